"""One training epoch of the reference driver on the device (GFlowNet100.py:278-321).

    log  = model.sample_states(s0, return_log=True)           gfx950 rollout + fill + reward
    loss = trajectory_balance_loss(Z, R, log.fwd_probs, log.back_probs)
           fwd_probs: the sampler's probabilities, backward = spai_logp_grad
           back_probs: BackwardPolicy, LSTM recurrence = spai_lstm_forward / _backward
    skip the update when the loss is NaN/Inf (GFlowNet100.py:298-300; one host sync, as there)
    scheduler.step(loss); loss.backward(); opt.step(); opt.zero_grad()
The ForwardPolicy's own backward (GATv2 x2 + mean pool + fc) runs the gfx950 kernels of
spai_policy_backward (policy._HipLogits; hidden sizes 4 and 8, the reference driver's hid = 4,
GFlowNet100.py:178-180); other hidden sizes differentiate the torch restatement on the device.
Adam is torch's (fused kernels on the device).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .utils import trajectory_balance_loss


@dataclass
class StepResult:
    log: object
    loss: torch.Tensor
    updated: bool


def train_step(model, opt, s0, scheduler=None) -> StepResult:
    """GFlowNet100.py:278-321 for one epoch (``model.train()`` then one batch)."""
    model.train()
    log = model.sample_states(s0, return_log=True)
    loss = trajectory_balance_loss(log.total_flow, log.rewards, log.fwd_probs, log.back_probs)
    if torch.isnan(loss) or torch.isinf(loss):
        return StepResult(log, loss.detach(), False)
    if scheduler is not None:
        scheduler.step(loss)
    loss.backward()
    opt.step()
    opt.zero_grad()
    return StepResult(log, loss.detach(), True)
