"""Trajectory log (reference: gflownet/log.py:10-164) holding device tensors.

After ``GFlowNet.sample_states`` the fields have the reference's shapes:
  ``actions`` / ``_actions``  [T, B] int64, -1 after a sample's terminal id E
  ``fwd_probs``               [B, T] fp32, 1.0 after the terminal
  ``back_probs``              [B, T] from the backward policy (log.py:123-164)
  ``rewards``                 [B] fp32 (gflownet.py:193: torch.tensor(..., dtype=log.rewards.dtype))
``fwd_probs`` is differentiable w.r.t. the policy logits when they require grad: the
sampler kernels are not differentiable, so the probabilities of the sampled order are
recomputed with torch ops from the fixed logits (closed form of the per-step masked
softmax of policy.py:65-73: p_t = w_{a_t} / (Z - sum_{s<t} w_{a_s}), w = exp(l)).
"""
from __future__ import annotations

import torch
from torch import Tensor


def trajectory_probs(logits: Tensor, actions_bt: Tensor) -> Tensor:
    """Differentiable [B, T] probabilities of the logged actions (-1 -> 1.0), fp64 internally."""
    l = logits.reshape(-1) if logits.dim() == 1 or logits.shape[0] == 1 else logits
    l64 = l.double()
    w = torch.exp(l64 - l64.detach().max(dim=-1, keepdim=True).values)
    Z = w.sum(-1, keepdim=True)
    valid = actions_bt >= 0
    idx = actions_bt.clamp(min=0)
    wa = (w.expand(actions_bt.shape[0], -1) if w.dim() == 1 or w.shape[0] == 1 else w).gather(1, idx)
    wa = torch.where(valid, wa, torch.zeros((), dtype=wa.dtype, device=wa.device))
    before = torch.cumsum(wa, 1) - wa
    p = wa / (Z.view(-1, 1) - before)
    return torch.where(valid, p, torch.ones((), dtype=p.dtype, device=p.device)).float()


class Log:
    def __init__(self, s0, backward_policy, total_flow, env):
        self._fwd_probs = []
        self._back_probs = None
        self._actions = []
        self.rewards = torch.zeros(len(s0))
        self.backward_policy = backward_policy
        self.total_flow = total_flow
        self.env = env
        self.num_samples = len(s0)
        # set by the MI355X sampler
        self._logits = None
        self._actions_bt = None
        self.removed = None
        self.counts = None

    def log(self, s, probs: Tensor, actions: Tensor, done: Tensor):
        """Per-step logging, log.py:24-89 semantics (used by custom loops)."""
        active = ~done.flatten().bool()
        fwd = torch.ones(actions.shape[0], device=actions.device)
        gathered = probs.gather(2, actions.unsqueeze(1)).view(-1)
        fwd[active] = gathered[active]
        self._fwd_probs.append(fwd)
        la = -torch.ones(self.num_samples, dtype=torch.long, device=actions.device)
        la[active] = actions.view(-1)[active]
        self._actions.append(la)

    def _set_rollout(self, logits: Tensor, actions_bt: Tensor, fwd_bt: Tensor):
        self._logits = logits
        self._actions_bt = actions_bt
        self._actions = actions_bt.t()
        self._fwd_probs = fwd_bt

    @property
    def fwd_probs(self) -> Tensor:
        if isinstance(self._fwd_probs, list):
            self._fwd_probs = torch.stack(self._fwd_probs, dim=0).t()
        if self._logits is not None and self._logits.requires_grad and torch.is_grad_enabled():
            return trajectory_probs(self._logits, self._actions_bt)
        return self._fwd_probs

    @property
    def actions(self) -> Tensor:
        if isinstance(self._actions, list):
            self._actions = torch.stack(self._actions, dim=0)
        return self._actions

    @property
    def back_probs(self) -> Tensor:
        if self._back_probs is None:
            bp = self.backward_policy(self.actions.t())
            self._back_probs = bp.reshape(self.num_samples, -1)
        return self._back_probs
