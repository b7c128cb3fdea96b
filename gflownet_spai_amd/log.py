"""Trajectory log (reference: gflownet/log.py:10-164) holding device tensors.

After ``GFlowNet.sample_states`` the fields have the reference's shapes:
  ``actions`` / ``_actions``  [T, B] int64, -1 after a sample's terminal id E
  ``fwd_probs``               [B, T] fp32, 1.0 after the terminal
  ``back_probs``              [B, T] from the backward policy (log.py:123-164)
  ``rewards``                 [B] fp32 (gflownet.py:193: torch.tensor(..., dtype=log.rewards.dtype))
``fwd_probs`` is differentiable w.r.t. the policy logits when they require grad: the
values are the sampler's, and the backward (``_TrajProbs``) is the gfx950 kernel
spai_logp_grad — the closed-form derivative of the per-step masked softmax of
policy.py:65-73 (p_t = w_{a_t} / (untouched mass + sum_{s>=t} w_{a_s}), w = exp(l)) in
O(T + E) per sample, instead of autograd through [B, E+1] temporaries.
"""
from __future__ import annotations

import torch
from torch import Tensor


def trajectory_probs(logits: Tensor, actions_bt: Tensor) -> Tensor:
    """Differentiable [B, T] probabilities of the logged actions (-1 -> 1.0), fp64 inside.

    p_t = w_{a_t} / (untouched mass + sum_{s>=t} w_{a_s}), w = exp(l - max l): the masked
    softmax of step t (policy.py:65-73) written with the remaining mass, so it stays
    accurate however much mass the trajectory removes."""
    l = logits.reshape(-1) if logits.dim() == 1 or logits.shape[0] == 1 else logits
    l64 = l.double()
    w = torch.exp(l64 - l64.detach().max(dim=-1, keepdim=True).values)
    B, T = actions_bt.shape
    W = w.expand(B, -1) if w.dim() == 1 else w
    valid = actions_bt >= 0
    idx = actions_bt.clamp(min=0)
    zero = torch.zeros((), dtype=W.dtype, device=W.device)
    wa = torch.where(valid, W.gather(1, idx), zero)
    chosen = torch.zeros(W.shape, dtype=torch.bool, device=W.device)
    rows = torch.arange(B, device=W.device).view(-1, 1).expand(B, T)
    chosen[rows[valid], actions_bt[valid]] = True
    untouched = torch.where(chosen, zero, W).sum(1, keepdim=True)
    suffix = torch.flip(torch.cumsum(torch.flip(wa, [1]), 1), [1])
    p = wa / (untouched + suffix)
    return torch.where(valid, p, torch.ones((), dtype=p.dtype, device=p.device)).float()


class _TrajProbs(torch.autograd.Function):
    """fwd_probs [B, T] of a rollout as a differentiable function of the logits: forward
    returns the sampler's probabilities, backward runs spai_logp_grad."""

    @staticmethod
    def forward(ctx, logits, probs_bt, actions_bt, removed, lmax):
        ctx.save_for_backward(logits, probs_bt, actions_bt, removed, lmax)
        return probs_bt.clone()

    @staticmethod
    def backward(ctx, g):
        from . import kernels

        logits, probs_bt, actions_bt, removed, lmax = ctx.saved_tensors
        grad = kernels.logp_grad(logits, lmax, actions_bt, probs_bt, g, removed)
        return grad.to(logits.dtype), None, None, None, None


class Log:
    def __init__(self, s0, backward_policy, total_flow, env):
        self._fwd_probs = []
        self._back_probs = None
        self._act_list = []
        self._act_tb = None  # [T, B] once known
        self.rewards = torch.zeros(len(s0))
        self.backward_policy = backward_policy
        self.total_flow = total_flow
        self.env = env
        self.num_samples = len(s0)
        # set by the MI355X sampler
        self._logits = None
        self._full = None  # (actions [B, cap] i64, fwd [B, cap] f32, T int32 device scalar)
        self._actions_bt = None
        self._lmax = None
        self.removed = None
        self.counts = None
        self.rewards_all = None  # fp64 rewards of every candidate of a columns-split step (all ranks')

    def log(self, s, probs: Tensor, actions: Tensor, done: Tensor):
        """Per-step logging, log.py:24-89 semantics (used by custom loops)."""
        active = ~done.flatten().bool()
        fwd = torch.ones(actions.shape[0], device=actions.device)
        gathered = probs.gather(2, actions.unsqueeze(1)).view(-1)
        fwd[active] = gathered[active]
        self._fwd_probs.append(fwd)
        la = -torch.ones(self.num_samples, dtype=torch.long, device=actions.device)
        la[active] = actions.view(-1)[active]
        self._act_list.append(la)

    def _set_rollout(self, logits: Tensor, actions_bt: Tensor, fwd_bt: Tensor, t_dev: Tensor | None = None,
                     lmax: Tensor | None = None):
        """actions_bt / fwd_bt: [B, T] or, with t_dev, [B, cap] buffers of which the first
        T = int(t_dev) columns are the trajectory (T is read lazily: no sync in the rollout);
        lmax: the logits' maximum the sampler used (the gradient kernel's weight scale)."""
        self._logits = logits
        self._lmax = lmax
        if t_dev is None:
            self._actions_bt, self._fwd_probs, self._act_tb = actions_bt, fwd_bt, actions_bt.t()
        else:
            self._full = (actions_bt, fwd_bt, t_dev)

    def _set_part(self, rank: int, world: int, group, bounds: Tensor):
        """The rollout was split over ``world`` processes by trajectory slices:
        this rank's buffers hold only the slice [bounds[b, 0], bounds[b, 1]) of each sample.
        ``local_slice`` reads the rank's part; the full log needs ``gather_parts()`` — a
        collective every rank of the group must call — before ``actions`` / ``fwd_probs``."""
        self._part = (rank, world, group, bounds)

    def local_slice(self):
        """(actions [B, cap], fwd [B, cap], bounds [B, 2]) of this rank's part (split rollouts)."""
        a, f, _ = self._full
        return a, f, self._part[3]

    def gather_parts(self) -> "Log":
        """Assemble the full trajectories of a slices-split rollout: one all_reduce of the
        zero-masked slices (disjoint, so the sum is exact).  A COLLECTIVE: call it on every rank
        of the group, or on none.  A no-op for an unsplit rollout."""
        part = getattr(self, "_part", None)
        if self._full is not None and part is not None and part[1] > 1:
            from .distributed import gather_slices
            a, f, t = self._full
            T = int(t)
            a, f = gather_slices(a, f, part[3], T, part[2])
            self._actions_bt, self._fwd_probs = a, f
            self._act_tb = a.t()
            self._full = None
        return self

    def _materialize(self):
        if self._full is not None:
            part = getattr(self, "_part", None)
            if part is not None and part[1] > 1:
                raise RuntimeError("this Log holds one rank's slice of a split rollout: call log.gather_parts() on "
                                   "every rank first (a collective), or read log.local_slice()")
            a, f, t = self._full
            T = int(t)
            self._actions_bt, self._fwd_probs = a[:, :T], f[:, :T]
            self._act_tb = self._actions_bt.t()
            self._full = None

    @property
    def _actions(self):
        """[T, B] after a rollout (gflownet.py:181 leaves log._actions as that tensor)."""
        self._materialize()
        if self._act_tb is None and self._act_list:
            self._act_tb = torch.stack(self._act_list, dim=0)
        return self._act_tb if self._act_tb is not None else self._act_list

    @property
    def fwd_probs(self) -> Tensor:
        self._materialize()
        if isinstance(self._fwd_probs, list):
            self._fwd_probs = torch.stack(self._fwd_probs, dim=0).t()
        if self._logits is not None and self._logits.requires_grad and torch.is_grad_enabled():
            if self._logits.is_cuda and self.removed is not None and self._lmax is not None:
                return _TrajProbs.apply(self._logits, self._fwd_probs, self._actions_bt, self.removed, self._lmax)
            return trajectory_probs(self._logits, self._actions_bt)
        return self._fwd_probs

    @property
    def actions(self) -> Tensor:
        return self._actions

    @property
    def back_probs(self) -> Tensor:
        if self._back_probs is None:
            bp = self.backward_policy(self.actions.t())
            self._back_probs = bp.reshape(self.num_samples, -1)
        return self._back_probs
