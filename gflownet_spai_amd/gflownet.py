"""Drop-in ``GFlowNet`` (reference: gflownet/gflownet.py:12-257) with the MI355X sampler.

``sample_states(s0, return_log=True) -> Log`` keeps the reference's contract.  The
policy's logits are state-independent within a rollout (gflownet.py:133,145: data_list
is built once from s0 and only the action mask changes), so they are produced ONCE per
rollout and the T-step loop runs on the device:

  mode="parity"     the reference's sampler step for step: per step B*(E+1) Exp(1) noise
                    from the torch CPU generator (exactly what Categorical(probs).sample()
                    draws, gflownet.py:148) and one fused masked-argmax kernel; bit-exact
                    actions vs the reference given the same torch seed.  O(T*B*E).
  mode="throughput" one-pass Gumbel-top-k (Philox, no host noise): all trajectories in
                    O(B*E) — distributionally identical to the sequential sampler.
Then ``env.update`` semantics: removal bitmaps -> fill -> residual -> rewards.
"""
from __future__ import annotations

from typing import List

import torch
from torch import Tensor, nn

from . import kernels
from .log import Log, trajectory_probs
from .preconditioner import Data


class GFlowNet(nn.Module):
    def __init__(self, forward_policy, backward_policy, env, *, mode: str = "parity", seed: int | None = None,
                 sample_base: int = 0, shard: tuple | None = None):
        super().__init__()
        if mode not in ("parity", "throughput"):
            raise ValueError("mode must be 'parity' or 'throughput'")
        self.register_buffer("total_flow", torch.ones(1))
        self.forward_policy = forward_policy
        self.backward_policy = backward_policy
        self.env = env
        self.mode = mode
        self._alpha_mean = None  # (key, mean over the batch of a constant sigmoid(alpha), pin)
        self.seed = int(torch.initial_seed() if seed is None else seed) & (2**64 - 1)
        self.sample_base = sample_base
        self.rollouts = 0  # Philox stream id of the next throughput rollout (host mirror)
        self._ctr = None   # the same counter on the device (advanced by the select phase itself)
        self._data_cache = {}
        # (rank, world, group): the columns split of DESIGN.md §6 (throughput mode).  Every rank
        # draws the same B candidates; rank r orders the r-th slice of every trajectory
        # (rollout parts) and fills lines shard_lines(n, r, world) of every candidate's M; one
        # all_reduce carries the parts' bucket weight sums and the squared residual partials.
        self.shard = shard
        if shard is not None:
            from .distributed import shard_lines
            rank, world, _ = shard
            self.lines = shard_lines(env.matrix_size, rank, world) if env is not None else None

    # ------------------------------------------------------------------ policy
    def policy_logits(self, data, batch_size: int):
        """(logits [E+1] fp32, alpha 0-d, lmax [B] or None) for this rollout.

        Uses ``forward_policy.logits_and_max(data, B)`` (ForwardPolicy here: the gfx950
        kernels also return the logits' maximum), else ``.logits(data)``, else the reference
        call contract ``forward(data, empty)`` -> probs and logits = log(probs) (a constant
        shift, irrelevant to sampling).  alpha is the mean of the B per-sample
        sigmoid(alpha) values, as gflownet.py:89."""
        lmax = None
        if hasattr(self.forward_policy, "logits_and_max"):
            logits, a, lmax = self.forward_policy.logits_and_max(data, batch_size)
        elif hasattr(self.forward_policy, "logits"):
            logits, a = self.forward_policy.logits(data)
        else:
            probs, a = self.forward_policy(data, torch.empty(0, dtype=torch.long))
            logits = torch.log(probs)
        if a.requires_grad or a._version != 0:
            alpha = torch.stack([a] * batch_size, dim=0).mean()
        else:  # a constant (the policy's cached sigmoid): its batch mean is cached with it
            key = (id(a), a.data_ptr(), batch_size)
            hit = self._alpha_mean
            if hit is None or hit[0] != key:
                hit = self._alpha_mean = (key, torch.stack([a] * batch_size, dim=0).mean(), a)  # a pins the id
            alpha = hit[1]
        return logits.reshape(-1), alpha, lmax

    def forward_probs(self, s, data_list, actions=None):
        """gflownet.py:47-123 (reference API; per-sample policy calls, not the hot path)."""
        if actions is None or len(actions) == 0:
            actions = torch.empty(0)
        else:
            actions = torch.stack(list(actions), dim=1) if torch.is_tensor(actions[0]) else torch.tensor(actions).t()
        probs, alphas = [], []
        for i, data in enumerate(data_list):
            act = actions[i, :] if actions.numel() > 0 else torch.empty(0, dtype=torch.long)
            p, a = self.forward_policy(data, act)
            probs.append(p)
            alphas.append(a)
        probs = torch.stack(probs, dim=0)
        if probs.size(0) > 1:
            tot = probs.sum(2)
            tot[tot == 0] = 1
            probs = probs / tot.unsqueeze(1)
        return probs, torch.stack(alphas, dim=0).mean()

    def state_to_data(self, s: List[Tensor]) -> list:
        """gflownet.py:223-257: one Data(x=ones(2N,1), edge_index, edge_attr) per state."""
        out = []
        for i, m in enumerate(s):
            if not m.is_sparse:
                raise ValueError(f"Tensor at index {i} is not a sparse tensor.")
            key = (m._indices().data_ptr(), m._values().data_ptr(), m._nnz(), self.env.matrix_size)
            hit = self._data_cache.get(key)
            if hit is None:  # states are never modified by a rollout: build each graph once
                dev = self.env.device
                d = Data(x=torch.ones((self.env.matrix_size * 2, 1), device=dev),
                         edge_index=m._indices().to(dev), edge_attr=m._values().float().to(dev))
                hit = self._data_cache[key] = (m, d)  # holding m pins its storage (key stays unique)
                if len(self._data_cache) > 8:
                    self._data_cache.pop(next(iter(self._data_cache)))
            out.append(hit[1])
        return out

    def _same_states(self, s0) -> bool:
        """True when every initial state is the same matrix (the drivers pass clones of one
        matrix, GFlowNet100.py:276): same storage, or equal indices and values (compared once per
        set of storages and versions).  Then one policy call serves every sample (the logits
        depend on the state only)."""
        key = tuple((m._indices().data_ptr(), m._values().data_ptr(), m._values()._version, m._nnz())
                    if m.is_sparse else id(m) for m in s0)
        memo = getattr(self, "_same_memo", None)
        if memo is not None and memo[0] == key:
            return memo[1]
        same = self._compare_states(s0)
        self._same_memo = (key, same, list(s0))  # the list pins the storages the key names
        return same

    @staticmethod
    def _compare_states(s0) -> bool:
        m0 = s0[0]
        for m in s0[1:]:
            if m is m0:
                continue
            if not (m.is_sparse and m0.is_sparse) or m.shape != m0.shape or m._nnz() != m0._nnz():
                return False
            i0, v0, i1, v1 = m0._indices(), m0._values(), m._indices(), m._values()
            if i0.data_ptr() == i1.data_ptr() and v0.data_ptr() == v1.data_ptr():
                continue
            if not (torch.equal(i0, i1.to(i0.device)) and torch.equal(v0, v1.to(v0.device))):
                return False
        return True

    def _rewards(self, removed, counts, alpha):
        return self.env.rewards_from_removed(removed, counts, alpha)

    # ------------------------------------------------------------------ sampler
    def sample_states(self, s0, return_log: bool = False):
        """gflownet.py:125-197: sample B trajectories from the initial states, score them, log."""
        if self.mode == "throughput":
            st = self.rollout_begin(s0)
            self.rollout_exchange(st)
            log = self.rollout_end(st)
            return log if return_log else None
        env = self.env
        B = len(s0)
        E = env.num_actions - 1
        log = Log(s0, self.backward_policy, self.total_flow, env)
        logits, alpha, lg, lmax, z = self._logits(s0, need_z=True)
        actions_bt, fwd_bt = self._parity_rollout(lg, B, lmax, z)
        removed, counts = kernels.actions_to_removed(actions_bt, E)
        rewards = self._rewards(removed, counts, alpha)
        log._set_rollout(logits, actions_bt, fwd_bt, lmax=lmax)
        log.removed, log.counts = removed, counts
        log.rewards = rewards.detach().to(torch.float32)
        return log if return_log else None

    def _logits(self, s0, need_z: bool = False):
        """(logits, alpha, sampler logits fp32 on the device, lmax [B], z [B] or None)."""
        env = self.env
        B = len(s0)
        E = env.num_actions - 1
        if self._same_states(s0):
            data_list = self.state_to_data(s0[:1])
            logits, alpha, lmax = self.policy_logits(data_list[0], B)
            if logits.numel() != E + 1:
                raise ValueError(f"policy produced {logits.numel()} logits for {E + 1} actions")
        else:
            # distinct initial states: one policy call per sample (gflownet.py:70-74 builds one
            # Data per sample), per-sample logit rows [B, E+1] for the sampler
            rows, alphas = [], []
            for d in self.state_to_data(s0):
                l, a, _ = self.policy_logits(d, 1)
                if l.numel() != E + 1:
                    raise ValueError(f"policy produced {l.numel()} logits for {E + 1} actions")
                rows.append(l)
                alphas.append(a)
            logits, alpha, lmax = torch.stack(rows, 0), torch.stack(alphas).mean(), None
        if lmax is not None and not need_z and logits.is_cuda and logits.dtype == torch.float32:
            return logits, alpha, logits.detach(), lmax, None  # the policy kernels produced the maximum
        lg, lmax, z = kernels.logits_stats(logits.detach().to(env.device), B)
        return logits, alpha, lg, lmax, z

    # The throughput step in three phases, so a caller can capture the collective-free ones in
    # HIP graphs (bench.py): begin = policy, select, fill of this rank's lines; exchange = the
    # split's one all_reduce (nothing on one GPU); end = merge (split only), sort of this rank's
    # trajectory slice with its fwd_probs, terminal step / padding, rewards, the Log.  No
    # phase synchronises with the host; the Philox stream id lives on the device and the select
    # phase advances it, so a replayed graph draws a fresh rollout.
    def rollout_begin(self, s0) -> dict:
        env = self.env
        B = len(s0)
        E = env.num_actions - 1
        logits, alpha, lg, lmax, _ = self._logits(s0)
        if self._ctr is None or self._ctr.device != lg.device:
            self._ctr = torch.tensor([self.rollouts], dtype=torch.int64, device=lg.device)
        self.rollouts += 1
        rank, world, group = self.shard if self.shard is not None else (0, 1, None)
        removed, counts, ws = kernels.rollout_select(lg, B, lmax, self.seed, 0, self.sample_base, self._ctr, rank,
                                                     world)
        lines = self.lines if self.shard is not None else (0, None)
        res2 = env.fill_partial(removed, *lines)
        return dict(s0=s0, B=B, E=E, logits=logits, alpha=alpha, lg=lg, lmax=lmax, removed=removed, counts=counts,
                    ws=ws, res2_part=res2, part=(rank, world, group))

    def rollout_exchange(self, st: dict) -> None:
        """ONE all_reduce over the split, in place on the rollout workspace's exchange array:
        the parts' bucket weight sums and winner counts (disjoint supports: the sum is exact and
        equals the one-GPU array) and the lines' squared residual partials.  The summed
        residuals are a view of that array (a captured ``rollout_end`` graph keeps reading it)."""
        rank, world, group = st["part"]
        if world == 1:
            st["res2"] = st["res2_part"]
            return
        from .distributed import exchange_parts
        st["res2"] = exchange_parts(kernels.exchange_array(st["ws"], st["E"], st["B"]), st["res2_part"], group)

    def rollout_end(self, st: dict) -> Log:
        env = self.env
        rank, world, group = st["part"]
        B, E, lg, lmax, counts, ws = st["B"], st["E"], st["lg"], st["lmax"], st["counts"], st["ws"]
        if world > 1:  # counts, T and the bucket positions need every part's buckets
            kernels.rollout_merge(lg, B, lmax, ws, rank, world, counts)
        actions, fwd = kernels.rollout_sort(lg, B, lmax, ws, rank, world)
        t_dev = kernels.rollout_finish(lg, B, lmax, counts, ws, actions, fwd, rank, world)
        rewards = env.rewards_from_res2(st["res2"], counts, st["alpha"])
        log = Log(st["s0"], self.backward_policy, self.total_flow, env)
        log._set_rollout(st["logits"], actions, fwd, t_dev, lmax=lmax)
        if world > 1:
            log._set_part(rank, world, group, kernels.part_bounds(ws, E, B, rank, world))
        log.removed, log.counts = st["removed"], counts
        log.rewards = rewards.detach().to(torch.float32)
        return log

    def _parity_rollout(self, lg: Tensor, B: int, lmax: Tensor, z: Tensor):
        E1 = lg.shape[-1]
        dev = lg.device
        chosen = torch.zeros(B, (E1 + 31) // 32, dtype=torch.int32, device=dev)
        active = torch.ones(B, dtype=torch.uint8, device=dev)
        zrem = z.clone()
        acts, probs = [], []
        while True:
            # exactly the draws of Categorical(probs).sample() -> multinomial fast path
            noise = torch.empty(B, E1).exponential_(1)
            a, p = kernels.parity_step(lg, B, noise, lmax, chosen, active, zrem)
            acts.append(a)
            probs.append(p)
            if not bool(active.any()):
                break
        actions_bt = torch.stack(acts, 1)
        # logged probabilities from the remaining mass (no running-sum cancellation)
        return actions_bt, trajectory_probs(lg, actions_bt)
