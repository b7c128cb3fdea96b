"""Multi-GPU layout of the hot path: one process per GPU, torch.distributed (RCCL over xGMI on
MI355X, gloo in the CPU tests).

Two ways to spread work:
  * columns (default of bench.py, the north star's split, strong scaling): every rank draws
    the same B candidates; rank r orders the r-th slice of every trajectory (rollout parts:
    a contiguous range of the presampled key buckets) and fills lines shard_lines(n, r, P) of
    every candidate's M.  ONE all_reduce per step carries the parts' bucket weight sums and
    winner counts and the squared residual partials (``exchange_parts``); the chosen M is
    assembled with ONE
    all_gather of equal-size ELL blocks (``allgather_lines``).
  * samples (strong scaling over a fixed global batch of B candidates, bench.py's default):
    rank r rolls out and fills candidates r*B/P .. (r+1)*B/P - 1 (the same Philox sample ids,
    hence the same draws, as a one-GPU batch); the step's exchange is one all_gather of the
    rewards and one reduce of the best candidate's M (``select_best_samples``).
  * candidates (weak scaling): rank r samples candidates with Philox sample ids
    r*B .. r*B+B-1 (``GFlowNet(sample_base=r*B)``); every candidate's trajectory, fill and
    reward live on one rank, so the step needs no collective.
The reference has no parallelism at all.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_lines(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced [begin, end) line range of ``rank`` (sizes differ by <= 1)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    q, r = divmod(n, world)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def allreduce_res2(res2: torch.Tensor, group=None) -> torch.Tensor:
    """Sum per-sample squared residual partials over the column shards (in place)."""
    dist.all_reduce(res2, op=dist.ReduceOp.SUM, group=group)
    return res2


def allgather_lines(m_local: torch.Tensor, n: int, group=None) -> torch.Tensor:
    """Assemble [B, n, W] line values from every rank's [B, n_r, W] block (one all_gather).

    Blocks are padded to ceil(n / P) lines so every rank contributes an equal-size chunk
    (the ring all-gather over xGMI is per-link bound: equal chunks keep every link busy)."""
    world = dist.get_world_size(group)
    B, n_loc, W = m_local.shape
    chunk = -(-n // world)
    buf = torch.zeros(B, chunk, W, dtype=m_local.dtype, device=m_local.device)
    buf[:, :n_loc] = m_local
    out = torch.empty(world, B, chunk, W, dtype=m_local.dtype, device=m_local.device)
    dist.all_gather_into_tensor(out.view(-1), buf.view(-1).contiguous(), group=group)
    parts = []
    for r in range(world):
        b, e = shard_lines(n, r, world)
        parts.append(out[r, :, : e - b])
    return torch.cat(parts, dim=1)


def select_best_samples(rewards_local: torch.Tensor, m_local: torch.Tensor, group=None, dst: int = 0):
    """The samples split's one exchange (no host round trip): every rank holds B/P candidates
    (global sample ids rank*B/P ...); ``rewards_local`` [B/P], ``m_local`` [B/P, n, W].  One
    all_gather makes the global rewards [B] known everywhere; the global argmax is found on the
    device, the owning rank contributes that candidate's M and every other rank zeros, and one
    reduce to ``dst`` delivers it there (x + 0 is exact).  Returns (rewards [B], best index
    [1] int64, M of the best candidate [n, W] -- valid on ``dst``)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    bl = rewards_local.numel()
    allr = torch.empty(world * bl, dtype=rewards_local.dtype, device=rewards_local.device)
    dist.all_gather_into_tensor(allr, rewards_local.contiguous(), group=group)
    best = torch.argmax(allr).view(1)
    mine = (best >= rank * bl) & (best < (rank + 1) * bl)
    pick = m_local.index_select(0, (best - rank * bl).clamp(0, bl - 1)).squeeze(0)
    out = torch.where(mine, pick, torch.zeros((), dtype=pick.dtype, device=pick.device)).contiguous()
    dist.reduce(out, dst=dist.get_global_rank(group, dst) if group is not None else dst, op=dist.ReduceOp.SUM,
                group=group)
    return allr, best, out


def gather_rewards(rewards: torch.Tensor, group=None) -> torch.Tensor:
    """[P*B] rewards of every rank's candidates, in rank order (for logging a global batch)."""
    world = dist.get_world_size(group)
    out = torch.empty(world * rewards.numel(), dtype=rewards.dtype, device=rewards.device)
    dist.all_gather_into_tensor(out, rewards.contiguous(), group=group)
    return out


def exchange_parts(xch: torch.Tensor, res2: torch.Tensor, group=None) -> torch.Tensor:
    """The split rollout's one collective, in place on the rollout workspace's exchange array
    (kernels.exchange_array: per-bucket weight sums and winner counts, each part non-zero on
    its own buckets only, so the sum is exact and equals the one-GPU array; then B slots):
    the lines' squared residual partials [B] go into the slots, one all_reduce sums
    everything, and the summed residuals (a view of the slots) are returned."""
    B = res2.numel()
    slots = xch[xch.numel() - B:]
    slots.copy_(res2.reshape(-1))
    dist.all_reduce(xch, op=dist.ReduceOp.SUM, group=group)
    return slots


def gather_slices(actions: torch.Tensor, fwd: torch.Tensor, bounds: torch.Tensor, T: int, group=None):
    """Full [B, T] trajectories from every rank's slice [bounds[b, 0], bounds[b, 1]) (the slices
    partition [0, T)): zero outside the slice, one all_reduce each (exact: one non-zero term)."""
    pos = torch.arange(T, device=actions.device).view(1, -1)
    mine = (pos >= bounds[:, :1]) & (pos < bounds[:, 1:])
    a = torch.where(mine, actions[:, :T], torch.zeros((), dtype=actions.dtype, device=actions.device)).contiguous()
    f = torch.where(mine, fwd[:, :T], torch.zeros((), dtype=fwd.dtype, device=fwd.device)).contiguous()
    dist.all_reduce(a, group=group)
    dist.all_reduce(f, group=group)
    return a, f
