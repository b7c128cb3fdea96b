"""Multi-GPU layout of the hot path: one process per GPU, torch.distributed (RCCL over xGMI on
MI355X, gloo in the CPU tests).

Two ways to spread work:
  * candidates (default, weak scaling): rank r samples candidates with Philox sample ids
    r*B .. r*B+B-1 (``GFlowNet(sample_base=r*B)``); every candidate's trajectory, fill and
    reward live on one rank, so the step needs no collective.
  * columns of one candidate (strong scaling of a single huge M): rank r owns lines
    [shard_lines(n, r, P)); the per-sample squared residuals are summed with ONE
    all_reduce of B fp64 (``PreconditionerEnv.rewards_from_removed(..., group=...)``) and M
    is assembled with ONE all_gather of equal-size ELL blocks (``allgather_lines``).
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


def gather_rewards(rewards: torch.Tensor, group=None) -> torch.Tensor:
    """[P*B] rewards of every rank's candidates, in rank order (for logging a global batch)."""
    world = dist.get_world_size(group)
    out = torch.empty(world * rewards.numel(), dtype=rewards.dtype, device=rewards.device)
    dist.all_gather_into_tensor(out, rewards.contiguous(), group=group)
    return out
