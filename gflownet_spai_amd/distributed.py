"""Multi-GPU layout of the hot path: one process per GPU, torch.distributed (RCCL over xGMI on
MI355X, gloo in the CPU tests).  The reference has no parallelism at all.

Three ways to spread the work; ``GFlowNet(shard=(rank, world, group), split=...)``:
  * columns (bench.py's default for --gpus > 1; the north star's "columns of M shard across the
    GPUs, one all-gather assembles M"): rank r rolls out ITS candidates (global sample ids
    r*Bl .. r*Bl + Bl - 1: the same Philox draws as a one-GPU batch of P*Bl), then
      1. one all_to_all of the removal bits: rank q receives, for every candidate, exactly the
         bits of its lines' action ids packed in line-major order, plus the candidate's removal
         count, whatever the matrix numbering (``PackPlan`` / spai_bitmap_pack /
         ``exchange_packed``);
      2. every rank fills lines ``shard_lines(n, r, P, align=256)`` of ALL P*Bl candidates;
      3. one all_reduce of the exact (integer-limb) squared-residual sums [P*Bl] — bit-identical
         to one GPU whatever P, because the shards are 256-line aligned and integer sums are
         associative (spai_hip.h SPAI_RES2_LIMBS);
      4. one all_gather of the best candidate's M lines (``allgather_lines``).
  * slices (strong scaling over the trajectory): every rank draws all E actions of the same B
    candidates and orders one contiguous slice of every trajectory; one all_reduce of the bucket
    sums + residual partials (``exchange_parts``).  The full log needs the explicit collective
    ``Log.gather_parts()`` on every rank.
  * samples (bench.py --shard samples): rank r rolls out and fills candidates r*B/P ..; one
    all_gather of the rewards and one reduce of the best candidate's M (``select_best_samples``).
  * candidates (weak scaling, ``GFlowNet(sample_base=r*B)``): no collective.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

LINE_ALIGN = 256  # lines per fill block (gram.hip / fill.hip kNT): the exact-sum invariance unit


def shard_lines(n: int, rank: int, world: int, align: int = 1) -> tuple[int, int]:
    """Contiguous, balanced [begin, end) line range of ``rank``.  With ``align`` > 1 the ranges
    are made of whole ``align``-line blocks (sizes differ by <= one block; the last is cut at n)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    if align < 1:
        raise ValueError("align must be >= 1")
    nb = -(-n // align)
    q, r = divmod(nb, world)
    b0 = rank * q + min(rank, r)
    b1 = b0 + q + (1 if rank < r else 0)
    return min(n, b0 * align), min(n, b1 * align)


def _host_staged(t: torch.Tensor, group) -> bool:
    """gloo has no device kernels for the ops used here: stage device tensors through the host."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_reduce_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM all_reduce (host-staged on gloo)."""
    if _host_staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


class _Done:
    def wait(self):
        return None


def all_gather_into_(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    """all_gather_into_tensor (host-staged and synchronous on gloo).  Returns ``out``, or with
    ``async_op`` a work handle whose ``wait()`` orders the current stream after the gather."""
    if _host_staged(inp, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, inp.cpu(), group=group)
        out.copy_(h)
        return _Done() if async_op else out
    w = dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)
    return w if async_op else out


def all_to_all_(out: torch.Tensor, inp: torch.Tensor, out_splits: list, in_splits: list, group=None,
                async_op: bool = False):
    """all_to_all_single with uneven splits; returns a work handle (``wait()`` orders the current
    stream after it on RCCL; host-staged and synchronous on gloo)."""
    if _host_staged(inp, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(h)
        return _Done()
    w = dist.all_to_all_single(out, inp, out_splits, in_splits, group=group, async_op=async_op)
    return w if async_op else _Done()


def allreduce_res2(res2: torch.Tensor, group=None) -> torch.Tensor:
    """Sum per-sample squared residual partials over the column shards (in place)."""
    return all_reduce_(res2, group)


def allgather_lines(m_local: torch.Tensor, n: int, group=None, align: int = 1) -> torch.Tensor:
    """Assemble [B, n, W] line values from every rank's [B, n_r, W] block (one all_gather);
    rank r's block is lines ``shard_lines(n, r, P, align)``.

    Blocks are padded to the largest shard so every rank contributes an equal-size chunk
    (the ring all-gather over xGMI is per-link bound: equal chunks keep every link busy)."""
    world = dist.get_world_size(group)
    B, n_loc, W = m_local.shape
    rng = [shard_lines(n, r, world, align) for r in range(world)]
    chunk = max(e - b for b, e in rng)
    if n_loc == chunk:
        buf = m_local.contiguous()
    else:
        buf = torch.zeros(B, chunk, W, dtype=m_local.dtype, device=m_local.device)
        buf[:, :n_loc] = m_local
    out = torch.empty(world, B, chunk, W, dtype=m_local.dtype, device=m_local.device)
    all_gather_into_(out.view(-1), buf.view(-1), group)
    if all(e - b == chunk for b, e in rng):
        return out.permute(1, 0, 2, 3).reshape(B, world * chunk, W)
    return torch.cat([out[r, :, : e - b] for r, (b, e) in enumerate(rng)], dim=1)


class LineGather:
    """``allgather_lines`` pipelined across steps: ``start(m_local)`` copies the rank's block into
    a persistent send buffer and launches the all_gather asynchronously (RCCL runs it on its own
    stream, so it overlaps whatever the current stream does next — the next step's rollout); the
    next ``start`` (or ``result`` / ``wait``) first orders the current stream after the previous
    gather, so the buffers are reused only once it has finished.  ``result()`` is the [B, n, W]
    assembly of the last started gather."""

    def __init__(self, n: int, group=None, align: int = 1):
        self.n, self.group, self.align = n, group, align
        self.work = None
        self.buf = self.out = None

    def wait(self) -> None:
        if self.work is not None:
            self.work.wait()
            self.work = None

    def start(self, m_local: torch.Tensor, rows: torch.Tensor | None = None) -> "LineGather":
        """rows: optional int64 index tensor on the device — gather only those candidates of
        m_local (copied straight into the send buffer, no intermediate)."""
        world = dist.get_world_size(self.group)
        B, n_loc, W = m_local.shape
        if rows is not None:
            B = rows.numel()
        self.rng = [shard_lines(self.n, r, world, self.align) for r in range(world)]
        chunk = max(e - b for b, e in self.rng)
        from .kernels import _timed
        with _timed("line_gather_wait"):  # (bench.py: the stream's wait for the previous gather)
            self.wait()  # the previous gather has read buf and written out
        if self.buf is None or self.buf.shape != (B, chunk, W) or self.buf.dtype != m_local.dtype:
            self.buf = torch.zeros(B, chunk, W, dtype=m_local.dtype, device=m_local.device)  # padding rows stay 0
            self.out = torch.empty(world, B, chunk, W, dtype=m_local.dtype, device=m_local.device)
        if rows is None:
            self.buf[:, :n_loc].copy_(m_local)
        elif n_loc == chunk:
            torch.index_select(m_local, 0, rows, out=self.buf)
        else:
            self.buf[:, :n_loc].copy_(m_local.index_select(0, rows))
        self.work = all_gather_into_(self.out.view(-1), self.buf.view(-1), self.group, async_op=True)
        return self

    def result(self) -> torch.Tensor:
        self.wait()
        world, B, chunk, W = self.out.shape
        if all(e - b == chunk for b, e in self.rng):
            return self.out.permute(1, 0, 2, 3).reshape(B, world * chunk, W)
        return torch.cat([self.out[r, :, : e - b] for r, (b, e) in enumerate(self.rng)], dim=1)


# ---------------------------------------------------------------- columns split: bitmap exchange
def word_spans(env, world: int) -> list:
    """[(w0, w1)] per rank: the bitmap words the action ids of rank q's lines span (one host
    sync).  For stencil matrices in row-major raw order a column shard's action ids are one
    contiguous range (its rows +- the stencil's reach), so a rank needs ~1/P of every bitmap; a
    randomly numbered matrix degrades to whole bitmaps (an all_gather's volume) — the product
    path exchanges line-major packed bits instead (``PackPlan``); the windows remain as a
    diagnostic of a numbering's locality."""
    act = env.pattern.act
    spans = []
    for q in range(world):
        b, e = shard_lines(env.matrix_size, q, world, LINE_ALIGN)
        a = act[b:e].reshape(-1)
        a = a[a >= 0]
        if a.numel() == 0:
            spans.append((0, 1))
            continue
        lo, hi = int(a.min()) >> 5, (int(a.max()) >> 5) + 1
        spans.append((lo, hi))
    return spans


class PackPlan:
    """The columns split's bitmap exchange plan for ``world`` ranks (built once per env and world,
    one host sync): per rank q the LINE-MAJOR action ids of its 256-line shard (``ids`` =
    all shards one after the other, ``seg`` [P+1] their bounds) and the packed word count
    ``wq[q]`` = ceil(nnz(shard q) / 32).  The send buffer of a rank with ``bl`` candidates is, per
    destination q, [bl][wq[q] + 1] words (q's bits packed in that order, then the removal count:
    spai_hip.h spai_bitmap_pack); rank r receives [P * bl, wq[r] + 1] and its fill reads the bits
    through ``local_pattern(env, r)``: the pattern with each of r's action ids replaced by its
    position in r's segment.  Every rank receives exactly nnz(shard) bits per candidate for any
    numbering of the matrix (action ids are raw COO positions, preconditioner.py:23-25).

    ``mode="window"`` (spai_window_pack; "auto" picks it when the windows total <= 1.25x the
    packed words, as for a stencil in row-major raw order, where rank q's ids span its rows +- the
    stencil's reach): q receives the contiguous bitmap words [lo[q], lo[q] + wq[q]) of its ids,
    copied without the gather, and reads them through ids shifted by 32 lo[q]."""

    WINDOW_SLACK = 1.25

    def __init__(self, env, world: int, mode: str = "auto"):
        if mode not in ("auto", "window", "gather"):
            raise ValueError(f"mode must be auto, window or gather, not {mode!r}")
        act = env.pattern.act
        dev = act.device
        self.world = world
        ids, seg, self.wq, self.lines, win = [], [0], [], [], []
        for q in range(world):
            b, e = shard_lines(env.matrix_size, q, world, LINE_ALIGN)
            a = act[b:e].reshape(-1)
            a = a[a >= 0]
            ids.append(a)
            seg.append(seg[-1] + a.numel())
            self.wq.append((a.numel() + 31) // 32)
            self.lines.append((b, e))
            win.append((int(a.min()) >> 5, (int(a.max()) >> 5) + 1) if a.numel() else (0, 0))
        self.ids = torch.cat(ids).to(torch.int32).contiguous()
        self.seg = torch.tensor(seg, dtype=torch.int64, device=dev)
        self.max_seg = max(seg[q + 1] - seg[q] for q in range(world))
        if mode == "auto":
            mode = "window" if sum(h - l for l, h in win) <= self.WINDOW_SLACK * sum(self.wq) else "gather"
        self.mode = mode
        if mode == "window":
            self.lo_words = [l for l, _ in win]
            self.wq = [h - l for l, h in win]
            self.lo = torch.tensor(self.lo_words, dtype=torch.int64, device=dev)
            self.span = torch.tensor(self.wq, dtype=torch.int64, device=dev)
            self.max_span = max(self.wq)
        self._off = {}
        self._local = {}

    def out_off(self, bl: int) -> torch.Tensor:
        """[P] int64 word offsets of the destinations' blocks in a send buffer of bl candidates."""
        if bl not in self._off:
            o = [0]
            for w in self.wq[:-1]:
                o.append(o[-1] + bl * (w + 1))
            self._off[bl] = (torch.tensor(o, dtype=torch.int64, device=self.seg.device), o[-1] + bl * (self.wq[-1] + 1))
        return self._off[bl]

    def send_words(self, bl: int) -> int:
        return self.out_off(bl)[1]

    def local_pattern(self, env, rank: int):
        """env.pattern with rank's action ids renumbered 0 .. nnz(shard) - 1 in line-major order
        (the bit positions of its received packed rows); other lines are left as they are."""
        if rank not in self._local:
            import dataclasses
            b, e = self.lines[rank]
            act = env.pattern.act.clone()
            blk = act[b:e]
            ok = blk >= 0
            if self.mode == "window":  # bit positions within the rank's word window
                loc = blk.to(torch.int64) - 32 * self.lo_words[rank]
            else:  # positions in the rank's line-major segment
                loc = torch.cumsum(ok.reshape(-1).to(torch.int64), 0).view_as(blk) - 1
            act[b:e] = torch.where(ok, loc.to(torch.int32), blk)
            self._local[rank] = dataclasses.replace(env.pattern, act=act)
        return self._local[rank]


def pack_bits_reference(removed: torch.Tensor, counts: torch.Tensor, plan: "PackPlan", bl: int) -> torch.Tensor:
    """torch restatement of spai_bitmap_pack / spai_window_pack (test infrastructure: the CPU gloo
    tests build the send buffer with it; the GPU tests check the kernels against it)."""
    out = []
    if plan.mode == "window":
        for q in range(plan.world):
            w = removed.view(torch.int32)[:, plan.lo_words[q]:plan.lo_words[q] + plan.wq[q]]
            out.append(torch.cat([w, counts.view(bl, 1).to(torch.int32)], 1).reshape(-1))
        return torch.cat(out)
    seg = plan.seg.tolist()
    for q in range(plan.world):
        a = plan.ids[seg[q]:seg[q + 1]].long().to(removed.device)
        words = plan.wq[q]
        bits = ((removed.view(torch.int32)[:, a >> 5].long() >> (a & 31)) & 1).to(torch.int64)  # [bl, m]
        pad = torch.zeros(bl, words * 32, dtype=torch.int64, device=removed.device)
        pad[:, :a.numel()] = bits
        w = (pad.view(bl, words, 32) << torch.arange(32, device=removed.device)).sum(2)
        w = torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)
        out.append(torch.cat([w, counts.view(bl, 1).to(torch.int32)], 1).reshape(-1))
    return torch.cat(out)


def exchange_packed(send: torch.Tensor, recv: torch.Tensor, plan: "PackPlan", bl: int, rank: int, group=None,
                    async_op: bool = False):
    """The columns split's all_to_all of packed rows: ``send`` [plan.send_words(bl)] int32 ->
    ``recv`` [P * bl, wq[rank] + 1] int32 (every candidate's packed bits of this rank's shard, then
    its removal count; global sample order: rank q's candidates are rows q*bl ..)."""
    in_splits = [bl * (w + 1) for w in plan.wq]
    out_splits = [bl * (plan.wq[rank] + 1)] * plan.world
    return all_to_all_(recv.view(-1), send, out_splits, in_splits, group, async_op)


def bitmap_pack_index(spans: list, bl: int, words: int, device) -> torch.Tensor:
    """int64 gather index over a rank's [bl * words + bl] buffer (bitmaps, then the bl removal
    counts) producing its all_to_all send buffer: for destination q, rows b = 0..bl-1 of
    (words w0_q .. w1_q - 1 of bitmap b, then count b)."""
    parts = []
    for w0, w1 in spans:
        rows = torch.arange(bl, device=device, dtype=torch.int64).view(-1, 1)
        cols = torch.arange(w0, w1, device=device, dtype=torch.int64).view(1, -1)
        blk = torch.cat([rows * words + cols, bl * words + rows], dim=1)  # [bl, span + 1]
        parts.append(blk.reshape(-1))
    return torch.cat(parts)


def exchange_bitmaps(send: torch.Tensor, recv: torch.Tensor, spans: list, bl: int, rank: int, group=None,
                     async_op: bool = False):
    """The columns split's all_to_all: ``send`` (from ``bitmap_pack_index``) -> ``recv`` int32
    [P * bl, span_r + 1] = every candidate's window of this rank's words + its removal count, in
    global sample order (rank q's candidates are rows q*bl ..)."""
    world = len(spans)
    span_r = spans[rank][1] - spans[rank][0]
    in_splits = [bl * (w1 - w0 + 1) for w0, w1 in spans]
    out_splits = [bl * (span_r + 1)] * world
    return all_to_all_(recv.view(-1), send, out_splits, in_splits, group, async_op)


# ---------------------------------------------------------------- samples split
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
    all_gather_into_(allr, rewards_local.contiguous(), group)
    best = torch.argmax(allr).view(1)
    mine = (best >= rank * bl) & (best < (rank + 1) * bl)
    pick = m_local.index_select(0, (best - rank * bl).clamp(0, bl - 1)).squeeze(0)
    out = torch.where(mine, pick, torch.zeros((), dtype=pick.dtype, device=pick.device)).contiguous()
    dst_g = dist.get_global_rank(group, dst) if group is not None else dst
    if _host_staged(out, group):
        h = out.cpu()
        dist.reduce(h, dst=dst_g, op=dist.ReduceOp.SUM, group=group)
        out.copy_(h)
    else:
        dist.reduce(out, dst=dst_g, op=dist.ReduceOp.SUM, group=group)
    return allr, best, out


def gather_rewards(rewards: torch.Tensor, group=None) -> torch.Tensor:
    """[P*B] rewards of every rank's candidates, in rank order (for logging a global batch)."""
    world = dist.get_world_size(group)
    out = torch.empty(world * rewards.numel(), dtype=rewards.dtype, device=rewards.device)
    return all_gather_into_(out, rewards.contiguous(), group)


# ---------------------------------------------------------------- slices split
def exchange_parts(xch: torch.Tensor, limbs: torch.Tensor, group=None) -> torch.Tensor:
    """The slices split's one collective, in place on the rollout workspace's exchange array
    (kernels.exchange_array: per-bucket weight sums and winner counts, each part non-zero on
    its own buckets only, then B * RES2_LIMBS caller slots): the lines' exact residual limbs
    [B, RES2_LIMBS] go into the slots and ONE all_reduce of the array's int64 bit patterns sums
    everything (a bucket entry has one non-zero term: its bits come through unchanged; the limbs
    add as integers).  Returns the summed limbs (a view of the slots)."""
    nl = limbs.numel()
    x64 = xch.view(torch.int64)
    slots = x64[x64.numel() - nl:].view_as(limbs)
    slots.copy_(limbs)
    all_reduce_(x64, group)
    return slots


def gather_slices(actions: torch.Tensor, fwd: torch.Tensor, bounds: torch.Tensor, T: int, group=None):
    """Full [B, T] trajectories from every rank's slice [bounds[b, 0], bounds[b, 1]) (the slices
    partition [0, T)): zero outside the slice, one all_reduce each (exact: one non-zero term)."""
    pos = torch.arange(T, device=actions.device).view(1, -1)
    mine = (pos >= bounds[:, :1]) & (pos < bounds[:, 1:])
    a = torch.where(mine, actions[:, :T], torch.zeros((), dtype=actions.dtype, device=actions.device)).contiguous()
    f = torch.where(mine, fwd[:, :T], torch.zeros((), dtype=fwd.dtype, device=fwd.device)).contiguous()
    all_reduce_(a, group)
    all_reduce_(f, group)
    return a, f
