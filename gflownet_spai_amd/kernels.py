"""Thin host wrappers over the C ABI (include/spai_hip.h) taking torch device tensors.

Each wrapper validates shapes on the host, allocates outputs with torch's caching
allocator on the current stream, and launches through ctypes.  No CPU fallback.
"""
from __future__ import annotations

import contextlib
import ctypes

import torch

from . import _lib
from .layout import Lines

_DT = {torch.float32: _lib.DTYPE_F32, torch.float64: _lib.DTYPE_F64}


def _l():
    return _lib.load()


# Optional per-launch HIP-event timing (bench.py): name -> list of (start, end) events,
# recorded on the stream the kernels are launched on (torch's current stream).
TIMERS: dict | None = None


@contextlib.contextmanager
def _timed(name: str):
    if TIMERS is None:
        yield
        return
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    yield
    e.record()
    TIMERS.setdefault(name, []).append((s, e))


def timer_ms(name: str) -> list:
    return [s.elapsed_time(e) for s, e in (TIMERS or {}).get(name, [])]


# single kernels inside the multi-kernel entry points (spai_kernel_timer_*): HIP events recorded
# by the library on the launch stream around each launch while armed (not under graph capture)
KERNEL_TIMERS = {"k_tile": 0, "k_sort2": 1, "k_qr_solve": 2, "k_gram_fill": 3}


def kernel_timers_available() -> bool:
    return hasattr(_l(), "spai_kernel_timer_arm")  # (absent from older variant libraries in A/B runs)


def kernel_timer_arm(on: bool, names=tuple(KERNEL_TIMERS)) -> None:
    for k in names:
        _lib.check(_l().spai_kernel_timer_arm(KERNEL_TIMERS[k], int(bool(on))), "spai_kernel_timer_arm")


def kernel_timer_read(names=tuple(KERNEL_TIMERS)) -> dict:
    """{kernel: (launches recorded, mean ms)} (waits for the recorded events)."""
    out = {}
    for k in names:
        cnt, ms = ctypes.c_int32(0), ctypes.c_double(0.0)
        _lib.check(_l().spai_kernel_timer_read(KERNEL_TIMERS[k], ctypes.byref(cnt), ctypes.byref(ms)),
                   "spai_kernel_timer_read")
        out[k] = (int(cnt.value), float(ms.value))
    return out


def logits_stats(logits: torch.Tensor, B: int):
    """lmax [B] fp32 and z [B] fp64 of logits [E+1] (shared) or [B, E+1]."""
    _lib.require_device(logits)
    shared = logits.dim() == 1
    lg = logits.contiguous().float()
    E1 = lg.shape[-1]
    lmax = torch.empty(B, dtype=torch.float32, device=lg.device)
    z = torch.empty(B, dtype=torch.float64, device=lg.device)
    nb = _l().spai_logits_stats_workspace_bytes(E1, B)
    ws = _lib.workspace(nb, lg.device, "stats")
    with _timed("logits_stats"):
        st = _l().spai_logits_stats(_lib.ptr(lg), 0 if shared else E1, E1, B, _lib.ptr(lmax), _lib.ptr(z),
                                      _lib.ptr(ws), ws.numel(), _lib.stream_ptr(lg.device))
    _lib.check(st, "spai_logits_stats")
    return lg, lmax, z


def parity_step(lg: torch.Tensor, B: int, noise: torch.Tensor, lmax, chosen, active, zrem):
    E1 = lg.shape[-1]
    out_a = torch.empty(B, dtype=torch.int64, device=lg.device)
    out_p = torch.empty(B, dtype=torch.float32, device=lg.device)
    noise = noise.to(lg.device, non_blocking=True).contiguous()
    if noise.shape != (B, E1):
        raise ValueError(f"noise shape {tuple(noise.shape)} != {(B, E1)}")
    nb = _l().spai_parity_step_workspace_bytes(E1, B)
    ws = _lib.workspace(nb, lg.device, "parity")
    _lib.check(_l().spai_parity_step(_lib.ptr(lg), 0 if lg.dim() == 1 else E1, E1, B, _lib.ptr(noise),
                                     _lib.ptr(lmax), _lib.ptr(chosen), chosen.shape[1], _lib.ptr(active),
                                     _lib.ptr(zrem), _lib.ptr(out_a), _lib.ptr(out_p), _lib.ptr(ws), ws.numel(),
                                     _lib.stream_ptr(lg.device)), "spai_parity_step")
    return out_a, out_p


def rollout_select(lg: torch.Tensor, B: int, lmax: torch.Tensor, seed: int, stream_id: int, sample_base: int = 0,
                   stream_ctr: torch.Tensor | None = None, part: int = 0, nparts: int = 1, ws_tag: str = "rollout",
                   out: torch.Tensor | None = None):
    """Phase 1 of the throughput rollout: removal bitmaps [B, ceil(E/32)] and counts [B] (for
    nparts > 1 the counts are written by rollout_merge, after the exchange).

    stream_ctr: optional device uint64 (int64 tensor) holding the Philox stream id, advanced
    by one on the device (graph replays draw fresh rollouts); part/nparts: this process orders
    buckets [nb*part/nparts, nb*(part+1)/nparts) of every sample (the slices split); out:
    optional int32 buffer [B * words + B] that receives the bitmaps, then the counts (the
    columns split gathers its all_to_all send buffer from it)."""
    _lib.require_device(lg)
    E = lg.shape[-1] - 1
    words = (E + 31) // 32
    if out is not None:
        if out.dtype != torch.int32 or out.numel() != B * words + B or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous int32 buffer of {B * words + B} elements")
        removed, counts = out[:B * words].view(B, words), out[B * words:]
    else:
        removed = torch.empty(B, words, dtype=torch.int32, device=lg.device)
        counts = torch.empty(B, dtype=torch.int32, device=lg.device)
    nb = _l().spai_rollout_workspace_bytes(E, B)
    if nb == 0:
        raise RuntimeError("spai_rollout_workspace_bytes failed: " + _l().spai_last_error().decode())
    ws = _lib.workspace(nb, lg.device, ws_tag)
    if stream_ctr is not None and (stream_ctr.dtype != torch.int64 or stream_ctr.numel() != 1 or
                                   stream_ctr.device != lg.device):
        raise ValueError("stream_ctr must be a 1-element int64 tensor on the logits' device")
    with _timed("rollout_select"):
        if isinstance(lmax, PendingMax):  # the policy's block maxima: reduced inside the select
            if lg.dim() != 1:
                raise ValueError("a deferred maximum needs one shared logits row")
            st = _l().spai_rollout_select_pm(_lib.ptr(lg), 0, E, B, _lib.ptr(lmax.out), _lib.ptr(lmax.parts),
                                             lmax.parts.numel(), seed & (2**64 - 1), stream_id & (2**64 - 1),
                                             _lib.ptr(stream_ctr), sample_base, part, nparts, _lib.ptr(removed),
                                             words, _lib.ptr(counts), _lib.ptr(ws), ws.numel(),
                                             _lib.stream_ptr(lg.device))
        else:
            st = _l().spai_rollout_select(_lib.ptr(lg), 0 if lg.dim() == 1 else E + 1, E, B, _lib.ptr(lmax),
                                          seed & (2**64 - 1), stream_id & (2**64 - 1), _lib.ptr(stream_ctr),
                                          sample_base, part, nparts, _lib.ptr(removed), words, _lib.ptr(counts),
                                          _lib.ptr(ws), ws.numel(), _lib.stream_ptr(lg.device))
    _lib.check(st, "spai_rollout_select")
    return removed, counts, ws


class PendingMax:
    """The logits' maximum not yet formed: ``parts`` holds the policy's fc block maxima
    (spai_policy_logits with B = 0) and rollout_select writes the maximum into ``out`` [B] inside its
    first launch (spai_rollout_select_pm) — one reduction launch fewer per step."""

    def __init__(self, out: torch.Tensor, parts: torch.Tensor):
        self.out, self.parts = out, parts


def rollout_order(lg, B, lmax, counts, ws):
    """Phase 2: ordered trajectories, no host round trip.

    Returns actions [B, E+1] int64 and fwd_probs [B, E+1] fp32 (only the first T columns
    are written) and T as a 1-element int32 device tensor."""
    E = lg.shape[-1] - 1
    actions = torch.empty(B, E + 1, dtype=torch.int64, device=lg.device)
    fwd = torch.empty(B, E + 1, dtype=torch.float32, device=lg.device)
    t_dev = torch.empty(1, dtype=torch.int32, device=lg.device)
    with _timed("rollout_order"):
        st = _l().spai_rollout_order(_lib.ptr(lg), 0 if lg.dim() == 1 else E + 1, E, B, _lib.ptr(lmax),
                                     _lib.ptr(counts), E + 1, _lib.ptr(actions), _lib.ptr(fwd), _lib.ptr(t_dev),
                                     _lib.ptr(ws), ws.numel(), _lib.stream_ptr(lg.device))
    _lib.check(st, "spai_rollout_order")
    return actions, fwd, t_dev


def exchange_array(ws: torch.Tensor, E: int, B: int) -> torch.Tensor:
    """fp64 view of the exchange array inside a rollout workspace: [B][2][kMaxB] bucket weight
    sums | winner counts (a part fills its own buckets, the rest are 0), then B * RES2_LIMBS
    slots the caller uses for the exact residual limbs.  The parts of a split rollout sum its
    int64 bit patterns (one all_reduce) before rollout_merge."""
    lib = _l()
    off, n = lib.spai_rollout_ws_offset(E, B, 2), lib.spai_rollout_ws_offset(E, B, 6)
    if off < 0 or n <= 0:
        raise ValueError("spai_rollout_ws_offset failed")
    return ws[off:off + n * 8].view(torch.float64)


def part_bounds(ws: torch.Tensor, E: int, B: int, part: int, nparts: int) -> torch.Tensor:
    """[B, 2] int64 trajectory slice [start, end) a part orders (device tensor, no sync; the last
    part's end is E + 1: it also writes the terminal step and the padding).  Valid after
    rollout_merge (or a one-part select)."""
    lib = _l()
    kmax = lib.spai_rollout_ws_offset(E, B, 3)
    o_bs, o_nb = lib.spai_rollout_ws_offset(E, B, 4), lib.spai_rollout_ws_offset(E, B, 5)
    bstart = ws[o_bs:o_bs + B * (kmax + 1) * 4].view(torch.int32).view(B, kmax + 1).long()
    nb = ws[o_nb:o_nb + B * 4].view(torch.int32).long()
    k0, k1 = (nb * part) // nparts, (nb * (part + 1)) // nparts
    start = bstart.gather(1, k0.view(B, 1))
    end = bstart.gather(1, k1.view(B, 1)) if part < nparts - 1 else torch.full_like(start, E + 1)
    return torch.cat([start, end], 1)


def _bstride(lg, E):
    return 0 if lg.dim() == 1 else E + 1


def rollout_merge(lg, B, lmax, ws, part: int, nparts: int, counts: torch.Tensor | None = None):
    """Split rollout, after the parts' exchange arrays are summed: counts [B], T, the bucket
    positions and the later-bucket masses.  Returns counts (int32 [B])."""
    E = lg.shape[-1] - 1
    if counts is None:
        counts = torch.empty(B, dtype=torch.int32, device=lg.device)
    with _timed("rollout_merge"):
        st = _l().spai_rollout_merge(_lib.ptr(lg), _bstride(lg, E), E, B, _lib.ptr(lmax), part, nparts,
                                     _lib.ptr(counts), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(lg.device))
    _lib.check(st, "spai_rollout_merge")
    return counts


def rollout_sort(lg, B, lmax, ws, part: int, nparts: int):
    """Sorts this part's buckets: actions [B, E+1] and fwd_probs [B, E+1] with the part's
    trajectory slice written (one-part select, or after rollout_merge)."""
    E = lg.shape[-1] - 1
    actions = torch.empty(B, E + 1, dtype=torch.int64, device=lg.device)
    fwd = torch.empty(B, E + 1, dtype=torch.float32, device=lg.device)
    with _timed("rollout_sort"):
        st = _l().spai_rollout_sort(_lib.ptr(lg), _bstride(lg, E), E, B, _lib.ptr(lmax), part, nparts, E + 1,
                                    _lib.ptr(actions), _lib.ptr(fwd), _lib.ptr(ws), ws.numel(),
                                    _lib.stream_ptr(lg.device))
    _lib.check(st, "spai_rollout_sort")
    return actions, fwd


def set_sort_blocks(blocks: int) -> None:
    """Persistent grid of the trajectory sort (spai_set_sort_blocks; 0 = one block per CU)."""
    _lib.check(_l().spai_set_sort_blocks(int(blocks)), "spai_set_sort_blocks")


def rollout_finish(lg, B, lmax, counts, ws, actions, fwd, part: int, nparts: int):
    """Terminal step and padding (last part) and T (int32 [1] device tensor)."""
    E = lg.shape[-1] - 1
    t_dev = torch.empty(1, dtype=torch.int32, device=lg.device)
    with _timed("rollout_finish"):
        st = _l().spai_rollout_finish(_lib.ptr(lg), _bstride(lg, E), E, B, _lib.ptr(lmax), _lib.ptr(counts), part,
                                      nparts, E + 1, _lib.ptr(actions), _lib.ptr(fwd), _lib.ptr(t_dev),
                                      _lib.ptr(ws), ws.numel(), _lib.stream_ptr(lg.device))
    _lib.check(st, "spai_rollout_finish")
    return t_dev


def narrow_values(a_lines: Lines) -> torch.Tensor:
    """A's values as the residual kernels read them: an fp64 A whose every value is exact in
    fp32 (stencils, integer-valued matrices) is handed over as fp32 — the same numbers, widened
    back exactly in the kernel, so every result keeps its bits — which halves the registers its
    13-wide lines take and lets k_resid_wide match a line's entry pairs once for 8 samples
    instead of 4.  Checked once per Lines object (one device->host sync) and cached on it."""
    v = a_lines.val
    if v.dtype != torch.float64:
        return v
    c = a_lines._narrow
    if c is None or c[0] is not v:
        f = v.float()
        c = (v, f if torch.equal(f.double(), v) else v)
        a_lines._narrow = c
    return c[1]


def residual_lines(m_idx: torch.Tensor, m_val: torch.Tensor, a_lines: Lines, line_begin: int = 0,
                   line_end: int | None = None, gram=None, pattern: Lines | None = None) -> torch.Tensor:
    """res2 [B] fp64 = sum over lines [begin, end) of ||sum_p M_b[l,p] A_line(idx_b[l,p]) - e_l||^2
    for B ARBITRARY sparse M_b in ELL lines: m_idx [B, n, W] or [n, W] (one index set for every
    sample) int32 with -1 = empty slot, m_val [B, n, W] fp32/fp64 (the generic SpMM residual of
    preconditioner.py:79-93; spai_residual_lines).

    ``gram`` (a CacheDict of ``pattern``'s Gram cache over these A lines: PreconditionerEnv keeps
    one for 13-wide patterns, kernels.cache_dict(env.gram, n) makes one of a 5/7-wide cache): lines
    whose index sets are slot-aligned sub-patterns of ``pattern`` take G, c from it instead of
    matching A (spai_residual_lines_gram; the same bits). Other widths and dtypes run the matching
    kernel."""
    _lib.require_device(m_val)
    if m_val.dim() == 2:
        m_val = m_val.unsqueeze(0)
    B, n, W = m_val.shape
    if line_end is None:
        line_end = n
    if m_val.dtype not in _DT or a_lines.val.dtype not in _DT:
        raise ValueError("M and A must be fp32 or fp64")
    m_idx = m_idx.to(torch.int32).contiguous()
    m_val = m_val.contiguous()
    if m_idx.shape[-2:] != (n, W) or (m_idx.dim() == 3 and m_idx.shape[0] != B):
        raise ValueError(f"m_idx shape {tuple(m_idx.shape)} does not match m_val {tuple(m_val.shape)}")
    a_val = narrow_values(a_lines)
    res2 = torch.empty(B, dtype=torch.float64, device=m_val.device)
    nb = _l().spai_residual_workspace_bytes(max(line_end - line_begin, 0), B)
    ws = _lib.workspace(nb, m_val.device, "residual")
    use_gram = (isinstance(gram, CacheDict) and pattern is not None and pattern.width == W and pattern.n == n
                and (W, a_lines.width) in ((5, 5), (5, 4), (5, 3), (7, 7), (7, 6), (7, 5), (13, 7), (13, 6), (13, 5))
                and a_val.dtype == torch.float32)
    with _timed("residual_lines"):
        if use_gram:
            st = _l().spai_residual_lines_gram(n, line_begin, line_end, W, _lib.ptr(m_idx),
                                               n * W if m_idx.dim() == 3 else 0, _lib.ptr(m_val), _DT[m_val.dtype],
                                               n * W, a_lines.width, _lib.ptr(a_lines.idx), _lib.ptr(a_val),
                                               _DT[a_val.dtype], _lib.ptr(pattern.idx), _lib.ptr(gram.table),
                                               _DT[gram.dtype], _lib.ptr(gram.entry), B, _lib.ptr(res2),
                                               _lib.ptr(ws), ws.numel(), _lib.stream_ptr(m_val.device))
        else:
            st = _l().spai_residual_lines(n, line_begin, line_end, W, _lib.ptr(m_idx),
                                          n * W if m_idx.dim() == 3 else 0, _lib.ptr(m_val), _DT[m_val.dtype], n * W,
                                          a_lines.width, _lib.ptr(a_lines.idx), _lib.ptr(a_val), _DT[a_val.dtype], B,
                                          _lib.ptr(res2), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(m_val.device))
    _lib.check(st, "spai_residual_lines_gram" if use_gram else "spai_residual_lines")
    return res2


def actions_to_removed(actions_bt: torch.Tensor, E: int):
    """Removal bitmaps + unique counts from a [B, T] int64 action tensor (-1 padded)."""
    _lib.require_device(actions_bt)
    a = actions_bt.to(torch.int64)
    B, T = a.shape
    words = (E + 31) // 32
    removed = torch.empty(B, words, dtype=torch.int32, device=a.device)
    counts = torch.empty(B, dtype=torch.int32, device=a.device)
    _lib.check(_l().spai_actions_to_removed(_lib.ptr(a), a.stride(0), a.stride(1), B, T, E, _lib.ptr(removed),
                                            words, _lib.ptr(counts), _lib.stream_ptr(a.device)),
               "spai_actions_to_removed")
    return removed, counts


def _fill_out(B: int, device, limbs: bool):
    if limbs:
        return None, torch.empty(B, _lib.RES2_LIMBS, dtype=torch.int64, device=device)
    return torch.empty(B, dtype=torch.float64, device=device), None


def fill_residual(pattern: Lines, a_lines: Lines, removed: torch.Tensor, lsq: bool, line_begin: int = 0,
                  line_end: int | None = None, store_m: bool = False, m_dtype=torch.float32, word_base: int = 0,
                  limbs: bool = False):
    """(res2 [B] fp64 = sum over lines [begin, end) of ||line residual||^2, or with ``limbs`` the
    exact sums [B, RES2_LIMBS] int64 to be summed across line shards; M values or None).
    ``removed`` [B, words]: row b holds bitmap words word_base .. word_base + words - 1 of sample b."""
    _lib.require_device(removed)
    if line_end is None:
        line_end = pattern.n
    removed = removed.contiguous()
    B, words = removed.shape
    if a_lines.val.dtype not in _DT:
        raise ValueError(f"A dtype {a_lines.val.dtype} not supported (fp32/fp64)")
    mode = _lib.FILL_LSQ if lsq else _lib.FILL_COPY
    if not lsq:
        m_dtype = torch.float32
    n_loc = line_end - line_begin
    res2, lb = _fill_out(B, removed.device, limbs)
    m = torch.empty(B, n_loc, pattern.width, dtype=m_dtype, device=removed.device) if store_m else None
    nb = _l().spai_fill_workspace_bytes(max(n_loc, 1), B)
    ws = _lib.workspace(nb, removed.device, "fill")
    with _timed("fill_residual"):
        st = _l().spai_fill_residual(mode, pattern.n, line_begin, line_end, pattern.width, _lib.ptr(pattern.idx),
                                       _lib.ptr(pattern.act), _lib.ptr(pattern.val), a_lines.width,
                                       _lib.ptr(a_lines.idx), _lib.ptr(a_lines.val), _DT[a_lines.val.dtype], B,
                                       _lib.ptr(removed), words, word_base, _lib.ptr(m), _DT[m_dtype], _lib.ptr(res2),
                                       _lib.ptr(lb), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(removed.device))
    _lib.check(st, "spai_fill_residual")
    return (lb if limbs else res2), m


def gram_build(pattern: Lines, a_lines: Lines) -> torch.Tensor:
    """Per-line Gram cache (fp64 [T + Wc, n]) of the LSQ fill / residual: built once per env."""
    _lib.require_device(pattern.idx)
    nb = _l().spai_gram_bytes(pattern.n, pattern.width)
    if nb == 0:
        raise NotImplementedError(f"no Gram kernel for width {pattern.width}")
    # zeroed: the padding lines of the last 64-line block stay exactly 0 (spai_gram_compact checks every entry)
    gram = torch.zeros(nb // 8, dtype=torch.float64, device=pattern.idx.device)
    _lib.check(_l().spai_gram_build(pattern.n, pattern.width, _lib.ptr(pattern.idx), a_lines.width,
                                    _lib.ptr(a_lines.idx), _lib.ptr(a_lines.val), _DT[a_lines.val.dtype],
                                    _lib.ptr(gram), _lib.stream_ptr(pattern.idx.device)), "spai_gram_build")
    return gram


def gram_compact(gram: torch.Tensor, pattern: Lines):
    """fp32 copy of an fp64 Gram cache if every entry survives the round trip exactly (then the
    fill is bit-identical from it and streams half the Gram bytes), else None.  One host sync
    (once per env)."""
    if pattern.width > 13:
        return None
    g32 = torch.empty(gram.numel(), dtype=torch.float32, device=gram.device)
    exact = torch.ones(1, dtype=torch.int32, device=gram.device)
    _lib.check(_l().spai_gram_compact(pattern.n, pattern.width, _lib.ptr(gram), _lib.ptr(g32), _lib.ptr(exact),
                                      _lib.stream_ptr(gram.device)), "spai_gram_compact")
    return g32 if int(exact.item()) == 1 else None


def _fill_lines_gram(mode, pattern: Lines, gram, line_begin: int, line_end: int, removed, word_base: int, m, m_dtype,
                     ws):
    """spai_fill_lines_gram from the full Gram cache, spai_fill_lines_gram_dict from its CacheDict."""
    B, words = removed.shape
    if isinstance(gram, CacheDict):
        st = _l().spai_fill_lines_gram_dict(mode, pattern.n, line_begin, line_end, pattern.width,
                                            _lib.ptr(pattern.act), _lib.ptr(pattern.val), _lib.ptr(gram.table),
                                            _DT[gram.dtype], _lib.ptr(gram.entry), B, _lib.ptr(removed), words,
                                            word_base, _lib.ptr(m), _DT[m_dtype], _lib.ptr(ws), ws.numel(),
                                            _lib.stream_ptr(removed.device))
    else:
        st = _l().spai_fill_lines_gram(mode, pattern.n, line_begin, line_end, pattern.width, _lib.ptr(pattern.act),
                                       _lib.ptr(pattern.val), _lib.ptr(gram), _DT[gram.dtype], B, _lib.ptr(removed),
                                       words, word_base, _lib.ptr(m), _DT[m_dtype], _lib.ptr(ws), ws.numel(),
                                       _lib.stream_ptr(removed.device))
    _lib.check(st, "spai_fill_lines_gram")


def fill_residual_gram(pattern: Lines, gram, removed: torch.Tensor, lsq: bool, line_begin: int = 0,
                       line_end: int | None = None, store_m: bool = False, m_dtype=torch.float32, word_base: int = 0,
                       limbs: bool = False):
    """fill_residual from the env's Gram cache (same outputs)."""
    _lib.require_device(removed)
    if line_end is None:
        line_end = pattern.n
    removed = removed.contiguous()
    B, words = removed.shape
    mode = _lib.FILL_LSQ if lsq else _lib.FILL_COPY
    if not lsq:
        m_dtype = torch.float32
    n_loc = line_end - line_begin
    res2, lb = _fill_out(B, removed.device, limbs)
    m = torch.empty(B, n_loc, pattern.width, dtype=m_dtype, device=removed.device) if store_m else None
    nb = _l().spai_fill_workspace_bytes(max(n_loc, 1), B)
    ws = _lib.workspace(nb, removed.device, "fill")
    with _timed("fill_residual"):  # the fill kernel alone (the bench's roofline kernel)
        _fill_lines_gram(mode, pattern, gram, line_begin, line_end, removed, word_base, m, m_dtype, ws)
    _lib.check(_l().spai_fill_reduce(n_loc, B, _lib.ptr(ws), _lib.ptr(res2), _lib.ptr(lb),
                                     _lib.stream_ptr(removed.device)), "spai_fill_reduce")
    return (lb if limbs else res2), m


def qr_max_rows(pattern: Lines, a_lines: Lines) -> int:
    """Largest row union |I| over the lines (the dense block A[I, slots] the QR fill factors);
    one host sync (once per env).  spai_qr_max_rows."""
    _lib.require_device(pattern.idx)
    out = torch.empty(1, dtype=torch.int32, device=pattern.idx.device)
    _lib.check(_l().spai_qr_max_rows(pattern.n, pattern.width, _lib.ptr(pattern.idx), a_lines.width,
                                     _lib.ptr(a_lines.idx), _lib.ptr(out), _lib.stream_ptr(pattern.idx.device)),
               "spai_qr_max_rows")
    return int(out.item())


def qr_cache(pattern: Lines, a_lines: Lines, max_rows: int):
    """The R cache of the QR fill (spai_qr_factor): per line the Householder R of its full block
    A[I, slots], Q^T e_l and the tail, fp64, built once per env (pattern widths <= 13 over A
    widths <= 7; the 13-wide solve re-reads its line's R per sample at one wave per SIMD).  None
    for wider lines (the fused spai_fill_lines_qr runs instead)."""
    _lib.require_device(pattern.idx)
    lib = _l()
    nb = lib.spai_qr_cache_bytes(pattern.n, pattern.width, a_lines.width)
    if nb == 0 or not (pattern.width <= 13 and a_lines.width <= 7):
        return None
    rc = torch.zeros(nb // 8, dtype=torch.float64, device=pattern.idx.device)
    av = narrow_values(a_lines)
    _lib.check(lib.spai_qr_factor(pattern.n, pattern.width, _lib.ptr(pattern.idx), _lib.ptr(pattern.act),
                                  a_lines.width, _lib.ptr(a_lines.idx), _lib.ptr(av), _DT[av.dtype], max_rows,
                                  _lib.ptr(rc), nb, _lib.stream_ptr(pattern.idx.device)), "spai_qr_factor")
    return rc


class CacheDict:
    """A per-line cache (the R cache, the Gram cache) held as its dictionary (spai_line_cache_dict):
    the distinct line entries ``table`` [entries * nq] and each line's entry ``entry`` [n] int32.
    Accepted wherever the full cache is."""

    def __init__(self, table: torch.Tensor, entry: torch.Tensor, entries: int):
        self.table, self.entry, self.entries = table, entry, entries

    @property
    def dtype(self):
        return self.table.dtype

    @property
    def nbytes(self) -> int:
        return self.table.numel() * self.table.element_size() + self.entry.numel() * self.entry.element_size()


QrDict = CacheDict  # (the R cache's dictionary)


def qr_class(W: int, WA: int) -> int:
    """Width class of the QR fill (qr.hip qr_class): 5, 7 or 13."""
    if W <= 5 and WA <= 5:
        return 5
    if W <= 7 and WA <= 7:
        return 7
    return 13


def qr_cache_q(wc: int) -> int:
    """Values per line of the R cache of width class wc: packed R, Q^T e, tail (qr.hip qr_cache_q)."""
    return wc * (wc + 1) // 2 + wc + 1


def qr_table_offset(n_lines: int, B: int) -> int:
    """Byte offset of spai_fill_lines_qr_cached's (entry, mask) table in its workspace."""
    return ((n_lines + 255) // 256 * B * 8 + 255) // 256 * 256


def cache_nbytes(cache) -> int:
    """Bytes one rollout's fill reads of a per-line cache (full tensor or CacheDict)."""
    return cache.nbytes if isinstance(cache, CacheDict) else cache.numel() * cache.element_size()


rcache_nbytes = cache_nbytes


def cache_dict(cache: torch.Tensor, n: int, max_frac: float = 0.25):
    """A per-line cache in the blocked layout ([ceil(n/64)][nq][64]) as a CacheDict when its lines
    have at most max_frac * n distinct entries (a stencil's interior lines share one: the same A
    values in the same relative positions give the same cached values bit for bit), else None
    (keep the full cache).  Env setup: one host round trip."""
    lib = _l()
    es = cache.element_size()
    nq = cache.numel() // ((n + 63) // 64 * 64)
    cap = max(1, int(n * max_frac))
    table = torch.empty(cap * nq, dtype=cache.dtype, device=cache.device)
    entry = torch.empty(n, dtype=torch.int32, device=cache.device)
    cnt = ctypes.c_int32(0)
    _lib.check(lib.spai_line_cache_dict(n, nq, es, _lib.ptr(cache), cache.numel() * es, cap, _lib.ptr(table),
                                        table.numel() * es, _lib.ptr(entry), ctypes.byref(cnt),
                                        _lib.stream_ptr(cache.device)), "spai_line_cache_dict")
    if cnt.value > cap:
        return None
    return CacheDict(table[:cnt.value * nq].clone(), entry, cnt.value)


def qr_dict(rcache: torch.Tensor, pattern: Lines, a_lines: Lines | None = None, max_frac: float = 0.25):
    """The R cache as a CacheDict, or None (cache_dict)."""
    return cache_dict(rcache, pattern.n, max_frac)


def _fill_lines_qr(pattern: Lines, a_lines: Lines, max_rows: int, removed: torch.Tensor, line_begin: int,
                   line_end: int, m, m_dtype, word_base: int, ws, rcache=None):
    B, words = removed.shape
    if rcache is not None:  # phase 2 only, from the env's R cache (full, or its dictionary)
        if isinstance(rcache, QrDict):
            nq = qr_cache_q(qr_class(pattern.width, a_lines.width))
            if rcache.table.dtype != torch.float64 or rcache.table.numel() != rcache.entries * nq:
                raise ValueError(f"the R cache dictionary holds {rcache.table.numel()} fp64 values, not "
                                 f"{rcache.entries} entries x {nq} (a Gram cache dictionary passed as an R cache?)")
            tab, ent, n_ent = rcache.table, rcache.entry, rcache.entries
        else:
            tab, ent, n_ent = rcache, None, 0
        with _timed("fill_residual"):  # the fill kernel alone
            st = _l().spai_fill_lines_qr_cached(pattern.n, line_begin, line_end, pattern.width, a_lines.width,
                                                _lib.ptr(pattern.act), _lib.ptr(tab), _lib.ptr(ent), n_ent, B,
                                                _lib.ptr(removed), words, word_base, _lib.ptr(m), _DT[m_dtype],
                                                _lib.ptr(ws), ws.numel(), _lib.stream_ptr(removed.device))
        _lib.check(st, "spai_fill_lines_qr_cached")
        return
    av = narrow_values(a_lines)  # fp32-exact A values are staged as fp32 (the same numbers)
    with _timed("fill_residual"):  # the fill kernel alone
        st = _l().spai_fill_lines_qr(pattern.n, line_begin, line_end, pattern.width, _lib.ptr(pattern.idx),
                                     _lib.ptr(pattern.act), a_lines.width, _lib.ptr(a_lines.idx), _lib.ptr(av),
                                     _DT[av.dtype], max_rows, B, _lib.ptr(removed), words, word_base, _lib.ptr(m),
                                     _DT[m_dtype], _lib.ptr(ws), ws.numel(), _lib.stream_ptr(removed.device))
    _lib.check(st, "spai_fill_lines_qr")


def fill_residual_qr(pattern: Lines, a_lines: Lines, max_rows: int, removed: torch.Tensor, line_begin: int = 0,
                     line_end: int | None = None, store_m: bool = False, m_dtype=torch.float64, word_base: int = 0,
                     limbs: bool = False, rcache=None):
    """The least-squares fill by Householder QR (spai_fill_lines_qr, or spai_fill_lines_qr_cached from
    an R cache, + spai_fill_reduce): same outputs as fill_residual with lsq=True (res2 [B] or exact
    limbs, M or None)."""
    _lib.require_device(removed)
    if line_end is None:
        line_end = pattern.n
    removed = removed.contiguous()
    B = removed.shape[0]
    n_loc = line_end - line_begin
    res2, lb = _fill_out(B, removed.device, limbs)
    m = torch.empty(B, n_loc, pattern.width, dtype=m_dtype, device=removed.device) if store_m else None
    nb = _l().spai_fill_workspace_bytes(max(n_loc, 1), B)
    if isinstance(rcache, QrDict):  # room for the cached fill's (entry, mask) table after the partials
        nb = max(nb, qr_table_offset(n_loc, B) + rcache.entries * 32 * 6 * 8)
    ws = _lib.workspace(nb, removed.device, "fill")
    _fill_lines_qr(pattern, a_lines, max_rows, removed, line_begin, line_end, m, m_dtype, word_base, ws, rcache)
    _lib.check(_l().spai_fill_reduce(n_loc, B, _lib.ptr(ws), _lib.ptr(res2), _lib.ptr(lb),
                                     _lib.stream_ptr(removed.device)), "spai_fill_reduce")
    return (lb if limbs else res2), m


def bitmap_pack(removed: torch.Tensor, counts: torch.Tensor, plan, out: torch.Tensor | None = None) -> torch.Tensor:
    """The columns split's all_to_all send buffer (spai_bitmap_pack): per destination q of
    ``plan`` (distributed.PackPlan) and candidate b, b's removal bits of q's line-major action ids
    packed 32 per word (or, plan.mode "window", spai_window_pack: q's contiguous word window), then
    counts[b]; int32 [plan.send_words(bl)]."""
    _lib.require_device(removed)
    bl, words = removed.shape
    off, total = plan.out_off(bl)
    if out is None:
        out = torch.empty(total, dtype=torch.int32, device=removed.device)
    if out.numel() != total or out.dtype != torch.int32 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous int32 buffer of {total} words")
    if removed.stride(1) != 1 or counts.dtype != torch.int32:
        raise ValueError("removed rows must be contiguous and counts int32")
    if plan.mode == "window" and max(lo + w for lo, w in zip(plan.lo_words, plan.wq)) > words:
        raise ValueError("the plan's word windows exceed the bitmap rows")
    with _timed("bitmap_pack"):
        if plan.mode == "window":  # contiguous word windows (spai_window_pack)
            st = _l().spai_window_pack(plan.world, bl, _lib.ptr(removed), removed.stride(0), _lib.ptr(counts),
                                       _lib.ptr(plan.lo), _lib.ptr(plan.span), _lib.ptr(off), plan.max_span,
                                       _lib.ptr(out), _lib.stream_ptr(removed.device))
        else:
            st = _l().spai_bitmap_pack(plan.world, bl, _lib.ptr(removed), removed.stride(0), _lib.ptr(counts),
                                       _lib.ptr(plan.ids), _lib.ptr(plan.seg), _lib.ptr(off), plan.max_seg,
                                       _lib.ptr(out), _lib.stream_ptr(removed.device))
    _lib.check(st, "spai_bitmap_pack" if plan.mode != "window" else "spai_window_pack")
    return out


def res2_from_limbs(limbs: torch.Tensor) -> torch.Tensor:
    """[B] fp64 squared residuals from exact sums [B, RES2_LIMBS] int64 (spai_res2_from_limbs)."""
    _lib.require_device(limbs)
    if limbs.dtype != torch.int64 or limbs.dim() != 2 or limbs.shape[1] != _lib.RES2_LIMBS:
        raise ValueError(f"limbs must be int64 [B, {_lib.RES2_LIMBS}]")
    limbs = limbs.contiguous()
    out = torch.empty(limbs.shape[0], dtype=torch.float64, device=limbs.device)
    _lib.check(_l().spai_res2_from_limbs(limbs.shape[0], _lib.ptr(limbs), _lib.ptr(out),
                                         _lib.stream_ptr(limbs.device)), "spai_res2_from_limbs")
    return out


def _reward_args(counts, alpha):
    return counts.to(torch.int32).contiguous(), alpha.detach().to(device=counts.device, dtype=torch.float32).reshape(1)


def rewards(res2: torch.Tensor, counts: torch.Tensor, nnz0: int, n: int, r0: float, f0: int, alpha: torch.Tensor):
    """(residual [B] fp64, reward [B] fp64, reward [B] fp32) with the reference's reward formula
    and type promotion (spai_rewards)."""
    B = res2.numel()
    c, a = _reward_args(counts, alpha)
    residual = torch.empty(B, dtype=torch.float64, device=res2.device)
    reward = torch.empty(B, dtype=torch.float64, device=res2.device)
    reward32 = torch.empty(B, dtype=torch.float32, device=res2.device)
    with _timed("rewards"):
        st = _l().spai_rewards(_lib.ptr(res2), _lib.ptr(c), B, nnz0, n, float(r0), float(f0), _lib.ptr(a),
                               _lib.ptr(residual), _lib.ptr(reward), _lib.ptr(reward32), _lib.stream_ptr(res2.device))
    _lib.check(st, "spai_rewards")
    return residual, reward, reward32


def fill_rewards_gram(pattern: Lines, gram, removed: torch.Tensor, lsq: bool, counts: torch.Tensor,
                      nnz0: int, r0: float, f0: int, alpha: torch.Tensor, store_m: bool = False,
                      m_dtype=torch.float32):
    """One GPU, all lines: the Gram-cached fill, then the exact residual sums and the rewards in
    one launch (spai_fill_lines_gram + spai_fill_reduce_rewards).  Returns (residual, reward,
    reward fp32, M or None)."""
    _lib.require_device(removed)
    removed = removed.contiguous()
    B, words = removed.shape
    n = pattern.n
    mode = _lib.FILL_LSQ if lsq else _lib.FILL_COPY
    if not lsq:
        m_dtype = torch.float32
    m = torch.empty(B, n, pattern.width, dtype=m_dtype, device=removed.device) if store_m else None
    ws = _lib.workspace(_l().spai_fill_workspace_bytes(n, B), removed.device, "fill")
    with _timed("fill_residual"):  # the fill kernel alone (the bench's roofline kernel)
        _fill_lines_gram(mode, pattern, gram, 0, n, removed, 0, m, m_dtype, ws)
    return _reduce_rewards(ws, n, B, counts, nnz0, r0, f0, alpha, removed.device) + (m,)


def _reduce_rewards(ws, n, B, counts, nnz0, r0, f0, alpha, device):
    """Exact residual sums of a whole-matrix fill's partials + the reward formula, one launch."""
    c, a = _reward_args(counts, alpha)
    residual = torch.empty(B, dtype=torch.float64, device=device)
    reward = torch.empty(B, dtype=torch.float64, device=device)
    reward32 = torch.empty(B, dtype=torch.float32, device=device)
    _lib.check(_l().spai_fill_reduce_rewards(n, B, _lib.ptr(ws), _lib.ptr(c), nnz0, n, float(r0), float(f0),
                                             _lib.ptr(a), _lib.ptr(residual), _lib.ptr(reward), _lib.ptr(reward32),
                                             _lib.stream_ptr(device)), "spai_fill_reduce_rewards")
    return residual, reward, reward32


def fill_rewards_qr(pattern: Lines, a_lines: Lines, max_rows: int, removed: torch.Tensor, counts: torch.Tensor,
                    nnz0: int, r0: float, f0: int, alpha: torch.Tensor, store_m: bool = False,
                    m_dtype=torch.float64, rcache=None):
    """fill_rewards_gram with the Householder-QR fill (spai_fill_lines_qr[_cached] + spai_fill_reduce_rewards)."""
    _lib.require_device(removed)
    removed = removed.contiguous()
    B = removed.shape[0]
    n = pattern.n
    m = torch.empty(B, n, pattern.width, dtype=m_dtype, device=removed.device) if store_m else None
    nb = _l().spai_fill_workspace_bytes(n, B)
    if isinstance(rcache, QrDict):  # room for the cached fill's (entry, mask) table after the partials
        nb = max(nb, qr_table_offset(n, B) + rcache.entries * 32 * 6 * 8)
    ws = _lib.workspace(nb, removed.device, "fill")
    _fill_lines_qr(pattern, a_lines, max_rows, removed, 0, n, m, m_dtype, 0, ws, rcache)
    return _reduce_rewards(ws, n, B, counts, nnz0, r0, f0, alpha, removed.device) + (m,)


def logp_grad(logits: torch.Tensor, lmax: torch.Tensor, actions_bt: torch.Tensor, probs_bt: torch.Tensor,
              gprobs_bt: torch.Tensor, removed: torch.Tensor) -> torch.Tensor:
    """dL/dlogits from dL/dprobs of a rollout's logged forward probabilities (spai_logp_grad).

    logits [E+1] or [1, E+1] (shared: the gradient is summed over the samples) or [B, E+1];
    actions/probs/gprobs [B, T] (row stride may exceed T); removed [B, ceil(E/32)]."""
    _lib.require_device(logits)
    E1 = logits.shape[-1]
    E = E1 - 1
    B, T = actions_bt.shape
    shared = logits.dim() == 1 or logits.shape[0] == 1
    lg = logits.detach().float()
    lg = lg.reshape(-1).contiguous() if shared else lg.contiguous()
    if not shared and lg.shape[0] != B:
        raise ValueError(f"per-sample logits {tuple(logits.shape)} for B={B}")

    def rows(t, dt):
        t = t.detach().to(dt)
        return t if t.stride(1) == 1 and t.stride(0) >= T else t.contiguous()

    a, p, g = rows(actions_bt, torch.int64), rows(probs_bt, torch.float32), rows(gprobs_bt, torch.float32)
    if removed.shape[0] != B or p.shape != (B, T) or g.shape != (B, T):
        raise ValueError("logp_grad: shapes of actions / probs / gprobs / removed disagree")
    lm = lmax.detach().float().reshape(-1).expand(B).contiguous() if lmax.numel() == 1 else lmax.float().contiguous()
    out = torch.empty(E1 if shared else (B, E1), dtype=torch.float32, device=lg.device)
    nb = _l().spai_logp_grad_workspace_bytes(E, T, B, 0 if shared else 1)
    ws = _lib.workspace(nb, lg.device, "logp_grad")
    st = _l().spai_logp_grad(_lib.ptr(lg), 0 if shared else E1, E, B, _lib.ptr(lm), _lib.ptr(a), a.stride(0), T,
                             _lib.ptr(p), p.stride(0), _lib.ptr(g), g.stride(0), _lib.ptr(removed), removed.shape[1],
                             _lib.ptr(out), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(lg.device))
    _lib.check(st, "spai_logp_grad")
    return out.view_as(logits) if shared else out


def _lstm_params(w_ih, w_hh, b_ih, b_hh):
    H = w_hh.shape[1]
    if w_ih.shape != (4 * H, 1) or w_hh.shape != (4 * H, H) or b_ih.shape != (4 * H,) or b_hh.shape != (4 * H,):
        raise ValueError("LSTM parameters must be input_dim=1: w_ih [4H,1], w_hh [4H,H], b_ih/b_hh [4H]")
    return H, [t.detach().float().contiguous() for t in (w_ih, w_hh, b_ih, b_hh)]


def lstm_forward(traj: torch.Tensor, lengths: torch.Tensor, w_ih, w_hh, b_ih, b_hh, keep_states: bool = False):
    """(h_last [B, H], states or None) of nn.LSTM(1, H) over each row's first lengths[b] ids; states
    is the flat buffer spai_lstm_backward reads (per-step (h, c), or 16-step checkpoints for H = 4)."""
    _lib.require_device(traj)
    H, ps = _lstm_params(w_ih, w_hh, b_ih, b_hh)
    tr = traj if traj.dtype == torch.int64 and traj.stride(1) == 1 else traj.to(torch.int64).contiguous()
    B, T = tr.shape
    n = lengths.to(device=tr.device, dtype=torch.int32).contiguous()
    h = torch.empty(B, H, dtype=torch.float32, device=tr.device)
    states = (torch.empty(_l().spai_lstm_states_floats(B, H, T), dtype=torch.float32, device=tr.device)
              if keep_states else None)
    with _timed("lstm_forward"):
        st = _l().spai_lstm_forward(B, H, _lib.ptr(tr), tr.stride(0), _lib.ptr(n), T, *[_lib.ptr(p) for p in ps],
                                    _lib.ptr(h), _lib.ptr(states), _lib.stream_ptr(tr.device))
    _lib.check(st, "spai_lstm_forward")
    return h, states


def lstm_backward(traj: torch.Tensor, lengths: torch.Tensor, w_ih, w_hh, b_ih, b_hh, states: torch.Tensor,
                  dh_last: torch.Tensor):
    """Per-sample fp64 gradient rows [B, 4H + 4H*H + 4H] (d w_ih | d w_hh | d bias) by BPTT."""
    H, ps = _lstm_params(w_ih, w_hh, b_ih, b_hh)
    tr = traj if traj.dtype == torch.int64 and traj.stride(1) == 1 else traj.to(torch.int64).contiguous()
    B, T = tr.shape
    if states is None or states.numel() != _l().spai_lstm_states_floats(B, H, T):
        raise ValueError("lstm_backward needs the states buffer of lstm_forward(keep_states=True) for this B, H, T")
    n = lengths.to(device=tr.device, dtype=torch.int32).contiguous()
    dh = dh_last.detach().float().contiguous()
    g = torch.empty(B, 8 * H + 4 * H * H, dtype=torch.float64, device=tr.device)
    nws = _l().spai_lstm_backward_workspace_bytes(B, H, T)
    ws = _lib.workspace(nws, tr.device, "lstm_backward") if nws else None
    with _timed("lstm_backward"):
        st = _l().spai_lstm_backward(B, H, _lib.ptr(tr), tr.stride(0), _lib.ptr(n), T, *[_lib.ptr(p) for p in ps],
                                     _lib.ptr(states), _lib.ptr(dh), _lib.ptr(g), _lib.ptr(ws), nws,
                                     _lib.stream_ptr(tr.device))
    _lib.check(st, "spai_lstm_backward")
    return g
