"""Drop-in ``PreconditionerEnv`` (reference: preconditioner.py:11-165) on the MI355X path.

Same constructor, attributes and methods as the reference; the work behind
``update`` / ``calculate_residual`` runs in libspai_hip.so:

  reference (per sample, Python)                 here (all samples, one launch each)
  ------------------------------------------     --------------------------------------------
  keep-list list-comp over E   utils.py:323      spai_actions_to_removed  -> removal bitmaps
  COO rebuild + 2x coalesce    utils.py:343-353  (none: M = shared pattern lines + bitmap)
                               utils.py:115-124
  torch.mm(M, A) SpGEMM        preconditioner:88 spai_fill_residual -> ||M A - I||_F^2 per sample
  sparse sub + norm            preconditioner:90   (fp64, never materialises M A)
  reward formula               preconditioner:137-165, 55-66  (torch ops, same type promotion)

Extensions (keyword-only, defaults = reference behaviour):
  side="MA" | "AM"    which residual: ||M A - I|| (reference) or ||A M - I|| (column SPAI)
  fill="copy" | "lsq" | "qr"  M = copied pattern values (reference) or per-line least squares:
                      "lsq" by the normal equations of the Gram cache (the bench path), "qr" by
                      Householder QR of each line's dense block A[I, J] (spai_fill_lines_qr)
  keep_m=False        keep the last batch's M values (LSQ) in ``self.last_m``
  rcache=True         fill="qr": factor every line's full block once per env (spai_qr_factor) and
                      solve each rollout's masked problems from that R cache; False: the fused
                      kernel refactors every call
  cache_dict=True     keep the Gram / R cache as its dictionary (kernels.CacheDict,
                      spai_line_cache_dict) when at most a quarter of the lines have distinct
                      entries — a stencil's interior lines share one: the same bits from fewer
                      HBM bytes (and two waves per SIMD for the 8-13-wide Gram fill; the
                      5/7-wide Gram fill keeps its full cache: no gain measured)
Documented deviations: alpha is taken from the ``alpha`` argument (the reference reads
the never-set ``self.alpha``, preconditioner.py:163); fp64 original matrices are
accepted (the reference raises in torch.mm, utils.py:350); a raw COO pattern with
duplicate entries raises ValueError (the reference's action ids are inconsistent then).
"""
from __future__ import annotations

from typing import List, Tuple

import torch
from torch import Tensor

from . import kernels
from .env import Env
from .layout import Lines, build_lines, lines_to_coo, raw_coo


class Data:
    """Keyword attribute bag standing in for torch_geometric.data.Data (preconditioner.py:25)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def __contains__(self, k):
        return k in self.__dict__


def _default_device():
    if not torch.cuda.is_available():
        raise RuntimeError("PreconditionerEnv needs an MI355X (no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


class PreconditionerEnv(Env):
    def __init__(self, matrix_size: int, initial_matrix: Tensor, original_matrix: Tensor, *, side: str = "MA",
                 fill: str = "copy", keep_m: bool = False, device=None, compact_gram: bool = True,
                 rcache: bool = True, cache_dict: bool = True):
        if side not in ("MA", "AM"):
            raise ValueError("side must be 'MA' or 'AM'")
        if fill not in ("copy", "lsq", "qr"):
            raise ValueError("fill must be 'copy', 'lsq' or 'qr'")
        self.device = torch.device(device) if device is not None else _default_device()
        self.side, self.fill, self.keep_m = side, fill, keep_m
        self._lsq = fill in ("lsq", "qr")  # M holds fitted values (not the pattern's)
        self.matrix_size = matrix_size
        self.init_nnz = initial_matrix.coalesce().indices().size(1)
        self.state_dim = self.init_nnz
        self.num_actions = self.init_nnz + 1
        self.matrix = initial_matrix.clone()
        self.original_matrix = original_matrix.clone()
        edge_index = self.matrix._indices()
        edge_attr = self.matrix._values()
        self.data = Data(edge_index=edge_index, edge_attr=edge_attr.float())

        orient = "row" if side == "MA" else "col"
        r, c, v = raw_coo(self.matrix)
        if r.numel() != self.init_nnz:
            raise ValueError("initial_matrix has duplicate raw entries; action ids would be ambiguous")
        self.pattern: Lines = build_lines(r, c, v, matrix_size, orient, self.device, torch.float32)
        a = self.original_matrix.coalesce()
        a_dtype = torch.float64 if a.dtype == torch.float64 else torch.float32
        ai = a.indices()
        self.a_lines: Lines = build_lines(ai[0], ai[1], a.values(), matrix_size, orient, self.device, a_dtype)
        self.last_m = None
        self.last_reward32 = None  # fp32 rewards of the last batch (Log.rewards)
        self.last_removed = None  # removal bitmaps [B, ceil(E/32)] of the last batch (assemble)
        self._word_spans = {}     # world -> per-rank bitmap word spans of the column shards
        # Gram cache of the fixed pattern (G = A_J^T A_J, c = A[l, J] per line): the per-rollout
        # fill then streams it instead of re-gathering A (pattern widths <= 13, A widths <= 7;
        # wider patterns use the generic kernels)
        # (not for fill="qr", which never reads it)
        self.gram = (kernels.gram_build(self.pattern, self.a_lines)
                     if self.pattern.width <= 13 and self.a_lines.width <= 7 and fill != "qr" else None)
        # the QR fill factors each line's dense block A[I, J]: its largest row union picks the kernel;
        # the factorisation of the FULL block is sample-independent, so it is done once here into the
        # R cache (rcache=False: refactor every call, the fused kernel)
        self.qr_rows = kernels.qr_max_rows(self.pattern, self.a_lines) if fill == "qr" else None
        self.rcache = (kernels.qr_cache(self.pattern, self.a_lines, self.qr_rows)
                       if fill == "qr" and rcache else None)
        if self.gram is not None and compact_gram:
            # integer stencils (and any A whose G, c are fp32-exact): the same cache in fp32
            g32 = kernels.gram_compact(self.gram, self.pattern)
            if g32 is not None:
                self.gram = g32
        if cache_dict:  # the caches' distinct line entries only (stencils: a handful); the 5/7-wide
            # Gram fill streams its full cache as fast (coalesced, 4 waves per SIMD either way)
            for name in ("gram", "rcache"):
                full = getattr(self, name)
                if full is None or (name == "gram" and self.pattern.width <= 7):
                    continue
                d = kernels.cache_dict(full, matrix_size)
                if d is not None:
                    setattr(self, name, d)

        self.orig_residual = self.calculate_residual(self.original_matrix, self.original_matrix)
        self._r0 = float(self.orig_residual)  # host copy: no device sync inside the reward formula
        self.orig_flops, _ = self.matrix_flops(self.original_matrix)

    # ------------------------------------------------------------------ hot path
    def update(self, sparse_matrices: List[Tensor], actions, alpha) -> List[Tensor]:
        """preconditioner.py:32-52: one reward per row of ``actions`` ([B, T], -1 padded)."""
        acts = torch.as_tensor(actions)
        if acts.dim() == 1:
            acts = acts.view(1, -1)
        acts = acts.to(self.device, torch.int64)
        removed, counts = kernels.actions_to_removed(acts, self.init_nnz)
        return list(self.rewards_from_removed(removed, counts, alpha).unbind(0))

    def rewards_from_removed(self, removed: Tensor, counts: Tensor, alpha, line_begin: int = 0,
                             line_end: int | None = None, group=None) -> Tensor:
        """[B] fp64 rewards from removal bitmaps; with ``group`` the lines are a shard and the
        per-sample squared norms are summed exactly across the process group (one all_reduce of
        the integer limbs: the same bits as one process when the shards are 256-line aligned)."""
        if group is None:
            if line_begin == 0 and (line_end is None or line_end == self.matrix_size):
                return self.fill_rewards(removed, counts, alpha)
            return self.rewards_from_res2(self.fill_partial(removed, line_begin, line_end), counts, alpha)
        from .distributed import all_reduce_
        limbs = all_reduce_(self.fill_partial(removed, line_begin, line_end, limbs=True), group)
        return self.rewards_from_res2(kernels.res2_from_limbs(limbs), counts, alpha)

    def fill_partial(self, removed: Tensor, line_begin: int = 0, line_end: int | None = None, word_base: int = 0,
                     limbs: bool = False, pattern: Lines | None = None) -> Tensor:
        """Fill lines [line_begin, line_end) of M for every sample and return the per-sample
        squared residual norms of those lines, [B] fp64 (kept in ``last_m`` / ``last_removed``);
        with ``limbs`` their exact sums [B, RES2_LIMBS] int64 instead (summable across line
        shards, spai_hip.h).  ``removed`` rows may be windows of the bitmaps starting at word
        ``word_base``, or packed rows read through ``pattern`` (the pattern with the shard's
        action ids renumbered: distributed.PackPlan.local_pattern, the columns split's exchange)."""
        kw = dict(store_m=self.keep_m, m_dtype=self.a_lines.val.dtype, word_base=word_base, limbs=limbs)
        pat = self.pattern if pattern is None else pattern
        if self.fill == "qr":
            res2, m = kernels.fill_residual_qr(pat, self.a_lines, self.qr_rows, removed, line_begin, line_end,
                                               rcache=self.rcache, **kw)
        elif self.gram is not None:
            res2, m = kernels.fill_residual_gram(pat, self.gram, removed, self._lsq, line_begin, line_end, **kw)
        else:
            res2, m = kernels.fill_residual(pat, self.a_lines, removed, self._lsq, line_begin, line_end, **kw)
        if self.keep_m:
            self.last_m = m
        # only whole bitmaps over all lines can be assembled: a window (the columns split's
        # all_to_all rows, whose last column is the removal count) or a line shard cannot
        whole = (pattern is None and word_base == 0 and removed.shape[1] == (self.init_nnz + 31) // 32
                 and line_begin == 0 and (line_end is None or line_end == self.matrix_size))
        self.last_removed = removed if whole else None
        return res2

    def pack_plan(self, world: int):
        """The columns split's bitmap exchange plan for ``world`` ranks (distributed.PackPlan; one
        host sync per world size, cached)."""
        plans = self.__dict__.setdefault("_pack_plans", {})
        if world not in plans:
            from .distributed import PackPlan
            plans[world] = PackPlan(self, world)
        return plans[world]

    def word_spans(self, world: int) -> list:
        """Bitmap word span [(w0, w1)] of each of ``world`` 256-line-aligned column shards
        (distributed.word_spans; one host sync per world size, cached)."""
        if world not in self._word_spans:
            from .distributed import word_spans
            self._word_spans[world] = word_spans(self, world)
        return self._word_spans[world]

    def rewards_from_res2(self, res2: Tensor, counts: Tensor, alpha) -> Tensor:
        """Residuals (``last_residual``) and rewards [B] fp64 from the summed squared norms (their
        fp32 copy, Log.rewards' dtype, in ``last_reward32``)."""
        if not torch.is_tensor(alpha):
            alpha = torch.tensor(float(alpha), dtype=torch.float32)
        self.last_residual, reward, self.last_reward32 = kernels.rewards(res2, counts, self.init_nnz,
                                                                         self.matrix_size, self._r0, self.orig_flops,
                                                                         alpha)
        return reward

    def fill_rewards(self, removed: Tensor, counts: Tensor, alpha) -> Tensor:
        """fill_partial over ALL lines + rewards_from_res2 (one GPU): with the Gram cache the exact
        residual sums and the reward formula run in one launch (spai_fill_reduce_rewards)."""
        if self.gram is None and self.fill != "qr":
            return self.rewards_from_res2(self.fill_partial(removed), counts, alpha)
        if not torch.is_tensor(alpha):
            alpha = torch.tensor(float(alpha), dtype=torch.float32)
        if self.fill == "qr":
            self.last_residual, reward, self.last_reward32, m = kernels.fill_rewards_qr(
                self.pattern, self.a_lines, self.qr_rows, removed, counts, self.init_nnz, self._r0, self.orig_flops,
                alpha, store_m=self.keep_m, m_dtype=self.a_lines.val.dtype, rcache=self.rcache)
        else:
            self.last_residual, reward, self.last_reward32, m = kernels.fill_rewards_gram(
                self.pattern, self.gram, removed, self.fill == "lsq", counts, self.init_nnz, self._r0,
                self.orig_flops, alpha, store_m=self.keep_m, m_dtype=self.a_lines.val.dtype)
        if self.keep_m:
            self.last_m = m
        self.last_removed = removed
        return reward

    def _performance(self, residual: Tensor, nnz: Tensor, alpha) -> Tensor:
        """preconditioner.py:137-165 with the reference's type promotion: alpha 0-d fp32,
        residual ratio fp64, flop ratio python-float -> fp32 product; sum in fp64."""
        dev = residual.device
        alpha = torch.as_tensor(alpha, dtype=torch.float32, device=dev) if not torch.is_tensor(alpha) else alpha.to(dev)
        rr = residual / self.orig_residual.to(dev) if self._r0 != 0 else torch.full_like(residual, float("inf"))
        flops = nnz.to(torch.float64) * (2.0 * self.matrix_size)
        cr = flops / self.orig_flops if self.orig_flops != 0 else torch.full_like(flops, float("inf"))
        t1 = alpha * (1 - rr)
        t2 = (1 - alpha) * (1 - cr).to(torch.float32)
        return t1 + t2

    # ------------------------------------------------------------------ reference API
    def reward(self, s: Tensor, traj_length: int, alpha) -> Tensor:
        r = self.evaluate_preconditioner(s, self.original_matrix, self.orig_residual, self.orig_flops, alpha)
        return r.to(torch.float64) * 1000

    def matrix_flops(self, matrix: Tensor) -> Tuple[int, int]:
        if matrix.is_sparse:
            non_zeros = matrix._values().numel()
            return non_zeros * matrix.shape[1] * 2, non_zeros
        non_zeros = torch.nonzero(matrix).size(0)
        return 2 * non_zeros, non_zeros

    def calculate_residual(self, updated_matrix: Tensor, original_matrix: Tensor) -> Tensor:
        """||M A - I||_F (or ||A M - I||_F for side='AM') of arbitrary sparse M, A on the GPU."""
        orient = self.pattern.orient
        n = self.matrix_size
        if original_matrix is self.original_matrix:
            a_lines = self.a_lines
        else:
            a = original_matrix.coalesce()
            ai = a.indices()
            a_lines = build_lines(ai[0], ai[1], a.values(), n, orient, self.device,
                                  torch.float64 if a.dtype == torch.float64 else torch.float32)
        m = updated_matrix.coalesce()
        mi = m.indices()
        mval = torch.float64 if m.dtype == torch.float64 else torch.float32
        pat = build_lines(mi[0], mi[1], m.values(), n, orient, self.device, mval)
        if pat.width <= 13 and a_lines.width <= 7:  # the generic SpMM residual kernel
            return torch.sqrt(kernels.residual_lines(pat.idx, pat.val, a_lines)[0])
        # wider lines (e.g. spilu L@U patterns): the LDS-hash line kernel of the copy fill
        pat = build_lines(mi[0], mi[1], m.values(), n, orient, self.device, torch.float32)
        removed = torch.zeros(1, max((m._nnz() + 31) // 32, 1), dtype=torch.int32, device=self.device)
        res2, _ = kernels.fill_residual(pat, a_lines, removed, lsq=False)
        return torch.sqrt(res2[0])

    def mask(self, s: Tensor) -> Tensor:
        return torch.ones(len(s), self.num_actions)

    def evaluate_preconditioner(self, updated_matrix: Tensor, original_matrix: Tensor, orig_residual, orig_flops,
                                alpha) -> Tensor:
        residual = self.calculate_residual(updated_matrix, original_matrix)
        _, non_zeros = self.matrix_flops(updated_matrix)
        return self._performance(residual.view(1), torch.tensor([non_zeros], device=residual.device), alpha)[0]

    # ------------------------------------------------------------------ products
    def assemble(self, b: int = 0, removed: Tensor | None = None) -> Tensor:
        """Sparse M of sample b of the last batch, as update_edges_and_convert_to_sparse returns
        it (gflownet/utils.py:295-356 + resize :89-126): coalesced [N, N] COO holding exactly the
        kept pattern entries (COPY: their pattern values; LSQ: the fitted values).  ``removed``
        defaults to the last batch's removal bitmaps."""
        if removed is None:
            removed = self.last_removed
        if removed is None:
            raise ValueError("no removal bitmaps: run update / rewards_from_removed first or pass removed")
        if self._lsq and self.last_m is None:
            raise ValueError("construct with keep_m=True to keep M")
        bits = removed[b].to(self.device)
        act = self.pattern.act.long()
        a = act.clamp(min=0)
        keep = (act >= 0) & (((bits[a >> 5] >> (a & 31)) & 1) == 0)
        vals = self.last_m[b] if self._lsq else self.pattern.val
        return lines_to_coo(self.pattern, vals, self.matrix_size, keep)
