"""HBM layout of the candidate pattern and of A: line-major ELL, built on the device.

The reference keeps the candidate pattern as a torch COO tensor whose RAW
``_indices()`` order defines the action ids (preconditioner.py:14-25) and rebuilds a
fresh COO matrix per sample (gflownet/utils.py:295-356).  Here the pattern is laid out
once, in the orientation of the residual that is evaluated:

  side "MA" (reference, preconditioner.py:79-93): line i = row i of M, A lines = rows of A
  side "AM" (north star, column SPAI):             line j = column j of M, A lines = cols of A

``Lines`` holds [n, W] int32 other-index (-1 padded), [n, W] int32 action id and [n, W]
values, entries of a line sorted by the other index.  All B samples share it; a sample
is only its removal bitmap (and, for LSQ fill, its [n, W] values).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch


@dataclass
class Lines:
    n: int
    width: int
    idx: torch.Tensor  # [n, width] int32, -1 = padding
    act: torch.Tensor  # [n, width] int32 action id (raw COO position), -1 = padding
    val: torch.Tensor  # [n, width] values (fp32 for a pattern, A's dtype for A lines)
    orient: str        # "row" | "col"
    # kernels.narrow_values' cache: (val it was computed from, fp32 copy if exact else val)
    _narrow: tuple | None = field(default=None, repr=False, compare=False)

    @property
    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.idx, self.act, self.val))


def raw_coo(t: torch.Tensor):
    """(rows, cols, vals) of a sparse COO tensor in RAW order (no coalesce)."""
    if not t.is_sparse:
        raise ValueError("The input tensor must be a sparse tensor.")
    ind = t._indices()
    return ind[0], ind[1], t._values()


def build_lines(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n: int, orient: str,
                device, val_dtype=None, width: int | None = None) -> Lines:
    """ELL lines of a raw COO matrix; action id of an entry = its raw position."""
    if orient not in ("row", "col"):
        raise ValueError(f"orient must be 'row' or 'col', got {orient!r}")
    rows = rows.to(device=device, dtype=torch.int64)
    cols = cols.to(device=device, dtype=torch.int64)
    vals = vals.to(device=device, dtype=val_dtype or vals.dtype)
    nnz = rows.numel()
    line, other = (rows, cols) if orient == "row" else (cols, rows)
    if nnz and (int(line.min()) < 0 or int(line.max()) >= n or int(other.min()) < 0 or int(other.max()) >= n):
        raise ValueError("sparse indices out of range for matrix_size")
    key = line * n + other
    order = torch.argsort(key, stable=True)
    ks = key[order]
    if nnz > 1 and bool((ks[1:] == ks[:-1]).any()):
        raise ValueError("duplicate (row, col) entries in the raw COO pattern are not supported; coalesce it first")
    ls = line[order]
    counts = torch.bincount(ls, minlength=n)
    w = int(counts.max()) if nnz else 0
    if width is None:
        width = max(w, 1)
    if w > width:
        raise ValueError(f"line width {w} exceeds {width}")
    start = torch.cumsum(counts, 0) - counts
    slot = torch.arange(nnz, device=device) - start[ls]
    flat = ls * width + slot
    idx = torch.full((n * width,), -1, dtype=torch.int32, device=device)
    act = torch.full((n * width,), -1, dtype=torch.int32, device=device)
    val = torch.zeros(n * width, dtype=vals.dtype, device=device)
    idx[flat] = other[order].to(torch.int32)
    act[flat] = order.to(torch.int32)
    val[flat] = vals[order]
    return Lines(n, width, idx.view(n, width), act.view(n, width), val.view(n, width), orient)


def lines_to_coo(lines: Lines, values: torch.Tensor, n: int, keep: torch.Tensor | None = None) -> torch.Tensor:
    """Assemble a coalesced [n, n] sparse COO matrix from per-line values aligned with
    ``lines``: padding slots and the slots where ``keep`` ([n, W] bool) is False are dropped,
    so the result holds exactly the kept entries (gflownet/utils.py:323-353)."""
    li = torch.arange(n, device=lines.idx.device).repeat_interleave(lines.width)
    oi = lines.idx.reshape(-1).long()
    ok = oi >= 0
    if keep is not None:
        ok &= keep.reshape(-1)
    li, oi, v = li[ok], oi[ok], values.reshape(-1)[ok]
    rows, cols = (li, oi) if lines.orient == "row" else (oi, li)
    return torch.sparse_coo_tensor(torch.stack([rows, cols]), v, (n, n)).coalesce()
