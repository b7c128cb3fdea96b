"""Host-side helpers with the reference's names (reference: gflownet/utils.py)."""
from __future__ import annotations

import os

import numpy as np
import torch
from torch import Tensor


def trajectory_balance_loss(total_flow: Tensor, rewards: Tensor, fwd_probs: Tensor, back_probs: Tensor) -> Tensor:
    """gflownet/utils.py:228-278: squared log-ratio of Z * prod pF and R * prod pB, each
    trajectory sum shifted by its batch maximum, averaged over the batch (eps = 1e-9)."""
    eps = 1e-9
    dt, dev = fwd_probs.dtype, fwd_probs.device
    log_pf = torch.log(fwd_probs + eps).sum(-1)
    log_pb = torch.log(back_probs.to(dev, dt) + eps).sum(-1)
    lhs = torch.log(total_flow.to(dev, dt) + eps) + (log_pf - log_pf.max(0, keepdim=True).values)
    rhs = torch.log(rewards.to(dev, dt) + eps) + (log_pb - log_pb.max(0, keepdim=True).values)
    return (lhs - rhs).pow(2).mean()


def read_mtx(file_path: str, threads: int = 0):
    """Matrix Market file -> (rows, cols, values float64, shape) host arrays in the order of
    scipy.io.mmread(path).tocoo(), parsed by the native multi-threaded reader (spai_mtx_read)."""
    import ctypes

    from . import _lib

    lib = _lib.load()
    path = os.fsencode(file_path)
    dims = np.zeros(4, np.int64)
    kinds = np.zeros(2, np.int32)
    _lib.check(lib.spai_mtx_header(path, dims.ctypes.data_as(ctypes.c_void_p), kinds.ctypes.data_as(ctypes.c_void_p)),
               "spai_mtx_header")
    cap = int(dims[3])
    rows, cols = np.empty(cap, np.int64), np.empty(cap, np.int64)
    vals = np.empty(cap, np.float64)
    nnz = ctypes.c_int64(0)
    _lib.check(lib.spai_mtx_read(path, rows.ctypes.data_as(ctypes.c_void_p), cols.ctypes.data_as(ctypes.c_void_p),
                                 vals.ctypes.data_as(ctypes.c_void_p), cap, int(threads), ctypes.byref(nnz)),
               "spai_mtx_read")
    k = nnz.value
    return rows[:k], cols[:k], vals[:k], (int(dims[0]), int(dims[1]))


def market_matrix_to_sparse_tensor(file_path: str) -> Tensor:
    """gflownet/utils.py:54-63: Matrix Market file -> fp64 COO tensor (uncoalesced, in mmread's
    raw order, which defines the action ids), read by the native parser."""
    rows, cols, vals, shape = read_mtx(file_path)
    idx = torch.from_numpy(np.vstack([rows, cols]))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(vals), shape)


def load_mtx_file(file_path: str):
    """GFlowNet100.py:44-46: csr_matrix(mmread(path)) (scipy CSR, duplicates summed), from the
    native reader."""
    import scipy.sparse as sp

    rows, cols, vals, shape = read_mtx(file_path)
    return sp.csr_matrix((vals, (rows, cols)), shape=shape)


def lu_candidate_matrix(A) -> Tensor:
    """GFlowNet100.py:126-153: the candidate pattern the driver samples from.  spilu(A) with
    scipy's defaults (SuperLU ILUTP), L = tril(ilu.L), U = triu(ilu.U), LU = L @ U (the factors in
    SuperLU's permuted order, as the driver takes them), as an fp32 COO tensor in LU.tocoo()
    order.  One-time host preprocessing, as in the reference; the rollout then runs on the GPU
    with this tensor as initial_matrix = original_matrix (GFlowNet100.py:173)."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla

    ilu = spla.spilu(sp.csc_matrix(A))
    L = sp.tril(ilu.L, format="csr")
    U = sp.triu(ilu.U, format="csr")
    coo = (L @ U).tocoo()
    idx = torch.from_numpy(np.vstack((coo.row, coo.col)).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(coo.data.astype(np.float32)), coo.shape)


def poisson_2d(grid: int, dtype=torch.float32) -> Tensor:
    """5-point Laplacian kron(I,T)+kron(T,I), T = tridiag(-1,2,-1), row-major COO (N = grid^2)."""
    n = grid * grid
    i = torch.arange(n)
    r, c = i // grid, i % grid
    rows, cols, vals = [i], [i], [torch.full((n,), 4.0)]
    for dr, dc in ((-1, 0), (1, 0), (0, -1), (0, 1)):
        ok = (r + dr >= 0) & (r + dr < grid) & (c + dc >= 0) & (c + dc < grid)
        rows.append(i[ok])
        cols.append(((r + dr) * grid + (c + dc))[ok])
        vals.append(torch.full((int(ok.sum()),), -1.0))
    rows, cols, vals = torch.cat(rows), torch.cat(cols), torch.cat(vals)
    order = torch.argsort(rows * n + cols)
    return torch.sparse_coo_tensor(torch.stack([rows[order], cols[order]]), vals[order].to(dtype), (n, n))


def thermal_like(grid: int, seed: int = 0, dtype=torch.float64) -> Tensor:
    """Synthetic stand-in for SuiteSparse thermal2 (C5: 1,227,087 unknowns, 8,579,355 nnz,
    ~7 nnz/row, SPD, unstructured): a steady heat-conduction matrix on a triangulated grid^2
    mesh — every node coupled to its 6 triangle neighbours (dx, dy) in {(+-1,0), (0,+-1),
    (1,-1), (-1,1)} with lognormal edge conductivities k_e (sigma 1: coefficient jumps of
    ~e^3 across the mesh), off-diagonals -k_e, diagonal = the node's conductance sum + 1e-3
    (a Robin-type anchor, so the matrix is SPD) — with the node numbering randomly permuted
    (no band or grid structure left in the ordering).  grid = 1108 gives 1,227,664 unknowns and
    8,584,786 nnz.  Coalesced COO (rows, then columns ascending)."""
    g = torch.Generator().manual_seed(seed)
    n = grid * grid
    i = torch.arange(n)
    r, c = i // grid, i % grid
    src, dst = [], []
    for dr, dc in ((0, 1), (1, 0), (1, -1)):  # each undirected edge once
        ok = (r + dr < grid) & (c + dc >= 0) & (c + dc < grid)
        src.append(i[ok])
        dst.append(((r + dr) * grid + (c + dc))[ok])
    src, dst = torch.cat(src), torch.cat(dst)
    k = torch.exp(torch.randn(src.numel(), generator=g, dtype=torch.float64))
    perm = torch.randperm(n, generator=g)
    src, dst = perm[src], perm[dst]
    diag = torch.full((n,), 1e-3, dtype=torch.float64)
    diag.index_add_(0, src, k)
    diag.index_add_(0, dst, k)
    rows = torch.cat([torch.arange(n), src, dst])
    cols = torch.cat([torch.arange(n), dst, src])
    vals = torch.cat([diag, -k, -k])
    order = torch.argsort(rows * n + cols)
    return torch.sparse_coo_tensor(torch.stack([rows[order], cols[order]]), vals[order].to(dtype), (n, n))


def poisson_3d(grid: int, dtype=torch.float64) -> Tensor:
    """7-point Laplacian on a grid^3 lattice (diag 6, off-diag -1), row-major COO."""
    n = grid ** 3
    i = torch.arange(n)
    x, y, z = i % grid, (i // grid) % grid, i // (grid * grid)
    rows, cols, vals = [i], [i], [torch.full((n,), 6.0)]
    for dx, dy, dz in ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)):
        ok = (x + dx >= 0) & (x + dx < grid) & (y + dy >= 0) & (y + dy < grid) & (z + dz >= 0) & (z + dz < grid)
        rows.append(i[ok])
        cols.append(((z + dz) * grid * grid + (y + dy) * grid + (x + dx))[ok])
        vals.append(torch.full((int(ok.sum()),), -1.0))
    rows, cols, vals = torch.cat(rows), torch.cat(cols), torch.cat(vals)
    order = torch.argsort(rows * n + cols)
    return torch.sparse_coo_tensor(torch.stack([rows[order], cols[order]]), vals[order].to(dtype), (n, n))


def axial_pattern_3d(grid: int, reach: int = 2, dtype=torch.float64) -> Tensor:
    """Candidate pattern of config C3 ("deeper learned pattern, nnz/col <= 13"): the 7-point
    star plus the axial neighbours at distance 2..reach on a grid^3 lattice (13 entries per
    interior column at reach 2, a subset of A^2's 25-point pattern, so it contains A).
    Values: A's stencil values (6 / -1) on A's entries, 0 beyond; the COPY fill copies them,
    the LSQ fill ignores them.  Row-major COO (action id = position)."""
    n = grid ** 3
    i = torch.arange(n)
    x, y, z = i % grid, (i // grid) % grid, i // (grid * grid)
    rows, cols, vals = [i], [i], [torch.full((n,), 6.0)]
    for d in range(1, reach + 1):
        for dx, dy, dz in ((d, 0, 0), (-d, 0, 0), (0, d, 0), (0, -d, 0), (0, 0, d), (0, 0, -d)):
            ok = (x + dx >= 0) & (x + dx < grid) & (y + dy >= 0) & (y + dy < grid) & (z + dz >= 0) & (z + dz < grid)
            rows.append(i[ok])
            cols.append(((z + dz) * grid * grid + (y + dy) * grid + (x + dx))[ok])
            vals.append(torch.full((int(ok.sum()),), -1.0 if d == 1 else 0.0))
    rows, cols, vals = torch.cat(rows), torch.cat(cols), torch.cat(vals)
    order = torch.argsort(rows * n + cols)
    return torch.sparse_coo_tensor(torch.stack([rows[order], cols[order]]), vals[order].to(dtype), (n, n))
