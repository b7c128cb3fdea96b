"""Host-side helpers with the reference's names (reference: gflownet/utils.py)."""
from __future__ import annotations

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


def market_matrix_to_sparse_tensor(file_path: str) -> Tensor:
    """gflownet/utils.py:54-63: Matrix Market file -> fp64 COO tensor (raw file order)."""
    import scipy.io

    m = scipy.io.mmread(file_path).tocoo()
    idx = torch.from_numpy(np.vstack([m.row, m.col]).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(m.data.astype(np.float64)), m.shape)


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
