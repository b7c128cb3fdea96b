"""GMRES evaluation of a preconditioner on the MI355X.

Reference: GFlowNet100.py:61-93 ``solve_with_gmres(A, b, M=None)`` =
``scipy.sparse.linalg.gmres(A, b, x0=0, M=M, maxiter=10260, callback=callback)`` (restart 20,
rtol 1e-5, left preconditioning, legacy callback = preconditioned relative residual per inner
iteration), and GFlowNet100.py:126-132 (the spilu baseline as a LinearOperator).

``_gmres`` restates scipy 1.15's ``gmres`` (scipy/sparse/linalg/_isolve/iterative.py) step for
step: Arnoldi with modified Gram-Schmidt, LAPACK ``lartg`` Givens rotations, the gh-8400 inner
tolerance control, the same breakdown and exit rules.  The Krylov basis and every length-n
vector live on the GPU; A v and M v run on ``spai_ell_spmv`` (row-ELL, fp64); the dot products
and axpys of the Gram-Schmidt are device ops; only the (restart+1)-sized Hessenberg column
crosses to the host once per inner iteration, where the rotations run in fp64 exactly as scipy
runs them.  Preconditioners: None, a sparse matrix (SPAI M: applied on the GPU) or a host
callable / LinearOperator (e.g. the spilu baseline: applied on the host, copied each way).
"""
from __future__ import annotations

import time
from typing import Callable

import numpy as np
import torch

from . import _lib, kernels
from .layout import Lines, build_lines


class DeviceOperator:
    """y = A x on the GPU for a square sparse A held as row-ELL lines (values fp32 or fp64)."""

    def __init__(self, A, device=None, dtype=None):
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if isinstance(A, Lines):
            if A.orient != "row":
                raise ValueError("DeviceOperator needs row lines")
            self.lines, self.n = A, A.n
        else:
            rows, cols, vals, n = _coo_of(A)
            vd = dtype or (torch.float64 if vals.dtype == torch.float64 else torch.float32)
            self.lines = build_lines(rows, cols, vals, n, "row", dev, vd)
            self.n = n
        self.shape = (self.n, self.n)
        self.device = self.lines.idx.device
        _lib.require_device(self.lines.idx)

    def matvec_into(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        L = self.lines
        dt = 1 if L.val.dtype == torch.float64 else 0  # SPAI_DTYPE_F64 / SPAI_DTYPE_F32
        st = kernels._l().spai_ell_spmv(self.n, L.width, _lib.ptr(L.idx), _lib.ptr(L.val), dt, _lib.ptr(x),
                                        _lib.ptr(y), _lib.stream_ptr(self.device))
        _lib.check(st, "spai_ell_spmv")
        return y

    def matvec(self, x: torch.Tensor) -> torch.Tensor:
        if x.dtype != torch.float64 or not x.is_contiguous() or x.device != self.device:
            raise ValueError("DeviceOperator.matvec takes a contiguous fp64 vector on its device")
        return self.matvec_into(x, torch.empty_like(x))


def _coo_of(A):
    """(rows, cols, vals, n) of a scipy sparse matrix or a torch sparse tensor, duplicates summed."""
    if isinstance(A, torch.Tensor):
        if not A.is_sparse:
            raise ValueError("A must be sparse")
        c = A.coalesce()
        return c.indices()[0], c.indices()[1], c.values(), int(A.shape[0])
    import scipy.sparse as sp
    if not sp.issparse(A):
        raise ValueError("A must be a scipy sparse matrix, a torch sparse tensor or Lines")
    c = sp.coo_matrix(A)
    c.sum_duplicates()
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt))  # noqa: E731
    vdt = np.float64 if c.dtype == np.float64 else np.float32
    return t(c.row, np.int64), t(c.col, np.int64), t(c.data, vdt), int(c.shape[0])


def _host_psolve(fn, device) -> Callable[[torch.Tensor], torch.Tensor]:
    def apply(v: torch.Tensor) -> torch.Tensor:
        out = np.asarray(fn(v.detach().cpu().numpy()), dtype=np.float64).reshape(-1)
        return torch.from_numpy(out).to(device)
    return apply


def _gmres(matvec, psolve, b: torch.Tensor, x0: torch.Tensor | None = None, *, rtol=1e-5, atol=0.0, restart=None,
           maxiter=None, callback=None):
    """scipy.sparse.linalg.gmres (legacy callback semantics) on torch vectors; returns (x, info).
    ``matvec``/``psolve`` map a length-n fp64 tensor to one on the same device."""
    from scipy.linalg import get_lapack_funcs

    n = b.numel()
    x = torch.zeros_like(b) if x0 is None else x0.clone()
    bnrm2 = float(torch.linalg.vector_norm(b))
    if atol is None or atol < 0:
        raise ValueError("atol must be a real, non-negative number")
    atol = max(float(atol), float(rtol) * bnrm2)
    if bnrm2 == 0:
        return b.clone(), 0
    eps = np.finfo(np.float64).eps
    if maxiter is None:
        maxiter = n * 10
    restart = min(20 if restart is None else restart, n)
    Mb_nrm2 = float(torch.linalg.vector_norm(psolve(b)))
    ptol_max_factor = 1.0
    ptol = Mb_nrm2 * min(ptol_max_factor, atol / bnrm2)
    presid = 0.0
    lartg = get_lapack_funcs("lartg", dtype=np.float64)
    v = torch.empty(restart + 1, n, dtype=torch.float64, device=b.device)
    h = np.zeros([restart, restart + 1], dtype=np.float64)
    givens = np.zeros([restart, 2], dtype=np.float64)
    hcol = torch.empty(restart + 3, dtype=torch.float64, device=b.device)
    inner_iter = 0
    rnorm = float("inf")
    for iteration in range(maxiter):
        if iteration == 0:
            r = b - matvec(x) if bool(x.any()) else b.clone()
            if float(torch.linalg.vector_norm(r)) < atol:
                return x, 0
        v[0] = psolve(r)
        tmp = float(torch.linalg.vector_norm(v[0]))
        v[0] *= 1 / tmp
        S = np.zeros(restart + 1, dtype=np.float64)
        S[0] = tmp
        breakdown = False
        for col in range(restart):
            w = psolve(matvec(v[col]))
            hcol[0] = torch.linalg.vector_norm(w)
            for k in range(col + 1):  # modified Gram-Schmidt, on the device
                t = torch.dot(v[k], w)
                hcol[1 + k] = t
                w -= t * v[k]
            hcol[col + 2] = torch.linalg.vector_norm(w)
            hh = hcol[:col + 3].cpu().numpy()  # the one host round trip of the inner iteration
            h0, h1 = hh[0], hh[col + 2]
            h[col, :col + 1] = hh[1:col + 2]
            h[col, col + 1] = h1
            v[col + 1] = w
            if h1 <= eps * h0:
                h[col, col + 1] = 0
                breakdown = True
            else:
                v[col + 1] *= 1 / h1
            for k in range(col):
                c, s = givens[k, 0], givens[k, 1]
                n0, n1 = h[col, [k, k + 1]]
                h[col, [k, k + 1]] = [c * n0 + s * n1, -np.conj(s) * n0 + c * n1]
            c, s, mag = lartg(h[col, col], h[col, col + 1])
            givens[col, :] = [c, s]
            h[col, [col, col + 1]] = mag, 0
            tmp = -np.conjugate(s) * S[col]
            S[[col, col + 1]] = [c * S[col], tmp]
            presid = np.abs(tmp)
            inner_iter += 1
            if callback is not None:
                callback(presid / bnrm2)
            if callback is not None and inner_iter == maxiter:
                break
            if presid <= ptol or breakdown:
                break
        if h[col, col] == 0:
            S[col] = 0
        y = np.zeros([col + 1], dtype=np.float64)
        y[:] = S[:col + 1]
        for k in range(col, 0, -1):
            if y[k] != 0:
                y[k] /= h[k, k]
                tmp = y[k]
                y[:k] -= tmp * h[k, :k]
        if y[0] != 0:
            y[0] /= h[0, 0]
        x += torch.from_numpy(y).to(b.device) @ v[:col + 1]
        r = b - matvec(x)
        rnorm = float(torch.linalg.vector_norm(r))
        if callback is not None and inner_iter == maxiter:
            return x, 0 if rnorm <= atol else maxiter
        if rnorm <= atol:
            break
        elif breakdown:
            break
        elif presid <= ptol:
            ptol_max_factor = max(eps, 0.25 * ptol_max_factor)
        else:
            ptol_max_factor = min(1.0, 1.5 * ptol_max_factor)
        ptol = presid * min(ptol_max_factor, atol / rnorm)
    info = 0 if rnorm <= atol else maxiter
    return x, info


def gmres(A, b, x0=None, *, M=None, rtol=1e-5, atol=0.0, restart=None, maxiter=None, callback=None, device=None):
    """scipy.sparse.linalg.gmres on the GPU: A (scipy / torch sparse, Lines or DeviceOperator),
    M None | sparse (applied on the GPU) | host callable or LinearOperator.  Returns (x, info)
    with x an fp64 device tensor."""
    Aop = A if isinstance(A, DeviceOperator) else DeviceOperator(A, device=device)
    dev = Aop.device
    bt = torch.as_tensor(np.asarray(b, dtype=np.float64).reshape(-1) if not isinstance(b, torch.Tensor) else b,
                         dtype=torch.float64).reshape(-1).to(dev).contiguous()
    if bt.numel() != Aop.n:
        raise ValueError(f"Shape mismatch: A is {Aop.shape}, but b is {tuple(bt.shape)}")
    if M is None:
        psolve = lambda v: v.clone()  # noqa: E731  (scipy's IdentityOperator returns a copy)
    elif isinstance(M, DeviceOperator):
        psolve = M.matvec
    elif isinstance(M, torch.Tensor) or hasattr(M, "tocoo") and not hasattr(M, "matvec"):
        psolve = DeviceOperator(M, device=dev).matvec
    else:
        import scipy.sparse as sp
        if sp.issparse(M):
            psolve = DeviceOperator(M, device=dev).matvec
        else:
            fn = M.matvec if hasattr(M, "matvec") else M
            psolve = _host_psolve(fn, dev)
    x0t = None if x0 is None else torch.as_tensor(np.asarray(x0, np.float64)).to(dev)
    return _gmres(lambda v: Aop.matvec(v.contiguous()), lambda v: psolve(v.contiguous()), bt, x0t, rtol=rtol,
                  atol=atol, restart=restart, maxiter=maxiter, callback=callback)


def solve_with_gmres(A, b, M=None, *, verbose: bool = True, device=None, maxiter: int = 10260):
    """GFlowNet100.py:61-93: (x, residuals, num_iterations, elapsed_time) of GMRES from x0 = 0
    with maxiter = 10260 (the driver's; a keyword lowers it for large evaluations), recording the
    legacy callback's preconditioned relative residual of every inner iteration; x is returned
    as a host numpy array like the reference's."""
    b = np.asarray(b, dtype=np.float64).reshape(-1) if not isinstance(b, torch.Tensor) else b.reshape(-1)
    n = A.n if isinstance(A, DeviceOperator) else A.shape[0]
    if b.shape[0] != n:
        raise ValueError(f"Shape mismatch: A is {tuple(A.shape)}, but b is {tuple(b.shape)}")
    residuals: list = []
    start = time.time()
    x, exit_code = gmres(A, b, M=M, maxiter=maxiter, callback=residuals.append, device=device)
    torch.cuda.synchronize(x.device)
    elapsed = time.time() - start
    if verbose:
        print("GMRES converged successfully." if exit_code == 0 else f"GMRES did not converge. Exit code: {exit_code}")
    return x.cpu().numpy(), residuals, len(residuals), elapsed


def spai_power_pattern(A, power: int = 1, device=None):
    """The power-pattern SPAI baseline: M with the sparsity of A^power,
    each column the least-squares solution of min ||A m_j - e_j|| (the env's LSQ fill, AM side,
    nothing removed).  Returns M as a sparse COO tensor on the device (A's dtype)."""
    import scipy.sparse as sp

    from .preconditioner import PreconditionerEnv
    rows, cols, vals, n = _coo_of(A)
    Acsr = sp.csr_matrix((vals.double().numpy(), (rows.numpy(), cols.numpy())), shape=(n, n))
    P = sp.csr_matrix(Acsr, copy=True)
    P.data[:] = 1.0
    Pk = P
    for _ in range(power - 1):
        Pk = Pk @ P
    Pk = Pk.tocoo()
    pat = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([Pk.row, Pk.col]).astype(np.int64)),
                                  torch.ones(Pk.nnz, dtype=torch.float32), (n, n))
    orig = torch.sparse_coo_tensor(torch.stack([rows, cols]), vals, (n, n))
    env = PreconditionerEnv(n, pat, orig, side="AM", fill="lsq", keep_m=True, device=device)
    words = (env.init_nnz + 31) // 32
    removed = torch.zeros(1, words, dtype=torch.int32, device=env.device)
    counts = torch.zeros(1, dtype=torch.int32, device=env.device)
    env.rewards_from_removed(removed, counts, torch.tensor(0.5))
    return env.assemble(0)
