"""GMRES evaluation (GFlowNet100.py:61-93): the device restatement of
scipy.sparse.linalg.gmres against scipy itself.  CPU: the host algorithm (_gmres) driven by
CPU torch vectors and scipy products.  GPU: solve_with_gmres with A and the SPAI M applied by
spai_ell_spmv, and the power-pattern SPAI baseline vs the oracle's column least squares."""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla
import torch

from gflownet_spai_amd.gmres import _gmres
from gflownet_spai_amd.utils import poisson_2d


def poisson_csr(g):
    A = poisson_2d(g, torch.float64).coalesce()
    return sp.csr_matrix((A.values().numpy(), tuple(A.indices().numpy())), shape=A.shape)


def nonsym(n, seed):
    rng = np.random.default_rng(seed)
    R = sp.random(n, n, density=4.0 / n, random_state=seed, format="csr")
    return (sp.identity(n) * 4 + R - R.T * 0.5 + sp.diags(rng.random(n))).tocsr()


def scipy_run(A, b, M=None, **kw):
    res = []
    x, info = spla.gmres(A, b, x0=np.zeros_like(b), M=M, callback=res.append, callback_type="legacy", **kw)
    return x, info, res


def host_run(A, b, M=None, **kw):
    res = []
    mv = lambda v: torch.from_numpy(A @ v.numpy())  # noqa: E731
    ps = (lambda v: v.clone()) if M is None else (lambda v: torch.from_numpy(M @ v.numpy()))  # noqa: E731
    x, info = _gmres(mv, ps, torch.from_numpy(b), callback=res.append, **kw)
    return x.numpy(), info, res


CASES = [("poisson16", lambda: poisson_csr(16), None), ("poisson16-jacobi", lambda: poisson_csr(16), "jacobi"),
         ("nonsym300", lambda: nonsym(300, 1), None), ("nonsym300-jacobi", lambda: nonsym(300, 2), "jacobi")]


def make_m(A, kind):
    return None if kind is None else sp.diags(1.0 / A.diagonal()).tocsr()


@pytest.mark.parametrize("name,mk,mkind", CASES)
@pytest.mark.parametrize("maxiter", [None, 10260, 7])
def test_host_algorithm_matches_scipy(name, mk, mkind, maxiter):
    A = mk()
    M = make_m(A, mkind)
    b = np.random.default_rng(0).standard_normal(A.shape[0])
    x0, i0, r0 = scipy_run(A, b, M, maxiter=maxiter)
    x1, i1, r1 = host_run(A, b, M, maxiter=maxiter)
    assert i1 == i0 and len(r1) == len(r0)
    np.testing.assert_allclose(r1, r0, rtol=1e-9, atol=1e-15)
    np.testing.assert_allclose(x1, x0, rtol=1e-9, atol=1e-12 * np.abs(x0).max())


def test_host_algorithm_restart_and_zero_rhs():
    A = nonsym(200, 3)
    b = np.random.default_rng(1).standard_normal(200)
    x0, i0, r0 = scipy_run(A, b, restart=5, maxiter=40)
    x1, i1, r1 = host_run(A, b, restart=5, maxiter=40)
    assert i1 == i0 and len(r1) == len(r0)
    np.testing.assert_allclose(r1, r0, rtol=1e-9)
    x, info = _gmres(lambda v: v, lambda v: v, torch.zeros(5, dtype=torch.float64))
    assert info == 0 and not x.any()


def test_solve_with_gmres_refuses_cpu():
    from gflownet_spai_amd import _lib
    from gflownet_spai_amd.gmres import DeviceOperator
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    with pytest.raises((_lib.SpaiUnavailable, RuntimeError, AssertionError)):
        DeviceOperator(poisson_csr(4), device="cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("name,mk,mkind", CASES)
def test_device_gmres_matches_scipy(name, mk, mkind):
    from gflownet_spai_amd.gmres import solve_with_gmres
    A = mk()
    M = make_m(A, mkind)
    b = np.random.default_rng(0).standard_normal(A.shape[0])
    x0, i0, r0 = scipy_run(A, b, M, maxiter=10260)
    x1, r1, it, _ = solve_with_gmres(A, b, M, verbose=False)
    assert it == len(r0) and it == len(r1)
    np.testing.assert_allclose(r1, r0, rtol=1e-8, atol=1e-15)
    np.testing.assert_allclose(x1, x0, rtol=1e-8, atol=1e-11 * np.abs(x0).max())


@pytest.mark.gpu
def test_device_gmres_host_preconditioner_ilu():
    """The driver's spilu baseline (GFlowNet100.py:126-132) as a host LinearOperator."""
    from gflownet_spai_amd.gmres import solve_with_gmres
    A = poisson_csr(20)
    ilu = spla.spilu(A.tocsc())
    M = spla.LinearOperator(A.shape, ilu.solve)
    b = np.ones(A.shape[0])
    x0, i0, r0 = scipy_run(A, b, M, maxiter=10260)
    x1, r1, it, _ = solve_with_gmres(A, b, M, verbose=False)
    assert it == len(r0)
    np.testing.assert_allclose(r1, r0, rtol=1e-8, atol=1e-15)


@pytest.mark.gpu
@pytest.mark.parametrize("power", [1, 2])
def test_power_pattern_spai_vs_lstsq_and_gmres(power):
    """SPAI on the pattern of A^power: every column is lstsq's min ||A m_j - e_j|| (oracle), and
    GMRES with it matches scipy's GMRES with the same M."""
    from gflownet_spai_amd.gmres import solve_with_gmres, spai_power_pattern
    A = poisson_csr(10)
    n = A.shape[0]
    M = spai_power_pattern(A, power).coalesce()
    Mcsc = sp.csc_matrix((M.values().double().cpu().numpy(), tuple(M.indices().cpu().numpy())), shape=(n, n))
    P = (abs(A) ** power).tocsc()
    for j in range(0, n, 7):
        J = P[:, j].indices
        m, *_ = np.linalg.lstsq(A[:, J].toarray(), np.eye(n)[:, j], rcond=None)
        np.testing.assert_allclose(Mcsc[J, j].toarray().ravel(), m, rtol=1e-6, atol=1e-9)
    b = np.random.default_rng(3).standard_normal(n)
    Mcsr = Mcsc.tocsr()
    x0, i0, r0 = scipy_run(A, b, Mcsr, maxiter=10260)
    x1, r1, it, _ = solve_with_gmres(A, b, M, verbose=False)
    assert it == len(r0)
    np.testing.assert_allclose(r1, r0, rtol=1e-7, atol=1e-15)
    assert it < len(scipy_run(A, b, None, maxiter=10260)[2])  # it preconditions
