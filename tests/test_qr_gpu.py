"""The least-squares fill by Householder QR (csrc/qr.hip, PreconditionerEnv(fill="qr")) against
the oracle's stacked Householder QR (oracle/spai_oracle.py lsq_fill) and numpy lstsq.

Bar (north star): M within 1e-6 relative Frobenius error, ||AM - I||_F within 1e-6; here much
tighter where the arithmetic allows (fp64 M: 1e-11).  Also: the QR and the normal-equations
(Gram) fill agree on well-conditioned stencils; on an ill-conditioned matrix the QR fill stays
at lstsq's accuracy where the normal equations lose it (they square the condition number); and
the exact per-block sums make 256-line-aligned shards bit-identical to one launch.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import spai_oracle as O

from .test_configs_gpu import _candidate, _lsq_vs_oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bits(removed_bool):
    """[K, E] bool -> [K, ceil(E/32)] int32 removal bitmaps on the device."""
    K, E = removed_bool.shape
    words = (E + 31) // 32
    pad = np.zeros((K, words * 32), bool)
    pad[:, :E] = removed_bool
    w = (pad.reshape(K, words, 32).astype(np.uint64) << np.arange(32, dtype=np.uint64)).sum(2).astype(np.uint32)
    return torch.from_numpy(w.view(np.int32)).to(DEV)


def _lines(A_sp, P_sp, n):
    Pc, Ac = P_sp.tocoo(), A_sp.tocoo()
    idx, act, _ = O.lines_from_coo(Pc.row, Pc.col, Pc.data, n, "col")
    a_idx, _, a_val = O.lines_from_coo(Ac.row, Ac.col, Ac.data.astype(np.float64), n, "col")
    return idx, act, a_idx, a_val


def _sp(t):
    c = t.coalesce()
    return sp.csr_matrix((c.values().double().numpy(), tuple(c.indices().numpy())), shape=tuple(c.shape))


@pytest.mark.parametrize("kind", ["2d", "3d13", "3d7"])
def test_qr_fill_vs_oracle_householder(kind):
    """fp64 stencils (2-D 5-point, 3-D with the 13-wide axial pattern, 3-D 7-point): every
    column's M within 1e-11 of the oracle's QR and the residual within 1e-11 of scipy's."""
    from gflownet_spai_amd import PreconditionerEnv, axial_pattern_3d, kernels, poisson_2d, poisson_3d
    if kind == "2d":
        A = poisson_2d(40, torch.float64)
        P = A
    else:
        A = poisson_3d(12)
        P = axial_pattern_3d(12) if kind == "3d13" else A
    n = A.shape[0]
    env = PreconditionerEnv(n, P, A, side="AM", fill="qr", keep_m=True)
    want_rows = {"2d": 13, "3d13": 55, "3d7": 25}[kind]
    assert env.qr_rows == want_rows
    A_sp, P_sp = _sp(A), _sp(P)
    idx, act, a_idx, a_val = _lines(A_sp, P_sp, n)
    rng = np.random.default_rng(7)
    E = env.init_nnz
    removed = rng.random((3, E)) < np.array([[0.0], [0.2], [0.5]])
    bits = _bits(removed)
    res2, m = kernels.fill_residual_qr(env.pattern, env.a_lines, env.qr_rows, bits, store_m=True,
                                       m_dtype=torch.float64)
    m = m.cpu().numpy()
    for b in range(3):
        keep = (idx >= 0) & ~removed[b][np.clip(act, 0, None)]
        m_ref = O.lsq_fill(idx, keep, a_idx, a_val)
        rel = np.linalg.norm(m[b] - m_ref) / np.linalg.norm(m_ref)
        assert rel < 1e-11, (b, rel)
        assert np.all(m[b][~keep] == 0)
        ref = O.residual_fro_fp64(A_sp.tocsc(), O.m_to_csc(idx, m[b], n, np.float64)) ** 2
        assert float(res2[b]) == pytest.approx(ref, rel=1e-11)
    # a few columns also against numpy lstsq directly
    A_csc = A_sp.tocsc()
    keep = (idx >= 0) & ~removed[1][np.clip(act, 0, None)]
    for j in (0, 1, n // 2, n - 1):
        mj, J = O.lsq_fill_lstsq(idx, keep, A_csc, j)
        slots = [p for p in range(idx.shape[1]) if keep[j, p]]
        np.testing.assert_allclose(m[1][j, slots], mj, rtol=1e-11, atol=1e-13)


def test_qr_and_gram_fills_agree_and_shards_are_exact():
    """On a well-conditioned stencil the QR fill and the normal-equations fill give the same M
    (1e-12) and residuals (1e-12); the QR fill's exact limbs over 256-line-aligned shards (any P)
    equal one launch bit for bit; the one-launch reward path equals the shard path."""
    from gflownet_spai_amd import PreconditionerEnv, kernels, poisson_2d
    from gflownet_spai_amd.distributed import LINE_ALIGN, shard_lines
    A = poisson_2d(96, torch.float64)
    n = A.shape[0]
    envq = PreconditionerEnv(n, A, A, side="AM", fill="qr", keep_m=True)
    envg = PreconditionerEnv(n, A, A, side="AM", fill="lsq", keep_m=True)
    rng = np.random.default_rng(3)
    removed = rng.random((5, envq.init_nnz)) < 0.3
    bits = _bits(removed)
    rq = envq.fill_partial(bits)
    mq = envq.last_m.clone()
    rg = envg.fill_partial(bits)
    np.testing.assert_allclose(rq.cpu().numpy(), rg.cpu().numpy(), rtol=1e-12)
    np.testing.assert_allclose(mq.cpu().numpy(), envg.last_m.cpu().numpy(), rtol=1e-11, atol=1e-13)
    for P in (2, 3, 7):
        lb = sum(envq.fill_partial(bits, *shard_lines(n, q, P, LINE_ALIGN), limbs=True) for q in range(P))
        assert torch.equal(kernels.res2_from_limbs(lb), rq)
    counts = torch.from_numpy(removed.sum(1).astype(np.int32)).to(DEV)
    rw = envq.fill_rewards(bits, counts, torch.tensor(0.5))
    assert torch.equal(envq.last_residual.double(), rq.sqrt())  # the same exact sums, one launch
    assert torch.equal(rw, envq.rewards_from_res2(rq, counts, torch.tensor(0.5)))


def test_qr_fill_ill_conditioned_matches_lstsq():
    """Nearly singular local blocks: A block-diagonal with dense 5 x 5 blocks ones + 1e-5 noise
    (pattern = A), so every line's block A[I, J] is one of them, condition ~1e5 - 1e7 (its normal
    equations ~1e10 - 1e14: the normal-equations fill drops the near-dependent columns of some
    blocks by its pivot floor and loses ~1e-4 on the others).  The QR fill matches numpy lstsq
    within 1e-6 (the north-star bar; ~cond x eps) on every line; the normal-equations fill is
    measured beside it."""
    from gflownet_spai_amd import PreconditionerEnv
    nb, w = 40, 5
    n = nb * w
    g = torch.Generator().manual_seed(5)
    blocks = 1.0 + 1e-5 * torch.randn(nb, w, w, generator=g, dtype=torch.float64)
    bi = torch.arange(nb).view(nb, 1, 1) * w
    rows = (bi + torch.arange(w).view(1, w, 1)).expand(nb, w, w).reshape(-1)
    cols = (bi + torch.arange(w).view(1, 1, w)).expand(nb, w, w).reshape(-1)
    A = torch.sparse_coo_tensor(torch.stack([rows, cols]), blocks.reshape(-1), (n, n))
    envq = PreconditionerEnv(n, A, A, side="AM", fill="qr", keep_m=True)
    envg = PreconditionerEnv(n, A, A, side="AM", fill="lsq", keep_m=True)
    assert envq.qr_rows == w
    bits = _bits(np.zeros((1, envq.init_nnz), bool))
    envq.fill_partial(bits)
    envg.fill_partial(bits)
    A_sp = _sp(A)
    idx, act, a_idx, a_val = _lines(A_sp, A_sp, n)
    keep = idx >= 0
    A_csc = A_sp.tocsc()
    mq, mg = envq.last_m[0].cpu().numpy(), envg.last_m[0].cpu().numpy()
    err_q = err_g = 0.0
    for j in range(n):
        mj, _ = O.lsq_fill_lstsq(idx, keep, A_csc, j)
        slots = [p for p in range(idx.shape[1]) if keep[j, p]]
        nr = np.linalg.norm(mj)
        err_q = max(err_q, np.linalg.norm(mq[j, slots] - mj) / nr)
        err_g = max(err_g, np.linalg.norm(mg[j, slots] - mj) / nr)
    assert err_q < 1e-6, err_q  # ~cond * eps: the worst block is near cond 1e8
    assert err_q < err_g, (err_q, err_g)


def test_qr_fill_c4_full_size_vs_oracle():
    """C4 1024^2 fp32 (the bench's configuration) with fill="qr": one throughput candidate's M
    over all 1,048,576 columns within 1e-6 of the oracle and ||AM - I||_F within 1e-6; the Gram
    fill's residual of the same candidate agrees within 1e-10."""
    from gflownet_spai_amd import PreconditionerEnv, poisson_2d
    A = poisson_2d(1024)
    n = A.shape[0]
    env = PreconditionerEnv(n, A, A, side="AM", fill="qr", keep_m=True)
    assert env.qr_rows == 13
    removed, log = _candidate(env, 1234)
    r, c, v, _ = O.poisson2d(1024)
    A_sp = sp.csr_matrix((v.astype(np.float64), (r, c)), shape=(n, n))
    _lsq_vs_oracle(env, A_sp, A_sp, removed)
    envg = PreconditionerEnv(n, A, A, side="AM", fill="lsq")
    res_g = envg.fill_partial(log.removed).sqrt()
    np.testing.assert_allclose(env.last_residual[:1].cpu().numpy(), res_g.cpu().numpy(), rtol=1e-10)


def _random_cols(n, k, seed, diag=None):
    """Sparse n x n COO with exactly k nonzeros per column: the diagonal (value ``diag``, default
    k + 1) and k - 1 distinct random rows (N(0, 1) values), so the row unions of k columns are
    nearly disjoint: |I| ~ k * WA (the wide-block QR instances)."""
    rng = np.random.default_rng(seed)
    rows = np.empty((n, k), np.int64)
    rows[:, 0] = np.arange(n)
    for j in range(n):
        o = rng.choice(n - 1, k - 1, replace=False)
        rows[j, 1:] = o + (o >= j)
    vals = rng.standard_normal((n, k))
    vals[:, 0] = k + 1.0 if diag is None else diag
    cols = np.repeat(np.arange(n), k)
    ind = torch.from_numpy(np.stack([rows.reshape(-1), cols]))
    # coalesced: the raw COO order (the env's action ids) is then the row-major order the oracle's
    # lines (built from scipy's CSR) number the entries by
    return torch.sparse_coo_tensor(ind, torch.from_numpy(vals.reshape(-1)), (n, n)).coalesce()


@pytest.mark.parametrize("kp,ka,lo,hi", [(5, 5, 17, 32), (7, 7, 33, 64), (13, 7, 65, 96)])
def test_qr_wide_row_unions_every_instance(kp, ka, lo, hi):
    """Random sparse A and pattern with nearly disjoint column supports, so the row unions |I| fall
    in the ranges of the larger group instances: <5,5,L8> (17-32 rows), <7,7,L16,NT128> (33-64) and
    <13,7,L32,RPL3> (65-96, the only group sum with the shfl_xor(16) step).  M from the fused kernel
    and from the R cache within 1e-10 of the oracle's QR; the residual vs scipy."""
    from gflownet_spai_amd import PreconditionerEnv, kernels
    n = 1500
    A = _random_cols(n, ka, 11)
    P = A if kp == ka else _random_cols(n, kp, 12)
    env = PreconditionerEnv(n, P, A, side="AM", fill="qr", keep_m=True)
    assert lo <= env.qr_rows <= hi, env.qr_rows
    assert env.rcache is not None  # (13-wide lines too: the cached solve re-reads R per sample)
    A_sp, P_sp = _sp(A), _sp(P)
    idx, act, a_idx, a_val = _lines(A_sp, P_sp, n)
    removed = np.random.default_rng(1).random((2, env.init_nnz)) < np.array([[0.0], [0.3]])
    bits = _bits(removed)
    outs = {"cached" if env.rcache is not None else "fused":
            kernels.fill_residual_qr(env.pattern, env.a_lines, env.qr_rows, bits, store_m=True,
                                     m_dtype=torch.float64, rcache=env.rcache)}
    outs["fused"] = kernels.fill_residual_qr(env.pattern, env.a_lines, env.qr_rows, bits, store_m=True,
                                             m_dtype=torch.float64)
    for name, (res2, m) in outs.items():
        m = m.cpu().numpy()
        for b in range(2):
            keep = (idx >= 0) & ~removed[b][np.clip(act, 0, None)]
            m_ref = O.lsq_fill(idx, keep, a_idx, a_val)
            rel = np.linalg.norm(m[b] - m_ref) / np.linalg.norm(m_ref)
            assert rel < 1e-10, (name, b, rel)
            ref = O.residual_fro_fp64(A_sp.tocsc(), O.m_to_csc(idx, m[b], n, np.float64)) ** 2
            assert float(res2[b]) == pytest.approx(ref, rel=1e-10), name


def test_qr_row_overflow_gives_nan():
    """A max_rows below the true largest |I| selects an instance too small for some lines: those
    lines' residual is NaN (the row-overflow path, rowl == -2), for the fused kernel and for an R
    cache built with the same wrong max_rows; never a silent wrong value."""
    from gflownet_spai_amd import PreconditionerEnv, kernels
    n = 600
    A = _random_cols(n, 5, 21)
    env = PreconditionerEnv(n, A, A, side="AM", fill="qr", keep_m=False)
    assert env.qr_rows > 16
    bits = _bits(np.zeros((1, env.init_nnz), bool))
    res2, _ = kernels.fill_residual_qr(env.pattern, env.a_lines, 16, bits)
    assert torch.isnan(res2).all()
    rc = kernels.qr_cache(env.pattern, env.a_lines, 16)
    res2c, _ = kernels.fill_residual_qr(env.pattern, env.a_lines, 16, bits, rcache=rc)
    assert torch.isnan(res2c).all()
    ok, _ = kernels.fill_residual_qr(env.pattern, env.a_lines, env.qr_rows, bits, rcache=env.rcache)
    assert torch.isfinite(ok).all()


@pytest.mark.parametrize("kind", ["2d", "3d7", "c5s", "3d13"])
def test_qr_cached_equals_fused(kind):
    """The R-cache path (phase 1 once per env, spai_fill_lines_qr_cached) against the fused kernel
    (phase 1 every call): the same reflections on the same numbers, only the rank floor's column
    norms are recomputed from R, so M and the residuals agree to rounding (1e-13) — and the cached
    path's exact per-block sums make 256-line-aligned shards bit-identical to one launch."""
    from gflownet_spai_amd import PreconditionerEnv, axial_pattern_3d, kernels, poisson_2d, poisson_3d, thermal_like
    from gflownet_spai_amd.distributed import LINE_ALIGN, shard_lines
    A = {"2d": lambda: poisson_2d(80, torch.float32), "3d7": lambda: poisson_3d(14), "3d13": lambda: poisson_3d(12),
         "c5s": lambda: thermal_like(40, 0, torch.float64)}[kind]()
    P = axial_pattern_3d(12) if kind == "3d13" else A  # 3d13: the C3 geometry (13-wide lines, cached solve)
    n = A.shape[0]
    envc = PreconditionerEnv(n, P, A, side="AM", fill="qr", keep_m=True)
    envf = PreconditionerEnv(n, P, A, side="AM", fill="qr", keep_m=True, rcache=False)
    assert envc.pattern.width == (13 if kind == "3d13" else envc.pattern.width)
    assert envc.rcache is not None and envf.rcache is None and envc.gram is None
    removed = np.random.default_rng(4).random((9, envc.init_nnz)) < 0.25  # 9: a chunk of 8 + 1
    bits = _bits(removed)
    rc = envc.fill_partial(bits)
    rf = envf.fill_partial(bits)
    np.testing.assert_allclose(rc.cpu().numpy(), rf.cpu().numpy(), rtol=1e-13)
    np.testing.assert_allclose(envc.last_m.cpu().numpy(), envf.last_m.cpu().numpy(), rtol=1e-12, atol=1e-14)
    for P in (2, 3):
        lb = sum(envc.fill_partial(bits, *shard_lines(n, q, P, LINE_ALIGN), limbs=True) for q in range(P))
        assert torch.equal(kernels.res2_from_limbs(lb), rc)
    counts = torch.from_numpy(removed.sum(1).astype(np.int32)).to(DEV)
    rw = envc.fill_rewards(bits, counts, torch.tensor(0.5))
    assert torch.equal(envc.last_residual.double(), rc.sqrt())
    assert torch.equal(rw, envc.rewards_from_res2(rc, counts, torch.tensor(0.5)))


@pytest.mark.parametrize("B", [1, 3])
def test_qr_cached_narrow_lines_and_small_batches(B):
    """A 1-D Laplacian (3-wide lines inside the 5-wide class: slots 3-4 are padding) with B = 1 and
    3 (partial sample chunks), over a line range that starts and ends inside 256-line blocks: the
    R-cache solve against the oracle's QR (1e-11) and the fused kernel (1e-13)."""
    from gflownet_spai_amd import PreconditionerEnv, kernels
    n = 1000
    i = torch.arange(n)
    rows = torch.cat([i, i[1:], i[:-1]])
    cols = torch.cat([i, i[:-1], i[1:]])
    vals = torch.cat([torch.full((n,), 2.0), torch.full((n - 1,), -1.0), torch.full((n - 1,), -1.0)]).double()
    A = torch.sparse_coo_tensor(torch.stack([rows, cols]), vals, (n, n)).coalesce()
    env = PreconditionerEnv(n, A, A, side="AM", fill="qr", keep_m=True)
    assert env.pattern.width == 3 and env.rcache is not None
    A_sp = _sp(A)
    idx, act, a_idx, a_val = _lines(A_sp, A_sp, n)
    removed = np.random.default_rng(9).random((B, env.init_nnz)) < 0.3
    bits = _bits(removed)
    lb, le = 256, 900  # a 256-aligned shard start, an end inside a block
    res_c, m_c = kernels.fill_residual_qr(env.pattern, env.a_lines, env.qr_rows, bits, lb, le, store_m=True,
                                          m_dtype=torch.float64, rcache=env.rcache)
    res_f, m_f = kernels.fill_residual_qr(env.pattern, env.a_lines, env.qr_rows, bits, lb, le, store_m=True,
                                          m_dtype=torch.float64)
    np.testing.assert_allclose(res_c.cpu().numpy(), res_f.cpu().numpy(), rtol=1e-13)
    np.testing.assert_allclose(m_c.cpu().numpy(), m_f.cpu().numpy(), rtol=1e-12, atol=1e-14)
    for b in range(B):
        keep = (idx >= 0) & ~removed[b][np.clip(act, 0, None)]
        m_ref = O.lsq_fill(idx, keep, a_idx, a_val, np.arange(lb, le))
        got = m_c[b].cpu().numpy()
        assert np.linalg.norm(got - m_ref) / np.linalg.norm(m_ref) < 1e-11


@pytest.mark.parametrize("kind", ["2d", "3d7", "1d", "random"])
def test_qr_dict_equals_full_cache(kind):
    """The R cache held as its dictionary (spai_line_cache_dict: the distinct line entries + each
    line's entry) against the full cache: the same values reach the same arithmetic, so M, the
    residual sums and the rewards are bit-identical, on one launch and on 256-line-aligned shards.
    Stencils have a handful of distinct entries (the interior lines share one); a random matrix
    has one per line and keeps the full cache."""
    from gflownet_spai_amd import PreconditionerEnv, kernels, poisson_2d, poisson_3d
    from gflownet_spai_amd.distributed import LINE_ALIGN, shard_lines
    if kind == "1d":
        n = 1000
        i = torch.arange(n)
        A = torch.sparse_coo_tensor(torch.stack([torch.cat([i, i[1:], i[:-1]]), torch.cat([i, i[:-1], i[1:]])]),
                                    torch.cat([torch.full((n,), 2.0), torch.full((2 * n - 2,), -1.0)]).double(),
                                    (n, n)).coalesce()
    elif kind == "random":
        A = _random_cols(1500, 5, 31)
    else:
        A = {"2d": lambda: poisson_2d(80, torch.float32), "3d7": lambda: poisson_3d(14)}[kind]()
    n = A.shape[0]
    envd = PreconditionerEnv(n, A, A, side="AM", fill="qr", keep_m=True)
    envf = PreconditionerEnv(n, A, A, side="AM", fill="qr", keep_m=True, cache_dict=False)
    assert torch.is_tensor(envf.rcache)
    if kind == "random":
        assert torch.is_tensor(envd.rcache)  # one entry per line: no dictionary
        return
    assert isinstance(envd.rcache, kernels.QrDict)
    assert envd.rcache.entries <= {"2d": 40, "3d7": 150, "1d": 6}[kind], envd.rcache.entries
    assert kernels.rcache_nbytes(envd.rcache) < kernels.rcache_nbytes(envf.rcache) / 4
    removed = np.random.default_rng(6).random((9, envd.init_nnz)) < 0.25
    bits = _bits(removed)
    rd, rf = envd.fill_partial(bits), envf.fill_partial(bits)
    assert torch.equal(rd, rf)
    assert torch.equal(envd.last_m, envf.last_m)
    for P in (2, 3):
        for q in range(P):
            lb, le = shard_lines(n, q, P, LINE_ALIGN)
            assert torch.equal(envd.fill_partial(bits, lb, le, limbs=True), envf.fill_partial(bits, lb, le, limbs=True))
    counts = torch.from_numpy(removed.sum(1).astype(np.int32)).to(DEV)
    assert torch.equal(envd.fill_rewards(bits, counts, torch.tensor(0.5)),
                       envf.fill_rewards(bits, counts, torch.tensor(0.5)))
    assert torch.equal(envd.last_m, envf.last_m)
