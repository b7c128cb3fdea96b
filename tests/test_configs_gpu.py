"""BASELINE.json configs on the GPU at their full sizes (VERDICT r1 "configs untested"):

  C2  256^2 5-pt fp32: the reference's own residuals / rewards (golden G4) on both sides
  C3  64^3 7-pt fp64 with the 13-wide axial candidate pattern (nnz/col <= 13): one throughput
      candidate's LSQ fill over all 262,144 columns and ||AM - I||_F vs the fp64 oracle
  C4  1024^2 5-pt fp32: one throughput candidate's LSQ fill over all 1,048,576 columns and
      ||AM - I||_F vs the oracle (the bench's configuration)
  plus assemble() against the reference's own assembled M (golden G7).

Tolerances (north star): M values within 1e-6 relative Frobenius error (fp32 storage) /
1e-11 (fp64), ||AM - I||_F within 1e-6 relative; index sets bit-exact.  The oracle's LSQ is
a stacked Householder QR in fp64 (oracle/spai_oracle.py lsq_fill), evaluated in column
chunks; its residual is scipy's A @ M in fp64.
"""
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import spai_oracle as O

from .conftest import GOLDEN
from .test_hip_parity import FixedLogits

pytestmark = pytest.mark.gpu
DEV = "cuda"


def removal_bits(removed_bool):
    words = (removed_bool.size + 31) // 32
    bits = np.zeros(words, np.uint32)
    ids = np.flatnonzero(removed_bool)
    np.bitwise_or.at(bits, ids >> 5, (np.uint32(1) << (ids & 31).astype(np.uint32)))
    return torch.from_numpy(bits.view(np.int32).reshape(1, words)).to(DEV)


def test_c2_reference_residuals_and_rewards_on_gpu():
    """C2 (golden G4): r0 and three removal sets (0 %, 5 %, 20 %), ||MA - I|| (reference side)
    and ||M^T A - I|| (= ||A M - I||, AM side) and the reference's reward at alpha 0.5."""
    from gflownet_spai_amd import PreconditionerEnv, poisson_2d
    case = json.load(open(os.path.join(GOLDEN, "meta.json")))["cases"]["c2_residual"]
    A = poisson_2d(256)
    n = 256 * 256
    for side, key in (("MA", "r_ma"), ("AM", "r_mta")):
        env = PreconditionerEnv(n, A, A, side=side)
        assert env.init_nnz == case["E"]
        assert float(env.orig_residual) == pytest.approx(case["r0"], rel=1e-15)
        for k, st in enumerate(case["sets"]):
            frac = float(st["recipe"].split("<")[1])
            removed = np.random.default_rng(1000 + k).random(env.init_nnz) < frac
            assert int(removed.sum()) == st["n_removed"]
            counts = torch.tensor([st["n_removed"]], dtype=torch.int32, device=DEV)
            rw = env.rewards_from_removed(removal_bits(removed), counts, torch.tensor(0.5))
            assert float(env.last_residual[0]) == pytest.approx(st[key], rel=1e-15)
            if side == "MA":
                assert float(rw[0]) == pytest.approx(st["reward"][0], rel=1e-12, abs=1e-12)


def _lsq_vs_oracle(env, A_sp, pat_sp, removed_row, chunk=65536, tol=1e-6):
    """Whole-matrix comparison of the env's stored M (sample 0) and residual with the oracle."""
    n = A_sp.shape[0]
    Pc, Ac = pat_sp.tocoo(), A_sp.tocoo()
    idx, act, _ = O.lines_from_coo(Pc.row, Pc.col, Pc.data, n, "col")
    a_idx, _, a_val = O.lines_from_coo(Ac.row, Ac.col, Ac.data.astype(np.float64), n, "col")
    keep = (idx >= 0) & ~removed_row[np.clip(act, 0, None)]
    m_gpu = env.last_m[0].cpu().numpy()
    num = den = 0.0
    for c0 in range(0, n, chunk):
        ids = np.arange(c0, min(c0 + chunk, n))
        m_ref = O.lsq_fill(idx, keep, a_idx, a_val, ids)
        num += float(((m_gpu[ids].astype(np.float64) - m_ref) ** 2).sum())
        den += float((m_ref ** 2).sum())
    rel = np.sqrt(num / den)
    assert rel < tol, rel
    # removed slots hold exactly 0 and the index set of M is the kept pattern
    assert np.all(m_gpu[~keep] == 0)
    res = O.residual_fro_fp64(A_sp.tocsc().astype(np.float64), O.m_to_csc(idx, m_gpu, n, m_gpu.dtype))
    assert float(env.last_residual[0]) == pytest.approx(res, rel=1e-6)
    return rel, res


def _candidate(env, seed, frac=0.2):
    """One throughput candidate with the bench's logits recipe (20 % expected removal)."""
    import bench
    from gflownet_spai_amd import GFlowNet
    E = env.num_actions - 1
    logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
    logits[E] = bench.terminal_logit(logits[:E].numpy(), frac)
    g = GFlowNet(FixedLogits(logits), None, env, mode="throughput", seed=seed)
    log = g.sample_states([env.matrix], return_log=True)
    bits = log.removed[0].cpu().numpy().view(np.uint32)
    removed = ((bits[:, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(-1)[:E].astype(bool)
    assert int(log.counts[0]) == int(removed.sum())
    return removed, log


def test_c4_lsq_fill_full_size_vs_oracle():
    """C4 1024^2 fp32 (BASELINE's metric config): one candidate's M over all 1,048,576
    columns within 1e-6 relative Frobenius error and ||AM - I||_F within 1e-6."""
    from gflownet_spai_amd import PreconditionerEnv, poisson_2d
    A = poisson_2d(1024)
    n = A.shape[0]
    env = PreconditionerEnv(n, A, A, side="AM", fill="lsq", keep_m=True)
    removed, _ = _candidate(env, 1234)
    r, c, v, _ = O.poisson2d(1024)
    A_sp = sp.csr_matrix((v.astype(np.float64), (r, c)), shape=(n, n))
    _lsq_vs_oracle(env, A_sp, A_sp, removed)


def test_c3_lsq_fill_13_wide_fp64_vs_oracle():
    """C3 64^3 7-pt fp64 with the 13-wide axial candidate pattern (|J| <= 13,
    |I| <= 37): one candidate's M over all 262,144 columns and ||AM - I||_F vs the oracle.
    The integer stencil's Gram cache round-trips through fp32, so the env streams it as fp32:
    the fill from the fp64 cache gives the same bits."""
    from gflownet_spai_amd import PreconditionerEnv, axial_pattern_3d, kernels, poisson_3d
    A = poisson_3d(64)
    P = axial_pattern_3d(64)
    n = A.shape[0]
    env = PreconditionerEnv(n, P, A, side="AM", fill="lsq", keep_m=True)
    assert env.pattern.width == 13 and env.gram is not None and env.gram.dtype == torch.float32
    removed, log = _candidate(env, 77)
    assert env.last_m.dtype == torch.float64
    g64 = kernels.gram_build(env.pattern, env.a_lines)
    res64, m64 = kernels.fill_residual_gram(env.pattern, g64, log.removed, True, store_m=True, m_dtype=torch.float64)
    assert torch.equal(m64, env.last_m)
    np.testing.assert_allclose(res64.double().sqrt().cpu().numpy(), env.last_residual.double().cpu().numpy(),
                               rtol=1e-15)
    Ai, Pi = A.coalesce(), P.coalesce()
    A_sp = sp.csr_matrix((Ai.values().numpy(), tuple(Ai.indices().numpy())), shape=(n, n))
    P_sp = sp.coo_matrix((Pi.values().numpy(), tuple(Pi.indices().numpy())), shape=(n, n))
    _lsq_vs_oracle(env, A_sp, P_sp, removed, tol=1e-11)


@pytest.mark.parametrize("m_dtype", [torch.float32, torch.float64])
def test_c3_wide_fill_fp32_and_fp64_gram_caches_bit_identical_over_shards(m_dtype):
    """C3's 13-wide LSQ fill (k_gram_fill_wide: fixed-count buffer stores of M, B = 10 = two
    sample chunks) from the env's fp32 Gram cache and from the fp64 cache of the same integer
    stencil: M and the residuals bit-identical, for fp32 and fp64 M, over the whole matrix and
    over 256-line-aligned shards (partial last blocks, line_begin > 0, M blocks that end inside a
    16-byte store) whose exact limbs sum to the one-launch bits."""
    from gflownet_spai_amd import PreconditionerEnv, axial_pattern_3d, kernels, poisson_3d
    from gflownet_spai_amd.distributed import LINE_ALIGN, shard_lines
    A = poisson_3d(64)
    P = axial_pattern_3d(64)
    n = A.shape[0]
    env = PreconditionerEnv(n, P, A, side="AM", fill="lsq")
    assert env.gram.dtype == torch.float32
    g64 = kernels.gram_build(env.pattern, env.a_lines)
    E = env.init_nnz
    rng = np.random.default_rng(91)
    rem = rng.random((10, E)) < rng.uniform(0.05, 0.5, (10, 1))
    bits = torch.cat([removal_bits(r) for r in rem])  # B = 10: two chunks of samples
    r32, m32 = kernels.fill_residual_gram(env.pattern, env.gram, bits, True, store_m=True, m_dtype=m_dtype)
    r64, m64 = kernels.fill_residual_gram(env.pattern, g64, bits, True, store_m=True, m_dtype=m_dtype)
    assert torch.equal(m32, m64) and torch.equal(r32, r64)
    for nparts in (3, 7):
        lb = 0
        for q in range(nparts):
            b, e = shard_lines(n, q, nparts, LINE_ALIGN)
            limbs, ms = kernels.fill_residual_gram(env.pattern, env.gram, bits, True, b, e, store_m=True,
                                                   m_dtype=m_dtype, limbs=True)
            assert torch.equal(ms, m64[:, b:e])
            lb = lb + limbs
        assert torch.equal(kernels.res2_from_limbs(lb), r64)


def test_c5_standin_lsq_fill_full_size_vs_oracle():
    """C5 stand-in (utils.thermal_like(1108): 1,227,664 unknowns, 8,584,786 nnz, 7 per row,
    lognormal conductivities, permuted numbering, fp64; thermal2 itself is not in the
    container): one candidate's LSQ M over all columns and ||AM - I||_F vs the oracle."""
    from gflownet_spai_amd import PreconditionerEnv, thermal_like
    A = thermal_like(1108)
    n = A.shape[0]
    env = PreconditionerEnv(n, A, A, side="AM", fill="lsq", keep_m=True)
    assert env.pattern.width == 7 and env.gram is not None and env.gram.dtype == torch.float64
    removed, _ = _candidate(env, 4321)
    Ai = A.coalesce()
    A_sp = sp.csr_matrix((Ai.values().numpy(), tuple(Ai.indices().numpy())), shape=(n, n))
    _lsq_vs_oracle(env, A_sp, A_sp, removed, tol=1e-9)


@pytest.mark.parametrize("fill", ["copy", "lsq"])
def test_assemble_matches_reference_m(fill):
    """assemble() returns update_edges_and_convert_to_sparse's M (golden G7: the reference's
    coalesced indices and fp32 values of three removal sets): COPY bit-exact; LSQ on the same
    index set with the fitted values."""
    from gflownet_spai_amd import PreconditionerEnv, kernels
    d = np.load(os.path.join(GOLDEN, "c1p_removal.npz"))
    g = np.load(os.path.join(GOLDEN, "c1p_assembled.npz"))
    n = int(d["n"])
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([d["rows"], d["cols"]]).astype(np.int64)),
                                torch.from_numpy(d["vals"]), (n, n))
    env = PreconditionerEnv(n, A, A, side="MA", fill=fill, keep_m=True)
    E = env.init_nnz
    sets = [int(k) for k in g["sets"]]
    acts = torch.from_numpy(np.where(d["removed"][sets], np.arange(E), -1))
    removed, counts = kernels.actions_to_removed(acts.to(DEV), E)
    env.rewards_from_removed(removed, counts, 0.5)
    off = 0
    for b, nnz in enumerate(g["nnz"]):
        M = env.assemble(b)
        assert M.is_coalesced() and M._nnz() == nnz
        assert np.array_equal(M.indices().cpu().numpy(), g["indices"][:, off:off + nnz])
        if fill == "copy":
            assert np.array_equal(M.values().cpu().numpy(), g["values"][off:off + nnz])
        off += nnz


def test_wide_fill_badly_scaled_columns_per_pivot_floor():
    """13-wide LSQ fill (k_gram_fill_wide) on a 3-D Laplacian whose every 5th column is scaled by
    1e-7 (G_kk ~ 1e-14 of its neighbours): the pivot floor is per pivot (1e-13 G_kk, as the
    narrow Gram kernel and fill.hip's k_line), so the small columns are solved, not dropped —
    M and ||AM - I||_F match the QR oracle.  (A floor relative to the line's largest diagonal
    would zero those slots.)"""
    from gflownet_spai_amd import PreconditionerEnv, axial_pattern_3d, kernels, poisson_3d
    grid = 10
    A0 = poisson_3d(grid).coalesce()
    n = A0.shape[0]
    scale = np.where(np.arange(n) % 5 == 0, 1e-7, 1.0)
    r, c = A0.indices().numpy()
    v = A0.values().numpy() * scale[c]
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([r, c])), torch.from_numpy(v), (n, n))
    P = axial_pattern_3d(grid)
    env = PreconditionerEnv(n, P, A, side="AM", fill="lsq", keep_m=True)
    assert env.pattern.width == 13 and env.gram is not None and env.gram.dtype == torch.float64
    E = env.init_nnz
    rng = np.random.default_rng(8)
    removed = rng.random(E) < 0.2
    acts = torch.from_numpy(np.where(removed, np.arange(E), -1))
    rb, counts = kernels.actions_to_removed(acts.view(1, -1).to(DEV), E)
    env.rewards_from_removed(rb, counts, 0.5)
    A_sp = sp.csr_matrix((v, (r, c)), shape=(n, n))
    Pi = P.coalesce()
    P_sp = sp.coo_matrix((Pi.values().numpy(), tuple(Pi.indices().numpy())), shape=(n, n))
    _lsq_vs_oracle(env, A_sp, P_sp, removed, tol=1e-8)


def test_rollouts_counter_is_the_device_stream_id():
    """GFlowNet.rollouts reads the device stream counter (graph replays advance it without the
    host) and setting it re-seeds the device counter: a replayed stream id draws the same
    removal sets again."""
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, poisson_2d
    A = poisson_2d(32)
    env = PreconditionerEnv(A.shape[0], A, A, side="AM", fill="lsq")
    E = env.num_actions - 1
    logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(4))
    logits[E] = 2.5
    g = GFlowNet(FixedLogits(logits), None, env, mode="throughput", seed=3)
    assert g.rollouts == 0
    logs = [g.sample_states([A] * 2, return_log=True) for _ in range(3)]
    assert g.rollouts == 3
    g.rollouts = 1
    again = g.sample_states([A] * 2, return_log=True)
    assert g.rollouts == 2
    assert torch.equal(again.removed, logs[1].removed) and not torch.equal(again.removed, logs[0].removed)
