"""HIP path (through the C ABI) vs the reference's golden vectors and the CPU oracle.

Bar: bit-exact for index work (sampled actions, removed sets, counts, orders); floats
within 1e-6 relative (north-star tolerance) unless the arithmetic is exact (integer
stencils in fp64: residuals of copy-filled Poisson matrices are exact).
"""
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import spai_oracle as O

from .conftest import GOLDEN

pytestmark = pytest.mark.gpu

DEV = "cuda"


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def coo(rows, cols, vals, n):
    return torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cols]).astype(np.int64)), torch.from_numpy(vals),
                                   (n, n))


class FixedLogits(torch.nn.Module):
    """Stand-in policy with the reference ForwardPolicy call contract (as in make_golden.py)."""

    def __init__(self, logits):
        super().__init__()
        self.l = torch.nn.Parameter(torch.as_tensor(logits).view(1, -1).clone())
        self.alpha = torch.nn.Parameter(torch.tensor(0.0))

    def logits(self, data):
        return self.l.to(DEV), torch.sigmoid(self.alpha).to(DEV)

    def forward(self, data, actions):
        x = self.l
        if actions.numel():
            m = torch.zeros_like(x, dtype=torch.bool)
            m[:, actions] = True
            x = x.masked_fill(m, float("-inf"))
        return torch.softmax(x, 1), torch.sigmoid(self.alpha)


def test_library_loaded_from_tree():
    from gflownet_spai_amd import _lib
    lib = _lib.load()
    assert lib.spai_abi_version() == _lib.ABI_VERSION
    assert os.path.dirname(_lib.LIB_PATH).endswith("gflownet_spai_amd")


@pytest.mark.parametrize("seed", range(4))
def test_parity_rollout_bit_exact_vs_reference(seed):
    from gflownet_spai_amd import BackwardPolicy, GFlowNet, PreconditionerEnv, trajectory_balance_loss
    d = load(f"c1_rollout_s{seed}.npz")
    n, B = int(d["n"]), int(d["B"])
    A = coo(d["rows"], d["cols"], d["vals"], n)
    env = PreconditionerEnv(n, A, A)
    E = env.num_actions - 1
    pol = FixedLogits(d["logits"])
    torch.manual_seed(0)
    bwd = BackwardPolicy(1, 4, E + 1).to(DEV)
    g = GFlowNet(pol, bwd, env, mode="parity")
    torch.manual_seed(int(d["seed"]))
    log = g.sample_states([A.clone() for _ in range(B)], return_log=True)
    assert np.array_equal(log.actions.cpu().numpy(), d["actions"])
    with torch.no_grad():
        np.testing.assert_allclose(log.fwd_probs.cpu().numpy(), d["fwd_probs"], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(log.rewards.cpu().numpy(), d["rewards"], rtol=1e-6)
    assert len(log._actions) == d["actions"].shape[0]
    loss = trajectory_balance_loss(log.total_flow, log.rewards, log.fwd_probs, log.back_probs)
    assert float(loss) == pytest.approx(float(d["loss"]), rel=1e-5)
    loss.backward()
    gref = d["logits_grad"]
    np.testing.assert_allclose(pol.l.grad.view(-1).numpy(), gref, rtol=2e-4, atol=2e-6 * np.abs(gref).max())


@pytest.mark.parametrize("name", ["c2_rollout.npz", "c4_rollout.npz", "c2long_rollout.npz", "longer_rollout.npz"])
def test_parity_rollout_bit_exact_vs_reference_large(name):
    """C2 (E = 326,656) and C4 (E = 5,238,784) reference rollouts (G6, make_golden.py g6), a
    LONG C2 rollout (G8: T = 4,605 steps, make_golden.py g8) and a 25,633-step rollout of the 72^2
    matrix (G9, make_golden.py g9: both samples remove all 25,632 actions, then the terminal —
    every step of the remaining-mass chain down to the last action): the HIP parity step reproduces the
    reference's actions from the same torch seed, its fwd_probs within 1e-6 and its rewards
    (copy fill, ||MA - I||).  The kernel ranks w_a / q_a with w_a = e^(l_a - lmax) instead of the
    reference's renormalised fp32 softmax p_a (a flip needs the two best ratios
    within ~3 ulp, ~1e-7 per step)."""
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, poisson_2d
    from .test_oracle_golden import large_rollout_logits
    d = load(name)
    grid, B = int(d["grid"]), int(d["B"])
    A = poisson_2d(grid)
    n = grid * grid
    env = PreconditionerEnv(n, A, A)
    logits = large_rollout_logits(d)
    assert env.num_actions == logits.numel()
    g = GFlowNet(FixedLogits(logits), None, env, mode="parity")
    torch.manual_seed(int(d["seed"]))
    log = g.sample_states([A.clone() for _ in range(B)], return_log=True)
    assert np.array_equal(log.actions.cpu().numpy(), d["actions"])
    with torch.no_grad():
        np.testing.assert_allclose(log.fwd_probs.cpu().numpy(), d["fwd_probs"], rtol=1e-6, atol=1e-12)
    np.testing.assert_allclose(log.rewards.cpu().numpy(), d["rewards"], rtol=1e-6)


@pytest.mark.parametrize("name", ["c1_removal.npz", "c1p_removal.npz", "rand64_removal.npz"])
def test_env_update_vs_reference(name):
    """PreconditionerEnv.update (copy fill) on both sides vs the reference and the fp64 oracle."""
    from gflownet_spai_amd import PreconditionerEnv
    d = load(name)
    n = int(d["n"])
    A = coo(d["rows"], d["cols"], d["vals"], n)
    Acsr = sp.csr_matrix((d["vals"].astype(np.float64), (d["rows"], d["cols"])), shape=(n, n))
    symmetric = abs(Acsr - Acsr.T).max() == 0
    exact = name != "rand64_removal.npz"  # integer stencils: every residual is exact in fp64
    removed = d["removed"]
    K = removed.shape[0]
    for side in ("MA", "AM"):
        env = PreconditionerEnv(n, A, A, side=side)
        E = env.num_actions - 1
        assert env.orig_flops == int(d["f0"]) and env.num_actions == int(d["num_actions"])
        assert float(env.orig_residual) == pytest.approx(float(d["r0"]), rel=0 if exact else 1e-6)
        T = max(int(removed.sum(1).max()), 1)
        acts = -np.ones((K, T + 1), np.int64)
        for k in range(K):
            ids = np.flatnonzero(removed[k])
            acts[k, :ids.size] = np.random.default_rng(k).permutation(ids)
            acts[k, ids.size] = E  # the terminal id is ignored (utils.py:323)
        for ia, al in enumerate(d["alphas"]):
            alpha = torch.tensor(al, dtype=torch.float32)
            rw = torch.stack(env.update(None, torch.from_numpy(acts), alpha)).cpu().numpy()
            res = env.last_residual.cpu().numpy()
            for k in range(K):
                mr, mc, mv = O.copy_fill_coo(d["rows"], d["cols"], d["vals"], removed[k], n)
                M = sp.csr_matrix((mv.astype(np.float64), (mr, mc)), shape=(n, n))
                ref64 = O.residual_fro_fp64(M, Acsr) if side == "MA" else O.residual_fro_fp64(Acsr, M)
                assert res[k] == pytest.approx(ref64, rel=1e-13, abs=1e-13)
                golden = d["r_ma"][k] if side == "MA" else (d["r_mta"][k] if symmetric else None)
                if golden is not None:
                    assert res[k] == pytest.approx(golden, rel=0 if exact else 1e-6)
                # reward formula + type promotion, bit-for-bit on our own residual
                want = O.reward(res[k], len(mr), alpha, float(env.orig_residual), env.orig_flops, n)
                assert rw[k] == pytest.approx(want, rel=1e-15, abs=1e-12)
                if side == "MA" and exact:
                    assert rw[k] == pytest.approx(d["reward"][k, ia], rel=1e-12, abs=1e-9)


def test_calculate_residual_and_reward_api():
    from gflownet_spai_amd import PreconditionerEnv
    d = load("c1_removal.npz")
    n = int(d["n"])
    A = coo(d["rows"], d["cols"], d["vals"], n)
    env = PreconditionerEnv(n, A, A)
    k = 20
    mr, mc, mv = O.copy_fill_coo(d["rows"], d["cols"], d["vals"], d["removed"][k], n)
    M = coo(mr, mc, mv, n)
    assert float(env.calculate_residual(M, A)) == d["r_ma"][k]
    r = env.reward(M, 5, torch.tensor(0.5))
    assert float(r) == pytest.approx(d["reward"][k, 0], rel=1e-12)
    assert env.matrix_flops(M) == (len(mr) * n * 2, len(mr))


@pytest.mark.parametrize("E,B,seed,stream", [(1216, 4, 0, 0), (1216, 3, 5, 9), (40, 2, 1, 0), (5000, 7, 2**40 + 3, 2**33 + 1)])
def test_throughput_rollout_bit_exact_vs_oracle(E, B, seed, stream):
    from gflownet_spai_amd import kernels
    rng = np.random.default_rng(E + B)
    logits = rng.standard_normal(E + 1).astype(np.float32)
    logits[E] = 3.5
    lg, lmax, z = kernels.logits_stats(torch.from_numpy(logits).to(DEV), B)
    removed, counts, ws = kernels.rollout_select(lg, B, lmax, seed, stream, sample_base=3)
    actions, fwd, t_dev = kernels.rollout_order(lg, B, lmax, counts, ws)
    counts_h = counts.cpu()
    T = int(t_dev)
    assert T == int(counts_h.max()) + 1
    actions, fwd = actions[:, :T], fwd[:, :T]
    r_o, a_o, f_o, c_o = O.throughput_rollout(logits, B, seed, stream, sample_base=3)
    assert np.array_equal(counts_h.numpy(), c_o)
    bits = removed.cpu().numpy().view(np.uint32)
    got = ((bits[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(B, -1)[:, :E].astype(bool)
    assert np.array_equal(got, r_o)
    assert np.array_equal(actions.cpu().numpy(), a_o.T)
    np.testing.assert_allclose(fwd.cpu().numpy(), f_o, rtol=1e-6)


def test_throughput_rollout_clustered_keys_overflow_path():
    """Keys clustered in a tiny part of the key range (one huge logit) overfill the MSD
    buckets; the exact rank-counting fallback must still give the oracle's order."""
    from gflownet_spai_amd import kernels
    E, B = 20000, 2
    logits = np.zeros(E + 1, np.float32)
    logits[7] = 1e30
    lg, lmax, z = kernels.logits_stats(torch.from_numpy(logits).to(DEV), B)
    removed, counts, ws = kernels.rollout_select(lg, B, lmax, 99, 1)
    actions, fwd, t_dev = kernels.rollout_order(lg, B, lmax, counts, ws)
    T = int(t_dev)
    r_o, a_o, f_o, c_o = O.throughput_rollout(logits, B, 99, 1)
    assert c_o.max() > 4096  # more winners than one 4096-record presample bucket
    assert np.array_equal(counts.cpu().numpy(), c_o)
    assert np.array_equal(actions[:, :T].cpu().numpy(), a_o.T)
    np.testing.assert_allclose(fwd[:, :T].cpu().numpy(), f_o, rtol=1e-6)


def test_throughput_rollout_tied_keys_oversized_bucket():
    """All 20,000 actions win with one and the same fp32 key (logit 1e30 swamps its Gumbel
    noise; the terminal's 9.9e29 loses to it) and fall into one bucket beyond k_sort2's
    8192-record LDS capacity: the k_sort2 block that meets it sorts it in global memory (ties by action id,
    as the oracle).  The terminal's own probability is 0/0 in both and is not compared."""
    from gflownet_spai_amd import kernels
    E, B = 20000, 2
    logits = np.full(E + 1, 1e30, np.float32)
    logits[E] = 9.9e29
    lg, lmax, z = kernels.logits_stats(torch.from_numpy(logits).to(DEV), B)
    removed, counts, ws = kernels.rollout_select(lg, B, lmax, 5, 3)
    actions, fwd, t_dev = kernels.rollout_order(lg, B, lmax, counts, ws)
    T = int(t_dev)
    big = ws_word(ws, E, B, 0)
    assert big == B  # the big path ran for every sample (one oversized bucket each)
    r_o, a_o, f_o, c_o = O.throughput_rollout(logits, B, 5, 3)
    assert (c_o == E).all()
    assert np.array_equal(counts.cpu().numpy(), c_o)
    assert np.array_equal(actions[:, :T].cpu().numpy(), a_o.T)
    np.testing.assert_allclose(fwd[:, :T - 1].cpu().numpy(), f_o[:, :T - 1], rtol=1e-6)
    # the order phase is idempotent: a second call on the same select lists each oversized
    # bucket once again (not twice) and reproduces the trajectory exactly
    actions2, fwd2, t2 = kernels.rollout_order(lg, B, lmax, counts, ws)
    assert ws_word(ws, E, B, 0) == B and int(t2) == T
    assert torch.equal(actions2[:, :T], actions[:, :T]) and torch.equal(fwd2[:, :T - 1], fwd[:, :T - 1])


def ws_word(ws, E, B, field):
    """int32 diagnostic word of the rollout workspace at the offset the library reports."""
    from gflownet_spai_amd import _lib
    off = _lib.load().spai_rollout_ws_offset(E, B, field)
    assert off >= 0 and off % 4 == 0
    return int(ws[off:off + 4].view(torch.int32)[0])


def test_full_size_c4_rollout_vs_oracle():
    """BASELINE's 1024^2 action space (E = 5,238,784) with the bench's logits: the removed set,
    the whole ordered trajectory and its probabilities of sample 0 vs the oracle."""
    from gflownet_spai_amd import kernels
    import bench
    E, B = 5238784, 2
    logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
    logits[E] = bench.terminal_logit(logits[:E].numpy(), 0.2)
    lg, lmax, z = kernels.logits_stats(logits.to(DEV), B)
    removed, counts, ws = kernels.rollout_select(lg, B, lmax, 1234, 0)
    actions, fwd, t_dev = kernels.rollout_order(lg, B, lmax, counts, ws)
    r_o, a_o, f_o, c_o = O.throughput_rollout(logits.numpy(), 1, 1234, 0)
    k = int(c_o[0])
    assert int(counts[0]) == k and int(t_dev) == int(counts.max()) + 1
    bits = removed[0].cpu().numpy().view(np.uint32)
    got = ((bits[:, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(-1)[:E].astype(bool)
    assert np.array_equal(got, r_o[0])
    assert np.array_equal(actions[0, :k + 1].cpu().numpy(), a_o[:k + 1, 0])
    np.testing.assert_allclose(fwd[0, :k + 1].cpu().numpy(), f_o[0, :k + 1], rtol=1e-6)


def test_throughput_sample_states_end_to_end():
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, poisson_2d
    A = poisson_2d(32)
    n = 32 * 32
    env = PreconditionerEnv(n, A, A, side="AM", fill="lsq", keep_m=True)
    E = env.num_actions - 1
    logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
    logits[E] = 6.0
    g = GFlowNet(FixedLogits(logits), None, env, mode="throughput", seed=42)
    log = g.sample_states([A] * 4, return_log=True)
    r_o, a_o, f_o, c_o = O.throughput_rollout(logits.numpy(), 4, 42, 0)
    assert np.array_equal(log.actions.cpu().numpy(), a_o)
    # LSQ fill vs the oracle (stacked QR, fp64) and ||AM-I|| from the stored fp32 M
    r, c, v, _ = O.poisson2d(32)
    idx, act, _ = O.lines_from_coo(r, c, v, n, "col")
    a_idx, _, a_val = O.lines_from_coo(r, c, v.astype(np.float64), n, "col")
    Acsc = sp.csc_matrix((v.astype(np.float64), (r, c)), shape=(n, n))
    for b in range(4):
        keep = (idx >= 0) & ~r_o[b][np.clip(act, 0, None)]
        m_ref = O.lsq_fill(idx, keep, a_idx, a_val)
        m_gpu = env.last_m[b].cpu().numpy().astype(np.float64)
        assert np.linalg.norm(m_gpu - m_ref) / np.linalg.norm(m_ref) < 1e-6
        res = O.residual_fro_fp64(Acsc, O.m_to_csc(idx, env.last_m[b].cpu().numpy(), n))
        assert float(env.last_residual[b]) == pytest.approx(res, rel=1e-10)


def test_lsq_fp64_3d_vs_oracle():
    """64^3 is the C3 config; a 12^3 7-pt fp64 lattice checks the fp64 LSQ kernel exactly."""
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, poisson_3d
    g3 = 12
    A = poisson_3d(g3)
    n = g3 ** 3
    env = PreconditionerEnv(n, A, A, side="AM", fill="lsq", keep_m=True)
    E = env.num_actions - 1
    logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(7))
    logits[E] = 7.0
    g = GFlowNet(FixedLogits(logits), None, env, mode="throughput", seed=3)
    g.sample_states([A] * 2, return_log=True)
    r_o, *_ = O.throughput_rollout(logits.numpy(), 2, 3, 0)
    r, c, v, _ = O.poisson3d(g3)
    idx, act, _ = O.lines_from_coo(r, c, v, n, "col")
    a_idx, _, a_val = O.lines_from_coo(r, c, v, n, "col")
    Acsc = sp.csc_matrix((v, (r, c)), shape=(n, n))
    for b in range(2):
        keep = (idx >= 0) & ~r_o[b][np.clip(act, 0, None)]
        m_ref = O.lsq_fill(idx, keep, a_idx, a_val)
        m_gpu = env.last_m[b].cpu().numpy()
        assert env.last_m.dtype == torch.float64
        assert np.linalg.norm(m_gpu - m_ref) / np.linalg.norm(m_ref) < 1e-12
        res = O.residual_fro_fp64(Acsc, O.m_to_csc(idx, m_gpu, n, np.float64))
        assert float(env.last_residual[b]) == pytest.approx(res, rel=1e-10)


def test_full_size_c4_residuals_vs_reference():
    """1024^2 (C4): r0 and one 20%-removed candidate against the reference's own numbers."""
    from gflownet_spai_amd import PreconditionerEnv, kernels, poisson_2d
    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))["cases"]["c4_residual"]
    A = poisson_2d(1024)
    n = 1024 * 1024
    for side, key in (("MA", "r_ma"), ("AM", "r_mta")):
        env = PreconditionerEnv(n, A, A, side=side)
        assert float(env.orig_residual) == pytest.approx(meta["r0"], rel=1e-15)
        st = meta["sets"][0]
        removed = np.random.default_rng(1000).random(env.init_nnz) < 0.2
        words = (env.init_nnz + 31) // 32
        bits = np.zeros(words, np.uint32)
        ids = np.flatnonzero(removed)
        np.bitwise_or.at(bits, ids >> 5, (np.uint32(1) << (ids & 31).astype(np.uint32)))
        rb = torch.from_numpy(bits.view(np.int32).reshape(1, words)).to(DEV)
        counts = torch.tensor([int(removed.sum())], dtype=torch.int32, device=DEV)
        rw = env.rewards_from_removed(rb, counts, torch.tensor(0.5))
        assert float(env.last_residual[0]) == pytest.approx(st[key], rel=1e-15)
        if side == "MA":
            assert float(rw[0]) == pytest.approx(st["reward"][0], rel=1e-12)


def test_edge_cases():
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, kernels
    d = load("c1_removal.npz")
    n = int(d["n"])
    A = coo(d["rows"], d["cols"], d["vals"], n)
    env = PreconditionerEnv(n, A, A)
    E = env.num_actions - 1
    # immediate terminal (nothing removed) and every edge removed
    env.update(None, torch.tensor([[E, -1], [E, -1]]), torch.tensor(0.5))
    assert float(env.last_residual[0]) == d["r_ma"][0]
    env.update(None, torch.arange(E + 1).view(1, -1), torch.tensor(0.5))
    assert float(env.last_residual[0]) == d["r_ma"][1] == pytest.approx(16.0)  # ||-I||_F = sqrt(256)
    # B = 1 (the reference crashes there, gflownet.py:121)
    logits = torch.full((E + 1,), -5.0)
    logits[E] = 20.0
    g = GFlowNet(FixedLogits(logits), None, env, mode="throughput", seed=1)
    log = g.sample_states([A], return_log=True)
    assert tuple(log.actions.shape) == (1, 1) and int(log.actions[0, 0]) == E
    # parity mode with B = 1 too
    g2 = GFlowNet(FixedLogits(logits), None, env, mode="parity")
    log2 = g2.sample_states([A], return_log=True)
    assert int(log2.actions[-1, 0]) == E
    # malformed input -> ValueError, widths beyond the compiled kernels -> NotImplementedError
    lg, lmax, z = kernels.logits_stats(logits.to(DEV), 1)
    with pytest.raises(ValueError):
        kernels.parity_step(lg, 1, torch.ones(1, 3), lmax, torch.zeros(1, (E + 32) // 32, dtype=torch.int32,
                                                                        device=DEV),
                            torch.ones(1, dtype=torch.uint8, device=DEV), z.clone())
    D = torch.ones(10, 10).to_sparse()
    dense_env = PreconditionerEnv(10, D, D)  # wide lines -> LDS hash kernel (copy fill)
    assert float(dense_env.orig_residual) == pytest.approx(np.sqrt(90 * 100 + 10 * 81), rel=1e-15)
    with pytest.raises(NotImplementedError):  # no LSQ kernel for 10-wide lines
        PreconditionerEnv(10, D, D, side="AM", fill="lsq").update(None, torch.tensor([[0, 100]]), 0.5)


def test_line_shards_sum_to_full_residual():
    """Column-sharded evaluation (the multi-GPU strong-scaling layout): the per-shard
    partials of ||AM - I||_F^2 sum to the unsharded value and the M blocks concatenate."""
    from gflownet_spai_amd import PreconditionerEnv, kernels, poisson_2d
    from gflownet_spai_amd.distributed import shard_lines
    A = poisson_2d(64)
    n = 64 * 64
    env = PreconditionerEnv(n, A, A, side="AM", fill="lsq")
    E = env.init_nnz
    rng = np.random.default_rng(3)
    acts = torch.from_numpy(np.where(rng.random((4, E)) < 0.25, np.arange(E), -1))
    removed, counts = kernels.actions_to_removed(acts.to(DEV), E)
    full, m_full = kernels.fill_residual(env.pattern, env.a_lines, removed, True, store_m=True)
    parts, blocks = [], []
    for r in range(3):
        b, e = shard_lines(n, r, 3)
        res2, m = kernels.fill_residual(env.pattern, env.a_lines, removed, True, b, e, store_m=True)
        parts.append(res2)
        blocks.append(m)
    np.testing.assert_allclose(sum(parts).cpu().numpy(), full.cpu().numpy(), rtol=1e-12)
    assert torch.equal(torch.cat(blocks, 1), m_full)


@pytest.mark.parametrize("side,fill,dims", [("AM", "lsq", 2), ("MA", "copy", 2), ("AM", "lsq", 3), ("AM", "copy", 3)])
def test_gram_cached_fill_matches_direct_kernel(side, fill, dims):
    """The env's Gram-cached fill (spai_gram_build + spai_fill_residual_gram, the bench path)
    gives the per-call kernel's (spai_fill_residual) residuals and M values, also per shard."""
    from gflownet_spai_amd import PreconditionerEnv, kernels, poisson_2d, poisson_3d
    from gflownet_spai_amd.distributed import shard_lines
    A = poisson_2d(48) if dims == 2 else poisson_3d(10)
    n = A.shape[0]
    env = PreconditionerEnv(n, A, A, side=side, fill=fill)
    assert env.gram is not None
    E = env.init_nnz
    rng = np.random.default_rng(11)
    acts = torch.from_numpy(np.where(rng.random((5, E)) < 0.3, np.arange(E), -1))
    removed, counts = kernels.actions_to_removed(acts.to(DEV), E)
    mdt = env.a_lines.val.dtype
    ref, m_ref = kernels.fill_residual(env.pattern, env.a_lines, removed, fill == "lsq", store_m=True, m_dtype=mdt)
    got, m_got = kernels.fill_residual_gram(env.pattern, env.gram, removed, fill == "lsq", store_m=True, m_dtype=mdt)
    np.testing.assert_allclose(got.cpu().numpy(), ref.cpu().numpy(), rtol=1e-12)
    tol = 1e-6 if m_got.dtype == torch.float32 else 1e-12
    np.testing.assert_allclose(m_got.cpu().numpy(), m_ref.cpu().numpy(), rtol=tol, atol=tol)
    parts = []
    for r in range(4):
        b, e = shard_lines(n, r, 4)
        res2, _ = kernels.fill_residual_gram(env.pattern, env.gram, removed, fill == "lsq", b, e)
        parts.append(res2)
    np.testing.assert_allclose(sum(parts).cpu().numpy(), got.cpu().numpy(), rtol=1e-12)


@pytest.mark.parametrize("side,fill,dims", [("AM", "lsq", 2), ("MA", "copy", 2), ("AM", "lsq", 3)])
def test_fp32_gram_cache_is_bit_identical(side, fill, dims):
    """The fp32 Gram cache (spai_gram_compact: integer stencils round-trip exactly) gives the
    fp64 cache's residuals and M values bit for bit; a matrix with non-fp32-exact products
    keeps the fp64 cache."""
    from gflownet_spai_amd import PreconditionerEnv, kernels, poisson_2d, poisson_3d
    A = poisson_2d(40) if dims == 2 else poisson_3d(9)
    n = A.shape[0]
    env32 = PreconditionerEnv(n, A, A, side=side, fill=fill, cache_dict=False)
    env64 = PreconditionerEnv(n, A, A, side=side, fill=fill, compact_gram=False, cache_dict=False)
    assert env32.gram.dtype == torch.float32 and env64.gram.dtype == torch.float64
    assert torch.equal(env32.gram.double(), env64.gram)
    E = env32.init_nnz
    rng = np.random.default_rng(5)
    acts = torch.from_numpy(np.where(rng.random((6, E)) < 0.3, np.arange(E), -1))
    removed, _ = kernels.actions_to_removed(acts.to(DEV), E)
    mdt = env64.a_lines.val.dtype
    r32, m32 = kernels.fill_residual_gram(env32.pattern, env32.gram, removed, fill == "lsq", store_m=True, m_dtype=mdt)
    r64, m64 = kernels.fill_residual_gram(env64.pattern, env64.gram, removed, fill == "lsq", store_m=True, m_dtype=mdt)
    assert torch.equal(r32, r64) and torch.equal(m32, m64)
    # a random-valued A: products are not fp32-exact, the env keeps fp64
    c = A.coalesce()
    vals = torch.from_numpy(np.random.default_rng(1).standard_normal(c._nnz()).astype(np.float32))
    R = torch.sparse_coo_tensor(c.indices(), vals.to(c.dtype), c.shape)
    assert PreconditionerEnv(n, R, R, side=side, fill=fill).gram.dtype == torch.float64


def _wide_pattern(dims, g):
    """13-wide candidate patterns (the nnz/col <= 13 rows of SURVEY §8a11): the 2-D A^2
    13-point pattern, and in 3-D the 7-point star plus the +-2 axial neighbours."""
    if dims == 2:
        r, c, v, n = O.poisson2d(g)
        A = sp.csr_matrix((v.astype(np.float64), (r, c)), shape=(n, n))
        P = (A @ A).tocoo()
        return A, P
    r, c, v, n = O.poisson3d(g)
    A = sp.csr_matrix((v, (r, c)), shape=(n, n))
    one = sp.diags([1.0, 1.0], [-2, 2], shape=(g, g))
    eye = sp.identity(g)
    far = sp.kron(sp.kron(one, eye), eye) + sp.kron(sp.kron(eye, one), eye) + sp.kron(sp.kron(eye, eye), one)
    P = (abs(A) + 0.5 * far).tocoo()
    return A, P


@pytest.mark.parametrize("dims,side,fill", [(2, "AM", "lsq"), (3, "AM", "lsq"), (2, "MA", "copy"), (3, "AM", "copy")])
def test_wide_pattern_gram_fill_vs_oracle(dims, side, fill):
    """Pattern width 13 (k_gram_fill_wide): LSQ values vs the oracle's Householder QR and the
    residual vs the oracle's fp64 ||AM - I||; COPY residual vs the uncached LDS-hash kernel."""
    from gflownet_spai_amd import PreconditionerEnv, kernels
    g = 24 if dims == 2 else 9
    A, P = _wide_pattern(dims, g)
    n = A.shape[0]
    dt = np.float32 if dims == 2 else np.float64
    Ac = A.tocoo()
    At = coo(Ac.row, Ac.col, Ac.data.astype(dt), n)
    Pt = coo(P.row, P.col, P.data.astype(dt), n)
    env = PreconditionerEnv(n, Pt, At, side=side, fill=fill, keep_m=True)
    assert env.pattern.width == 13 and env.gram is not None
    E = env.init_nnz
    rng = np.random.default_rng(21)
    rem = rng.random((3, E)) < np.array([[0.0], [0.3], [0.8]])
    acts = torch.from_numpy(np.where(rem, np.arange(E), -1))
    removed, counts = kernels.actions_to_removed(acts.to(DEV), E)
    rw = env.rewards_from_removed(removed, counts, 0.5)
    assert torch.isfinite(rw).all()
    if fill == "lsq":
        idx, act, _ = O.lines_from_coo(P.row, P.col, P.data, n, "col")
        a_idx, _, a_val = O.lines_from_coo(Ac.row, Ac.col, Ac.data, n, "col")
        Acsc = A.tocsc()
        tol = 1e-6 if dt == np.float32 else 1e-11
        for b in range(3):
            keep = (idx >= 0) & ~rem[b][np.clip(act, 0, None)]
            m_ref = O.lsq_fill(idx, keep, a_idx, a_val)
            m_gpu = env.last_m[b].cpu().numpy().astype(np.float64)
            assert np.linalg.norm(m_gpu - m_ref) / np.linalg.norm(m_ref) < tol
            res = O.residual_fro_fp64(Acsc, O.m_to_csc(idx, env.last_m[b].cpu().numpy(), n, dt))
            assert float(env.last_residual[b]) == pytest.approx(res, rel=1e-8)
        j = n // 2 + 3  # one interior column against numpy lstsq as well
        keep = (idx >= 0) & ~rem[1][np.clip(act, 0, None)]
        m_ls, J = O.lsq_fill_lstsq(idx, keep, Acsc, j)
        got = env.last_m[1][j].cpu().numpy().astype(np.float64)[keep[j] & (idx[j] >= 0)]
        np.testing.assert_allclose(got, m_ls, rtol=tol * 10, atol=tol)
    else:
        ref, _ = kernels.fill_residual(env.pattern, env.a_lines, removed, False, store_m=False,
                                       m_dtype=env.a_lines.val.dtype)
        got, _ = kernels.fill_residual_gram(env.pattern, env.gram, removed, False)
        np.testing.assert_allclose(got.cpu().numpy(), ref.cpu().numpy(), rtol=1e-12)


def test_sample_states_distinct_initial_states():
    """Different initial states per sample get their own policy call and logit row (the
    reference runs the policy on each s0[b], gflownet.py:70-74); identical states share one."""
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, poisson_2d

    class EdgeLogits(torch.nn.Module):
        calls = 0

        def logits(self, data):
            EdgeLogits.calls += 1
            l = torch.cat([data.edge_attr.float().reshape(-1) * 0.7, torch.tensor([3.0], device=DEV)])
            return l, torch.tensor(0.5, device=DEV)

    A = poisson_2d(12)
    n = 144
    A2 = torch.sparse_coo_tensor(A._indices(), A._values() * 1.5, A.shape)
    env = PreconditionerEnv(n, A, A, side="AM", fill="lsq")
    g = GFlowNet(EdgeLogits(), None, env, mode="throughput", seed=3)
    log = g.sample_states([A, A2, A], return_log=True)
    assert EdgeLogits.calls == 3
    acts = log.actions.cpu().numpy()
    for b, M in enumerate([A, A2, A]):
        lb = np.concatenate([M._values().numpy().astype(np.float32) * np.float32(0.7), [3.0]]).astype(np.float32)
        _, a_o, f_o, c_o = O.throughput_rollout(lb, 1, 3, 0, sample_base=b)
        k = int(c_o[0])
        assert np.array_equal(acts[:k + 1, b], a_o[:, 0])
        np.testing.assert_allclose(log.fwd_probs[b, :k + 1].detach().cpu().numpy(), f_o[0], rtol=1e-6)
    EdgeLogits.calls = 0
    A3 = torch.sparse_coo_tensor(A._indices().clone(), A._values().clone(), A.shape)
    g.sample_states([A, A3, A], return_log=True)  # equal content, other storage: one call
    assert EdgeLogits.calls == 1


@pytest.mark.parametrize("P", [2, 3, 5])
def test_split_rollout_parts_reassemble_bit_exact(P):
    """The multi-GPU split played by P parts in one process: every part's select
    gives the complete removed sets and fills the exchange array for its own buckets only; the
    parts' arrays are summed (what the all_reduce does); each part's merge then reproduces the
    one-part counts, and its sort + finish write its trajectory slice.  The slices tile [0, T)
    and reassemble the one-part rollout bit for bit (actions and fwd_probs)."""
    from gflownet_spai_amd import kernels
    E, B = 300000, 3
    rng = np.random.default_rng(P)
    logits = rng.standard_normal(E + 1).astype(np.float32)
    logits[E] = 1.2
    lg, lmax, _ = kernels.logits_stats(torch.from_numpy(logits).to(DEV), B)
    removed1, counts1, ws1 = kernels.rollout_select(lg, B, lmax, 17, 4)
    a1, f1, t1 = kernels.rollout_order(lg, B, lmax, counts1, ws1)
    T = int(t1)
    parts = []
    for q in range(P):
        rq, _, wq = kernels.rollout_select(lg, B, lmax, 17, 4, 0, None, q, P, ws_tag=f"part{q}")
        assert torch.equal(rq, removed1)
        parts.append(wq)
    from gflownet_spai_amd import _lib
    nbk = B * 2 * _lib.load().spai_rollout_ws_offset(E, B, 3)  # the bucket part (then B caller slots)
    xs = [kernels.exchange_array(wq, E, B)[:nbk] for wq in parts]
    # disjoint supports: each bucket's entries come from exactly one part
    nz = sum((x != 0).int() for x in xs)
    assert int(nz.max()) <= 1
    total = sum(x.clone() for x in xs)
    one = kernels.exchange_array(ws1, E, B)[:nbk]
    assert torch.equal(total, one)
    acts = torch.full((B, T), -7, dtype=torch.int64, device=DEV)
    fwds = torch.full((B, T), -7.0, device=DEV)
    covered = torch.zeros((B, T), dtype=torch.int32, device=DEV)
    for q, wq in enumerate(parts):
        kernels.exchange_array(wq, E, B)[:nbk].copy_(total)
        cq = kernels.rollout_merge(lg, B, lmax, wq, q, P)
        assert torch.equal(cq, counts1)
        aq, fq = kernels.rollout_sort(lg, B, lmax, wq, q, P)
        tq = kernels.rollout_finish(lg, B, lmax, cq, wq, aq, fq, q, P)
        assert int(tq) == T
        bd = kernels.part_bounds(wq, E, B, q, P).cpu()
        for b in range(B):
            s0, e0 = int(bd[b, 0]), min(int(bd[b, 1]), T)
            acts[b, s0:e0] = aq[b, s0:e0]
            fwds[b, s0:e0] = fq[b, s0:e0]
            covered[b, s0:e0] += 1
    assert bool((covered == 1).all())
    assert torch.equal(acts, a1[:, :T])
    assert torch.equal(fwds, f1[:, :T])
    r_o, a_o, f_o, c_o = O.throughput_rollout(logits, B, 17, 4)
    assert np.array_equal(acts.cpu().numpy(), a_o.T)


def test_stream_counter_and_graph_replay():
    """The Philox stream id read from the device counter equals the host argument and advances
    by one per select; a HIP graph of GFlowNet.sample_states replays fresh rollouts (streams
    1, 2, ...) identical to the oracle's, with M and rewards recomputed each replay."""
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, kernels, poisson_2d
    E, B = 5000, 2
    logits = np.random.default_rng(3).standard_normal(E + 1).astype(np.float32)
    logits[E] = 2.0
    lg, lmax, _ = kernels.logits_stats(torch.from_numpy(logits).to(DEV), B)
    ctr = torch.tensor([41], dtype=torch.int64, device=DEV)
    r_a, c_a, _ = kernels.rollout_select(lg, B, lmax, 9, 0, 0, ctr)
    assert int(ctr) == 42
    r_b, c_b, _ = kernels.rollout_select(lg, B, lmax, 9, 41)
    assert torch.equal(r_a, r_b) and torch.equal(c_a, c_b)

    A = poisson_2d(24)
    n = 24 * 24
    env = PreconditionerEnv(n, A, A, side="AM", fill="lsq", keep_m=True)
    El = env.num_actions - 1
    lgt = torch.randn(El + 1, generator=torch.Generator().manual_seed(5))
    lgt[El] = 4.0
    g = GFlowNet(FixedLogits(lgt).to(DEV), None, env, mode="throughput", seed=11)  # no H2D copy in capture
    s0 = [A] * 3
    with torch.no_grad():
        log0 = g.sample_states(s0, return_log=True)  # stream 0, eager (also warms every cache)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            g.sample_states(s0, return_log=True)  # stream 1 (warm-up on the capture stream)
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(graph):
            logc = g.sample_states(s0, return_log=True)  # captured: not executed
        outs = []
        for _ in range(2):
            graph.replay()
            torch.cuda.synchronize()
            outs.append((logc._full[0].clone(), logc._full[2].clone(), env.last_m.clone(), logc.rewards.clone()))
    _, a_0, _, _ = O.throughput_rollout(lgt.numpy(), 3, 11, 0)
    assert np.array_equal(log0.actions.cpu().numpy(), a_0)
    for k, (acts, t, m, rw) in enumerate(outs):
        _, a_o, _, c_o = O.throughput_rollout(lgt.numpy(), 3, 11, 2 + k)
        T = int(t)
        assert T == a_o.shape[0]
        assert np.array_equal(acts[:, :T].cpu().numpy(), a_o.T)
    assert not torch.equal(outs[0][2], outs[1][2])  # the fill ran again on the new removal sets


def _inexact(v, rng):
    """fp64 values that are NOT exact in fp32 (so the kernels read them as fp64, not narrowed)."""
    return v * (1.0 + 2.0 ** -40 * rng.integers(1, 1000, v.shape))


@pytest.mark.parametrize("dims,W,adt,mdt,side,exact", [(2, 5, np.float32, np.float32, "col", True),
                                                        (2, 7, np.float32, np.float64, "row", True),
                                                        (3, 7, np.float64, np.float64, "col", True),
                                                        (3, 7, np.float64, np.float64, "col", False),
                                                        (3, 13, np.float64, np.float32, "row", True),
                                                        (3, 13, np.float64, np.float64, "col", True),
                                                        (3, 13, np.float64, np.float64, "row", False)])
def test_residual_lines_arbitrary_m_vs_scipy(dims, W, adt, mdt, side, exact):
    """The generic batched SpMM residual (spai_residual_lines) of B DISTINCT random sparse M
    (random indices anywhere in [0, n), random values, empty slots) against scipy's exact fp64
    ||M A - I||_F^2 (row lines) / ||A M - I||_F^2 (column lines), per sample; one shared index
    set too (idx stride 0); line ranges sum to the whole.  fp64 A with fp32-exact values runs
    narrowed (kernels.narrow_values); `exact=False` keeps the fp64-A kernels covered."""
    from gflownet_spai_amd import kernels
    from gflownet_spai_amd.layout import build_lines
    r, c, v, n = (O.poisson2d(12, adt) if dims == 2 else O.poisson3d(6, adt))
    if not exact:
        v = _inexact(v, np.random.default_rng(1))
    A = sp.csr_matrix((v.astype(np.float64), (r, c)), shape=(n, n))
    a_lines = build_lines(torch.from_numpy(r), torch.from_numpy(c), torch.from_numpy(v), n, side, DEV)
    assert (kernels.narrow_values(a_lines).dtype == torch.float32) == (exact or adt == np.float32)
    rng = np.random.default_rng(W)
    B = 3 if W < 13 else 11  # 13-wide: chunks of 8 (fp32-exact A) or 4 samples, and a partial chunk
    idx = rng.integers(0, n, (B, n, W)).astype(np.int32)
    idx[rng.random((B, n, W)) < 0.3] = -1
    for b in range(B):  # distinct indices inside a line (the ELL lines of a sparse matrix)
        for l in range(n):
            row = idx[b, l]
            seen = set()
            for p in range(W):
                if row[p] in seen:
                    row[p] = -1
                elif row[p] >= 0:
                    seen.add(int(row[p]))
    val = rng.standard_normal((B, n, W)).astype(mdt)
    got = kernels.residual_lines(torch.from_numpy(idx).to(DEV), torch.from_numpy(val).to(DEV), a_lines).cpu().numpy()
    I = sp.identity(n, format="csr")
    for b in range(B):
        ok = idx[b] >= 0
        lines, slots = np.nonzero(ok)
        other = idx[b][ok]
        vals = val[b][ok].astype(np.float64)
        M = sp.csr_matrix((vals, (lines, other) if side == "row" else (other, lines)), shape=(n, n))
        P = (M @ A) if side == "row" else (A @ M)
        ref = sp.linalg.norm(P - I) ** 2
        assert got[b] == pytest.approx(ref, rel=1e-12)
    # one index set for every sample (stride 0) and a split into line ranges
    shared = kernels.residual_lines(torch.from_numpy(idx[0]).to(DEV), torch.from_numpy(val[:1]).to(DEV), a_lines)
    assert float(shared[0]) == pytest.approx(float(got[0]), rel=1e-14)
    h = n // 2
    parts = (kernels.residual_lines(torch.from_numpy(idx).to(DEV), torch.from_numpy(val).to(DEV), a_lines, 0, h) +
             kernels.residual_lines(torch.from_numpy(idx).to(DEV), torch.from_numpy(val).to(DEV), a_lines, h, n))
    np.testing.assert_allclose(parts.cpu().numpy(), got, rtol=1e-13)


@pytest.mark.parametrize("W,mdt", [(7, np.float64), (7, np.float32), (13, np.float64)])
def test_residual_lines_multiblock_batch8(W, mdt):
    """Many blocks and a full chunk: B = 8 samples of an fp64 3-D Laplacian's pattern (W = 7) or
    the 13-wide axial pattern, 25 % of the slots removed per sample, random values, at
    n = 16^3 (16 blocks of 256 lines) vs scipy's fp64 ||A M_b - I||_F^2."""
    from gflownet_spai_amd import axial_pattern_3d, kernels
    from gflownet_spai_amd.layout import build_lines
    r, c, v, n = O.poisson3d(16, np.float64)
    A = sp.csr_matrix((v, (r, c)), shape=(n, n))
    a_lines = build_lines(torch.from_numpy(r), torch.from_numpy(c), torch.from_numpy(v), n, "col", DEV)
    if W == 7:
        pat = a_lines.idx.cpu().numpy()
    else:
        P = axial_pattern_3d(16, 2).coalesce()
        pr, pc = P.indices()
        pat = build_lines(pr, pc, P.values(), n, "col", DEV).idx.cpu().numpy()
    rng = np.random.default_rng(11)
    B = 8
    idx = np.repeat(pat[None], B, 0).copy()
    idx[rng.random(idx.shape) < 0.25] = -1
    val = rng.standard_normal(idx.shape).astype(mdt)
    got = kernels.residual_lines(torch.from_numpy(idx).to(DEV), torch.from_numpy(val).to(DEV), a_lines).cpu().numpy()
    I = sp.identity(n, format="csr")
    for b in range(B):
        ok = idx[b] >= 0
        lines, _ = np.nonzero(ok)
        M = sp.csr_matrix((val[b][ok].astype(np.float64), (idx[b][ok], lines)), shape=(n, n))
        assert got[b] == pytest.approx(sp.linalg.norm(A @ M - I) ** 2, rel=1e-12)


def test_residual_lines_matches_fused_lsq_fill_residual():
    """||A M - I||_F^2 of the candidates' stored LSQ fills M (distinct kept index sets per
    sample) through the generic kernel equals the fused fill kernel's residual (which takes it
    from the factorisation; they differ by d^T G d, d = fp32 rounding of M)."""
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, kernels, poisson_2d
    A = poisson_2d(32)
    env = PreconditionerEnv(1024, A, A, side="AM", fill="lsq", keep_m=True)
    E = env.num_actions - 1
    lg = torch.randn(E + 1, generator=torch.Generator().manual_seed(2))
    lg[E] = 1.0
    log = GFlowNet(FixedLogits(lg), None, env, mode="throughput", seed=3).sample_states([A] * 4, return_log=True)
    pat = env.pattern
    bits = log.removed.view(torch.int32)
    act = pat.act.long().clamp(min=0)
    rem = ((bits[:, act >> 5] >> (act & 31)) & 1).bool()
    idx = torch.where(rem | (pat.idx < 0), torch.full_like(pat.idx, -1), pat.idx)
    got = kernels.residual_lines(idx, env.last_m, env.a_lines)
    ref = env.last_residual.double() ** 2
    np.testing.assert_allclose(got.cpu().numpy(), ref.cpu().numpy(), rtol=1e-6)


@pytest.mark.parametrize("dims,exact", [(2, True), (3, True), (3, False)])
def test_residual_lines_shared_pattern_and_conflicting_lanes(dims, exact):
    """k_resid_shared (2-D: A's own 5-wide pattern, fp32) and k_resid_wide (3-D: the 13-wide
    axial C3 pattern, fp64; fp32-exact A values: chunks of 8 samples, otherwise 4): B = 9
    samples that are sub-patterns of ONE line pattern (random removals per sample: one index
    matching per line and chunk) except sample 3, which puts a different valid index into one
    slot of ~10 % of the lines (those lanes evaluate every sample of the chunk on its own index
    set).  Each sample vs scipy's exact fp64 ||A M_b - I||_F^2, and bit for bit vs the same
    sample evaluated alone (both paths apply the same operations in the same order)."""
    from gflownet_spai_amd import axial_pattern_3d, kernels
    from gflownet_spai_amd.layout import build_lines
    dt = np.float32 if dims == 2 else np.float64
    r, c, v, n = O.poisson2d(16, dt) if dims == 2 else O.poisson3d(7, dt)
    if not exact:
        v = _inexact(v, np.random.default_rng(2))
    A = sp.csr_matrix((v.astype(np.float64), (r, c)), shape=(n, n))
    a_lines = build_lines(torch.from_numpy(r), torch.from_numpy(c), torch.from_numpy(v), n, "col", DEV)
    if dims == 2:
        pat = a_lines.idx.cpu().numpy()  # [n, 5], -1 padded
    else:
        P = axial_pattern_3d(7, 2).coalesce()
        pr, pc = P.indices()
        pat = build_lines(pr, pc, P.values(), n, "col", DEV).idx.cpu().numpy()  # [n, 13]
        assert pat.shape[1] == 13
    rng = np.random.default_rng(5)
    B, W = 9, pat.shape[1]
    idx = np.repeat(pat[None], B, 0).copy()
    idx[rng.random(idx.shape) < 0.25] = -1
    conflict = rng.random(n) < 0.1
    for l in np.nonzero(conflict)[0]:
        p = int(np.argmax(pat[l] >= 0))
        new = int(rng.integers(0, n))
        while new in set(pat[l].tolist()):
            new = int(rng.integers(0, n))
        idx[3, l, p] = new
    val = rng.standard_normal((B, n, W)).astype(dt)
    got = kernels.residual_lines(torch.from_numpy(idx).to(DEV), torch.from_numpy(val).to(DEV), a_lines).cpu().numpy()
    I = sp.identity(n, format="csr")
    for b in range(B):
        ok = idx[b] >= 0
        lines, _ = np.nonzero(ok)
        M = sp.csr_matrix((val[b][ok].astype(np.float64), (idx[b][ok], lines)), shape=(n, n))
        assert got[b] == pytest.approx(sp.linalg.norm(A @ M - I) ** 2, rel=1e-12)
        alone = kernels.residual_lines(torch.from_numpy(idx[b:b + 1]).to(DEV), torch.from_numpy(val[b:b + 1]).to(DEV),
                                       a_lines).cpu().numpy()
        assert alone[0] == got[b]


@pytest.mark.parametrize("geom,mdt", [("3d13", torch.float64), ("3d13", torch.float32), ("2d5", torch.float32),
                                      ("3d7", torch.float64)])
def test_residual_lines_gram_cache_bit_identical(geom, mdt):
    """spai_residual_lines_gram (the 13-wide C3 geometry with the env's Gram cache dictionary; the
    5-wide 2-D and 7-wide 3-D stencil patterns with a dictionary made from the env's full cache)
    against the index-matching kernel (spai_residual_lines) bit for bit, B = 9 samples: every
    sample a slot-aligned sub-pattern of the env's pattern (random removals -> -1), except sample
    3, which puts a foreign index into one slot of ~10 % of the lines (those lines are matched from
    A by the lean fallback).  Also a fully aligned batch, and both against scipy's
    ||A M_b - I||_F^2."""
    from gflownet_spai_amd import PreconditionerEnv, axial_pattern_3d, kernels, poisson_2d, poisson_3d
    if geom == "3d13":
        A, P = poisson_3d(16), axial_pattern_3d(16)
    else:
        A = P = poisson_2d(40) if geom == "2d5" else poisson_3d(12)
    n = A.shape[0]
    env = PreconditionerEnv(n, P, A, side="AM", fill="lsq")
    W = env.pattern.width
    assert W == int(geom[2:])
    gram = env.gram if W == 13 else kernels.cache_dict(env.gram, n)
    assert isinstance(gram, kernels.CacheDict)
    pat = env.pattern.idx.cpu().numpy()
    rng = np.random.default_rng(21)
    B = 9
    idx = np.repeat(pat[None], B, 0).copy()
    idx[rng.random(idx.shape) < 0.25] = -1
    aligned = idx.copy()
    for l in np.nonzero(rng.random(n) < 0.1)[0]:
        p = int(np.argmax(pat[l] >= 0))
        new = int(rng.integers(0, n))
        while new in set(pat[l].tolist()):
            new = int(rng.integers(0, n))
        idx[3, l, p] = new
    val = torch.from_numpy(rng.standard_normal((B, n, W))).to(mdt)
    c = A.coalesce()
    Asp = sp.csr_matrix((c.values().double().numpy(), (c.indices()[0].numpy(), c.indices()[1].numpy())), shape=(n, n))
    I = sp.identity(n, format="csr")
    for ix in (aligned, idx):
        ti = torch.from_numpy(ix).to(DEV)
        ref = kernels.residual_lines(ti, val.to(DEV), env.a_lines)
        got = kernels.residual_lines(ti, val.to(DEV), env.a_lines, gram=gram, pattern=env.pattern)
        assert torch.equal(got, ref)
        g = got.cpu().numpy()
        for b in (0, 3):
            ok = ix[b] >= 0
            lines, _ = np.nonzero(ok)
            M = sp.csr_matrix((val[b].double().numpy()[ok], (ix[b][ok], lines)), shape=(n, n))
            assert g[b] == pytest.approx(sp.linalg.norm(Asp @ M - I) ** 2, rel=1e-12)
    # line shards sum to the whole (256-line blocks: the same partial sums)
    ti = torch.from_numpy(idx).to(DEV)
    h = 256 * (n // 512)
    parts = (kernels.residual_lines(ti, val.to(DEV), env.a_lines, 0, h, gram=gram, pattern=env.pattern) +
             kernels.residual_lines(ti, val.to(DEV), env.a_lines, h, n, gram=gram, pattern=env.pattern))
    np.testing.assert_allclose(parts.cpu().numpy(), got.cpu().numpy(), rtol=1e-13)


def test_residual_lines_gram_noninteger_stencil_bit_identical():
    """the Gram-cached residual on a stencil with non-integer fp64 values (its Gram cache
    stays fp64, compact_gram=False, and is not fp32-exact): spai_residual_lines_gram with the cache's
    dictionary (25 distinct entries, the fp64 16-byte entry loads) against the index-matching kernel
    bit for bit — the cache's products must be summed in line_gram's order — and against scipy."""
    from gflownet_spai_amd import PreconditionerEnv, kernels, poisson_2d
    g = 40
    base = poisson_2d(g, torch.float64).coalesce()
    r, c = base.indices()
    n = g * g
    # a translation-invariant 5-point stencil with unequal, non-integer coefficients
    dr, dc = r // g - c // g, r % g - c % g
    f64 = lambda x: torch.full(r.shape, x, dtype=torch.float64)  # (fp64 values, none exact in fp32)
    v = torch.where(r == c, f64(4.37), torch.where(dr == 0, torch.where(dc > 0, f64(-1.13), f64(-0.91)),
                                                   torch.where(dr > 0, f64(-1.27), f64(-0.79))))
    assert not torch.equal(v.float().double(), v)
    A = torch.sparse_coo_tensor(base.indices(), v, (n, n))
    env = PreconditionerEnv(n, A, A, side="AM", fill="lsq", compact_gram=False)
    assert env.gram.dtype == torch.float64
    gram = kernels.cache_dict(env.gram, n)
    assert isinstance(gram, kernels.CacheDict) and gram.entries == 25
    W = env.pattern.width
    pat = env.pattern.idx.cpu().numpy()
    rng = np.random.default_rng(5)
    B = 8
    idx = np.repeat(pat[None], B, 0).copy()
    idx[rng.random(idx.shape) < 0.3] = -1
    val = torch.from_numpy(rng.standard_normal((B, n, W)))
    ti = torch.from_numpy(idx).to(DEV)
    ref = kernels.residual_lines(ti, val.to(DEV), env.a_lines)
    got = kernels.residual_lines(ti, val.to(DEV), env.a_lines, gram=gram, pattern=env.pattern)
    assert torch.equal(got, ref)
    Asp = sp.csr_matrix((v.numpy(), (r.numpy(), c.numpy())), shape=(n, n))
    I = sp.identity(n, format="csr")
    for b in (0, 5):
        ok = idx[b] >= 0
        lines, _ = np.nonzero(ok)
        M = sp.csr_matrix((val[b].numpy()[ok], (idx[b][ok], lines)), shape=(n, n))
        assert float(got[b]) == pytest.approx(sp.linalg.norm(Asp @ M - I) ** 2, rel=1e-12)


@pytest.mark.parametrize("kind", ["2d_lsq", "2d_copy", "3d_axial", "3d_axial_f64"])
def test_gram_dict_is_bit_identical(kind):
    # (the env holds 5/7-wide Gram caches in full; the dictionary is built here explicitly)
    """The Gram cache held as its dictionary (spai_line_cache_dict + spai_fill_lines_gram_dict; the
    13-wide fill re-reads its entry per sample at two waves per SIMD) against the full cache: M,
    the residual sums (one launch, 256-line-aligned shards) and the rewards bit for bit, for the
    5-wide and the 13-wide (C3 geometry) fills, fp32 and fp64 caches."""
    from gflownet_spai_amd import PreconditionerEnv, axial_pattern_3d, kernels, poisson_2d, poisson_3d
    from gflownet_spai_amd.distributed import LINE_ALIGN, shard_lines
    fill, side = ("copy", "MA") if kind == "2d_copy" else ("lsq", "AM")
    if kind.startswith("2d"):
        A = P = poisson_2d(70)
    else:
        A, P = poisson_3d(16), axial_pattern_3d(16)
        if kind.endswith("f64"):  # non-fp32-exact values: the fp64 cache
            c = A.coalesce()
            A = torch.sparse_coo_tensor(c.indices(), c.values() * (1.0 + 1e-9), c.shape).coalesce()
    n = A.shape[0]
    envd = PreconditionerEnv(n, P, A, side=side, fill=fill, keep_m=True)
    envf = PreconditionerEnv(n, P, A, side=side, fill=fill, keep_m=True, cache_dict=False)
    assert isinstance(envd.gram, kernels.CacheDict) == (envd.pattern.width > 7) and torch.is_tensor(envf.gram)
    if not isinstance(envd.gram, kernels.CacheDict):
        envd.gram = kernels.cache_dict(envd.gram, n)
    assert envd.gram.dtype == envf.gram.dtype == (torch.float64 if kind.endswith("f64") else torch.float32)
    assert kernels.cache_nbytes(envd.gram) < kernels.cache_nbytes(envf.gram) / 4
    E = envd.init_nnz
    rng = np.random.default_rng(12)
    acts = torch.from_numpy(np.where(rng.random((9, E)) < 0.25, np.arange(E), -1))
    removed, counts = kernels.actions_to_removed(acts.to(DEV), E)
    rd, rf = envd.fill_partial(removed), envf.fill_partial(removed)
    assert torch.equal(rd, rf) and torch.equal(envd.last_m, envf.last_m)
    for q in range(3):
        lb, le = shard_lines(n, q, 3, LINE_ALIGN)
        assert torch.equal(envd.fill_partial(removed, lb, le, limbs=True), envf.fill_partial(removed, lb, le, limbs=True))
    assert torch.equal(envd.fill_rewards(removed, counts, torch.tensor(0.5)),
                       envf.fill_rewards(removed, counts, torch.tensor(0.5)))


@pytest.mark.parametrize("overlap", ["sort", "fill", "select"])
def test_overlap_modes_graph_replay_bit_identical(overlap):
    """The fill + rewards on a second captured stream beside the trajectory sort (overlap="sort":
    forked after the sort's launch; "fill": after the select; "select": issued after the sort but
    depending on the select only): graph replays give the same actions, fwd_probs, M and rewards
    bit for bit as the one-stream step (overlap=False) on the same Philox streams, QR fill."""
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, poisson_2d
    A = poisson_2d(32)
    n = 32 * 32
    env = PreconditionerEnv(n, A, A, side="AM", fill="qr", keep_m=True)
    El = env.num_actions - 1
    lgt = torch.randn(El + 1, generator=torch.Generator().manual_seed(8))
    lgt[El] = 4.0
    s0 = [A] * 4
    res = {}
    for ov in (False, overlap):
        g = GFlowNet(FixedLogits(lgt).to(DEV), None, env, mode="throughput", seed=13, overlap=ov)
        with torch.no_grad():
            g.sample_states(s0, return_log=True)  # stream 0, eager (warms every cache)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                g.sample_states(s0, return_log=True)  # stream 1
            torch.cuda.current_stream().wait_stream(side)
            with torch.cuda.graph(graph):
                logc = g.sample_states(s0, return_log=True)
            outs = []
            for _ in range(2):  # streams 2, 3
                graph.replay()
                torch.cuda.synchronize()
                T = int(logc._full[2])
                outs.append((logc._full[0][:, :T].clone(), logc._full[1][:, :T].clone(), env.last_m.clone(),
                             logc.rewards.clone()))
        res[ov] = outs
    for (a0, f0, m0, r0), (a1, f1, m1, r1) in zip(res[False], res[overlap]):
        assert torch.equal(a0, a1) and torch.equal(f0, f1) and torch.equal(m0, m1) and torch.equal(r0, r1)
