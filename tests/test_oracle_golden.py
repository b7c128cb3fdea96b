"""The CPU oracle against the golden vectors captured from the reference itself
(tests/golden/make_golden.py), plus the oracle's own known-answer tests.

These pin the oracle before any HIP result is compared with it.
"""
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import spai_oracle as O

from .conftest import GOLDEN

ROLLOUTS = [f"c1_rollout_s{s}.npz" for s in range(4)]
REMOVALS = ["c1_removal.npz", "c1p_removal.npz", "rand64_removal.npz"]


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def test_philox_known_answers():
    # Random123 philox4x32_10 KAT vectors
    assert [int(x) for x in O.philox4x32_10(0, 0, 0, 0, 0, 0)] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    ff = 0xFFFFFFFF
    assert [int(x) for x in O.philox4x32_10(ff, ff, ff, ff, ff, ff)] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6,
                                                                          0x6D5451FD]
    assert [int(x) for x in O.philox4x32_10(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344, 0xA4093822,
                                             0x299F31D0)] == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_det_logf_accuracy():
    x = np.concatenate([np.logspace(-30, 30, 20001).astype(np.float32), np.float32([1.0, 0.5, 2.0, 6e-8, 16.6])])
    err = np.abs(O.det_logf(x).astype(np.float64) - np.log(x.astype(np.float64)))
    assert err.max() < 2e-5 * max(1.0, np.abs(np.log(x)).max() / 70)
    assert O.det_logf(np.float32([1.0]))[0] == 0.0


@pytest.mark.parametrize("name", ROLLOUTS)
def test_parity_rollout_matches_reference(name):
    d = load(name)
    torch.manual_seed(int(d["seed"]))
    acts, fwd = O.parity_rollout(d["logits"], int(d["B"]))
    assert np.array_equal(acts.numpy(), d["actions"])
    assert np.array_equal(fwd.numpy(), d["fwd_probs"])


def large_rollout_logits(d):
    E = int(d["grid"]) ** 2 * 5 - 4 * int(d["grid"])
    logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(int(d["logit_seed"])))
    logits[E] = float(d["terminal_logit"])
    return logits


@pytest.mark.parametrize("name", ["c2_rollout.npz", "c4_rollout.npz", "longer_rollout.npz"])
def test_parity_rollout_matches_reference_large(name):
    """C2 / C4 reference rollouts (G6) and the 25,633-step 72^2 rollout (G9, every action removed
    before the terminal): the oracle's sequential sampler with the reference's normalisation
    chain reproduces actions and fwd_probs bit for bit from the seeds."""
    d = load(name)
    torch.manual_seed(int(d["seed"]))
    k = 2000 if name == "longer_rollout.npz" else None  # G9: its first 2,000 steps here (the GPU test runs all)
    acts, fwd = O.parity_rollout(large_rollout_logits(d), int(d["B"]), max_steps=k)
    assert np.array_equal(acts.numpy(), d["actions"][:k])
    assert np.array_equal(fwd.numpy(), d["fwd_probs"][:, :k])


@pytest.mark.parametrize("name", REMOVALS)
def test_copy_fill_residual_reward_match_reference(name):
    d = load(name)
    n = int(d["n"])
    for k in range(d["removed"].shape[0]):
        mr, mc, mv = O.copy_fill_coo(d["rows"], d["cols"], d["vals"], d["removed"][k], n)
        assert len(mr) == d["nnz_m"][k]
        r = O.residual_ma_torch(mr, mc, mv, d["rows"], d["cols"], d["vals"], n)
        assert r == d["r_ma"][k]
        for ia, al in enumerate(d["alphas"]):
            rw = O.reward(r, len(mr), torch.tensor(al, dtype=torch.float32), d["r0"], int(d["f0"]), n)
            assert rw == d["reward"][k, ia]


@pytest.mark.parametrize("name", REMOVALS)
def test_fp64_residual_both_sides_vs_reference(name):
    """The fp64 scipy residual used for the north-star side agrees with the reference:
    ||M A - I|| (r_ma) and ||A M - I|| == ||M^T A - I|| (reference calculate_residual(M^T, A))."""
    d = load(name)
    n = int(d["n"])
    A = sp.csr_matrix((d["vals"].astype(np.float64), (d["rows"], d["cols"])), shape=(n, n))
    for k in range(d["removed"].shape[0]):
        mr, mc, mv = O.copy_fill_coo(d["rows"], d["cols"], d["vals"], d["removed"][k], n)
        M = sp.csr_matrix((mv.astype(np.float64), (mr, mc)), shape=(n, n))
        rel = 1e-12 if name != "rand64_removal.npz" else 1e-6  # reference SpGEMM runs in fp32
        assert O.residual_fro_fp64(M, A) == pytest.approx(d["r_ma"][k], rel=rel)
        if np.allclose(A.toarray(), A.toarray().T):
            assert O.residual_fro_fp64(A, M) == pytest.approx(d["r_mta"][k], rel=rel)


def test_full_size_golden_residuals():
    """C2 and C4 (256^2, 1024^2) residuals of the reference, recomputed by the fp64 oracle."""
    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))
    for tag, grid in (("c2_residual", 256), ("c4_residual", 1024)):
        case = meta["cases"][tag]
        r, c, v, n = O.poisson2d(grid)
        A = sp.csr_matrix((v.astype(np.float64), (r, c)), shape=(n, n))
        assert O.residual_fro_fp64(A, A) == pytest.approx(case["r0"], rel=1e-13)
        for k, st in enumerate(case["sets"]):
            frac = float(st["recipe"].split("<")[1])
            removed = np.random.default_rng(1000 + k).random(len(r)) < frac
            assert removed.sum() == st["n_removed"]
            keep = ~removed
            M = sp.csr_matrix((v[keep].astype(np.float64), (r[keep], c[keep])), shape=(n, n))
            assert O.residual_fro_fp64(M, A) == pytest.approx(st["r_ma"], rel=1e-13)
            assert O.residual_fro_fp64(A, M) == pytest.approx(st["r_mta"], rel=1e-13)
            rw = O.reward(st["r_ma"], int(keep.sum()), torch.tensor(0.5), case["r0"], case["f0"], n)
            assert rw == pytest.approx(st["reward"][0], rel=1e-12)


def test_throughput_rollout_structure():
    """Gumbel-top-k oracle: trajectories are the removed sets in key order, then E."""
    rng = np.random.default_rng(0)
    logits = rng.standard_normal(301).astype(np.float32)
    logits[-1] = 3.0
    removed, actions, fwd, counts = O.throughput_rollout(logits, 5, seed=7, stream=3)
    E = 300
    for b in range(5):
        k = counts[b]
        assert set(actions[:k, b].tolist()) == set(np.flatnonzero(removed[b]).tolist())
        assert actions[k, b] == E and np.all(actions[k + 1:, b] == -1)
        t = O.arrival_times(logits, b, 7, 3)
        assert np.all(np.diff(t[actions[:k, b]]) >= 0) and np.all(t[actions[:k, b]] < t[E])
        assert np.all(fwd[b, k + 1:] == 1.0) and np.all(fwd[b, :k + 1] > 0)


def test_det_expf_accuracy_and_range():
    """det_expf: within 2 ulp of the correctly rounded e^x over its range, exact at 0, the
    overflow/underflow clamps, and r_E = 1 exactly (the terminal's inverse rate)."""
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-87.3, 88.7, 200000), rng.uniform(-3, 3, 100000)]).astype(np.float32)
    got = O.det_expf(x).astype(np.float64)
    ref = np.exp(x.astype(np.float64))
    ulp = np.spacing(ref.astype(np.float32)).astype(np.float64)
    assert np.max(np.abs(got - ref) / ulp) < 2.0
    assert O.det_expf(np.float32([0.0]))[0] == 1.0
    assert O.det_expf(np.float32([89.0]))[0] == np.inf and O.det_expf(np.float32([-88.0]))[0] == 0.0
    lg = rng.standard_normal(50).astype(np.float32)
    assert O.inverse_rates(lg)[-1] == 1.0


def test_arrival_race_matches_gumbel_keys():
    """t_a < t_E decides the same removed set as the Gumbel keys l_a - ln q_a > l_E - ln q_E
    (equal up to fp32 rounding at exact near-ties), and ascending t is descending key order."""
    rng = np.random.default_rng(6)
    logits = rng.standard_normal(20001).astype(np.float32)
    logits[-1] = 1.2
    for b in range(3):
        t = O.arrival_times(logits, b, 5, 9).astype(np.float64)
        q = -O.det_logf(O.philox_u(logits.size, b, 5, 9)).astype(np.float64)
        key = logits.astype(np.float64) - np.log(q)
        agree = (t[:-1] < t[-1]) == (key[:-1] > key[-1])
        assert agree.mean() > 0.9995
        win = np.flatnonzero(t[:-1] < t[-1])
        o = win[np.argsort(t[win], kind="stable")]
        assert np.mean(np.diff(key[o]) <= 1e-5) > 0.999


def test_gumbel_topk_matches_sequential_distribution():
    """Distributional parity with the reference sampler (gflownet.py:148 loop): the
    marginal removal probability of every action under Gumbel-top-k equals the one of
    sequential sampling without replacement until the terminal id (Monte Carlo)."""
    rng = np.random.default_rng(1)
    E = 12
    logits = (rng.standard_normal(E + 1) * 0.7).astype(np.float32)
    logits[E] = 1.0
    R = 6000
    seq = np.zeros(E)
    w = np.exp(logits.astype(np.float64))
    for _ in range(R):
        avail = np.ones(E + 1, bool)
        while True:
            p = np.where(avail, w, 0)
            a = rng.choice(E + 1, p=p / p.sum())
            if a == E:
                break
            avail[a] = False
            seq[a] += 1
    gum = np.zeros(E)
    for s in range(R // 50):
        removed, *_ = O.throughput_rollout(logits, 50, seed=11, stream=s)
        gum += removed.sum(0)
    p_seq, p_gum = seq / R, gum / R
    tol = 4.5 * np.sqrt(p_seq * (1 - p_seq) * 2 / R) + 1e-3
    assert np.all(np.abs(p_seq - p_gum) < tol), (p_seq, p_gum)


def test_lsq_fill_matches_lstsq():
    """Stacked-QR LS fill vs per-column numpy lstsq (AM side, column lines)."""
    rng = np.random.default_rng(3)
    for grid in (6, 9):
        r, c, v, n = O.poisson2d(grid, np.float64)
        idx, act, val = O.lines_from_coo(r, c, v, n, "col")
        a_idx, _, a_val = O.lines_from_coo(r, c, v, n, "col")
        keep = (rng.random(idx.shape) > 0.3) & (idx >= 0)
        m = O.lsq_fill(idx, keep, a_idx, a_val)
        A = sp.csc_matrix((v, (r, c)), shape=(n, n))
        for j in range(n):
            ref, J = O.lsq_fill_lstsq(idx, keep, A, j)
            got = m[j][keep[j] & (idx[j] >= 0)]
            np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)
        # the fill is the LS minimiser: residual of each column <= that of any perturbation
        M = O.m_to_csc(idx, m, n, np.float64)
        base = O.residual_fro_fp64(A, M)
        pert = O.m_to_csc(idx, np.where(keep, m + 1e-3 * rng.standard_normal(m.shape), 0), n, np.float64)
        assert O.residual_fro_fp64(A, pert) >= base


def test_trajectory_balance_loss_reference():
    from gflownet_spai_amd.log import trajectory_probs
    from gflownet_spai_amd.policy import BackwardPolicy
    from gflownet_spai_amd.utils import trajectory_balance_loss

    for name in ROLLOUTS:
        d = load(name)
        B, E = int(d["B"]), d["logits"].size - 1
        logits = torch.tensor(d["logits"], requires_grad=True)
        acts_bt = torch.tensor(d["actions"]).t().contiguous()
        fp = trajectory_probs(logits, acts_bt)
        np.testing.assert_allclose(fp.detach().numpy(), d["fwd_probs"], rtol=1e-6, atol=1e-9)
        torch.manual_seed(0)
        bwd = BackwardPolicy(1, 4, E + 1)
        bp = bwd.torch_forward(acts_bt).reshape(B, -1)
        np.testing.assert_allclose(bp.detach().numpy(), d["back_probs"], rtol=1e-5, atol=1e-7)
        loss = trajectory_balance_loss(torch.ones(1), torch.tensor(d["rewards"]), fp, bp)
        ref_loss = O.trajectory_balance_loss(torch.ones(1), torch.tensor(d["rewards"]), torch.tensor(d["fwd_probs"]),
                                             torch.tensor(d["back_probs"]))
        assert float(loss) == pytest.approx(float(d["loss"]), rel=1e-6)
        assert float(ref_loss) == pytest.approx(float(d["loss"]), rel=1e-6)
        loss.backward()
        np.testing.assert_allclose(logits.grad.numpy(), d["logits_grad"], rtol=2e-4,
                                   atol=2e-6 * np.abs(d["logits_grad"]).max())
