"""Reference-API pieces that need no GPU: GFlowNet.forward_probs (gflownet/gflownet.py:47-123)
against the reference's logged per-step probabilities, and the G7 assembled-M fixture
against the oracle's copy fill."""
import os

import numpy as np
import pytest
import torch

from oracle import spai_oracle as O

from .conftest import GOLDEN
from .test_hip_parity import FixedLogits


class CpuLogits(FixedLogits):
    def logits(self, data):  # pragma: no cover - forward_probs uses forward()
        raise AssertionError


@pytest.mark.parametrize("seed", range(4))
def test_forward_probs_reproduce_reference_step_probabilities(seed):
    """forward_probs(s, data_list, history) at every step t of a reference rollout gives, at the
    action the reference took, exactly the probability the reference logged (fwd_probs[b, t])
    for the samples still active; rows are renormalised (B > 1) and alpha = mean sigmoid."""
    from gflownet_spai_amd import GFlowNet
    d = np.load(os.path.join(GOLDEN, f"c1_rollout_s{seed}.npz"))
    B = int(d["B"])
    acts = torch.from_numpy(d["actions"])  # [T, B]
    T = acts.shape[0]
    g = GFlowNet(CpuLogits(d["logits"]), None, None)
    data_list = [None] * B
    for t in range(T):
        hist = [acts[s] for s in range(t)]
        with torch.no_grad():
            probs, alpha = g.forward_probs(None, data_list, hist)
        assert probs.shape == (B, 1, d["logits"].size)
        assert float(alpha) == pytest.approx(0.5)
        np.testing.assert_allclose(probs.sum(2).numpy(), 1.0, rtol=1e-5)
        for b in range(B):
            a = int(acts[t, b])
            if a < 0:
                continue
            assert float(probs[b, 0, a]) == pytest.approx(float(d["fwd_probs"][b, t]), rel=1e-6)


def test_assembled_m_fixture_matches_copy_fill():
    """G7: the reference's assembled M (kept entries, coalesced) == the oracle's copy fill."""
    d = np.load(os.path.join(GOLDEN, "c1p_removal.npz"))
    g = np.load(os.path.join(GOLDEN, "c1p_assembled.npz"))
    n = int(d["n"])
    off = 0
    for k, nnz in zip(g["sets"], g["nnz"]):
        mr, mc, mv = O.copy_fill_coo(d["rows"], d["cols"], d["vals"], d["removed"][k], n)
        order = np.lexsort((mc, mr))
        assert len(mr) == nnz
        assert np.array_equal(g["indices"][:, off:off + nnz], np.stack([mr[order], mc[order]]))
        assert np.array_equal(g["values"][off:off + nnz], mv[order])
        off += nnz


def test_thermal_like_standin_structure():
    """The C5 stand-in generator (utils.thermal_like): symmetric, <= 7 entries per row,
    diagonally dominant with positive diagonal (SPD), a permuted numbering (no band), and at
    full size thermal2's scale (1.23 M unknowns, 8.58 M nnz)."""
    import numpy as np
    import scipy.sparse as sp
    from gflownet_spai_amd import thermal_like
    A = thermal_like(40, seed=3).coalesce()
    n = A.shape[0]
    i = A.indices().numpy()
    M = sp.csr_matrix((A.values().numpy(), (i[0], i[1])), shape=(n, n))
    assert abs(M - M.T).max() == 0
    assert np.diff(M.indptr).max() <= 7
    d = M.diagonal()
    off = np.asarray(abs(M).sum(1)).ravel() - d
    assert np.all(d > off)  # strictly diagonally dominant (the 1e-3 anchor)
    bw = np.abs(i[0] - i[1]).max()
    assert bw > n // 2  # numbering scattered: no band left
    assert np.all(np.linalg.eigvalsh(M.toarray()) > 0)


def test_narrow_values_exact_only_and_cached():
    """kernels.narrow_values hands A's fp64 values to the residual kernels as fp32 only when
    every value survives the round trip (the same numbers), caches the copy on the Lines object
    and recomputes it when the values tensor is replaced."""
    from gflownet_spai_amd import kernels
    from gflownet_spai_amd.layout import build_lines
    r = torch.tensor([0, 0, 1, 1, 2])
    c = torch.tensor([0, 1, 0, 1, 2])
    exact = build_lines(r, c, torch.tensor([4.0, -1.0, -1.0, 4.0, 0.5], dtype=torch.float64), 3, "row", "cpu")
    v32 = kernels.narrow_values(exact)
    assert v32.dtype == torch.float32 and torch.equal(v32.double(), exact.val)
    assert kernels.narrow_values(exact) is v32  # cached
    inexact = build_lines(r, c, torch.tensor([4.0, -1.0, 0.1, 4.0, 0.5], dtype=torch.float64), 3, "row", "cpu")
    assert kernels.narrow_values(inexact) is inexact.val  # 0.1 is not an fp32 number: stays fp64
    exact.val = exact.val * (1 + 2.0 ** -40)
    assert kernels.narrow_values(exact) is exact.val  # new values, checked again
    f32 = build_lines(r, c, torch.ones(5), 3, "row", "cpu")
    assert kernels.narrow_values(f32) is f32.val
