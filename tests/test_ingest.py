"""Ingest: the native Matrix Market reader against scipy.io.mmread (the
reference's reader, gflownet/utils.py:54-63, GFlowNet100.py:44-46), the spilu L@U candidate
pattern of GFlowNet100.py:126-153, and (GPU) an env built from a file."""
import os

import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp
import torch

from gflownet_spai_amd.utils import (load_mtx_file, lu_candidate_matrix, market_matrix_to_sparse_tensor,
                                     poisson_2d, read_mtx)

HERE = os.path.dirname(os.path.abspath(__file__))


def write(tmp_path, name, header, size, lines):
    p = tmp_path / name
    p.write_text(header + "\n% a comment\n%\n" + size + "\n" + "\n".join(lines) + "\n")
    return str(p)


def ref_coo(path):
    """gflownet/utils.py:54-63 restated: mmread -> tocoo -> (row, col, float64 data)."""
    m = scipy.io.mmread(path).tocoo()
    return m.row.astype(np.int64), m.col.astype(np.int64), m.data.astype(np.float64), m.shape


def same(path, threads=0):
    r, c, v, shape = read_mtx(path, threads)
    rr, rc, rv, rshape = ref_coo(path)
    assert shape == rshape
    assert np.array_equal(r, rr) and np.array_equal(c, rc)
    assert np.array_equal(v, rv)  # correctly rounded on both sides: bit-identical


@pytest.mark.parametrize("field", ["real", "integer", "pattern"])
@pytest.mark.parametrize("sym", ["general", "symmetric", "skew-symmetric"])
def test_reader_matches_mmread(tmp_path, field, sym):
    rng = np.random.default_rng(len(field) * 7 + len(sym))
    n, k = 37, 150
    i = rng.integers(1, n + 1, k)
    j = rng.integers(1, n + 1, k)
    if sym != "general":  # lower triangle, as (skew-)symmetric files store it
        i, j = np.maximum(i, j), np.minimum(i, j)
        if sym == "skew-symmetric":
            keep = i != j
            i, j = i[keep], j[keep]
    vals = rng.standard_normal(i.size) * 10.0 ** rng.integers(-12, 12, i.size)
    lines = []
    for a, b, v in zip(i, j, vals):
        if field == "real":
            lines.append(f"{a} {b} {float(v)!r}")
        elif field == "integer":
            lines.append(f"{a} {b} {int(v * 1000) % 100000 - 50000}")
        else:
            lines.append(f"{a} {b}")
    p = write(tmp_path, "m.mtx", f"%%MatrixMarket matrix coordinate {field} {sym}", f"{n} {n} {len(lines)}", lines)
    same(p)


def test_reader_multichunk_order_and_whitespace(tmp_path):
    """Several MB so the body is split over threads; tabs, CRLF and blank lines in between."""
    rng = np.random.default_rng(7)
    n, k = 5000, 200_000
    i, j = rng.integers(1, n + 1, k), rng.integers(1, n + 1, k)
    i, j = np.maximum(i, j), np.minimum(i, j)
    v = rng.standard_normal(k)
    body = []
    for t, (a, b, x) in enumerate(zip(i, j, v)):
        sep = "\t" if t % 3 == 0 else " "
        body.append(f"{a}{sep}{b}{sep}{x:.17g}" + ("\r" if t % 5 == 0 else ""))
        if t % 1000 == 999:
            body.append("")
    p = write(tmp_path, "big.mtx", "%%MatrixMarket matrix coordinate real symmetric", f"{n} {n} {k}", body)
    assert os.path.getsize(p) > 4 << 20
    for threads in (1, 3, 8):
        same(p, threads)


def test_sparse_tensor_and_csr_like_reference(tmp_path):
    A = poisson_2d(6).coalesce()
    r, c = A.indices().numpy() + 1
    v = A.values().numpy()
    low = r >= c
    lines = [f"{a} {b} {x}" for a, b, x in zip(r[low], c[low], v[low])]
    p = write(tmp_path, "p.mtx", "%%MatrixMarket matrix coordinate real symmetric", f"36 36 {len(lines)}", lines)
    t = market_matrix_to_sparse_tensor(p)
    rr, rc, rv, _ = ref_coo(p)
    assert t.dtype == torch.float64 and not t.is_coalesced()
    assert np.array_equal(t._indices().numpy(), np.vstack([rr, rc]))
    assert np.array_equal(t._values().numpy(), rv)
    M = load_mtx_file(p)
    ref = sp.csr_matrix(scipy.io.mmread(p))
    assert (M != ref).nnz == 0 and np.array_equal(M.toarray(), A.to_dense().numpy())


@pytest.mark.parametrize("text,err", [
    ("%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n", NotImplementedError),
    ("%%MatrixMarket matrix coordinate complex general\n2 2 1\n1 1 1 0\n", NotImplementedError),
    ("%%MatrixMarket matrix coordinate real general\n2 2 2\n1 1 1.0\n", ValueError),       # too few entries
    ("%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1.0\n", ValueError),       # index out of range
    ("%%MatrixMarket matrix coordinate real symmetric\n2 3 1\n1 1 1.0\n", ValueError),     # non-square symmetric
    ("not a header\n", ValueError),
])
def test_reader_rejects_like_the_reference(tmp_path, text, err):
    p = tmp_path / "bad.mtx"
    p.write_text(text)
    with pytest.raises(err):
        read_mtx(str(p))


def test_reader_missing_file():
    with pytest.raises(ValueError):
        read_mtx("/nonexistent/x.mtx")


def test_lu_candidate_matrix_is_the_drivers():
    """GFlowNet100.py:126-153 restated inline on the same A: identical indices and fp32 values."""
    import scipy.sparse.linalg as spla
    A = poisson_2d(8).coalesce()
    Acsr = sp.csr_matrix((A.values().double().numpy(), tuple(A.indices().numpy())), shape=A.shape)
    t = lu_candidate_matrix(Acsr)
    ilu = spla.spilu(Acsr)
    LU = (sp.tril(ilu.L, format="csr") @ sp.triu(ilu.U, format="csr")).tocoo()
    assert t.dtype == torch.float32 and tuple(t.shape) == A.shape
    assert np.array_equal(t._indices().numpy(), np.vstack((LU.row, LU.col)))
    assert np.array_equal(t._values().numpy(), torch.FloatTensor(LU.data).numpy())
    assert t._nnz() >= A._nnz()  # ILU fill only adds entries to A's pattern


@pytest.mark.gpu
def test_env_from_mtx_file_copy_fill_vs_oracle(tmp_path):
    """A symmetric MTX file -> native reader -> L@U candidate -> PreconditionerEnv on the GPU:
    the env's action ids are the raw COO positions and its copy-fill residuals match the fp64
    oracle on random removal sets."""
    from oracle import spai_oracle as O
    from gflownet_spai_amd import PreconditionerEnv
    A = poisson_2d(12).coalesce()
    r, c = A.indices().numpy() + 1
    v = A.values().numpy()
    low = r >= c
    lines = [f"{a} {b} {x}" for a, b, x in zip(r[low], c[low], v[low])]
    p = write(tmp_path, "a.mtx", "%%MatrixMarket matrix coordinate real symmetric", f"144 144 {len(lines)}", lines)
    C = lu_candidate_matrix(load_mtx_file(p))
    n = C.shape[0]
    rows, cols = C._indices().numpy()
    vals = C._values().numpy()
    env = PreconditionerEnv(n, C, C)
    E = env.num_actions - 1
    assert E == C._nnz()
    Ccsr = sp.csr_matrix((vals.astype(np.float64), (rows, cols)), shape=(n, n))
    rng = np.random.default_rng(0)
    K = 6
    removed = rng.random((K, E)) < 0.3
    T = int(removed.sum(1).max())
    acts = -np.ones((K, T + 1), np.int64)
    for k in range(K):
        ids = np.flatnonzero(removed[k])
        acts[k, :ids.size] = rng.permutation(ids)
        acts[k, ids.size] = E
    env.update(None, torch.from_numpy(acts), torch.tensor(0.5))
    res = env.last_residual.cpu().numpy()
    for k in range(K):
        mr, mc, mv = O.copy_fill_coo(rows, cols, vals, removed[k], n)
        M = sp.csr_matrix((mv.astype(np.float64), (mr, mc)), shape=(n, n))
        assert res[k] == pytest.approx(O.residual_fro_fp64(M, Ccsr), rel=1e-12)


@pytest.mark.gpu
def test_lu_candidate_driver_config_64_vs_oracle():
    """The reference driver's own configuration at 64^2: the candidate is
    spilu's L@U of a 4,096-unknown Poisson matrix (GFlowNet100.py:126-153) with lines up to ~230
    wide, and initial_matrix = original_matrix = that candidate (GFlowNet100.py:173), side MA, copy
    fill (preconditioner.py:32-52).  env.update on 8 random removal sets (5-80 % removed) and on a
    throughput rollout's removal sets: every ||M C - I||_F (the any-width copy residual, k_line_hash)
    against the fp64 oracle, and every reward against the reference formula."""
    from oracle import spai_oracle as O
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv
    A = poisson_2d(64).coalesce()
    Acsr = sp.csr_matrix((A.values().double().numpy(), tuple(A.indices().numpy())), shape=A.shape)
    C = lu_candidate_matrix(Acsr)
    n = C.shape[0]
    rows, cols = C._indices().numpy()
    vals = C._values().numpy()
    assert np.bincount(rows, minlength=n).max() > 13 * 10  # lines far wider than the stencil kernels'
    env = PreconditionerEnv(n, C, C)
    E = env.num_actions - 1
    assert E == C._nnz()
    Ccsr = sp.csr_matrix((vals.astype(np.float64), (rows, cols)), shape=(n, n))
    rng = np.random.default_rng(64)
    fracs = np.array([0.05, 0.1, 0.2, 0.3, 0.4, 0.5, 0.65, 0.8])
    K = fracs.size
    removed = rng.random((K, E)) < fracs[:, None]
    T = int(removed.sum(1).max())
    acts = -np.ones((K, T + 1), np.int64)
    for k in range(K):
        ids = np.flatnonzero(removed[k])
        acts[k, :ids.size] = rng.permutation(ids)
        acts[k, ids.size] = E
    alpha = 0.5
    rw = torch.stack(env.update(None, torch.from_numpy(acts), torch.tensor(alpha))).cpu().numpy()
    res = env.last_residual.cpu().numpy()
    r0 = O.residual_fro_fp64(Ccsr, Ccsr)
    for k in range(K):
        mr, mc, mv = O.copy_fill_coo(rows, cols, vals, removed[k], n)
        M = sp.csr_matrix((mv.astype(np.float64), (mr, mc)), shape=(n, n))
        ref = O.residual_fro_fp64(M, Ccsr)
        assert res[k] == pytest.approx(ref, rel=1e-12)
        assert rw[k] == pytest.approx(O.reward(ref, E - int(removed[k].sum()), alpha, r0, 2 * E * n, n), rel=1e-9)

    # a throughput rollout over this candidate: its removal sets are the oracle's, its residuals too
    class Fixed(torch.nn.Module):
        def __init__(self, l):
            super().__init__()
            self.l = l

        def logits(self, data):
            return self.l.to(env.device), torch.tensor(0.5, device=env.device)

    lg = torch.randn(E + 1, generator=torch.Generator().manual_seed(3))
    lg[E] = 2.0
    with torch.no_grad():
        log = GFlowNet(Fixed(lg), None, env, mode="throughput", seed=9).sample_states([C] * 4, return_log=True)
    rem_o, a_o, _, c_o = O.throughput_rollout(lg.numpy(), 4, 9, 0)
    assert np.array_equal(log.counts.cpu().numpy(), c_o)
    assert np.array_equal(log.actions.cpu().numpy(), a_o)
    res = env.last_residual.cpu().numpy()
    for k in range(4):
        mr, mc, mv = O.copy_fill_coo(rows, cols, vals, rem_o[k], n)
        M = sp.csr_matrix((mv.astype(np.float64), (mr, mc)), shape=(n, n))
        assert res[k] == pytest.approx(O.residual_fro_fp64(M, Ccsr), rel=1e-12)
