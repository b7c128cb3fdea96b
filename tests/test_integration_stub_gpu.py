"""INTEGRATION.md's reference-side ctypes binding, executed as published (the code block is read
from the document, not copied), on the reference's own golden removal sets: its ||M A - I||_F
must equal the reference's ``calculate_residual`` values (preconditioner.py:79-93) captured in
tests/golden (exact for the integer stencils, 1e-6 relative for the random-valued 64 x 64 case)
and its nnz(M) the reference's M._nnz()."""
import os

import numpy as np
import pytest
import torch

from .abi_header import integration_stub
from .conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _stub_namespace():
    from gflownet_spai_amd import _lib
    os.environ["SPAI_HIP_LIB"] = _lib.LIB_PATH
    ns = {"__name__": "spai_binding"}
    exec(compile(integration_stub(), "INTEGRATION.md:spai_binding.py", "exec"), ns)
    return ns


@pytest.mark.parametrize("name,exact", [("c1_removal.npz", True), ("c1p_removal.npz", True),
                                        ("rand64_removal.npz", False)])
def test_integration_stub_reproduces_reference_residuals(name, exact):
    ns = _stub_namespace()
    d = np.load(os.path.join(GOLDEN, name))
    n = int(d["n"])
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([d["rows"], d["cols"]]).astype(np.int64)),
                                torch.from_numpy(d["vals"]), (n, n))
    removed = d["removed"]
    K, E = removed.shape
    T = int(removed.sum(1).max()) + 1
    acts = -np.ones((K, T), np.int64)
    for k in range(K):
        ids = np.flatnonzero(removed[k])
        acts[k, :ids.size] = np.random.default_rng(k).permutation(ids)
        acts[k, ids.size] = E  # the terminal id is ignored (utils.py:323)
    res, nnz = ns["residuals"](A, A, torch.from_numpy(acts))
    res = res.cpu().numpy()
    assert np.array_equal(nnz.cpu().numpy(), d["nnz_m"])
    if exact:
        assert np.array_equal(res, d["r_ma"])
    else:
        np.testing.assert_allclose(res, d["r_ma"], rtol=1e-6)


def test_integration_stub_maps_status_to_exceptions():
    """The stub's _ok maps SPAI_ERR_INVALID to ValueError with spai_last_error()'s text (the
    reference raises ValueError for bad input, gflownet/utils.py:100-121)."""
    ns = _stub_namespace()
    lib = ns["_lib"]
    rc = lib.spai_fill_residual(7, 10, 0, 10, 5, None, None, None, 5, None, None, 0, 1, None, 1, 0, None, 0,
                                None, None, None, 0, None)
    with pytest.raises(ValueError, match="fill_mode"):
        ns["_ok"](rc)
