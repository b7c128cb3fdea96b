"""The C-ABI library loads without a GPU and exports every entry point include/spai_hip.h
declares, with the signatures the ctypes binding uses (no compute calls here)."""
import ctypes
import os
import re

import pytest

from gflownet_spai_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "spai_hip.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(spai_[a-z0-9_]+)\s*\(", text)))


def test_header_lists_the_bound_functions():
    assert header_functions() == sorted(_lib.SIGNATURES)


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspai_hip.so not built (run build())")
def test_library_exports_every_symbol():
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.spai_abi_version() == _lib.ABI_VERSION
    assert isinstance(lib.spai_last_error(), bytes)


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspai_hip.so not built (run build())")
def test_argument_validation_without_gpu():
    """Argument checks run before any HIP call, so they are exercisable on a CPU host."""
    lib = _lib.load()
    rc = lib.spai_fill_residual(7, 10, 0, 10, 5, None, None, None, 5, None, None, 0, 1, None, 1, 0, None, 0,
                                None, None, None, 0, None)
    assert rc == _lib.SPAI_ERR_INVALID
    assert b"fill_mode" in lib.spai_last_error()
    rc = lib.spai_rollout_select(None, 0, 10, 1, None, 0, 0, None, 0, 0, 1, None, 1, None, None, 0, None)
    assert rc == _lib.SPAI_ERR_INVALID
    rc = lib.spai_rollout_sort(None, 0, 10, 1, None, 2, 2, 11, None, None, None, 0, None)
    assert rc == _lib.SPAI_ERR_INVALID and b"null pointer" in lib.spai_last_error()
    rc = lib.spai_rollout_merge(None, 0, 10, 1, None, 0, 2, None, None, 0, None)
    assert rc == _lib.SPAI_ERR_INVALID and b"null pointer" in lib.spai_last_error()
    assert lib.spai_rollout_ws_offset(1000, 2, 6) == 2 * 2 * 1024 + 2 * 8
    assert lib.spai_rollout_ws_offset(1000, 2, 3) == 1024 and lib.spai_rollout_ws_offset(1000, 2, 9) == -1
    assert 0 < lib.spai_rollout_ws_offset(1000, 2, 2) < lib.spai_rollout_workspace_bytes(1000, 2)
    with pytest.raises(ValueError):
        _lib.check(rc, "spai_rollout_select")
    assert lib.spai_fill_workspace_bytes(1000, 4) >= 1000 * 4 * 8
    assert lib.spai_logits_stats_workspace_bytes(10, 2) > 0
