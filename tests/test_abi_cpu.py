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
    assert lib.spai_rollout_ws_offset(1000, 2, 6) == 2 * 2 * 2048 + 2 * 8
    assert lib.spai_rollout_ws_offset(1000, 2, 3) == 2048 and lib.spai_rollout_ws_offset(1000, 2, 9) == -1
    assert 0 < lib.spai_rollout_ws_offset(1000, 2, 2) < lib.spai_rollout_workspace_bytes(1000, 2)
    with pytest.raises(ValueError):
        _lib.check(rc, "spai_rollout_select")
    assert lib.spai_fill_workspace_bytes(1000, 4) >= 1000 * 4 * 8
    assert lib.spai_logits_stats_workspace_bytes(10, 2) > 0
    # the Gram-cached residual: null cache, misaligned cache, and widths outside 5 / 7 / 13 (rejected
    # before any device access: the pointers below are never dereferenced)
    p = 4096
    args = lambda W, WA, gram, a_dt: (100, 0, 100, W, p, 0, p, _lib.DTYPE_F32, 0, WA, p, p, a_dt, p, gram,
                                      _lib.DTYPE_F32, p, 1, p, p, 1 << 20, None)
    rc = lib.spai_residual_lines_gram(*args(13, 7, None, _lib.DTYPE_F32))
    assert rc == _lib.SPAI_ERR_INVALID and b"null pointer" in lib.spai_last_error()
    rc = lib.spai_residual_lines_gram(*args(13, 7, p + 4, _lib.DTYPE_F32))
    assert rc == _lib.SPAI_ERR_INVALID and b"16-byte aligned" in lib.spai_last_error()
    for W, WA, a_dt in ((9, 7, _lib.DTYPE_F32), (5, 7, _lib.DTYPE_F32), (13, 7, _lib.DTYPE_F64)):
        rc = lib.spai_residual_lines_gram(*args(W, WA, p, a_dt))
        assert rc == _lib.SPAI_ERR_UNSUPPORTED and b"spai_residual_lines" in lib.spai_last_error()


def test_binding_signatures_match_header_parameter_lists():
    """_lib.SIGNATURES (the package's ctypes binding) agrees with include/spai_hip.h argument for
    argument: same count and, per position, the ctypes type the header's C type needs."""
    from .abi_header import parse_header
    hdr = parse_header()
    assert sorted(hdr) == sorted(_lib.SIGNATURES)
    for name, (res, args) in _lib.SIGNATURES.items():
        h_res, h_args, h_names = hdr[name]
        assert res is h_res, (name, res, h_res)
        assert len(args) == len(h_args), (name, len(args), len(h_args))
        for i, (a, h) in enumerate(zip(args, h_args)):
            assert a is h, (name, h_names[i], a, h)


def test_integration_stub_matches_header():
    """The reference-side binding published in INTEGRATION.md binds every function it calls with
    the header's parameter list (ABI 17), and calls each with that many arguments."""
    import ast
    from .abi_header import integration_stub, parse_header
    hdr = parse_header()
    src = integration_stub()
    tree = ast.parse(src)
    alias = {"_P": ctypes.c_void_p, "_I": ctypes.c_int32, "_L": ctypes.c_int64, "_Z": ctypes.c_size_t}
    bound = {}
    for node in ast.walk(tree):
        if not isinstance(node, ast.Assign):
            continue
        targets = node.targets[0].elts if isinstance(node.targets[0], ast.Tuple) else [node.targets[0]]
        values = node.value.elts if isinstance(node.value, ast.Tuple) and len(targets) > 1 else [node.value]
        for t, v in zip(targets, values):
            if isinstance(t, ast.Attribute) and t.attr == "argtypes" and isinstance(t.value, ast.Attribute):
                bound[t.value.attr] = [alias[e.id] for e in v.elts]
    assert {"spai_actions_to_removed", "spai_fill_residual", "spai_fill_workspace_bytes"} <= set(bound)
    for name, args in bound.items():
        h_args = hdr[name][1]
        assert len(args) == len(h_args), (name, len(args), len(h_args))
        assert all(a is h for a, h in zip(args, h_args)), name
    calls = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute) and node.func.attr.startswith("spai_"):
            calls.setdefault(node.func.attr, []).append(len(node.args))
    assert calls["spai_fill_residual"] == [23] and calls["spai_actions_to_removed"] == [10]
    for name, ns in calls.items():
        assert all(k == len(hdr[name][1]) for k in ns), name


def test_sharded_gflownet_needs_an_explicit_split_and_aligned_lines():
    """A sharded GFlowNet must name its split (the splits read s0 differently); both splits use
    256-line-aligned shards (the exact residual sums are invariant only for aligned shards)."""
    import types
    from gflownet_spai_amd import GFlowNet
    from gflownet_spai_amd.distributed import LINE_ALIGN
    env = types.SimpleNamespace(matrix_size=96 * 96)
    with pytest.raises(ValueError, match="split"):
        GFlowNet(None, None, env, mode="throughput", shard=(0, 3, None))
    GFlowNet(None, None, env, mode="throughput", shard=(0, 1, None))  # one rank: no split needed
    for split in ("columns", "slices"):
        rngs = [GFlowNet(None, None, env, mode="throughput", shard=(r, 3, None), split=split).lines for r in range(3)]
        assert rngs[0][0] == 0 and rngs[-1][1] == env.matrix_size
        assert all(rngs[i][1] == rngs[i + 1][0] for i in range(2))
        assert all(b % LINE_ALIGN == 0 for b, _ in rngs)


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspai_hip.so not built (run build())")
def test_kernel_timer_arguments_without_gpu():
    """spai_kernel_timer_*: out-of-range kernels are rejected; an armed timer with no launch recorded
    reads back zero launches (neither call touches the device then)."""
    lib = _lib.load()
    assert lib.spai_kernel_timer_arm(4, 1) == _lib.SPAI_ERR_INVALID and b"out of range" in lib.spai_last_error()
    assert lib.spai_kernel_timer_arm(-1, 0) == _lib.SPAI_ERR_INVALID
    cnt, ms = ctypes.c_int32(-1), ctypes.c_double(-1.0)
    assert lib.spai_kernel_timer_read(9, ctypes.byref(cnt), ctypes.byref(ms)) == _lib.SPAI_ERR_INVALID
    assert lib.spai_kernel_timer_read(0, None, None) == _lib.SPAI_ERR_INVALID
    for k in range(4):
        assert lib.spai_kernel_timer_arm(k, 1) == _lib.SPAI_OK
        assert lib.spai_kernel_timer_read(k, ctypes.byref(cnt), ctypes.byref(ms)) == _lib.SPAI_OK
        assert cnt.value == 0 and ms.value == 0.0
        assert lib.spai_kernel_timer_arm(k, 0) == _lib.SPAI_OK
