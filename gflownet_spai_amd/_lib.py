"""ctypes binding of libspai_hip.so (the C ABI declared in include/spai_hip.h).

The shared library is built in-tree (``gflownet_spai_amd/libspai_hip.so``) by
``__graft_entry__.build()`` / ``make -C gflownet_spai_amd/csrc``.  There is no
CPU fallback: if the library is missing or no GPU is present, every compute entry
point raises.  Status codes map to the exception types the reference raises
(ValueError for bad input, ``gflownet/utils.py:100-121``; RuntimeError otherwise).
"""
from __future__ import annotations

import ctypes
import os

import torch

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libspai_hip.so")
if os.environ.get("SPAI_LIB_VARIANT"):  # A/B timing of kernel variants built under build/variants/
    LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "variants",
                            os.environ["SPAI_LIB_VARIANT"])

SPAI_OK, SPAI_ERR_INVALID, SPAI_ERR_HIP, SPAI_ERR_UNSUPPORTED = 0, 1, 2, 3
FILL_COPY, FILL_LSQ = 0, 1  # (the Householder-QR fill has its own entry point)
DTYPE_F32, DTYPE_F64 = 0, 1
ABI_VERSION = 20
RES2_LIMBS = 8  # SPAI_RES2_LIMBS

_c_i32, _c_i64, _c_u64, _c_sz, _c_p = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/spai_hip.h one-to-one.
SIGNATURES = {
    "spai_abi_version": (ctypes.c_int, []),
    "spai_last_error": (ctypes.c_char_p, []),
    "spai_kernel_timer_arm": (ctypes.c_int, [_c_i32, _c_i32]),
    "spai_kernel_timer_read": (ctypes.c_int, [_c_i32, _c_p, _c_p]),
    "spai_logits_stats_workspace_bytes": (_c_sz, [_c_i32, _c_i32]),
    "spai_logits_stats": (ctypes.c_int, [_c_p, _c_i64, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_sz, _c_p]),
    "spai_parity_step_workspace_bytes": (_c_sz, [_c_i32, _c_i32]),
    "spai_parity_step": (ctypes.c_int, [_c_p, _c_i64, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_p,
                                        _c_p, _c_p, _c_p, _c_sz, _c_p]),
    "spai_rollout_workspace_bytes": (_c_sz, [_c_i32, _c_i32]),
    "spai_rollout_select": (ctypes.c_int, [_c_p, _c_i64, _c_i32, _c_i32, _c_p, _c_u64, _c_u64, _c_p, _c_i32, _c_i32,
                                           _c_i32, _c_p, _c_i32, _c_p, _c_p, _c_sz, _c_p]),
    "spai_rollout_select_pm": (ctypes.c_int, [_c_p, _c_i64, _c_i32, _c_i32, _c_p, _c_p, _c_i32, _c_u64, _c_u64, _c_p,
                                              _c_i32, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p, _c_sz, _c_p]),
    "spai_policy_lmax_parts": (ctypes.c_int32, [_c_i32]),
    "spai_rollout_merge": (ctypes.c_int, [_c_p, _c_i64, _c_i32, _c_i32, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_sz,
                                          _c_p]),
    "spai_rollout_sort": (ctypes.c_int, [_c_p, _c_i64, _c_i32, _c_i32, _c_p, _c_i32, _c_i32, _c_i64, _c_p, _c_p,
                                         _c_p, _c_sz, _c_p]),
    "spai_rollout_finish": (ctypes.c_int, [_c_p, _c_i64, _c_i32, _c_i32, _c_p, _c_p, _c_i32, _c_i32, _c_i64, _c_p,
                                           _c_p, _c_p, _c_p, _c_sz, _c_p]),
    "spai_rollout_order": (ctypes.c_int, [_c_p, _c_i64, _c_i32, _c_i32, _c_p, _c_p, _c_i64, _c_p, _c_p, _c_p, _c_p,
                                          _c_sz, _c_p]),
    "spai_actions_to_removed": (ctypes.c_int, [_c_p, _c_i64, _c_i64, _c_i32, _c_i32, _c_i32, _c_p, _c_i32, _c_p,
                                               _c_p]),
    "spai_fill_workspace_bytes": (_c_sz, [_c_i32, _c_i32]),
    "spai_rewards": (ctypes.c_int, [_c_p, _c_p, _c_i32, _c_i64, _c_i32, ctypes.c_double, ctypes.c_double, _c_p, _c_p,
                                    _c_p, _c_p, _c_p]),
    "spai_fill_reduce_rewards": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_p, _c_i64, _c_i32, ctypes.c_double,
                                                ctypes.c_double, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "spai_gram_bytes": (_c_sz, [_c_i32, _c_i32]),
    "spai_gram_build": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p, _c_i32, _c_p, _c_p]),
    "spai_fill_residual_gram": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_i32, _c_i32,
                                               _c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p, _c_sz, _c_p]),
    "spai_gram_compact": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "spai_fill_lines_gram": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_i32, _c_i32,
                                            _c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_sz, _c_p]),
    "spai_policy_params": (_c_sz, [_c_i32, _c_i32, _c_i32]),
    "spai_policy_workspace_bytes": (_c_sz, [_c_i32, _c_i32, _c_i32]),
    "spai_policy_logits": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
                                          _c_i32, _c_p, _c_p, _c_i32, _c_i32, _c_p, _c_sz, _c_p]),
    "spai_policy_rows_constant": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_p, _c_p]),
    "spai_rollout_ws_offset": (_c_i64, [_c_i32, _c_i32, _c_i32]),
    "spai_residual_workspace_bytes": (_c_sz, [_c_i32, _c_i32]),
    "spai_residual_lines": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_i64, _c_p, _c_i32, _c_i64,
                                           _c_i32, _c_p, _c_p, _c_i32, _c_i32, _c_p, _c_p, _c_sz, _c_p]),
    "spai_residual_lines_gram": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_i64, _c_p, _c_i32, _c_i64,
                                                _c_i32, _c_p, _c_p, _c_i32, _c_p, _c_p, _c_i32, _c_p, _c_i32, _c_p,
                                                _c_p, _c_sz, _c_p]),
    "spai_logp_grad_workspace_bytes": (_c_sz, [_c_i32, _c_i32, _c_i32, _c_i32]),
    "spai_logp_grad": (ctypes.c_int, [_c_p, _c_i64, _c_i32, _c_i32, _c_p, _c_p, _c_i64, _c_i32, _c_p, _c_i64, _c_p,
                                      _c_i64, _c_p, _c_i32, _c_p, _c_p, _c_sz, _c_p]),
    "spai_lstm_forward": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_i64, _c_p, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p,
                                         _c_p, _c_p]),
    "spai_policy_backward_workspace_bytes": (_c_sz, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32]),
    "spai_policy_backward": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
                                            _c_p, _c_p, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_sz, _c_p]),
    "spai_ell_spmv":(ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_p, _c_i32, _c_p, _c_p, _c_p]),
    "spai_mtx_header": (ctypes.c_int, [ctypes.c_char_p, _c_p, _c_p]),
    "spai_mtx_read": (ctypes.c_int, [ctypes.c_char_p, _c_p, _c_p, _c_p, _c_i64, _c_i32, _c_p]),
    "spai_lstm_states_floats": (_c_sz, [_c_i32, _c_i32, _c_i32]),
    "spai_lstm_backward_workspace_bytes": (_c_sz, [_c_i32, _c_i32, _c_i32]),
    "spai_lstm_backward": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_i64, _c_p, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_p,
                                          _c_p, _c_p, _c_p, _c_sz, _c_p]),
    "spai_fill_reduce": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_p, _c_p, _c_p]),
    "spai_fill_residual": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_i32, _c_p, _c_p,
                                          _c_i32, _c_i32, _c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p, _c_p, _c_sz,
                                          _c_p]),
    "spai_res2_from_limbs": (ctypes.c_int, [_c_i32, _c_p, _c_p, _c_p]),
    "spai_qr_max_rows": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p, _c_p]),
    "spai_fill_lines_qr": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_i32, _c_p, _c_p, _c_i32,
                                          _c_i32, _c_i32, _c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_sz, _c_p]),
    "spai_set_sort_blocks": (ctypes.c_int, [_c_i32]),
    "spai_bitmap_pack": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_p, _c_p]),
    "spai_window_pack": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_p, _c_p]),
    "spai_qr_cache_bytes": (_c_sz, [_c_i32, _c_i32, _c_i32]),
    "spai_qr_factor": (ctypes.c_int, [_c_i32, _c_i32, _c_p, _c_p, _c_i32, _c_p, _c_p, _c_i32, _c_i32, _c_p, _c_sz,
                                      _c_p]),
    "spai_fill_lines_qr_cached": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_i32,
                                                 _c_i32, _c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_sz, _c_p]),
    "spai_line_cache_dict": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_p, _c_sz, _c_i32, _c_p, _c_sz, _c_p, _c_p,
                                            _c_p]),
    "spai_fill_lines_gram_dict": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_p, _c_p, _c_p, _c_i32,
                                                 _c_p, _c_i32, _c_p, _c_i32, _c_i32, _c_p, _c_i32, _c_p, _c_sz, _c_p]),
}

_lib = None


class SpaiUnavailable(RuntimeError):
    """libspai_hip.so is missing or cannot run here (no GPU)."""


def load():
    """Load and type the library (no GPU needed just to load)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SpaiUnavailable(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                              "or `make -C gflownet_spai_amd/csrc`")
    lib = ctypes.CDLL(LIB_PATH)
    variant = bool(os.environ.get("SPAI_LIB_VARIANT"))  # an A/B build may predate newer entry points
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.spai_abi_version() != ABI_VERSION and not variant:
        raise SpaiUnavailable(f"libspai_hip ABI {lib.spai_abi_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def require_device(t: torch.Tensor):
    if not t.is_cuda:
        raise SpaiUnavailable("gflownet_spai_amd runs on the MI355X only (tensor on %s); there is no CPU path" % t.device)


def check(status: int, where: str):
    if status == SPAI_OK:
        return
    msg = f"{where}: {load().spai_last_error().decode(errors='replace')}"
    if status == SPAI_ERR_INVALID:
        raise ValueError(msg)
    if status == SPAI_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise RuntimeError(msg)


def ptr(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_ws_cache: dict = {}


def workspace(nbytes: int, device, tag: str) -> torch.Tensor:
    """Caller-owned workspace (a byte tensor from torch's caching allocator), reused per
    (tag, device, current stream) so concurrent streams never share one."""
    key = (tag, str(device), torch.cuda.current_stream(device).cuda_stream)
    ws = _ws_cache.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _ws_cache[key] = ws
    return ws
