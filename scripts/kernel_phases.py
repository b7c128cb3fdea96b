"""Per-phase wall-clock of k_sort2, k_tile and k_splitters' splitter blocks (variant build with -DSPAI_PROF):
  make -C gflownet_spai_amd/csrc BUILD=../../build/prof OUT=../../build/variants/libspai_prof.so EXTRA=-DSPAI_PROF
  SPAI_LIB_VARIANT=libspai_prof.so python scripts/kernel_phases.py
Phase times are summed over the blocks of each kernel (thread 0's view, stamps after the
phase's barrier) and divided by the rollouts and by the resident block count."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gflownet_spai_amd import _lib, kernels  # noqa: E402

E, B, iters = 5238784, int(os.environ.get("B", 8)), 10
logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
logits[E] = bench.terminal_logit(logits[:E].numpy(), 0.2)
lg, lmax, z = kernels.logits_stats(logits.cuda(), B)
lib = _lib.load()
buf = (ctypes.c_ulonglong * 64)()
for it in range(iters + 1):
    removed, counts, ws = kernels.rollout_select(lg, B, lmax, 1234, it)
    kernels.rollout_order(lg, B, lmax, counts, ws)
    torch.cuda.synchronize()
    if it == 0:
        lib.spai_debug_prof(buf, 1)  # warm-up: discard
lib.spai_debug_prof(buf, 0)
ncu = torch.cuda.get_device_properties(0).multi_processor_count
kern = {
    "k_sort2": (0, ["wait", "flush", "map", "mapbar", "issue", "minmax", "subcount", "subscan", "scatter", "rank", "place",
                 "wscan", "store"], ncu),
    "k_tile": (32, ["prologue", "keys", "atomics", "offsets", "win_place", "win_write", "list", "lut_rounds"], ncu),
    "k_splitters": (16, ["counts", "keys", "hist", "scan", "splitters", "lut"], B),
}
for name, (base, phases, resident) in kern.items():
    tot = sum(buf[base + i] for i in range(len(phases)))
    print(f"{name}: per resident block slot (us, {resident} slots, {iters} rollouts)")
    for i, nm in enumerate(phases):
        print(f"  {nm:11s} {buf[base + i] / 100.0 / iters / resident:8.2f}  ({100.0 * buf[base + i] / max(tot, 1):.1f}%)")
    print(f"  total       {tot / 100.0 / iters / resident:8.2f}")
