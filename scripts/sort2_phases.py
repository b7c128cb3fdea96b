"""Per-phase wall-clock of k_sort2 (variant build with -DSPAI_PROF):
SPAI_LIB_VARIANT=libspai_prof.so python scripts/sort2_phases.py"""
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
buf = (ctypes.c_ulonglong * 16)()
names = ["table", "gather", "minmax", "subcount", "subscan", "scatter", "rank", "place", "wscan", "store"]
for it in range(iters + 1):
    removed, counts, ws = kernels.rollout_select(lg, B, lmax, 1234, it)
    kernels.rollout_order(lg, B, lmax, counts, ws)
    torch.cuda.synchronize()
    if it == 0:
        lib.spai_debug_sort2_prof(buf, 1)  # first iteration is warm-up: read and reset
lib.spai_debug_sort2_prof(buf, 0)
tot = sum(buf[i] for i in range(len(names)))
nblk = torch.cuda.get_device_properties(0).multi_processor_count
print(f"k_sort2 per-block time by phase (us, averaged over {iters} rollouts and {nblk} blocks):")
for i, nm in enumerate(names):
    us = buf[i] / 100.0 / iters / nblk  # wall_clock64 runs at 100 MHz
    print(f"  {nm:9s} {us:8.2f}  ({100.0 * buf[i] / max(tot, 1):.1f}%)")
print(f"  total     {tot / 100.0 / iters / nblk:8.2f}")
