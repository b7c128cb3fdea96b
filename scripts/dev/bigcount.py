"""How many buckets exceed k_sort2's LDS capacity (the oversized slow path) over 20 C4 rollouts."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import bench
from gflownet_spai_amd import kernels, _lib
E, B = 5238784, 8
logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
logits[E] = bench.terminal_logit(logits[:E].numpy(), 0.2)
lg, lmax, z = kernels.logits_stats(logits.cuda(), B)
lib = _lib.load()
tot = 0
for it in range(int(os.environ.get("ROLL", 20))):
    removed, counts, ws = kernels.rollout_select(lg, B, lmax, 1234, it)
    kernels.rollout_order(lg, B, lmax, counts, ws)
    off = lib.spai_rollout_ws_offset(E, B, 0)
    tot += int(ws[off:off + 4].view(torch.int32).item())
print(os.environ.get("SPAI_LIB_VARIANT", "tree"), "oversized buckets rollouts:", os.environ.get("ROLL", 20), tot)
