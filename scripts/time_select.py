"""Event timing of spai_rollout_select alone at C4 (B=8, bench logits)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gflownet_spai_amd import kernels  # noqa: E402

E, B = 5238784, 8
logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
logits[E] = bench.terminal_logit(logits[:E].numpy(), 0.2)
lg, lmax, z = kernels.logits_stats(logits.cuda(), B)
ts = []
for it in range(12):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    kernels.rollout_select(lg, B, lmax, 1234, it)
    e1.record()
    torch.cuda.synchronize()
    if it >= 2:
        ts.append(e0.elapsed_time(e1))
print(f"dbg={os.environ.get('SPAI_DBG', '0')} select {sum(ts) / len(ts) * 1e3:.1f} us")
