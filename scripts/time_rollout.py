"""Event timing of rollout_select / rollout_order at C4 (B=8, bench logits).

Reports the median (and min) over ITERS rollouts; A/B comparisons of library builds
(SPAI_LIB_VARIANT) should run in the same gpurun call, alternating."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gflownet_spai_amd import kernels  # noqa: E402

E, B, iters = 5238784, int(os.environ.get("B", 8)), int(os.environ.get("ITERS", 30))
logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
logits[E] = bench.terminal_logit(logits[:E].numpy(), 0.2)
lg, lmax, z = kernels.logits_stats(logits.cuda(), B)
ts, to = [], []
for it in range(iters + 3):
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    removed, counts, ws = kernels.rollout_select(lg, B, lmax, 1234, it)
    e1.record()
    kernels.rollout_order(lg, B, lmax, counts, ws)
    e2.record()
    torch.cuda.synchronize()
    if it >= 3:
        ts.append(e0.elapsed_time(e1) * 1e3)
        to.append(e1.elapsed_time(e2) * 1e3)
print(f"{os.environ.get('SPAI_LIB_VARIANT', 'default'):>22s}: select {statistics.median(ts):6.1f} us (min {min(ts):6.1f})"
      f"  order {statistics.median(to):6.1f} us (min {min(to):6.1f})  winners/sample {counts.float().mean().item():.0f}")
