"""A/B timing of the throughput rollout phases at C4 (B=8, bench-like logits): HIP-event
averages of spai_rollout_select and spai_rollout_order over 10 rollouts after 2 warm-ups.
Run once per library build (SPAI_LIB_VARIANT=libspai_x.so picks build/variants/libspai_x.so),
under `rocprofv3 --kernel-trace --stats` for the per-kernel split."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gflownet_spai_amd import kernels  # noqa: E402

E, B = int(os.environ.get("E", 5238784)), int(os.environ.get("B", 8))
logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
logits[E] = bench.terminal_logit(logits[:E].numpy(), float(os.environ.get("FRAC", 0.2)))
lg, lmax, z = kernels.logits_stats(logits.cuda(), B)
sel, order, cnt = [], [], []
for it in range(12):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    removed, counts, ws = kernels.rollout_select(lg, B, lmax, 1234, it)
    ev[1].record()
    kernels.rollout_order(lg, B, lmax, counts, ws)
    ev[2].record()
    torch.cuda.synchronize()
    if it >= 2:
        sel.append(ev[0].elapsed_time(ev[1]))
        order.append(ev[1].elapsed_time(ev[2]))
        cnt.append(float(counts.double().mean()))
print(json.dumps({"variant": os.environ.get("SPAI_LIB_VARIANT", "tree"), "select_us": 1e3 * sum(sel) / len(sel),
                  "order_us": 1e3 * sum(order) / len(order), "winners_mean": sum(cnt) / len(cnt)}))
