"""k_tile time (library kernel timer) over repeated spai_rollout_select calls at C4, B=8, for
timing-ablation builds (build/variants/<name>.so via SPAI_LIB_VARIANT; their samples are wrong):
  python scripts/tile_ablate.py [name]"""
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
for it in range(3):
    kernels.rollout_select(lg, B, lmax, 1234, it)
torch.cuda.synchronize()
kernels.kernel_timer_arm(True, ["k_tile"])
for it in range(30):
    kernels.rollout_select(lg, B, lmax, 1234, it)
torch.cuda.synchronize()
kernels.kernel_timer_arm(False, ["k_tile"])
cnt, ms = kernels.kernel_timer_read(["k_tile"])["k_tile"]
print(f"{sys.argv[1] if len(sys.argv) > 1 else 'tree'}: k_tile {ms * 1e3:.1f} us ({cnt} launches)", flush=True)
