"""Debug view of the sample-sort workspace after spai_rollout_select (C4 bench logits)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gflownet_spai_amd import kernels  # noqa: E402

kTile, kMaxB, kSampM, kSampNT = 16384, 2048, 65536, 256


def carve(E, B):
    off = 0
    out = {}

    def take(name, n, sz):
        nonlocal off
        out[name] = (off, n, sz)
        off = (off + n * sz + 255) // 256 * 256
    ntiles = (E + kTile - 1) // kTile
    M = 1
    while M * 2 <= E and M * 2 <= kSampM:
        M *= 2
    nsb = (M + kSampNT - 1) // kSampNT
    take("ctl", B * kMaxB + B + 1, 4)
    take("samp_cnt", B * nsb, 4)
    take("samp", B * M, 4)
    take("nb", B, 4)
    take("spl", B * kMaxB, 4)
    take("staging", B * ntiles * kTile, 8)
    take("tcount", B * kMaxB * ntiles, 4)
    take("tloc", B * kMaxB * ntiles, 4)
    take("tile_wrest", B * ntiles, 8)
    take("bstart", B * (kMaxB + 1), 4)
    return out, ntiles, M, nsb


def view(ws, lay, name, dtype):
    o, n, sz = lay[name]
    return ws[o:o + n * sz].view(dtype)


E = 5238784
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
logits[E] = bench.terminal_logit(logits[:E].numpy(), 0.2)
lg, lmax, z = kernels.logits_stats(logits.cuda(), B)
removed, counts, ws = kernels.rollout_select(lg, B, lmax, 1234, 0)
torch.cuda.synchronize()
lay, ntiles, M, nsb = carve(E, B)
nb = view(ws, lay, "nb", torch.int32).cpu().numpy()
bstart = view(ws, lay, "bstart", torch.int32).view(B, kMaxB + 1).cpu().numpy()
scnt = view(ws, lay, "samp_cnt", torch.int32).view(B, nsb).cpu().numpy()
spl = view(ws, lay, "spl", torch.int32).view(B, kMaxB).cpu().numpy().view(np.uint32)
print("counts", counts.cpu().numpy(), "M", M, "nsb", nsb, "ntiles", ntiles)
for b in range(min(B, 3)):
    sizes = np.diff(bstart[b, :nb[b] + 1])
    print(f"b={b} nb={nb[b]} sampled winners={scnt[b].sum()} sizes: min {sizes.min()} mean {sizes.mean():.0f} "
          f"max {sizes.max()} >8192: {(sizes > 8192).sum()} sorted_spl={bool(np.all(np.diff(spl[b, :nb[b]-1].astype(np.int64)) >= 0))}")
    print("  first sizes", sizes[:12], "last", sizes[-6:])
    print("  spl head", spl[b, :6], "tail", spl[b, max(0, nb[b] - 7):nb[b] - 1])
