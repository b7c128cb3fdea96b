"""Diagnostics for the trajectory ordering pipeline at bench scale (GPU box only)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from gflownet_spai_amd import kernels
import bench

E = int(sys.argv[1]) if len(sys.argv) > 1 else 5238784
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
logits[E] = bench.terminal_logit(logits[:E].numpy(), 0.2)
dev = torch.device("cuda", 0)
lg, lmax, z = kernels.logits_stats(logits.to(dev), B)
removed, counts, ws = kernels.rollout_select(lg, B, lmax, 1234, 0)
torch.cuda.synchronize()
t0 = time.time()
actions, fwd, t_dev = kernels.rollout_order(lg, B, lmax, counts, ws)
torch.cuda.synchronize()
print("order s", time.time() - t0, "counts", counts.tolist(), "T", int(t_dev))

# replicate the carve of trajectory.hip to read nbk / bucket_start
def al(x): return (x + 255) // 256 * 256
nblk = (E + 1023) // 1024
off = 0
lay = {}
def take(name, n, sz):
    global off
    lay[name] = (off, n, sz); off = al(off + n * sz)
nb = B * nblk; stage = nb * 1024; cap = B * E
for name, n, sz in [("block_counts", nb, 4), ("block_min", nb, 4), ("block_max", nb, 4), ("block_wrest", nb, 8),
                    ("wrest", B, 8), ("klo", B, 8), ("kscale", B, 8), ("nbk", B, 4), ("seg", B, 4), ("tdev", 1, 4),
                    ("st_ord", stage, 4), ("st_act", stage, 4), ("part_hist", B * 64 * 16384, 4),
                    ("bucket_start", B * 16385, 4)]:
    take(name, n, sz)
def get(name, dt):
    o, n, sz = lay[name]
    return ws[o:o + n * sz].view(dt).cpu().numpy()
nbk = get("nbk", torch.int32); bs = get("bucket_start", torch.int32).reshape(B, 16385)
lo = get("klo", torch.float64); hi = get("kscale", torch.float64)
for b in range(B):
    sz = np.diff(bs[b, :nbk[b] + 1])
    print(b, "nbk", nbk[b], "klo", lo[b], "kscale", hi[b], "bucket max", sz.max(), "mean", sz.mean(), ">2048:", (sz > 2048).sum())
if len(sys.argv) > 3:
    from oracle import spai_oracle as O
    r_o, a_o, f_o, c_o = O.throughput_rollout(logits.numpy(), 1, 1234, 0)
    T = int(t_dev)
    print("sample0 match:", np.array_equal(actions[0, :c_o[0] + 1].cpu().numpy(), a_o[:, 0][:c_o[0] + 1]),
          "fwd maxrel", float(np.max(np.abs(fwd[0, :c_o[0] + 1].cpu().numpy() - f_o[0, :c_o[0] + 1]) / f_o[0, :c_o[0] + 1])))
