"""Trajectory-sort diagnostics on one GPU: per rollout of a bench config, the bucket sizes the
select phase produced (largest, number above k_sort2's LDS capacity), the oversized-bucket count
the sort met (workspace field 0) and the sort's HIP-event time.  Finds what sets k_sort2's worst
case (the C5 stand-in's 935 us launches).

  python scripts/sort_diag.py [--config c5s] [--rollouts 40] [--batch 8]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KCAP2 = 8192  # trajectory.hip kCap2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5s")
    ap.add_argument("--rollouts", type=int, default=40)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import bench
    from gflownet_spai_amd import PreconditionerEnv, kernels

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    A, P = bench.config_matrices(args.config)
    env = PreconditionerEnv(A.shape[0], P, A, side="AM", fill="copy", device=dev)
    pol = bench.make_policy(env, P, dev)
    from gflownet_spai_amd.preconditioner import Data
    n = env.matrix_size
    data = Data(x=torch.ones(2 * n, 1, device=dev), edge_index=P._indices().to(dev), edge_attr=P._values().float().to(dev))
    with torch.no_grad():
        lg, _ = pol.logits(data)
    lg = lg.reshape(-1).contiguous().float()
    B = args.batch
    E = lg.numel() - 1
    lg, lmax, _ = kernels.logits_stats(lg, B)
    lib = kernels._l()
    o_big, o_bs, o_nb = (lib.spai_rollout_ws_offset(E, B, f) for f in (0, 4, 5))
    kmax = lib.spai_rollout_ws_offset(E, B, 3)
    recs = []
    for i in range(args.rollouts):
        removed, counts, ws = kernels.rollout_select(lg, B, lmax, 1234, i)
        bs = ws[o_bs:o_bs + B * (kmax + 1) * 4].view(torch.int32).view(B, kmax + 1).cpu().numpy()
        nb = ws[o_nb:o_nb + B * 4].view(torch.int32).cpu().numpy()
        sizes = np.concatenate([np.diff(bs[b, :nb[b] + 1]) for b in range(B)])
        kk = [int(np.argmax(np.diff(bs[b, :nb[b] + 1]))) for b in range(B)]
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        actions, fwd = kernels.rollout_sort(lg, B, lmax, ws, 0, 1)
        e.record()
        kernels.rollout_finish(lg, B, lmax, counts, ws, actions, fwd, 0, 1)
        torch.cuda.synchronize()
        big = int(ws[o_big:o_big + 4].view(torch.int32).item())
        rec = {"rollout": i, "sort_ms": s.elapsed_time(e), "buckets": int(sizes.size), "mean": float(sizes.mean()),
               "max": int(sizes.max()), "over_cap": int((sizes > KCAP2).sum()), "oversized_met": big,
               "argmax_bucket_per_sample": kk, "nb": nb.tolist(), "counts": counts.cpu().tolist()}
        recs.append(rec)
        print(json.dumps({k: rec[k] for k in ("rollout", "sort_ms", "buckets", "mean", "max", "over_cap",
                                              "oversized_met", "argmax_bucket_per_sample")}), flush=True)
    t = np.array([r["sort_ms"] for r in recs])
    summ = {"config": args.config, "B": B, "E": E, "rollouts": len(recs), "sort_ms_mean": float(t.mean()),
            "sort_ms_max": float(t.max()), "rollouts_with_oversized": int(sum(r["over_cap"] > 0 for r in recs)),
            "max_bucket": int(max(r["max"] for r in recs)),
            "sort_ms_mean_without_oversized": float(np.mean([r["sort_ms"] for r in recs if r["over_cap"] == 0] or [0])),
            "sort_ms_mean_with_oversized": float(np.mean([r["sort_ms"] for r in recs if r["over_cap"] > 0] or [0]))}
    print(json.dumps(summ))
    if args.out:
        json.dump({"summary": summ, "rollouts": recs}, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
