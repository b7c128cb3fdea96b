"""Isolated timing of the cached QR fill (k_qr_solve, spai_fill_lines_qr_cached) on one GPU: M stored
or not (the store stream's share of the kernel), batch sizes, the R cache in full or as its
dictionary.  Kernel time from the library's per-launch HIP events (spai_kernel_timer_*).

  python scripts/qr_fill_bench.py [--config c4] [--batches 8,16] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gflownet_spai_amd import PreconditionerEnv, kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--batches", default="8,16")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    A, P = bench.config_matrices(args.config)
    n = A.shape[0]
    for dic in (True, False):
        env = PreconditionerEnv(n, P, A, side="AM", fill="qr", keep_m=True, device=dev, cache_dict=dic)
        E = env.num_actions - 1
        logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
        logits[E] = bench.terminal_logit(logits[:E].numpy(), 0.2)
        for B in [int(x) for x in args.batches.split(",")]:
            lgs, lmax, _ = kernels.logits_stats(logits.to(dev), B)
            removed, counts, _ = kernels.rollout_select(lgs, B, lmax, 7, 0)
            for store in (True, False):
                def run():
                    return kernels.fill_residual_qr(env.pattern, env.a_lines, env.qr_rows, removed, store_m=store,
                                                    m_dtype=env.a_lines.val.dtype, rcache=env.rcache)
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                kernels.kernel_timer_arm(True, ["k_qr_solve"])
                for _ in range(args.iters):
                    run()
                torch.cuda.synchronize()
                kernels.kernel_timer_arm(False, ["k_qr_solve"])
                cnt, ms = kernels.kernel_timer_read(["k_qr_solve"])["k_qr_solve"]
                rec = {"config": args.config, "dict": dic, "B": B, "store_m": store, "kernel_ms": ms, "launches": cnt,
                       "m_bytes": B * n * env.pattern.width * env.a_lines.val.element_size() if store else 0}
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
