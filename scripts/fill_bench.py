"""Isolated timing of spai_fill_residual (LSQ / COPY) at C4 for several batch sizes.
--path line times the fill that forms each line's Gram from A in the launch (fill.hip k_line,
spai_fill_residual) instead of reading the env's Gram cache (gram.hip, the bench's path).

Working sets at B >= 16 exceed the 256 MiB Infinity Cache, so the GB/s figure there is an
HBM figure.  usage: python scripts/fill_bench.py [--config c4] [--batches 8,32] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gflownet_spai_amd import PreconditionerEnv, kernels, poisson_2d, poisson_3d  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--batches", default="8,32")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--path", default="gram", choices=["gram", "line"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    dims, grid, dtype, _ = bench.CONFIGS[args.config]
    A = poisson_2d(grid, dtype) if dims == 2 else poisson_3d(grid, dtype)
    n = A.shape[0]
    out = []
    for fill in ("lsq", "copy"):
        env = PreconditionerEnv(n, A, A, side="AM", fill=fill, keep_m=True, device=dev)
        E = env.num_actions - 1
        logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123))
        logits[E] = bench.terminal_logit(logits[:E].numpy(), 0.2)
        lg = logits.to(dev)
        for B in [int(x) for x in args.batches.split(",")]:
            lgs, lmax, _ = kernels.logits_stats(lg, B)
            removed, counts, _ = kernels.rollout_select(lgs, B, lmax, 7, 0)
            def run():
                if args.path == "line":
                    return kernels.fill_residual(env.pattern, env.a_lines, removed, fill == "lsq",
                                                 store_m=os.environ.get("NO_STORE") is None,
                                                 m_dtype=env.a_lines.val.dtype)
                return kernels.fill_residual_gram(env.pattern, env.gram, removed, fill == "lsq",
                                                  store_m=os.environ.get("NO_STORE") is None,
                                                  m_dtype=env.a_lines.val.dtype)
            for _ in range(2):
                run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.iters):
                run()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / args.iters
            fb = bench.fill_bytes(env, B, store_m=os.environ.get("NO_STORE") is None)
            rec = {"path": args.path, "fill": fill, "B": B, "ms": ms, "bytes": fb, "GBps": fb / ms / 1e6,
                   "frac": fb / ms / 1e6 / bench.HBM_PEAK_GBS, "columns_per_s": B * n / ms * 1e3}
            out.append(rec)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
