"""Isolated timing of spai_residual_lines (the generic ||A M_b - I||_F^2) at C4 / C3.

M_b = the candidate pattern (A's own lines) with an independent 25 % of the slots removed per
sample and random values (the GFlowNet candidates' structure); --distinct gives every sample
random indices instead (the per-sample path).  Prints ms per launch and the fraction of the HBM
roofline at bytes(A) + B x bytes(M_b).
--wide (C3): M on the 13-wide axial candidate pattern of the bench's C3 config with fp64 values
(k_resid_row16), instead of A's own 7-wide pattern.
usage: python scripts/resid_bench.py [--config c4] [--batch 8] [--iters 20] [--distinct] [--wide]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gflownet_spai_amd import PreconditionerEnv, axial_pattern_3d, kernels, poisson_2d, poisson_3d  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--distinct", action="store_true")
    ap.add_argument("--wide", action="store_true")
    ap.add_argument("--dry", action="store_true", help="print the inputs, launch nothing")
    ap.add_argument("--mf64", action="store_true", help="fp64 M values on A's own pattern")
    ap.add_argument("--pad", action="store_true", help="idx / M as views of larger buffers (overrun probe)")
    ap.add_argument("--inexact", action="store_true", help="A values perturbed off fp32 (fp64-A kernels)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    dims, grid, dtype, _ = bench.CONFIGS[args.config]
    A = poisson_2d(grid, dtype) if dims == 2 else poisson_3d(grid, dtype)
    if args.inexact:
        A = A.coalesce()
        A = torch.sparse_coo_tensor(A.indices(), A.values() * (1 + 2.0 ** -40 * torch.arange(A._nnz()) % 7), A.shape)
    n = A.shape[0]
    env = PreconditionerEnv(n, A, A, side="AM", fill="copy", device=dev)
    a = env.a_lines
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(0)
    pat = a.idx
    mdt = torch.float64 if args.mf64 else torch.float32
    if args.wide:  # the C3 candidate pattern (13-wide), fp64 M
        env = PreconditionerEnv(n, axial_pattern_3d(grid, 2), A, side="AM", fill="copy", device=dev)
        pat, mdt = env.pattern.idx, torch.float64
    W = pat.shape[1]
    if args.distinct:
        idx = torch.randint(0, n, (B, n, W), generator=g, device=dev, dtype=torch.int32)
        idx = torch.sort(idx, dim=2).values
        dup = torch.zeros_like(idx, dtype=torch.bool)
        dup[:, :, 1:] = idx[:, :, 1:] == idx[:, :, :-1]
        idx[dup] = -1
    else:
        idx = pat.unsqueeze(0).repeat(B, 1, 1)
    idx[torch.rand(idx.shape, generator=g, device=dev) < 0.25] = -1
    idx = idx.contiguous()
    m = torch.randn((B, n, W), generator=g, device=dev, dtype=mdt)
    if args.pad:
        bi = torch.full((B * n * W + 65536,), -1, dtype=idx.dtype, device=dev)
        bi[: B * n * W] = idx.reshape(-1)
        bm = torch.zeros(B * n * W + 65536, dtype=m.dtype, device=dev)
        bm[: B * n * W] = m.reshape(-1)
        idx, m = bi[: B * n * W].view(B, n, W), bm[: B * n * W].view(B, n, W)
    if args.dry:
        av = kernels.narrow_values(a)
        print(json.dumps({"idx": [list(idx.shape), list(idx.stride()), str(idx.dtype), int(idx.min()), int(idx.max()),
                                  idx.data_ptr() % 256],
                          "m": [list(m.shape), list(m.stride()), str(m.dtype), m.data_ptr() % 256],
                          "a_idx": [list(a.idx.shape), list(a.idx.stride()), int(a.idx.min()), int(a.idx.max()),
                                    a.idx.data_ptr() % 256],
                          "a_val": [list(av.shape), list(av.stride()), str(av.dtype), av.data_ptr() % 256],
                          "n": n, "W": W, "B": B, "a_width": a.width}))
        return
    kernels.residual_lines(idx, m, a)
    kernels.TIMERS = {}
    for _ in range(args.iters):
        kernels.residual_lines(idx, m, a)
    torch.cuda.synchronize()
    ms = sum(kernels.timer_ms("residual_lines")) / args.iters
    av = kernels.narrow_values(a)
    nbytes = a.idx.numel() * 4 + av.numel() * av.element_size() + B * n * W * (4 + m.element_size())
    print(json.dumps({"config": args.config, "B": B, "W": W, "distinct": args.distinct, "ms": ms, "bytes": nbytes,
                      "frac": nbytes / (ms * 1e-3) / 8e12}))


if __name__ == "__main__":
    main()
