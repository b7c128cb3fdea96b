"""Preconditioner quality by GMRES (GFlowNet100.py:61-93, 126-132) on one
MI355X: iterations and time of solve_with_gmres(A, b, M) for M = none, the driver's spilu
baseline (host LinearOperator), the power-pattern SPAI baselines (pattern of A, A^2; LSQ fill
on the GPU) and GFlowNet-sampled SPAI patterns (throughput rollout of the bench policy, LSQ
fill), plus the spai_ell_spmv roofline (HIP events over repeated products).
usage: python scripts/gmres_eval.py [--matrix poisson|thermal] [--grid 256] [--maxiter 10260] [--no-spilu]
                                    [--out gpurun_out/gmres.json]
(--matrix thermal --grid 1108: the C5 stand-in, utils.thermal_like, 1.23 M unknowns, fp64)"""
import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gflownet_spai_amd import BackwardPolicy, GFlowNet, PreconditionerEnv, poisson_2d, thermal_like  # noqa: E402
from gflownet_spai_amd.gmres import DeviceOperator, solve_with_gmres, spai_power_pattern  # noqa: E402


def spmv_roofline(op: DeviceOperator, reps=200):
    n, W = op.n, op.lines.width
    x = torch.randn(n, dtype=torch.float64, device=op.device)
    y = torch.empty_like(x)
    for _ in range(5):
        op.matvec_into(x, y)
    s = torch.cuda.current_stream(op.device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        op.matvec_into(x, y)
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    vb = op.lines.val.element_size()
    algo = n * W * (4 + vb) + 8 * n + 8 * n  # lines + y + x once
    return {"n": n, "W": W, "avg_us": us, "algorithmic_bytes": algo, "GB_s": algo / us / 1e3,
            "frac_of_8TBs": algo / us / 1e3 / 8000.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--matrix", default="poisson", choices=["poisson", "thermal"])
    ap.add_argument("--maxiter", type=int, default=10260)
    ap.add_argument("--no-spilu", action="store_true")
    ap.add_argument("--powers", default="1,2")
    ap.add_argument("--samples", type=int, default=2)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.matrix == "poisson":
        A32 = poisson_2d(args.grid, torch.float32)
        A64 = poisson_2d(args.grid, torch.float64).coalesce()
    else:
        A64 = thermal_like(args.grid).coalesce()
        A32 = torch.sparse_coo_tensor(A64.indices(), A64.values().float(), A64.shape)
    n = A64.shape[0]
    Acsr = sp.csr_matrix((A64.values().numpy(), tuple(A64.indices().numpy())), shape=(n, n))
    b = np.random.default_rng(0).standard_normal(n)
    Aop = DeviceOperator(Acsr, device=dev)
    out = {"matrix": (f"{args.grid}^2 5-pt Poisson" if args.matrix == "poisson" else
                      f"thermal2-like synthetic (utils.thermal_like({args.grid}))") + f" (n={n}, nnz={Acsr.nnz}), fp64",
           "b": "N(0,1), seed 0",
           "gmres": f"restart 20, rtol 1e-5, maxiter {args.maxiter} (GFlowNet100.py:81 uses 10260)", "runs": {}}

    def run(name, M, nnz=None):
        solve_with_gmres(Aop, b, M, verbose=False, maxiter=2) if name == "warmup" else None
        x, res, it, el = solve_with_gmres(Aop, b, M, verbose=False, maxiter=args.maxiter)
        rel = float(np.linalg.norm(b - Acsr @ x) / np.linalg.norm(b))
        out["runs"][name] = {"iterations": it, "seconds": el, "true_rel_residual": rel, "nnz_M": nnz}
        print(name, out["runs"][name], flush=True)

    run("warmup", None)
    out["runs"].pop("warmup")
    run("none", None)
    if not args.no_spilu:
        t0 = time.perf_counter()
        ilu = spla.spilu(Acsr.tocsc())
        out["spilu_seconds"] = time.perf_counter() - t0
        run("spilu (host LinearOperator, GFlowNet100.py:126-132)", spla.LinearOperator(Acsr.shape, ilu.solve),
            int(ilu.L.nnz + ilu.U.nnz))
    for p in (int(x) for x in args.powers.split(",")):
        M = spai_power_pattern(A64, p, device=dev).coalesce()
        run(f"SPAI pattern(A^{p}) LSQ", M, int(M._nnz()))
        if p == 1:
            out["spmv_A"] = spmv_roofline(Aop)
            out["spmv_M"] = spmv_roofline(DeviceOperator(M, device=dev))
    # GFlowNet-sampled patterns of A (bench policy: ~20% of the entries removed), LSQ fill
    env = PreconditionerEnv(n, A32, A64, side="AM", fill="lsq", keep_m=True, device=dev)
    fwd = bench.make_policy(env, A32, dev)
    torch.manual_seed(0)
    bwd = BackwardPolicy(1, 4, env.num_actions).to(dev)
    g = GFlowNet(fwd, bwd, env, mode="throughput", seed=1234)
    with torch.no_grad():
        log = g.sample_states([A32] * args.samples, return_log=True)
    for s in range(args.samples):
        M = env.assemble(s).coalesce()
        run(f"GFlowNet sample {s} LSQ", M, int((M.values() != 0).sum()))
    line = json.dumps(out)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    print(line)


if __name__ == "__main__":
    main()
