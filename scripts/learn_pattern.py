"""Train the GFlowNet on one MI355X with the reference driver's loop and compare the learned
SPAI pattern with power-pattern SPAI by GMRES (GFlowNet100.py:278-321 epoch loop, :61-93
solve_with_gmres).

Reference hyper-parameters (GFlowNet100.py:32-34, 178-181, 266-267): ForwardPolicy(-1, 4, E+1)
and BackwardPolicy(1, 4, E+1) at their seeded random init, Adam lr 5e-4 over both,
ReduceLROnPlateau(factor 0.2, patience 10) stepped with the loss, batch 2, initial states =
clones of A.  Sampler: throughput mode (Philox exponential race, one pass per rollout), LSQ fill
of M on the kept pattern, reward on ||A M - I||_F (side AM) with the reference formula.

Per epoch the record holds loss, rewards, removed counts, residuals, mean sigmoid(alpha), lr
and the wall time.  After training, B_eval candidates are drawn from the trained and from the
untrained policy; the best of each (highest reward) is evaluated by GMRES (restart 20, rtol
1e-5, as the reference) beside M = none and the power-pattern SPAI of A and A^2.

usage: python scripts/learn_pattern.py [--matrix poisson|thermal] [--grid 256] [--epochs 1000]
                                       [--budget-s 240] [--out gpurun_out/learn.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gflownet_spai_amd import (BackwardPolicy, ForwardPolicy, GFlowNet, PreconditionerEnv, poisson_2d,  # noqa: E402
                               thermal_like)
from gflownet_spai_amd.gmres import DeviceOperator, solve_with_gmres, spai_power_pattern  # noqa: E402
from gflownet_spai_amd.train import train_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--matrix", default="poisson", choices=["poisson", "thermal"])
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=1000)
    ap.add_argument("--budget-s", type=float, default=240.0, help="stop training after this many seconds")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--lr", type=float, default=5e-4)
    ap.add_argument("--no-plateau", action="store_true", help="constant lr (no ReduceLROnPlateau)")
    ap.add_argument("--eval-batch", type=int, default=8)
    ap.add_argument("--maxiter", type=int, default=10260)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if args.matrix == "poisson":
        A64 = poisson_2d(args.grid, torch.float64).coalesce()
        name = f"{args.grid}^2 5-pt Poisson"
    else:
        A64 = thermal_like(args.grid).coalesce()
        name = f"thermal2-like synthetic (utils.thermal_like({args.grid}))"
    A32 = torch.sparse_coo_tensor(A64.indices(), A64.values().float(), A64.shape).coalesce()
    n = A64.shape[0]
    Acsr = sp.csr_matrix((A64.values().numpy(), tuple(A64.indices().numpy())), shape=(n, n))
    env = PreconditionerEnv(n, A32, A64, side="AM", fill="lsq", keep_m=True, device=dev)
    E = env.num_actions - 1

    torch.manual_seed(0)  # the policies' random init (seeded, as the reference's notebook runs)
    fwd = ForwardPolicy(-1, 4, E + 1).to(dev)
    bwd = BackwardPolicy(1, 4, E + 1).to(dev)
    model = GFlowNet(fwd, bwd, env, mode="throughput", seed=2024)
    init_state = {k: v.detach().clone() for k, v in fwd.state_dict().items()}
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    sched = None if args.no_plateau else torch.optim.lr_scheduler.ReduceLROnPlateau(opt, factor=0.2, patience=10)
    s0 = [A32] * args.batch
    hist = []
    t_start = time.perf_counter()
    for ep in range(args.epochs):
        t0 = time.perf_counter()
        res = train_step(model, opt, s0, sched)
        log = res.log
        rw = log.rewards_all.double().cpu().numpy() if getattr(log, "rewards_all", None) is not None else \
            log.rewards.double().cpu().numpy()
        rec = {"epoch": ep, "loss": float(res.loss), "updated": bool(res.updated),
               "reward_mean": float(rw.mean()), "reward_max": float(rw.max()),
               "removed_mean": float(log.counts.double().mean()), "removed_frac": float(log.counts.double().mean()) / E,
               "residual_mean": float(env.last_residual.double().mean()),
               "alpha": float(torch.sigmoid(fwd.alpha.detach())), "lr": opt.param_groups[0]["lr"],
               "seconds": time.perf_counter() - t0}
        hist.append(rec)
        if ep % 25 == 0:
            print(json.dumps(rec), flush=True)
        if time.perf_counter() - t_start > args.budget_s:
            break
    train_s = time.perf_counter() - t_start

    b = np.random.default_rng(0).standard_normal(n)
    Aop = DeviceOperator(Acsr, device=dev)
    out = {"matrix": f"{name} (n={n}, nnz={Acsr.nnz}), candidate pattern = A, LSQ fill, reward on ||AM-I||_F",
           "driver": f"GFlowNet100.py:278-321 loop: batch {args.batch}, Adam lr {args.lr}, "
                     f"{'constant lr' if args.no_plateau else 'ReduceLROnPlateau(0.2, 10)'}, "
                     f"ForwardPolicy(-1, 4, E+1) + BackwardPolicy(1, 4, E+1) seeded random init, throughput sampler",
           "E": E, "r0": env._r0, "epochs_run": len(hist), "train_seconds": train_s,
           "history": hist, "gmres": f"restart 20, rtol 1e-5, maxiter {args.maxiter}, b ~ N(0,1) seed 0", "runs": {}}

    def run(label, M, extra=None):
        x, _, it, el = solve_with_gmres(Aop, b, M, verbose=False, maxiter=args.maxiter)
        rel = float(np.linalg.norm(b - Acsr @ x) / np.linalg.norm(b))
        r = {"iterations": it, "seconds": el, "true_rel_residual": rel}
        if M is not None:
            r["nnz_M"] = int((M.coalesce().values() != 0).sum())
        r.update(extra or {})
        out["runs"][label] = r
        print(label, json.dumps(r), flush=True)

    def best_sample(label):
        with torch.no_grad():
            log = model.sample_states([A32] * args.eval_batch, return_log=True)
        rw = log.rewards_all.double()
        k = int(torch.argmax(rw))
        M = env.assemble(k).coalesce()
        run(label, M, {"reward": float(rw[k]), "residual_AM_fro": float(env.last_residual[k]),
                       "removed": int(log.counts[k]), "rewards_all": [float(v) for v in rw.cpu()]})

    run("warmup", None)
    out["runs"].pop("warmup")
    run("none", None)
    for p in ((1, 2) if args.matrix == "poisson" else (1,)):  # thermal: A^2 is 19 wide (fill kernels <= 13)
        M = spai_power_pattern(A64, p, device=dev).coalesce()
        res = env.calculate_residual(M, env.original_matrix)
        run(f"SPAI pattern(A^{p}) LSQ", M, {"residual_AM_fro": float(res)})
    best_sample("GFlowNet trained: best of eval batch")
    fwd.load_state_dict(init_state)
    best_sample("GFlowNet untrained (seeded init): best of eval batch")
    line = json.dumps(out)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            f.write(line + "\n")
    print(json.dumps({k: v for k, v in out.items() if k != "history"}))


if __name__ == "__main__":
    main()
