"""Timing of one training epoch (GFlowNet100.py:278-321) on one MI355X, by phase:
sample_states | back_probs (LSTM forward) | loss | backward (logp_grad, LSTM BPTT, policy)
| Adam.  usage: python scripts/train_bench.py [--config c2|c4] [--batch B] [--steps K]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gflownet_spai_amd import BackwardPolicy, GFlowNet, PreconditionerEnv, kernels, poisson_2d, poisson_3d  # noqa: E402
from gflownet_spai_amd.utils import trajectory_balance_loss  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    dims, grid, dtype, text = bench.CONFIGS[args.config]
    A = poisson_2d(grid, dtype) if dims == 2 else poisson_3d(grid, dtype)
    n = A.shape[0]
    env = PreconditionerEnv(n, A, A, side="AM", fill="lsq", device=dev)
    E = env.num_actions - 1
    fwd = bench.make_policy(env, A, dev)
    fwd.requires_grad_(True)
    torch.manual_seed(0)
    bwd = BackwardPolicy(1, 4, E + 1).to(dev)
    model = GFlowNet(fwd, bwd, env, mode="throughput", seed=1234)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    s0 = [A] * args.batch
    rec = []
    for it in range(args.steps + 1):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev[0].record()
        log = model.sample_states(s0, return_log=True)
        fp = log.fwd_probs
        ev[1].record()
        bp = log.back_probs
        ev[2].record()
        loss = trajectory_balance_loss(log.total_flow, log.rewards.clamp(min=1.0), fp, bp)
        ev[3].record()
        loss.backward()
        ev[4].record()
        opt.step()
        opt.zero_grad()
        ev[5].record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if it == 0:
            continue  # warm-up
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(5)]
        rec.append({"wall_ms": wall * 1e3, "sample_ms": ms[0], "back_probs_ms": ms[1], "loss_ms": ms[2],
                    "backward_ms": ms[3], "adam_ms": ms[4], "T": int(log.fwd_probs.shape[1]),
                    "loss": float(loss)})
    out = {"config": text, "B": args.batch, "E": E, "steps": rec,
           "lstm_ns_per_step": 1e6 * rec[-1]["back_probs_ms"] / rec[-1]["T"]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
