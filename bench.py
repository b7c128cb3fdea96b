"""Benchmark of the SPAI-via-GFlowNet hot path on MI355X (BASELINE.json metric).

One step = one ``GFlowNet.sample_states`` call over a batch of B candidate preconditioners
of the 1024^2 5-point Poisson matrix (config C4, fp32): ForwardPolicy logits (GATv2 x2 +
mean pool + fc on the state graph, random-init weights), throughput rollout (Gumbel-top-k,
20 % expected removal, ordered trajectory log + forward probabilities), least-squares fill
of M (column SPAI) and the ||A M - I||_F reward, all inputs resident in HBM.
columns/s = (B * N * world) / step time (max over ranks).  Multi-GPU: one process per
GPU, each rank samples its own B candidates (Philox sample ids rank*B..), no collective in
the step (weak scaling).  Prints ONE JSON line on rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2|c3] [--batch B]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (dims, grid, dtype, workload text); candidate pattern = A (2-D) or the 13-wide axial
    # pattern (C3: nnz/col <= 13, utils.axial_pattern_3d)
    "c4": (2, 1024, torch.float32, "C4: 1024^2 5-pt Poisson (1,048,576 x 1,048,576 CSR, fp32), pattern = A"),
    "c2": (2, 256, torch.float32, "C2: 256^2 5-pt Poisson (65,536 x 65,536 CSR, fp32), pattern = A"),
    "c3": (3, 64, torch.float64, "C3: 64^3 7-pt 3-D Laplacian (262,144 x 262,144, fp64), 13-wide axial pattern "
                                 "(nnz/col <= 13)"),
}


def config_matrices(cfg: str):
    """(A, candidate pattern) of a bench config."""
    from gflownet_spai_amd import axial_pattern_3d, poisson_2d, poisson_3d
    dims, grid, dtype, _ = CONFIGS[cfg]
    if dims == 2:
        A = poisson_2d(grid, dtype)
        return A, A
    return poisson_3d(grid, dtype), axial_pattern_3d(grid, 2, dtype)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 TB/s measured copy)


def terminal_logit(logits: np.ndarray, frac: float) -> float:
    """l_E with E[#removed]/E = frac: P(key_a > key_E) = sigmoid(l_a - l_E) (two Gumbels)."""
    l = logits.astype(np.float64)
    lo, hi = -50.0, 50.0
    for _ in range(100):
        mid = 0.5 * (lo + hi)
        f = np.mean(1.0 / (1.0 + np.exp(-(l - mid))))
        lo, hi = (mid, hi) if f > frac else (lo, mid)
    return 0.5 * (lo + hi)


def make_policy(env, A, dev, hid: int = 4):
    """Random-init ForwardPolicy of the reference's architecture (policy.py:24-33:
    node_features=-1, hidden_dim=4 as GFlowNet100.py:178-181), seeded; the terminal row's
    fc bias is then set so the expected removed fraction is 20 %, so the
    sampler's workload matches the configured one.  The policy runs inside every step."""
    from gflownet_spai_amd import ForwardPolicy
    from gflownet_spai_amd.preconditioner import Data

    torch.manual_seed(123)
    E = env.num_actions - 1
    pol = ForwardPolicy(-1, hid, E + 1).to(dev)
    n = env.matrix_size
    data = Data(x=torch.ones(2 * n, 1, device=dev), edge_index=A._indices().to(dev),
                edge_attr=A._values().float().to(dev))
    with torch.no_grad():
        lg, _ = pol.logits(data)
        lg = lg.reshape(-1).double().cpu().numpy()
        pol.fc.bias[E] += terminal_logit(lg[:E], 0.2) - lg[E]
    pol.requires_grad_(False)  # sampling only: no autograd bookkeeping in the step
    return pol


def fill_bytes(env, B, store_m: bool = True) -> float:
    """Algorithmic HBM bytes of one fill + ||AM-I|| launch.

    Gram-cached path (the env's default for widths <= 7): per line the action ids and the
    Gram values (T + Wc, fp32 when the cache round-trips exactly, else fp64), per sample the
    removal bitmap and the stored values of M."""
    n, W = env.pattern.n, env.pattern.width
    s = env.a_lines.val.element_size() if env.fill == "lsq" else 4
    per_sample = math.ceil(env.init_nnz / 32) * 4 + (n * W * s if store_m else 0) + 8
    if getattr(env, "gram", None) is not None:
        line = n * W * 4 + env.gram.numel() * env.gram.element_size() + (n * W * 4 if env.fill == "copy" else 0)
    else:
        sa = env.a_lines.val.element_size()
        line = n * W * (4 + 4 + 4) + n * env.a_lines.width * (4 + sa)
    return line + B * per_sample


def measured_traffic(cfg: str, B: int, overlap: bool):
    """HBM bytes per launch of the roofline kernel from the committed PMC profile of this
    exact workload (profiles/fill_traffic.json, written by scripts/collect_profiles.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `bench.py`), else None."""
    path = os.path.join(ROOT, "profiles", "fill_traffic.json")
    try:
        rec = json.load(open(path))
    except (OSError, ValueError):
        return None
    if rec.get("config") == cfg and rec.get("batch") == B:
        return float(rec["hbm_bytes_per_launch"])
    return None


def cpu_baseline(cfg, B, budget_s: float, logits=None):
    """The oracle (numpy, single thread) on a bounded sample of the same workload (the
    policy's logits are taken as given: the CPU leg times the rollout, fill and residual)."""
    from oracle import spai_oracle as O
    import scipy.sparse as sp

    dims, grid, dtype, _ = CONFIGS[cfg]
    npd = np.float32 if dtype == torch.float32 else np.float64
    r, c, v, n = O.poisson2d(grid, npd) if dims == 2 else O.poisson3d(grid, npd)
    E = len(r)
    if logits is None:
        logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(123)).numpy()
        logits[E] = terminal_logit(logits[:E], 0.2)
    t0 = time.perf_counter()
    removed, actions, fwd, counts = O.throughput_rollout(logits, 1, seed=1234, stream=0)
    t_roll = time.perf_counter() - t0
    idx, act, _ = O.lines_from_coo(r, c, v, n, "col")
    a_idx, _, a_val = O.lines_from_coo(r, c, v.astype(np.float64), n, "col")
    keep = (idx >= 0) & ~removed[0][np.clip(act, 0, None)]
    cols = min(n, 16384)
    done, t_fill = 0, 0.0
    A = sp.csc_matrix((v.astype(np.float64), (r, c)), shape=(n, n))
    while done < n and t_fill < budget_s:
        ids = np.arange(done, min(done + cols, n))
        t0 = time.perf_counter()
        m = O.lsq_fill(idx, keep, a_idx, a_val, ids)
        sub = idx[ids]
        ok = sub >= 0
        Ms = sp.csc_matrix((m[ok], (sub[ok], np.nonzero(ok)[0])), shape=(n, ids.size))
        P = (A @ Ms).tocoo()
        diag = P.data[P.row == ids[P.col]].sum()
        _ = np.sqrt(max((P.data ** 2).sum() - 2 * diag + ids.size, 0.0))
        t_fill += time.perf_counter() - t0
        done = ids[-1] + 1
    per_col = t_fill / done
    t_sample = t_roll + per_col * n  # one candidate over all N columns
    return {"value": n / t_sample, "unit": "columns/s", "cores": 1, "kind": "port",
            "sample": f"oracle/spai_oracle.py (numpy): 1 full rollout over E={E} ({t_roll:.2f}s, the bench policy's "
                      f"logits given) + LSQ fill and ||AM-I|| over the first {done} of {n} columns ({t_fill:.2f}s), "
                      f"extrapolated to N columns; policy forward not included"}


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` run directly: start the N ranks (one process per GPU) under
    torch.distributed.run on 127.0.0.1 as child processes and return their exit status.
    The parent has not initialised the GPU (no HIP call before this point)."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard", default="candidates", choices=["candidates", "columns"],
                    help="candidates: B candidates per rank (weak scaling, no collective); columns: the same B "
                         "candidates on every rank, lines of M split across ranks, one all_reduce of the squared "
                         "residuals and one all_gather of M per step (strong scaling)")
    ap.add_argument("--overlap", action="store_true",
                    help="run the fill/reward on a side stream concurrent with the trajectory sort (measured ~1%% "
                         "slower: the sort's persistent blocks hold nearly all LDS, so the two serialise anyway)")
    ap.add_argument("--no-overlap", action="store_true", help="(default; kept for old command lines)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # one child process per GPU; nothing here touched the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with "
                 f"torch.distributed.run --nproc-per-node {args.gpus} or without WORLD_SIZE")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, kernels, poisson_2d, poisson_3d

    dims, grid, dtype, text = CONFIGS[args.config]
    A, P = config_matrices(args.config)
    n = A.shape[0]
    env = PreconditionerEnv(n, P, A, side="AM", fill="lsq", keep_m=True, device=dev)
    E = env.num_actions - 1
    B = args.batch
    columns = args.shard == "columns"
    shard = None
    if columns and world > 1:
        from gflownet_spai_amd.distributed import allgather_lines, shard_lines
        lb, le = shard_lines(n, rank, world)
        shard = (lb, le, None)
    model = GFlowNet(make_policy(env, P, dev), None, env, mode="throughput", seed=1234,
                     sample_base=0 if columns else rank * B, overlap=args.overlap and not args.no_overlap, line_shard=shard)
    s0 = [P] * B

    def step():
        log = model.sample_states(s0, return_log=True)
        if shard is not None:
            log.m_full = allgather_lines(env.last_m, n)  # M of every candidate on every rank (one all_gather)
        return log

    for _ in range(args.warmup):
        step()

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    kernels.TIMERS = {}
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        log = step()
    barrier()
    dt = (time.perf_counter() - t0) / args.steps
    phases = {k: float(np.mean(kernels.timer_ms(k))) for k in kernels.TIMERS}
    kernels.TIMERS = None
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    res = env.last_residual.double().cpu().numpy()
    counts = log.counts.cpu().numpy()

    if rank == 0:
        fill_ms = phases.get("fill_residual", float("nan"))
        fb = fill_bytes(env, B)
        if shard is not None:  # the rank's fill covers its own lines only (rank 0: the first, largest shard)
            fb *= (shard[1] - shard[0]) / n
        achieved = fb / (fill_ms * 1e-3) / 1e9
        traffic = measured_traffic(args.config, B, args.overlap and not args.no_overlap)
        out = {
            "metric": "SPAI columns/sec + final ||AM-I||_F, 2D Poisson 1024^2, at 1/2/4/8 GPU",
            "value": B * n * (1 if columns else world) / dt,
            "unit": "columns/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if columns else "weak",
            "vs_baseline": None,
            "dtype": "f32 storage, f64 solve/accumulate",
            "data": "synthetic (random-init seeded ForwardPolicy GATv2x2+fc, hid=4, evaluated on the state graph in "
                    "every step; terminal fc bias set for 20% expected removal; Poisson matrix from its stencil)",
            "config": {"workload": text + (f", B={B} candidates, lines of M sharded over the GPUs (all_reduce of "
                                               "||.||^2, all_gather of M)" if columns else
                                               f", B={B} candidates per GPU") +
                                   ": ForwardPolicy logits + throughput rollout + LSQ fill + ||AM-I||_F",
                       "N": n, "E": E, "global_batch": B * (1 if columns else world),
                       "parallelism": f"{'columns' if columns else 'candidates'} sharded x{world}"},
            "final_residual_fro": float(res[0]),
            "final_residual_fro_mean": float(res.mean()),
            "removed_per_candidate_mean": float(counts.mean()),
            "phases_ms": phases,
            "roofline": {"kernel": "k_gram_fill<5,f32,LSQ> (spai_fill_residual_gram: LSQ fill of M + ||AM-I||^2)",
                         "bound": "hbm",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "bytes_per_launch": fb, "avg_launch_ms": fill_ms},
        }
        if not args.no_cpu_baseline and world == 1:
            with torch.no_grad():
                lg_host = model.forward_policy.logits(model.state_to_data(s0[:1])[0])[0].reshape(-1).cpu().numpy()
            out["cpu_baseline"] = cpu_baseline(args.config, B, args.cpu_budget, lg_host)
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
