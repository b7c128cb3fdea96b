"""Benchmark of the SPAI-via-GFlowNet hot path on MI355X (BASELINE.json metric).

One step = one ``GFlowNet.sample_states`` call over a batch of B candidate preconditioners
of the 1024^2 5-point Poisson matrix (config C4, fp32): ForwardPolicy logits (GATv2 x2 +
mean pool + fc on the state graph, random-init weights), throughput rollout (Gumbel-top-k,
20 % expected removal, ordered trajectory log + forward probabilities), least-squares fill
of M (column SPAI; Householder QR: every line's full block A[I, slots] factored once per env
into an R cache, the masked re-triangularisation per step) and the ||A M - I||_F reward, all
inputs resident in HBM.

Multi-GPU (one process per GPU; `--gpus N` starts the N ranks itself, or run it under
torch.distributed.run), DESIGN.md §6:
  --shard columns (default; the north star's column split, weak scaling): every GPU rolls out
      --batch candidates (global sample ids rank*batch ..: the same Philox draws as one GPU with
      the whole batch); one all_to_all ships each GPU the bitmap words of its 256-line-aligned
      column shard for every candidate; every GPU fills + scores its lines of ALL P*batch
      candidates; one all_reduce of the exact residual sums (bit-identical to one GPU); one
      all_gather assembles the best candidate's M.  value = P*batch*N / step (also reported
      without the M all_gather).  --strong: --batch is the global batch instead.
  --shard slices: the same B candidates on every rank, one slice of every trajectory per rank.
  --shard samples (strong scaling): the global batch split over the ranks; one all_gather of the
      rewards and one reduce of the best candidate's M to rank 0.
  --shard candidates (weak scaling): --batch candidates per rank, no collective.
The timed steps replay HIP graphs of every maximal run of collective-free phases
(GFlowNet.rollout_phases; one GPU: up to --steps-per-graph whole steps per graph), the
collectives run eagerly between them; the Philox stream id lives on the device, so every replay
draws a fresh rollout.  --pipeline (default): consecutive steps alternate between two stream
lanes and step k+1 waits only for step k's select, so its policy and select run beside step k's
sort, fill and padding (one GPU: GFlowNet(pipeline=True); the columns split: two copies of its
program with their own buffers); every step still does all of its work, with the same bits as
steps run one after the other (tests/test_pipeline_gpu.py, tests/test_bench_dist_gpu.py).  The
per-phase HIP-event timings come from an eager pass of the same step.  Prints ONE JSON line on
rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2|c3] [--batch B]
"""
import argparse
import contextlib
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
    "c2lu": ("lu", 256, torch.float32, "C2 L@U: the reference driver's own candidate (GFlowNet100.py:126-153,173): "
                                       "spilu L@U of the 256^2 5-pt Poisson matrix (65,536 unknowns, 2,162,871 nnz, "
                                       "lines up to 744 wide, fp32) as initial_matrix = original_matrix"),
    "c5s": ("thermal", 1108, torch.float64, "C5 stand-in: synthetic thermal2-like heat-conduction matrix "
                                            "(1,227,664 x 1,227,664, 8,584,786 nnz, 7 per row, lognormal "
                                            "conductivities, randomly permuted numbering, fp64), pattern = A"),
}


def config_matrices(cfg: str):
    """(A, candidate pattern) of a bench config."""
    from gflownet_spai_amd import axial_pattern_3d, poisson_2d, poisson_3d, thermal_like
    dims, grid, dtype, _ = CONFIGS[cfg]
    if dims == "lu":  # GFlowNet100.py:126-153: the driver samples from spilu's L@U, original = initial
        import scipy.sparse as sp
        from gflownet_spai_amd.utils import lu_candidate_matrix
        A = poisson_2d(grid, torch.float64).coalesce()
        C = lu_candidate_matrix(sp.csr_matrix((A.values().numpy(), tuple(A.indices().numpy())), shape=A.shape))
        return C, C
    if dims == "thermal":
        A = thermal_like(grid, 0, dtype)
        return A, A
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
    from gflownet_spai_amd import kernels
    n, W = env.pattern.n, env.pattern.width
    s = env.a_lines.val.element_size() if env._lsq else 4
    per_sample = math.ceil(env.init_nnz / 32) * 4 + (n * W * s if store_m else 0) + 8
    if getattr(env, "rcache", None) is not None:  # QR fill: the action ids + the env-constant R cache
        line = n * W * 4 + kernels.rcache_nbytes(env.rcache)
    elif getattr(env, "gram", None) is not None:
        line = n * W * 4 + kernels.cache_nbytes(env.gram) + (n * W * 4 if env.fill == "copy" else 0)
    else:
        sa = env.a_lines.val.element_size()
        line = n * W * (4 + 4 + 4) + n * env.a_lines.width * (4 + sa)
    return line + B * per_sample


def survey_fill_bytes(env, B, store_m: bool = True) -> float:
    """SURVEY.md §8(d)'s algorithmic bytes of one LSQ fill + ||AM-I|| launch, with A counted as
    A itself (not the Gram cache the kernel streams instead): bytes(A) = nnz_A (s_A + 4) + 4 (N + 1),
    the pattern 4 nnz_P + 4 (N + 1), and per sample the removal bitmap + the M values s_M nnz_P."""
    n = env.pattern.n
    nnz_a = int((env.a_lines.idx >= 0).sum())
    nnz_p = env.init_nnz
    s_a = env.a_lines.val.element_size()
    s_m = s_a if env._lsq else 4
    per_sample = math.ceil(nnz_p / 32) * 4 + (s_m * nnz_p if store_m else 0) + 8
    return nnz_a * (s_a + 4) + 4 * (n + 1) + 4 * nnz_p + 4 * (n + 1) + B * per_sample


def measured_traffic(cfg: str, B: int, kernel: str | None = None):
    """HBM bytes per launch of the roofline kernel from the committed PMC profile of this
    exact workload (profiles/fill_traffic.json, written by scripts/collect_profiles.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `bench.py`; ``kernel``: only a
    record of that kernel), else None."""
    path = os.path.join(ROOT, "profiles", "fill_traffic.json")
    try:
        rec = json.load(open(path))
    except (OSError, ValueError):
        return None
    if "config" in rec:  # single-record form
        rec = {rec["config"]: rec}
    rec = rec.get(cfg, {})
    if rec.get("batch") == B and (kernel is None or kernel + "<" in rec.get("kernel", "")):
        return float(rec["hbm_bytes_per_launch"]), rec.get("source", "profiles/fill_traffic.json")
    return None


def cpu_baseline(cfg, B, budget_s: float, logits, T_mean: float):
    """The reference's CPU path restated with its own torch ops (oracle/spai_oracle.py:
    reference_step = masked softmax + renormalisations + Categorical(probs).sample() per step,
    gflownet.py:116-148, policy.py:65-73; reference_update_residual = keep-mask COO M +
    coalesce + sparse torch.mm + identity subtraction + torch.norm, utils.py:315-353,
    preconditioner.py:79-93), on all the threads torch uses on this host, over a BOUNDED sample
    of the same workload: a few sampler steps over the full [B, E+1] action space and one
    candidate's env.update, extrapolated to the batch (T_mean steps: the GPU run's mean
    trajectory length; B updates).  The reference has no least-squares fill: its env.update is
    the copy fill (the ForwardPolicy forward is not timed: PyG is absent).  A secondary field
    times the oracle's numpy Gumbel-top-k rollout + LSQ fill (1 thread) on part of the columns."""
    from oracle import spai_oracle as O

    A, P = config_matrices(cfg)
    Pc, Ac = P.coalesce(), A.coalesce()
    r, c = (t.numpy() for t in Pc.indices())
    v = Pc.values().float().numpy()
    n = A.shape[0]
    E = len(r)
    lg_t = torch.as_tensor(np.asarray(logits, np.float32)).view(1, -1)
    assert lg_t.shape[1] == E + 1
    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(0)
    hist, t_steps, steps = [], 0.0, 0
    t_budget = 0.4 * budget_s
    while steps < 3 or (t_steps < t_budget and steps < 40):
        t0 = time.perf_counter()
        a, _ = O.reference_step(lg_t, B, hist, g)
        t_steps += time.perf_counter() - t0
        hist.append(a.view(B))
        steps += 1
    t_step = t_steps / steps
    A_t = torch.sparse_coo_tensor(Ac.indices(), Ac.values().float(), (n, n))
    removed = np.random.default_rng(1).random(E) < 0.2
    t0 = time.perf_counter()
    O.reference_update_residual(r, c, v, removed, n, A_t)
    t_upd = time.perf_counter() - t0
    t_batch = T_mean * t_step + B * t_upd
    out = {"value": B * n / t_batch, "unit": "columns/s", "cores": threads, "kind": "port",
           "host_cpus": os.cpu_count(), "torch_threads": threads,
           "sample": f"reference ops in torch-CPU ({threads} threads of {os.cpu_count()} CPUs): {steps} sampler steps "
                     f"over [B={B}, E+1={E + 1}] ({t_step * 1e3:.1f} ms/step) and one env.update copy fill + "
                     f"||MA-I||_F ({t_upd:.2f} s), extrapolated to the batch: {T_mean:.0f} steps (the GPU run's "
                     f"mean trajectory length) + {B} updates"}
    if A.shape == P.shape and Ac._nnz() == E:  # secondary (pattern = A): numpy Gumbel-top-k + LSQ fill, 1 thread
        idx, act, _ = O.lines_from_coo(r, c, v, n, "col")
        a_idx, _, a_val = O.lines_from_coo(r, c, v.astype(np.float64), n, "col")
        t0 = time.perf_counter()
        rem, *_ = O.throughput_rollout(np.asarray(logits, np.float32), 1, 1234, 0)
        t_roll = time.perf_counter() - t0
        keep = (idx >= 0) & ~rem[0][np.clip(act, 0, None)]
        cols = min(n, 65536)
        t0 = time.perf_counter()
        O.lsq_fill(idx, keep, a_idx, a_val, np.arange(cols))
        t_fill = (time.perf_counter() - t0) * n / cols
        out["numpy_gumbel_lsq"] = {"value": n / (t_roll + t_fill), "unit": "columns/s", "cores": 1,
                                   "sample": f"oracle numpy Gumbel-top-k rollout ({t_roll:.2f} s) + LSQ fill of "
                                             f"{cols} columns extrapolated to {n}"}
    return out


def generic_residual_leg(env, log, cfg: str, reps: int = 10):
    """The generic SpMM residual (spai_residual_lines: ||A M_b - I||_F^2 of B arbitrary sparse
    M_b, preconditioner.py:79-93 for any M) on the step's B candidates: their stored LSQ values
    with each candidate's own kept index set (removed slots -> -1).  Timed with HIP events on
    the launch stream; algorithmic bytes per launch = bytes(A) + B x bytes(M_b) (SURVEY §8d
    with A shared by the batch: the kernel reads each line of A once for all B samples).  Also checks the result against the fused fill kernel's
    residual (they differ by d^T G d, d = the fp32 rounding of M)."""
    from gflownet_spai_amd import kernels
    pat, a = env.pattern, env.a_lines
    bits = log.removed.view(torch.int32)
    act = pat.act.long().clamp(min=0)
    rem = ((bits[:, act >> 5] >> (act & 31)) & 1).bool()
    idx = torch.where(rem | (pat.idx < 0), torch.full_like(pat.idx, -1), pat.idx).contiguous()
    m = env.last_m.contiguous()
    B, n, W = m.shape
    # 13-wide lines: G, c from the pattern's Gram cache dictionary (the index matching done once per
    # env, untimed: the env's own cache, or one built here when the env keeps none — the QR fill
    # reads its R cache; spai_residual_lines_gram, bit-identical to the matching kernel).  5/7-wide
    # lines keep the matching kernel: their matching is cheap (C4: 80 us from the dictionary vs 70)
    gram = env.gram if W > 7 else None
    if gram is None and W > 7:
        gram = kernels.gram_build(pat, a)
        g32 = kernels.gram_compact(gram, pat)
        gram = g32 if g32 is not None else gram
    if torch.is_tensor(gram):
        gram = kernels.cache_dict(gram, pat.n)
    kw = dict(gram=gram, pattern=pat) if gram is not None else {}
    res2 = kernels.residual_lines(idx, m, a, **kw)  # warm-up
    kernels.TIMERS = {}
    for _ in range(reps):
        res2 = kernels.residual_lines(idx, m, a, **kw)
    torch.cuda.synchronize()
    ms = float(np.mean(kernels.timer_ms("residual_lines")))
    kernels.TIMERS = None
    ref = env.last_residual.double() ** 2
    rel = float(((res2 - ref).abs() / ref).max())
    av = kernels.narrow_values(a)  # fp64 A with fp32-exact values is read as fp32 (same numbers)
    bytes_a = a.idx.numel() * 4 + av.numel() * av.element_size()
    bytes_m = n * W * (4 + m.element_size())
    name = "k_resid_gram" if gram is not None else ("k_resid_shared" if W <= 7 else "k_resid_wide")
    extra = (f"; G, c from the pattern's Gram cache dictionary ({gram.entries} entries, "
             f"{kernels.cache_nbytes(gram)} B)" if gram is not None else "")
    out = roofline_obj(f"{name}<{W},{a.width},{str(av.dtype)[6:]},{str(m.dtype)[6:]}> (||A M_b - I||_F^2 of "
                       f"B={B} arbitrary sparse M_b: the step's LSQ fills with their own kept index sets; "
                       f"bytes = bytes(A) + B x bytes(M_b){extra})", bytes_a + B * bytes_m, ms,
                       traffic=measured_traffic(cfg + "_residual", B, name))
    out["max_rel_diff_vs_fused_fill"] = rel
    return out


def select_bytes(env, B: int, winners: float) -> float:
    """Algorithmic HBM bytes of the select phase (k_presample + k_splitters + k_tile + k_bsum,
    DESIGN.md §3): the shared logits row read once and its inverse rates / weights written
    once (k_presample), read once more by k_tile (the B samples of a tile share them through
    L2), the B removal bitmaps and 12 bytes per staged winner."""
    E1 = env.num_actions
    return 4 * E1 + 2 * 8 * E1 + B * 4 * math.ceil((E1 - 1) / 32) + 12 * winners


def rollout_bytes(env, B: int) -> float:
    """SURVEY.md §8(d)'s algorithmic bytes of the throughput rollout: the logits once per batch,
    4 (E + 1), and the B removal bitmaps, B ceil(E / 8).  One k_tile launch covers all of it (every
    action of every sample), so these are also k_tile's algorithmic bytes per launch."""
    E1 = env.num_actions
    return 4 * E1 + B * math.ceil((E1 - 1) / 8)


def pmc_record(cfg: str, B: int, kernel: str):
    """The committed PMC summary of ``kernel`` for this workload (profiles/fill_traffic.json key
    ``<cfg>_<kernel>``): (HBM bytes per launch, VALU wave-instructions per launch, source) or None."""
    path = os.path.join(ROOT, "profiles", "fill_traffic.json")
    try:
        rec = json.load(open(path)).get(f"{cfg}_{kernel}", {})
    except (OSError, ValueError):
        return None
    if rec.get("batch") != B:
        return None
    return float(rec["hbm_bytes_per_launch"]), rec.get("valu_insts_per_launch"), rec.get("source")


VALU_CLOCK_GHZ = 2.4  # MI355X_MICROARCH.md: peak engine clock
N_SIMDS = 256 * 4


def roofline_obj(kernel, nbytes, ms, traffic=None):
    """traffic: (HBM bytes per launch, source) from a committed PMC pass of the same workload
    (measured_traffic: NOT measured in this run; `traffic_source` names the file), or None."""
    achieved = nbytes / (ms * 1e-3) / 1e9
    tb, src = traffic if traffic is not None else (None, None)
    return {"kernel": kernel, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": tb, "traffic_source": src, "bytes_per_launch": nbytes,
            "avg_launch_ms": ms}


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
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard", default="columns", choices=["columns", "slices", "samples", "candidates"])
    ap.add_argument("--strong", action="store_true",
                    help="columns split: --batch is the GLOBAL batch (batch/P rollouts per GPU) instead of per GPU")
    ap.add_argument("--assemble", default="best", choices=["best", "all", "none"])
    ap.add_argument("--pipeline", action=argparse.BooleanOptionalAction, default=True,
                    help="one GPU: consecutive steps on two alternating stream lanes, step k+1's policy and "
                         "select beside step k's sort, fill and padding (GFlowNet(pipeline=True); every step "
                         "still does all of its work; --no-pipeline: one step after the other)")
    ap.add_argument("--side", default="auto", choices=["auto", "AM", "MA"],
                    help="reward side: ||AM - I|| (the north star's column SPAI) or ||MA - I|| (the reference's "
                         "calculate_residual); auto: MA for c2lu (the driver's configuration), else AM")
    ap.add_argument("--fill", default="auto", choices=["auto", "lsq", "qr", "copy"],
                    help="least-squares fill: Householder QR from the env's R cache (qr, the north star's algorithm) "
                         "or the normal equations from the Gram cache (lsq); auto: qr where the cached QR solve is "
                         "compiled (pattern lines <= 7 wide: c2, c4, c5s), lsq for c3's 13-wide lines")
    ap.add_argument("--no-graph", action="store_true", help="time eager steps (host launches) instead of graph replays")
    ap.add_argument("--steps-per-graph", type=int, default=8,
                    help="one GPU: at most this many consecutive steps captured in one HIP graph (the largest count "
                         "that divides --steps; 1: one graph replay per step)")
    ap.add_argument("--overlap", default="sort", choices=["sort", "fill", "select", "none"],
                    help="one GPU: the fill + rewards on a second stream beside the trajectory sort, the sort "
                         "launched first (sort) or the fill first (fill); none: one stream")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (nccl = RCCL over xGMI; gloo only to rehearse the flow)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every rank on GPU 0 (rehearsal of the multi-rank flow on a one-GPU box, with --backend gloo)")
    ap.add_argument("--sort-blocks", type=int, default=0,
                    help="persistent blocks of the trajectory sort (0: one per CU); fewer leave CUs to the fill "
                         "running beside it (--overlap)")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group and run the --shard split's multi-GPU step even at one rank "
                         "(--gpus 1 --backend nccl: the columns split's graph segments, all_to_all and pipelined M "
                         "all_gather through a one-rank RCCL group)")
    ap.add_argument("--dump", default=None,
                    help="write the last assembled step (Philox stream id, rewards of every candidate, the assembled "
                         "M) to this .pt file (rank 0; tests/test_bench_dist_gpu.py)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # one child process per GPU; nothing here touched the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with "
                 f"torch.distributed.run --nproc-per-node {args.gpus} or without WORLD_SIZE")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_gpu:  # rehearsal of the multi-rank flow on a one-GPU box (with --backend gloo)
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_on = world > 1 or args.dist
    if dist_on:
        import torch.distributed as dist
        if "RANK" not in os.environ:  # --dist on one GPU without a launcher: a one-rank group on 127.0.0.1
            import socket
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(port))
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, kernels
    from gflownet_spai_amd.distributed import LINE_ALIGN
    if args.sort_blocks:
        kernels.set_sort_blocks(args.sort_blocks)

    dims, grid, dtype, text = CONFIGS[args.config]
    if args.fill == "auto":
        args.fill = {"c3": "lsq", "c2lu": "copy"}.get(args.config, "qr")
    if args.side == "auto":
        args.side = "MA" if args.config == "c2lu" else "AM"
    A, P = config_matrices(args.config)
    n = A.shape[0]
    env = PreconditionerEnv(n, P, A, side=args.side, fill=args.fill, keep_m=True, device=dev)
    E = env.num_actions - 1
    shard = args.shard if dist_on else "columns"  # one GPU: every split is the same one-GPU step
    if shard in ("samples", "slices") or (shard == "columns" and args.strong):
        if args.batch % world:
            sys.exit(f"bench.py: --shard {shard} needs the batch ({args.batch}) divisible by the GPU count ({world})")
        B, bl, strong = args.batch, args.batch // world if shard != "slices" else args.batch, True
    else:  # columns (weak: --batch rollouts per GPU, fill of every candidate by column shard) / candidates
        B, bl, strong = args.batch * world, args.batch, False
    base = {"samples": rank * bl, "candidates": rank * bl}.get(shard, 0)
    split = {"columns": "columns", "slices": "slices"}.get(shard) if dist_on else None
    model = GFlowNet(make_policy(env, P, dev), None, env, mode="throughput", seed=1234, sample_base=base,
                     shard=(rank, world, None) if split else None, split=split or "columns",
                     overlap=False if args.overlap == "none" else args.overlap,
                     pipeline=args.pipeline and not dist_on)
    s0 = [P] * bl
    assembled = {}
    do_assemble = [args.assemble != "none" and dist_on and shard != "candidates"]
    # the M all_gather of a step runs asynchronously and overlaps the next step's rollout; the
    # timed region still ends after the last one (gather.wait() before the closing barrier).
    # GFlowNet gives both splits 256-line-aligned shards (its .lines): the gather uses the same
    from gflownet_spai_amd.distributed import LineGather
    gather = LineGather(n, align=LINE_ALIGN) if do_assemble[0] else None

    def assemble(log, m=None):
        if not do_assemble[0]:
            return
        if m is None:
            m = env.last_m  # columns: [B, this shard's lines, W] of EVERY candidate; slices: the same B on every rank
        if shard == "samples":  # global rewards everywhere, the best candidate's M on rank 0
            from gflownet_spai_amd.distributed import select_best_samples
            assembled["r"], assembled["best"], assembled["m"] = select_best_samples(log.rewards, m)
            return
        if args.assemble == "best":  # the candidate with the highest reward: the preconditioner kept
            gather.start(m, rows=torch.argmax(log.rewards_all).view(1))
        else:
            gather.start(m)

    phases = model.rollout_phases()

    def eager_step():
        st = {"s0": s0}
        for i, (fn, kind) in enumerate(phases):
            model.run_phase(fn, kind, st, timer=f"phase{i}_{fn.__name__.strip('_')}")
        with kernels._timed("assemble"):
            assemble(st["log"])
        return st["log"]

    def barrier():
        if dist_on:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    with torch.no_grad():
        for _ in range(args.warmup):
            log = eager_step()
        # eager pass with per-phase HIP events (on the stream the kernels run on)
        kernels.TIMERS = {}
        k_eager = max(1, min(args.steps, 10))
        barrier()
        t0 = time.perf_counter()
        for _ in range(k_eager):
            log = eager_step()
        barrier()
        dt_eager = (time.perf_counter() - t0) / k_eager
        phase_ms = {k: float(np.mean(kernels.timer_ms(k))) for k in kernels.TIMERS}
        kernels.TIMERS = None
        if dist_on:  # every rank's phase times, max over ranks (the collectives wait on the slowest rank)
            names = sorted(phase_ms)
            t = torch.tensor([phase_ms[k] for k in names], device=dev, dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            phase_ms_max = dict(zip(names, t.tolist()))
        kernel_ms = {}
        if kernels.kernel_timers_available():
            # single kernels inside the multi-kernel entry points (k_tile, k_sort2, the fill): HIP events
            # around each launch on its stream, in a second eager pass (their records would add to the
            # phase times above)
            kernels.kernel_timer_arm(True)
            for _ in range(k_eager):
                log = eager_step()
            barrier()
            kernels.kernel_timer_arm(False)
            kernel_ms = {k: ms for k, (cnt, ms) in kernels.kernel_timer_read().items() if cnt > 0}

        use_graph = not args.no_graph
        if use_graph:
            if gather is not None:
                gather.wait()  # no RCCL gather in flight while a graph is captured
            # capture every maximal run of collective-free phases as one HIP graph (one GPU: the
            # whole step is one graph); the collectives run eagerly between the replays
            model.pipeline_join()
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                eager_step()
                model.pipeline_join()
            torch.cuda.current_stream(dev).wait_stream(side)
            barrier()
            # --pipeline with a split (columns): two copies of the step's program, each captured on its
            # own stream with its own buffers and memory pool, replayed alternately on two stream
            # lanes; step k+1 waits only for step k's select (the Philox stream counter), so its
            # select and bitmap pack run beside step k's exchange, fill and reductions.  The
            # collectives stay eager and are issued in the same order on every rank.
            xpipe = dist_on and args.pipeline and split is not None

            def build(st, cs):
                program, pool_, run = [], [None], []

                def capture(run):
                    """One graph of consecutive device phases; its program entry keeps the first phase's
                    stream order (kind "side": replayed on the model's side stream, forked from the
                    current one; "join": after the side stream's work)."""
                    kind = run[0][1]
                    g = torch.cuda.CUDAGraph()
                    if dist_on:  # no collective of the previous eager phase still in flight on RCCL's stream
                        torch.cuda.synchronize()
                    # a side segment runs beside later main segments: its own memory pool (graphs that
                    # share a pool may reuse each other's freed blocks, safe only when replayed in order)
                    gp = None if kind == "side" else pool_[0]
                    # thread_local: a HIP call from an RCCL helper thread cannot invalidate this capture
                    with torch.cuda.graph(g, pool=gp, stream=cs,
                                          capture_error_mode="thread_local" if dist_on else "global"):
                        for f, _k in run:
                            f(st)
                        model.pipeline_join()  # (a pipelined step's lanes rejoin inside its capture)
                    if kind != "side":
                        pool_[0] = g.pool()
                    if kind == "side":
                        sstream = model._side_stream(dev)

                        def rep():
                            sstream.wait_stream(torch.cuda.current_stream(dev))
                            with torch.cuda.stream(sstream):
                                g.replay()
                        return rep
                    if kind == "join":
                        sstream = model._side_stream(dev)

                        def rep():
                            torch.cuda.current_stream(dev).wait_stream(sstream)
                            g.replay()
                        return rep
                    return g.replay

                # segments: maximal runs of device phases, cut at every collective, around every "side"
                # phase and before every "join" phase
                for fn, kind in phases + [(None, True)]:
                    if fn is not None and kind is not True and kind != "side" and not (kind == "join" and run):
                        run.append((fn, kind))
                        continue
                    if run:
                        program.append(("graph:" + "+".join(f.__name__.strip("_") for f, _k in run), capture(run)))
                        run = []
                    if fn is None:
                        break
                    if kind is True:
                        fn(st)  # a collective, eagerly (allocates its persistent buffers before the next capture)
                        program.append((fn.__name__.strip("_"), lambda f=fn, st=st: f(st)))
                    elif kind == "side":
                        program.append(("graph(side):" + fn.__name__.strip("_"), capture([(fn, kind)])))
                    else:  # "join" opens the next segment
                        run.append((fn, kind))
                return program, pool_[0]

            progs = []
            for bt in (["A", "B"] if xpipe else [""]):
                stp = {"s0": s0, "bt": bt}
                program, pool = build(stp, torch.cuda.Stream(dev) if xpipe else None)
                # (this program's Log, M and residual: what its replays write)
                progs.append({"program": program, "log": stp["log"], "m": env.last_m, "res": env.last_residual,
                              "lane": torch.cuda.Stream(dev, priority=-1) if xpipe else None})
            glog = progs[0]["log"]
            pstate = {"i": 0, "sel": None, "last": progs[0], "pending": None}

            def step(host=None):
                pr = progs[pstate["i"]]
                pstate["i"] = (pstate["i"] + 1) % len(progs)
                ln = pr["lane"]
                ctx = contextlib.nullcontext()
                if ln is not None:  # fork the lane after the previous step's select (via the caller's stream)
                    c = torch.cuda.current_stream(dev)
                    if pstate["sel"] is not None:
                        c.wait_event(pstate["sel"])
                    ln.wait_stream(c)
                    ctx = torch.cuda.stream(ln)
                with ctx:
                    for i, (name, p) in enumerate(pr["program"]):
                        if host is None:
                            p()
                        else:  # host issue time per program entry (diagnostic pass)
                            t = time.perf_counter()
                            p()
                            host.setdefault(name, []).append(time.perf_counter() - t)
                        if ln is not None and i == 0:  # the select phase: what the next step waits for
                            ev = torch.cuda.Event()
                            ev.record(ln)
                            pstate["sel"] = ev
                t = time.perf_counter()
                if ln is None:
                    with ctx:
                        assemble(pr["log"], pr["m"])
                else:  # the PREVIOUS step's M gather, on its own lane after this step's program: RCCL runs
                    # its collectives in issue order, so this step's bitmap all_to_all goes first
                    flush_assemble()
                    pstate["pending"] = pr
                if host is not None:
                    host.setdefault("assemble", []).append(time.perf_counter() - t)
                pstate["last"] = pr
                return pr["log"]

            def flush_assemble():
                pr = pstate.get("pending")
                if pr is not None:
                    with torch.cuda.stream(pr["lane"]):
                        assemble(pr["log"], pr["m"])
                    pstate["pending"] = None

            for _ in range(max(1, args.warmup)):
                log = step()
            flush_assemble()
            # a step without collectives (one GPU): spg consecutive steps in ONE graph, so the
            # ~12 us between two graph launches is paid once per spg steps (every step is still a
            # whole sample_states: its own select, sort, fill and Log, its own Philox stream id)
            spg = max(1, args.steps_per_graph) if all(not k for _, k in phases) else 1
            while args.steps % spg:  # the largest count <= --steps-per-graph that divides the timed steps
                spg -= 1
            if spg > 1:
                gm = torch.cuda.CUDAGraph()
                model.pipeline_join()
                with torch.cuda.graph(gm, pool=pool):
                    for _ in range(spg):
                        stm = {"s0": s0}
                        for f, _c in phases:
                            f(stm)
                    model.pipeline_join()  # --pipeline: consecutive steps overlap inside the graph
                mlog = stm["log"]
                gm.replay()
        else:
            step = eager_step
            spg = 1

            def flush_assemble():
                pass

        def steps(k):  # k timed steps: the remainder as single steps, then whole multi-step graphs
            out = None
            if spg > 1:
                for _ in range(k % spg):
                    out = step()
                for _ in range(k // spg):
                    gm.replay()  # the last capture: env.last_* and mlog name its last step's buffers
                    out = mlog
                return out
            for _ in range(k):
                out = step()
            return out

        barrier()
        t0 = time.perf_counter()
        log = steps(args.steps)
        flush_assemble()
        if gather is not None:
            gather.wait()
        barrier()
        dt = (time.perf_counter() - t0) / args.steps
        dt_noasm = dt
        if args.dump and rank == 0:  # the last timed step: its stream id, every candidate's reward, M
            res = pstate["last"]["res"] if use_graph and spg == 1 else env.last_residual
            dump = {"stream_id": model.rollouts - 1, "rewards_all": log.rewards_all.double().cpu(),
                    "residual": res.double().cpu(), "shard": shard, "world": world}
            if gather is not None and args.assemble != "none":
                dump["m_assembled"] = gather.result().cpu()
            torch.save(dump, args.dump)
        if do_assemble[0]:  # the same steps without the M all_gather (reported apart)
            do_assemble[0] = False
            barrier()
            t0 = time.perf_counter()
            log = steps(args.steps)
            flush_assemble()
            barrier()
            dt_noasm = (time.perf_counter() - t0) / args.steps
            do_assemble[0] = True
        host_us = None
        if use_graph and dist_on:  # host issue time of each program entry (a pass after the timed steps)
            host = {}
            for _ in range(k_eager):
                step(host)
            flush_assemble()
            if gather is not None:
                gather.wait()
            barrier()
            host_us = {k: 1e6 * float(np.mean(v)) for k, v in host.items()}
    if dist_on:
        t = torch.tensor([dt, dt_eager, dt_noasm], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt, dt_eager, dt_noasm = float(t[0]), float(t[1]), float(t[2])
    res = env.last_residual.double().cpu().numpy()
    counts = log.counts.cpu().numpy()

    if rank == 0:
        # the fill kernel's own launch time (kernel timers), else its phase
        fill_ms = kernel_ms.get("k_qr_solve" if args.fill == "qr" else "k_gram_fill",
                                phase_ms.get("fill_residual", float("nan")))
        fb = fill_bytes(env, B if shard == "columns" else bl)
        if split:  # the rank's fill covers its own lines only (rank 0: the first shard)
            fb *= (model.lines[1] - model.lines[0]) / n
        gram_t = "f32" if env.gram is not None and env.gram.dtype == torch.float32 else "f64"
        workload = text + {
            "columns": (f", {bl} rollouts per GPU x {world} GPUs = B={B} candidates; columns of M sharded over the "
                        f"GPUs (256-line-aligned shards, fill + ||AM-I|| of every candidate per shard)" +
                        (": one all_to_all of the bitmap windows, one all_reduce of the exact residual sums, one "
                         "all_gather of the best candidate's M" if world > 1 else "")),
            "slices": f", B={B} candidates, trajectory slices + lines of M per GPU over {world} GPUs (one all_reduce, "
                      f"{args.assemble} M all_gather)",
            "samples": f", B={B} candidates split over {world} GPUs ({bl} per GPU; one all_gather of the rewards "
                       f"and one reduce of the best candidate's M per step)",
            "candidates": f", B={bl} candidates per GPU, no collective"}[shard]
        metric = {"c4": "SPAI columns/sec + final ||AM-I||_F, 2D Poisson 1024^2, at 1/2/4/8 GPU",
                  "c2": "SPAI columns/sec + final ||AM-I||_F, 2D Poisson 256^2 (C2)",
                  "c3": "SPAI columns/sec + final ||AM-I||_F, 3D Laplacian 64^3 fp64 (C3)",
                  "c5s": "SPAI columns/sec + final ||AM-I||_F, thermal2-like stand-in fp64 (C5 stand-in)",
                  "c2lu": "SPAI columns/sec + final ||MA-I||_F, the driver's L@U candidate of 256^2 Poisson (copy fill)"
                  }[args.config]
        out = {
            "metric": metric,
            "value": B * n / dt,
            "unit": "columns/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32 storage, f64 solve/accumulate" if dtype == torch.float32 else "f64",
            "data": "synthetic (random-init seeded ForwardPolicy GATv2x2+fc, hid=4, evaluated on the state graph in "
                    "every step; terminal fc bias set for 20% expected removal; matrix from its stencil)",
            "config": {"workload": workload + ": ForwardPolicy logits + throughput rollout + " +
                                   ("copy fill (the reference's)" if args.fill == "copy" else "LSQ fill") +
                                   (" (Householder QR)" if args.fill == "qr" else "") + f" + ||{args.side[0]}"
                                   f"{args.side[1]}-I||_F",
                       "N": n, "E": E, "global_batch": B, "rollouts_per_gpu": bl,
                       "parallelism": f"{shard} sharded x{world}"},
            "value_without_assembly": B * n / dt_noasm,
            "ms_per_step_without_assembly": dt_noasm * 1e3,
            "graph": use_graph,
            "steps_per_graph": spg,
            "pipeline": bool(args.pipeline and (not dist_on or split is not None)),
            "ms_per_step_eager": dt_eager * 1e3,
            "final_residual_fro": float(res[0]),
            "final_residual_fro_mean": float(res.mean()),
            "removed_per_candidate_mean": float(counts.mean()),
            "phases_ms": phase_ms,
            "roofline": roofline_obj(f"k_gram_fill<{env.pattern.width},{gram_t},LSQ> (LSQ fill of M + ||AM-I||^2; A "
                                     f"reaches it through the env-constant Gram cache)" if args.fill != "copy" else
                                     f"k_line{'_hash' if env.pattern.width > 7 else ''} (the reference's copy fill + "
                                     f"||{args.side[0]}{args.side[1]}-I||^2 of lines up to {env.pattern.width} wide)",
                                     fb, fill_ms, measured_traffic(args.config, bl)),
        }
        if args.fill == "qr":  # the Householder-QR fill reads A itself: SURVEY §8(d)'s bytes are its bytes
            sbq = survey_fill_bytes(env, B if shard == "columns" else bl)
            if split:
                sbq *= (model.lines[1] - model.lines[0]) / n
            if env.rcache is not None:  # phase 2 from the R cache: its bytes are the cache + the per-sample stream
                tabled = (isinstance(env.rcache, kernels.QrDict) and env.rcache.entries <= 4096 and
                          kernels.qr_class(env.pattern.width, env.a_lines.width) == 5)
                head = (f"k_qr_table<5> + k_qr_lookup<5> (LSQ fill of M by Householder QR: every (dictionary entry, "
                        f"keep mask) masked re-triangularisation of the cached R solved once per call "
                        f"({env.rcache.entries} entries x 32 masks), each (line, sample) reading its M and residual "
                        f"from that table" if tabled else
                        f"k_qr_solve<{env.pattern.width}> (LSQ fill of M by Householder QR: masked "
                        f"re-triangularisation of each line's cached R")
                out["roofline"] = roofline_obj(
                    head + f" (the full block A[I, slots] factored once per env, rows {env.qr_rows}"
                    + (f"; the cache as its dictionary: {env.rcache.entries} distinct line entries"
                       if isinstance(env.rcache, kernels.QrDict) else "") +
                    ") + ||AM-I||^2)", fb, fill_ms, measured_traffic(args.config + "_qr", bl))
            else:
                out["roofline"] = roofline_obj(f"k_qr_fill<{env.pattern.width},rows {env.qr_rows}> (LSQ fill of M by "
                                               f"Householder QR of each line's block A[I, J] + ||AM-I||^2)", sbq,
                                               fill_ms, measured_traffic(args.config + "_qr", bl))
        # the same launch at SURVEY §8(d)'s bytes (A counted as bytes(A), not as the Gram cache)
        sb = survey_fill_bytes(env, B if shard == "columns" else bl)
        if split:
            sb *= (model.lines[1] - model.lines[0]) / n
        out["roofline"]["bytes_survey_8d"] = sb
        out["roofline"]["frac_survey_8d"] = sb / (fill_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
        # achieved / frac at SURVEY §8(d)'s algorithmic bytes (the contract's figure); the bytes the
        # kernel streams instead (the env-constant Gram / R cache, or its dictionary, for A) beside them
        rf = out["roofline"]
        rf["bytes_cache_counted"], rf["frac_cache_counted"] = rf["bytes_per_launch"], rf["frac"]
        rf["bytes_per_launch"], rf["achieved"] = sb, sb / (fill_ms * 1e-3) / 1e9
        rf["frac"] = rf["achieved"] / HBM_PEAK_GBS
        # the fill (the reward kernel the north star's >= 40 % names) is reported as roofline_fill;
        # the headline roofline is the step's DOMINANT kernel, k_tile (the rollout's select)
        out["roofline_fill"] = out.pop("roofline")
        out["kernel_ms"] = kernel_ms
        tile_ms = kernel_ms.get("k_tile")
        if tile_ms:
            rb = rollout_bytes(env, bl)
            pm = pmc_record(args.config, bl, "tile")
            rt = roofline_obj("k_tile (throughput rollout select: Philox4x32-10 + fp32 arrival time per (action, "
                              "sample), removal bitmaps, bucket grouping of the winners; bytes = SURVEY 8(d) rollout: "
                              "4 (E+1) logits + B ceil(E/8) bitmaps)", rb, tile_ms,
                              (pm[0], pm[2]) if pm else None)
            if pm:
                rt["traffic_over_bytes"] = pm[0] / rb
                if pm[1]:  # issue-time bound: a wave64 VALU instruction holds a SIMD for 4 cycles
                    issue_ms = pm[1] * 4 / N_SIMDS / (VALU_CLOCK_GHZ * 1e9) * 1e3
                    rt["valu"] = {"wave_insts_per_launch": pm[1],
                                  "lane_insts_per_action_sample": pm[1] * 64 / ((env.num_actions - 1) * bl),
                                  "issue_ms_at_peak_clock": issue_ms, "issue_frac_of_launch": issue_ms / tile_ms,
                                  "source": pm[2]}
            out["roofline"] = rt
        else:  # (a library without the kernel timers: the fill stays the headline)
            out["roofline"] = out["roofline_fill"]
        if not dist_on:
            sel = roofline_obj("rollout_select phase: k_presample + k_splitters + k_tile + k_bsum (k_tile ~80 % of "
                               "it; VALU/latency-bound, not bandwidth-bound: DESIGN.md §3); bytes = the implementation's "
                               "own streams (logits, rates/weights, bitmaps, 12-byte staged winners)",
                               select_bytes(env, bl, float(counts.sum())),
                               phase_ms.get("rollout_select", float("nan")))
            sel["bytes_survey_8d"] = rollout_bytes(env, bl)
            sel["frac_survey_8d"] = sel["bytes_survey_8d"] / (sel["avg_launch_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS
            out["roofline_select"] = sel
            if env.pattern.width <= 13 and env.a_lines.width <= 7:  # (the generic residual's widths)
                with torch.no_grad():
                    out["roofline_residual"] = generic_residual_leg(env, log, args.config)
        if dist_on:  # the multi-GPU step explains itself: collective phases, max over ranks (HIP events on the
            # compute stream: the time it waits for each collective), the group and the library
            out["phases_ms_max_over_ranks"] = phase_ms_max
            col = {"bitmap_all_to_all_issue": "_c_send", "bitmap_all_to_all_wait": "_c_recv",
                   "limb_all_reduce": "_c_reduce", "slices_all_reduce": "rollout_exchange"}
            out["collectives_ms"] = {name: v for name, key in col.items()
                                     for k, v in phase_ms_max.items() if k.endswith(key)}
            if "line_gather_wait" in phase_ms_max:
                out["collectives_ms"]["line_gather_wait"] = phase_ms_max["line_gather_wait"]
            if host_us is not None:  # rank 0's host time to issue each graph replay / eager collective
                out["host_issue_us"] = host_us
                out["host_issue_us_total"] = sum(host_us.values())
            out["world_size"] = torch.distributed.get_world_size()
            out["backend"] = torch.distributed.get_backend()
            if args.backend == "nccl":
                v = torch.cuda.nccl.version()
                out["rccl_version"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        if not args.no_cpu_baseline and not dist_on:
            with torch.no_grad():
                lg_host = model.forward_policy.logits(model.state_to_data(s0[:1])[0])[0].reshape(-1).cpu().numpy()
            out["cpu_baseline"] = cpu_baseline(args.config, B, args.cpu_budget, lg_host, float(counts.mean()) + 1)
        print(json.dumps(out), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
