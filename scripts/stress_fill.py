"""Repeat the parity rollout golden check and Gram-vs-direct fill in one process (flake hunt)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gflownet_spai_amd import GFlowNet, PreconditionerEnv, kernels, poisson_2d  # noqa: E402
from tests.test_hip_parity import FixedLogits, coo, load  # noqa: E402

bad = 0
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    for seed in range(4):
        d = load(f"c1_rollout_s{seed}.npz")
        n = int(d["n"])
        A = coo(d["rows"], d["cols"], d["vals"], n)
        env = PreconditionerEnv(n, A, A)
        torch.manual_seed(int(d["seed"]))
        g = GFlowNet(FixedLogits(d["logits"]), None, env, mode="parity")
        log = g.sample_states([A] * int(d["B"]), return_log=True)
        ok_a = np.array_equal(log.actions.cpu().numpy(), d["actions"])
        rw = log.rewards.cpu().numpy()
        ok_r = np.allclose(rw, d["rewards"], rtol=1e-6)
        if not (ok_a and ok_r):
            bad += 1
            print("MISMATCH rep", rep, "seed", seed, ok_a, rw, d["rewards"],
                  env.last_residual.cpu().numpy(), flush=True)
    for B in (1, 3, 4, 5, 8):
        Ap = poisson_2d(40)
        n = Ap.shape[0]
        for fill in ("copy", "lsq"):
            env = PreconditionerEnv(n, Ap, Ap, side="AM", fill=fill)
            E = env.init_nnz
            rng = np.random.default_rng(rep * 10 + B)
            acts = torch.from_numpy(np.where(rng.random((B, E)) < 0.3, np.arange(E), -1))
            removed, counts = kernels.actions_to_removed(acts.cuda(), E)
            ref, _ = kernels.fill_residual(env.pattern, env.a_lines, removed, fill == "lsq")
            got, _ = kernels.fill_residual_gram(env.pattern, env.gram, removed, fill == "lsq")
            if not np.allclose(got.cpu().numpy(), ref.cpu().numpy(), rtol=1e-12):
                bad += 1
                print("GRAM MISMATCH", rep, B, fill, got.cpu().numpy(), ref.cpu().numpy(), flush=True)
print("stress done, mismatches:", bad)
