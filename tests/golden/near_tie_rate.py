"""Measure how often parity mode's scoring can disagree with the reference's sampler chain.

Test infrastructure (build container only, CPU): it evaluates the reference's per-step chain
with torch-CPU ops as ``oracle.spai_oracle.reference_step`` restates it (policy.py:65-73 masked
softmax, gflownet/gflownet.py:116-119 row renormalisation, Categorical's own renormalisation and
multinomial's argmax(p / q), gflownet.py:148), pinned by the G6/G8 reference rollouts.

Per active sample-step it records
  * the relative gap between the two best scores of the reference chain, (s1 - s2) / s1;
  * whether the kernel's form argmax(exp(l - lmax) / q) (rollout.hip k_parity_partial;
    numpy's fp32 exp stands in for the device expf, both within ~1 ulp) picks another action.
A flip needs the gap to be below the relative rounding difference of the two forms (a few fp32
ulp, < 1e-6), so the count of gaps below 1e-6 bounds the flip rate from above.

It also evaluates the C2 softmax under two of torch's CPU kernels (ATEN_CPU_CAPABILITY=default
and the host's best vector ISA) and counts the probabilities whose bits differ: the reference's
own fp32 chain is not reproducible bit for bit across hosts.

Usage: python tests/golden/near_tie_rate.py [steps] [out.json]
"""
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.spai_oracle import poisson2d  # noqa: E402

THRESH = (1e-7, 1e-6, 1e-5, 1e-4, 1e-3)


def c2_logits(seed=21, terminal=5.0):
    """The G8 recipe (make_golden.py g8): C2 5-pt Poisson, E = 326,656."""
    E = poisson2d(256)[0].size
    lg = torch.randn(E + 1, generator=torch.Generator().manual_seed(seed))
    lg[E] = terminal
    return lg


def step_chain(logits, B, hist, gen):
    """reference_step's ops, also returning the scores p / q and the noise."""
    A1 = logits.shape[1]
    acts = torch.stack(hist, 1) if hist else torch.empty(B, 0, dtype=torch.long)
    probs = []
    for b in range(B):
        x = logits
        if acts.shape[1] > 0:
            mask = torch.ones_like(x, dtype=torch.bool)
            mask[:, acts[b][acts[b] >= 0]] = 0
            x = x.masked_fill(~mask, float("-inf"))
        probs.append(torch.softmax(x, dim=1))
    pa = torch.stack(probs, 0)
    if B > 1:
        s = pa.sum(2)
        s[s == 0] = 1
        pa = pa / s.unsqueeze(1)
    p2 = pa.reshape(-1, A1)
    p2 = p2 / p2.sum(-1, keepdim=True)
    q = torch.empty_like(p2).exponential_(1, generator=gen)
    return p2 / q, q, acts


def softmax_bits(capability: str) -> np.ndarray:
    env = dict(os.environ, ATEN_CPU_CAPABILITY=capability)
    code = ("import sys, torch, numpy as np; sys.path.insert(0, %r); from tests.golden.near_tie_rate import c2_logits;"
            "p = torch.softmax(c2_logits().view(1, -1), 1); np.save(sys.argv[1], p.numpy());"
            "print(torch.backends.cpu.get_cpu_capability())") % os.path.dirname(os.path.dirname(HERE))
    out = f"/tmp/softmax_{capability}.npy"
    cap = subprocess.run([sys.executable, "-c", code, out], env=env, capture_output=True, text=True, check=True)
    return np.load(out), cap.stdout.strip()


def _per_entry(a, b):
    r = a.astype(np.float64).ravel() / b.astype(np.float64).ravel()
    dev = np.abs(r / np.median(r) - 1.0)
    return {"per_entry_rel_dev_after_common_scale": {"p50": float(np.percentile(dev, 50)),
                                                     "p99": float(np.percentile(dev, 99)), "max": float(dev.max()),
                                                     "frac_below_6e-8": float(np.mean(dev < 6e-8))}}


def main():
    steps_goal = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    out_path = sys.argv[2] if len(sys.argv) > 2 else None
    torch.set_num_threads(int(os.environ.get("NT_THREADS", "4")))
    logits = c2_logits().view(1, -1)
    E = logits.shape[1] - 1
    lmax = float(logits.max())
    w_all = np.exp((logits.view(-1).numpy() - np.float32(lmax)).astype(np.float32)).astype(np.float32)
    B = 2
    gen = torch.Generator().manual_seed(1234)
    n_steps = flips = traj = 0
    below = {t: 0 for t in THRESH}
    min_gap = 1.0
    t0 = time.time()
    while n_steps < steps_goal:
        hist, done = [], torch.zeros(B, dtype=torch.bool)
        traj += 1
        while not bool(done.all()) and n_steps < steps_goal:
            sc, q, acts = step_chain(logits, B, hist, gen)
            a_ref = torch.argmax(sc, dim=-1)
            for b in range(B):
                if done[b]:
                    continue
                top = torch.topk(sc[b], 2).values
                gap = float((top[0] - top[1]) / top[0])
                min_gap = min(min_gap, gap)
                for t in THRESH:
                    below[t] += gap < t
                # the kernel's form: exp(l - lmax) / q, chosen actions scored 0
                w = w_all.copy()
                if acts.shape[1]:
                    taken = acts[b][acts[b] >= 0].numpy()
                    w[taken] = 0
                s = w / q[b].numpy()
                flips += int(np.argmax(s)) != int(a_ref[b])
                n_steps += 1
            la = torch.where(done, torch.full((B,), -1), a_ref)
            hist.append(la)
            done |= a_ref == E
            if n_steps % 5000 < B:
                print(f"{n_steps} steps, {traj} trajectories, flips {flips}, below {below}, "
                      f"{time.time() - t0:.0f} s", flush=True)
    p_def, cap_def = softmax_bits("default")
    p_vec, cap_vec = softmax_bits(torch.backends.cpu.get_cpu_capability())
    res = {
        "config": "C2 256^2 Poisson, E = 326,656, G8 logits (seed 21, terminal 5.0), B = 2",
        "sample_steps": n_steps, "trajectories": traj, "flips_vs_exp_over_q": flips,
        "gap_below": {f"{t:g}": below[t] for t in THRESH}, "min_relative_gap": min_gap,
        "softmax_bits_differ_between_cpu_kernels": {
            "capabilities": [cap_def, cap_vec],
            "entries_differing": int((p_def.view(np.uint32) != p_vec.view(np.uint32)).sum()),
            "entries": int(p_def.size),
            "max_rel_diff": float(np.max(np.abs(p_def.astype(np.float64) - p_vec) / p_vec)),
            # the part that can change an argmax: per-entry deviation after the common scale
            **_per_entry(p_def, p_vec)},
        "seconds": round(time.time() - t0, 1), "torch": torch.__version__,
    }
    print(json.dumps(res, indent=1))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
