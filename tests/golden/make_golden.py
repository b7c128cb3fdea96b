"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Runs ONLY in the build container, where the read-only reference lives at
/root/reference.  It never runs on the GPU box and nothing it imports is copied
into the repository: the committed fixtures are data only (inputs + the
reference's outputs).

How the reference is made importable: every hot-path module
imports ``torch_geometric`` at top level, which is not installed and cannot be
fetched.  ``preconditioner.py`` and ``gflownet/*`` use ``torch_geometric.data.Data``
purely as a keyword attribute bag (``preconditioner.py:25``,
``gflownet/gflownet.py:248``, ``gflownet/utils.py:311``), so a probe-only bag is
placed on ``sys.path`` from a temp dir.  ``torch_geometric.nn`` gets placeholders
that raise if used: the GATv2 ``ForwardPolicy`` is NOT exercised (its numerics
are "parity unpinned").  All arithmetic captured below is the reference's own
code running on torch ATen.

Harness-side workarounds for the reference's latent bugs:
  * ``evaluate_preconditioner`` reads ``self.alpha`` (never set): ``update`` is
    wrapped to set ``env.alpha = alpha`` from its argument first.
  * B >= 2 only (``gflownet.py:121`` UnboundLocalError at B == 1).
  * fp32 matrices only (``utils.py:350`` forces M to fp32).
  * ``gc.collect`` is patched to a no-op for speed (no numeric effect).
  * the policy is a stand-in with ``ForwardPolicy.forward``'s contract
    (``policy.py:34-73`` after the fc): fixed logits -> masked_fill(-inf) on the
    action history -> softmax, plus sigmoid(alpha).  Valid because the
    reference's logits are state-independent within a rollout.

Usage:  python tests/golden/make_golden.py            (writes *.npz + meta.json)
        python tests/golden/make_golden.py g6         (C2/C4 parity rollouts, appended)
        python tests/golden/make_golden.py g7         (C1 assembled M of three removal sets, appended)
        python tests/golden/make_golden.py g8         (C2 long parity rollout, T > 1000, appended)
        python tests/golden/make_golden.py g9         (72^2 parity rollout with T >= 20000, appended)
"""
import gc
import json
import os
import sys
import tempfile
import time

import numpy as np
import scipy.sparse as sp
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _import_reference():
    d = tempfile.mkdtemp(prefix="pyg_probe_")
    os.makedirs(os.path.join(d, "torch_geometric"))
    with open(os.path.join(d, "torch_geometric", "__init__.py"), "w") as f:
        f.write("")
    with open(os.path.join(d, "torch_geometric", "data.py"), "w") as f:
        f.write("class Data:\n"
                "    def __init__(self, **kw):\n"
                "        self.__dict__.update(kw)\n"
                "    def __contains__(self, k):\n"
                "        return k in self.__dict__\n")
    with open(os.path.join(d, "torch_geometric", "nn.py"), "w") as f:
        f.write("class GATv2Conv:\n"
                "    def __init__(self, *a, **k):\n"
                "        raise NotImplementedError('probe stub')\n"
                "def global_mean_pool(*a, **k):\n"
                "    raise NotImplementedError('probe stub')\n")
    sys.path[:0] = [d, REF]
    import preconditioner  # noqa: E402
    import policy  # noqa: E402
    from gflownet import gflownet as gfn_mod  # noqa: E402
    from gflownet import utils as ref_utils  # noqa: E402
    gc.collect = lambda *a, **k: 0
    return preconditioner, policy, gfn_mod, ref_utils


def poisson2d(n, dtype=np.float32):
    t = sp.diags([-np.ones(n - 1), 2 * np.ones(n), -np.ones(n - 1)], [-1, 0, 1])
    i = sp.identity(n)
    return (sp.kron(i, t) + sp.kron(t, i)).tocoo().astype(dtype)


def to_torch_coo(rows, cols, vals, n, coalesce=False):
    t = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cols]).astype(np.int64)),
                                torch.from_numpy(vals), (n, n))
    return t.coalesce() if coalesce else t


class FixedLogitPolicy(torch.nn.Module):
    """Stand-in with ForwardPolicy.forward's call contract (policy.py:34-73)."""

    def __init__(self, logits):
        super().__init__()
        self.logits = torch.nn.Parameter(logits.view(1, -1).clone())
        self.alpha = torch.nn.Parameter(torch.tensor(0.0))

    def forward(self, data, actions):
        x = self.logits
        if actions.numel() > 0:
            mask = torch.ones_like(x, dtype=torch.bool)
            mask[:, actions] = 0
            x = x.masked_fill(~mask, float("-inf"))
        return torch.softmax(x, dim=1), torch.sigmoid(self.alpha)


def make_env(preconditioner, A_t, n):
    env = preconditioner.PreconditionerEnv(matrix_size=n, initial_matrix=A_t, original_matrix=A_t)
    orig_update = env.update

    def update(s, actions, alpha):
        env.alpha = alpha  # SURVEY §0.7a workaround: use the passed alpha
        return orig_update(s, actions, alpha)

    env.update = update
    return env


def removal_case(preconditioner, ref_utils, env, n, removed_ids, alphas):
    """Reference pattern->M (utils.py:295-356) and residual/reward (preconditioner.py:55-165)."""
    acts = [torch.tensor(int(a)) for a in removed_ids]
    M = ref_utils.update_edges_and_convert_to_sparse(env.data, acts, n)
    M = ref_utils.resize_sparse_tensor(M, (n, n))
    r_ma = env.calculate_residual(M, env.original_matrix)
    r_mta = env.calculate_residual(M.t().coalesce(), env.original_matrix)
    rewards = []
    for a in alphas:
        env.alpha = torch.tensor(a, dtype=torch.float32)
        rewards.append(float(env.reward(M, len(removed_ids), env.alpha)))
    return float(r_ma), float(r_mta), M._nnz(), rewards


def main():
    preconditioner, policy, gfn_mod, ref_utils = _import_reference()
    meta = {"torch": torch.__version__, "numpy": np.__version__,
            "generated": time.strftime("%Y-%m-%d"), "cases": {}}
    rng = np.random.default_rng(20241024)
    alphas = [0.5, 0.3]

    # ---------------- G1 + G3: C1 (16x16 grid) env + removal sets ----------------
    for tag, permute in (("c1", False), ("c1p", True)):
        A = poisson2d(16)
        rows, cols, vals = A.row.astype(np.int64), A.col.astype(np.int64), A.data.astype(np.float32)
        # row-major (coalesced) order, optionally a random raw order (action id = raw position)
        order = np.lexsort((cols, rows))
        if permute:
            order = rng.permutation(order)
        rows, cols, vals = rows[order], cols[order], vals[order]
        n = 256
        A_t = to_torch_coo(rows, cols, vals, n)
        env = make_env(preconditioner, A_t, n)
        E = env.num_actions - 1
        sets = [np.zeros(0, np.int64), np.arange(E, dtype=np.int64), np.array([0]), np.array([E - 1])]
        for k in (1, 2, 5, 17, 60, 200, 600, 1000, 1200):
            for _ in range(3):
                sets.append(np.sort(rng.choice(E, size=k, replace=False)).astype(np.int64))
        recs = [removal_case(preconditioner, ref_utils, env, n, s, alphas) for s in sets]
        removed = np.zeros((len(sets), E), np.bool_)
        for i, s in enumerate(sets):
            removed[i, s] = True
        np.savez_compressed(os.path.join(HERE, f"{tag}_removal.npz"),
                            rows=rows, cols=cols, vals=vals, n=n,
                            num_actions=env.num_actions, r0=float(env.orig_residual),
                            f0=env.orig_flops, removed=removed,
                            r_ma=np.array([r[0] for r in recs]), r_mta=np.array([r[1] for r in recs]),
                            nnz_m=np.array([r[2] for r in recs]),
                            reward=np.array([r[3] for r in recs]), alphas=np.array(alphas))
        meta["cases"][f"{tag}_removal"] = {"n": n, "E": E, "sets": len(sets), "permuted_raw_order": permute}
        print(tag, "r0", float(env.orig_residual), "E", E)

    # ---------------- G5: random non-symmetric fp32 matrix (non-integer arithmetic) ----------------
    n = 64
    R = sp.random(n, n, density=0.08, random_state=7, format="coo", dtype=np.float64)
    R = (R + sp.identity(n) * 2.0).tocoo()
    R.data = (rng.standard_normal(R.nnz) * 0.7).astype(np.float32)
    order = rng.permutation(R.nnz)
    rows, cols, vals = R.row[order].astype(np.int64), R.col[order].astype(np.int64), R.data[order].astype(np.float32)
    A_t = to_torch_coo(rows, cols, vals, n)
    env = make_env(preconditioner, A_t, n)
    E = env.num_actions - 1
    sets = [np.zeros(0, np.int64)] + [np.sort(rng.choice(E, size=k, replace=False)) for k in (1, 3, 10, 40, 100, E - 5)]
    recs = [removal_case(preconditioner, ref_utils, env, n, s, alphas) for s in sets]
    removed = np.zeros((len(sets), E), np.bool_)
    for i, s in enumerate(sets):
        removed[i, s] = True
    np.savez_compressed(os.path.join(HERE, "rand64_removal.npz"),
                        rows=rows, cols=cols, vals=vals, n=n, num_actions=env.num_actions,
                        r0=float(env.orig_residual), f0=env.orig_flops, removed=removed,
                        r_ma=np.array([r[0] for r in recs]), r_mta=np.array([r[1] for r in recs]),
                        nnz_m=np.array([r[2] for r in recs]), reward=np.array([r[3] for r in recs]),
                        alphas=np.array(alphas))
    meta["cases"]["rand64_removal"] = {"n": n, "E": E, "sets": len(sets)}

    # ---------------- G2: C1 rollouts through GFlowNet.sample_states ----------------
    A = poisson2d(16)
    order = np.lexsort((A.col, A.row))
    rows, cols, vals = A.row[order].astype(np.int64), A.col[order].astype(np.int64), A.data[order].astype(np.float32)
    n = 256
    A_t = to_torch_coo(rows, cols, vals, n)
    for seed, term_logit, B in ((0, 4.0, 4), (1, 4.0, 4), (2, 6.0, 3), (3, 2.5, 2)):
        env = make_env(preconditioner, A_t, n)
        E = env.num_actions - 1
        g = torch.Generator().manual_seed(123 + seed)
        logits = torch.randn(E + 1, generator=g)
        logits[E] = term_logit
        fwd = FixedLogitPolicy(logits)
        torch.manual_seed(0)
        bwd = policy.BackwardPolicy(1, 4, E + 1)
        model = gfn_mod.GFlowNet(fwd, bwd, env)
        s0 = [A_t.clone() for _ in range(B)]
        torch.manual_seed(seed)
        t0 = time.time()
        lg = model.sample_states(s0, return_log=True)
        dt = time.time() - t0
        loss = ref_utils.trajectory_balance_loss(lg.total_flow, lg.rewards, lg.fwd_probs, lg.back_probs)
        loss.backward()
        np.savez_compressed(os.path.join(HERE, f"c1_rollout_s{seed}.npz"),
                            rows=rows, cols=cols, vals=vals, n=n, logits=logits.numpy(), seed=seed, B=B,
                            actions=lg.actions.numpy(), fwd_probs=lg.fwd_probs.detach().numpy(),
                            rewards=lg.rewards.numpy(), back_probs=lg.back_probs.detach().numpy(),
                            loss=float(loss), logits_grad=fwd.logits.grad.view(-1).numpy(),
                            alpha_grad=0.0 if fwd.alpha.grad is None else float(fwd.alpha.grad))
        meta["cases"][f"c1_rollout_s{seed}"] = {"B": B, "T": int(lg.actions.shape[0]),
                                               "terminal_logit": term_logit, "loss": float(loss),
                                               "seconds": round(dt, 3)}
        print("rollout", seed, "T", lg.actions.shape[0], "loss", float(loss), "rewards", lg.rewards.tolist())

    # ---------------- G4: C2 / C4 single-candidate residuals (recipe-regenerable removal sets) ----------------
    for tag, grid, fracs in (("c2", 256, (0.0, 0.05, 0.2)), ("c4", 1024, (0.2,))):
        A = poisson2d(grid)
        order = np.lexsort((A.col, A.row))
        rows, cols, vals = A.row[order].astype(np.int64), A.col[order].astype(np.int64), A.data[order].astype(np.float32)
        n = grid * grid
        A_t = to_torch_coo(rows, cols, vals, n)
        t0 = time.time()
        env = make_env(preconditioner, A_t, n)
        t_init = time.time() - t0
        E = env.num_actions - 1
        out = {"n": n, "E": E, "r0": float(env.orig_residual), "f0": env.orig_flops,
               "env_init_s": round(t_init, 3), "sets": []}
        for k, frac in enumerate(fracs):
            removed = np.flatnonzero(np.random.default_rng(1000 + k).random(E) < frac)
            t0 = time.time()
            r_ma, r_mta, nnz_m, rew = removal_case(preconditioner, ref_utils, env, n, removed, alphas)
            out["sets"].append({"recipe": f"np.random.default_rng({1000 + k}).random(E) < {frac}",
                                "n_removed": int(removed.size), "r_ma": r_ma, "r_mta": r_mta,
                                "nnz_m": nnz_m, "reward": rew, "seconds": round(time.time() - t0, 3)})
        meta["cases"][f"{tag}_residual"] = out
        print(tag, json.dumps(out)[:400])

    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


def parity_rollouts_large():
    """G6: reference rollouts at C2 (256^2) and C4 (1024^2) through GFlowNet.sample_states.

    Terminal-biased fixed logits keep T small (the reference loop costs a policy call and a
    [B, E+1] multinomial per step).  Stored: the recipe of the logits (regenerable from the
    seed), the torch seed of the rollout (the sampler's Exp(1) noise is regenerable from it),
    and the reference's actions, fwd_probs and rewards.  Appends to meta.json."""
    preconditioner, policy, gfn_mod, ref_utils = _import_reference()
    meta_path = os.path.join(HERE, "meta.json")
    meta = json.load(open(meta_path))
    for tag, grid, logit_seed, term_logit, seed, B in (("c2", 256, 7, 11.5, 11, 2), ("c4", 1024, 8, 14.2, 12, 2)):
        A = poisson2d(grid)
        order = np.lexsort((A.col, A.row))
        rows, cols, vals = A.row[order].astype(np.int64), A.col[order].astype(np.int64), A.data[order].astype(np.float32)
        n = grid * grid
        A_t = to_torch_coo(rows, cols, vals, n)
        env = make_env(preconditioner, A_t, n)
        E = env.num_actions - 1
        logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(logit_seed))
        logits[E] = term_logit
        model = gfn_mod.GFlowNet(FixedLogitPolicy(logits), None, env)
        s0 = [A_t.clone() for _ in range(B)]
        torch.manual_seed(seed)
        t0 = time.time()
        lg = model.sample_states(s0, return_log=True)
        dt = time.time() - t0
        np.savez_compressed(os.path.join(HERE, f"{tag}_rollout.npz"), grid=grid, logit_seed=logit_seed,
                            terminal_logit=term_logit, seed=seed, B=B, actions=lg.actions.numpy(),
                            fwd_probs=lg.fwd_probs.detach().numpy(), rewards=lg.rewards.numpy())
        meta["cases"][f"{tag}_rollout"] = {
            "B": B, "T": int(lg.actions.shape[0]), "E": E, "grid": grid,
            "logits": f"torch.randn(E + 1, generator=torch.Generator().manual_seed({logit_seed})); [E] = {term_logit}",
            "rollout_seed": f"torch.manual_seed({seed}) before sample_states", "seconds": round(dt, 3)}
        print(tag, "T", lg.actions.shape[0], "rewards", lg.rewards.tolist(), "s", round(dt, 1))
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1)


def parity_rollout_long():
    """G8: a LONG reference rollout at C2 (256^2, E = 326,656) through GFlowNet.sample_states:
    the terminal logit is set so that a sample stops with probability ~2.8e-4 per step (T > 1,000 steps
    of the reference's fp32 masked softmax -> renormalisation -> Categorical chain
    (policy.py:65-73, gflownet.py:116-119,148), B = 2.  Stored like G6.  Appends to meta.json."""
    preconditioner, policy, gfn_mod, ref_utils = _import_reference()
    meta_path = os.path.join(HERE, "meta.json")
    meta = json.load(open(meta_path))
    tag, grid, logit_seed, term_logit, seed, B = "c2long", 256, 21, 5.0, 31, 2
    A = poisson2d(grid)
    order = np.lexsort((A.col, A.row))
    rows, cols, vals = A.row[order].astype(np.int64), A.col[order].astype(np.int64), A.data[order].astype(np.float32)
    n = grid * grid
    A_t = to_torch_coo(rows, cols, vals, n)
    env = make_env(preconditioner, A_t, n)
    E = env.num_actions - 1
    logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(logit_seed))
    logits[E] = term_logit
    model = gfn_mod.GFlowNet(FixedLogitPolicy(logits), None, env)
    s0 = [A_t.clone() for _ in range(B)]
    torch.manual_seed(seed)
    t0 = time.time()
    lg = model.sample_states(s0, return_log=True)
    dt = time.time() - t0
    np.savez_compressed(os.path.join(HERE, f"{tag}_rollout.npz"), grid=grid, logit_seed=logit_seed,
                        terminal_logit=term_logit, seed=seed, B=B, actions=lg.actions.numpy(),
                        fwd_probs=lg.fwd_probs.detach().numpy(), rewards=lg.rewards.numpy())
    meta["cases"][f"{tag}_rollout"] = {
        "B": B, "T": int(lg.actions.shape[0]), "E": E, "grid": grid,
        "logits": f"torch.randn(E + 1, generator=torch.Generator().manual_seed({logit_seed})); [E] = {term_logit}",
        "rollout_seed": f"torch.manual_seed({seed}) before sample_states", "seconds": round(dt, 3),
        "cpu": torch.backends.cpu.get_cpu_capability()}
    print(tag, "T", lg.actions.shape[0], "rewards", lg.rewards.tolist(), "s", round(dt, 1))
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1)


def parity_rollout_longer(terminal=-6.0, seed=41, min_t=20000, grid=72, B=2):
    """G9: a reference rollout at least ``min_t`` steps long (pin parity mode past
    T = 2e4), stored like G8.  On C2 (256^2, E = 326,656) the reference keeps every step's state
    and evaluates the residual per step: the first attempt held 15.5 GB after 2 h without
    finishing a draw (T = 2e4 would need ~80 GB), so the long draw runs on the 72^2 Poisson
    matrix (E = 25,632) with the terminal logit at -6, which removes most of the actions before
    it stops.  If the draw is shorter than ``min_t`` the next seed is tried.  Appends to
    meta.json."""
    preconditioner, policy, gfn_mod, ref_utils = _import_reference()
    meta_path = os.path.join(HERE, "meta.json")
    meta = json.load(open(meta_path))
    tag, logit_seed = "longer", 21
    A = poisson2d(grid)
    order = np.lexsort((A.col, A.row))
    rows, cols, vals = A.row[order].astype(np.int64), A.col[order].astype(np.int64), A.data[order].astype(np.float32)
    n = grid * grid
    A_t = to_torch_coo(rows, cols, vals, n)
    env = make_env(preconditioner, A_t, n)
    E = env.num_actions - 1
    logits = torch.randn(E + 1, generator=torch.Generator().manual_seed(logit_seed))
    logits[E] = terminal
    while True:
        model = gfn_mod.GFlowNet(FixedLogitPolicy(logits), None, env)
        s0 = [A_t.clone() for _ in range(B)]
        torch.manual_seed(seed)
        t0 = time.time()
        with torch.no_grad():  # values only: without it every step's autograd graph ([B, E+1] tensors) is kept
            lg = model.sample_states(s0, return_log=True)
        dt = time.time() - t0
        T = int(lg.actions.shape[0])
        print(tag, "seed", seed, "T", T, "s", round(dt, 1), flush=True)
        if T >= min_t:
            break
        seed += 1
    np.savez_compressed(os.path.join(HERE, f"{tag}_rollout.npz"), grid=grid, logit_seed=logit_seed,
                        terminal_logit=terminal, seed=seed, B=B, actions=lg.actions.numpy(),
                        fwd_probs=lg.fwd_probs.detach().numpy(), rewards=lg.rewards.numpy())
    meta["cases"][f"{tag}_rollout"] = {
        "B": B, "T": T, "E": E, "grid": grid,
        "logits": f"torch.randn(E + 1, generator=torch.Generator().manual_seed({logit_seed})); [E] = {terminal}",
        "rollout_seed": f"torch.manual_seed({seed}) before sample_states", "seconds": round(dt, 3),
        "cpu": torch.backends.cpu.get_cpu_capability()}
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1)


def assembled_m():
    """G7: the reference's M (update_edges_and_convert_to_sparse + resize_sparse_tensor,
    utils.py:295-356, 89-126) for three removal sets of the permuted-raw-order C1 pattern
    (c1p_removal.npz sets 2, 5, 20): coalesced indices and values, concatenated."""
    preconditioner, policy, gfn_mod, ref_utils = _import_reference()
    d = np.load(os.path.join(HERE, "c1p_removal.npz"))
    n = int(d["n"])
    A_t = to_torch_coo(d["rows"], d["cols"], d["vals"], n)
    env = make_env(preconditioner, A_t, n)
    sets, idx, vals, nnz = [2, 5, 20], [], [], []
    for k in sets:
        acts = [torch.tensor(int(a)) for a in np.flatnonzero(d["removed"][k])]
        M = ref_utils.resize_sparse_tensor(ref_utils.update_edges_and_convert_to_sparse(env.data, acts, n), (n, n))
        M = M.coalesce()
        idx.append(M.indices().numpy())
        vals.append(M.values().numpy())
        nnz.append(M._nnz())
    np.savez_compressed(os.path.join(HERE, "c1p_assembled.npz"), sets=np.array(sets), nnz=np.array(nnz),
                        indices=np.concatenate(idx, 1), values=np.concatenate(vals))
    meta_path = os.path.join(HERE, "meta.json")
    meta = json.load(open(meta_path))
    meta["cases"]["c1p_assembled"] = {"removal_sets": sets, "nnz": nnz, "dtype": str(vals[0].dtype)}
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1)
    print("assembled", nnz)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "g6":
        parity_rollouts_large()
    elif len(sys.argv) > 1 and sys.argv[1] == "g7":
        assembled_m()
    elif len(sys.argv) > 1 and sys.argv[1] == "g8":
        parity_rollout_long()
    elif len(sys.argv) > 1 and sys.argv[1] == "g9":
        parity_rollout_longer()
    else:
        main()
