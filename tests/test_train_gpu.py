"""Training-side kernels on the MI355X through the C ABI, against the
oracle (itself pinned by the reference's logits.grad / back_probs, tests/test_train_cpu.py).

Tolerances: gradients of the logged probabilities 1e-5 relative to the largest entry (the
kernel takes the sampler's fp32 probabilities as given); LSTM fp32 recurrence vs the fp64
oracle 1e-5 relative (back_probs) / 1e-4 (BPTT weight gradients, fp64-accumulated)."""
import os

import numpy as np
import pytest
import torch

from oracle import spai_oracle as O

from .conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROLLOUTS = [f"c1_rollout_s{s}.npz" for s in range(4)]


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def tb_grad_wrt_probs(d):
    fp = torch.tensor(d["fwd_probs"], requires_grad=True)
    loss = O.trajectory_balance_loss(torch.ones(1), torch.tensor(d["rewards"]), fp, torch.tensor(d["back_probs"]))
    loss.backward()
    return fp.grad.numpy()


def removed_bitmaps(actions_bt, E):
    from gflownet_spai_amd import kernels

    return kernels.actions_to_removed(torch.as_tensor(actions_bt).to(DEV), E)[0]


def close(got, ref, rel):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    np.testing.assert_allclose(got, ref, rtol=rel, atol=rel * max(np.abs(ref).max(), 1e-30))


@pytest.mark.parametrize("name", ROLLOUTS)
def test_logp_grad_vs_reference_logits_grad(name):
    from gflownet_spai_amd import kernels

    d = load(name)
    E = d["logits"].size - 1
    acts_bt = torch.tensor(d["actions"].T.copy())
    gp = tb_grad_wrt_probs(d)
    lg = torch.tensor(d["logits"], device=DEV)
    lmax = lg.max().reshape(1)
    got = kernels.logp_grad(lg, lmax, acts_bt.to(DEV), torch.tensor(d["fwd_probs"], device=DEV),
                            torch.tensor(gp, device=DEV), removed_bitmaps(acts_bt, E)).cpu().numpy()
    close(got, O.logp_grad(d["logits"], acts_bt.numpy(), d["fwd_probs"], gp), 1e-5)
    ref = d["logits_grad"].astype(np.float64)
    np.testing.assert_allclose(got, ref, rtol=2e-4, atol=2e-6 * np.abs(ref).max())


@pytest.mark.parametrize("shared", [True, False])
def test_logp_grad_throughput_rollout_vs_oracle(shared):
    """A C2-sized throughput rollout (E = 326,656, ~65K removals per sample: many chunks),
    random upstream gradients, shared and per-sample logits."""
    from gflownet_spai_amd import kernels

    E, B = 326656, 3
    g = torch.Generator().manual_seed(11)
    lg_h = torch.randn(E + 1 if shared else (B, E + 1), generator=g)
    if shared:
        lg_h[E] = 3.5
    else:
        lg_h[:, E] = 3.5
    lg = lg_h.to(DEV)
    lgs, lmax, _ = kernels.logits_stats(lg, B)
    removed, counts, ws = kernels.rollout_select(lgs, B, lmax, 5, 2)
    acts, fwd, t_dev = kernels.rollout_order(lgs, B, lmax, counts, ws)
    T = int(t_dev)
    acts, fwd = acts[:, :T], fwd[:, :T]
    gp = torch.randn(B, T, generator=g).to(DEV)
    got = kernels.logp_grad(lg, lmax, acts, fwd, gp, removed).cpu().numpy()
    a_h, f_h, g_h = acts.cpu().numpy(), fwd.cpu().numpy(), gp.cpu().numpy()
    if shared:
        close(got, O.logp_grad(lg_h.numpy(), a_h, f_h, g_h), 1e-5)
    else:
        for b in range(B):
            close(got[b], O.logp_grad(lg_h[b].numpy(), a_h[b:b + 1], f_h[b:b + 1], g_h[b:b + 1]), 1e-5)


def test_tb_loss_gradient_through_sample_states():
    """log.fwd_probs backward (spai_logp_grad) == autograd through the fp64 torch
    restatement (log.trajectory_probs) on the same rollout."""
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv, poisson_2d
    from gflownet_spai_amd.log import trajectory_probs
    from gflownet_spai_amd.utils import trajectory_balance_loss

    A = poisson_2d(32)
    env = PreconditionerEnv(1024, A, A, side="AM", fill="lsq", device=DEV)
    E = env.num_actions - 1

    class Fixed(torch.nn.Module):
        def __init__(self):
            super().__init__()
            l = torch.randn(1, E + 1, generator=torch.Generator().manual_seed(3))
            l[0, E] = 2.0
            self.l = torch.nn.Parameter(l.to(DEV))

        def logits(self, data):
            return self.l, torch.tensor(0.5, device=DEV)

    pol = Fixed()
    model = GFlowNet(pol, None, env, mode="throughput", seed=9)
    log = model.sample_states([A] * 4, return_log=True)
    bp = torch.full_like(log.fwd_probs.detach(), 0.5)
    rewards = torch.tensor([3.0, 5.0, 7.0, 11.0], device=DEV)
    loss = trajectory_balance_loss(log.total_flow, rewards, log.fwd_probs, bp)
    loss.backward()
    got = pol.l.grad.clone()
    pol.l.grad = None
    fp = trajectory_probs(pol.l, log._actions_bt)
    trajectory_balance_loss(log.total_flow, rewards, fp, bp).backward()
    close(got.cpu().numpy(), pol.l.grad.cpu().numpy(), 1e-5)


def _lstm_case(H, B, T, lens, hi, seed):
    torch.manual_seed(seed)
    lstm = torch.nn.LSTM(1, H, batch_first=True)
    rng = np.random.default_rng(seed)
    traj = rng.integers(0, hi, size=(B, T))
    for b, n in enumerate(lens):
        traj[b, n:] = -1
    return lstm, traj


@pytest.mark.parametrize("H,hi,lens", [(2, 100, None), (4, 100, None), (8, 100, None),
                                       # action-id-sized inputs (gates saturate, a cell counts steps)
                                       (4, 5_000_000, None),
                                       # block edges of the H = 4 checkpointed path (16-step blocks)
                                       (4, 1000, [16, 15, 17, 47, 48, 49, 32, 2])])
def test_lstm_forward_backward_vs_oracle(H, hi, lens):
    from gflownet_spai_amd import kernels

    T = 3000 if lens is None else max(lens)
    lens = lens or [T, 2999, 1500, 64, 1]
    B = len(lens)
    lstm, traj = _lstm_case(H, B, T, lens, hi, H)
    P = [lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0]
    Pd = [p.detach().to(DEV) for p in P]
    tr = torch.tensor(traj, device=DEV)
    n = torch.tensor(lens, device=DEV, dtype=torch.int32)
    h, states = kernels.lstm_forward(tr, n, *Pd, keep_states=True)
    hl, _ = O.lstm_forward(traj, *(p.detach().numpy() for p in P))
    close(h.cpu().numpy(), hl, 1e-5)
    dh = np.random.default_rng(1).standard_normal((B, H))
    rows = kernels.lstm_backward(tr, n, *Pd, states, torch.tensor(dh, device=DEV, dtype=torch.float32))
    g = rows.sum(0).cpu().numpy()
    g_ih, g_hh, g_b = O.lstm_backward(traj, *(p.detach().numpy() for p in P), dh)
    R = 4 * H
    close(g[:R], g_ih.reshape(-1), 1e-4)
    close(g[R:R + R * H], g_hh.reshape(-1), 1e-4)
    close(g[R + R * H:], g_b, 1e-4)


@pytest.mark.parametrize("name", ROLLOUTS)
def test_backward_policy_vs_reference_back_probs(name):
    from gflownet_spai_amd.policy import BackwardPolicy

    d = load(name)
    B, E = int(d["B"]), d["logits"].size - 1
    torch.manual_seed(0)
    bwd = BackwardPolicy(1, 4, E + 1).to(DEV)
    bp = bwd(torch.tensor(d["actions"].T.copy(), device=DEV)).reshape(B, -1)
    np.testing.assert_allclose(bp.detach().cpu().numpy(), d["back_probs"], rtol=1e-5, atol=1e-7)


def test_backward_policy_gradients_vs_torch_lstm():
    """Every BackwardPolicy parameter gradient of sum(log back_probs) against the nn.LSTM
    restatement (torch autograd on the CPU, fp32)."""
    from gflownet_spai_amd.policy import BackwardPolicy

    B, T, E = 4, 700, 900
    torch.manual_seed(2)
    bwd = BackwardPolicy(1, 4, E + 1)
    rng = np.random.default_rng(2)
    traj = rng.integers(0, E, size=(B, T))
    for b, n in enumerate([T, 650, 300, 2]):
        traj[b, n:] = -1
    w = torch.tensor(rng.standard_normal((B, T)), dtype=torch.float32)
    (torch.log(bwd.torch_forward(torch.tensor(traj)).reshape(B, T) + 1e-9) * w).sum().backward()
    ref = {k: p.grad.clone() for k, p in bwd.named_parameters()}
    gpu = bwd.to(DEV)
    gpu.zero_grad()
    (torch.log(gpu(torch.tensor(traj, device=DEV)).reshape(B, T) + 1e-9) * w.to(DEV)).sum().backward()
    for k, p in gpu.named_parameters():
        close(p.grad.cpu().numpy(), ref[k].numpy(), 1e-4)


def test_train_step_end_to_end():
    """GFlowNet100.py's epoch on the device: HIP ForwardPolicy + BackwardPolicy, TB loss,
    Adam; the update happens, is finite, and repeats from the same state (to rounding: the
    ForwardPolicy's torch-restatement backward accumulates with atomics)."""
    from torch.optim import Adam

    from gflownet_spai_amd import BackwardPolicy, ForwardPolicy, GFlowNet, PreconditionerEnv, poisson_2d
    from gflownet_spai_amd.train import train_step

    A = poisson_2d(16)
    out = []
    for _ in range(2):
        env = PreconditionerEnv(256, A, A, side="AM", fill="lsq", device=DEV)
        E = env.num_actions - 1
        torch.manual_seed(0)
        fwd = ForwardPolicy(-1, 4, E + 1).to(DEV)
        with torch.no_grad():
            fwd.fc.bias[E] += 6.0  # short trajectories
        bwd = BackwardPolicy(1, 4, E + 1).to(DEV)
        model = GFlowNet(fwd, bwd, env, mode="throughput", seed=4)
        opt = Adam(model.parameters(), lr=1e-3)
        before = [p.detach().clone() for p in model.parameters()]
        res = [train_step(model, opt, [A] * 3) for _ in range(3)]
        after = [p.detach().clone() for p in model.parameters()]
        assert all(r.loss.isfinite() for r in res if r.updated)
        assert any(r.updated for r in res)
        assert any(not torch.equal(a, b) for a, b in zip(before, after))
        out.append((torch.stack([r.loss for r in res]).cpu(), [a.cpu() for a in after]))
    torch.testing.assert_close(out[0][0], out[1][0], rtol=1e-4, atol=1e-6)
    for a, b in zip(out[0][1], out[1][1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)
