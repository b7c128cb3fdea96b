"""Training-side oracle pinned on the CPU: the closed-form gradient of
the logged forward probabilities against the reference's own logits.grad (golden
rollouts), and the numpy LSTM forward / BPTT against the golden back_probs and torch
autograd.  The HIP kernels are compared with these in tests/test_train_gpu.py."""
import os

import numpy as np
import pytest
import torch

from oracle import spai_oracle as O

from .conftest import GOLDEN

ROLLOUTS = [f"c1_rollout_s{s}.npz" for s in range(4)]


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def tb_grad_wrt_probs(d):
    """dL/dfwd_probs of the reference TB loss at the golden rollout (torch autograd, fp32)."""
    fp = torch.tensor(d["fwd_probs"], requires_grad=True)
    loss = O.trajectory_balance_loss(torch.ones(1), torch.tensor(d["rewards"]), fp, torch.tensor(d["back_probs"]))
    loss.backward()
    return fp.grad.numpy()


@pytest.mark.parametrize("name", ROLLOUTS)
def test_logp_grad_oracle_matches_reference_logits_grad(name):
    d = load(name)
    gp = tb_grad_wrt_probs(d)
    acts_bt = d["actions"].T
    got = O.logp_grad(d["logits"], acts_bt, d["fwd_probs"], gp)
    ref = d["logits_grad"].astype(np.float64)
    np.testing.assert_allclose(got, ref, rtol=2e-4, atol=2e-6 * np.abs(ref).max())


def test_logp_grad_oracle_vs_autograd_random():
    """Against torch fp64 autograd through the per-step masked softmax (policy.py:65-73)."""
    rng = np.random.default_rng(5)
    E = 60
    l = rng.standard_normal(E + 1)
    for k in (0, 1, 7, E):
        order = rng.permutation(E)[:k].tolist() + [E]
        lt = torch.tensor(l, requires_grad=True)
        mask = torch.zeros(E + 1, dtype=torch.bool)
        ps = []
        for a in order:
            p = torch.softmax(lt.masked_fill(mask, float("-inf")), 0)[a]
            ps.append(p)
            mask = mask.clone()
            mask[a] = True
        p = torch.stack(ps)
        gp = torch.tensor(rng.standard_normal(len(order)))
        (p * gp).sum().backward()
        got = O.logp_grad(l, np.array([order]), p.detach().numpy()[None], gp.numpy()[None])
        np.testing.assert_allclose(got, lt.grad.numpy(), rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("name", ROLLOUTS)
def test_lstm_oracle_matches_reference_back_probs(name):
    from gflownet_spai_amd.policy import BackwardPolicy

    d = load(name)
    B, E = int(d["B"]), d["logits"].size - 1
    torch.manual_seed(0)  # make_golden.py: BackwardPolicy(1, 4, E + 1) under manual_seed(0)
    bwd = BackwardPolicy(1, 4, E + 1)
    L = bwd.lstm
    bp = O.backward_probs(d["actions"].T, *(t.detach().numpy() for t in (L.weight_ih_l0, L.weight_hh_l0,
                                                                          L.bias_ih_l0, L.bias_hh_l0)),
                          bwd.fc.weight.detach().numpy(), bwd.fc.bias.detach().numpy())
    np.testing.assert_allclose(bp.reshape(B, -1), d["back_probs"], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("H", [2, 4, 8])
def test_lstm_oracle_backward_vs_torch_autograd(H):
    torch.manual_seed(H)
    lstm = torch.nn.LSTM(1, H, batch_first=True).double()
    rng = np.random.default_rng(H)
    B, T = 3, 40
    traj = rng.integers(0, 50, size=(B, T))
    lens = [T, 25, 1]
    for b, n in enumerate(lens):
        traj[b, n:] = -1
    x = torch.tensor(traj, dtype=torch.float64).unsqueeze(-1)
    packed = torch.nn.utils.rnn.pack_padded_sequence(x, torch.tensor(lens), batch_first=True, enforce_sorted=False)
    _, (h, _) = lstm(packed)
    dh = torch.tensor(rng.standard_normal((B, H)))
    (h[-1] * dh).sum().backward()
    P = [lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0]
    hl, _ = O.lstm_forward(traj, *(p.detach().numpy() for p in P))
    np.testing.assert_allclose(hl, h[-1].detach().numpy(), rtol=1e-12, atol=1e-14)
    g_ih, g_hh, g_b = O.lstm_backward(traj, *(p.detach().numpy() for p in P), dh.numpy())
    np.testing.assert_allclose(g_ih, P[0].grad.numpy(), rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(g_hh, P[1].grad.numpy(), rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(g_b, P[2].grad.numpy(), rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(g_b, P[3].grad.numpy(), rtol=1e-10, atol=1e-13)


def test_backward_policy_refuses_cpu_tensors():
    from gflownet_spai_amd._lib import SpaiUnavailable
    from gflownet_spai_amd.policy import BackwardPolicy

    bwd = BackwardPolicy(1, 4, 10)
    with pytest.raises(SpaiUnavailable):
        bwd(torch.zeros(2, 3, dtype=torch.long))
