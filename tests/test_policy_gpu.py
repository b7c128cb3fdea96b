"""HIP ForwardPolicy (spai_policy_logits through the C ABI) vs the fp32 torch restatement
and the fp64 numpy oracle; gradients through the recompute backward; end to end through
GFlowNet.sample_states.

Tolerances (fp32 GATv2 with online softmax and a different summation order than the torch
reference): logits within 2e-5 relative to max|logit| (+1e-6 absolute); lmax bit-exact to
the max of the returned logits; sampled index sets bit-exact given the same logits.
"""
import numpy as np
import pytest
import torch

from gflownet_spai_amd import GFlowNet, PreconditionerEnv, poisson_2d
from gflownet_spai_amd.policy import ForwardPolicy
from gflownet_spai_amd.preconditioner import Data
from oracle import spai_oracle as O

from .test_policy_cpu import layer_params, random_graph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def close(got, ref, rel=2e-5):
    got = np.asarray(got, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    scale = max(1.0, np.abs(ref).max())
    err = np.abs(got - ref).max()
    assert err <= rel * scale + 1e-6, f"max abs err {err:.3e} (scale {scale:.3e})"


def randomise(pol, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in pol.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.5)
    return pol


@pytest.mark.parametrize("fin,hid", [(1, 4), (1, 8), (2, 16), (4, 32), (1, 32)])
def test_policy_logits_random_features(fin, hid):
    torch.manual_seed(fin * 100 + hid)
    n = 300
    ei, ea = random_graph(n // 2, 1200, seed=hid)
    x = np.random.default_rng(hid).standard_normal((n, fin)).astype(np.float32)
    pol = randomise(ForwardPolicy(fin, hid, 1500), fin + hid).to(DEV)
    data = Data(x=torch.from_numpy(x).to(DEV), edge_index=torch.from_numpy(ei).to(DEV),
                edge_attr=torch.from_numpy(ea).to(DEV))
    with torch.no_grad():
        got, a, lmax = pol.logits_and_max(data, 3)
        ref, a_ref = pol.torch_logits(data)
    assert got.shape == (1, 1201)
    close(got.cpu(), ref.cpu())
    assert torch.equal(lmax.cpu(), got.max().cpu().repeat(3))
    assert float(a) == float(a_ref)
    orc = O.forward_policy_logits(x, ei, ea, layer_params(pol.gat1.cpu().double()),
                                  layer_params(pol.gat2.cpu().double()), pol.fc.weight.detach().cpu().numpy(),
                                  pol.fc.bias.detach().cpu().numpy(), 1201)
    close(got.cpu(), orc)


@pytest.mark.parametrize("grid,fast", [(16, True), (256, True), (16, False), (256, False)])
def test_policy_logits_state_graph(grid, fast):
    """The reference's own input: state_to_data's x = ones(2N, 1) over A's raw COO pattern,
    through the constant-row closed form (fast) and through the general GATv2 kernels."""
    A = poisson_2d(grid)
    n = grid * grid
    E = A._nnz()
    pol = randomise(ForwardPolicy(-1, 4, E + 7), grid).to(DEV)
    pol.const_fast_path = fast
    data = Data(x=torch.ones(2 * n, 1, device=DEV), edge_index=A._indices().to(DEV),
                edge_attr=A._values().float().to(DEV))
    with torch.no_grad():
        got, _, lmax = pol.logits_and_max(data, 2)
        ref, _ = pol.torch_logits(data)
    assert pol.rows_constant(data.x)
    close(got.cpu(), ref.cpu())
    assert float(lmax[0]) == float(got.max())
    # known answer: with x = ones the pooled embedding is graph-independent
    p1 = layer_params(pol.gat1.cpu().double())
    h1 = np.maximum(O.gatv2_layer_ones_answer(p1["W_l"], p1["b_l"], p1["bias"], 1), 0.0)
    p2 = layer_params(pol.gat2.cpu().double())
    h2 = np.maximum(h1 @ p2["W_l"].T + p2["b_l"] + p2["bias"], 0.0)
    lg = pol.fc.weight.detach().cpu().double().numpy()[:E + 1] @ h2[0] + pol.fc.bias.detach().cpu().double().numpy()[:E + 1]
    close(got.cpu(), lg)


@pytest.mark.parametrize("fin,hid", [(1, 4), (2, 8), (4, 4), (1, 16)])
def test_policy_gradients_match_torch(fin, hid):
    """spai_policy_backward (hid 4, 8) and the torch-restatement path (hid 16) against autograd
    through the torch restatement of the same network."""
    torch.manual_seed(3)
    n = 200
    ei, ea = random_graph(n // 2, 700, seed=3)
    x = torch.randn(n, fin)
    pol = randomise(ForwardPolicy(fin, hid, 800), 11).to(DEV)
    data = Data(x=x.to(DEV), edge_index=torch.from_numpy(ei).to(DEV), edge_attr=torch.from_numpy(ea).to(DEV))
    assert pol._hip_backward_ok(data) == (hid in (4, 8))
    w = torch.randn(1, 701, device=DEV)
    lg, a, _ = pol.logits_and_max(data)
    ((lg * w).sum() + a).backward()
    got = {k: p.grad.clone() for k, p in pol.named_parameters()}
    pol.zero_grad()
    lg2, a2 = pol.torch_logits(data)
    ((lg2 * w).sum() + a2).backward()
    for k, p in pol.named_parameters():
        if p.grad is None:
            assert got[k] is None or float(got[k].abs().max()) == 0.0
            continue
        close(got[k].cpu(), p.grad.cpu(), rel=1e-4)


def test_sample_states_with_forward_policy():
    """End to end: HIP policy -> throughput rollout (lmax from the policy kernels) ->
    LSQ fill -> reward; trajectories bit-exact vs the oracle given the policy's logits."""
    A = poisson_2d(16)
    env = PreconditionerEnv(256, A, A, side="AM", fill="lsq", keep_m=True)
    E = env.num_actions - 1
    pol = randomise(ForwardPolicy(-1, 4, E + 1), 5).to(DEV)
    with torch.no_grad():
        pol.fc.bias[E] += 2.0
    g = GFlowNet(pol, None, env, mode="throughput", seed=9)
    log = g.sample_states([A] * 3, return_log=True)
    data = g.state_to_data([A])[0]
    with torch.no_grad():
        lg, _ = pol.logits(data)
    r_o, a_o, f_o, c_o = O.throughput_rollout(lg.cpu().numpy().reshape(-1), 3, 9, 0)
    assert np.array_equal(log.actions.cpu().numpy(), a_o)
    assert np.array_equal(log.counts.cpu().numpy(), c_o)
    np.testing.assert_allclose(log.fwd_probs.detach().cpu().numpy(), f_o, rtol=1e-6)
    # the differentiable probabilities reach the policy parameters
    loss = torch.log(log.fwd_probs).sum()
    loss.backward()
    assert pol.fc.weight.grad is not None and float(pol.fc.weight.grad.abs().sum()) > 0


def lp(layer):
    import copy
    return layer_params(copy.deepcopy(layer).cpu().double())


@pytest.mark.parametrize("fin,hid", [(1, 4), (2, 8), (4, 16), (1, 32)])
def test_policy_const_rows_closed_form_matches_general(fin, hid):
    """Identical non-unit rows (x = c for every node): the closed form and the general kernels
    agree with each other and with the fp64 oracle; a single differing row is detected and
    takes the general kernels."""
    n = 400
    ei, ea = random_graph(n // 2, 1500, seed=fin + hid)
    row = np.random.default_rng(hid).standard_normal(fin).astype(np.float32)
    x = np.tile(row, (n, 1))
    pol = randomise(ForwardPolicy(fin, hid, 1700), 7 * hid).to(DEV)
    data = Data(x=torch.from_numpy(x).to(DEV), edge_index=torch.from_numpy(ei).to(DEV),
                edge_attr=torch.from_numpy(ea).to(DEV))
    outs = []
    for fast in (True, False):
        pol.const_fast_path = fast
        with torch.no_grad():
            got, _, lmax = pol.logits_and_max(data, 2)
        assert float(lmax[1]) == float(got.max())
        outs.append(got.cpu())
    assert pol.rows_constant(data.x)
    close(outs[0], outs[1])
    orc = O.forward_policy_logits(x, ei, ea, lp(pol.gat1),
                                  lp(pol.gat2), pol.fc.weight.detach().cpu().numpy(),
                                  pol.fc.bias.detach().cpu().numpy(), 1501)
    close(outs[0], orc)
    # one row differs -> not constant (re-checked after the in-place change), general path
    pol.const_fast_path = True
    with torch.no_grad():
        data.x[n - 1, 0] += 1.0
    assert not pol.rows_constant(data.x)
    x2 = data.x.cpu().numpy()
    with torch.no_grad():
        got, _, _ = pol.logits_and_max(data, 1)
    orc2 = O.forward_policy_logits(x2, ei, ea, lp(pol.gat1),
                                   lp(pol.gat2), pol.fc.weight.detach().cpu().numpy(),
                                   pol.fc.bias.detach().cpu().numpy(), 1501)
    close(got.cpu(), orc2)


@pytest.mark.parametrize("grid", [16, 256])
def test_deferred_max_in_select(grid):
    """The logits maximum deferred to the rollout (spai_policy_logits with B = 0 leaves the fc block
    maxima; spai_rollout_select_pm reduces them in an extra block of its first launch): the same
    lmax as the policy's own reduction and bit-identical select outputs; a no-grad sample_states
    (which defers) matches the oracle."""
    from gflownet_spai_amd import kernels
    A = poisson_2d(grid)
    env = PreconditionerEnv(grid * grid, A, A, side="AM", fill="lsq")
    E = env.num_actions - 1
    pol = randomise(ForwardPolicy(-1, 4, E + 1), grid).to(DEV)
    with torch.no_grad():
        pol.fc.bias[E] += 2.0
    g = GFlowNet(pol, None, env, mode="throughput", seed=5)
    data = g.state_to_data([A])[0]
    with torch.no_grad():
        lg, _, lmax = pol.logits_and_max(data, 3)
        lg2, _, pend = pol.logits_and_max(data, 3, defer_max=True)
        assert isinstance(pend, kernels.PendingMax) and torch.equal(lg, lg2)
        r1, c1, _ = kernels.rollout_select(lg.reshape(-1), 3, lmax, 5, 7)
        r1, c1 = r1.clone(), c1.clone()
        r2, c2, _ = kernels.rollout_select(lg2.reshape(-1), 3, pend, 5, 7)
        assert torch.equal(pend.out, lmax) and float(lmax[0]) == float(lg.max())
        assert torch.equal(r1, r2) and torch.equal(c1, c2)
        log = g.sample_states([A] * 3, return_log=True)
    r_o, a_o, f_o, c_o = O.throughput_rollout(lg.cpu().numpy().reshape(-1), 3, 5, 0)
    assert np.array_equal(log.actions.cpu().numpy(), a_o) and np.array_equal(log.counts.cpu().numpy(), c_o)
    np.testing.assert_allclose(log.fwd_probs.detach().cpu().numpy(), f_o, rtol=1e-6)
