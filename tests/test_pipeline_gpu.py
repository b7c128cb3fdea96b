"""Pipelined throughput steps (GFlowNet(pipeline=True), bench.py --pipeline): consecutive steps on
two alternating stream lanes, step k+1's policy and select beside step k's sort, fill and padding.
Every step must produce exactly the bits of the same step run alone: the same Philox stream id,
the same trajectories, step probabilities, rewards and M.  Checked eagerly step by step and
through bench.py's multi-step HIP graphs (the last timed step, dumped and recomputed).
Reference loop being pipelined: gflownet/gflownet.py:125-197 (one sample_states call per step).
"""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _setup(cfg, fill):
    import bench
    from gflownet_spai_amd import PreconditionerEnv
    A, P = bench.config_matrices(cfg)
    dev = torch.device("cuda", 0)
    env = PreconditionerEnv(A.shape[0], P, A, side="AM", fill=fill, keep_m=True, device=dev)
    return bench, env, P, dev


@pytest.mark.parametrize("fill", ["qr", "lsq"])
def test_pipelined_steps_bit_identical_to_sequential(fill):
    from gflownet_spai_amd import GFlowNet
    bench, env, P, dev = _setup("c2", fill)
    pol = bench.make_policy(env, P, dev)
    nsteps = 5
    with torch.no_grad():
        seq = GFlowNet(pol, None, env, mode="throughput", seed=99)
        ref = []
        for _ in range(nsteps):
            log = seq.sample_states([P] * 8, return_log=True)
            torch.cuda.synchronize()
            ref.append((log.actions.clone(), log.fwd_probs.clone(), log.rewards_all.clone(), env.last_m.clone()))
        pl = GFlowNet(pol, None, env, mode="throughput", seed=99, pipeline=True)
        logs = []
        for _ in range(nsteps):
            log = pl.sample_states([P] * 8, return_log=True)
            logs.append((log, env.last_m))
        pl.pipeline_join()
        torch.cuda.synchronize()
    assert pl.rollouts == seq.rollouts == nsteps
    for (a, f, r, m), (log, lm) in zip(ref, logs):
        assert torch.equal(log.actions, a)
        assert torch.equal(log.fwd_probs, f)
        assert torch.equal(log.rewards_all, r)
        assert torch.equal(lm, m)


def test_bench_pipelined_graph_step_matches_sequential(tmp_path):
    dump = tmp_path / "pl.pt"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c2", "--pipeline", "--steps", "10",
           "--steps-per-graph", "5", "--warmup", "2", "--no-cpu-baseline", "--dump", str(dump)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["pipeline"] is True and line["steps_per_graph"] == 5
    d = torch.load(dump, weights_only=True)
    from gflownet_spai_amd import GFlowNet
    bench, env, P, dev = _setup("c2", "qr")
    with torch.no_grad():
        model = GFlowNet(bench.make_policy(env, P, dev), None, env, mode="throughput", seed=1234)
        model.rollouts = int(d["stream_id"])
        log = model.sample_states([P] * 8, return_log=True)
    assert torch.equal(log.rewards_all.double().cpu(), d["rewards_all"])
    assert torch.equal(env.last_residual.double().cpu(), d["residual"])
