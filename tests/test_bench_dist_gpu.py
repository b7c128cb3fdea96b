"""The multi-GPU columns step as bench.py runs it, through RCCL, on the one GPU of the box.

Two ranks cannot share one GPU under RCCL (its duplicate-GPU check), so the
multi-rank exchange itself first runs on the driver's 8-GPU node.  What one GPU can run is the
WHOLE columns-split step of bench.py on a one-rank RCCL group (``--gpus 1 --dist --backend
nccl``): the line-major packed bitmap all_to_all issued asynchronously beside rollout_sort, the
graph segments captured between the eager collectives, the exact limb all_reduce, and the
pipelined M all_gather (LineGather) still in flight when the next step's graph replays.  The bench
is launched as a fresh child process (its own HIP context and process group) and dumps its last
step; this test recomputes that step with the one-GPU product path (same seed, same Philox
stream id) and requires the rewards of every candidate and the assembled M bit for bit.
Reference loops being split: gflownet/gflownet.py:135-183, preconditioner.py:37-51.
"""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("fill", ["qr", "lsq"])
def test_bench_columns_step_under_rccl_matches_one_gpu(tmp_path, fill):
    dump = tmp_path / f"dist_{fill}.pt"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c2", "--gpus", "1", "--dist", "--backend",
           "nccl", "--fill", fill, "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--dump", str(dump)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    # the bench line explains the multi-GPU step: the collective phases (max over ranks), the group, RCCL
    import json
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["world_size"] == 1 and line["backend"] == "nccl" and line["rccl_version"]
    col = line["collectives_ms"]
    for k in ("bitmap_all_to_all_issue", "bitmap_all_to_all_wait", "limb_all_reduce", "line_gather_wait"):
        assert k in col and col[k] >= 0.0, (k, col)
    assert set(line["phases_ms_max_over_ranks"]) == set(line["phases_ms"])
    d = torch.load(dump, weights_only=True)
    assert d["shard"] == "columns" and d["world"] == 1 and "m_assembled" in d

    sys.path.insert(0, ROOT)
    import bench
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv
    A, P = bench.config_matrices("c2")
    n = A.shape[0]
    dev = torch.device("cuda", 0)
    genv = PreconditionerEnv(n, P, A, side="AM", fill=fill, keep_m=True, device=dev)
    with torch.no_grad():
        model = GFlowNet(bench.make_policy(genv, P, dev), None, genv, mode="throughput", seed=1234)
        model.rollouts = int(d["stream_id"])
        log = model.sample_states([P] * 8, return_log=True)
    assert torch.equal(log.rewards_all.double().cpu(), d["rewards_all"])
    assert torch.equal(genv.last_residual.double().cpu(), d["residual"])
    best = int(torch.argmax(log.rewards_all))
    assert torch.equal(genv.last_m[best].cpu(), d["m_assembled"][0])


def test_bench_columns_two_ranks_gloo_pipelined_matches_one_gpu(tmp_path):
    """The multi-rank flow of the driver's scaling run on the one GPU: two ranks (gloo,
    host-staged collectives, both on GPU 0), the columns split with its two alternating graph
    programs (--pipeline, the default) and the deferred M gather.  Rank 0 dumps the last timed
    step: every one of the 2 x 8 candidates' rewards and the assembled best M must equal one GPU
    rolling out all 16 candidates at that stream id, bit for bit."""
    dump = tmp_path / "cols2.pt"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c2", "--gpus", "2", "--backend", "gloo",
           "--share-gpu", "--steps", "4", "--warmup", "1", "--no-cpu-baseline", "--dump", str(dump)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["world_size"] == 2 and line["pipeline"] is True
    d = torch.load(dump, weights_only=True)
    assert d["shard"] == "columns" and d["world"] == 2

    sys.path.insert(0, ROOT)
    import bench
    from gflownet_spai_amd import GFlowNet, PreconditionerEnv
    A, P = bench.config_matrices("c2")
    n = A.shape[0]
    dev = torch.device("cuda", 0)
    genv = PreconditionerEnv(n, P, A, side="AM", fill="qr", keep_m=True, device=dev)
    with torch.no_grad():
        model = GFlowNet(bench.make_policy(genv, P, dev), None, genv, mode="throughput", seed=1234)
        model.rollouts = int(d["stream_id"])
        log = model.sample_states([P] * 16, return_log=True)
    assert torch.equal(log.rewards_all.double().cpu(), d["rewards_all"])
    best = int(torch.argmax(log.rewards_all))
    assert torch.equal(genv.last_m[best].cpu(), d["m_assembled"][0])
