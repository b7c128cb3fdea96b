"""Which HIP-graph capture of a pipelined throughput step fails: captures of increasing scope,
each announced (flushed) before it starts, so the last line printed names the failing one.

  python scripts/pipeline_capture_diag.py [--config c2]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gflownet_spai_amd import GFlowNet, PreconditionerEnv  # noqa: E402


def say(*a):
    print(*a, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    A, P = bench.config_matrices(args.config)
    env = PreconditionerEnv(A.shape[0], P, A, side="AM", fill="qr", keep_m=True, device=dev)
    pol = bench.make_policy(env, P, dev)
    s0 = [P] * 8

    # 1. plain fork/join of a priority stream inside a capture, a dangling event record on it
    x = torch.zeros(1 << 20, device=dev)
    ln = torch.cuda.Stream(dev, priority=-1)
    g = torch.cuda.graph
    say("1a fork/join priority stream")
    gr = torch.cuda.CUDAGraph()
    with g(gr):
        ln.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(ln):
            x.add_(1)
        torch.cuda.current_stream(dev).wait_stream(ln)
    gr.replay()
    torch.cuda.synchronize()
    say("1b + dangling event on the forked stream")
    gr = torch.cuda.CUDAGraph()
    with g(gr):
        ln.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(ln):
            x.add_(1)
            ev = torch.cuda.Event()
            ev.record(ln)
            x.add_(1)
        torch.cuda.current_stream(dev).wait_stream(ln)
    gr.replay()
    torch.cuda.synchronize()
    if os.environ.get("DIAG_NESTED"):  # crashes hipStreamEndCapture on ROCm 7 (r6): a stream forked from a forked stream
      say("1c two-level fork C -> ln -> sd")
      sd = torch.cuda.Stream(dev, priority=-1)
      gr = torch.cuda.CUDAGraph()
      with g(gr):
          ln.wait_stream(torch.cuda.current_stream(dev))
          with torch.cuda.stream(ln):
              x.add_(1)
              sd.wait_stream(ln)
              with torch.cuda.stream(sd):
                  x.mul_(2)
              ln.wait_stream(sd)
          torch.cuda.current_stream(dev).wait_stream(ln)
      gr.replay()
      torch.cuda.synchronize()
    say("1d allocation on the forked stream inside the capture")
    gr = torch.cuda.CUDAGraph()
    with g(gr):
        ln.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(ln):
            y = torch.empty(1 << 20, device=dev)
            y.copy_(x)
        torch.cuda.current_stream(dev).wait_stream(ln)
    gr.replay()
    torch.cuda.synchronize()

    for overlap in (False,):
        model = GFlowNet(pol, None, env, mode="throughput", seed=5, pipeline=True, overlap=overlap)
        with torch.no_grad():
            for _ in range(2):
                model.sample_states(s0)
            model.pipeline_join()
            torch.cuda.synchronize()
            for nsteps in (1, 2, 5):
                say(f"2 pipelined capture overlap={overlap} steps={nsteps}")
                gr = torch.cuda.CUDAGraph()
                with g(gr):
                    for _ in range(nsteps):
                        model.sample_states(s0)
                    model.pipeline_join()
                gr.replay()
                torch.cuda.synchronize()
    say("all captures ok")


if __name__ == "__main__":
    main()
