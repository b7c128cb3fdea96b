"""Practical HBM rates on this MI355X for the stream shapes of the fill kernel (k_gram_fill at
C4, B = 8: 110 MB read — Gram cache, action ids, bitmaps — and 168 MB written — M): a
write-only stream, a read-only stream and a copy (torch's own kernels, HIP-event timed), and
from them the time a streaming kernel of the fill's read/write mix would take.  Prints one JSON line.

usage: python scripts/hbm_probe.py [--iters 50]
"""
import argparse
import json

import torch


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3  # s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    wr_bytes, rd_bytes = 168 * 2 ** 20, 110 * 2 ** 20
    w = torch.empty(wr_bytes // 4, dtype=torch.float32, device=dev)
    r = torch.rand(rd_bytes // 4, dtype=torch.float32, device=dev)
    out = {}
    t = timed(lambda: w.fill_(1.0), args.iters)
    out["write_only_GBps"] = wr_bytes / t / 1e9
    t = timed(lambda: r.sum(), args.iters)
    out["read_only_GBps"] = rd_bytes / t / 1e9
    # copy: read 110 MB + write 110 MB in one kernel
    c = torch.empty_like(r)
    t_copy = timed(lambda: c.copy_(r), args.iters)
    out["copy_GBps"] = 2 * rd_bytes / t_copy / 1e9
    # the fill's mix at these rates: 110 MB read + 110 MB written as a copy, the other 58 MB
    # write-only (an estimate of the best a streaming kernel of that mix reaches)
    t_mix = t_copy + (wr_bytes - rd_bytes) / (out["write_only_GBps"] * 1e9)
    out["fill_mix_estimate"] = {"us": t_mix * 1e6, "GBps": (wr_bytes + rd_bytes) / t_mix / 1e9}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
