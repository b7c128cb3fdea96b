"""Ingest timing: the native Matrix Market reader (spai_mtx_read) vs scipy.io.mmread (the
reference's reader, gflownet/utils.py:54-63) on a thermal2-sized synthetic symmetric file
(1,228,045 rows, the lower triangle of a 7-point-like pattern: ~4.9 M stored entries, ~8.5 M
after mirroring, like thermal2's 8.58 M).  thermal2 itself is not in the container.
usage: python scripts/mtx_bench.py [--out profiles/ingest_r1.json] [--path /tmp/thermal2_like.mtx]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gflownet_spai_amd.utils import read_mtx  # noqa: E402


def make(path, n=1_228_045, seed=0):
    rng = np.random.default_rng(seed)
    offs = (0, 1, 3, 1100)  # diagonal + three sub-diagonals: ~4 stored entries per row
    rows, cols = [], []
    for o in offs:
        i = np.arange(o, n)
        keep = rng.random(i.size) < (1.0 if o == 0 else 0.97)
        rows.append(i[keep] + 1)
        cols.append(i[keep] - o + 1)
    r, c = np.concatenate(rows), np.concatenate(cols)
    v = rng.standard_normal(r.size)
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real symmetric\n% synthetic thermal2-sized\n")
        f.write(f"{n} {n} {r.size}\n")
        np.savetxt(f, np.column_stack([r, c, v]), fmt=["%d", "%d", "%.16e"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", default="/tmp/thermal2_like.mtx")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if not os.path.exists(args.path):
        make(args.path)
    size = os.path.getsize(args.path)
    out = {"file": "synthetic thermal2-sized symmetric real MTX", "bytes": size, "cpus": os.cpu_count()}
    for threads in (1, 0):
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            r, c, v, shape = read_mtx(args.path, threads)
            best = min(best, time.perf_counter() - t0)
        out[f"native_s_threads_{threads or 'all'}"] = best
    out["nnz_after_mirroring"] = int(r.size)
    import scipy.io
    t0 = time.perf_counter()
    m = scipy.io.mmread(args.path).tocoo()
    out["scipy_mmread_tocoo_s"] = time.perf_counter() - t0
    out["identical_to_mmread"] = bool(np.array_equal(m.row, r) and np.array_equal(m.col, c)
                                      and np.array_equal(m.data, v))
    line = json.dumps(out)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
