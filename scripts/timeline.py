"""Step timeline from a rocprofv3 kernel trace (``--kernel-trace --output-format csv``): the last
``--steps`` steps (a step starts at each launch of ``--marker``), per step the period, the union
of kernel busy time, and the idle gaps between kernels with the kernels on either side.

  python scripts/timeline.py <dir with *_kernel_trace.csv> [--marker k_presample] [--steps 5]
"""
import argparse
import csv
import glob
import os


def load(path):
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {path}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             f'{r.get("Stream_Id", "?")}/{r.get("Queue_Id", "?")}'))
    rows.sort()
    return rows


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--marker", default="k_presample")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--gap-us", type=float, default=3.0)
    args = ap.parse_args()
    rows = load(args.path)
    starts = [i for i, r in enumerate(rows) if args.marker in r[2]]
    if len(starts) < args.steps + 1:
        raise SystemExit(f"{len(starts)} marker launches")
    for s in range(len(starts) - args.steps - 1, len(starts) - 1):
        seg = rows[starts[s]:starts[s + 1]]
        t0, t1 = seg[0][0], rows[starts[s + 1]][0]
        busy, end, gaps = 0, t0, []
        prev = None
        for st, en, nm, q in seg:
            if st > end:
                if (st - end) / 1e3 >= args.gap_us:
                    gaps.append(((st - end) / 1e3, short(prev[2]) if prev else "-", short(nm)))
                busy += en - st
                end = en
            elif en > end:
                busy += en - end
                end = en
            prev = (st, en, nm)
        print(f"step {s}: period {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, {len(seg)} kernels")
        for g in gaps:
            print(f"   gap {g[0]:7.1f} us  after {g[1]}  before {g[2]}")
    # kernel list of the last step with stream ids
    s = len(starts) - 2
    print("last step kernels (start offset us, duration us, stream/queue, name):")
    t0 = rows[starts[s]][0]
    for st, en, nm, q in rows[starts[s]:starts[s + 1]]:
        print(f"  {(st - t0) / 1e3:8.1f} {(en - st) / 1e3:7.1f}  {q:>6}  {short(nm)}")


if __name__ == "__main__":
    main()
