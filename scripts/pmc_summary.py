"""Summarise rocprofv3 outputs into profiles/: kernel stats table and per-kernel PMC averages.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports half of
the bytes of wide coalesced reads on gfx950, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
(Uncalibrated for other access widths; both terms are listed separately.)
usage: python scripts/pmc_summary.py <tag> [prof_dir] [pmc_dir]
"""
import collections
import csv
import json
import os
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
prof = sys.argv[2] if len(sys.argv) > 2 else f"gpurun_out/prof_{tag}"
pmc = sys.argv[3] if len(sys.argv) > 3 else f"gpurun_out/pmc_{tag}"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out_dir = os.path.join(root, "profiles")
os.makedirs(out_dir, exist_ok=True)


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0][:80]


summary = {"tag": tag, "kernels": {}}
stats = os.path.join(prof, "run_kernel_stats.csv")
if os.path.exists(stats):
    rows = list(csv.DictReader(open(stats)))
    lines = ["| kernel | calls | avg us | total ms | % |", "|---|---|---|---|---|"]
    for r in rows[:30]:
        k = short(r["Name"])
        lines.append(f"| {k} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")
        summary["kernels"].setdefault(k, {})["avg_us"] = float(r["AverageNs"]) / 1e3
        summary["kernels"][k]["calls"] = int(r["Calls"])
    with open(os.path.join(out_dir, f"kernel_stats_{tag}.md"), "w") as f:
        f.write(f"# rocprofv3 --kernel-trace --stats ({tag})\n\nCommand: `rocprofv3 --kernel-trace --stats "
                f"--output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline` on one MI355X.\n\n")
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(out_dir, f"kernel_stats_{tag}.csv"), "w") as f:
        f.write(open(stats).read())
if os.path.isdir(pmc):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(os.listdir(pmc)):
        p = os.path.join(pmc, d, "run_counter_collection.csv")
        if os.path.exists(p):
            for r in csv.DictReader(open(p)):
                agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        e = summary["kernels"].setdefault(k, {})
        e["pmc"] = avg
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["hbm_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
with open(os.path.join(out_dir, f"pmc_{tag}.json"), "w") as f:
    json.dump(summary, f, indent=1)
print(json.dumps({k: {kk: (round(vv, 1) if isinstance(vv, float) else None) for kk, vv in v.items() if kk != "pmc"}
                  for k, v in summary["kernels"].items() if "spai" in k}, indent=0)[:3000])
