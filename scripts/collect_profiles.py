"""Summarise a rocprofv3 --kernel-trace --stats run and the separate PMC passes of the same
bench command into profiles/: kernel_stats_<tag>.md/.csv, pmc_<tag>.json and
fill_traffic.json (HBM bytes per launch of the roofline kernel, read back by bench.py).

HBM traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: MI355X_MICROARCH.md §HBM
(FETCH_SIZE reports half of the bytes of coalesced reads on gfx950; calibrated here against
the fill kernel's known read bytes).
usage: python scripts/collect_profiles.py <tag> <prof_dir> <pmc_dir|-> [--config c4 --batch 8 --out profiles]
"""
import argparse
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOF_KERNELS = {"c4": "k_gram_fill<5, ", "c2": "k_gram_fill<5, ", "c3": "k_gram_fill_wide<13, "}  # LSQ fill, any Gram type
ROOF_KERNELS_QR = {"c4": "k_qr_lookup<5, ", "c2": "k_qr_lookup<5, ", "c5s": "k_qr_solve<7, ", "c3": "k_qr_solve<13, "}


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0][:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("prof")
    ap.add_argument("pmc")
    ap.add_argument("--config", default="c4")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles"))
    ap.add_argument("--cmd", default="python bench.py --steps 10 --warmup 2 --no-cpu-baseline")
    ap.add_argument("--fill", default="lsq", choices=["lsq", "qr"], help="the bench command's fill (its roofline kernel)")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    stats = os.path.join(args.prof, "run_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    lines = ["| kernel | calls | avg us | total ms | % |", "|---|---|---|---|---|"]
    summary = {"tag": args.tag, "command": args.cmd, "kernels": {}}
    for r in rows:
        k = short(r["Name"])
        summary["kernels"].setdefault(k, {})["avg_us"] = float(r["AverageNs"]) / 1e3
        summary["kernels"][k]["calls"] = int(r["Calls"])
        if len(lines) < 32:
            lines.append(f"| {k} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                         f"{float(r['TotalDurationNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")
    with open(os.path.join(args.out, f"kernel_stats_{args.tag}.md"), "w") as f:
        f.write(f"# rocprofv3 --kernel-trace --stats ({args.tag})\n\nCommand on one MI355X: "
                f"`rocprofv3 --kernel-trace --stats --output-format csv -- {args.cmd}`\n\n" + "\n".join(lines) + "\n")
    shutil.copy(stats, os.path.join(args.out, f"kernel_stats_{args.tag}.csv"))
    if args.pmc == "-":  # kernel stats only (no PMC passes in this run)
        return
    pmc = json.load(open(os.path.join(args.pmc, "summary.json")))
    for k, e in pmc.items():
        kk = k.replace("spai::", "")
        match = [n for n in summary["kernels"] if n.replace("spai::", "").replace("void ", "").startswith(kk.replace("void ", ""))]
        dst = summary["kernels"].setdefault(match[0] if match else k, {})
        dst.update(e)
    with open(os.path.join(args.out, f"pmc_{args.tag}.json"), "w") as f:
        json.dump(summary, f, indent=1)
    if args.fill == "qr":
        roof = [(k, v) for k, v in summary["kernels"].items()
                if ROOF_KERNELS_QR[args.config] in k and "hbm_bytes_per_launch" in v]
    else:
        roof = [(k, v) for k, v in summary["kernels"].items()
                if ROOF_KERNELS[args.config] in k and "true" in k and "hbm_bytes_per_launch" in v]
    key = args.config + ("_qr" if args.fill == "qr" else "")
    if roof:
        k, v = roof[0]
        rec = {"config": args.config, "batch": args.batch, "kernel": k, "avg_us": v.get("avg_us"),
               "hbm_bytes_per_launch": v["hbm_bytes_per_launch"], "FETCH_SIZE_KB": v["pmc"].get("FETCH_SIZE"),
               "WRITE_SIZE_KB": v["pmc"].get("WRITE_SIZE"), "source": f"profiles/pmc_{args.tag}.json",
               "command": args.cmd}
        # the cached QR fill's (entry, mask) table kernel runs before the lookup in the same call
        tab = [(k2, v2) for k2, v2 in summary["kernels"].items() if "k_qr_table<" in k2 and "hbm_bytes_per_launch" in v2]
        if "k_qr_lookup<" in k and tab:
            rec["kernel"] = f"{tab[0][0]} + {k}"
            rec["hbm_bytes_per_launch"] += tab[0][1]["hbm_bytes_per_launch"]
            rec["avg_us"] = (rec["avg_us"] or 0.0) + (tab[0][1].get("avg_us") or 0.0)
        path = os.path.join(args.out, "fill_traffic.json")
        try:
            allrec = json.load(open(path))
        except (OSError, ValueError):
            allrec = {}
        if "config" in allrec:  # older single-record form
            allrec = {allrec["config"]: allrec}
        allrec[key] = rec
        # the generic residual leg's kernel (bench roofline_residual), when it ran in this command
        res = [(k, v) for k, v in summary["kernels"].items()
               if ("k_resid_shared<" in k or "k_resid_wide<" in k or "k_resid_gram<" in k) and "hbm_bytes_per_launch" in v]
        if res:
            k, v = res[0]
            allrec[args.config + "_residual"] = {
                "config": args.config, "batch": args.batch, "kernel": k, "avg_us": v.get("avg_us"),
                "hbm_bytes_per_launch": v["hbm_bytes_per_launch"], "FETCH_SIZE_KB": v["pmc"].get("FETCH_SIZE"),
                "WRITE_SIZE_KB": v["pmc"].get("WRITE_SIZE"), "source": f"profiles/pmc_{args.tag}.json",
                "command": args.cmd}
        # the rollout's dominant kernels (bench roofline: k_tile; k_sort2 for reference), with the
        # VALU instruction count the bench's issue-time estimate uses
        for short_name, key2 in (("k_tile", "_tile"), ("k_sort2", "_sort")):
            kk = [(k, v) for k, v in summary["kernels"].items() if k.replace("spai::", "").startswith(short_name)
                  and "hbm_bytes_per_launch" in v]
            if kk:
                k, v = kk[0]
                allrec[args.config + key2] = {
                    "config": args.config, "batch": args.batch, "kernel": k, "avg_us": v.get("avg_us"),
                    "hbm_bytes_per_launch": v["hbm_bytes_per_launch"], "valu_insts_per_launch": v["pmc"].get("SQ_INSTS_VALU"),
                    "FETCH_SIZE_KB": v["pmc"].get("FETCH_SIZE"), "WRITE_SIZE_KB": v["pmc"].get("WRITE_SIZE"),
                    "source": f"profiles/pmc_{args.tag}.json", "command": args.cmd}
        json.dump(allrec, open(path, "w"), indent=1)
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
