#!/bin/bash
# LDS / VALU counters of the rollout kernels: two rocprofv3 --pmc passes over scripts/ab_rollout.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_rollout
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d $O/p -o run -- python scripts/ab_rollout.py > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/q -o run -- python scripts/ab_rollout.py > $O/log2 2>&1 || { tail -5 $O/log2; exit 1; }
python - $O/p/run_counter_collection.csv $O/q/run_counter_collection.csv <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "spai" in k:
        a = {c: sum(v) / len(v) for c, v in d.items()}
        print("%-28s VALU %.3g LDS %.3g WAIT_LDS %.3g BANK %.3g (%.2f per LDS instr)" % (k, a["SQ_INSTS_VALU"], a["SQ_INSTS_LDS"], a["SQ_WAIT_INST_LDS"], a["SQ_LDS_BANK_CONFLICT"], a["SQ_LDS_BANK_CONFLICT"] / max(a["SQ_INSTS_LDS"], 1)))
        gui = max(a.get("GRBM_GUI_ACTIVE", 1), 1)
        # quad-cycle counters summed over waves; per-SIMD busy fractions over 1024 SIMDs x GUI cycles
        print("%-28s   VALU-busy %.2f LDS-busy %.2f wave-cycles/GUI %.1f wait-any/wave-cycles %.2f" % ("",
              4 * a["SQ_ACTIVE_INST_VALU"] / (1024 * gui), 4 * a["SQ_ACTIVE_INST_LDS"] / (1024 * gui),
              4 * a["SQ_WAVE_CYCLES"] / (1024 * gui), a["SQ_WAIT_INST_ANY"] / max(a["SQ_WAVE_CYCLES"], 1)))
PY
