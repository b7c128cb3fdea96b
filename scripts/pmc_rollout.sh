#!/bin/bash
# LDS / VALU counters of the rollout kernels (one rocprofv3 --pmc pass over scripts/ab_rollout.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_rollout
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d $O/p -o run -- python scripts/ab_rollout.py > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
python - $O/p/run_counter_collection.csv <<'PY'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "spai" in k:
        a = {c: sum(v) / len(v) for c, v in d.items()}
        print("%-40s VALU %.3g LDS %.3g WAIT_LDS %.3g BANK %.3g (%.2f per LDS instr)" % (k, a["SQ_INSTS_VALU"], a["SQ_INSTS_LDS"], a["SQ_WAIT_INST_LDS"], a["SQ_LDS_BANK_CONFLICT"], a["SQ_LDS_BANK_CONFLICT"] / max(a["SQ_INSTS_LDS"], 1)))
PY
