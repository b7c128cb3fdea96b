#!/bin/bash
# PMC passes over a command (each its own rocprofv3 run, kernel-trace only), summary per kernel.
# usage: scripts/pmc_kernels.sh <outdir> <cmd...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
i=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -k 10 ${PMC_TIMEOUT:-200} rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; [ $i -le 4 ] && exit $rc; fi
done
python - "$OUT" <<'PY'
import csv, collections, glob, json, sys
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {}
for k, d in sorted(agg.items()):
    if "spai" not in k:
        continue
    a = {c: sum(v) / len(v) for c, v in d.items()}
    e = {"pmc": a}
    if "FETCH_SIZE" in a and "WRITE_SIZE" in a:
        # MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports half of coalesced read bytes on gfx950
        e["hbm_bytes_per_launch"] = (2 * a["FETCH_SIZE"] + a["WRITE_SIZE"]) * 1024
    summary[k] = e
    print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(a.items())))
json.dump(summary, open(f"{out}/summary.json", "w"), indent=1)
PY
