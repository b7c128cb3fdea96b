#!/bin/bash
# Experiment: k_sort2 bucket order (tree: XCD-aware, libnoxcd: plain) — rollout parity tests,
# interleaved A/B of the C4 bench, per-phase stamps (libspai_prof) and FETCH_SIZE of k_sort2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/exp_${TAG:-sort}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_parity.py -x -q --timeout 120 --timeout-method thread -k "rollout or order or sort or throughput" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ROUNDS=${ROUNDS:-2} bash scripts/gpu_ab.sh "$@" || exit 1
SPAI_LIB_VARIANT=libspai_prof.so timeout -k 10 200 python scripts/kernel_phases.py > $O/phases.log 2>&1 || { tail -20 $O/phases.log; exit 1; }
cat $O/phases.log
for v in tree "$@"; do
  if [ "$v" = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_$v -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
  python - $O/pmc_$v "$v" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if "k_sort2" in k or "k_tile" in k:
            d[k].append(float(r["Counter_Value"]))
for k, v in d.items():
    print(sys.argv[2], k, "FETCH_SIZE KB avg", sum(v) / len(v), "x2 MB", 2 * sum(v) / len(v) / 1000)
PY
done
