#!/bin/bash
# Bucket-region staging: whole -m gpu suite, interleaved A/B vs the given variants, k_sort2/k_tile
# FETCH/WRITE sizes; then (LEARN=1) the constant-lr training runs of scripts/learn_pattern.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/exp_${TAG:-region}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ROUNDS=${ROUNDS:-3} bash scripts/gpu_ab.sh "$@" || exit 1
for v in tree "$@"; do
  if [ "$v" = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_${v}_$c -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_${v}_$c.log 2>&1 || { tail -5 $O/pmc_${v}_$c.log; exit 1; }
  done
  python - $O "$v" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(f"{sys.argv[1]}/pmc_{sys.argv[2]}_*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if any(x in k for x in ("k_sort2", "k_tile", "k_bsum", "k_pad")):
            d[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(d.items()):
    print(sys.argv[2], k, c, "MB", round(sum(v) / len(v) / 1000 * (2 if c == "FETCH_SIZE" else 1), 1))
PY
done
unset SPAI_LIB_VARIANT
if [ "${LEARN:-0}" = 1 ]; then
  timeout -k 10 400 python -u scripts/learn_pattern.py --matrix poisson --grid 256 --epochs 1000 --budget-s 150 --lr 1e-2 --no-plateau --out $O/learn_c2_const.json > $O/learn_c2_const.log 2>&1 || { tail -20 $O/learn_c2_const.log; exit 1; }
  tail -3 $O/learn_c2_const.log | cut -c1-1500
  timeout -k 10 400 python -u scripts/learn_pattern.py --matrix thermal --grid 256 --epochs 1000 --budget-s 150 --lr 1e-2 --no-plateau --out $O/learn_th_const.json > $O/learn_th_const.log 2>&1 || { tail -20 $O/learn_th_const.log; exit 1; }
  tail -3 $O/learn_th_const.log | cut -c1-1500
fi
