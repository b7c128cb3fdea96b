#!/bin/bash
# A/B of rollout kernels: for each variant (tree = the in-tree library, else
# build/variants/<name>), HIP-event phase times and a rocprofv3 kernel-stats table.
# usage: scripts/ab_rollout.sh tree libspai_old.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in "$@"; do
  if [ "$v" = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi
  timeout -k 10 200 python scripts/ab_rollout.py || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/$v -o run -- \
    python scripts/ab_rollout.py > gpurun_out/ab/$v.log 2>&1 || { tail -5 gpurun_out/ab/$v.log; exit 1; }
  python - gpurun_out/ab/$v/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print("   %-60s %6s %9.1f us" % (r["Name"].replace("(anonymous namespace)::", "")[:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
