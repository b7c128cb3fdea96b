#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_$TAG/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_$TAG/bench.log
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -3
exit $rc
