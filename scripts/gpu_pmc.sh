#!/bin/bash
# PMC counter passes (each its own rocprofv3 run, kernel-trace only; no sys/runtime traces).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for CTRS in "${@}"; do
  i=$((i+1))
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- \
    python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($CTRS) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
