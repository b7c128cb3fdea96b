#!/bin/bash
# GPU-box check: parity tests, smoke, short bench lines. Each GPU step has its own time limit;
# the script stops at the first failure (no GPU step runs after a crash, abort or timeout).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-10}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
for cfg in ${BENCH_CONFIGS:-c4 c3}; do
  timeout -k 10 400 python bench.py --config $cfg --steps $STEPS --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench_$cfg.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"; tail -2 gpurun_out/bench_$cfg.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
