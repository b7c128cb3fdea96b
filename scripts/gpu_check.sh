#!/bin/bash
# GPU-box check: parity tests, smoke, short bench. Stops at the first crash/timeout
# (exit 124/134/137/139); an ordinary pytest failure (exit 1) still runs smoke + bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-10}
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -3 gpurun_out/smoke.log
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 400 python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc3=$?; echo "bench rc=$rc3"; tail -3 gpurun_out/bench.log
exit $(( rc > rc3 ? rc : rc3 ))
