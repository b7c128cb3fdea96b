#!/bin/bash
# A/B of library variants (build/variants/<lib>) against the tree library on the C4 bench:
# optional GPU tests first (TESTS = a pytest -k expression, or "all"), then ROUNDS interleaved
# bench runs each, ms/step and the per-phase HIP-event times printed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  K=(); [ "$TESTS" != all ] && K=(-k "$TESTS")
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -1 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/ab_tests.log | head -30; exit $rc; }
fi
for r in $(seq 1 ${ROUNDS:-2}); do
for v in tree "$@"; do
  if [ "$v" = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi
  timeout -k 10 300 python bench.py --config ${CFG:-c4} --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  tail -1 gpurun_out/ab_$v.log | python scripts/ab_line.py $v
done
done
