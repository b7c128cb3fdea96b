#!/bin/bash
# Quick GPU check of a rollout/fill change: the whole -m gpu suite, then the C4 bench line on the
# tree library and on each build/variants/<lib> given (phase times + ms/step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -1 gpurun_out/quick_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/quick_tests.log | head -20; exit $rc; }
for v in tree "$@"; do
  if [ "$v" = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi
  timeout -k 10 300 python bench.py --config ${CFG:-c4} --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/quick_bench_$v.log 2>&1 || { tail -20 gpurun_out/quick_bench_$v.log; exit 1; }
  tail -1 gpurun_out/quick_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['phases_ms'].items()})"
done
