#!/bin/bash
# Fill-kernel change check on one MI355X: the fill/residual GPU tests on the tree library,
# then fill_bench A/B of the tree against build/variants/<libs>, then the C4 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "gram or lsq or fill or c4 or c3 or c2 or c5 or residual or assemble or edge" > gpurun_out/ab_fill_tests.log 2>&1
rc=$?; tail -1 gpurun_out/ab_fill_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/ab_fill_tests.log | head; exit $rc; }
BATCHES=8 bash scripts/ab_fill.sh tree "$@" > gpurun_out/ab_fill.log 2>&1 || { tail -20 gpurun_out/ab_fill.log; exit 1; }
cat gpurun_out/ab_fill.log
CFG=c3 BATCHES=8 bash scripts/ab_fill.sh tree "$@" > gpurun_out/ab_fill_c3.log 2>&1 || { tail -20 gpurun_out/ab_fill_c3.log; exit 1; }
cat gpurun_out/ab_fill_c3.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench.log 2>&1 || { tail -20 gpurun_out/ab_bench.log; exit 1; }
tail -1 gpurun_out/ab_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'], d['roofline'])"
