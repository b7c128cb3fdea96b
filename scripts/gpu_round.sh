#!/bin/bash
# Round evidence on one MI355X: the whole -m gpu suite, smoke, rocprofv3 kernel stats of the C4
# bench (QR fill, the default) and of the LSQ-fill bench, then the bench lines themselves (C4,
# C4 --fill lsq, C3).
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r5}
O=gpurun_out/round_$TAG
mkdir -p $O
step() { echo "== $1"; }
if [ -z "$SKIP_TESTS" ]; then
  step pytest
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
CMD="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
step rocprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $CMD > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
step rocprof_lsq
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lsq -o run -- $CMD --fill lsq > $O/prof_lsq.log 2>&1 || { tail -20 $O/prof_lsq.log; exit 1; }
step bench
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
step bench_lsq
timeout -k 10 300 python bench.py --fill lsq --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_lsq.log 2>&1 || { tail -20 $O/bench_lsq.log; exit 1; }
tail -1 $O/bench_lsq.log | cut -c1-400
step bench_c3
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | cut -c1-400
