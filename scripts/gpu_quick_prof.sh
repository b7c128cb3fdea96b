#!/bin/bash
# Quick GPU iteration: selected parity tests, then a rocprofv3 kernel-stats run of a short
# bench (no PMC).  usage: TESTS="tests/test_policy_gpu.py" TAG=x scripts/gpu_quick_prof.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-quick}
O=gpurun_out/quick_$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
python scripts/prof_stats.py $O/prof 30 ${TRACE:-0}
