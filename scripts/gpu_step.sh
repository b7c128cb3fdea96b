#!/bin/bash
# One GPU call of a development iteration: optional pytest selection, then bench lines and an
# optional rocprofv3 kernel-stats pass, each step under its own time limit, stopping at the first
# failure.  usage: TAG=x TESTS="tests/test_qr_gpu.py" BENCH="--fill qr;--fill lsq" PROF="--fill qr" scripts/gpu_step.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-dev}
mkdir -p $O
if [ -n "$TESTS" ]; then
  echo "== pytest $TESTS"
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
IFS=';' read -ra BL <<< "$BENCH"
i=0
for b in "${BL[@]}"; do
  i=$((i+1))
  echo "== bench $b"
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $b > $O/bench$i.log 2>&1 || { tail -20 $O/bench$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench$i.log').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), 'ms', {k: round(v,4) for k,v in d['phases_ms'].items()}, 'roof', d['roofline']['kernel'][:24], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3), round(d['roofline']['frac_cache_counted'],3))"
done
if [ -n "$PROF" ]; then
  echo "== rocprof $PROF"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline $PROF > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  python scripts/prof_stats.py $O/prof 2>/dev/null | head -30 || true
fi
