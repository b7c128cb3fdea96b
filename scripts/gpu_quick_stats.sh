#!/bin/bash
# rocprofv3 kernel stats of a short C4 bench run (+ the last step's timeline), printed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/qs_${TAG:-x}
mkdir -p $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- \
  python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
f=$(find $D -name "run_kernel_stats.csv" | head -1); dd=$(dirname $f)
python scripts/prof_stats.py $dd 30 ${TAIL:-0}
tail -1 $D/bench.log | cut -c1-300
