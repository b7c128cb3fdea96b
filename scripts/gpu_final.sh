#!/bin/bash
# End-of-session evidence on one MI355X: rocprofv3 kernel stats of the C4 bench, then the default
# bench line (as the driver runs it) and the C3 line.  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r3d}
O=gpurun_out/round_$TAG
mkdir -p $O gpurun_out/profiles
CMD="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $CMD > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | cut -c1-300
