#!/bin/bash
# Profile evidence for one bench config on one MI355X (no tests): rocprofv3 kernel stats,
# the PMC passes, the profiles/ summaries (copied to gpurun_out/profiles), then the bench line.
# usage: TAG=r2b CONFIG=c4 scripts/gpu_prof.sh     (every GPU step has its own time limit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r2}
CONFIG=${CONFIG:-c4}
FILL=${FILL:-lsq}
O=gpurun_out/prof_${TAG}_$CONFIG
mkdir -p $O gpurun_out/profiles
CMD="python bench.py --config $CONFIG --fill $FILL --steps 10 --warmup 2 --no-cpu-baseline ${PROF_ARGS:-}"
echo "== rocprof $CONFIG"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $CMD > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo "== pmc $CONFIG"
PMC_TIMEOUT=300 scripts/pmc_kernels.sh $O/pmc $CMD > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python scripts/collect_profiles.py ${TAG}_$CONFIG $O/prof $O/pmc --config $CONFIG --fill $FILL --cmd "$CMD" > $O/collect.log 2>&1 || { cat $O/collect.log; exit 1; }
cp profiles/kernel_stats_${TAG}_$CONFIG.* profiles/pmc_${TAG}_$CONFIG.json profiles/fill_traffic.json gpurun_out/profiles/
echo "== bench $CONFIG"
timeout -k 10 400 python bench.py --config $CONFIG --fill $FILL ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
