#!/bin/bash
# Round evidence on one MI355X: parity tests, smoke, rocprof kernel stats + PMC passes of the
# bench, profile summaries (also copied to gpurun_out/profiles), then the bench line itself.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
O=gpurun_out/round_$TAG
mkdir -p $O
step() { echo "== $1"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
CMD="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
step rocprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $CMD > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
step pmc
PMC_TIMEOUT=300 scripts/pmc_kernels.sh $O/pmc $CMD > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python scripts/collect_profiles.py $TAG $O/prof $O/pmc --cmd "$CMD" > $O/collect.log 2>&1 || { cat $O/collect.log; exit 1; }
mkdir -p gpurun_out/profiles && cp profiles/kernel_stats_$TAG.* profiles/pmc_$TAG.json profiles/fill_traffic.json gpurun_out/profiles/
step bench
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
