#!/bin/bash
# C3 profiles on one MI355X: rocprofv3 stats + PMC passes of the C3 bench, summarised into
# profiles/ (kernel_stats_r3c_c3.*, pmc_r3c_c3.json, the c3 records of fill_traffic.json).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/round_r3c_c3
mkdir -p $O gpurun_out/profiles
CMD="python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $CMD > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
PMC_TIMEOUT=300 scripts/pmc_kernels.sh $O/pmc $CMD > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python scripts/collect_profiles.py r3c_c3 $O/prof $O/pmc --config c3 --cmd "$CMD" > $O/collect.log 2>&1 || { cat $O/collect.log; exit 1; }
cp profiles/kernel_stats_r3c_c3.* profiles/pmc_r3c_c3.json profiles/fill_traffic.json gpurun_out/profiles/
head -14 profiles/kernel_stats_r3c_c3.md
