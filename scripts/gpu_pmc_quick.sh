#!/bin/bash
# PMC passes of the C4 bench (per-kernel summary printed for the spai kernels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_${TAG:-x}
PMC_TIMEOUT=240 bash scripts/pmc_kernels.sh $O python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O.txt 2>&1
rc=$?; grep -E "k_tile|k_sort2|k_gram_fill|k_fixed|k_splitters|k_pad|k_fc|k_resid|pass" $O.txt | cut -c1-900; exit $rc
