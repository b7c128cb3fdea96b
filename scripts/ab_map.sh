#!/bin/bash
# GPU A/B of the in-tree rollout kernels against build/variants/ libraries: rollout parity
# tests on the tree library, then HIP-event / rocprof kernel times of each variant.
# usage: scripts/ab_map.sh libspai_head.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K="throughput or split or stream_counter or full_size_c4_rollout or sample_states"
timeout -k 10 300 python -u -m pytest tests/test_hip_parity.py -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/t_tree.log 2>&1
rc=$?; tail -2 gpurun_out/t_tree.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/t_tree.log | head; exit $rc; }
bash scripts/ab_rollout.sh tree "$@" || exit 1
[ -f build/variants/libspai_prof.so ] && SPAI_LIB_VARIANT=libspai_prof.so timeout -k 10 120 python scripts/kernel_phases.py
exit 0
