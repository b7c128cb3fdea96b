#!/bin/bash
# A/B of the generic residual kernel: the bench's roofline_residual leg per library variant
# (tree = the in-tree library).  usage: scripts/ab_resid.sh tree rc8.so rc4.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for v in "$@"; do
  if [ "$v" = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi
  timeout -k 10 200 python bench.py --config ${CFG:-c4} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab/resid_$v.log 2>&1 || { tail -5 gpurun_out/ab/resid_$v.log; exit 1; }
  tail -1 gpurun_out/ab/resid_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline_residual']; print('$v', d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['max_rel_diff_vs_fused_fill'])"
done
