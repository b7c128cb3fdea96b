#!/bin/bash
# A/B of the 13-wide generic residual kernels: the tree library (after its residual parity tests)
# and the library variants given (build/variants/<name>.so; "old" = the tree with
# SPAI_RESID_WIDE_OLD, the thread-per-line k_resid_wide).  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/resid_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_parity.py -m gpu -x -q -k "residual" \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in tree "$@" tree; do
  unset SPAI_RESID_WIDE_OLD SPAI_LIB_VARIANT
  if [ $v = old ]; then export SPAI_RESID_WIDE_OLD=1; elif [ $v != tree ]; then export SPAI_LIB_VARIANT=$v; fi
  timeout -k 10 300 python bench.py --config ${CFG:-c3} --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  tail -1 $O/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline_residual']; print('$v', round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), round(r['frac'],3), r['max_rel_diff_vs_fused_fill'])"
done
