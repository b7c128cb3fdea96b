#!/bin/bash
# Round-6 same-box A/B: the tests named in TESTS on the tree library, the isolated QR fill of each
# library (scripts/qr_fill_bench.py), then interleaved C4 bench lines (scripts/gpu_ab.sh) of the
# tree library and the variants given as arguments (build/variants/<name>.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then  # on the tree library and (VTESTS=1) on every variant
  for v in tree ${VTESTS:+"$@"}; do
    if [ "$v" = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi
    timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -k "not library_loaded" \
      > gpurun_out/ab_r6_tests_$v.log 2>&1 \
      || { tail -40 gpurun_out/ab_r6_tests_$v.log; exit 1; }
    echo "tests $v: $(tail -1 gpurun_out/ab_r6_tests_$v.log)"
  done
  unset SPAI_LIB_VARIANT
fi
if [ -n "$QRB" ]; then
  for v in tree "$@"; do
    if [ "$v" = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi
    timeout -k 10 300 python scripts/qr_fill_bench.py --config c4 --batches 8 > gpurun_out/qrb_$v.log 2>&1 || { tail -20 gpurun_out/qrb_$v.log; exit 1; }
    echo "qrb $v: $(grep '^{' gpurun_out/qrb_$v.log | python -c "import sys,json; print([(d['dict'], d['store_m'], round(d['kernel_ms']*1e3,1)) for d in map(json.loads, sys.stdin)])")"
  done
  unset SPAI_LIB_VARIANT
fi
TESTS= STEPS=${STEPS:-30} ROUNDS=${ROUNDS:-2} bash scripts/gpu_ab.sh "$@"
