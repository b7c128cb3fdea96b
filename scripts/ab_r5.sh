#!/bin/bash
# Round-5 same-box A/B drivers (DESIGN.md §5 records each result).  usage on the GPU box:
#   bash scripts/ab_r5.sh <case>
# A "variant" is a library built under build/variants/<name>.so (make -C gflownet_spai_amd/csrc
# BUILD=... OUT=../../build/variants/<name>.so EXTRA=-D...) or "base.so" = the last commit's
# sources (git archive HEAD); scripts/gpu_ab.sh interleaves it with the tree library.
#   wavem   per-wave M staging in the QR solve       (variant wavem.so: EXTRA=-DQRS_WAVE_M)
#   blockm  per-block M staging in the Gram fills     (variant blockm.so: EXTRA="-DQRS_BLOCK_M -DFILL_BLOCK_M")
#   base    any change against base.so: the tests named in TESTS, then C4 (QR), then CFGS
#   ovl     overlap="sort" vs "select" (no variant)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
RUN_TESTS="$TESTS"; unset TESTS  # (gpu_ab.sh reads TESTS as a -k expression)
mkdir -p gpurun_out
tests() {
  [ -z "$1" ] && return 0
  timeout -k 10 900 python -u -m pytest $1 -m gpu -x -q --timeout 300 --timeout-method thread -k "${2:-not library_loaded}" \
    > gpurun_out/ab_r5_tests.log 2>&1 || { tail -40 gpurun_out/ab_r5_tests.log; exit 1; }
  tail -1 gpurun_out/ab_r5_tests.log
}
case "$1" in
  wavem)
    SPAI_LIB_VARIANT=wavem.so tests tests/test_qr_gpu.py
    ROUNDS=3 BENCH_ARGS="--fill qr" bash scripts/gpu_ab.sh wavem.so || exit 1 ;;
  blockm)
    tests "tests/test_qr_gpu.py tests/test_hip_parity.py tests/test_configs_gpu.py tests/test_columns_split_gpu.py" ""
    for a in "--fill qr" "--fill lsq"; do ROUNDS=2 BENCH_ARGS="$a" bash scripts/gpu_ab.sh blockm.so || exit 1; done
    ROUNDS=2 CFG=c3 bash scripts/gpu_ab.sh blockm.so || exit 1 ;;
  base)
    tests "${RUN_TESTS:-tests/test_qr_gpu.py tests/test_hip_parity.py}" ""
    ROUNDS=${ROUNDS:-3} BENCH_ARGS="--fill qr" bash scripts/gpu_ab.sh base.so || exit 1
    for c in ${CFGS:-}; do ROUNDS=2 CFG=$c bash scripts/gpu_ab.sh base.so || exit 1; done ;;
  ovl)
    for r in 1 2 3 4; do for o in sort select; do
      timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --overlap $o > gpurun_out/ovl_$o.log 2>&1 \
        || { tail -20 gpurun_out/ovl_$o.log; exit 1; }
      tail -1 gpurun_out/ovl_$o.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$o', round(d['ms_per_step'],4))"
    done; done ;;
  *) echo "usage: $0 wavem|blockm|base|ovl"; exit 2 ;;
esac
