set -o pipefail
cd $GRAFT_REPO_ROOT
SPAI_LIB_VARIANT=wavem.so timeout -k 10 600 python -u -m pytest tests/test_qr_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not library_loaded" > gpurun_out/abw_tests.log 2>&1 || { tail -30 gpurun_out/abw_tests.log; exit 1; }
tail -1 gpurun_out/abw_tests.log
ROUNDS=3 BENCH_ARGS="--fill qr" bash scripts/gpu_ab.sh wavem.so || exit 1
ROUNDS=1 BENCH_ARGS="--fill lsq" bash scripts/gpu_ab.sh || exit 1
ROUNDS=1 CFG=c3 bash scripts/gpu_ab.sh || exit 1
