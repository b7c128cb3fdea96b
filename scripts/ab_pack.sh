set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_qr_gpu.py tests/test_columns_split_gpu.py tests/test_bench_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abpack_tests.log 2>&1 || { tail -40 gpurun_out/abpack_tests.log; exit 1; }
tail -1 gpurun_out/abpack_tests.log
ROUNDS=3 BENCH_ARGS="--fill qr" bash scripts/gpu_ab.sh base.so || exit 1
