set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_qr_gpu.py tests/test_hip_parity.py tests/test_configs_gpu.py tests/test_columns_split_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/abm_tests.log 2>&1 || { tail -30 gpurun_out/abm_tests.log; exit 1; }
tail -1 gpurun_out/abm_tests.log
ROUNDS=2 BENCH_ARGS="--fill qr" bash scripts/gpu_ab.sh blockm.so || exit 1
ROUNDS=2 BENCH_ARGS="--fill lsq" bash scripts/gpu_ab.sh blockm.so || exit 1
ROUNDS=2 CFG=c3 bash scripts/gpu_ab.sh blockm.so || exit 1
