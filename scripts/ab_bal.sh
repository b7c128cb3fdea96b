set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 800 python -u -m pytest tests/test_hip_parity.py tests/test_columns_split_gpu.py tests/test_policy_gpu.py tests/test_train_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abbal_tests.log 2>&1 || { tail -40 gpurun_out/abbal_tests.log; exit 1; }
tail -1 gpurun_out/abbal_tests.log
ROUNDS=2 BENCH_ARGS="--fill qr" bash scripts/gpu_ab.sh base.so || exit 1
ROUNDS=2 CFG=c2 bash scripts/gpu_ab.sh base.so || exit 1
