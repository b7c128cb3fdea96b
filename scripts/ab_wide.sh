set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_configs_gpu.py tests/test_hip_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abwide_tests.log 2>&1 || { tail -30 gpurun_out/abwide_tests.log; exit 1; }
tail -1 gpurun_out/abwide_tests.log
ROUNDS=3 CFG=c3 bash scripts/gpu_ab.sh left.so || exit 1
