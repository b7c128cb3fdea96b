cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "residual or c3 or assemble" > gpurun_out/res_tests.log 2>&1; rc=$?; tail -1 gpurun_out/res_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/res_tests.log | head -20; exit $rc; }
CFG=c3 bash scripts/ab_resid.sh tree libbase.so || exit 1
for v in tree libbase.so; do if [ $v = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi; timeout -k 10 120 python scripts/resid_bench.py --config c3 --distinct 2>&1 | tail -1 || exit 1; done
