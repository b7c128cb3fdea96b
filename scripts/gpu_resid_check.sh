#!/bin/bash
# GPU check of the generic residual / SpMV kernels: their parity tests, the C3 bench line
# (roofline_residual) and the ELL SpMV roofline on the C5 stand-in.  Each GPU step has its own
# time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/resid_check
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_parity.py tests/test_gmres.py -m gpu -x -q -k "residual or gmres or spmv" \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['ms_per_step'], json.dumps(d['roofline_residual']))"
timeout -k 10 300 python scripts/resid_bench.py --config c3 > $O/resid_c3.log 2>&1 || { tail -20 $O/resid_c3.log; exit 1; }
tail -1 $O/resid_c3.log
timeout -k 10 400 python scripts/gmres_eval.py --matrix thermal --grid 1108 --maxiter 40 --no-spilu --powers 1 --samples 1 \
  --out $O/gmres_c5s.json > $O/gmres.log 2>&1 || { tail -20 $O/gmres.log; exit 1; }
python -c "import json; d=json.load(open('$O/gmres_c5s.json')); print(json.dumps(d.get('spmv_A')))"
