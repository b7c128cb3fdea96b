#!/bin/bash
# Round 3 evidence on one MI355X: the round script (parity tests, smoke, rocprof stats + PMC of the C4 bench, C4 bench line),
# the C3 bench line and the ELL SpMV roofline on the banded 2-D Poisson matrix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/round_r3c
mkdir -p $O
unset SPAI_LIB_VARIANT
TAG=r3c bash scripts/gpu_round.sh || exit 1
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
cp $O/bench_c3.log gpurun_out/profiles/ 2>/dev/null
tail -1 $O/bench_c3.log | head -c 400; echo
timeout -k 10 300 python scripts/gmres_eval.py --matrix poisson --grid 1024 --maxiter 40 --no-spilu --powers 1 --samples 1 \
  --out $O/gmres_poisson.json > $O/gmres.log 2>&1 || { tail -5 $O/gmres.log; exit 1; }
python -c "import json; print(json.load(open('$O/gmres_poisson.json')).get('spmv_A'))"
