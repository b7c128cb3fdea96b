#!/bin/bash
# The multi-GPU bench flow rehearsed on ONE MI355X: 2 ranks share GPU 0 over gloo (host-staged
# collectives), for each split; then the N=1 bench line.  Not a scaling measurement.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sh in ${SPLITS:-columns samples slices}; do
  timeout -k 10 300 python bench.py --gpus ${RANKS:-2} --backend gloo --share-gpu --shard $sh --steps 5 --warmup 2 \
    --config ${CFG:-c2} --no-cpu-baseline > gpurun_out/rehearsal_$sh.log 2>&1 || { tail -30 gpurun_out/rehearsal_$sh.log; exit 1; }
  tail -1 gpurun_out/rehearsal_$sh.log | cut -c1-600
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rehearsal_n1.log 2>&1 || { tail -20 gpurun_out/rehearsal_n1.log; exit 1; }
tail -1 gpurun_out/rehearsal_n1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N1', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['phases_ms'].items()})"
