#!/bin/bash
# Round evidence bench lines on one MI355X: C4 as the driver runs it (with the CPU baseline), the
# other configs without it, the one-rank RCCL columns step (its collective fields), C2 L@U.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r6}
O=gpurun_out/$TAG
mkdir -p $O
echo "== c4 (driver command)"
timeout -k 10 600 python bench.py > $O/bench_c4_full.log 2>&1 || { tail -20 $O/bench_c4_full.log; exit 1; }
tail -1 $O/bench_c4_full.log | cut -c1-300
for c in ${CFGS:-c2 c3 c5s c2lu}; do
  echo "== $c"
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$c.log 2>&1 \
    || { tail -20 $O/bench_$c.log; exit 1; }
  tail -1 $O/bench_$c.log | cut -c1-200
done
echo "== c4 --fill lsq"
timeout -k 10 400 python bench.py --fill lsq --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c4_lsq.log 2>&1 \
  || { tail -20 $O/bench_c4_lsq.log; exit 1; }
tail -1 $O/bench_c4_lsq.log | cut -c1-200
echo "== c4 --dist (one-rank RCCL columns step)"
timeout -k 10 400 python bench.py --gpus 1 --dist --backend nccl --steps 10 --warmup 2 --no-cpu-baseline \
  > $O/bench_c4_dist.log 2>&1 || { tail -20 $O/bench_c4_dist.log; exit 1; }
tail -1 $O/bench_c4_dist.log | cut -c1-200
