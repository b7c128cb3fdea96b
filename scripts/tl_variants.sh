#!/bin/bash
# Kernel-trace timelines of the one-rank RCCL columns step under env variants (VARS="name=ENV=V ...").
export TMPDIR=/tmp; O=gpurun_out/${TAG:-tlv}; mkdir -p $O
for v in ${VARS:-base=X=0}; do
  n=${v%%=*}; e=${v#*=}
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$n -o run -- python bench.py --gpus 1 --dist --backend nccl --steps 20 --warmup 3 --no-cpu-baseline > $O/tl_$n.log 2>&1 || exit 1
  echo "== $n"
  grep "^{" $O/tl_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:d.get(k) for k in ['ms_per_step','ms_per_step_without_assembly']})"
  python scripts/timeline.py $O/tl_$n --steps 2 > $O/tl_$n.txt 2>&1; cat $O/tl_$n.txt
done
