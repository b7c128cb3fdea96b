set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3 4; do for o in sort select; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --overlap $o > gpurun_out/ovl_$o.log 2>&1 || { tail -20 gpurun_out/ovl_$o.log; exit 1; }
  tail -1 gpurun_out/ovl_$o.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$o', round(d['ms_per_step'],4))"
done; done
