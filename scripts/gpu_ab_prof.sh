#!/bin/bash
# Kernel-level A/B of library variants (build/variants/<lib>) against the tree library: optional
# GPU tests (TESTS = a pytest -k expression), then ROUNDS interleaved rocprofv3 kernel-stats runs
# of the C4 bench per library, printing the average duration of the kernels named in KERNELS.
# usage: TESTS="rollout" KERNELS="k_max k_bsum k_bscan" scripts/gpu_ab_prof.sh base.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/abp_tests.log 2>&1
  rc=$?; tail -1 gpurun_out/abp_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/abp_tests.log | head -30; exit $rc; }
fi
for r in $(seq 1 ${ROUNDS:-2}); do
for v in tree "$@"; do
  if [ "$v" = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi
  O=gpurun_out/abp_${v}_$r
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python bench.py --config ${CFG:-c4} --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $O.log 2>&1 || { tail -20 $O.log; exit 1; }
  python - "$O" "$v" "${KERNELS}" <<'EOF'
import csv, json, sys
d, v, ks = sys.argv[1], sys.argv[2], sys.argv[3].split()
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
out = {}
for k in ks:
    for r in rows:
        if k in r["Name"]:
            out[k] = round(float(r["AverageNs"]) / 1e3, 2)
            break
line = open(f"{d}.log").read().strip().splitlines()[-1]
print(v, round(json.loads(line)["ms_per_step"], 4), out)
EOF
done
done
