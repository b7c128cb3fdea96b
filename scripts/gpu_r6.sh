#!/bin/bash
# Round-6 GPU driver (one MI355X).  Steps (space-separated in STEPS, run in order, each under its
# own time limit; the script stops at the first failure):
#   tests   the whole -m gpu suite (or TESTS=<pytest args>)
#   smoke   __graft_entry__.smoke()
#   diag    scripts/sort_diag.py on c5s and c4 (bucket sizes vs k_sort2 time)
#   ab      scripts/gpu_ab.sh: the tree library against the variants in VARIANTS (build/variants/*.so)
#   bench   the C4 bench line (and BENCH_CFGS configs)
#   prof    rocprofv3 kernel stats of the C4 bench (TAG names the profiles)
#   pmc     PMC passes of the C4 bench (scripts/pmc_kernels.sh)
#   phases  scripts/kernel_phases.py on the SPAI_PROF variant (build/variants/libspai_prof.so)
#   qrbench scripts/qr_fill_bench.py (the cached QR fill alone: M stored or not, batch sizes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r6}
O=gpurun_out/$TAG
mkdir -p $O
for st in ${STEPS:-tests bench}; do
  echo "== $st"
  case $st in
    tests)
      timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
        > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
      tail -1 $O/pytest.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    diag)
      for c in ${DIAG_CFGS:-c5s c4}; do
        timeout -k 10 300 python scripts/sort_diag.py --config $c --rollouts ${DIAG_N:-30} --out $O/sort_diag_$c.json \
          > $O/sd_$c.log 2>&1 || { tail -20 $O/sd_$c.log; exit 1; }
        tail -1 $O/sd_$c.log
      done ;;
    ab)
      TESTS= STEPS=30 ROUNDS=${ROUNDS:-3} bash scripts/gpu_ab.sh $VARIANTS || exit 1 ;;
    bench)
      for c in ${BENCH_CFGS:-c4}; do
        timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} \
          > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 1; }
        tail -1 $O/bench_$c.log | cut -c1-600
      done ;;
    prof)
      for c in ${PROF_CFGS:-c4}; do
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- \
          python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_$c.log 2>&1 \
          || { tail -20 $O/prof_$c.log; exit 1; }
      done ;;
    pmc)
      for c in ${PMC_CFGS:-c4}; do
        PMC_TIMEOUT=300 bash scripts/pmc_kernels.sh $O/pmc_$c python bench.py --config $c --steps 10 --warmup 2 \
          --no-cpu-baseline > $O/pmc_$c.log 2>&1 || { tail -20 $O/pmc_$c.log; exit 1; }
      done ;;
    qrbench)
      timeout -k 10 300 python scripts/qr_fill_bench.py --config ${QR_CFG:-c4} > $O/qr_fill_bench.log 2>&1 || { tail -20 $O/qr_fill_bench.log; exit 1; }
      cat $O/qr_fill_bench.log | grep '^{' ;;
    phases)
      SPAI_LIB_VARIANT=libspai_prof.so timeout -k 10 300 python scripts/kernel_phases.py > $O/phases.log 2>&1 || { tail -20 $O/phases.log; exit 1; }
      cat $O/phases.log ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
