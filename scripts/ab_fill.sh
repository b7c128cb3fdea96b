#!/bin/bash
# A/B of the fill kernel: fill_bench per variant (tree = the in-tree library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  if [ "$v" = tree ]; then unset SPAI_LIB_VARIANT; else export SPAI_LIB_VARIANT=$v; fi
  echo "== $v"
  timeout -k 10 200 python scripts/fill_bench.py --config ${CFG:-c4} --batches ${BATCHES:-8} --iters 20 || exit 1
done
