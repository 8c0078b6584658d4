#!/bin/bash
# One GPU call: quick f16x3 correctness (op-level + reference fixtures) of the in-tree
# library, then an A/B of bench.py between it and each variant library given (alternating,
# REPS times, one box).  Each GPU step under its own timeout; stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ab
rm -rf $O && mkdir -p $O
PT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT tests/test_gpu_ops.py -m gpu -k "split or scaling" > $O/ops.log 2>&1 || { echo "ops rc=$?"; exit 1; }
timeout -k 10 300 $PT tests/test_gpu_parity.py -m gpu -k "f16x3" > $O/parity.log 2>&1 || { echo "parity rc=$?"; exit 1; }
for rep in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline skip > $O/base_$rep.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    SPFF_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline skip > $O/${n}_$rep.log 2>&1 || { echo "bench $n rc=$?"; exit 1; }
  done
done
echo "[r03_ab] done"
