#!/bin/bash
# A/B: bench.py (10 steps) with the in-tree lib and each variant lib given, twice, one box
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/abv_base_$rep.log 2>&1 || exit $?
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    SPFF_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/abv_${n}_$rep.log 2>&1 || exit $?
  done
done
