#!/bin/bash
# GPU call: correctness of the touched kernels, then conv-kernel A/B of variant libraries
# (scripts/build_variant.py) against the in-tree library on the same box.
#   bash scripts/r03_ab.sh [TESTS] -- variantA.so variantB.so ...
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${AB_TESTS:-"tests/test_gpu_ops.py tests/test_gpu_parity.py"}
if [ -n "$T" ]; then
  timeout -k 10 600 python -u -m pytest $T -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1
  t=$?; echo "tests rc=$t"; tail -2 gpurun_out/ab_tests.log
  [ $t -le 1 ] || exit $t
fi
OUT=gpurun_out/ab_kbench.log
: > $OUT
for lib in base "$@"; do
  [ -n "${KV_SKIP:-}" ] && break
  echo "=== $lib" >> $OUT
  if [ "$lib" = base ]; then
    timeout -k 10 240 python scripts/kbench.py --math bf16x6 --iters 10 --ops ${KV_OPS:-fwd,dgrad,wgrad} >> $OUT 2>&1 || exit $?
  else
    SPFF_LIB=$lib timeout -k 10 240 python scripts/kbench.py --math bf16x6 --iters 10 --ops ${KV_OPS:-fwd,dgrad,wgrad} >> $OUT 2>&1 || exit $?
  fi
done
for lib in base "$@"; do
  if [ "$lib" = base ]; then
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/ab_bench_base.log 2>&1 || exit $?
  else
    SPFF_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/ab_bench_$(basename $lib .so).log 2>&1 || exit $?
  fi
done
echo "[r03_ab] done"
