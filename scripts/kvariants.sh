#!/bin/bash
# Compare conv-kernel variants (scripts/build_variant.py) on the fwd/dgrad layers:
#   bash scripts/kvariants.sh variants/libA.so variants/libB.so ...   (base = in-tree lib)
set -u
mkdir -p gpurun_out
OUT=gpurun_out/kvariants.log
: > $OUT
for lib in base "$@"; do
  echo "=== $lib" >> $OUT
  if [ "$lib" = base ]; then
    timeout -k 10 240 python scripts/kbench.py --math bf16x6 --iters 10 --ops ${KV_OPS:-fwd,dgrad} >> $OUT 2>&1 || exit $?
  else
    SPFF_LIB=$lib timeout -k 10 240 python scripts/kbench.py --math bf16x6 --iters 10 --ops ${KV_OPS:-fwd,dgrad} >> $OUT 2>&1 || exit $?
  fi
done
