#!/bin/bash
# GPU call: per-layer kernel timings (scripts/kbench.py) of the in-tree library and of
# variant libraries (scripts/build_variant.py) on the same box, no bench runs.
#   KV_OPS=fwd bash scripts/r03_kdiag.sh variantA.so variantB.so ...
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/kdiag.log
: > $OUT
for lib in base "$@"; do
  echo "=== $lib" >> $OUT
  if [ "$lib" = base ]; then
    timeout -k 10 240 python scripts/kbench.py --math bf16x6 --iters 10 --ops ${KV_OPS:-fwd,dgrad,wgrad} >> $OUT 2>&1 || exit $?
  else
    SPFF_LIB=$lib timeout -k 10 240 python scripts/kbench.py --math bf16x6 --iters 10 --ops ${KV_OPS:-fwd,dgrad,wgrad} >> $OUT 2>&1 || exit $?
  fi
done
echo "[r03_kdiag] done"
