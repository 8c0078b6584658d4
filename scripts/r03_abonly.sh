#!/bin/bash
# A/B only: bench.py (20 steps) with the in-tree library and each variant library given,
# alternating, REPS times, one box.  Each run under its own timeout; stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/abo
rm -rf $O && mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for lib in "" "$@"; do
    n=${lib:+$(basename "$lib" .so)}; n=${n:-base}
    SPFF_LIB=${lib:-spff-unet-spcct_amd/innovative3D/_lib/libspff_hip.so} timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline skip > $O/${n}_$rep.log 2>&1 || { echo "ab $n rc=$?"; exit 1; }
  done
done
echo "[r03_abonly] done"
