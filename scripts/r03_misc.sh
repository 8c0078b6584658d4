#!/bin/bash
# One GPU call: per-kernel SQ counters of the default bench step (r03_pmcall.sh), then the
# 3DUNet and SwinUNETR workload bench lines with the default arithmetic.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/misc
bash scripts/r03_pmcall.sh || exit 1
timeout -k 10 300 python bench.py --workload unet3d --steps 10 --warmup 3 > gpurun_out/misc/bench_unet3d.log 2>&1 || { echo "unet3d rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --workload swin --steps 10 --warmup 3 > gpurun_out/misc/bench_swin.log 2>&1 || { echo "swin rc=$?"; exit 1; }

# A/B of the variant libraries given as arguments (bench.py, 20 steps, alternating, twice)
for rep in 1 2; do
  for lib in "" "$@"; do
    n=${lib:+$(basename "$lib" .so)}; n=${n:-base}
    SPFF_LIB=${lib:-spff-unet-spcct_amd/innovative3D/_lib/libspff_hip.so} timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline skip > gpurun_out/misc/ab_${n}_$rep.log 2>&1 || { echo "ab $n rc=$?"; exit 1; }
  done
done
echo "[r03_misc] ab done"
