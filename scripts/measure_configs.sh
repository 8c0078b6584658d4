#!/bin/bash
# One GPU call: the non-headline bench lines (3DUNet, SwinUNETR, registry layout, the whole
# 5 x 512^3 volume on one GPU) with their CPU baselines, plus a rocprofv3 kernel-stats pass
# of each of the first three, into gpurun_out/configs$ROUND.  Each GPU step under its own
# timeout; the call stops at the first failing step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/configs${ROUND:-}
rm -rf $O && mkdir -p $O
for w in unet3d swin registry; do
  echo "[configs] $w"
  timeout -k 10 500 python bench.py --workload $w > $O/bench_$w.log 2>&1 || { echo "bench $w rc=$?"; exit 1; }
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --cpu-baseline skip > $O/prof_$w.log 2>&1 || { echo "prof $w rc=$?"; exit 1; }
done
if [ "${STRONG:-1}" = 1 ]; then
  echo "[configs] volume512 strong"
  timeout -k 10 600 python bench.py --workload volume512 --strong --steps 2 --warmup 1 --cpu-baseline skip > $O/bench_strong1.log 2>&1 || { echo "strong rc=$?"; exit 1; }
fi
echo "[configs] done"
