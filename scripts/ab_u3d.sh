#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload unet3d --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/abu_base_$rep.log 2>&1 || exit $?
  SPFF_LIB=variants/libspff_x32.so timeout -k 10 300 python bench.py --workload unet3d --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/abu_x32_$rep.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profu3d -o run --output-format csv -- python3 bench.py --workload unet3d --steps 3 --warmup 1 --cpu-baseline skip > gpurun_out/profu3d.log 2>&1
