#!/bin/bash
# One GPU call: the other bench workloads with the default arithmetic -- ONE 5 x 512^3 volume
# on one GPU (lean layout; the 1-GPU point of config 4's same-volume comparison) and the
# registry-layout batch.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/wl
timeout -k 10 600 python bench.py --workload volume512 --strong --steps 2 --warmup 1 --cpu-baseline skip > gpurun_out/wl/bench_strong1.log 2>&1 || { echo "strong rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --workload registry --batch 2 --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/wl/bench_registry.log 2>&1 || { echo "registry rc=$?"; exit 1; }
echo "[r03_workloads] done"
