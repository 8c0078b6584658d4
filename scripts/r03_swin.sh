#!/bin/bash
# GPU call: SwinUNETR tests on the MFMA window attention, then bench --workload swin with
# the MFMA kernels and with the VALU kernels (SPFF_ATTN_VALU=1) on the same box.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_swin.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/swin_tests.log 2>&1
t=$?; echo "swin tests rc=$t"; tail -2 gpurun_out/swin_tests.log
[ $t -le 1 ] || exit $t
timeout -k 10 300 python bench.py --workload swin --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/swin_bench_mfma.log 2>&1 || exit $?
SPFF_ATTN_VALU=1 timeout -k 10 300 python bench.py --workload swin --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/swin_bench_valu.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/swin_prof -o run --output-format csv -- python3 bench.py --workload swin --steps 3 --warmup 1 --cpu-baseline skip > gpurun_out/swin_prof.log 2>&1 || exit $?
echo "[r03_swin] done"
