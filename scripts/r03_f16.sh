#!/bin/bash
# One GPU call for the f16x3 conv arithmetic: op-level accuracy vs fp64 (and the operand
# scaling far outside fp16's range), whole-network parity on the reference fixtures,
# per-layer kernel rates, the bench line of both arithmetics, and the config-2 oracle
# test.  Each GPU step under its own timeout; the call stops at the first failing step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/f16
rm -rf $O && mkdir -p $O
step() { echo "[r03_f16] $1 $(date +%T)"; }
PT="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider"
step ops
timeout -k 10 300 $PT tests/test_gpu_ops.py -m gpu -k "split or scaling" > $O/ops.log 2>&1 || { echo "ops rc=$?"; exit 1; }
step parity
timeout -k 10 400 $PT tests/test_gpu_parity.py -m gpu -k "f16x3" > $O/parity.log 2>&1 || { echo "parity rc=$?"; exit 1; }
if [ "${F16_KBENCH:-0}" = 1 ]; then
  step kbench
  timeout -k 10 300 python scripts/kbench.py --math f16x3 --iters 10 > $O/kbench_f16x3.log 2>&1 || { echo "kbench rc=$?"; exit 1; }
  timeout -k 10 300 python scripts/kbench.py --math bf16x6 --iters 10 > $O/kbench_bf16x6.log 2>&1 || { echo "kbench rc=$?"; exit 1; }
fi
step bench
timeout -k 10 300 python bench.py --math f16x3 --cpu-baseline skip > $O/bench_f16x3.log 2>&1 || { echo "bench rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --cpu-baseline skip > $O/bench_bf16x6.log 2>&1 || { echo "bench rc=$?"; exit 1; }
step prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --math f16x3 --steps 3 --warmup 1 --cpu-baseline skip > $O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
if [ "${F16_SIZES:-1}" = 1 ]; then
  step sizes
  timeout -k 10 900 $PT tests/test_gpu_baseline_sizes.py -m gpu -k "config2 and f16x3" > $O/sizes.log 2>&1 || { echo "sizes rc=$?"; exit 1; }
fi
step done
