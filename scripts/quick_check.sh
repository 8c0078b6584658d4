#!/bin/bash
# GPU box: conv op tests + small-fixture parity, one bench line, one FETCH_SIZE pass
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/qc_tests.log 2>&1 || { echo "tests rc=$?"; tail -5 gpurun_out/qc_tests.log; exit 1; }
tail -1 gpurun_out/qc_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/qc_bench.log 2>&1 || exit $?
if [ "${QC_PMC:-1}" = 1 ]; then
  rm -rf gpurun_out/qc_fetch
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/qc_fetch -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip > gpurun_out/qc_fetch.log 2>&1 || exit $?
fi
