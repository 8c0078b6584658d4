#!/bin/bash
# GPU call: quick f16x3 correctness of ONE variant library (op-level + reference fixtures,
# through SPFF_LIB), then the bench A/B of r03_abonly.sh against the in-tree library.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/abc
PT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider"
SPFF_LIB=$1 timeout -k 10 300 $PT tests/test_gpu_ops.py -m gpu -k "split or scaling" > gpurun_out/abc/ops.log 2>&1 || { echo "ops rc=$?"; exit 1; }
SPFF_LIB=$1 timeout -k 10 300 $PT tests/test_gpu_parity.py -m gpu -k "f16x3" > gpurun_out/abc/parity.log 2>&1 || { echo "parity rc=$?"; exit 1; }
bash scripts/r03_abonly.sh "$@"
