#!/bin/bash
# One GPU call for a library change: the GPU suite, an A/B of the workloads $AB_WORKLOADS
# (default: registry, 3DUNet) against the HEAD library (abvar/libspff_head.so, built by
# scripts/build_rev.py), then scripts/measure.sh (ROUND=$MROUND) for the patch bench line and
# its PMC key.  Used for the elementwise-grid floor (O=ew) and the weight-prep grids (O=pack).
# Each GPU step under its own timeout; the call stops at the first failing step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${O:-ew}
rm -rf $O && mkdir -p $O
echo "[ew] suite"
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "suite rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in 1 2 3; do
  for w in ${AB_WORKLOADS:-registry unet3d}; do
    for lib in new head; do
      if [ $lib = new ]; then
        timeout -k 10 200 python bench.py --workload $w --cpu-baseline skip > $O/tmp.log 2>&1 || { echo "bench $w $lib rc=$?"; tail -20 $O/tmp.log; exit 1; }
      else
        SPFF_LIB=abvar/libspff_head.so timeout -k 10 200 python bench.py --workload $w --cpu-baseline skip > $O/tmp.log 2>&1 || { echo "bench $w $lib rc=$?"; tail -20 $O/tmp.log; exit 1; }
      fi
      tail -1 $O/tmp.log >> $O/ab_${w}_${lib}.jsonl
      echo "round $r $w $lib: $(tail -1 $O/tmp.log | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3))')" | tee -a $O/ab_summary.txt
    done
  done
done
echo "[ew] measure"
ROUND=${MROUND:-5e} M3_KBENCH=0 bash scripts/measure.sh || exit 1
echo "[ew] done"
