#!/bin/bash
# A/B of whole-step time on ONE box: bench.py alternating between the in-tree library
# ("base") and variant libraries (SPFF_LIB), ROUNDS times; the JSON lines go to
# gpurun_out/ab_<i>.jsonl.  Usage: scripts/ab_bench.sh ROUNDS lib1 [lib2 ...]
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  i=0
  for lib in base "$@"; do
    if [ "$lib" = base ]; then
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/ab_tmp.log 2>&1 || exit $?
    else
      SPFF_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/ab_tmp.log 2>&1 || exit $?
    fi
    tail -1 gpurun_out/ab_tmp.log >> gpurun_out/ab_$i.jsonl
    echo "round $r lib $i ($lib): $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab_tmp.log').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3))")" | tee -a gpurun_out/ab_summary.txt
    i=$((i+1))
  done
done
