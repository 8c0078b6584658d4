#!/bin/bash
# rocprofv3 kernel stats of bench.py for the in-tree lib and each variant lib, one box
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
i=0
for lib in base "$@"; do
  if [ "$lib" = base ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline skip > gpurun_out/pv$i.log 2>&1 || exit $?
  else
    SPFF_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline skip > gpurun_out/pv$i.log 2>&1 || exit $?
  fi
  echo "$i $lib" >> gpurun_out/pv_index.txt
  i=$((i+1))
done
