#!/bin/bash
# rocprofv3 kernel stats of the swin bench for the in-tree lib and variant libs
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
i=0
for lib in base "$@"; do
  if [ "$lib" = base ]; then unset SPFF_LIB; else export SPFF_LIB=$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/av$i -o run --output-format csv -- python3 bench.py --workload swin --steps 2 --warmup 1 --cpu-baseline skip > gpurun_out/av$i.log 2>&1 || exit $?
  echo "$i $lib" >> gpurun_out/av_index.txt
  i=$((i+1))
done
