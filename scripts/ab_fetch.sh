#!/bin/bash
# Per-kernel HBM read A/B: one rocprofv3 --pmc FETCH_SIZE pass of a 1-step bench per lib
# (in-tree lib + each variant lib given); conv-kernel summary -> gpurun_out/abf_<name>.txt
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in base "$@"; do
  n=$(basename "$lib" .so)
  rm -rf gpurun_out/abf_$n
  if [ "$lib" = base ]; then
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/abf_$n -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip > gpurun_out/abf_$n.log 2>&1 || exit $?
  else
    SPFF_LIB=$lib timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/abf_$n -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip > gpurun_out/abf_$n.log 2>&1 || exit $?
  fi
  f=$(find gpurun_out/abf_$n -name "*counter_collection.csv" | head -1)
  python3 - "$f" > gpurun_out/abf_$n.txt <<'PY'
import collections, csv, sys
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] == "FETCH_SIZE" and "k_conv3d" in r["Kernel_Name"]:
        acc[r["Kernel_Name"].split("(")[0]].append(2 * float(r["Counter_Value"]) * 1024)
for k, v in sorted(acc.items()):
    print(f"{len(v):4d} {sum(v) / len(v) / 1e9:7.3f} GB/launch (2 x FETCH) {k}")
PY
  echo "== $n"; cat gpurun_out/abf_$n.txt
  rm -rf gpurun_out/abf_$n
done
