#!/bin/bash
# Per-kernel A/B: rocprofv3 kernel stats of a short bench run with the in-tree lib and
# each variant lib given (one box); summaries -> gpurun_out/kst_<name>.txt
#   KST_PAT: regex of the kernel names to print (default: all, top 25)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in base "$@"; do
  n=$(basename "$lib" .so)
  rm -rf gpurun_out/kst_$n
  if [ "$lib" = base ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kst_$n -o run -- python3 bench.py --steps 4 --warmup 2 --cpu-baseline skip > gpurun_out/kst_$n.log 2>&1 || exit $?
  else
    SPFF_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kst_$n -o run -- python3 bench.py --steps 4 --warmup 2 --cpu-baseline skip > gpurun_out/kst_$n.log 2>&1 || exit $?
  fi
  f=$(find gpurun_out/kst_$n -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "${KST_PAT:-.}" > gpurun_out/kst_$n.txt <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
pat = re.compile(sys.argv[2])
rows = [r for r in rows if pat.search(r['Name'])]
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:25]:
    print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f}us {float(r['TotalDurationNs'])/6e6:8.3f}ms/step {r['Name'][:110]}")
PY
  echo "== $n"; cat gpurun_out/kst_$n.txt
  find gpurun_out/kst_$n -name "*.csv" ! -name "*kernel_stats.csv" -delete
done
