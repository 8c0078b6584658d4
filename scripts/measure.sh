#!/bin/bash
# One GPU call: default bench line, rocprofv3 kernel stats of the same command, per-layer
# conv kernel rates, and the two PMC traffic passes (FETCH_SIZE / WRITE_SIZE) keyed to
# the bench workload (scripts/pmc_traffic.py), into gpurun_out/m$ROUND (default 4).  Each GPU step under its own timeout;
# the call stops at the first failing step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/m${ROUND:-4}
rm -rf $O && mkdir -p $O
run() { echo "[measure] $1"; }
# (the profiler passes run the eager step: the same kernels as the graph replays the bench
# line times, each launch visible to the kernel trace and the counter collection)
PARGS="${BENCH_ARGS:-} --graph off"
run bench
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
run prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline skip ${PARGS} > $O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
if [ "${M3_KBENCH:-1}" = 1 ]; then
  run kbench
  timeout -k 10 300 python scripts/kbench.py --math ${KB_MATH:-f16x3} --iters 10 > $O/kbench.log 2>&1 || { echo "kbench rc=$?"; exit 1; }
fi
if [ "${M3_PMC:-1}" = 1 ]; then
  run pmc
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip ${PARGS} > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch rc=$?"; exit 1; }
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip ${PARGS} > $O/pmc_write.log 2>&1 || { echo "pmc write rc=$?"; exit 1; }
  python scripts/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/pmc_conv.json $O/pmc_hbm_per_kernel.csv --bench-log $O/pmc_fetch.log > $O/pmc_traffic.log 2>&1 || { echo "pmc_traffic rc=$?"; exit 1; }
fi
if [ "${M3_PMCALL:-0}" = 1 ]; then
  # SQ wave-state / MFMA-busy / LDS counters per kernel (two passes; scripts/pmc_summary.py)
  run pmcall
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $O/pmcall_a -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip ${PARGS} > $O/pmcall_a.log 2>&1 || { echo "pmcall a rc=$?"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $O/pmcall_b -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip ${PARGS} > $O/pmcall_b.log 2>&1 || { echo "pmcall b rc=$?"; exit 1; }
  python scripts/pmc_summary.py $O/pmcall_a/run_counter_collection.csv $O/pmcall_b/run_counter_collection.csv > $O/pmcall_summary.txt 2>&1
fi
echo "[measure] done"
