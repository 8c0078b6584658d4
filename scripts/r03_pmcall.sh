#!/bin/bash
# GPU call: SQ wave-state / MFMA / LDS counters of every kernel of one bench step (two
# separate --pmc passes), summarised per kernel by scripts/pmc_summary.py.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pmcall
mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $O/a -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip ${BENCH_ARGS:-} > $O/a.log 2>&1 || { echo "pass a rc=$?"; tail -5 $O/a.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $O/b -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip ${BENCH_ARGS:-} > $O/b.log 2>&1 || { echo "pass b rc=$?"; tail -5 $O/b.log; exit 1; }
python scripts/pmc_summary.py $O/a/run_counter_collection.csv $O/b/run_counter_collection.csv > $O/summary.txt 2>&1

echo "[r03_pmcall] done"
