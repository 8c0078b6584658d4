set -e
mkdir -p gpurun_out
timeout -k 10 300 python scripts/dbg_dgrad_coherence.py > gpurun_out/dbg.log 2>&1
timeout -k 10 900 python scripts/dbg_cfg2_dskip64.py >> gpurun_out/dbg.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/bench_sa.log 2>&1
