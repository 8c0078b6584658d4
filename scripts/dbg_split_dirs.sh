#!/bin/bash
# diagnostics: f32 vs split-bf16 engine on a fixture with the split limited to one direction
set -u
mkdir -p gpurun_out
timeout -k 10 300 python scripts/dbg_math.py --no-stats > gpurun_out/dbg_dir_both.log 2>&1 &&
SPFF_DEBUG_SPLIT=fwd timeout -k 10 300 python scripts/dbg_math.py --no-stats > gpurun_out/dbg_dir_fwd.log 2>&1 &&
SPFF_DEBUG_SPLIT=dgrad timeout -k 10 300 python scripts/dbg_math.py --no-stats > gpurun_out/dbg_dir_dgrad.log 2>&1
