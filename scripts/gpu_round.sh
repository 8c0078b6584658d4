#!/bin/bash
# GPU-box runner: each GPU step under its own timeout; continue only after a
# clean exit (0) or an ordinary test failure (1).  Anything else (fault, abort,
# segfault, timeout) ends the call.  Usage: scripts/gpu_round.sh STEP...
#   STEP in: tests | smoke | bench | benchfull | prof | pmc
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
for step in "$@"; do
  case "$step" in
    tests) timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$? ;;
    sel) timeout -k 10 ${SEL_T:-900} python -u -m pytest ${SEL} -m gpu -v -s --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sel${SEL_TAG:-}.log 2>&1; rc=$? ;;
    dp) timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dp.log 2>&1; rc=$? ;;
    sizes) timeout -k 10 1000 python -u -m pytest tests/test_gpu_baseline_sizes.py -m gpu -x -v -s --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sizes.log 2>&1; rc=$? ;;
    memory) timeout -k 10 400 python -u -m pytest tests/test_gpu_memory.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_memory.log 2>&1; rc=$? ;;
    strong1) timeout -k 10 600 python bench.py --workload volume512 --strong --steps 2 --warmup 1 > gpurun_out/bench_strong1.log 2>&1; rc=$? ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$? ;;
    bench) timeout -k 10 600 python bench.py --steps 3 --warmup 1 --cpu-steps 1 > gpurun_out/bench_quick.log 2>&1; rc=$? ;;
    benchu3d) timeout -k 10 600 python bench.py --workload unet3d --steps 10 --warmup 3 > gpurun_out/bench_unet3d.log 2>&1; rc=$? ;;
    bench512) timeout -k 10 900 python bench.py --workload volume512 --steps 3 --warmup 1 > gpurun_out/bench512.log 2>&1; rc=$? ;;
    benchfull) timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1; rc=$? ;;
    prof) (cd "$GRAFT_REPO_ROOT" && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline skip > gpurun_out/prof.log 2>&1); rc=$? ;;
    pmc) (cd "$GRAFT_REPO_ROOT" && timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip > gpurun_out/pmc_fetch.log 2>&1 && timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline skip > gpurun_out/pmc_write.log 2>&1 && python scripts/pmc_traffic.py gpurun_out/pmc_fetch/run_counter_collection.csv gpurun_out/pmc_write/run_counter_collection.csv gpurun_out/pmc_conv.json gpurun_out/pmc_hbm_per_kernel.csv --bench-log gpurun_out/pmc_fetch.log > gpurun_out/pmc_traffic.log 2>&1); rc=$? ;;
    kbench) timeout -k 10 300 python scripts/kbench.py > gpurun_out/kbench.log 2>&1; rc=$? ;;
    kbx) (timeout -k 10 300 python scripts/kbench.py --math bf16x6 > gpurun_out/kbx.log 2>&1 && timeout -k 10 300 python scripts/kbench.py --math bf16x3 >> gpurun_out/kbx.log 2>&1); rc=$? ;;
    train) timeout -k 10 600 python -m pytest tests/test_gpu_train.py -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_train.log 2>&1; rc=$? ;;
    dskip) timeout -k 10 400 python scripts/dbg_math.py --no-stats --dskip > gpurun_out/dbg_dskip.log 2>&1; rc=$? ;;
    sharded) timeout -k 10 600 python -m pytest tests/test_gpu_sharded.py -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_sharded.log 2>&1; rc=$? ;;
    optim) timeout -k 10 300 python -m pytest tests/test_gpu_optim.py -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_optim.log 2>&1; rc=$? ;;
    parity) timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_parity.log 2>&1; rc=$? ;;
    unet3d) timeout -k 10 600 python -u -m pytest tests/test_gpu_unet3d.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_unet3d.log 2>&1; rc=$? ;;
    split) timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -k split > gpurun_out/pytest_split.log 2>&1; rc=$? ;;
    kpmc) (cd "$GRAFT_REPO_ROOT" && timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d gpurun_out/kpmc -o run -- python3 scripts/kbench.py --iters 1 --layers ${KPMC_LAYERS:-dec1} --math ${KPMC_MATH:-bf16x6} > gpurun_out/kpmc.log 2>&1 && timeout -k 10 600 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d gpurun_out/kpmc2 -o run -- python3 scripts/kbench.py --iters 1 --layers ${KPMC_LAYERS:-dec1} --math ${KPMC_MATH:-bf16x6} >> gpurun_out/kpmc.log 2>&1); rc=$? ;;
    swin) timeout -k 10 600 python -u -m pytest tests/test_gpu_swin.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_swin.log 2>&1; rc=$? ;;
    benchswin) timeout -k 10 600 python bench.py --workload swin --steps 10 --warmup 3 > gpurun_out/bench_swin.log 2>&1; rc=$? ;;
    profswin) (cd "$GRAFT_REPO_ROOT" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profswin -o run --output-format csv -- python3 bench.py --workload swin --steps 3 --warmup 1 --cpu-baseline skip > gpurun_out/profswin.log 2>&1); rc=$? ;;
    profu3d) (cd "$GRAFT_REPO_ROOT" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profu3d -o run --output-format csv -- python3 bench.py --workload unet3d --steps 3 --warmup 1 --cpu-baseline skip > gpurun_out/profu3d.log 2>&1); rc=$? ;;
    graph) timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-baseline skip --graph on > gpurun_out/bench_graph.log 2>&1; rc=$? ;;
    dry2) (timeout -k 10 400 python bench.py --gpus 2 --one-gpu --size 64 --steps 2 --warmup 1 > gpurun_out/dry2_patch.log 2>&1 && timeout -k 10 400 python bench.py --gpus 2 --one-gpu --workload unet3d --steps 2 --warmup 1 > gpurun_out/dry2_unet3d.log 2>&1); rc=$? ;;
    gprobe3) timeout -k 10 300 python -u scripts/graph_probe3.py f16x3 > gpurun_out/gprobe3.log 2>&1 && timeout -k 10 300 python -u scripts/graph_probe3.py f32 >> gpurun_out/gprobe3.log 2>&1; rc=$? ;;
    probe) timeout -k 10 600 python -u scripts/oracle_det_probe.py 4 > gpurun_out/oracle_det_probe.log 2>&1; rc=$? ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "[gpu_round] $step rc=$rc" | tee -a gpurun_out/steps.log
  ok $rc || { echo "[gpu_round] stopping after $step (rc=$rc)"; exit $rc; }
done
