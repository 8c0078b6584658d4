#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: voxels/s of SPFF-UNet forward + loss +
backward (weight grads; optimizer step excluded, as in the metric's
definition) on a batch of 2 x 5-channel 128^3 patches (K=13,
base 32) per GPU, synthetic data resident in HBM before the timed region.

    python bench.py [--gpus N --steps K --warmup W]     (N > 1: starts its own N ranks)
    torchrun --nproc-per-node N bench.py --gpus N ...   (data parallel, RCCL)

With --gpus N > 1 and no launcher (WORLD_SIZE unset) the parent process starts N fresh
children with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set
(`launch_ranks`) before any device call and exits with the first non-zero child code.
Under a launcher, --gpus must equal WORLD_SIZE.

One process per GPU; N > 1 is batch data parallelism (weak scaling): each rank
runs its own batch, the valid-voxel count is all-reduced before the loss so
the CE mean is the global one, and the flat gradient is all-reduced (RCCL).
Rank 0 prints one JSON line.  The CPU baseline (rank 0, N=1) times the CPU
oracle (oracle/spff_oracle.py, PyTorch-CPU restatement of the reference path)
on the same batch on the host cores (all physical cores the process is allotted).
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
for _p in (str(ROOT), str(ROOT / "spff-unet-spcct_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from build_ext import build_record  # noqa: E402  (source digest the library was built from)

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 = f32 vector peak
# dense bf16 MFMA: 256 CUs x 4 SIMDs x 1024 flop/clk (32x32x16 in 32 cycles) x 2.4 GHz
BF16_MFMA_PEAK_TFLOPS = 256 * 4 * 1024 * 2.4e9 / 1e12
# fp32-equivalent peak of each conv arithmetic: bf16x6 runs 6 bf16 MFMA products per
# fp32 multiply-add, bf16x3 runs 3
MATH_PEAK = {"f32": FP32_MFMA_PEAK_TFLOPS, "bf16x6": BF16_MFMA_PEAK_TFLOPS / 6,
             "bf16x3": BF16_MFMA_PEAK_TFLOPS / 3, "f16x3": BF16_MFMA_PEAK_TFLOPS / 3}
# what each conv arithmetic is, in one line, with where its accuracy is measured
CONV_MATH_ACCURACY = {
    "f32": "fp32 MFMA (an fp32 fma chain)",
    "bf16x6": "fp32 operands split exactly into 3 bf16 planes, 6 products, fp32 accumulate",
    "bf16x3": "2 bf16 planes, 3 products (~2^-17 per product; opt-in)",
    "f16x3": ("each operand scaled by a power of two from its max |element| and split into 2 fp16 "
              "planes (<= 2^-22 |x|), 3 products, fp32 accumulate; measured against fp64: below "
              "the fp32 MFMA path's error in all 29 per-op cases and as close as it at config 2 "
              "(logits 1.2e-5, gradients <= 4.5e-5 rel. L2; profiles/r03/f16x3/)"),
}
MATH_KERNEL = {"f32": "k_conv3d_fwd (fp32 MFMA 3x3x3 implicit GEMM, fwd+dgrad)",
               "bf16x6": "k_conv3d_fwd_x<.,.,3> (3-plane split-bf16 MFMA 3x3x3 implicit GEMM, "
                         "fwd+dgrad)",
               "bf16x3": "k_conv3d_fwd_x<.,.,2> (2-plane split-bf16 MFMA 3x3x3 implicit GEMM, "
                         "fwd+dgrad)",
               "f16x3": "k_conv3d_fwd_x<.,.,12> (2-plane scaled-fp16 MFMA 3x3x3 implicit GEMM, "
                        "fwd+dgrad)"}
HBM_PEAK_GBS = 8000.0


def build_model(K, base, in_ch, D, device, seed=0):
    import innovative3D.models as M
    from innovative3D.weightgen import synth_state
    core = M.build_spct_energyfilm_fourier(num_classes=K, base=base, in_channels=in_ch)
    for b in core._blocks():
        b.fgate._ensure_mask(D, "cpu")
    st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=seed)
    core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    return core.to(device), st


def host_cpu_info():
    """Host CPU topology (lscpu-style): physical cores = distinct (package, core) pairs
    in /proc/cpuinfo; logical CPUs; the CPUs this process may run on; OMP_NUM_THREADS."""
    phys, logical = set(), 0
    try:
        pkg = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k = k.strip()
            if k == "processor":
                logical += 1
            elif k == "physical id":
                pkg = v.strip()
            elif k == "core id":
                core = v.strip()
                phys.add((pkg, core))
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    cg = cgroup_cpu_allotment()
    allot = [aff] + [v for v in (cg.get("quota_cpus"), cg.get("cpuset_cpus")) if v]
    return {"physical_cores": len(phys) or None, "logical_cpus": logical or os.cpu_count(),
            "affinity_cpus": aff, "omp_num_threads": omp or None, "cgroup": cg,
            "allotment_cpus": min(allot)}


def _cpulist_len(s):
    """number of CPUs in a kernel cpu-list string such as '0-15,32-47'"""
    n = 0
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        n += (int(b) - int(a) + 1) if b else 1
    return n


def cgroup_cpu_allotment():
    """This process's CPU allotment from its cgroup, walking from its own cgroup up to the
    root (the tightest limit wins): v2 `cpu.max` (quota / period) and
    `cpuset.cpus.effective`, or v1 `cpu.cfs_quota_us / cpu.cfs_period_us` and
    `cpuset.effective_cpus`.  Raw strings are kept as the record."""
    rec = {"version": None, "quota_cpus": None, "cpuset_cpus": None, "raw": {}}
    try:
        lines = open("/proc/self/cgroup").read().split("\n")
    except OSError:
        return rec
    base = pathlib.Path("/sys/fs/cgroup")
    v2 = [ln.split(":", 2)[2] for ln in lines if ln.startswith("0::")]
    quotas, cpusets = [], []
    if v2 and (base / "cgroup.controllers").exists():
        rec["version"] = 2
        p = base / v2[0].lstrip("/")
        chain = [p] + list(p.parents)
        for d in chain:
            if not str(d).startswith(str(base)):
                break
            try:
                q, per = (d / "cpu.max").read_text().split()[:2]
                rec["raw"].setdefault("cpu.max", []).append(f"{d}: {q} {per}")
                if q != "max":
                    quotas.append(int(q) / int(per))
            except (OSError, ValueError):
                pass
            try:
                s = (d / "cpuset.cpus.effective").read_text().strip()
                if s:
                    rec["raw"].setdefault("cpuset.cpus.effective", []).append(f"{d}: {s}")
                    cpusets.append(_cpulist_len(s))
            except (OSError, ValueError):
                pass
    else:
        rec["version"] = 1
        for ln in lines:
            parts = ln.split(":", 2)
            if len(parts) < 3:
                continue
            ctrls, path = parts[1].split(","), parts[2].lstrip("/")
            for c in ctrls:
                root = base / (c if (base / c).exists() else parts[1])
                d = root / path
                for dd in [d] + list(d.parents):
                    if not str(dd).startswith(str(root)):
                        break
                    try:
                        if c == "cpu":
                            q = int((dd / "cpu.cfs_quota_us").read_text())
                            per = int((dd / "cpu.cfs_period_us").read_text())
                            rec["raw"].setdefault("cfs", []).append(f"{dd}: {q} {per}")
                            if q > 0:
                                quotas.append(q / per)
                        elif c == "cpuset":
                            s = (dd / "cpuset.effective_cpus").read_text().strip()
                            rec["raw"].setdefault("cpuset", []).append(f"{dd}: {s}")
                            if s:
                                cpusets.append(_cpulist_len(s))
                    except (OSError, ValueError):
                        pass
    if quotas:
        rec["quota_cpus"] = max(1, int(min(quotas)))
    if cpusets:
        rec["cpuset_cpus"] = min(cpusets)
    return rec


def baseline_threads():
    """All physical cores the process may use ("the node's own host cores"):
    min(physical cores, the process's real CPU allotment = affinity mask, cgroup quota,
    cgroup cpuset).  OMP_NUM_THREADS is a per-GPU-share convention, not an allotment: it
    is reported, and timed as a second labelled figure (`per_gpu_share`)."""
    h = host_cpu_info()
    n = min(h["physical_cores"] or h["allotment_cpus"], h["allotment_cpus"])
    return max(1, n), h


def cpu_baseline(st, K, base, x_cpu, y_cpu, depth, steps):
    """Oracle (PyTorch-CPU restatement of the reference) fwd+loss+bwd on the host cores, on
    the SAME inputs the GPU run uses (BASELINE.md 'CPU baseline timing': x ~ N(0,1) seed 0,
    labels with 1 % ignore): the WHOLE config-2 batch by default (depth = 0), so nothing is
    extrapolated; `depth` > 0 restricts it to sample 0, depths [0, depth) (a debugging aid).
    Threads = min(physical cores, the process's real allotment: affinity, cgroup quota and
    cpuset; `baseline_threads`).  When OMP_NUM_THREADS (the box's per-GPU CPU share) is
    smaller, the same batch is also timed on that many threads as `per_gpu_share`."""
    from oracle import spff_oracle as O
    threads, host = baseline_threads()
    in_ch = x_cpu.shape[1]
    cfg = O.SpffCfg(in_ch=in_ch, num_classes=K, base=base)
    if depth and depth < x_cpu.shape[2]:
        x = x_cpu[0:1, :, :depth].contiguous()
        y = y_cpu[0:1, :depth].contiguous()
    else:
        x, y = x_cpu.contiguous(), y_cpu.contiguous()
    D = x.shape[2]
    st_d = {k: v for k, v in st.items() if not k.endswith("._mask")}
    # masks for the sample depth (all ones, as in the reference)
    import numpy as np
    for k in list(st_d):
        if k.endswith("freq_mask"):
            st_d[k] = np.ones((1, 1, D // 2 + 1, 1, 1), np.float32)
    P = O.params_from_state(st_d)
    vox = x.shape[0] * D * x.shape[3] * x.shape[4]
    full = x_cpu.shape[0] * x_cpu.shape[2] * x_cpu.shape[3] * x_cpu.shape[4]

    def timed(nthreads, nsteps, warm):
        torch.set_num_threads(nthreads)
        times = []
        for i in range(nsteps + warm):
            t0 = time.perf_counter()
            O.fwd_bwd(P, x, y, cfg)
            if i >= warm:
                times.append(time.perf_counter() - t0)
        return statistics.median(times), times

    med, times = timed(threads, steps, 1)
    shape = "x".join(map(str, x.shape))
    what = (f"the GPU run's whole batch ({shape}, synthetic_batch seed 0, K={K}, base {base}); "
            "no extrapolation") if vox == full else (
            f"sample 0, depths 0..{D - 1} of the GPU run's batch ({shape}) = 1/{full // vox} of "
            "the headline voxels")
    out = {"value": vox / med, "unit": "voxels/s", "cores": torch.get_num_threads(),
           "kind": "port", "host": host, "s_per_step": times, "voxels_per_step": vox,
           "threads_rule": "min(physical cores, allotment = min(affinity, cgroup quota, cgroup "
                           "cpuset))",
           "sample": f"oracle fwd+ce_plus_macro_dice+bwd on {what}; median of {steps} steps "
                     f"after 1 warm-up ({med:.2f} s/step) on {torch.get_num_threads()} threads"}
    share = host.get("omp_num_threads")
    if share and share < threads:
        med2, t2 = timed(share, 1, 1)
        out["per_gpu_share"] = {"value": vox / med2, "cores": share, "s_per_step": t2,
                                "note": "same batch on OMP_NUM_THREADS threads (the box's "
                                        "per-GPU CPU share convention)"}
    return out


def unet3d_flops(B, D, H, W, K, f=32, cin=1):
    """Algorithmic fwd+bwd FLOPs of one 3DUNet step at backbone shape B x D x H x W:
    3x3x3 convs (fwd, input grad except the first conv, weight grad), the 2x2x2
    ConvTransposes (x3) and the 1x1x1 head (x3, input grad included)."""
    fl = 0.0
    chans = [(cin, f), (f, 2 * f), (2 * f, 4 * f), (4 * f, 8 * f), (8 * f, 16 * f),
             (16 * f, 8 * f), (8 * f, 4 * f), (4 * f, 2 * f), (2 * f, f)]
    lvls = [0, 1, 2, 3, 4, 3, 2, 1, 0]
    for i, ((ci, co), l) in enumerate(zip(chans, lvls)):
        V = B * (D >> l) * (H >> l) * (W >> l)
        for a, b_ in ((ci, co), (co, co)):
            mm = 2.0 * V * a * b_ * 27
            fl += mm * (3 if not (i == 0 and a == ci) else 2)
    for u in range(4):
        Vlow = B * (D >> (4 - u)) * (H >> (4 - u)) * (W >> (4 - u))
        fl += 3 * 2.0 * Vlow * (16 * f >> u) * 8 * (8 * f >> u)
    fl += 3 * 2.0 * B * D * H * W * f * K
    return fl


def bench_unet3d(args, world, rank, device):
    """BASELINE configs[2]: the 3DUNet variant (Cicek3DUNet + depth adapter,
    registry "3DUNet") on batch 4 x 1 x 5 x 96 x 96 per GPU: train-mode forward,
    the wrapper's weighted CE, backward (optimizer excluded, as in the headline
    metric).  N > 1: batch data parallelism (per-replica BatchNorm statistics,
    synchronised BatchNorm (innovative3D.distributed.sync_batchnorm: the batch moments
    and the backward's per-channel sums all-reduced, so N ranks normalise exactly as one
    device on the N x 4 batch), global valid count, gradient all-reduce."""
    import innovative3D.models as M
    from innovative3D.weightgen import synth_state
    from innovative3D.synthetic import synthetic_batch
    from innovative3D.distributed import allreduce_gradients, global_valid_count, sync_batchnorm
    K, Bt, D0, HW = args.classes, 4, 5, 96
    m = M.LitCicek3DUNet_DepthAdapter_Published(num_classes=K)
    sd = m.state_dict()
    st = synth_state([(k, tuple(v.shape)) for k, v in sd.items()], seed=0)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    m = m.to(device).train()
    m.backbone.math = args.math
    sync_batchnorm(m)  # (world 1: nothing to synchronise)
    x, y = synthetic_batch(Bt, 1, D0, HW, HW, K, ignore_frac=0.01, seed=1000 + rank, device=device)
    params = list(m.parameters())

    def step():
        for q in params:
            q.grad = None
        logits = m(x)
        cnt = global_valid_count(y, 255) if world > 1 else None
        from innovative3D.models import _WeightedCE
        loss, _conf = _WeightedCE.apply(logits, y, K, 255, None) if cnt is None else \
            _weighted_ce_global(logits, y, K, cnt)
        loss.backward()
        allreduce_gradients(params)
        return loss

    def _weighted_ce_global(logits, y_, K_, cnt):
        from innovative3D import _engine as E

        class _F(torch.autograd.Function):
            @staticmethod
            def forward(ctx, lg):
                lcl = lg.permute(0, 2, 3, 4, 1).contiguous()
                out4, dl, conf = E.weighted_ce_forward(lcl, y_, K_, 255, None, count_override=cnt)
                ctx.dl = dl
                return out4[0]

            @staticmethod
            def backward(ctx, g):
                E.scale_(ctx.dl, g.reshape(1))
                return ctx.dl.permute(0, 4, 1, 2, 3)
        return _F.apply(logits), None

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    from innovative3D import _engine as E
    E.conv_prof_enable(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    cprof = E.conv_prof_collect()
    E.conv_prof_enable(False)
    ranks = rank_report(elapsed, args.steps, device) if world > 1 else None
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    vox = Bt * D0 * HW * HW
    value = world * vox * args.steps / elapsed
    fl = unet3d_flops(Bt, 16, HW, HW, K)
    out = {
        "metric": "voxels/sec fwd+bwd, 3DUNet variant (Cicek3DUNet + depth adapter 5->16->5), "
                  "1-ch 5x96x96 patches",
        "value": value, "unit": "voxels/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "conv_math": args.math,
        "data": "synthetic (x~N(0,1), labels U[0,K) with 1% ignore=255; weights from weightgen seed 0)",
        "config": {"workload": f"3DUNet fwd+weighted CE+bwd, batch {Bt} x 1ch x {D0} x {HW} x {HW} "
                               f"per GPU (backbone at 16 x {HW} x {HW}), K={K}, base 32, "
                               "BatchNorm train mode" + (", synchronised over the ranks"
                                                         if world > 1 else "") +
                               " (BASELINE configs[2])",
                   "global_batch": Bt * world, "shape": [Bt, 1, D0, HW, HW],
                   "parallelism": f"dp{world}"},
        "loss": float(loss.item()),
        "backbone_voxels_per_s": value * 16 / D0,
        "step_tflops": fl * world * args.steps / elapsed / 1e12 / world,
        "algorithmic_flops_per_step": fl,
        "roofline": conv_class_roofline(cprof, args.steps, args.math, elapsed / args.steps * 1e3),
        "cpu_baseline": None,
    }
    if ranks:
        out["ranks"] = ranks
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        out["cpu_baseline"] = cpu_baseline_unet3d(st, K, args.cpu_steps)
        out["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def conv_class_roofline(prof, steps, math, step_ms):
    """`roofline` of a workload whose step is not an SPFF plan (3DUNet, SwinUNETR): the 3x3x3
    fwd/dgrad conv launches (the same k_conv3d_fwd_x kernel as the headline's dominant
    kernel), timed live with HIP events on their stream by the library-wide conv profiler
    (spff_conv_prof_*), algorithmic fp32 flops 2 V Cin Cout 27 per launch; the weight
    gradient and each class's share of the step beside it."""
    prof = {k: v for k, v in prof.items() if k.startswith("conv_")}
    ms = prof["conv_fwd"][0] + prof["conv_dgrad"][0]
    fl = prof["conv_fwd"][1] + prof["conv_dgrad"][1]
    nl = prof["conv_fwd"][2] + prof["conv_dgrad"][2]
    achieved = fl / (ms * 1e-3) / 1e12 if ms > 0 else None
    peak = MATH_PEAK[math]
    return {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
            "frac": (achieved / peak) if achieved else None, "traffic": None,
            "kernel": MATH_KERNEL[math], "avg_launch_ms": ms / max(1, nl), "launches": int(nl),
            "algorithmic_flops_per_launch": fl / max(1, nl),
            "per_class_ms_per_step": {k: v[0] / steps for k, v in prof.items()},
            "per_class_tflops": {k: (v[1] / (v[0] * 1e-3) / 1e12 if v[0] > 0 else None)
                                 for k, v in prof.items()},
            "conv_share_of_step": sum(v[0] for v in prof.values()) / steps / step_ms,
            "note": ("3x3x3 conv classes timed by the library-wide conv profiler (HIP events "
                     "around each launch on its stream, spff_conv_prof_*); achieved = fwd + "
                     "dgrad algorithmic flops / their summed durations; traffic not "
                     "collected for this workload")}


def cpu_baseline_unet3d(st, K, steps):
    """unet3d_oracle (PyTorch-CPU restatement of the reference) fwd + weighted CE + bwd."""
    from oracle import unet3d_oracle as U
    from innovative3D.synthetic import synthetic_batch
    threads, _host = baseline_threads()
    torch.set_num_threads(threads)
    P, B = U.params_from_state(st)
    cfg = U.UNet3DCfg(num_classes=K, base=32, in_ch=1, target_depth=16)
    x, y = synthetic_batch(4, 1, 5, 96, 96, K, ignore_frac=0.01, seed=123)
    times = []
    for i in range(steps + 1):
        t0 = time.perf_counter()
        U.fwd_bwd(P, B, x, y, cfg)
        if i > 0:
            times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": 4 * 5 * 96 * 96 / med, "unit": "voxels/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"unet3d_oracle fwd+weighted CE+bwd on the full 4x1x5x96x96 batch; "
                      f"median of {steps} steps after 1 warm-up ({med:.2f} s/step)"}


def swin_flops(B, D, H, W, K, f=12, cin=1, heads=(1, 2, 4, 8), w=7, mlp=2.0):
    """Algorithmic fwd+bwd FLOPs of one SwinUNETR step (registry config) at input
    B x D x H x W: 3x3x3 / 1x1 convs of the residual blocks (fwd, input grad except
    on the network input, weight grad), the Swin stages' linear layers (x3), window
    attention over the padded windows (QK^T and PV: 4 n^2 C per window forward,
    8 n^2 C backward), transposed convs (x3), patch embedding (x2) and the head (x3)."""
    vol = lambda l: B * (D >> l) * (H >> l) * (W >> l)  # noqa: E731
    fl = 0.0
    rbs = [(0, cin, f, True), (1, f, f, False), (2, 2 * f, 2 * f, False), (3, 4 * f, 4 * f, False),
           (5, 16 * f, 16 * f, False), (4, 16 * f, 8 * f, False), (3, 8 * f, 4 * f, False),
           (2, 4 * f, 2 * f, False), (1, 2 * f, f, False), (0, 2 * f, f, False)]
    for L, ci, co, first in rbs:
        V = vol(L)
        fl += 2.0 * V * ci * co * 27 * (2 if first else 3) + 2.0 * V * co * co * 27 * 3
        if ci != co:
            fl += 2.0 * V * ci * co * (2 if first else 3)
    for s in range(4):
        T, C = vol(s + 1), f << s
        hid = int(C * mlp)
        fl += 3 * 2.0 * T * (3 * C * C + C * C + 2 * C * hid) + 3 * 2.0 * (T // 8) * 8 * C * 2 * C
        dims = [(D >> (s + 1)), (H >> (s + 1)), (W >> (s + 1))]
        ws = [min(w, d) for d in dims]
        nwin = B
        for d, k in zip(dims, ws):
            nwin *= -(-d // k)
        n = ws[0] * ws[1] * ws[2]
        fl += 12.0 * n * n * C * nwin
    for u, (ci, co) in enumerate(((16 * f, 8 * f), (8 * f, 4 * f), (4 * f, 2 * f), (2 * f, f),
                                  (f, f))):
        fl += 3 * 2.0 * vol(5 - u) * ci * 8 * co
    fl += 2 * 2.0 * vol(1) * 8 * cin * f + 3 * 2.0 * vol(0) * f * K
    return fl


def bench_swin(args, world, rank, device):
    """BASELINE configs[4]: the SwinUNETR variant (registry "SwinUNETR": MONAI 1.5.2
    SwinUNETR, feature 12, depths 1, heads 1/2/4/8, window 7) on batch 2 x 1 x 128^3
    per GPU: forward, the Lit loss (0.5 soft-Dice + 0.5 CE), backward (optimizer
    excluded).  N > 1: batch data parallelism with the gradient all-reduced."""
    import innovative3D.models as M
    from innovative3D.config import variant
    from innovative3D.weightgen import synth_state
    from innovative3D.synthetic import synthetic_batch
    from innovative3D.distributed import allreduce_gradients
    K, Bt, S_ = args.classes, 2, 128
    lit = variant("SwinUNETR")[1](num_classes=K)
    sd = lit.state_dict()
    st = synth_state([(k, tuple(v.shape)) for k, v in sd.items()
                      if not k.endswith("relative_position_index")], seed=0)
    sd.update({k: torch.from_numpy(v) for k, v in st.items()})
    lit.load_state_dict(sd)
    lit = lit.to(device)
    lit.model.model.math = args.math
    x, y = synthetic_batch(Bt, 1, S_, S_, S_, K, ignore_frac=0.01, seed=1000 + rank, device=device)
    params = list(lit.parameters())

    def step():
        for q in params:
            q.grad = None
        logits = lit(x)
        loss = M._SwinLoss.apply(logits, y, K, 255, False, 0.5)
        loss.backward()
        if world > 1:  # DDP semantics (the reference trains it under Lightning DDP): mean
            allreduce_gradients(params)
            for q in params:
                q.grad.div_(world)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    from innovative3D import _engine as E
    E.conv_prof_enable(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    cprof = E.conv_prof_collect()
    E.conv_prof_enable(False)
    ranks = rank_report(elapsed, args.steps, device) if world > 1 else None
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    vox = Bt * S_ ** 3
    value = world * vox * args.steps / elapsed
    fl = swin_flops(Bt, S_, S_, S_, K)
    out = {
        "metric": "voxels/sec fwd+bwd, SwinUNETR variant (MONAI 1.5.2 SwinUNETR, registry "
                  "settings), 1-ch 128^3 patches",
        "value": value, "unit": "voxels/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "conv_math": args.math,
        "data": "synthetic (x~N(0,1), labels U[0,K) with 1% ignore=255; weights from weightgen seed 0)",
        "config": {"workload": f"SwinUNETR fwd+0.5 softDice+0.5 CE+bwd, batch {Bt} x 1ch x {S_}^3 "
                               f"per GPU, K={K}, feature 12, depths (1,1,1,1), heads (1,2,4,8), "
                               "window 7 (BASELINE configs[4])",
                   "global_batch": Bt * world, "shape": [Bt, 1, S_, S_, S_],
                   "parallelism": f"dp{world}"},
        "loss": float(loss.item()),
        "step_tflops": fl * args.steps / elapsed / 1e12,
        "algorithmic_flops_per_step": fl,
        "parity": "unpinned (MONAI absent offline); engine vs the restated oracle: tests/test_gpu_swin.py",
        "roofline": conv_class_roofline(cprof, args.steps, args.math, elapsed / args.steps * 1e3),
        "cpu_baseline": None,
    }
    if ranks:
        out["ranks"] = ranks
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        out["cpu_baseline"] = cpu_baseline_swin(st, K, args.cpu_steps)
        out["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_swin(st, K, steps):
    """swin_oracle (PyTorch-CPU restatement) fwd + Lit loss + bwd on 1 x 1 x 128^3."""
    from oracle import swin_oracle as S
    from innovative3D.synthetic import synthetic_batch
    threads, _host = baseline_threads()
    torch.set_num_threads(threads)
    P = S.params_from_state(st, prefix="model.model.")
    cfg = S.SwinCfg(num_classes=K)
    x, y = synthetic_batch(1, 1, 128, 128, 128, K, ignore_frac=0.01, seed=123)
    times = []
    for i in range(steps + 1):
        t0 = time.perf_counter()
        S.fwd_bwd(P, x, y, cfg)
        if i > 0:
            times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": 128 ** 3 / med, "unit": "voxels/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"swin_oracle fwd+loss+bwd on 1x1x128^3 (half the batch); median of "
                      f"{steps} steps after 1 warm-up ({med:.2f} s/step)"}


def time_loss_pass(xshape, y, K, device, reps=10):
    """The loss pass (k_loss + its finaliser: K*4 B logits and an 8 B label read, K*4 B
    dlogits written per voxel -- SURVEY §8(d)'s fourth memory-bound pass), timed with HIP
    events on the stream it runs on, on channel-last logits of this step's shape and the
    step's labels, with the global valid count given as the data-parallel runner gives it.
    Outside the timed step (the engine's own call, same sizes)."""
    from innovative3D import _engine as E
    B, _c, D, H, W = xshape
    g = torch.Generator(device=device).manual_seed(7)
    lcl = torch.randn(B, D, H, W, K, device=device, generator=g)
    cnt = (y != 255).sum().reshape(1).to(torch.int64)
    E.ce_dice_forward(lcl, y, K, 255, 1e-6, cnt)
    torch.cuda.synchronize()
    # HIP events around the pass's own launches on its stream (the library-wide recorder:
    # class loss_pass = confusion zeroing + k_loss + finaliser, k_loss alone beside it), so
    # host-side gaps between the Python calls are not counted
    E.conv_prof_enable(True)
    for _ in range(reps):
        E.ce_dice_forward(lcl, y, K, 255, 1e-6, cnt)
    torch.cuda.synchronize()
    pr = E.conv_prof_collect()
    E.conv_prof_enable(False)
    ms = pr["loss_pass"][0] / max(1, pr["loss_pass"][2])
    mk = pr["k_loss"][0] / max(1, pr["k_loss"][2])
    by = float(B * D * H * W) * (K * 4 + 8 + K * 4)
    del lcl
    return {"achieved_GBps": by / (ms * 1e-3) / 1e9, "frac": by / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "ms_per_call": ms, "algorithmic_bytes_per_call": by,
            "k_loss_ms": mk, "k_loss_frac": by / (mk * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "note": ("timed after the step loop on logits of the step's shape (one call per "
                     "step): HIP events around the pass's launches (confusion zeroing, k_loss, "
                     "finaliser) on its stream, mean of the calls")}


def rank_report(elapsed_local, steps, device):
    """World size, backend and every rank's own ms/step (all ranks must call)."""
    t = torch.tensor([elapsed_local], dtype=torch.float64, device=device)
    ts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(ts, t)
    return {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()),
            "ms_per_step_by_rank": [float(v.item()) / steps * 1e3 for v in ts]}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, child_cmd=None, env=None):
    """`bench.py --gpus N` without an external launcher: start N FRESH child processes
    (`sys.executable bench.py <argv>`), one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR (127.0.0.1) / MASTER_PORT set, exactly what `torch.distributed.run` would
    set, then wait for all of them.  The parent never touches the GPU (no torch.cuda call
    before or after), so each child initialises HIP and RCCL on its own device.  Returns
    the first non-zero child exit code (in rank order), else 0; when one child fails the
    others are given the process-group timeout to fail their collectives, then killed."""
    import subprocess
    cmd = list(child_cmd or [sys.executable, str(pathlib.Path(__file__).resolve())]) + list(argv)
    base = dict(os.environ if env is None else env)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    base.setdefault("MASTER_PORT", str(_free_port()))
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                 LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", SPFF_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen(cmd, env=e))
    rcs = [None] * n
    deadline = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if deadline is None and any(rc not in (None, 0) for rc in rcs):
            deadline = time.time() + float(base.get("SPFF_BENCH_KILL_AFTER", "120"))
        if deadline is not None and time.time() > deadline:
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.kill()
                    rcs[i] = p.wait()
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--size", type=int, default=128, help="D = H = W")
    ap.add_argument("--in-ch", type=int, default=5)
    ap.add_argument("--classes", type=int, default=13)
    ap.add_argument("--base", type=int, default=32)
    ap.add_argument("--cpu-baseline", choices=("auto", "skip"), default="auto")
    ap.add_argument("--math", choices=("f32", "bf16x6", "bf16x3", "f16x3"), default="f16x3",
                    help="conv arithmetic: f16x3 (default) = each operand scaled by a power of "
                         "two from its max |element| and split into 2 fp16 planes, 3 products, "
                         "fp32 accumulate (measured as close to fp64 as the f32 path); bf16x6 = "
                         "3 exact bf16 planes, 6 products")
    ap.add_argument("--workload", choices=("patch128", "volume512", "registry", "unet3d", "swin"),
                    default="patch128",
                    help="patch128 = the headline (BASELINE configs[1]): batch data parallelism; "
                         "volume512 = BASELINE configs[3]: one 5 x (64 N) x 512 x 512 volume "
                         "depth-sharded over the N ranks (64-slice slab per rank, RCCL halos); "
                         "registry = one batch of --batch registry-layout volumes 1 x 5 x hw x hw "
                         "height-sharded over the N ranks (hw / N rows each; strong scaling); "
                         "unet3d = BASELINE configs[2]: the 3DUNet variant, batch 4 x 1 x 5 x 96^2; "
                         "swin = BASELINE configs[4]: the SwinUNETR variant, batch 2 x 1 x 128^3")
    ap.add_argument("--slab-depth", type=int, default=64)
    ap.add_argument("--strong", action="store_true",
                    help="volume512: strong scaling -- ONE 5 x D x 512 x 512 volume (D = "
                         "--volume-depth, 512 = the north star's volume) split into N slabs of "
                         "D / N; N = 1 runs it whole on one GPU (lean memory layout)")
    ap.add_argument("--volume-depth", type=int, default=512)
    ap.add_argument("--memory", choices=("auto", "full", "lean"), default="auto",
                    help="saved-activation layout (include/spff.h SPFF_MEM_*)")
    ap.add_argument("--hw", type=int, default=512)
    ap.add_argument("--one-gpu", action="store_true",
                    help="functional dry run: every rank on cuda:0 with host-staged gloo "
                         "collectives (e.g. 8 ranks of --workload volume512 --strong on a "
                         "1-GPU box); the timings are not a scaling measurement")
    ap.add_argument("--coll-timeout", type=float, default=600.0,
                    help="seconds before a collective is declared failed (process group timeout)")
    ap.add_argument("--cpu-depth", type=int, default=0,
                    help="0 (default) = time the CPU oracle on the whole batch; > 0 = sample 0, "
                         "depths [0, cpu-depth) only")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="time the step as a captured HIP graph replayed K times (one GPU, SPFF "
                         "workloads), the eager loop of the same K steps beside it; auto = on "
                         "for patch128 at N = 1.  The replay's loss must equal the eager "
                         "step's bit for bit, else value falls back to the eager time")
    ap.add_argument("--pmc", default=str(ROOT / "profiles" / "r06_pmc_conv.json"),
                    help="per-launch HBM traffic summary from rocprofv3 --pmc "
                         "(scripts/pmc_traffic.py); used only when its workload key matches")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            # no external launcher: start the N ranks here, before anything touches the GPU
            raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE="
                         f"{os.environ['WORLD_SIZE']} ranks")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("SPFF_BENCH_STUB") == "1":
        # launcher test hook (tests/test_bench_launch_cpu.py): report the rank layout and
        # stop before any device call
        print(json.dumps({"stub": True, "rank": rank, "local_rank": local, "world_size": world,
                          "launched": os.environ.get("SPFF_BENCH_LAUNCHED") == "1",
                          "master": [os.environ.get("MASTER_ADDR"),
                                     os.environ.get("MASTER_PORT")]}), flush=True)
        return
    if world > 1 and not args.one_gpu:
        n_dev = torch.cuda.device_count()  # does not initialise HIP on this image
        if local >= n_dev:
            raise SystemExit(f"bench.py: rank {rank} needs device {local}, {n_dev} visible")
    device = torch.device("cuda", 0 if args.one_gpu else local)
    torch.cuda.set_device(device)
    if world > 1:
        # a dead or wedged peer fails the collective after this long instead of hanging the
        # job (SURVEY §5 failure detection; the reference sets NCCL_ASYNC_ERROR_HANDLING)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        import datetime
        if args.one_gpu:  # RCCL refuses two ranks on one device: host-staged gloo
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.coll_timeout))
        else:
            dist.init_process_group("nccl", device_id=device,
                                    timeout=datetime.timedelta(seconds=args.coll_timeout))

    if args.graph == "on" and (world > 1 or args.workload in ("unet3d", "swin")):
        raise SystemExit("bench.py --graph on: one GPU, SPFF workloads")
    use_graph = args.graph == "on" or (args.graph == "auto" and world == 1 and
                                       args.workload == "patch128")
    if args.workload == "unet3d":
        return bench_unet3d(args, world, rank, device)
    if args.workload == "swin":
        return bench_swin(args, world, rank, device)

    from innovative3D.distributed import DataParallelSPFF
    from innovative3D.synthetic import synthetic_batch

    K = args.classes
    sharded = args.workload == "volume512"
    registry = args.workload == "registry"
    if registry:  # the registry layout [B, 1, 5, H, W] sharded along H
        from innovative3D.sharded import HeightShardedSPFF, height_bounds
        B, HW = args.batch, args.hw
        off, Hl = height_bounds(HW, world, rank)
        core, st = build_model(K, args.base, 1, 5, device)
        core.math = args.math
        core.memory = args.memory
        x, y = synthetic_batch(B, 1, 5, HW, HW, K, ignore_frac=0.01, seed=0)
        x = x[:, :, :, off:off + Hl].contiguous().to(device)
        y = y[:, :, off:off + Hl].contiguous().to(device)
        runner = HeightShardedSPFF(core, K, 255) if world > 1 else DataParallelSPFF(core, K, 255)
        vox_step = B * 5 * Hl * HW
    elif sharded:  # weak scaling: a fixed slab per rank, global depth = slab * world;
        # --strong: one volume of --volume-depth slices, D / world per rank
        from innovative3D.sharded import DepthShardedSPFF
        B, HW = 1, args.hw
        if args.strong:
            if args.volume_depth % world:
                raise SystemExit(f"--volume-depth {args.volume_depth} not divisible by {world}")
            Dl = args.volume_depth // world
        else:
            Dl = args.slab_depth
        core, st = build_model(K, args.base, args.in_ch, Dl * world, device)
        core.math = args.math
        core.memory = args.memory
        x, y = synthetic_batch(1, args.in_ch, Dl, HW, HW, K, ignore_frac=0.01, seed=1000 + rank,
                               device=device)
        runner = DepthShardedSPFF(core, K, 255) if world > 1 else DataParallelSPFF(core, K, 255)
        vox_step = Dl * HW * HW
    else:
        B, S = args.batch, args.size
        core, st = build_model(K, args.base, args.in_ch, S, device)
        core.math = args.math
        core.memory = args.memory
        # rank r's batch = synthetic_batch(seed r): rank 0 holds BASELINE.md's config-2
        # inputs (seed 0), the ones tests/test_gpu_baseline_sizes.py checks against the oracle
        x_cpu, y_cpu = synthetic_batch(B, args.in_ch, S, S, S, K, ignore_frac=0.01, seed=rank)
        x, y = x_cpu.to(device), y_cpu.to(device)
        runner = DataParallelSPFF(core, K, 255)
        vox_step = B * S * S * S

    def step():
        loss, _conf = runner.step(x, y)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    plan = core._plan

    def timed(fn, n):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = None
        for _ in range(n):
            r = fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0, r

    # 1. the timed region: K steps with nothing but the step's own launches in it (the
    #    per-class HIP events of 2. add a queue packet before and after every profiled launch,
    #    ~1 ms per step of gaps: measured separately, never inside the timed region)
    elapsed, loss = timed(step, args.steps)
    graph_rec = None
    if use_graph:
        # the step captured once into a HIP graph (torch.cuda.CUDAGraph over the engine's
        # launches: no host syncs, static shapes, the plan's workspace fixed) and replayed:
        # the same kernels, without the host round trips between them
        eager = elapsed
        try:
            side = torch.cuda.Stream(device)
            side.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(side):
                step()
            torch.cuda.current_stream(device).wait_stream(side)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                gloss = step()
            for _ in range(2):
                g.replay()
            g_elapsed, _ = timed(g.replay, args.steps)
            # the engine is deterministic: a replay on the same inputs reproduces the eager
            # step's loss bit for bit (tests/test_gpu_graph.py); anything else means the
            # capture missed work, and the eager time stands
            same = float(gloss) == float(loss)
            graph_rec = {"eager_ms_per_step": eager / args.steps * 1e3,
                         "graph_ms_per_step": g_elapsed / args.steps * 1e3,
                         "replay_loss_equals_eager": same,
                         "note": ("value = the graph replays" if same else
                                  "value = the EAGER loop: the replay's loss differed") +
                                 "; both loops without profiling events"}
            if same:
                elapsed, loss = g_elapsed, gloss
            else:
                print(f"bench.py: HIP-graph replay loss {float(gloss)!r} != eager {float(loss)!r}; "
                      "reporting the eager time", file=sys.stderr, flush=True)
        except RuntimeError as e:
            # a capture the runtime refuses: the eager loop above stands (and says why)
            torch.cuda.synchronize()
            graph_rec = {"eager_ms_per_step": eager / args.steps * 1e3, "error": repr(e)[:300],
                         "note": "value = the EAGER loop: the HIP-graph capture failed"}
            print(f"bench.py: HIP-graph capture failed ({e!r}); reporting the eager time",
                  file=sys.stderr, flush=True)

    # 2. per-class kernel timing: a separate pass of K eager steps with HIP events around the
    #    engine's launches on its stream (and, sharded, around the collective callbacks)
    plan.prof_enable(True)
    plan.prof_collect()
    plan.coll_timing = world > 1 and (sharded or registry)
    plan.coll_collect()
    prof_elapsed, _ = timed(step, args.steps)
    prof = plan.prof_collect()
    plan.prof_enable(False)
    coll = plan.coll_collect() if plan.coll_timing else {}
    plan.coll_timing = False
    elapsed_local = elapsed
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    value = world * vox_step * args.steps / elapsed

    # dominant kernel: the fwd/dgrad conv kernel (forward + input-grad convs), timed live
    ms = prof["conv_fwd"][0] + prof["conv_dgrad"][0]
    fl = prof["conv_fwd"][1] + prof["conv_dgrad"][1]
    nl = prof["conv_fwd"][2] + prof["conv_dgrad"][2]
    cb = prof["conv_fwd"][3] + prof["conv_dgrad"][3]
    achieved = fl / (ms * 1e-3) / 1e12 if ms > 0 else None
    # roofline.traffic: the PMC measurement is used only for the workload it was taken on
    # (scripts/pmc_traffic.py stores the bench line's workload_key); otherwise null
    if registry:
        shape = [B, 1, 5, HW, HW]
    elif sharded:
        shape = [1, args.in_ch, Dl * world, HW, HW]
    else:
        shape = [B, args.in_ch, S, S, S]
    wkey = {"workload": args.workload, "shape": shape, "classes": K, "base": args.base,
            "math": args.math, "n_gpus": world, "memory_layout": plan.layout}
    traffic, traffic_src = None, {"file": None, "matched": False}
    try:
        pm = json.loads(pathlib.Path(args.pmc).read_text())
        traffic_src["file"] = str(pathlib.Path(args.pmc).resolve().relative_to(ROOT))
        # the summary counts for THIS kernel build only: same workload key and the same
        # library sources (a kernel change makes a committed measurement stale -> null)
        same = pm.get("lib_sources_sha256") == build_record()["lib_sources_sha256"]
        traffic_src["same_sources"] = same
        if pm.get("workload_key") == wkey and same:
            traffic = pm.get("hbm_bytes_per_launch")
            traffic_src["matched"] = True
        else:
            traffic_src["pmc_workload_key"] = pm.get("workload_key")
    except Exception:
        pass
    peak = MATH_PEAK[args.math]
    roof = {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
            "frac": (achieved / peak) if achieved else None, "traffic": traffic,
            "kernel": MATH_KERNEL[args.math],
            "peak_note": ("algorithmic fp32 flops (2*V*Cin*Cout*27 per conv); peak = the "
                          f"{args.math} arithmetic's fp32-equivalent MFMA peak"
                          + ("" if args.math == "f32" else
                             f" = dense bf16 MFMA {BF16_MFMA_PEAK_TFLOPS:.0f} / "
                             f"{6 if args.math == 'bf16x6' else 3} products")),
            "frac_of_fp32_mfma_peak": (achieved / FP32_MFMA_PEAK_TFLOPS) if achieved else None,
            "avg_launch_ms": ms / max(1, nl), "launches": int(nl),
            "algorithmic_flops_per_launch": fl / max(1, nl),
            "compulsory_bytes_per_launch": cb / max(1, nl),
            "traffic_over_compulsory": (traffic / (cb / nl)) if (traffic and nl and cb) else None,
            "traffic_note": ("PMC HBM bytes per launch of this kernel (2 x FETCH_SIZE + WRITE_SIZE, "
                             "rocprofv3 --pmc passes of this same bench workload); null when the "
                             "summary's workload key or library sources differ from this run's"),
            "traffic_source": traffic_src,
            "per_class_ms_per_step": {k: v[0] / args.steps for k, v in prof.items()},
            "per_class_tflops": {k: (v[1] / (v[0] * 1e-3) / 1e12 if v[0] > 0 else None)
                                 for k, v in prof.items() if k not in plan.MEM_CLASSES},
            "step_tflops": value / world * 2462016 / 1e12}
    # the HBM-bound passes (each judged on its own algorithmic bytes =
    # operands read once + result written once), timed live like the conv kernels
    mem = {}
    tb = tm = 0.0
    for k in plan.MEM_CLASSES:
        ms_k, _f, n_k, by = prof[k]
        if ms_k > 0:
            gbs = by / (ms_k * 1e-3) / 1e9
            mem[k] = {"achieved_GBps": gbs, "frac": gbs / HBM_PEAK_GBS, "launches": int(n_k),
                      "algorithmic_bytes_per_launch": by / max(1, n_k),
                      "ms_per_step": ms_k / args.steps}
            tb += by
            tm += ms_k
    if not (sharded or registry):
        mem["loss"] = time_loss_pass(tuple(x.shape), y, K, device)
    roof["memory_bound"] = {
        "peak_GBps": HBM_PEAK_GBS, "kernels": mem,
        "aggregate": {"achieved_GBps": tb / (tm * 1e-3) / 1e9 if tm else None,
                      "frac": (tb / (tm * 1e-3) / 1e9 / HBM_PEAK_GBS) if tm else None},
        "note": ("slab_reduce = per-(b,c,d) hw-reductions (IN statistics, gate sums; C*4 B per "
                 "input tensor per voxel, incl. the split combine); act_apply = IN/gate apply "
                 "(8*C B/voxel); in_bwd_apply = IN backward apply (12*C B/voxel); HIP events "
                 "on the engine stream; loss = k_loss + finaliser (K*4 + 8 + K*4 B/voxel), not "
                 "in the aggregate")}
    if registry:
        cfg = {"workload": f"SPFF-UNet fwd+ce_plus_macro_dice+bwd, batch {B} x 1ch x 5 x {HW} x "
                           f"{HW} (registry layout) height-sharded into {world} x {Hl}-row slabs, "
                           f"K={K}, base {args.base}",
               "global_batch": B, "shape": [B, 1, 5, HW, HW], "parallelism": f"height{world}"}
        metric = f"voxels/sec fwd+bwd, SPFF-UNet registry layout {B}x1x5x{HW}x{HW}, " \
                 "height-sharded over N GPUs (strong scaling)"
    elif sharded:
        cfg = {"workload": f"SPFF-UNet fwd+ce_plus_macro_dice+bwd, one 1 x {args.in_ch}ch x "
                           f"{Dl * world} x {HW} x {HW} volume depth-sharded into {world} x "
                           f"{Dl}-slice slabs (BASELINE configs[3] at 8 GPUs), K={K}, base {args.base}",
               "global_batch": 1, "shape": [1, args.in_ch, Dl * world, HW, HW],
               "parallelism": f"depth{world}", "memory_layout": plan.layout,
               "workspace_GiB": plan.ws_bytes / 2 ** 30}
        metric = ("voxels/sec fwd+bwd, SPFF-UNet 5-ch volume depth-sharded (512^3 at 8 GPUs)"
                  if not args.strong else
                  f"voxels/sec fwd+bwd, SPFF-UNet one 5x{args.volume_depth}x{HW}x{HW} volume, "
                  f"depth-sharded over N GPUs (strong scaling)")
    else:
        cfg = {"workload": f"SPFF-UNet fwd+ce_plus_macro_dice+bwd, batch {B} x {args.in_ch}ch x "
                           f"{S}^3 per GPU, K={K}, base {args.base}",
               "global_batch": B * world, "shape": [B, args.in_ch, S, S, S],
               "parallelism": f"dp{world}"}
        metric = "voxels/sec fwd+bwd, SPFF-UNet 5-ch 128^3 patch"
    out = {
        "metric": metric,
        "value": value, "unit": "voxels/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if ((sharded and args.strong) or registry) else "weak",
        "vs_baseline": None,
        "dtype": "f32", "conv_math": args.math,
        "conv_math_accuracy": CONV_MATH_ACCURACY.get(args.math),
        "data": "synthetic (x~N(0,1), labels U[0,K) with 1% ignore=255; weights from weightgen seed 0)",
        "config": cfg,
        "workload_key": wkey,
        "loss": float(loss.item()),
        "roofline": roof,
        "cpu_baseline": None,
        "build": build_record(),
    }
    if graph_rec:
        out["hip_graph"] = graph_rec
    out["profiled_pass_ms_per_step"] = prof_elapsed / args.steps * 1e3
    if world > 1:
        out["ranks"] = rank_report(elapsed_local, args.steps, device)
        bk = getattr(runner, "bucketer", None)
        out["collectives"] = {
            "per_step": {k: {"calls": v["calls"] / args.steps, "ms": v["ms"] / args.steps,
                             "MB": v["bytes"] / args.steps / 1e6} for k, v in coll.items()},
            # the bucketed gradient all-reduces of the last step (issued during its backward)
            "grad_allreduce_buckets_last_step": len(bk.launched) if bk else None,
            "grad_allreduce_MB": (sum(b - a for a, b in bk.launched) * 4 / 1e6) if bk else None,
            "backend": dist.get_backend(),
            "note": ("HIP events around each spff_coll callback's work on its stream (rank 0); "
                     "halos on the side stream overlap the interior conv tiles, so their time "
                     "is the exchange's own duration" + ("; --one-gpu: every rank shares one "
                     "GPU through host-staged gloo, so these times are not a scaling "
                     "measurement" if args.one_gpu else ""))}
        out["f16_absmax_ms_per_step"] = prof["f16_absmax"][0] / args.steps
    if rank == 0 and world == 1 and args.cpu_baseline == "auto" and not (sharded or registry):
        out["cpu_baseline"] = cpu_baseline(st, K, args.base, x_cpu, y_cpu, args.cpu_depth,
                                           args.cpu_steps)
        out["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
        if "per_gpu_share" in out["cpu_baseline"]:
            out["gpu_over_cpu_per_gpu_share"] = value / out["cpu_baseline"]["per_gpu_share"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
