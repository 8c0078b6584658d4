"""Batch data parallelism for the SPFF engine: one process per GPU,
torch.distributed over RCCL ("nccl" backend on ROCm), xGMI between GPUs.

The reference trains on one device only (train.py:1486-1503); this
module is new.  Exactness argument: InstanceNorm, the FourierGate/SpectralSE
means and the channel-SE pool are all per sample, so a rank's forward on its
own samples is exactly the single-device forward restricted to them.  The
cross-sample couplings are the loss terms (DP row):

* the CE mean is normalised by the GLOBAL number of non-ignored voxels (one
  int64 all-reduce before the loss), so each rank's CE term is its share of
  the global mean and its dlogits are exactly the global-batch dlogits;
* the reported loss and hard-Dice (helpers.py:782-803, logged per step at
  models.py:486-507) come from ONE fp64 all-reduce of [CE share, K x (K+1)
  confusion counts] -- the global CE and the confusion of the whole batch, so
  the values equal the single-device ones (the Dice term carries no gradient);
* the weight gradient is a plain SUM over ranks.  It is all-reduced in
  buckets while the backward is still running: the engine reports each block's
  finished parameter-gradient range (spff_plan_set_grad_hook) in the order the
  backward completes them, and ``GradBucketer`` issues an async all-reduce of
  every contiguous run that has reached the bucket size.  RCCL's stream waits
  on the compute stream at issue time, so each all-reduce overlaps the
  remaining backward kernels.
"""
from __future__ import annotations

from typing import Callable, Iterable, List, Optional

import torch
import torch.distributed as dist

from . import _engine as E


def world(group=None) -> int:
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def _multi(group, force: bool = False) -> bool:
    """collectives are issued: more than one rank, or ``force`` on an initialised group"""
    if world(group) > 1:
        return True
    return bool(force) and dist.is_available() and dist.is_initialized()


def global_valid_count(labels: torch.Tensor, ignore_index: int = 255, group=None,
                       count_fn: Optional[Callable] = None, force: bool = False) -> torch.Tensor:
    """All-reduced number of labels != ignore_index (int64 tensor on labels' device).
    ``count_fn`` defaults to the HIP counting kernel."""
    cnt = (count_fn or E.count_valid)(labels, ignore_index)
    if _multi(group, force):
        dist.all_reduce(cnt, group=group)
    return cnt


def allreduce_gradients(params: Iterable[torch.nn.Parameter], group=None,
                        force: bool = False) -> None:
    """SUM-all-reduce every .grad with ONE collective over a flat buffer."""
    if not _multi(group, force):
        return
    gs: List[torch.Tensor] = [p.grad for p in params if p.grad is not None]
    if not gs:
        return
    flat = torch.cat([g.reshape(-1) for g in gs])
    dist.all_reduce(flat, group=group)
    o = 0
    for g in gs:
        n = g.numel()
        g.copy_(flat[o:o + n].view_as(g))
        o += n


def allreduce_confusion(conf: torch.Tensor, group=None) -> torch.Tensor:
    if world(group) > 1:
        dist.all_reduce(conf, group=group)
    return conf


def global_loss(ce_share: torch.Tensor, conf: torch.Tensor, num_classes: int,
                smooth: float = 1e-6, group=None, force: bool = False):
    """(loss, ce, conf) of the whole global batch from this rank's CE share (CE
    normalised by the global valid count) and its confusion counts, with one
    fp64 all-reduce and no host sync.  loss = fp32(ce) + fp32(0.5 * dice_loss),
    as the reference adds the python-float Dice term to the fp32 CE tensor
    (helpers.py:797-803)."""
    from .helpers import dice_loss_from_confusion_t
    K = int(num_classes)
    buf = torch.cat([ce_share.detach().reshape(1).to(torch.float64),
                     conf.detach().reshape(-1).to(torch.float64)])
    if _multi(group, force):
        dist.all_reduce(buf, group=group)
    ce = buf[0].to(torch.float32)
    conf_g = buf[1:].round().to(torch.int64).view(conf.shape)
    dice = dice_loss_from_confusion_t(conf_g, K, smooth)
    loss = ce + (0.5 * dice).to(torch.float32)
    return loss, ce, conf_g


class GradBucketer:
    """Overlaps the gradient all-reduce with the engine's backward.

    ``ready(off, n)`` is called (through the engine's grad hook, in stream
    order) when floats [off, off + n) of the flat gradient are final.  Adjacent
    ranges are merged; a merged run of >= ``bucket_bytes`` is all-reduced
    asynchronously at once.  ``finish()`` all-reduces what is left and makes the
    current stream wait for every collective."""

    def __init__(self, group=None, bucket_bytes: int = 4 << 20):
        self.group, self.bucket_floats = group, max(1, bucket_bytes // 4)
        self.flat: Optional[torch.Tensor] = None
        self.runs: List[list] = []        # pending [start, end, stream] runs, disjoint
        self.works = []
        self.launched: List[tuple] = []   # (start, end) of every issued all-reduce
        self.begun = 0                    # begin() calls (DataParallelSPFF checks coverage)
        self.covered = set()              # id() of the parameters whose gradient went through

    def begin(self, flat: torch.Tensor) -> None:
        self.flat, self.runs, self.works, self.launched = flat, [], [], []
        self.begun += 1

    def cover(self, param_ids) -> None:
        """called by the engine's autograd op after a backward through this bucketer:
        the parameters (ids) whose gradients the buckets all-reduced"""
        self.covered.update(param_ids)

    def abort(self) -> None:
        """Error exit of a backward that had begun: wait for the all-reduces already
        issued (peers that issued the same ones can complete them) and drop the rest."""
        works, self.works, self.runs = self.works, [], []
        for w in works:
            try:
                w.wait()
            except Exception:  # noqa: BLE001 -- the original error is what propagates
                pass

    def _stream_key(self):
        """the stream ready() was called on (device tensors; None on the host): a run's
        all-reduce is ordered after the work of the stream that reported it, so runs
        reported on different streams are never merged"""
        f = self.flat
        if f is None or not f.is_cuda:
            return None
        return torch.cuda.current_stream(f.device).cuda_stream

    def _launch(self, a: int, b: int, key=None) -> None:
        self.launched.append((a, b))
        f = self.flat
        if key is not None and key != self._stream_key():
            with torch.cuda.stream(torch.cuda.ExternalStream(key, device=f.device)):
                self.works.append(dist.all_reduce(f[a:b], group=self.group, async_op=True))
            return
        self.works.append(dist.all_reduce(f[a:b], group=self.group, async_op=True))

    def ready(self, off: int, n: int) -> None:
        a, b = int(off), int(off) + int(n)
        key = self._stream_key()
        keep = []
        for r in self.runs:
            if r[2] == key and r[1] == a:
                a = r[0]
            elif r[2] == key and r[0] == b:
                b = r[1]
            else:
                keep.append(r)
        if b - a >= self.bucket_floats:
            self.runs = keep
            self._launch(a, b, key)
        else:
            self.runs = keep + [[a, b, key]]

    def finish(self) -> None:
        for a, b, key in sorted(self.runs, key=lambda r: r[0]):
            self._launch(a, b, key)
        self.runs = []
        for w in self.works:
            w.wait()
        self.works = []


class DataParallelSPFF:
    """Minimal DDP for an engine module (SPFF core or any Lit wrapper): ``step(x, y)``
    runs forward, the global-count loss, backward with the bucketed, overlapped
    gradient all-reduce, and returns (loss, conf) of the GLOBAL batch -- the
    values a single device would report for the concatenated batch.

    The bucketer is attached as ``grad_hook`` to EVERY submodule (the engine reads it
    from whichever module calls its plan: the core, ``.backbone`` of the 3DUNet wrapper,
    ``.model.model`` of the Swin wrapper).  If no plan took the hook during a step
    (a backward that did not run through the engine), the gradients are all-reduced
    after the backward instead, so ranks can never keep unreduced gradients."""

    def __init__(self, module: torch.nn.Module, num_classes: int, ignore_index: int = 255,
                 group=None, bucket_bytes: int = 4 << 20, overlap: bool = True,
                 force_collectives: bool = False):
        """``force_collectives``: issue every collective even when the group has one rank
        (a world-1 RCCL group then runs the whole device path -- the count, the bucketed
        all-reduces on the engine's backward and the loss all-reduce -- on one GPU;
        tests/test_gpu_dp.py::test_rccl_world1_bucketed_step)."""
        self.module, self.K, self.ignore, self.group = module, int(num_classes), ignore_index, group
        self.force = bool(force_collectives)
        self.params = [p for p in module.parameters()]
        self.core = getattr(module, "model", module)
        self.bucketer = GradBucketer(group, bucket_bytes) if overlap else None

    def _set_hook(self, hook) -> None:
        for m in self.module.modules():
            m.grad_hook = hook

    def step(self, x: torch.Tensor, y: torch.Tensor):
        from .helpers import ce_dice_parts
        for p in self.params:
            p.grad = None
        n = world(self.group)
        multi = n > 1 or (self.force and dist.is_available() and dist.is_initialized())
        hook = self.bucketer if (multi and self.bucketer is not None) else None
        begun = hook.begun if hook is not None else 0
        if hook is not None:
            hook.covered.clear()
        self._set_hook(hook)
        try:
            logits = self.module(x)
            self.last_logits = logits.detach()
            cnt = global_valid_count(y, self.ignore, self.group, force=self.force) if multi else None
            loss_loc, conf, ce = ce_dice_parts(logits, y, self.K, self.ignore,
                                               count_override=cnt)
            loss_loc.backward()
        finally:
            self._set_hook(None)
        if multi:
            allreduce_uncovered(self.params, hook if (hook is not None and hook.begun != begun)
                                else None, self.group, force=self.force)
        if not multi:
            return loss_loc.detach(), conf
        loss, _ce, conf_g = global_loss(ce, conf, self.K, group=self.group, force=self.force)
        return loss, conf_g


def allreduce_uncovered(params: Iterable[torch.nn.Parameter], bucketer: Optional[GradBucketer],
                        group=None, force: bool = False) -> int:
    """All-reduce (one flat collective) every .grad the bucketer did NOT reduce during
    the backward: the parameters no engine op reported through ``bucketer.cover`` (a
    parameter of a wrapper outside the plan, or all of them when no plan took the
    hook).  Returns the number of tensors reduced here.  Every rank sees the same
    module structure and the same engine ops, so every rank issues the same call."""
    done = bucketer.covered if bucketer is not None else set()
    rest = [p for p in params if p.grad is not None and id(p) not in done]
    allreduce_gradients(rest, group, force=force)
    return len(rest)


def sync_batchnorm(module: torch.nn.Module, group=None, host_staged=None):
    """Synchronised BatchNorm for the 3DUNet variant's data parallelism: every engine
    BatchNorm3d of ``module`` (the Cicek3DUNet backbone, or the Lit wrapper around it)
    all-reduces its batch moments over ``group`` in the forward and its two per-channel
    sums in the backward (spff_unet3d_set_sync_bn), so a step on N ranks of B samples
    normalises exactly as one device on the N B-sample batch and every rank keeps the same
    running statistics (torch.nn.SyncBatchNorm semantics).  The
    BN weight / bias gradients stay per-rank partial sums, SUM-all-reduced with the rest of
    the gradient.  World 1: nothing to synchronise (returns None).  Returns the collective
    (innovative3D.sharded.TorchDepthColl: RCCL on device tensors, host-staged for gloo)."""
    from .sharded import TorchDepthColl
    if world(group) <= 1:
        for m in module.modules():
            if hasattr(m, "_bn_modules"):
                m.sync_bn = None
        return None
    coll = TorchDepthColl(group, host_staged=host_staged)
    n = 0
    for m in module.modules():
        if hasattr(m, "_bn_modules"):  # the engine backbone (models.Cicek3DUNet)
            m.sync_bn = coll
            n += 1
    if not n:
        raise ValueError("sync_batchnorm: no engine 3DUNet backbone in the module")
    return coll
