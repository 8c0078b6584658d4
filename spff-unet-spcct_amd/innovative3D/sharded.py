"""Depth sharding of one volume across the GPUs of a node (BASELINE config 4:
a 5 x 512^3 volume, 8 x 64 depth slabs).

D is never pooled by the network (pools and up-convolutions act on H, W), so
rank r owns global depths [r * D_loc, (r + 1) * D_loc) at every level.  The
engine (include/spff.h, spff_cfg.shard_world / shard_rank) runs the path on its
slab and calls back, in stream order, for the only cross-slab couplings:

  * a one-slice halo per side before every 3x3x3 convolution (forward input,
    backward dy) -- ``halo``;
  * fp64 all-reduces of the InstanceNorm moments, the channel-SE pool, the
    partial rfft spectra of the FourierGate (forward s1, backward dw) and the
    SE gradient contraction -- ``allreduce``.

Height sharding (``HeightShardedSPFF``; SURVEY.md §8(e): "in the registry
layout (D = 5), shard H instead, in multiples of 8 rows") splits the registry
input [B, 1, 5, H, W] into row slabs of a multiple of 8 rows, so the three
(1,2,2) pools and the up-convolutions stay rank-local.  The engine
(spff_cfg.shard_axis = SPFF_SHARD_HEIGHT) exchanges one boundary ROW per side
before every 3x3x3 convolution through the same ``halo`` callback (a staging
slab of two rows per side), all-reduces the InstanceNorm moments as above, and
all-reduces the per-(b, c, d) gate sums (fp32), after which the EnergyFiLM /
FourierGate / SpectralSE / SE algebra is evaluated replicated (rank 0 keeps its
parameter gradients).  Any batch size.

The loss is normalised by the GLOBAL valid-voxel count and the flat weight
gradient is all-reduced once per step, as in innovative3D.distributed.  The
algorithm is pinned against the unsharded oracle by tests/test_sharded_cpu.py
(gloo, world 2 and 4) and the engine against the unsharded engine by
tests/test_gpu_sharded.py.
"""
from __future__ import annotations

import datetime

import torch
import torch.distributed as dist

from . import distributed as Dd


class TorchDepthColl:
    """spff_coll over a torch.distributed group.  Device tensors go straight to
    the backend (RCCL: all_reduce and batched point-to-point send / recv on the
    current stream); ``host_staged`` (default for gloo) copies through host
    memory, which lets several ranks share one GPU in tests.

    Failure detection: a host-staged exchange waits at most ``timeout``
    seconds for its peers and then raises, which the engine turns into a failed step
    (SPFF_ECOLL -> innovative3D._engine.SpffCollError naming the collective and the
    peer) instead of a hang.  Device (RCCL) collectives are stream-ordered -- blocking
    the host on them would serialise the halo exchange the engine overlaps with the
    interior tiles -- so they are bounded by the process group's own timeout
    (init_process_group(timeout=...), with TORCH_NCCL_ASYNC_ERROR_HANDLING=1, as
    bench.py / train.py set), whose watchdog fails the job when a peer stalls."""

    def __init__(self, group=None, host_staged=None, timeout: float = 300.0):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.host = (dist.get_backend(group) == "gloo") if host_staged is None else host_staged
        self.timeout = datetime.timedelta(seconds=float(timeout))

    def _peer(self, r):
        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def _wait(self, works, what: str) -> None:
        for w in works:
            try:
                ok = w.wait(timeout=self.timeout)
            except Exception as e:  # noqa: BLE001
                raise RuntimeError(f"rank {self.rank}: {what} did not complete within "
                                   f"{self.timeout.total_seconds():.0f} s ({e})") from e
            if ok is False:
                raise RuntimeError(f"rank {self.rank}: {what} did not complete within "
                                   f"{self.timeout.total_seconds():.0f} s")

    def allreduce(self, t: torch.Tensor) -> None:
        if self.host:
            c = t.cpu()
            self._wait([dist.all_reduce(c, group=self.group, async_op=True)],
                       f"all-reduce of {c.numel()} {str(c.dtype)[6:]} over {self.world} ranks")
            t.copy_(c)
        else:
            dist.all_reduce(t, group=self.group)

    def halo(self, slab: torch.Tensor, sl: int, d_local: int) -> None:
        """slab: [(d_local + 2) * sl] view -- [left halo | d_local slices | right halo]."""
        first, last = slab[sl:2 * sl], slab[d_local * sl:(d_local + 1) * sl]
        left, right = slab[:sl], slab[(d_local + 1) * sl:]
        r, w = self.rank, self.world
        if self.host:
            first_c, last_c = first.cpu(), last.cpu()
            left_c, right_c = torch.empty_like(first_c), torch.empty_like(first_c)
            ops = []
            if r > 0:
                ops += [dist.P2POp(dist.isend, first_c, self._peer(r - 1), self.group),
                        dist.P2POp(dist.irecv, left_c, self._peer(r - 1), self.group)]
            if r + 1 < w:
                ops += [dist.P2POp(dist.isend, last_c, self._peer(r + 1), self.group),
                        dist.P2POp(dist.irecv, right_c, self._peer(r + 1), self.group)]
            self._wait(dist.batch_isend_irecv(ops) if ops else [],
                       f"halo exchange with ranks {[q for q in (r - 1, r + 1) if 0 <= q < w]}")
            if r > 0:
                left.copy_(left_c)
            if r + 1 < w:
                right.copy_(right_c)
            return
        ops = []
        if r > 0:
            ops += [dist.P2POp(dist.isend, first.contiguous(), self._peer(r - 1), self.group),
                    dist.P2POp(dist.irecv, left, self._peer(r - 1), self.group)]
        if r + 1 < w:
            ops += [dist.P2POp(dist.isend, last.contiguous(), self._peer(r + 1), self.group),
                    dist.P2POp(dist.irecv, right, self._peer(r + 1), self.group)]
        for op in dist.batch_isend_irecv(ops) if ops else []:
            op.wait()


def _default_overlap(coll) -> bool:
    """Bucketed gradient all-reduces during the backward, interleaved with the halo
    exchanges.  On RCCL both go through the group's one communicator (batched
    point-to-point selects the device's collective communicator, as all_reduce does)
    and are issued from the host in the plan's fixed order, identical on every rank,
    so they cannot cross.  That path has only run host-staged (gloo) and at world 1
    on RCCL, so it stays opt-in for device collectives (SPFF_SHARD_OVERLAP=1) until a
    multi-GPU run has exercised it; without it the flat gradient is all-reduced once
    after the backward (allreduce_uncovered)."""
    import os
    if getattr(coll, "host", True):
        return True
    return os.environ.get("SPFF_SHARD_OVERLAP", "0") == "1"


def height_bounds(H: int, world: int, rank: int):
    """(offset, rows) of rank's slab of a height-H volume (H / world a multiple of 8)."""
    if H % (8 * world):
        raise ValueError(f"height {H} does not split into {world} slabs of a multiple of 8 rows")
    h = H // world
    return rank * h, h


def shard_bounds(D: int, world: int, rank: int):
    """(offset, depth) of rank's slab of a depth-D volume (D divisible by world)."""
    if D % world:
        raise ValueError(f"depth {D} not divisible by {world} shards")
    d = D // world
    return rank * d, d


class DepthShardedSPFF:
    """``step(x_slab, y_slab)``: forward of this rank's slab through the sharded
    engine, the global-count loss, backward and the flat gradient all-reduce.
    Returns (loss, confusion) with the hard-Dice term from the all-reduced
    confusion, i.e. the values of the unsharded step."""

    axis = 0  # SPFF_SHARD_DEPTH

    def __init__(self, core: torch.nn.Module, num_classes: int, ignore_index: int = 255,
                 group=None, coll=None, timeout: float = 300.0, bucket_bytes: int = 4 << 20,
                 overlap: bool | None = None):
        self.core, self.K, self.ignore, self.group = core, int(num_classes), ignore_index, group
        self.coll = coll or TorchDepthColl(group, timeout=timeout)
        if overlap is None:
            overlap = _default_overlap(self.coll)
        core.shard = (self.coll.world, self.coll.rank, self.axis)
        core.shard_coll = self.coll
        self.params = [p for p in core.parameters()]
        # the flat weight gradient is SUM-all-reduced in buckets WHILE the backward runs
        # (the engine's grad hook, as innovative3D.distributed.DataParallelSPFF does)
        self.bucketer = Dd.GradBucketer(group, bucket_bytes) if overlap else None

    def step(self, x: torch.Tensor, y: torch.Tensor):
        from .helpers import ce_dice_parts
        for p in self.params:
            p.grad = None
        hook = self.bucketer if self.coll.world > 1 else None
        begun = hook.begun if hook is not None else 0
        if hook is not None:
            hook.covered.clear()
        self.core.grad_hook = hook
        try:
            logits = self.core(x)
            self.last_logits = logits.detach()
            cnt = Dd.global_valid_count(y, self.ignore, self.group)
            loss_loc, conf, ce = ce_dice_parts(logits, y, self.K, self.ignore, count_override=cnt)
            loss_loc.backward()
        finally:
            self.core.grad_hook = None
        # whatever the bucketer did not cover (everything, if the plan never took the hook)
        Dd.allreduce_uncovered(self.params, hook if (hook is not None and hook.begun != begun)
                               else None, self.group)
        # the global value: summed CE shares + 0.5 * Dice of the summed confusion
        loss, _ce, conf_g = Dd.global_loss(ce, conf, self.K, group=self.group)
        return loss, conf_g


class HeightShardedSPFF(DepthShardedSPFF):
    """``step(x_slab, y_slab)`` on this rank's H-slab (``height_bounds``) of a
    registry-layout batch [B, 1, 5, H, W] / labels [B, 5, H, W]; same return
    values as the unsharded step."""

    axis = 1  # SPFF_SHARD_HEIGHT
