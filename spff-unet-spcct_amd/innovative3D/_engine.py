"""ctypes binding of libspff_hip.so (include/spff.h) + the torch glue around it.

There is deliberately no CPU / PyTorch fallback: if the HIP library is
missing or the tensors are not on a ROCm device, every entry point raises.
"""
from __future__ import annotations

import collections
import ctypes
import os
import pathlib
import threading
import weakref
from typing import Dict, List, Optional, Tuple

import torch

_LIB_PATH = pathlib.Path(__file__).resolve().parent / "_lib" / "libspff_hip.so"
_lib = None
_lib_lock = threading.Lock()


class SpffError(RuntimeError):
    pass


class SpffCollError(SpffError):
    """A shard-group collective (spff_coll callback: halo exchange or all-reduce) failed,
    e.g. a peer rank died or timed out; the engine returned SPFF_ECOLL."""


SPFF_ECOLL = -4


class spff_cfg(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int), ("in_ch", ctypes.c_int), ("depth", ctypes.c_int),
        ("height", ctypes.c_int), ("width", ctypes.c_int), ("num_classes", ctypes.c_int),
        ("base", ctypes.c_int), ("ksd", ctypes.c_int), ("use_efilm", ctypes.c_int),
        ("use_fgate", ctypes.c_int), ("use_se", ctypes.c_int), ("use_specse", ctypes.c_int),
        ("math", ctypes.c_int), ("shard_world", ctypes.c_int), ("shard_rank", ctypes.c_int),
        ("memory_mode", ctypes.c_int), ("shard_axis", ctypes.c_int),
        ("efilm_hidden", ctypes.c_int), ("efilm_pe_dims", ctypes.c_int),
        ("fgate_learn_phase", ctypes.c_int),
    ]


class spff_unet3d_cfg(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int), ("in_ch", ctypes.c_int), ("depth", ctypes.c_int),
        ("height", ctypes.c_int), ("width", ctypes.c_int), ("target_depth", ctypes.c_int),
        ("num_classes", ctypes.c_int), ("base", ctypes.c_int), ("math", ctypes.c_int),
        ("reserved", ctypes.c_int * 7),
    ]


class spff_swin_cfg(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int), ("in_ch", ctypes.c_int), ("depth", ctypes.c_int),
        ("height", ctypes.c_int), ("width", ctypes.c_int), ("num_classes", ctypes.c_int),
        ("feature_size", ctypes.c_int), ("window", ctypes.c_int), ("heads", ctypes.c_int * 4),
        ("mlp_ratio", ctypes.c_float), ("math", ctypes.c_int), ("reserved", ctypes.c_int * 6),
    ]


# spff_coll (include/spff.h): the shard group's collectives, called back by the engine
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.c_int, ctypes.c_void_p)
HALO_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                           ctypes.c_int, ctypes.c_void_p)


class spff_coll(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("allreduce", ALLREDUCE_FN), ("halo", HALO_FN)]


# spff_grad_ready_fn (include/spff.h): dparams[off, off + n) final during spff_backward
GRAD_READY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_void_p)


# saved-activation layout (include/spff.h SPFF_MEM_*)
MEMORY_MODES = {"auto": 0, "full": 1, "lean": 2}


def default_memory() -> str:
    """Saved-activation layout for new plans: $SPFF_MEMORY, else "auto" (lean from 2^26
    voxels per plan)."""
    m = os.environ.get("SPFF_MEMORY", "auto")
    if m not in MEMORY_MODES:
        raise SpffError(f"SPFF_MEMORY={m!r}: expected one of {sorted(MEMORY_MODES)}")
    return m


# conv arithmetic (include/spff.h SPFF_MATH_*)
MATH_F32, MATH_BF16X6, MATH_BF16X3, MATH_F16X3 = 0, 1, 2, 3
MATH_NAMES = {"f32": MATH_F32, "bf16x6": MATH_BF16X6, "bf16x3": MATH_BF16X3,
              "f16x3": MATH_F16X3}


def default_math() -> str:
    """Conv arithmetic for new plans: $SPFF_MATH, else "f16x3" (scaled fp16 planes, measured
    as close to fp64 as the fp32 MFMA path)."""
    m = os.environ.get("SPFF_MATH", "f16x3")
    if m not in MATH_NAMES:
        raise SpffError(f"SPFF_MATH={m!r}: expected one of {sorted(MATH_NAMES)}")
    return m


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_S = ctypes.c_size_t

_SIGS = {
    "spff_plan_create": (_I, [ctypes.POINTER(spff_cfg), ctypes.POINTER(_P)]),
    "spff_plan_set_coll": (_I, [_P, ctypes.POINTER(spff_coll)]),
    "spff_plan_destroy": (None, [_P]),
    "spff_plan_set_grad_hook": (_I, [_P, GRAD_READY_FN, _P]),
    "spff_last_error": (ctypes.c_char_p, []),
    "spff_num_params": (_I, [_P]),
    "spff_param_info": (_I, [_P, _I, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_I),
                             ctypes.POINTER(_L), ctypes.POINTER(_L), ctypes.POINTER(_L)]),
    "spff_param_floats": (_L, [_P]),
    "spff_workspace_bytes": (_S, [_P]),
    "spff_forward": (_I, [_P, _P, _P, _P, _P, _P]),
    "spff_backward": (_I, [_P, _P, _P, _P, _P, _P]),
    "spff_saved_tensor": (_I, [_P, _P, ctypes.c_char_p, ctypes.POINTER(_P), ctypes.POINTER(_L),
                               ctypes.POINTER(_I)]),
    "spff_debug_set": (_I, [_P, _I, _I]),
    "spff_prof_enable": (_I, [_P, _I]),
    "spff_prof_collect": (_I, [_P, ctypes.POINTER(ctypes.c_double), _I]),
    "spff_upconv_ws_bytes": (ctypes.c_size_t, [_I, _I, _I, _I, _I, _I]),
    "spff_upconv_fwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "spff_upconv_dgrad": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "spff_upconv_wgrad": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "spff_unet3d_set_sync_bn": (_I, [_P, _P, _I]),
    "spff_conv_prof_enable": (_I, [_I]),
    "spff_conv_prof_collect": (_I, [ctypes.POINTER(ctypes.c_double), _I]),
    "spff_loss_ws_bytes": (_S, [_L, _I]),
    "spff_loss": (_I, [_P, _P, _L, _I, _I, ctypes.c_double, _P, _P, _P, _P, _P, _P]),
    "spff_confusion": (_I, [_P, _P, _L, _I, _I, _P, _P]),
    "spff_count_valid": (_I, [_P, _L, _I, _P, _P]),
    "spff_scale": (_I, [_P, _L, _P, _P]),
    "spff_conv3d_ws_bytes": (_S, [_I, _I, _I, _I, _I, _I, _I]),
    "spff_conv3d_fwd": (_I, [_P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "spff_conv3d_dgrad": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "spff_adam_step": (_I, [_P, _P, _P, _P, _L, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                            ctypes.c_double, ctypes.c_double, _I, _L, _P]),
    "spff_conv3d_fwd_ex": (_I, [_P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "spff_conv3d_dgrad_ex": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "spff_conv3d_wgrad_ex": (_I, [_P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "spff_conv3d_wgrad": (_I, [_P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    # 3DUNet baseline variant (BASELINE config 3)
    "spff_unet3d_create": (_I, [ctypes.POINTER(spff_unet3d_cfg), ctypes.POINTER(_P)]),
    "spff_unet3d_destroy": (None, [_P]),
    "spff_unet3d_num_params": (_I, [_P]),
    "spff_unet3d_param_info": (_I, [_P, _I, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_I),
                                    ctypes.POINTER(_L), ctypes.POINTER(_L), ctypes.POINTER(_L)]),
    "spff_unet3d_param_floats": (_L, [_P]),
    "spff_unet3d_num_buffers": (_I, [_P]),
    "spff_unet3d_buffer_info": (_I, [_P, _I, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_L),
                                     ctypes.POINTER(_L)]),
    "spff_unet3d_buffer_floats": (_L, [_P]),
    "spff_unet3d_workspace_bytes": (_S, [_P]),
    "spff_unet3d_forward": (_I, [_P, _P, _P, _P, _I, _P, _P, _P]),
    "spff_unet3d_backward": (_I, [_P, _P, _P, _P, _P, _P]),
    "spff_unet3d_saved_tensor": (_I, [_P, _P, ctypes.c_char_p, ctypes.POINTER(_P),
                                      ctypes.POINTER(_L), ctypes.POINTER(_I)]),
    # SwinUNETR variant (BASELINE config 5)
    "spff_swin_create": (_I, [ctypes.POINTER(spff_swin_cfg), ctypes.POINTER(_P)]),
    "spff_swin_destroy": (None, [_P]),
    "spff_swin_num_params": (_I, [_P]),
    "spff_swin_param_info": (_I, [_P, _I, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_I),
                                  ctypes.POINTER(_L), ctypes.POINTER(_L), ctypes.POINTER(_L)]),
    "spff_swin_param_floats": (_L, [_P]),
    "spff_swin_workspace_bytes": (_S, [_P]),
    "spff_swin_forward": (_I, [_P, _P, _P, _P, _P, _P]),
    "spff_swin_backward": (_I, [_P, _P, _P, _P, _P, _P]),
    "spff_swin_saved_tensor": (_I, [_P, _P, ctypes.c_char_p, ctypes.POINTER(_P),
                                    ctypes.POINTER(_L), ctypes.POINTER(_I)]),
    "spff_swin_loss_ws_bytes": (_S, [_I, _I]),
    # data path
    "spff_rasterize_ellipses": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "spff_resize_bilinear_aa": (_I, [_P, _I, _I, _I, _P, _I, _I, _P, _P]),
    "spff_grid_aug_ws_bytes": (_S, [_I]),
    "spff_grid_aug": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, ctypes.c_uint64, _P, _P, _P, _P]),
    "spff_swin_loss": (_I, [_P, _P, _I, _L, _I, _I, _I, ctypes.c_double, _P, _P, _P, _P]),
    "spff_loss_ex": (_I, [_P, _P, _L, _I, _I, ctypes.c_double, _P, _P, _I, _P, _P, _P, _P, _P]),
}
EXPORTED = tuple(_SIGS)


def lib_path() -> pathlib.Path:
    return pathlib.Path(os.environ.get("SPFF_LIB", str(_LIB_PATH)))


def lib():
    """Load libspff_hip.so (raises if it is missing -- no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is None:
            p = lib_path()
            if not p.exists():
                raise SpffError(
                    f"libspff_hip.so not found at {p}; build it with "
                    f"`python spff-unet-spcct_amd/build_ext.py` (hipcc, gfx950)")
            L = ctypes.CDLL(str(p))
            for name, (res, args) in _SIGS.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().spff_last_error()
        raise SpffError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(t: torch.Tensor, what: str):
    if not (t.is_cuda and torch.version.hip is not None):
        raise SpffError(f"{what}: the SPFF engine runs only on a ROCm (HIP) device; got a tensor "
                        f"on {t.device}. There is no CPU fallback.")


class Plan:
    """One engine plan (shape + flags) and its device workspace.

    The workspace holds the saved activations of the most recent forward until
    the matching backward (``generation`` guards against interleaving)."""

    def __init__(self, batch, in_ch, depth, height, width, num_classes, base=32, ksd=3,
                 efilm=True, fgate=True, se=True, specse=True, device=None, math=None,
                 shard_world=1, shard_rank=0, memory=None, shard_axis=0, efilm_hidden=32,
                 efilm_pe_dims=16, fgate_learn_phase=False):
        math = default_math() if math is None else math
        if math not in MATH_NAMES:
            raise SpffError(f"math={math!r}: expected one of {sorted(MATH_NAMES)}")
        memory = default_memory() if memory is None else memory
        if memory not in MEMORY_MODES:
            raise SpffError(f"memory={memory!r}: expected one of {sorted(MEMORY_MODES)}")
        cfg = spff_cfg()
        cfg.math = MATH_NAMES[math]
        cfg.memory_mode = MEMORY_MODES[memory]
        self.memory = memory
        # the layout the engine resolves (engine.hip build_plan: lean from 2^26 voxels on auto)
        self.layout = ("lean" if memory == "lean" or
                       (memory == "auto" and batch * depth * height * width >= 1 << 26)
                       else "full")
        cfg.shard_world, cfg.shard_rank = int(shard_world), int(shard_rank)
        # 0 = SPFF_SHARD_DEPTH (BASELINE config 4), 1 = SPFF_SHARD_HEIGHT (registry layout)
        cfg.shard_axis = int(shard_axis)
        self.math = math
        self.shard = (int(shard_world), int(shard_rank), int(shard_axis))
        cfg.batch, cfg.in_ch, cfg.depth, cfg.height, cfg.width = batch, in_ch, depth, height, width
        cfg.num_classes, cfg.base, cfg.ksd = num_classes, base, ksd
        cfg.use_efilm, cfg.use_fgate, cfg.use_se, cfg.use_specse = (int(bool(efilm)), int(bool(fgate)),
                                                                    int(bool(se)), int(bool(specse)))
        # EnergyFiLM3D(hidden, pe_dims) / FourierGate3D(learn_phase) of the blocks
        cfg.efilm_hidden, cfg.efilm_pe_dims = int(efilm_hidden), int(efilm_pe_dims)
        cfg.fgate_learn_phase = int(bool(fgate_learn_phase))
        self.cfg = cfg
        self.key = (batch, in_ch, depth, height, width, num_classes, base, ksd, bool(efilm),
                    bool(fgate), bool(se), bool(specse), math, self.shard, memory,
                    int(efilm_hidden), int(efilm_pe_dims), bool(fgate_learn_phase))
        L = lib()
        h = ctypes.c_void_p()
        check(L.spff_plan_create(ctypes.byref(cfg), ctypes.byref(h)), "spff_plan_create")
        self._h = h
        self.params: List[Tuple[str, Tuple[int, ...], int, int]] = []
        for i in range(L.spff_num_params(h)):
            name = ctypes.c_char_p()
            nd = ctypes.c_int()
            shape = (ctypes.c_int64 * 5)()
            off = ctypes.c_int64()
            n = ctypes.c_int64()
            check(L.spff_param_info(h, i, ctypes.byref(name), ctypes.byref(nd), shape,
                                    ctypes.byref(off), ctypes.byref(n)), "spff_param_info")
            self.params.append((name.value.decode(), tuple(shape[k] for k in range(nd.value)),
                                off.value, n.value))
        self.nfloats = int(L.spff_param_floats(h))
        self.ws_bytes = int(L.spff_workspace_bytes(h))
        self.device = device
        self._ws: Optional[torch.Tensor] = None
        self.generation = 0

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None and _lib is not None:
                _lib.spff_plan_destroy(self._h)
        except Exception:
            pass

    def set_coll(self, impl) -> None:
        """Attach a depth-sharding collective implementation: an object with
        ``allreduce(t)`` (in-place sum of a device tensor over the group) and
        ``halo(slab, slice, d_local)`` (``slab`` = the [d_local + 2] x slice view
        whose first / last slices receive the neighbours' boundary slices), e.g.
        innovative3D.sharded.TorchDepthColl.  The engine calls them in stream
        order with pointers into this plan's workspace."""
        def view(ptr, n, dtype):
            ws = self._ws
            off = ptr - ws.data_ptr()
            esz = 8 if dtype == torch.float64 else 4
            if off < 0 or off % esz or off + n * esz > ws.numel():
                raise SpffError("collective buffer outside the plan workspace")
            return ws[off:off + n * esz].view(dtype)

        def _timed(kind, nbytes, stream, dev, fn):
            """fn(); with coll_timing on, bracketed by HIP events on the stream the engine
            handed the callback (where the collective's work is issued)"""
            if not self.coll_timing:
                return fn()
            st = (torch.cuda.ExternalStream(stream, device=dev) if stream
                  else torch.cuda.current_stream(dev))
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            fn()
            b.record(st)
            self._coll_ev.append((kind, nbytes, a, b))

        def _allreduce(ctx, buf, n, dt, stream):
            try:
                t = view(buf, n, torch.float64 if dt == 1 else torch.float32)
                nb = t.numel() * t.element_size()
                cur = torch.cuda.current_stream(t.device)
                if stream and stream != cur.cuda_stream:
                    # issue the all-reduce on the stream the engine handed over (where
                    # its timing events are recorded and the buffer is ordered), as
                    # _halo does
                    with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=t.device)):
                        _timed("allreduce", nb, stream, t.device, lambda: impl.allreduce(t))
                else:
                    _timed("allreduce", nb, stream, t.device, lambda: impl.allreduce(t))
                return 0
            except Exception as e:  # noqa: BLE001 -- reported through the engine status
                self.coll_error = e
                return 1

        def _halo(ctx, interior, sl, d_local, stream):
            try:
                slab = view(interior - 4 * sl, (d_local + 2) * sl, torch.float32)
                cur = torch.cuda.current_stream(slab.device)
                # 2 slices sent (and 2 received) per rank at most
                nb = 2 * 4 * int(sl)
                if stream and stream != cur.cuda_stream:
                    # the engine's side stream (halo exchange overlapping the interior
                    # depth tiles of the next convolution): issue the exchange there
                    with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=slab.device)):
                        _timed("halo", nb, stream, slab.device,
                               lambda: impl.halo(slab, int(sl), int(d_local)))
                else:
                    _timed("halo", nb, stream, slab.device,
                           lambda: impl.halo(slab, int(sl), int(d_local)))
                return 0
            except Exception as e:  # noqa: BLE001
                self.coll_error = e
                return 1
        self.coll_timing = getattr(self, "coll_timing", False)
        self._coll_ev = []
        self._coll_fns = (ALLREDUCE_FN(_allreduce), HALO_FN(_halo))  # keep alive
        self._coll = spff_coll(None, self._coll_fns[0], self._coll_fns[1])
        self.coll_impl = impl
        self.coll_error = None
        check(lib().spff_plan_set_coll(self._h, ctypes.byref(self._coll)), "spff_plan_set_coll")

    def coll_collect(self) -> Dict[str, Dict[str, float]]:
        """{kind: {calls, ms, bytes}} of the shard-group collective callbacks since the
        last collect (coll_timing on: HIP events around each callback's work on its
        stream; a halo on the side stream overlaps the interior conv tiles, so its time
        is the exchange's duration, not the step time it costs).  Syncs on the events."""
        out: Dict[str, Dict[str, float]] = {}
        for kind, nb, a, b in getattr(self, "_coll_ev", []):
            b.synchronize()
            r = out.setdefault(kind, {"calls": 0, "ms": 0.0, "bytes": 0.0})
            r["calls"] += 1
            r["ms"] += a.elapsed_time(b)
            r["bytes"] += nb
        self._coll_ev = []
        return out

    def workspace(self, device) -> torch.Tensor:
        if self._ws is None or self._ws.device != device:
            self._ws = _alloc_workspace(self, device)
        return self._ws

    def forward(self, x: torch.Tensor, flat: torch.Tensor, out: Optional[torch.Tensor] = None):
        """x [B,Cin,D,H,W] contiguous fp32 -> logits channel-last [B,D,H,W,K]."""
        c = self.cfg
        require_device(x, "SPFF forward")
        if tuple(x.shape) != (c.batch, c.in_ch, c.depth, c.height, c.width):
            raise SpffError(f"input shape {tuple(x.shape)} does not match plan")
        x = x.contiguous()
        if x.dtype != torch.float32:
            raise SpffError("SPFF engine computes in fp32; got " + str(x.dtype))
        if out is None:
            out = torch.empty((c.batch, c.depth, c.height, c.width, c.num_classes),
                              dtype=torch.float32, device=x.device)
        ws = self.workspace(x.device)
        self.generation += 1
        self.coll_error = None
        self._check(lib().spff_forward(self._h, _ptr(x), _ptr(flat), _ptr(out), _ptr(ws),
                                       _stream(x.device)), "spff_forward")
        return out

    def _check(self, rc: int, what: str) -> None:
        """check(), raising SpffCollError chained to the callback's own exception when a
        shard-group collective failed (SPFF_ECOLL)"""
        if rc == SPFF_ECOLL:
            msg = lib().spff_last_error()
            err = getattr(self, "coll_error", None)
            raise SpffCollError(f"{what} failed ({rc}): {msg.decode() if msg else ''}"
                                + (f" -- {err!r}" if err is not None else "")) from err
        check(rc, what)

    def backward(self, dlogits_cl: torch.Tensor, flat: torch.Tensor,
                 dflat: Optional[torch.Tensor] = None, grad_hook=None) -> torch.Tensor:
        """``grad_hook``: an object with begin(dflat), ready(off, n) and finish()
        (innovative3D.distributed.GradBucketer); ready() is called while the
        backward is being enqueued, as each parameter group's gradient becomes
        final, and finish() after it."""
        dlogits_cl = dlogits_cl.contiguous()
        if dflat is None:
            dflat = torch.empty(self.nfloats, dtype=torch.float32, device=dlogits_cl.device)
        ws = self.workspace(dlogits_cl.device)
        L = lib()
        self.coll_error = None
        if grad_hook is None:
            self._check(L.spff_backward(self._h, _ptr(dlogits_cl), _ptr(flat), _ptr(dflat),
                                        _ptr(ws), _stream(dlogits_cl.device)), "spff_backward")
            return dflat
        covered = [0]
        err = []

        dev = dlogits_cl.device
        main_stream = torch.cuda.current_stream(dev).cuda_stream

        def _ready(_ctx, off, n, stream):
            try:
                covered[0] += int(n)
                if stream and stream != main_stream:
                    # the engine's weight-gradient stream (those floats are final in its
                    # order): the bucket's all-reduce is issued there
                    with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=dev)):
                        grad_hook.ready(int(off), int(n))
                else:
                    grad_hook.ready(int(off), int(n))
                return 0
            except Exception as e:  # noqa: BLE001 -- reported through the engine status
                err.append(e)
                return 1
        fn = GRAD_READY_FN(_ready)
        grad_hook.begin(dflat)
        ok = False
        try:
            check(L.spff_plan_set_grad_hook(self._h, fn, None), "spff_plan_set_grad_hook")
            try:
                rc = L.spff_backward(self._h, _ptr(dlogits_cl), _ptr(flat), _ptr(dflat), _ptr(ws),
                                     _stream(dlogits_cl.device))
            finally:
                L.spff_plan_set_grad_hook(self._h, GRAD_READY_FN(), None)
            if err:
                raise SpffError(f"gradient hook failed: {err[0]!r}") from err[0]
            self._check(rc, "spff_backward")
            if covered[0] != self.nfloats:
                raise SpffError(f"gradient hook covered {covered[0]} of {self.nfloats} floats")
            grad_hook.finish()
            ok = True
        finally:
            if not ok and hasattr(grad_hook, "abort"):
                # join the bucket all-reduces already issued, so peers that issued the
                # same ones complete them, then let the error propagate (the process
                # group's timeout ends any collective a peer is left waiting in)
                grad_hook.abort()
        return dflat

    PROF_CLASSES = ("conv_fwd", "conv_dgrad", "conv_wgrad", "gemm", "slab_reduce", "act_apply",
                    "in_bwd_apply", "f16_absmax")
    MEM_CLASSES = ("slab_reduce", "act_apply", "in_bwd_apply", "f16_absmax")

    def prof_enable(self, on: bool = True):
        check(lib().spff_prof_enable(self._h, int(bool(on))), "spff_prof_enable")

    def prof_collect(self) -> Dict[str, Tuple[float, float, int, float]]:
        """{class: (total_ms, algorithmic_flops, launches, compulsory_bytes)} since the last
        collect."""
        n = len(self.PROF_CLASSES)
        buf = (ctypes.c_double * (4 * n))()
        check(lib().spff_prof_collect(self._h, buf, n), "spff_prof_collect")
        return {c: (buf[4 * i], buf[4 * i + 1], int(buf[4 * i + 2]), buf[4 * i + 3])
                for i, c in enumerate(self.PROF_CLASSES)}

    def debug_set(self, key: int, value: int):
        """spff_debug_set: key 0 = stop the backward after N decoder blocks, key 1 = store
        the GEMM-applied block outputs too (saved("dec1.out") etc.), key 2 = 0: the encoder
        output gradients by a k_maxpool_bwd_add pass instead of PoolAdd in their readers."""
        check(lib().spff_debug_set(self._h, int(key), int(value)), "spff_debug_set")

    def saved(self, name: str) -> torch.Tensor:
        """Copy of a saved intermediate as a channel-last [V, C] tensor (debug/tests):
        fp32, or uint8 for the max-pool argmax bytes "poolN.idx"."""
        ws = self._ws
        if ws is None:
            raise SpffError("no forward has run")
        ptr = ctypes.c_void_p()
        nv = ctypes.c_int64()
        ch = ctypes.c_int()
        check(lib().spff_saved_tensor(self._h, _ptr(ws), name.encode(), ctypes.byref(ptr),
                                      ctypes.byref(nv), ctypes.byref(ch)), "spff_saved_tensor")
        off = ptr.value - ws.data_ptr()
        n = nv.value * ch.value
        if name.endswith(".idx"):
            return ws[off:off + n].view(nv.value, ch.value).clone()
        return ws[off:off + 4 * n].view(torch.float32).view(nv.value, ch.value).clone()


# Plans (and the workspace each pins: ~2.6 KB per voxel) belong to the module
# that created them: a small LRU of shapes per (module, tag) -- so alternating
# shapes (a partial last batch, validation at another size) do not rebuild and
# re-allocate a multi-GB workspace on every switch -- dropped with the module (weak
# keys), or explicitly by release_plans().  At most PLAN_CACHE plans per (module,
# tag), and older ones are evicted first while their workspaces together would exceed
# PLAN_CACHE_FRACTION of the device memory (a 5 x 512^3 plan alone is 211 GiB).
_OWNER_PLANS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
_ANON_PLANS: Dict[tuple, object] = {}
PLAN_CACHE = int(os.environ.get("SPFF_PLAN_CACHE", "3"))
PLAN_CACHE_FRACTION = 0.4


def _all_plans():
    for slots in list(_OWNER_PLANS.values()):
        for lru in slots.values():
            yield from list(lru.values())
    yield from list(_ANON_PLANS.values())


def release_workspace(plan) -> None:
    """Free a cached plan's workspace (the plan stays; the next forward allocates a new
    one).  A backward still pending on that workspace's activations then fails loudly
    (its plan generation no longer matches) instead of reading freed memory."""
    if getattr(plan, "_ws", None) is not None:
        plan._ws = None
        plan.generation = getattr(plan, "generation", 0) + 1


def _alloc_workspace(plan, device) -> torch.Tensor:
    """The plan's workspace.  If the device is out of memory, the workspaces of the OTHER
    cached plans on the same device (validation shapes, a partial last batch: see
    _owned_plan) are released, torch's cache is emptied and the allocation retried:
    first only plans with no backward pending on their workspace (``_pending_gen``, set
    by the engine ops' autograd forward, cleared by their backward), then, as a last
    resort, those too (their pending backward then fails loudly, see release_workspace).
    A failure after that raises.  SPFF_PLAN_CACHE=1 keeps one plan per module and tag
    (round 2's behaviour: the previous shape's workspace is freed before a new shape's
    is built)."""
    device = torch.device(device)
    try:
        return torch.empty(plan.ws_bytes, dtype=torch.uint8, device=device)
    except torch.OutOfMemoryError:
        pass

    def same_device(q):
        ws = getattr(q, "_ws", None)
        return ws is not None and ws.device == device

    for last_resort in (False, True):
        for q in _all_plans():
            if q is plan or not same_device(q):
                continue
            if not last_resort and getattr(q, "_pending_gen", None) == getattr(q, "generation", 0):
                continue
            release_workspace(q)
        torch.cuda.empty_cache()
        try:
            return torch.empty(plan.ws_bytes, dtype=torch.uint8, device=device)
        except torch.OutOfMemoryError:
            if last_resort:
                raise


def _device_bytes() -> int:
    try:
        if torch.cuda.is_available():
            return int(torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory)
    except Exception:  # noqa: BLE001
        pass
    return 64 << 30


def _owned_plan(owner, tag: str, key: tuple, make):
    if owner is None:
        if key not in _ANON_PLANS:
            _ANON_PLANS[key] = make()
        return _ANON_PLANS[key]
    slots = _OWNER_PLANS.get(owner)
    if slots is None:
        slots = {}
        _OWNER_PLANS[owner] = slots
    lru = slots.setdefault(tag, collections.OrderedDict())
    if key in lru:
        lru.move_to_end(key)
        return lru[key]
    plan = make()  # host-side only: the workspace is allocated at first use
    budget = PLAN_CACHE_FRACTION * _device_bytes()
    while lru and (len(lru) >= PLAN_CACHE or
                   sum(getattr(q, "ws_bytes", 0) for q in lru.values())
                   + getattr(plan, "ws_bytes", 0) > budget):
        lru.popitem(last=False)  # free the least recently used plan's workspace first
    lru[key] = plan
    return plan


def release_plans(owner=None) -> None:
    """Drop the engine plans (and workspaces) of ``owner`` -- every module-owned
    and anonymous plan when owner is None."""
    if owner is None:
        _OWNER_PLANS.clear()
        _ANON_PLANS.clear()
    else:
        _OWNER_PLANS.pop(owner, None)


def shard_key(shard) -> Tuple[int, int, int]:
    """(world, rank[, axis]) -> (world, rank, axis); axis 0 = depth, 1 = height"""
    sh = tuple(int(v) for v in shard)
    return sh if len(sh) == 3 else (sh[0], sh[1], 0)


def get_plan(owner=None, tag: str = "", **kw) -> Plan:
    """The plan of ``owner`` (an nn.Module) for tag ``tag`` and this shape/flag set."""
    key = (kw["batch"], kw["in_ch"], kw["depth"], kw["height"], kw["width"], kw["num_classes"],
           kw.get("base", 32), kw.get("ksd", 3), bool(kw.get("efilm", True)),
           bool(kw.get("fgate", True)), bool(kw.get("se", True)), bool(kw.get("specse", True)),
           kw.get("math") or default_math(), shard_key(kw.get("shard", (1, 0))),
           kw.get("memory") or default_memory(), int(kw.get("efilm_hidden", 32)),
           int(kw.get("efilm_pe_dims", 16)), bool(kw.get("fgate_learn_phase", False)))

    def make():
        kk = dict(kw)
        kk["shard_world"], kk["shard_rank"], kk["shard_axis"] = shard_key(kk.pop("shard", (1, 0)))
        return Plan(**kk)
    return _owned_plan(owner, tag, key, make)


class UNet3DPlan:
    """Engine plan of the 3DUNet baseline variant (include/spff.h spff_unet3d_*):
    Cicek3DUNet + the depth adapter of LitCicek3DUNet_DepthAdapter_Published
    (reference models.py:718-777).  Parameters are one flat fp32 buffer in
    reference state-dict order (``params``), BatchNorm running statistics a
    second one (``buffers``)."""

    def __init__(self, batch, in_ch, depth, height, width, num_classes, base=32, target_depth=0,
                 device=None, math=None):
        math = default_math() if math is None else math
        if math not in MATH_NAMES:
            raise SpffError(f"math={math!r}: expected one of {sorted(MATH_NAMES)}")
        cfg = spff_unet3d_cfg()
        cfg.batch, cfg.in_ch, cfg.depth, cfg.height, cfg.width = batch, in_ch, depth, height, width
        cfg.target_depth, cfg.num_classes, cfg.base = int(target_depth), num_classes, base
        cfg.math = MATH_NAMES[math]
        self.cfg, self.math, self.device = cfg, math, device
        L = lib()
        h = ctypes.c_void_p()
        check(L.spff_unet3d_create(ctypes.byref(cfg), ctypes.byref(h)), "spff_unet3d_create")
        self._h = h
        self.params: List[Tuple[str, Tuple[int, ...], int, int]] = []
        for i in range(L.spff_unet3d_num_params(h)):
            name, nd = ctypes.c_char_p(), ctypes.c_int()
            shape, off, n = (ctypes.c_int64 * 5)(), ctypes.c_int64(), ctypes.c_int64()
            check(L.spff_unet3d_param_info(h, i, ctypes.byref(name), ctypes.byref(nd), shape,
                                           ctypes.byref(off), ctypes.byref(n)),
                  "spff_unet3d_param_info")
            self.params.append((name.value.decode(), tuple(shape[k] for k in range(nd.value)),
                                off.value, n.value))
        self.buffers: List[Tuple[str, int, int]] = []
        for i in range(L.spff_unet3d_num_buffers(h)):
            name, off, n = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_int64()
            check(L.spff_unet3d_buffer_info(h, i, ctypes.byref(name), ctypes.byref(off),
                                            ctypes.byref(n)), "spff_unet3d_buffer_info")
            self.buffers.append((name.value.decode(), off.value, n.value))
        self.nfloats = int(L.spff_unet3d_param_floats(h))
        self.nbuf = int(L.spff_unet3d_buffer_floats(h))
        self.ws_bytes = int(L.spff_unet3d_workspace_bytes(h))
        self._ws: Optional[torch.Tensor] = None
        self.generation = 0

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None and _lib is not None:
                _lib.spff_unet3d_destroy(self._h)
        except Exception:
            pass

    def workspace(self, device) -> torch.Tensor:
        if self._ws is None or self._ws.device != device:
            self._ws = _alloc_workspace(self, device)
        return self._ws

    def set_sync_bn(self, impl) -> None:
        """Synchronised BatchNorm over a data-parallel group (spff_unet3d_set_sync_bn):
        ``impl`` has ``allreduce(t)`` (in-place sum of a device tensor over the group) and
        ``world``, e.g. innovative3D.sharded.TorchDepthColl; None restores per-replica
        statistics."""
        L = lib()
        if impl is None or int(getattr(impl, "world", 1)) <= 1:
            check(L.spff_unet3d_set_sync_bn(self._h, None, 1), "spff_unet3d_set_sync_bn")
            self._sync = None
            return

        def _allreduce(ctx, buf, n, dt, stream):
            try:
                ws = self._ws
                off = buf - ws.data_ptr()
                esz = 8 if dt == 1 else 4
                if off < 0 or off % esz or off + n * esz > ws.numel():
                    raise SpffError("collective buffer outside the plan workspace")
                t = ws[off:off + n * esz].view(torch.float64 if dt == 1 else torch.float32)
                cur = torch.cuda.current_stream(t.device)
                if stream and stream != cur.cuda_stream:
                    with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=t.device)):
                        impl.allreduce(t)
                else:
                    impl.allreduce(t)
                return 0
            except Exception as e:  # noqa: BLE001 -- reported through the engine status
                self.coll_error = e
                return 1

        def _no_halo(ctx, interior, sl, d_local, stream):
            return 1
        self._sync_fns = (ALLREDUCE_FN(_allreduce), HALO_FN(_no_halo))  # keep alive
        self._sync = spff_coll(None, self._sync_fns[0], self._sync_fns[1])
        self.coll_error = None
        check(L.spff_unet3d_set_sync_bn(self._h, ctypes.byref(self._sync), int(impl.world)),
              "spff_unet3d_set_sync_bn")

    def forward(self, x: torch.Tensor, flat: torch.Tensor, bufs: torch.Tensor, training: bool,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x [B,Cin,D,H,W] fp32 -> logits channel-last [B,D,H,W,K]; training updates bufs."""
        c = self.cfg
        require_device(x, "3DUNet forward")
        if tuple(x.shape) != (c.batch, c.in_ch, c.depth, c.height, c.width):
            raise SpffError(f"input shape {tuple(x.shape)} does not match plan")
        if x.dtype != torch.float32:
            raise SpffError("the engine computes in fp32; got " + str(x.dtype))
        x = x.contiguous()
        if out is None:
            out = torch.empty((c.batch, c.depth, c.height, c.width, c.num_classes),
                              dtype=torch.float32, device=x.device)
        ws = self.workspace(x.device)
        self.generation += 1
        check(lib().spff_unet3d_forward(self._h, _ptr(x), _ptr(flat), _ptr(bufs), int(bool(training)),
                                        _ptr(out), _ptr(ws), _stream(x.device)),
              "spff_unet3d_forward")
        return out

    def backward(self, dlogits_cl: torch.Tensor, flat: torch.Tensor, grad_hook=None) -> torch.Tensor:
        """``grad_hook`` (GradBucketer protocol): this plan reports its whole
        gradient as ready once the backward is enqueued (no per-block hook)."""
        dlogits_cl = dlogits_cl.contiguous()
        dflat = torch.empty(self.nfloats, dtype=torch.float32, device=dlogits_cl.device)
        ws = self.workspace(dlogits_cl.device)
        check(lib().spff_unet3d_backward(self._h, _ptr(dlogits_cl), _ptr(flat), _ptr(dflat),
                                         _ptr(ws), _stream(dlogits_cl.device)),
              "spff_unet3d_backward")
        _whole_buffer_hook(grad_hook, dflat)
        return dflat

    def saved(self, name: str) -> torch.Tensor:
        ws = self._ws
        if ws is None:
            raise SpffError("no forward has run")
        ptr, nv, ch = ctypes.c_void_p(), ctypes.c_int64(), ctypes.c_int()
        check(lib().spff_unet3d_saved_tensor(self._h, _ptr(ws), name.encode(), ctypes.byref(ptr),
                                             ctypes.byref(nv), ctypes.byref(ch)),
              "spff_unet3d_saved_tensor")
        off = ptr.value - ws.data_ptr()
        n = nv.value * ch.value
        return ws[off:off + 4 * n].view(torch.float32).view(nv.value, ch.value).clone()


def _whole_buffer_hook(grad_hook, dflat: torch.Tensor) -> None:
    if grad_hook is None:
        return
    grad_hook.begin(dflat)
    grad_hook.ready(0, int(dflat.numel()))
    grad_hook.finish()


def get_unet3d_plan(owner=None, tag: str = "", **kw) -> UNet3DPlan:
    """UNet3D plans, owned like get_plan."""
    key = ("unet3d", kw["batch"], kw["in_ch"], kw["depth"], kw["height"], kw["width"],
           kw["num_classes"], kw.get("base", 32), kw.get("target_depth", 0),
           kw.get("math") or default_math())
    return _owned_plan(owner, "unet3d:" + tag, key, lambda: UNet3DPlan(**kw))


class SwinPlan:
    """One spff_swin plan (SwinUNETR variant) + its workspace."""

    def __init__(self, batch, in_ch, depth, height, width, num_classes, feature_size=12,
                 window=7, heads=(1, 2, 4, 8), mlp_ratio=2.0, device=None, math=None):
        math = math or default_math()
        if math not in MATH_NAMES:
            raise SpffError(f"math={math!r}: expected one of {sorted(MATH_NAMES)}")
        cfg = spff_swin_cfg()
        cfg.batch, cfg.in_ch, cfg.depth, cfg.height, cfg.width = batch, in_ch, depth, height, width
        cfg.num_classes, cfg.feature_size, cfg.window = num_classes, feature_size, window
        for i, h in enumerate(heads):
            cfg.heads[i] = int(h)
        cfg.mlp_ratio = float(mlp_ratio)
        cfg.math = MATH_NAMES[math]
        self.cfg, self.math, self.device = cfg, math, device
        L = lib()
        h = ctypes.c_void_p()
        check(L.spff_swin_create(ctypes.byref(cfg), ctypes.byref(h)), "spff_swin_create")
        self._h = h
        self.params: List[Tuple[str, Tuple[int, ...], int, int]] = []
        for i in range(L.spff_swin_num_params(h)):
            name, nd = ctypes.c_char_p(), ctypes.c_int()
            shape, off, n = (ctypes.c_int64 * 5)(), ctypes.c_int64(), ctypes.c_int64()
            check(L.spff_swin_param_info(h, i, ctypes.byref(name), ctypes.byref(nd), shape,
                                         ctypes.byref(off), ctypes.byref(n)),
                  "spff_swin_param_info")
            self.params.append((name.value.decode(), tuple(shape[k] for k in range(nd.value)),
                                off.value, n.value))
        self.nfloats = int(L.spff_swin_param_floats(h))
        self.ws_bytes = int(L.spff_swin_workspace_bytes(h))
        self._ws: Optional[torch.Tensor] = None
        self.generation = 0

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None and _lib is not None:
                _lib.spff_swin_destroy(self._h)
        except Exception:
            pass

    def workspace(self, device) -> torch.Tensor:
        if self._ws is None or self._ws.device != device:
            self._ws = _alloc_workspace(self, device)
        return self._ws

    def forward(self, x: torch.Tensor, flat: torch.Tensor,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x [B,Cin,D,H,W] fp32 -> logits channel-last [B,D,H,W,K]."""
        c = self.cfg
        require_device(x, "SwinUNETR forward")
        if tuple(x.shape) != (c.batch, c.in_ch, c.depth, c.height, c.width):
            raise SpffError(f"input shape {tuple(x.shape)} does not match plan")
        if x.dtype != torch.float32:
            raise SpffError("the engine computes in fp32; got " + str(x.dtype))
        x = x.contiguous()
        if out is None:
            out = torch.empty((c.batch, c.depth, c.height, c.width, c.num_classes),
                              dtype=torch.float32, device=x.device)
        ws = self.workspace(x.device)
        self.generation += 1
        check(lib().spff_swin_forward(self._h, _ptr(x), _ptr(flat), _ptr(out), _ptr(ws),
                                      _stream(x.device)), "spff_swin_forward")
        return out

    def backward(self, dlogits_cl: torch.Tensor, flat: torch.Tensor,
                 dflat: Optional[torch.Tensor] = None, grad_hook=None) -> torch.Tensor:
        """``grad_hook`` as UNet3DPlan.backward: the whole gradient at once."""
        dlogits_cl = dlogits_cl.contiguous()
        if dflat is None:
            dflat = torch.empty(self.nfloats, dtype=torch.float32, device=dlogits_cl.device)
        ws = self.workspace(dlogits_cl.device)
        check(lib().spff_swin_backward(self._h, _ptr(dlogits_cl), _ptr(flat), _ptr(dflat), _ptr(ws),
                                       _stream(dlogits_cl.device)), "spff_swin_backward")
        _whole_buffer_hook(grad_hook, dflat)
        return dflat

    def saved(self, name: str) -> torch.Tensor:
        ws = self._ws
        if ws is None:
            raise SpffError("no forward has run")
        ptr, nv, ch = ctypes.c_void_p(), ctypes.c_int64(), ctypes.c_int()
        check(lib().spff_swin_saved_tensor(self._h, _ptr(ws), name.encode(), ctypes.byref(ptr),
                                           ctypes.byref(nv), ctypes.byref(ch)),
              "spff_swin_saved_tensor")
        off = ptr.value - ws.data_ptr()
        n = nv.value * ch.value
        return ws[off:off + 4 * n].view(torch.float32).view(nv.value, ch.value).clone()


def get_swin_plan(owner=None, tag: str = "", **kw) -> SwinPlan:
    """SwinUNETR plans, owned like get_plan."""
    key = ("swin", kw["batch"], kw["in_ch"], kw["depth"], kw["height"], kw["width"],
           kw["num_classes"], kw.get("feature_size", 12), kw.get("window", 7),
           tuple(kw.get("heads", (1, 2, 4, 8))), float(kw.get("mlp_ratio", 2.0)),
           kw.get("math") or default_math())
    return _owned_plan(owner, "swin:" + tag, key, lambda: SwinPlan(**kw))


def swin_loss_forward(logits_cl: torch.Tensor, labels: torch.Tensor, K: int, ignore_index: int,
                      include_bg: bool, ce_weight: float):
    """LitSwinUNETR_Published._loss on the HIP kernels: returns (out4, dlogits_cl)."""
    require_device(logits_cl, "SwinUNETR loss")
    logits_cl = logits_cl.contiguous()
    B = logits_cl.shape[0]
    labels = labels.to(device=logits_cl.device, dtype=torch.int64).contiguous()
    V = labels.numel()
    if logits_cl.numel() != V * K or V % B:
        raise SpffError(f"logits ({tuple(logits_cl.shape)}) / labels ({tuple(labels.shape)}) mismatch")
    dev = logits_cl.device
    out4 = torch.empty(4, dtype=torch.float32, device=dev)
    dl = torch.empty_like(logits_cl)
    ws = torch.empty(int(lib().spff_swin_loss_ws_bytes(B, K)), dtype=torch.uint8, device=dev)
    check(lib().spff_swin_loss(_ptr(logits_cl), _ptr(labels), B, V // B, K, int(ignore_index),
                               int(bool(include_bg)), float(ce_weight), _ptr(out4), _ptr(dl),
                               _ptr(ws), _stream(dev)), "spff_swin_loss")
    return out4, dl


# ------------------------------------------------------------- data path ops --
def rasterize_ellipses(rois: torch.Tensor, frames: int, height: int, width: int) -> torch.Tensor:
    """rois [n, 5] int32 (x0, y0, w0, h0, label) on the device -> labels [F, H, W] int64."""
    require_device(rois, "rasterize_ellipses")
    rois = rois.to(torch.int32).contiguous()
    lab = torch.empty((frames, height, width), dtype=torch.int64, device=rois.device)
    check(lib().spff_rasterize_ellipses(_ptr(rois), rois.shape[0], frames, height, width,
                                        _ptr(lab), _stream(rois.device)), "spff_rasterize_ellipses")
    return lab


def resize_bilinear_aa(frames: torch.Tensor, height: int, width: int) -> torch.Tensor:
    """[N, h, w] fp32 -> [N, height, width] (F.interpolate bilinear, antialias)."""
    require_device(frames, "resize_bilinear_aa")
    x = frames.to(torch.float32).contiguous()
    n, hin, win = x.shape
    out = torch.empty((n, height, width), dtype=torch.float32, device=x.device)
    tmp = torch.empty((n, hin, width), dtype=torch.float32, device=x.device)
    check(lib().spff_resize_bilinear_aa(_ptr(x), n, hin, win, _ptr(out), height, width, _ptr(tmp),
                                        _stream(x.device)), "spff_resize_bilinear_aa")
    return out


def grid_aug(x: torch.Tensor, y: Optional[torch.Tensor], maps: torch.Tensor, prm: torch.Tensor,
             seed: int, out_hw) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """x [B,F,H,W] fp32 (+ y int64) -> augmented [B,F,Ho,Wo]; maps [B,H+W] int32 and
    prm [B,8] fp32 on the device (see include/spff.h spff_grid_aug)."""
    require_device(x, "grid_aug")
    x = x.contiguous()
    B, F_, H, W = x.shape
    Ho, Wo = out_hw
    xo = torch.empty((B, F_, Ho, Wo), dtype=torch.float32, device=x.device)
    yo = None
    if y is not None:
        y = y.to(device=x.device, dtype=torch.int64).contiguous()
        yo = torch.empty((B, F_, Ho, Wo), dtype=torch.int64, device=x.device)
    ws = torch.empty(int(lib().spff_grid_aug_ws_bytes(B)), dtype=torch.uint8, device=x.device)
    check(lib().spff_grid_aug(_ptr(x), _ptr(y), B, F_, H, W, _ptr(maps.contiguous()),
                              _ptr(prm.contiguous()), ctypes.c_uint64(int(seed) & (2**64 - 1)),
                              _ptr(xo), _ptr(yo), _ptr(ws), _stream(x.device)), "spff_grid_aug")
    return xo, yo


# ------------------------------------------------------------------ loss ops --
def loss_ws(device) -> torch.Tensor:
    n = int(lib().spff_loss_ws_bytes(0, 1))
    return torch.empty(n, dtype=torch.uint8, device=device)


def ce_dice_forward(logits_cl: torch.Tensor, labels: torch.Tensor, K: int, ignore_index: int,
                    smooth: float, count_override: Optional[torch.Tensor] = None):
    """Returns (out4, dlogits_cl, conf[K, K+1])."""
    require_device(logits_cl, "ce_plus_macro_dice_loss")
    logits_cl = logits_cl.contiguous()
    labels = labels.to(device=logits_cl.device, dtype=torch.int64).contiguous()
    V = labels.numel()
    if logits_cl.numel() != V * K:
        raise SpffError(f"logits ({tuple(logits_cl.shape)}) / labels ({tuple(labels.shape)}) mismatch")
    dev = logits_cl.device
    out4 = torch.empty(4, dtype=torch.float32, device=dev)
    dl = torch.empty_like(logits_cl)
    conf = torch.empty(K * (K + 1), dtype=torch.int64, device=dev)
    ws = loss_ws(dev)
    check(lib().spff_loss(_ptr(logits_cl), _ptr(labels), V, K, int(ignore_index), float(smooth),
                          _ptr(count_override), _ptr(out4), _ptr(dl), _ptr(conf), _ptr(ws),
                          _stream(dev)), "spff_loss")
    return out4, dl, conf.view(K, K + 1)


def weighted_ce_forward(logits_cl: torch.Tensor, labels: torch.Tensor, K: int, ignore_index: int,
                        class_weights: Optional[torch.Tensor] = None,
                        count_override: Optional[torch.Tensor] = None):
    """The 3DUNet wrapper's _weighted_softmax_ce (models.py:779-799):
    sum_v w[y_v] nll_v / max(N_valid, 1).  Returns (out4, dlogits_cl, conf)."""
    require_device(logits_cl, "weighted softmax CE")
    logits_cl = logits_cl.contiguous()
    labels = labels.to(device=logits_cl.device, dtype=torch.int64).contiguous()
    V = labels.numel()
    if logits_cl.numel() != V * K:
        raise SpffError(f"logits ({tuple(logits_cl.shape)}) / labels ({tuple(labels.shape)}) mismatch")
    dev = logits_cl.device
    cw = None
    if class_weights is not None:
        cw = class_weights.to(device=dev, dtype=torch.float32).contiguous()
        if cw.numel() != K:
            raise SpffError(f"class_weights has {cw.numel()} entries, expected {K}")
    out4 = torch.empty(4, dtype=torch.float32, device=dev)
    dl = torch.empty_like(logits_cl)
    conf = torch.empty(K * (K + 1), dtype=torch.int64, device=dev)
    ws = loss_ws(dev)
    check(lib().spff_loss_ex(_ptr(logits_cl), _ptr(labels), V, K, int(ignore_index), 1e-6,
                             _ptr(count_override), _ptr(cw), 1, _ptr(out4), _ptr(dl), _ptr(conf),
                             _ptr(ws), _stream(dev)), "spff_loss_ex")
    return out4, dl, conf.view(K, K + 1)


def confusion(logits_cl: torch.Tensor, labels: torch.Tensor, K: int,
              ignore_index: Optional[int]) -> torch.Tensor:
    require_device(logits_cl, "per_class_metrics_3d")
    logits_cl = logits_cl.contiguous()
    labels = labels.to(device=logits_cl.device, dtype=torch.int64).contiguous()
    conf = torch.empty(K * (K + 1), dtype=torch.int64, device=logits_cl.device)
    ign = -(2 ** 31) if ignore_index is None else int(ignore_index)
    check(lib().spff_confusion(_ptr(logits_cl), _ptr(labels), labels.numel(), K, ign, _ptr(conf),
                               _stream(logits_cl.device)), "spff_confusion")
    return conf.view(K, K + 1)


def count_valid(labels: torch.Tensor, ignore_index: int) -> torch.Tensor:
    require_device(labels, "count_valid")
    labels = labels.to(torch.int64).contiguous()
    cnt = torch.empty(1, dtype=torch.int64, device=labels.device)
    check(lib().spff_count_valid(_ptr(labels), labels.numel(), int(ignore_index), _ptr(cnt),
                                 _stream(labels.device)), "spff_count_valid")
    return cnt


def scale_(x: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    check(lib().spff_scale(_ptr(x), x.numel(), _ptr(scale.to(torch.float32).contiguous()),
                           _stream(x.device)), "spff_scale")
    return x


def to_channels_last(t: torch.Tensor) -> torch.Tensor:
    """[B,C,D,H,W] -> contiguous [B,D,H,W,C] (a free view for channels_last_3d)."""
    return t.permute(0, 2, 3, 4, 1).contiguous()


CONV_PROF_CLASSES = ("conv_fwd", "conv_dgrad", "conv_wgrad", "loss_pass", "k_loss")


def conv_prof_enable(on: bool = True) -> None:
    """Library-wide conv timing (every 3x3x3 conv launch of any plan; HIP events on the
    launch's stream) -- the 3DUNet / SwinUNETR bench lines' roofline source."""
    check(lib().spff_conv_prof_enable(int(bool(on))), "spff_conv_prof_enable")


def conv_prof_collect() -> Dict[str, Tuple[float, float, int]]:
    """{class: (ms, algorithmic fp32 flops, launches)} since the last enable / collect."""
    n = len(CONV_PROF_CLASSES)
    buf = (ctypes.c_double * (4 * n))()
    check(lib().spff_conv_prof_collect(buf, n), "spff_conv_prof_collect")
    return {c: (buf[4 * i], buf[4 * i + 1], int(buf[4 * i + 2]))
            for i, c in enumerate(CONV_PROF_CLASSES)}
