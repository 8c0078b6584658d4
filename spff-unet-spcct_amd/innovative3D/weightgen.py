"""Deterministic synthetic parameter generator (host-side utility, no GPU).

The reference ships no checkpoints, and there is no network to fetch any, so
every parity fixture, test and benchmark in this repo initialises SPFF-UNet
parameters from this generator.  Each tensor is drawn from its own numpy
``default_rng([seed, crc32(name)])`` stream, so the values depend only on
(seed, state-dict key, shape) -- not on module construction order -- and the
reference model (``tests/golden/make_golden.py``), the CPU oracle and the HIP
engine all see bit-identical weights.

Distribution rules (chosen to keep activations O(1) like PyTorch's default
kaiming-uniform init, while making every affine term non-trivial so parity
tests exercise it):

* conv / linear weights (ndim >= 2): U(-1/sqrt(fan_in), 1/sqrt(fan_in)),
  fan_in = prod(shape[1:]) (PyTorch's convention, also for ConvTranspose3d);
* InstanceNorm affine ``weight`` (1-D): 1 + 0.1 * N(0,1);
* biases (1-D): U(-0.1, 0.1);
* ``mag_scale``: 1 + 0.1 * N(0,1)  (FourierGate, models.py:1523);
* ``freq_mask`` / ``_mask``: all ones unless ``mask_jitter`` > 0 -- the
  reference creates it lazily as ones and never optimises it;
* BatchNorm buffers (3DUNet): ``running_mean`` U(-0.1, 0.1), ``running_var``
  U(0.5, 1.5) (a valid variance), ``num_batches_tracked`` 0.
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterable, Tuple

import numpy as np

__all__ = ["synth_param", "synth_state"]


def synth_param(name: str, shape: Tuple[int, ...], seed: int = 0,
                mask_jitter: float = 0.0) -> np.ndarray:
    rng = np.random.default_rng([int(seed), zlib.crc32(name.encode("utf-8"))])
    shape = tuple(int(s) for s in shape)
    leaf = name.rsplit(".", 1)[-1]
    if leaf in ("freq_mask", "_mask"):
        out = np.ones(shape, dtype=np.float64)
        if mask_jitter > 0:
            out = out + mask_jitter * rng.standard_normal(shape)
    elif leaf == "running_var":
        out = rng.uniform(0.5, 1.5, size=shape)
    elif leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    elif leaf == "mag_scale":
        out = 1.0 + 0.1 * rng.standard_normal(shape)
    elif len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        b = 1.0 / np.sqrt(max(1, fan_in))
        out = rng.uniform(-b, b, size=shape)
    elif leaf == "weight":
        out = 1.0 + 0.1 * rng.standard_normal(shape)
    else:
        out = rng.uniform(-0.1, 0.1, size=shape)
    return out.astype(np.float32)


def synth_state(named_shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int = 0,
                mask_jitter: float = 0.0) -> Dict[str, np.ndarray]:
    """Generate a full state dict.  ``_mask`` and ``freq_mask`` are the same
    tensor in the reference (models.py:1532-1535), so both keys get the values
    generated for the ``freq_mask`` name."""
    out: Dict[str, np.ndarray] = {}
    for name, shape in named_shapes:
        gen_name = name[:-len("_mask")] + "freq_mask" if name.endswith("._mask") else name
        out[name] = synth_param(gen_name, shape, seed, mask_jitter)
    return out
