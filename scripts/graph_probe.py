#!/usr/bin/env python3
"""Probe: the SPFF step (forward + ce_plus_macro_dice + backward, bench.py's default
workload) captured once into a HIP graph (torch.cuda.graph) and replayed, against the eager
step: gradients and loss must be bitwise equal (the engine is deterministic), then ms/step of
both."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "spff-unet-spcct_amd")]

import torch  # noqa: E402

from bench import build_model  # noqa: E402
from innovative3D.distributed import DataParallelSPFF  # noqa: E402
from innovative3D.synthetic import synthetic_batch  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    core, _ = build_model(13, 32, 5, 128, dev)
    core.math = "f16x3"
    x, y = synthetic_batch(2, 5, 128, 128, 128, 13, ignore_frac=0.01, seed=0)
    x, y = x.to(dev), y.to(dev)
    runner = DataParallelSPFF(core, 13, 255)

    def step():
        loss, _conf = runner.step(x, y)
        return loss

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ref_loss = float(step())
    ref = [p.grad.clone() for p in core.parameters()]
    # capture
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gl = step()
    g.replay()
    torch.cuda.synchronize()
    same = all(torch.equal(p.grad, r) for p, r in zip(core.parameters(), ref))
    print(f"graph replay: loss {float(gl):.8f} vs eager {ref_loss:.8f}; gradients bitwise equal: {same}",
          flush=True)
    for name, fn in (("eager", step), ("graph", g.replay)) * 5:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(30):
            fn()
        torch.cuda.synchronize()
        print(f"{name}: {(time.perf_counter() - t) / 30 * 1e3:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
