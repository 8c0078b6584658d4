#!/usr/bin/env python3
"""Summarise scripts/ab_bench.sh output: per library, ms/step of every round and the mean
per-class ms/step (roofline.per_class_ms_per_step) -- gpurun_out/ab_<i>.jsonl."""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_[0-9]*.jsonl")):
    rows = [json.loads(line) for line in open(f) if line.strip()]
    ms = [r["ms_per_step"] for r in rows]
    pc = {}
    for r in rows:
        for k, v in r["roofline"]["per_class_ms_per_step"].items():
            pc.setdefault(k, []).append(v)
    print(f"{f}: ms/step {' '.join(f'{m:.3f}' for m in ms)} (mean {sum(ms) / len(ms):.3f})  frac "
          f"{rows[-1]['roofline']['frac']:.3f}")
    print("   " + "  ".join(f"{k} {sum(v) / len(v):.3f}" for k, v in pc.items()))
