#!/usr/bin/env python3
"""Summarise gpurun_out/abv_*.log bench lines (scripts/ab_variants.sh)."""
import glob
import json

for f in sorted(glob.glob("gpurun_out/abv_*.log")):
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print(f, "no result")
        continue
    d = json.loads(lines[-1])
    r = d["roofline"]
    print(f"{f[15:-4]:24s} {d['ms_per_step']:7.2f} ms  conv {r['achieved']:6.1f} TF ({r['frac']:.3f})  " +
          " ".join(f"{k}={v:.2f}" for k, v in r["per_class_ms_per_step"].items()))
