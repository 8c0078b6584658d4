#!/usr/bin/env python3
"""Compare gpurun_out/cfg2_<tag>.npz gradient dumps against cfg2_<ref>.npz:
per-parameter relative L2, worst first."""
import sys

import numpy as np

ref = np.load(f"gpurun_out/cfg2_{sys.argv[1]}.npz")
for tag in sys.argv[2:]:
    z = np.load(f"gpurun_out/cfg2_{tag}.npz")
    rows = []
    for k in ref.files:
        a, b = ref[k].astype(np.float64), z[k].astype(np.float64)
        rows.append((np.linalg.norm(a - b) / max(np.linalg.norm(a), 1e-30), k))
    rows.sort(reverse=True)
    print(tag, " ".join(f"{k}={r:.1e}" for r, k in rows[:5]))
