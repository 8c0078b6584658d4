#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per spff kernel (sums over dispatches).

    python scripts/pmc_summary.py gpurun_out/kpmc/run_counter_collection.csv \
        [gpurun_out/kpmc2/run_counter_collection.csv ...]

Derived (MI355X: 256 CUs x 4 SIMDs, 8 XCDs): clock = GRBM_GUI_ACTIVE / 8 / kernel time
(rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs), MFMA share = SQ_VALU_MFMA_BUSY_CYCLES /
(1024 SIMDs x GRBM_GUI_ACTIVE / 8), and the SQ wave-state split (SQ_* count quad-cycles)."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(dict)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "spff::" not in name:
            continue
        short = name.split("(")[0].replace("void ", "")
        acc[short][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[short][(path, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, c in acc.items():
    ns = sum(dur[k].values()) / max(1, len({p for p, _ in dur[k]}))  # per counter pass
    line = [f"{k}: {ns / 1e6:.3f} ms"]
    if c.get("GRBM_GUI_ACTIVE"):
        line.append(f"clock {c['GRBM_GUI_ACTIVE'] / 8 / ns:.2f} GHz")
        if c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            line.append(f"MFMA busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (128 * c['GRBM_GUI_ACTIVE']):.3f}")
    w = c.get("SQ_WAVE_CYCLES")
    if w:
        for n in ("SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if n in c:
                line.append(f"{n[3:]} {c[n] / w:.3f}")
    if c.get("SQ_LDS_IDX_ACTIVE"):
        line.append(f"LDS conflict share {c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:.3f}")
    line += [f"{n}={v:.3g}" for n, v in sorted(c.items()) if n in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS")]
    print("  ".join(line))
