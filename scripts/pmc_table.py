#!/usr/bin/env python3
"""Per-kernel HBM traffic table from the two rocprofv3 --pmc passes of
scripts/gpu_round.sh pmc (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE),
with each kernel's average launch time from the same passes' kernel traces.

    python scripts/pmc_table.py gpurun_out/pmc_fetch gpurun_out/pmc_write out.csv
"""
import collections
import csv
import pathlib
import sys

fdir, wdir, out = map(pathlib.Path, sys.argv[1:4])


def load(d, counter):
    val = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(d / "run_counter_collection.csv")):
        if r["Counter_Name"] == counter and "spff::" in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            val[k] += float(r["Counter_Value"]) * 1024
            n[k].add(r["Dispatch_Id"])
    return val, {k: len(v) for k, v in n.items()}


def times(d):
    t = collections.defaultdict(list)
    for r in csv.DictReader(open(d / "run_kernel_trace.csv")):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        t[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return t


fv, fn = load(fdir, "FETCH_SIZE")
wv, _ = load(wdir, "WRITE_SIZE")
tt = times(fdir)
rows = []
for k in fv:
    L = fn[k]
    hbm = (2 * fv[k] + wv.get(k, 0.0)) / L
    ms = sum(tt[k]) / len(tt[k]) if tt.get(k) else float("nan")
    rows.append((k, L, 2 * fv[k], wv.get(k, 0.0), hbm, ms, hbm / ms / 1e6 if ms == ms else 0))
rows.sort(key=lambda r: -r[4] * r[1])
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "launches", "fetch_bytes_x2", "write_bytes", "hbm_bytes_per_launch",
                "ms_per_launch", "GBps"])
    for r in rows:
        w.writerow([r[0], r[1], int(r[2]), int(r[3]), int(r[4]), f"{r[5]:.4f}", f"{r[6]:.1f}"])
print(open(out).read()[:1200])
