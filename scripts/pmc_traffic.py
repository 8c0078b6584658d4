#!/usr/bin/env python3
"""Per-launch HBM traffic of the dominant conv kernel from two rocprofv3 --pmc
passes of bench.py (FETCH_SIZE, WRITE_SIZE; scripts/gpu_round.sh pmc), with
MI355X_MICROARCH.md's gfx950 correction: FETCH_SIZE reports half the bytes of
16-B/lane streaming reads, so traffic = 2 x FETCH_SIZE + WRITE_SIZE (both in KB).

    python scripts/pmc_traffic.py gpurun_out/pmc_fetch/run_counter_collection.csv \
        gpurun_out/pmc_write/run_counter_collection.csv profiles/r03_pmc_conv.json \
        [per_kernel.csv] [--bench-log gpurun_out/pmc_fetch.log]

--bench-log: the profiled bench.py run's output; its JSON line's `workload_key` and
build digest are stored with the traffic, and bench.py uses the traffic only for a run
with the same workload key (otherwise `roofline.traffic` is null).
"""
import csv
import json
import statistics
import sys

KERNEL = "k_conv3d_fwd_x"


def per_dispatch(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            out[int(r["Dispatch_Id"])] = (float(r["Counter_Value"]), r["Kernel_Name"].split("(")[0])
    return out


bench_line = None
if "--bench-log" in sys.argv:
    i = sys.argv.index("--bench-log")
    for ln in open(sys.argv[i + 1]):
        if ln.startswith("{") and '"workload_key"' in ln:
            bench_line = json.loads(ln)
    del sys.argv[i:i + 2]

fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], "WRITE_SIZE")
f_kb = [v for v, _ in fetch.values()]
w_kb = [v for v, _ in write.values()]
fetch_b = 2 * statistics.fmean(f_kb) * 1024
write_b = statistics.fmean(w_kb) * 1024
res = {"kernel": KERNEL, "launches_fetch": len(f_kb), "launches_write": len(w_kb),
       "fetch_bytes_per_launch_corrected": fetch_b, "write_bytes_per_launch": write_b,
       "hbm_bytes_per_launch": fetch_b + write_b,
       "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, --kernel-trace), "
                 "bench.py --steps 1 --warmup 1; traffic = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B), "
                 "averaged over the fwd+dgrad launches"}
if bench_line is not None:
    res["workload_key"] = bench_line["workload_key"]
    res["lib_sources_sha256"] = bench_line.get("build", {}).get("lib_sources_sha256")
    res["compulsory_bytes_per_launch"] = bench_line["roofline"]["compulsory_bytes_per_launch"]
    res["traffic_over_compulsory"] = res["hbm_bytes_per_launch"] / res["compulsory_bytes_per_launch"]
json.dump(res, open(sys.argv[3], "w"), indent=1)
print(json.dumps(res, indent=1))

# per-kernel table of the same two passes (all spff kernels): corrected HBM bytes and the
# effective bandwidth over the traced duration -- the memory-bound kernels' evidence.
if len(sys.argv) > 4:
    import collections
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0, 0])
    for path, ctr, idx in ((sys.argv[1], "FETCH_SIZE", 0), (sys.argv[2], "WRITE_SIZE", 1)):
        for r in csv.DictReader(open(path)):
            if "spff::" not in r["Kernel_Name"] or r["Counter_Name"] != ctr:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            a = agg[k]
            a[idx] += float(r["Counter_Value"]) * 1024 * (2 if idx == 0 else 1)
            if idx == 0:
                a[2] += 1
                a[3] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    with open(sys.argv[4], "w") as f:
        f.write("kernel,launches,fetch_bytes_x2,write_bytes,hbm_bytes_per_launch,ms_per_launch,GBps\n")
        for k, (fb, wb, n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][0] - kv[1][1]):
            f.write(f"\"{k}\",{n},{fb:.0f},{wb:.0f},{(fb + wb) / max(1, n):.0f},"
                    f"{ns / max(1, n) / 1e6:.4f},{(fb + wb) / max(1, ns):.1f}\n")
