#!/usr/bin/env python3
"""Write profiles/<round>/README.md (+ copies of the stats CSV and the bench JSON
line) from a rocprofv3 --kernel-trace --stats run of bench.py.

    python scripts/prof_readme.py gpurun_out/prof/run_kernel_stats.csv \
        gpurun_out/bench_quick.log profiles/r01 --steps 4 --note "..."
"""
import argparse
import csv
import json
import pathlib
import shutil

ap = argparse.ArgumentParser()
ap.add_argument("stats")
ap.add_argument("bench_log")
ap.add_argument("out_dir")
ap.add_argument("--steps", type=float, default=4.0, help="profiled steps (warmup + timed)")
ap.add_argument("--cmd", default="rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run "
                "--output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline skip")
ap.add_argument("--note", default="")
ap.add_argument("--what", default="SPFF-UNet fwd+loss+bwd, batch 2 x 5 x 128^3, K=13, base 32")
ap.add_argument("--bench-json", default="bench_quick.json")
a = ap.parse_args()
out = pathlib.Path(a.out_dir)
out.mkdir(parents=True, exist_ok=True)
rows = list(csv.DictReader(open(a.stats)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
lines = [f"# {out.name} rocprofv3 --kernel-trace --stats summary", "",
         f"Command (on the MI355X box, repo root): `{a.cmd}`", "",
         f"{a.steps:g} steps profiled (warm-up + timed) of {a.what}.  Total kernel time "
         f"{tot / 1e6:.1f} ms = "
         f"{tot / 1e6 / a.steps:.1f} ms/step.", ""]
if a.note:
    lines += [a.note, ""]
lines += ["| kernel | calls | total ms | ms/step | avg us | % |", "|---|---:|---:|---:|---:|---:|"]
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].split("(")[0].replace("void ", "")
    lines.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                 f"{float(r['TotalDurationNs']) / 1e6 / a.steps:.2f} | "
                 f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
bench = [x for x in open(a.bench_log) if x.startswith("{")]
if bench:
    d = json.loads(bench[-1])
    (out / a.bench_json).write_text(json.dumps(d, indent=1) + "\n")
    r = d.get("roofline") or {}
    lines += ["", f"Bench line of the same build: {d['value'] / 1e6:.2f} Mvox/s, "
              f"{d['ms_per_step']:.1f} ms/step, conv math `{d.get('conv_math', 'f32')}`"
              + (f"; dominant kernel {r.get('kernel')}: {r.get('achieved', 0):.1f} TFLOP/s = "
                 f"{100 * (r.get('frac') or 0):.1f} % of {r.get('peak', 0):.1f}, average launch "
                 f"{r.get('avg_launch_ms', 0):.3f} ms (HIP events)." if r else ".")]
shutil.copy(a.stats, out / ("kernel_stats_" + a.bench_json.replace(".json", ".csv")))
(out / "README.md").write_text("\n".join(lines) + "\n")
print((out / "README.md").read_text()[:1500])
