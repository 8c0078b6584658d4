"""Summarise a rocprofv3 kernel_stats.csv as ms/step (usage: kstats.py CSV STEPS)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {int(r['Calls']):6d} calls "
          f"{float(r['AverageNs'])/1e3:9.1f} us avg {float(r['Percentage']):5.1f}%  {r['Name'][:80]}")
print(f"total {tot/1e6/steps:.2f} ms/step")
