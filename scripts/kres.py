#!/usr/bin/env python3
"""Per-kernel register summary of a hipcc -Rpass-analysis=kernel-resource-usage log:
    hipcc ... -Rpass-analysis=kernel-resource-usage 2> log; python scripts/kres.py log [filter]"""
import re
import subprocess
import sys

txt = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cur = None
rows = {}
for line in txt.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1)] = m.group(2)
names = list(rows)
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
except OSError:
    dem = names
for n, d in zip(names, dem):
    d = d.split("(")[0]
    if flt in d:
        r = rows[n]
        print(f"{d:70s} V{r.get('VGPRs')} A{r.get('AGPRs')} Vsp{r.get('VGPRs Spill')} S{r.get('TotalSGPRs')} Ssp{r.get('SGPRs Spill')} occ{r.get('Occupancy')}")
