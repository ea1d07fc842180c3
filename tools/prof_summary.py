#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace csv: time per step by kernel and by launch shape."""
import collections
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
agg = collections.defaultdict(lambda: [0, 0.0])
tot = 0.0
for r in rows:
    dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += dt
    k = (r["Kernel_Name"].split("(")[0][:48], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[k][0] += 1
    agg[k][1] += dt
print(f"total kernel time {tot / 1e3 / steps:.2f} ms/step, {len(rows) / steps:.0f} launches/step")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{t / steps:9.1f} us/step {n / steps:6.0f}/step avg {t / n:8.1f}  {k}")
