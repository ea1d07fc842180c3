#!/usr/bin/env python3
"""Average per-dispatch PMC values of kernels matching a substring: pmc_read.py TAG [kernel-substr]"""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "vq3d"
vals = collections.defaultdict(list)
for path in sorted(glob.glob(f"gpurun_out/pmc_{tag}_*/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
for c, v in sorted(vals.items()):
    print(f"{c:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
