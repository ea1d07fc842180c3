#!/usr/bin/env python3
"""Per-kernel average PMC values over rocprofv3 --pmc passes: pmc_kernels.py DIR_GLOB [substr]

Every counter_collection.csv under the directories matching DIR_GLOB is read; values are summed
per (dispatch, counter) over the XCD / shader-engine instances and averaged per kernel name."""
import collections
import csv
import glob
import re
import sys

pat = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "vq3d"
per = collections.defaultdict(float)
names = {}
for path in sorted(glob.glob(pat)):
    for f in glob.glob(f"{path}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"].replace(", ", "_"):
                continue
            k = re.sub(r"\(.*$", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))[:60]
            key = (f, r["Dispatch_Id"])
            names[key] = k
            per[(key, r["Counter_Name"])] += float(r["Counter_Value"])
agg = collections.defaultdict(list)
for (key, c), v in per.items():
    agg[(names[key], c)].append(v)
kern = sorted({k for k, _ in agg})
for k in kern:
    print(k)
    for (kk, c), v in sorted(agg.items()):
        if kk == k:
            print(f"    {c:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
