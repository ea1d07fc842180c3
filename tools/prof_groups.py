#!/usr/bin/env python3
"""Last training step of a rocprofv3 --kernel-trace database grouped by (kernel, grid):
    python tools/prof_groups.py DB [TOP] [FILTER]"""
import collections
import re
import sqlite3
import sys

rows = sqlite3.connect(sys.argv[1]).execute(
    "select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels order by start").fetchall()
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
flt = sys.argv[3] if len(sys.argv) > 3 else ""
adam = [i for i, r in enumerate(rows) if "adam" in r[0]]
seg = rows[adam[-2] + 1: adam[-1] + 1]
print(f"last step: {len(seg)} kernels, span {(seg[-1][2] - seg[0][1]) / 1e6:.2f} ms")
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    n = re.sub(r"\(.*$", "", r[0].replace("(anonymous namespace)::", ""))[:56]
    k = (n, r[3] // max(1, r[6]), r[4], r[5], r[6])
    agg[k][0] += 1
    agg[k][1] += (r[2] - r[1]) / 1e3
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    if flt in k[0]:
        print(f"{t:9.0f} us {n:5d}x {t / n:8.1f}  {k[0]}  wg={k[1]}x{k[2]}x{k[3]} ({k[4]})")
