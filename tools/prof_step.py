#!/usr/bin/env python3
"""Kernel time of the LAST training step in a rocprofv3 --kernel-trace database, delimited by the
Adam kernel (one per step): per-kernel totals, launch count, busy time vs the step's span.

    python tools/prof_step.py gpurun_out/prof/run_results.db [TOP]
"""
import collections
import re
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = sqlite3.connect(db).execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
adam = [i for i, r in enumerate(rows) if "adam" in r[0]]
if len(adam) < 2:
    sys.exit("need two Adam launches in the trace")
seg = rows[adam[-2] + 1: adam[-1] + 1]
span = (seg[-1][2] - seg[0][1]) / 1e3
busy = sum(r[2] - r[1] for r in seg) / 1e3


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*$", "", n)
    return n[:70]


agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    k = short(r[0])
    agg[k][0] += 1
    agg[k][1] += (r[2] - r[1]) / 1e3
print(f"last step: {len(seg)} kernels, span {span / 1e3:.2f} ms, busy {busy / 1e3:.2f} ms")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{t:10.1f} us {n:6d}x {t / n:8.1f} avg  {k}")
