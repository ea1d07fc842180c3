#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (--kernel-trace): time per step by kernel name + grid.

    python tools/prof_db.py gpurun_out/prof/run_results.db STEPS [TOP] [--by-name]
"""
import collections
import sqlite3
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3].isdigit() else 40
by_name = "--by-name" in sys.argv
c = sqlite3.connect(path)
rows = c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, duration, start, end from kernels").fetchall()
agg = collections.defaultdict(lambda: [0, 0.0])
tot = 0.0
for name, gx, gy, gz, wx, dur, st, en in rows:
    dt = dur / 1e3
    tot += dt
    short = name.split("(")[0][:60]
    k = short if by_name else (short, gx // max(wx, 1), gy, gz)
    agg[k][0] += 1
    agg[k][1] += dt
span = (max(r[7] for r in rows) - min(r[6] for r in rows)) / 1e6
print(f"total kernel time {tot / 1e3 / steps:.2f} ms/step, {len(rows) / steps:.0f} launches/step, "
      f"trace span {span:.1f} ms")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{t / steps:9.1f} us/step {n / steps:6.0f}/step avg {t / n:8.1f}  {k}")
