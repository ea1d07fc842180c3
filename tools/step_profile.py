#!/usr/bin/env python3
"""Per-step kernel breakdown from a rocprofv3 --kernel-trace run of bench.py.

    python tools/step_profile.py <rocprofv3 output dir> [TOP] [--json OUT]

A step is delimited by the Adam kernel (one launch per training step); the LAST complete step
of the trace is summarised: launches, span, busy time, and the kernels ranked by their total
time in the step (name without the argument list + grid).  --json writes the ranking that
bench.py reads to pick the dominant kernel (profiles/r02_step_top.json).
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def load(d):
    paths = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = []
    for p in paths:
        for r in csv.DictReader(open(p)):
            rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0),
                         int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)))
    rows.sort(key=lambda r: r[1])
    return rows


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*$", "", n)
    return n.strip()[:90]


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 40
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    rows = load(d)
    adam = [i for i, r in enumerate(rows) if "adam" in r[0]]
    if len(adam) < 2:
        sys.exit("need two Adam launches in the trace")
    seg = rows[adam[-2] + 1: adam[-1] + 1]
    span = (seg[-1][2] - seg[0][1]) / 1e3
    busy = sum(r[2] - r[1] for r in seg) / 1e3
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        k = f"{short(r[0])} [grid {r[3] // max(r[4], 1)}]"
        agg[k][0] += 1
        agg[k][1] += (r[2] - r[1]) / 1e3
    print(f"last step: {len(seg)} kernels, span {span / 1e3:.2f} ms, busy {busy / 1e3:.2f} ms")
    ranked = sorted(agg.items(), key=lambda kv: -kv[1][1])
    for k, (n, t) in ranked[:top]:
        print(f"{t:10.1f} us {n:6d}x {t / n:8.1f} avg  {k}")
    byname = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        k = short(r[0])
        byname[k][0] += 1
        byname[k][1] += (r[2] - r[1]) / 1e3
    if out:
        json.dump({"source": os.path.abspath(d), "launches": len(seg), "span_us": span, "busy_us": busy,
                   "by_name_grid": [{"kernel": k, "launches": n, "total_us": t, "avg_us": t / n}
                                    for k, (n, t) in ranked[:top]],
                   "by_name": [{"kernel": k, "launches": n, "total_us": t, "avg_us": t / n}
                               for k, (n, t) in sorted(byname.items(), key=lambda kv: -kv[1][1])[:top]]},
                  open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
