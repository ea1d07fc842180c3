#!/usr/bin/env python3
"""Average duration of the dominant-kernel launches that bench.py's roofline measurement issues
(the last N launches of the fused 18-channel block forward, bench.DOM), from a rocprofv3
--kernel-trace CSV, to cross-check bench.py's HIP-event figure.

    python3 tools/dominant_from_trace.py gpurun_out/stats/run_kernel_trace.csv [N]
"""
import csv
import json
import re
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    rows = [r for r in csv.DictReader(open(path)) if "k_preact_mid_fwd" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the roofline launches are the last n of the trace with the dominant launch geometry
    grid = (rows[-1]["Grid_Size_X"], rows[-1]["LDS_Block_Size"])
    sel = [r for r in rows if (r["Grid_Size_X"], r["LDS_Block_Size"]) == grid][-n:]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]
    m = re.search(r"k_preact_mid_fwd", sel[-1]["Kernel_Name"])
    print(json.dumps({"kernel": m.group(0) if m else sel[-1]["Kernel_Name"][:80], "launches": len(d),
                      "avg_us": sum(d) / len(d), "min_us": min(d), "max_us": max(d)}))


if __name__ == "__main__":
    main()
