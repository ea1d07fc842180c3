#!/usr/bin/env python3
"""Launch one of bench.py's kernel probes (default: the dominant one of profiles/r02_step_top.json)
N times with the Infinity Cache flushed in between, for rocprofv3 PMC passes (one counter
block per run, MI355X_MICROARCH.md §HBM):

  rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run --output-format csv -- \
      python3 tools/dominant_kernel.py k_pm_bwd2
  rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run --output-format csv -- \
      python3 tools/dominant_kernel.py k_pm_bwd2
  python3 tools/pmc_traffic.py k_pm_bwd2 gpurun_out/pmc_f gpurun_out/pmc_w > profiles/r02_pmc_k_pm_bwd2.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def dominant():
    for e in json.load(open(bench.STEP_TOP))["by_name"]:
        k = bench.probe_for(e["kernel"])
        if k:
            return k
    return "k_pm_bwd2"


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else dominant()
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda:0")
    launch = bench.PROBES[kind](dev, kind)[0]
    # a 300 MB READ sweep between launches evicts the inputs from L2 and the Infinity Cache without
    # leaving dirty lines whose write-back would be counted in the next launch's WRITE_SIZE
    flush = torch.ones(300 * 2 ** 20 // 4, device=dev)
    sink = torch.empty((), device=dev)
    torch.cuda.synchronize()
    for _ in range(n):
        torch.sum(flush, dim=0, out=sink)
        launch()
    torch.cuda.synchronize()
    print(kind)


if __name__ == "__main__":
    main()
