#!/usr/bin/env python3
"""Average launch time of bench.py kernel probes (resident production-shape inputs, 20 launches
in a HIP graph, HIP events on the replay stream):  python3 tools/probe_time.py k_pm_fwd k_pm_bwd2"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for kind in sys.argv[1:]:
        launch, algo, flops, desc = bench.PROBES[kind](dev, kind)
        ts = sorted(bench.timed_launch(dev, launch) for _ in range(3))
        t = ts[1]
        print(f"{kind:14s} {t * 1e6:8.1f} us  {algo / t / 1e9:7.0f} GB/s  {desc}", flush=True)


if __name__ == "__main__":
    main()
