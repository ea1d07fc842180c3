#!/usr/bin/env python3
"""Launch the dominant kernel (bench.py DOM: fused 18-channel PreAct block forward @128x128x32,
bf16) N times with the Infinity Cache flushed in between, for rocprofv3 PMC passes:

  rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run --output-format csv -- \
      python3 tools/dominant_kernel.py
  rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run --output-format csv -- \
      python3 tools/dominant_kernel.py
  python3 tools/pmc_traffic.py gpurun_out/pmc_f gpurun_out/pmc_w > profiles/pmc_dominant.json
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main(n=int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    dev = torch.device("cuda:0")
    launch, _, _ = bench.dominant_setup(dev)
    flush = torch.empty(300 * 2 ** 20 // 4, device=dev)  # evicts the inputs from the Infinity Cache
    for _ in range(n):
        flush.zero_()
        launch()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
