#!/usr/bin/env python3
"""Launch the dominant kernel (bench.py DOM: 3x3x3 circular conv 9->9 @128x128x32, bf16) N
times, for rocprofv3 PMC passes:

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
from vq3d import ops  # noqa: E402


def main(n=int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    dev = torch.device("cuda:0")
    h, w, d = bench.DOM["grid"]
    g = torch.Generator(device=dev).manual_seed(7)
    x = (torch.randn((1, bench.DOM["cin"], h, w, d), device=dev, generator=g) * 0.5).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last_3d)
    wt = torch.randn((bench.DOM["cout"], bench.DOM["cin"], 3, 3, 3), device=dev, generator=g) * 0.1
    # evict the inputs from the Infinity Cache between launches (300 MB write)
    flush = torch.empty(300 * 2 ** 20 // 4, device=dev)
    for _ in range(n):
        flush.zero_()
        ops.conv_fwd(x, wt, ops.ConvGeom(3, 1, 1, True))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
