#!/usr/bin/env python3
"""Launch one 1x1x1 conv pass N times (for rocprofv3 PMC passes on a single kernel).

    python3 tools/pw_kernel.py CIN COUT H W D {fwd|dgrad|wgrad} [N]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))

import torch  # noqa: E402

from vq3d import ops  # noqa: E402


def main():
    cin, cout, h, w, d = [int(v) for v in sys.argv[1:6]]
    mode = sys.argv[6]
    n = int(sys.argv[7]) if len(sys.argv) > 7 else 5
    dev = torch.device("cuda:0")
    cl = torch.channels_last_3d
    x = torch.randn((1, cin, h, w, d), device=dev).bfloat16().contiguous(memory_format=cl)
    g = torch.randn((1, cout, h, w, d), device=dev).bfloat16().contiguous(memory_format=cl)
    wt = torch.randn((cout, cin, 1, 1, 1), device=dev) * 0.1
    dw = torch.zeros_like(wt)
    a, b = torch.zeros(1, device=dev), torch.zeros(1, device=dev)
    g1 = ops.ConvGeom(1)
    flush = torch.empty(300 * 2 ** 20 // 4, device=dev)
    for _ in range(n):
        flush.zero_()
        if mode == "fwd":
            ops.conv_fwd(x, wt, g1, pro=(a, b), act=(a, b))
        elif mode == "dgrad":
            ops.conv_bwd(g, x, wt, g1, pro=(a, b), aux=x, addend=x if cin == cout else None)
        else:
            ops.conv_bwd(g, x, wt, g1, pro=(a, b), want_gx=False, dw=dw)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
