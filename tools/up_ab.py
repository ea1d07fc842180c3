#!/usr/bin/env python3
"""Launch times of the step's upsample shapes (trilinear x2 and its adjoint, bf16), one process:
    VQ3D_LIB=... python3 tools/up_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from conv_ab import timed  # noqa: E402
from vq3d import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    cl = torch.channels_last_3d
    for (c, h, w, d) in ((4, 256, 256, 64), (9, 128, 128, 32), (16, 64, 64, 16)):
        x = torch.randn((1, c, h, w, d), device=dev).bfloat16().contiguous(memory_format=cl)
        gy = torch.randn((1, c, 2 * h, 2 * w, 2 * d), device=dev).bfloat16().contiguous(memory_format=cl)
        aux = torch.randn_like(x)
        ab = torch.full((1,), 0.1, device=dev)
        pre = torch.zeros(1, device=dev)
        tf = timed(lambda: ops.upsample2x(x))
        tb = timed(lambda: ops.upsample2x_bwd(gy, x.shape, aux=aux, aux_b=ab, dpro_pre=pre, dpro_post=pre))
        by = x.numel() * 2 * 9
        print(f"upsample c{c} {h}x{w}x{d}: fwd {tf * 1e6:7.1f} us ({by / tf / 1e9:5.0f} GB/s)  "
              f"bwd {tb * 1e6:7.1f} us ({by / tb / 1e9:5.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
