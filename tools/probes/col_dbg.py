"""Debug: the (2, 1) column block's errors per tensor vs the float64 reference (VQ3D_LIB picks the build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import test_gpu_preact_col as T  # noqa: E402

dev = torch.device("cuda:0")
for half in T.HALF:
    T._H[0] = half
    for shape in T.SHAPES:
        b, c, h, w, d = shape
        if c != 2:
            continue
        blk = T._block(c, seed=h + d + c)
        gen = torch.Generator().manual_seed(7)
        x = T.rb(torch.randn(shape, generator=gen, dtype=torch.float64))
        gy = T.rb(torch.randn(shape, generator=gen, dtype=torch.float64))
        ry, rgx, rgp = T._ref_strict(blk, x, gy)
        m, y, xg = T._run(blk, x, gy, dev)
        errs = {"y": T.rel(y, ry), "gx": T.rel(xg.grad, rgx)}
        for n, p in m.named_parameters():
            errs[n] = T.rel(p.grad, rgp[n].reshape(p.shape))
        print(half, shape, {k: f"{v:.1e}" for k, v in errs.items()}, flush=True)
