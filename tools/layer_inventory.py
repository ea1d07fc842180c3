#!/usr/bin/env python3
"""List every conv / upsample launch of one training step (shapes only, no GPU): the host
path runs on CPU tensors with the C-ABI calls recorded instead of executed.

    python3 tools/layer_inventory.py [config] [H W D]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from vq3d import _lib as L  # noqa: E402

rec = collections.Counter()


def fake_call(name, *args):
    if name.startswith("vq3d_conv3d"):
        d = args[0]._obj
        key = (name[12:], "bf16" if d.dtype == 1 else "f32", d.cin + d.cin2, d.cout, (d.in_h, d.in_w, d.in_d),
               d.kernel, d.stride, "circ" if d.pad_mode else "zero")
        rec[key] += 1
    elif name.startswith("vq3d_upsample"):
        rec[(name[5:], args[2], tuple(args[3:6]))] += 1
    return 0


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "3l_pub"
    mkw, size, batch = bench.CONFIGS[cfg][:3]
    if len(sys.argv) > 4:
        size = tuple(int(v) for v in sys.argv[2:5])
    L.call = fake_call
    L.ptr = lambda t: t.data_ptr()
    L.stream = lambda: None
    import vq3d
    from vq3d import functional as F
    F.grad_buf = lambda p: torch.zeros_like(p) if p is not None else None
    model = vq3d.VQVAE(vq3d.default_args(**mkw))
    x = torch.rand((batch, 1) + size) * 4.5 - 0.5
    nvs = torch.full((batch,), size[2], dtype=torch.int64)
    loss = model.training_step((x, nvs), 0)
    loss.backward()
    for k, n in sorted(rec.items(), key=lambda kv: str(kv[0])):
        print(n, k)


if __name__ == "__main__":
    main()
