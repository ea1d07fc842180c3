#!/usr/bin/env python3
"""Time the wide-block kernels (preact_wide.hip) one by one on resident tensors.

    python3 tools/wide_micro.py [H W D] [iters]

Per-call times (HIP events around a graph replay of `iters` calls) of the forward launch, the
bwd_data launch and the bwd_weight pair, for one 72-channel / branch-36 block."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))

import torch  # noqa: E402

from block_micro import timed  # noqa: E402


def main():
    from vq3d import _lib as L
    from vq3d import layers as VL
    from vq3d import ops
    from vq3d.flat import FlatParams
    from vq3d.functional import StackPlan
    h, w, d = [int(v) for v in sys.argv[1:4]] if len(sys.argv) > 3 else (32, 32, 8)
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    blk = VL.PreActFixupResBlock(72, 72, mode="same").to(dev)
    FlatParams(blk.parameters(), dev)
    with torch.no_grad():
        for p in blk.parameters():
            p.normal_(0, 0.1)
    cl = torch.channels_last_3d
    x = torch.randn((1, 72, h, w, d), device=dev).contiguous(memory_format=cl)
    g = torch.randn((1, 72, h, w, d), device=dev).contiguous(memory_format=cl)
    plan = StackPlan([blk])
    ptab, _ = plan.tables(dev)
    img, per = ops.preact_wide_pack(ptab, 1, 72, 36, dev)
    out, t2, t3 = ops.preact_wide_fwd(x, img.data_ptr(), blk)
    gx = torch.empty_like(x)
    nws = int(L.query("vq3d_preact_wide_workspace_bytes", 1, h, w, d))
    ws = torch.empty(nws, dtype=torch.uint8, device=dev)
    prm = ops._preact_params(blk)
    names = {"dw1": blk.branch_conv1.weight, "dw2": blk.branch_conv2.weight, "dw3": blk.branch_conv3.weight,
             "dbias1a": blk.bias1a, "dbias1b": blk.bias1b, "dbias2a": blk.bias2a, "dbias2b": blk.bias2b,
             "dbias3a": blk.bias3a, "dbias3b": blk.bias3b, "dscale": blk.scale, "dbias4": blk.bias4}
    gr = L.PreactGrads(*[ops._p(names[n].grad) for n, _ in L.PreactGrads._fields_])

    def fwd():
        L.call("vq3d_preact_wide_fwd", L.BF16, 1, 72, 36, h, w, d, L.ptr(x), ctypes.c_void_p(img.data_ptr()),
               ctypes.byref(prm), L.ptr(out), L.ptr(t2), L.ptr(t3), L.stream())

    def bwd_data():
        L.call("vq3d_preact_wide_bwd_data", L.BF16, 1, 72, 36, h, w, d, L.ptr(g), L.ptr(x), L.ptr(t2), L.ptr(t3),
               ctypes.c_void_p(img.data_ptr()), ctypes.byref(prm), L.ptr(ws), ctypes.c_size_t(nws), L.ptr(gx),
               L.stream())

    def bwd_weight():
        L.call("vq3d_preact_wide_bwd_weight", L.BF16, 1, 72, 36, h, w, d, L.ptr(g), L.ptr(x), L.ptr(t2), L.ptr(t3),
               ctypes.byref(prm), ctypes.byref(gr), L.ptr(ws), ctypes.c_size_t(nws), L.stream())

    def pack():
        L.call("vq3d_preact_wide_pack", L.BF16, 1, 72, 36, L.ptr(ptab), L.ptr(img), L.stream())
    bwd_data()
    res = {n: timed(f, iters) for n, f in (("pack", pack), ("fwd", fwd), ("bwd_data", bwd_data),
                                            ("bwd_weight", bwd_weight))}
    print(f"wide C72 BR36 {h}x{w}x{d}:", {k: round(v, 1) for k, v in res.items()}, "us per call")


if __name__ == "__main__":
    main()
