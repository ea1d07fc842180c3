#!/usr/bin/env python3
"""Micro-benchmark the 1x1x1 conv backward-data with its fused epilogue options, one at a time
(graph replay, HIP events): which part of the PreAct conv1 backward costs what.

    python3 tools/pw_micro.py CIN COUT H W D [iters]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))

import torch  # noqa: E402

from vq3d import ops  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            for _ in range(iters):
                fn()
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    cin, cout, h, w, d = [int(v) for v in sys.argv[1:6]]
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
    dev = torch.device("cuda:0")
    cl = torch.channels_last_3d
    x = torch.randn((1, cin, h, w, d), device=dev).bfloat16().contiguous(memory_format=cl)
    g = torch.randn((1, cout, h, w, d), device=dev).bfloat16().contiguous(memory_format=cl)
    add = torch.randn_like(x)
    wt = torch.randn((cout, cin, 1, 1, 1), device=dev) * 0.1
    a, b = torch.zeros(1, device=dev), torch.zeros(1, device=dev)
    dpre, dpost = torch.zeros(1, device=dev), torch.zeros(1, device=dev)
    g1 = ops.ConvGeom(1)
    cases = {
        "fwd plain": lambda: ops.conv_fwd(x, wt, g1),
        "fwd pro+act": lambda: ops.conv_fwd(x, wt, g1, pro=(a, b), act=(a, b)),
        "dgrad plain": lambda: ops.conv_bwd(g, x, wt, g1, want_gx=True, dw=None),
        "dgrad +aux": lambda: ops.conv_bwd(g, x, wt, g1, pro=(a, b), aux=x),
        "dgrad +aux+addend": lambda: ops.conv_bwd(g, x, wt, g1, pro=(a, b), aux=x, addend=add),
        "dgrad +aux+addend+partials": lambda: ops.conv_bwd(g, x, wt, g1, pro=(a, b), aux=x, addend=add,
                                                           dpro_pre=dpre, dpro_post=dpost),
    }
    for name, fn in cases.items():
        # conv_bwd also runs the weight gradient when dw is given; keep dgrad-only timings
        t = timeit(fn, iters)
        print(f"{cin}->{cout} {h}x{w}x{d} {name:30s} {t:9.1f} us")


if __name__ == "__main__":
    main()
