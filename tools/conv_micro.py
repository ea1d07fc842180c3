#!/usr/bin/env python3
"""Micro-benchmark one conv launch (forward or backward-data / weight) of the vq3d library.

    python3 tools/conv_micro.py CIN COUT H W D K S P CIRC [fwd|dgrad|wgrad] [bf16|fp32] [iters]
Prints the average launch time (HIP events around a graph replay of `iters` launches) and
algorithmic GB/s."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))

import torch  # noqa: E402

from vq3d import ops  # noqa: E402


def main():
    cin, cout, h, w, d, k, s, p, circ = [int(v) for v in sys.argv[1:10]]
    mode = sys.argv[10] if len(sys.argv) > 10 else "fwd"
    dt = torch.bfloat16 if (sys.argv[11] if len(sys.argv) > 11 else "bf16") == "bf16" else torch.float32
    iters = int(sys.argv[12]) if len(sys.argv) > 12 else 20
    dev = torch.device("cuda:0")
    geom = ops.ConvGeom(k, s, p, bool(circ))
    x = torch.randn((1, cin, h, w, d), device=dev).to(dt).contiguous(memory_format=torch.channels_last_3d)
    wt = torch.randn((cout, cin, k, k, k), device=dev) * 0.1
    oh, ow, od = geom.out(h), geom.out(w), geom.out(d)
    g = torch.randn((1, cout, oh, ow, od), device=dev).to(dt).contiguous(memory_format=torch.channels_last_3d)
    dw = torch.zeros_like(wt)

    def run():
        if mode == "fwd":
            ops.conv_fwd(x, wt, geom)
        elif mode == "dgrad":
            ops.conv_bwd(g, x, wt, geom, want_gx=True, dw=None) if False else _dgrad_only()
        else:
            _wgrad_only()

    import ctypes
    from vq3d import _lib as L

    def _dgrad_only():
        desc, _ = ops.conv_desc(x.dtype, 1, cin, 0, cout, h, w, d, geom, 0)
        gx = torch.empty_like(x)
        epi = L.DgradEpilogue()
        ws, wsb = ops._ws(desc, L.PASS_BWD_DATA, x.device)
        L.call("vq3d_conv3d_bwd_data", ctypes.byref(desc), L.ptr(g), None, L.ptr(wt), None, ctypes.byref(epi),
               L.ptr(gx), None, None, None, None if ws is None else L.ptr(ws), wsb, L.stream())

    def _wgrad_only():
        desc, _ = ops.conv_desc(x.dtype, 1, cin, 0, cout, h, w, d, geom, 0)
        ws, wsb = ops._ws(desc, L.PASS_BWD_WEIGHT, x.device)
        L.call("vq3d_conv3d_bwd_weight", ctypes.byref(desc), L.ptr(x), None, L.ptr(g), None, None, L.ptr(wt), None,
               L.ptr(dw), None, None, None, None if ws is None else L.ptr(ws), wsb, L.stream())

    for _ in range(3):
        run()
    # capture the launches in a HIP graph so host-side (Python / ctypes) overhead is not timed
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            for _ in range(iters):
                run()
    graph.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    graph.replay()
    e1.record(st)
    e1.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / iters
    byt = (x.numel() + g.numel()) * x.element_size()
    print(f"{mode} {cin}->{cout} {h}x{w}x{d} k{k}s{s}p{p}c{circ} {str(dt)[6:]}: {t * 1e6:9.1f} us  "
          f"{byt / t / 1e9:8.1f} GB/s algorithmic")


if __name__ == "__main__":
    main()
