#!/usr/bin/env python3
"""Launch times of a list of conv shapes in one process (A/B of two library builds via VQ3D_LIB).

    VQ3D_LIB=.../libvq3d_b.so python3 tools/conv_ab.py [SHAPE ...]
SHAPE = "cin,cout,h,w,d,k,s,p,circ,mode" (mode fwd | dgrad | wgrad); default: the step's k^3
shapes on the lines / generic engines.  Each time is the median of 3 HIP-graph replays of 20
launches (HIP events on the replay stream)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))

import torch  # noqa: E402

from vq3d import _lib as L  # noqa: E402
from vq3d import ops  # noqa: E402

DEFAULT = [
    "4,4,512,512,128,3,1,1,1,fwd", "4,4,512,512,128,3,1,1,1,dgrad", "4,4,512,512,128,3,1,1,1,wgrad",
    "4,4,512,512,128,4,2,1,1,fwd", "4,4,512,512,128,4,2,1,1,wgrad",
    "9,9,256,256,64,3,1,1,1,fwd", "9,9,256,256,64,3,1,1,1,dgrad",
    "8,8,256,256,64,4,2,1,1,fwd",
    "8,8,128,128,32,3,1,1,1,fwd", "8,8,128,128,32,3,1,1,1,dgrad",
    "16,16,64,64,16,3,1,1,1,fwd", "16,16,64,64,16,3,1,1,1,dgrad",
    "32,32,32,32,8,3,1,1,1,fwd", "32,32,32,32,8,3,1,1,1,dgrad",
    "64,64,16,16,4,3,1,1,1,fwd", "64,64,16,16,4,3,1,1,1,dgrad",
]


def timed(run, iters=20):
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            for _ in range(iters):
                run()
    graph.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        graph.replay()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 1e3 / iters)
    return sorted(ts)[1]


def one(spec, dev):
    f = spec.split(",")
    cin, cout, h, w, d, k, s, p, circ = [int(v) for v in f[:9]]
    mode = f[9]
    geom = ops.ConvGeom(k, s, p, bool(circ))
    cl = torch.channels_last_3d
    x = torch.randn((1, cin, h, w, d), device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    wt = torch.randn((cout, cin, k, k, k), device=dev) * 0.1
    g = torch.randn((1, cout, geom.out(h), geom.out(w), geom.out(d)), device=dev).to(torch.bfloat16).contiguous(
        memory_format=cl)
    dw = torch.zeros_like(wt)
    desc, _ = ops.conv_desc(x.dtype, 1, cin, 0, cout, h, w, d, geom, 0)
    if mode == "fwd":
        def run():
            ops.conv_fwd(x, wt, geom)
    elif mode == "dgrad":
        gx = torch.empty_like(x)
        epi = L.DgradEpilogue()
        ws, wsb = ops._ws(desc, L.PASS_BWD_DATA, dev)

        def run():
            L.call("vq3d_conv3d_bwd_data", ctypes.byref(desc), L.ptr(g), None, L.ptr(wt), None, ctypes.byref(epi),
                   L.ptr(gx), None, None, None, None if ws is None else L.ptr(ws), wsb, L.stream())
    else:
        ws, wsb = ops._ws(desc, L.PASS_BWD_WEIGHT, dev)

        def run():
            L.call("vq3d_conv3d_bwd_weight", ctypes.byref(desc), L.ptr(x), None, L.ptr(g), None, None, L.ptr(wt),
                   None, L.ptr(dw), None, None, None, None if ws is None else L.ptr(ws), wsb, L.stream())
    t = timed(run)
    byt = (x.numel() + g.numel()) * 2
    print(f"{spec:34s} {t * 1e6:9.1f} us  {byt / t / 1e9:7.0f} GB/s", flush=True)


def main():
    dev = torch.device("cuda:0")
    for spec in sys.argv[1:] or DEFAULT:
        one(spec, dev)


if __name__ == "__main__":
    main()
