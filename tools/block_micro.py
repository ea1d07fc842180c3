#!/usr/bin/env python3
"""Time one fused PreAct block (forward / backward) on resident bf16 tensors.

    python3 tools/block_micro.py [C BR H W D] [iters]

Prints the per-call forward and backward time (HIP events around a graph replay of `iters`
calls) for the block path the model dispatches (ops.preact_*), plus algorithmic bytes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))

import torch  # noqa: E402

CL = torch.channels_last_3d


def timed(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            for _ in range(iters):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    from vq3d import layers as VL
    from vq3d import ops
    from vq3d.flat import FlatParams
    a = [int(v) for v in sys.argv[1:6]] if len(sys.argv) > 5 else [18, 9, 128, 128, 32]
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
    c, br, h, w, d = a
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    blk = VL.PreActFixupResBlock(c, c, mode="same").to(dev)
    FlatParams(blk.parameters(), dev)
    with torch.no_grad():
        for p in blk.parameters():
            p.normal_(0, 0.2)
    x = (torch.randn((1, c, h, w, d), device=dev) * 0.5).to(torch.bfloat16).contiguous(memory_format=CL)
    g = (torch.randn((1, c, h, w, d), device=dev) * 0.5).to(torch.bfloat16).contiguous(memory_format=CL)
    names = {"dw1": blk.branch_conv1.weight, "dw2": blk.branch_conv2.weight, "dw3": blk.branch_conv3.weight,
             "dbias1a": blk.bias1a, "dbias1b": blk.bias1b, "dbias2a": blk.bias2a, "dbias2b": blk.bias2b,
             "dbias3a": blk.bias3a, "dbias3b": blk.bias3b, "dscale": blk.scale, "dbias4": blk.bias4}
    grads = {n: p.grad for n, p in names.items()}
    if ops.preact_mid_supported(x, br):
        fwd = lambda: ops.preact_mid_fwd(x, blk)  # noqa: E731
        out, t2, t3 = fwd()
        bwd = lambda: ops.preact_mid_bwd(g, x, t2, t3, blk, grads)  # noqa: E731
        kind = "mid"
    elif ops.preact_small_supported(x, br):
        fwd = lambda: ops.preact_small_fwd(x, blk)  # noqa: E731
        out, t2, t3 = fwd()
        bwd = lambda: ops.preact_small_bwd(g, x, t2, t3, blk, grads)  # noqa: E731
        kind = "small"
    else:
        raise SystemExit("no fused block kernel for this shape")
    # calibration: torch copies of the block's input (18.9 MB at 128^2 x 32 x 18) and of a 4x
    # larger buffer
    big = torch.empty(x.numel() * 4, dtype=torch.bfloat16, device=dev)
    big_dst = torch.empty_like(big)
    xc = torch.empty_like(x)
    tc = timed(lambda: xc.copy_(x), iters)
    tcb = timed(lambda: big_dst.copy_(big), iters)
    print(f"copy {x.numel() * 2 / 1e6:.1f} MB: {tc:7.1f} us ({2 * x.numel() * 2 / tc / 1e3:7.1f} GB/s r+w); "
          f"copy {big.numel() * 2 / 1e6:.1f} MB: {tcb:7.1f} us ({2 * big.numel() * 2 / tcb / 1e3:7.1f} GB/s r+w)")
    if kind == "mid":  # per kernel (vq3d_preact_mid_*_stages), preallocated outputs
        bufs = (out, t2, t3)
        gx = torch.empty_like(x)
        ws = ops.workspace(ops.L.query("vq3d_preact_mid_workspace_bytes", 1, h, w, d), dev)
        ops.preact_mid_bwd(g, x, t2, t3, blk, grads, bufs=(gx, ws))
        per = {f"fwd{k}": timed(lambda k=k: ops.preact_mid_fwd(x, blk, stages=k, bufs=bufs), iters) for k in (1, 2)}
        per.update({f"bwd{k}": timed(lambda k=k: ops.preact_mid_bwd(g, x, t2, t3, blk, grads, stages=k,
                                                                      bufs=(gx, ws)), iters) for k in (1, 2, 4, 8, 16)})
        print("per kernel us:", {k: round(v, 1) for k, v in per.items()})
    tf = timed(fwd, iters)
    tb = timed(bwd, iters)
    nv = h * w * d
    fb = nv * (2 * c + 2 * br) * 2
    bb = nv * (3 * c + 2 * br) * 2
    print(f"{kind} C{c} BR{br} {h}x{w}x{d}: fwd {tf:8.1f} us ({fb / tf / 1e3:7.1f} GB/s alg), "
          f"bwd {tb:8.1f} us ({bb / tb / 1e3:7.1f} GB/s alg)")


if __name__ == "__main__":
    main()
