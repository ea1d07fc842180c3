#!/usr/bin/env python3
"""Per-call-site GPU time of one training step: every libvq3d C-ABI call is bracketed by
HIP events on the launch stream and the times are aggregated by call signature (entry point +
conv descriptor), so each layer shape's share of the step is visible.

    python3 tools/call_timing.py [config] [--steps N] [--top K]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from vq3d import _lib as L  # noqa: E402


def sig(name, args):
    if name.startswith("vq3d_conv3d"):
        d = args[0]._obj
        pro = "+pro" if d.pro_kind else ""
        return (f"{name[12:]:11s} c{d.cin + d.cin2:>3}->{d.cout:<3} {d.in_h}x{d.in_w}x{d.in_d} "
                f"k{d.kernel}s{d.stride}{'c' if d.pad_mode else 'z'}{pro}")
    if name.startswith("vq3d_upsample"):
        return f"{name[5:]} c{args[2]} {args[3]}x{args[4]}x{args[5]}"
    return name


def main():
    p = argparse.ArgumentParser()
    p.add_argument("config", nargs="?", default="3l_pub")
    p.add_argument("--steps", type=int, default=1)
    p.add_argument("--top", type=int, default=60)
    a = p.parse_args()
    import vq3d
    mkw, size, batch = bench.CONFIGS[a.config][:3]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = vq3d.VQVAE(vq3d.default_args(compute_dtype="bf16", **mkw)).to(dev)
    opt = model.configure_optimizers()
    x = (torch.rand((batch, 1) + size, generator=torch.Generator().manual_seed(1234)) * 4.5 - 0.5).to(dev)
    nvs = torch.full((batch,), size[2], dtype=torch.int64, device=dev)

    def step():
        opt.zero_grad()
        loss = model.training_step((x, nvs), 0)
        loss.backward()
        opt.step()

    step()
    torch.cuda.synchronize()
    rec = []
    orig = L.call

    def timed(name, *args):
        s = torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r = orig(name, *args)
        e1.record(s)
        rec.append((sig(name, args), e0, e1))
        return r

    L.call = timed
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(a.steps):
        step()
    t1.record()
    torch.cuda.synchronize()
    L.call = orig
    total = t0.elapsed_time(t1) / a.steps
    agg = collections.defaultdict(lambda: [0, 0.0])
    for k, e0, e1 in rec:
        agg[k][0] += 1
        agg[k][1] += e0.elapsed_time(e1)
    covered = sum(v[1] for v in agg.values()) / a.steps
    print(f"step {total:.2f} ms, {len(rec) / a.steps:.0f} calls/step, {covered:.2f} ms inside calls")
    byname = collections.defaultdict(float)
    for k, (n, t) in agg.items():
        byname[k.split()[0]] += t / a.steps
    print("by entry: " + ", ".join(f"{k} {v:.1f}" for k, v in sorted(byname.items(), key=lambda kv: -kv[1])))
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / a.steps:9.3f} ms {n // a.steps:5d}x {t / n * 1e3:8.1f} us  {k}")


if __name__ == "__main__":
    main()
