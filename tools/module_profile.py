#!/usr/bin/env python3
"""Per-module GPU time of one eager training step of bench.py's workload (level streams off, so
the step is one serial stream): HIP events recorded on the current stream by forward pre / post
hooks and full backward pre / post hooks of the model's modules.

    python3 tools/module_profile.py [--config 3l_pub] [--top 60] [--depth 4]

Modules at depth <= --depth below the model (plus every BlockStack, Quantizer and Conv3d) are
timed; nested modules are included in their parents' times.  A fused run (one BlockStack launch
sequence) shows as its BlockStack."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="3l_pub")
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--depth", type=int, default=4)
    a = ap.parse_args()
    import bench
    import vq3d
    from vq3d import ops
    from vq3d.utils import synthetic_volume
    mkw, size, batch, _ = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    ops.set_overlap_levels(False)
    torch.manual_seed(0)
    model = vq3d.VQVAE(vq3d.default_args(compute_dtype="bf16", base_lr=1e-4, **mkw)).to(dev)
    model.train()
    opt = model.configure_optimizers()
    x = torch.cat([synthetic_volume((1, 1) + tuple(size), i) for i in range(batch)]).to(dev)
    nvs = torch.full((batch,), size[2], dtype=torch.int64, device=dev)

    def step():
        opt.zero_grad()
        loss = model.training_step((x, nvs), 0)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    events, handles = [], []
    keep = ("BlockStack", "Quantizer", "Conv3d", "PreActFixupResBlock", "DownBlock", "UpBlock",
            "PreQuantizationConditioning", "Encoder2", "Decoder")

    def rec(name, kind):
        def hook(*_):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            events.append((name, kind, e))
        return hook
    for name, m in model.named_modules():
        depth = name.count(".") + 1 if name else 0
        if not name or type(m).__name__ not in keep or (depth > a.depth and type(m).__name__ not in
                                                          ("BlockStack", "Quantizer", "Conv3d")):
            continue
        handles.append(m.register_forward_pre_hook(rec(name, "f0")))
        handles.append(m.register_forward_hook(rec(name, "f1")))
        handles.append(m.register_full_backward_pre_hook(rec(name, "b0")))
        handles.append(m.register_full_backward_hook(rec(name, "b1")))
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    step()
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record()
    torch.cuda.synchronize()
    for h in handles:
        h.remove()
    total = e0.elapsed_time(e1)
    open_ = {}
    acc = {}
    for name, kind, e in events:
        if kind in ("f0", "b0"):
            open_[(name, kind[0])] = e
        else:
            s = open_.pop((name, kind[0]), None)
            if s is not None:
                t = s.elapsed_time(e)
                d = acc.setdefault(name, [0.0, 0.0])
                d[0 if kind[0] == "f" else 1] += t
    print(f"step {total:.2f} ms (eager, one stream, hooks on)")
    rows = sorted(acc.items(), key=lambda kv: -(kv[1][0] + kv[1][1]))
    print(f"{'module':60s} {'fwd ms':>8s} {'bwd ms':>8s}  class")
    mods = dict(model.named_modules())
    for name, (f, b) in rows[:a.top]:
        m = mods[name]
        extra = ""
        if type(m).__name__ == "PreActFixupResBlock":
            extra = f" {m.in_channels}->{m.out_channels} {m.mode}"
        elif type(m).__name__ == "BlockStack":
            extra = f" x{len(m)}"
        print(f"{name:60s} {f:8.3f} {b:8.3f}  {type(m).__name__}{extra}")


if __name__ == "__main__":
    main()
