#!/usr/bin/env python3
"""Training-step health check of the bench workload: loss, gradient and parameter finiteness per
step, eager then HIP-graph replay; on the first non-finite value the forward activations of every
top-level module are checked to name where it starts.

    python3 tools/nan_hunt.py [config] [--eager N] [--replay N]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

WATCH = os.environ.get("NAN_WATCH", "decoder.up.0")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("config", nargs="?", default="3l_pub")
    p.add_argument("--eager", type=int, default=6)
    p.add_argument("--replay", type=int, default=20)
    a = p.parse_args()
    import vq3d
    from vq3d import parallel
    from vq3d.utils import synthetic_volume
    mkw, size, batch = bench.CONFIGS[a.config][:3]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = vq3d.VQVAE(vq3d.default_args(compute_dtype="bf16", base_lr=1e-4, **mkw)).to(dev)
    model.train()
    opt = model.configure_optimizers()
    allreduce = parallel.GradientAllReduce(model)
    x = torch.cat([synthetic_volume((1, 1) + size, i) for i in range(batch)]).to(dev)
    nvs = torch.full((batch,), size[2], dtype=torch.int64, device=dev)
    bad, amax = {}, {}

    def hook(name):
        def f(mod, inp, out):
            if inp and torch.is_tensor(inp[0]) and inp[0].is_floating_point() and not torch.isfinite(inp[0]).all():
                bad.setdefault(name + " <input>", tuple(inp[0].shape))
            outs = out if isinstance(out, (tuple, list)) else (out,)
            for o in outs:
                if torch.is_tensor(o) and o.is_floating_point():
                    if name not in bad and not torch.isfinite(o).all():
                        bad[name] = tuple(o.shape)
                    amax[name] = float(o.detach().float().abs().max())
                    break
        return f
    hooks = [mod.register_forward_hook(hook(name)) for name, mod in model.named_modules()
             if name and (name.count(".") <= 2 or name.startswith(WATCH))]

    def step(i):
        opt.zero_grad()
        loss = model.training_step((x, nvs), i)
        loss.backward()
        allreduce()
        opt.step()
        return loss

    def health(tag, loss):
        torch.cuda.synchronize()
        g = model.flat.grad if hasattr(model.flat, "grad") and model.flat.grad is not None else None
        gf = bool(torch.isfinite(g).all()) if g is not None else None
        pf = bool(torch.isfinite(model.flat.data).all())
        print(f"{tag}: loss {float(loss.detach()):.6f} grads finite {gf} params finite {pf}"
              + (f" first non-finite module outputs {dict(list(bad.items())[:6])}" if bad else ""), flush=True)
        return bool(torch.isfinite(loss)) and pf

    prev = {}
    for i in range(a.eager):
        amax.clear()
        ok = health(f"eager step {i}", step(i))
        if not ok:
            for k, v in amax.items():
                if k.startswith(WATCH):
                    print(f"  {k:40s} max|out| {v:12.4g}  (previous step {prev.get(k, float('nan')):12.4g})")
            return 1
        prev = dict(amax)
    for h in hooks:  # no host syncs inside the capture
        h.remove()
    graph, static = bench.capture(step, a.eager)
    print("captured", flush=True)
    for i in range(a.replay):
        graph.replay()
        if not health(f"replay {i}", static):
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
