#!/usr/bin/env python3
"""Which host calls issue device copies / fills in one eager training step (torch profiler,
CPU op stacks), to account for __amd_rocclr_copyBuffer launches in the kernel trace."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    import vq3d
    cfg = sys.argv[1] if len(sys.argv) > 1 else "2l_dflt"
    mkw, size, batch = bench.CONFIGS[cfg]
    size = (64, 64, 32)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = vq3d.VQVAE(vq3d.default_args(compute_dtype="bf16", **mkw)).to(dev)
    opt = model.configure_optimizers()
    x = (torch.rand((batch, 1) + size) * 4.5 - 0.5).to(dev)
    nvs = torch.full((batch,), size[2], dtype=torch.int64, device=dev)

    def step():
        opt.zero_grad()
        loss = model.training_step((x, nvs), 0)
        loss.backward()
        opt.step()

    step()
    step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
        step()
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        if any(k in ev.name for k in ("copy", "Memcpy", "memcpy", "fill", "zero", "clone", "contiguous")):
            stack = [s for s in (ev.stack or []) if "vq3d" in s or "bench" in s or "model" in s][:3]
            cnt[(ev.name, tuple(stack))] += 1
    for (name, stack), n in cnt.most_common(25):
        print(n, name, " <- ".join(stack))


if __name__ == "__main__":
    main()
