#!/usr/bin/env python3
"""Loss of the first N eager training steps of a model config at a volume size (diagnostics):
    python3 tools/loss_steps.py H W D [N] [--cfg 3l_pub|2l] [--lr 1e-4]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))

import torch  # noqa: E402

import vq3d  # noqa: E402
from vq3d import ops  # noqa: E402

CFG = {"3l_pub": dict(n_bottleneck_blocks=3, n_pre_quantization_blocks=50, n_post_quantization_blocks=50,
                      n_post_upscale_blocks=3, n_post_downscale_blocks=2, num_embeddings=[128, 256, 512]),
       "2l": dict(n_bottleneck_blocks=2, n_pre_quantization_blocks=2, n_post_quantization_blocks=2,
                  n_post_upscale_blocks=2, n_post_downscale_blocks=2, num_embeddings=[128, 256])}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("size", type=int, nargs=3)
    p.add_argument("n", type=int, nargs="?", default=4)
    p.add_argument("--cfg", default="3l_pub")
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--perturb", type=float, default=0.0)
    a = p.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = vq3d.VQVAE(vq3d.default_args(base_lr=a.lr, **CFG[a.cfg]))
    if a.perturb:
        g = torch.Generator().manual_seed(1)
        with torch.no_grad():
            for _, q in sorted(m.named_parameters()):
                q.add_(a.perturb * torch.randn(q.shape, generator=g))
    m = m.to(dev)
    m.train()
    opt = m.configure_optimizers()
    size = tuple(a.size)
    x = (torch.rand((1, 1) + size, generator=torch.Generator().manual_seed(2)) * 4.5 - 0.5).to(dev)
    for i in range(a.n):
        opt.zero_grad()
        loss = m.training_step((x, torch.tensor([size[2]])), i)
        loss.backward()
        ops.join_side()
        opt.step()
        torch.cuda.synchronize()
        gn = float(torch.sqrt(sum((q.grad.double() ** 2).sum() for q in m.parameters() if q.grad is not None)))
        print(f"{a.cfg} {size} step {i}: loss {float(loss.detach()):.6f} grad-norm {gn:.4e}", flush=True)


if __name__ == "__main__":
    main()
