#!/usr/bin/env python3
"""Host enqueue time of one eager training step of bench.py's workload against its GPU time: the
eager step is GPU-bound while the host issues its ~1,350 launches faster than the GPU runs them.

    python3 tools/host_time.py [--steps 10]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import bench
    import vq3d
    from vq3d.utils import synthetic_volume
    mkw, size, batch, _ = bench.CONFIGS["3l_pub"]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = vq3d.VQVAE(vq3d.default_args(compute_dtype="bf16", base_lr=1e-4, **mkw)).to(dev)
    model.train()
    opt = model.configure_optimizers()
    x = synthetic_volume((1, 1) + tuple(size), 0).to(dev)
    nvs = torch.full((1,), size[2], dtype=torch.int64, device=dev)

    def step():
        opt.zero_grad()
        loss = model.training_step((x, nvs), 0)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    host = []
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        t = time.perf_counter()
        step()
        host.append(time.perf_counter() - t)
    e1.record()
    torch.cuda.synchronize()
    gpu = e0.elapsed_time(e1) / a.steps
    # the host's own cost of a step, measured with the GPU idle (each step synchronised first)
    idle = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        step()
        idle.append(time.perf_counter() - t)
    torch.cuda.synchronize()
    print(f"eager step: GPU {gpu:.2f} ms/step; host enqueue while streaming {1e3 * sum(host) / len(host):.2f} ms/step; "
          f"host enqueue from an idle queue {1e3 * min(idle):.2f} ms (min) / {1e3 * sum(idle) / len(idle):.2f} ms (mean)")


if __name__ == "__main__":
    main()
