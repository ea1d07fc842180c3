#!/usr/bin/env python3
"""Throughput of the 3D VQ-VAE-2 training step (enc + VQ + dec, fwd + bwd + Adam) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3l_pub]

N > 1 runs under torch.distributed.run, one process per GPU (RCCL); each rank trains on its
own synthetic 512x512x128 volume (weak scaling: batch 1 per GPU, BASELINE.json configs[2]).
Rank 0 prints ONE JSON line.  Default workload = the BASELINE metric's configuration:
3-layer VQ-VAE with the reference's published block counts (50 pre-q / 50 post-q / 3 post-up /
2 post-down, K = 128/256/512, slurm-jobs/train_vqvae_3d.job:76-86), bf16 activations.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (model kwargs, volume (H, W, D), batch per GPU)
    "3l_pub": (dict(n_bottleneck_blocks=3, n_pre_quantization_blocks=50, n_post_quantization_blocks=50,
                    n_post_upscale_blocks=3, n_post_downscale_blocks=2, num_embeddings=[128, 256, 512]),
               (512, 512, 128), 1),
    "3l_dflt": (dict(n_bottleneck_blocks=3, num_embeddings=[256]), (512, 512, 128), 1),
    "2l_pub": (dict(n_bottleneck_blocks=2, n_pre_quantization_blocks=150, n_post_quantization_blocks=150,
                    n_post_upscale_blocks=5, n_post_downscale_blocks=5, num_embeddings=[128, 256]),
               (256, 256, 128), 2),
    "2l_dflt": (dict(n_bottleneck_blocks=2, num_embeddings=[256]), (256, 256, 128), 2),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="3l_pub", choices=sorted(CONFIGS))
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--size", type=int, nargs=3, default=None, help="override the volume H W D")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--profile-steps", action="store_true", help="print per-step times to stderr")
    return p.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    import vq3d
    from vq3d import parallel
    from vq3d.utils import synthetic_volume

    rank, world, local, dev = parallel.init_from_env()
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    mkw, size, batch = CONFIGS[a.config]
    if a.size:
        size = tuple(a.size)
    torch.manual_seed(0)
    args = vq3d.default_args(compute_dtype=a.dtype, base_lr=1e-4 * world, **mkw)
    model = vq3d.VQVAE(args).to(dev)
    model.train()
    opt = model.configure_optimizers()
    allreduce = parallel.GradientAllReduce(model)
    # this rank's synthetic volumes, resident in HBM before timing
    idx = parallel.shard_indices(0, rank, world, batch)
    x = torch.cat([synthetic_volume((1, 1) + size, i) for i in idx]).to(dev)
    nvs = torch.full((batch,), size[2], dtype=torch.int64, device=dev)

    def step(i):
        opt.zero_grad()
        loss = model.training_step((x, nvs), i)
        loss.backward()
        allreduce()
        opt.step()
        return loss

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    per = []
    for i in range(a.steps):
        ts = time.perf_counter()
        loss = step(a.warmup + i)
        if a.profile_steps:
            torch.cuda.synchronize()
            per.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    if a.profile_steps and rank == 0:
        print("per-step s:", [round(v, 4) for v in per], file=sys.stderr)
    final_loss = float(loss)
    vols = world * batch * a.steps
    res = {
        "metric": "volumes/sec (enc+VQ+dec fwd+bwd) at 512x512x128",
        "value": vols / elapsed,
        "unit": "volumes/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1000.0 * elapsed / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": a.dtype,
        "data": "synthetic (torch.rand*4.5-0.5 volumes, reference init weights, seed 0)",
        "config": {"workload": f"vqvae_{a.config}_train_step", "volume": list(size), "batch_per_gpu": batch,
                   "global_batch": batch * world, "parallelism": f"dp{world}", "final_loss": final_loss},
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
