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
    p.add_argument("--serial-wgrad", action="store_true",
                   help="run weight gradients on the main stream (default: side stream, overlapped)")
    p.add_argument("--eager", action="store_true",
                   help="launch every kernel from Python each step instead of replaying a captured HIP graph")
    return p.parse_args()


# ---------------------------------------------------------------------------------------------- roofline
# Dominant kernel of the path = the one with the largest share of the step's kernel time in the
# rocprofv3 kernel trace of this bench (profiles/r01_step_breakdown_v9.txt): the fused forward of
# the 18-channel PreActFixupResBlock at 128x128x32 (preact_mid.hip, 50 launches per step, decoder
# bottom level).  Algorithmic bytes per launch = bf16 x (18 ch) read + out (18 ch), t2 (9 ch),
# t3 (9 ch) written + the three fp32 weight tensors.
DOM = dict(channels=18, branch=9, grid=(128, 128, 32))
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_dominant.json")
DOM_NAME = "vq3d preact_mid_fwd: fused PreActFixupResBlock 18ch/branch 9 @128x128x32 bf16"


def dominant_setup(dev, seed=7):
    """(launch(), algorithmic bytes, flops) of one dominant-kernel launch on resident inputs."""
    import torch

    from vq3d import layers as VL
    from vq3d import ops
    torch.manual_seed(seed)
    blk = VL.PreActFixupResBlock(DOM["channels"], DOM["channels"], mode="same").to(dev)
    h, w, d = DOM["grid"]
    g = torch.Generator(device=dev).manual_seed(seed)
    x = (torch.randn((1, DOM["channels"], h, w, d), device=dev, generator=g) * 0.5).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last_3d)
    assert ops.preact_mid_supported(x, DOM["branch"])

    def launch():
        return ops.preact_mid_fwd(x, blk)
    nvox = h * w * d
    c, b = DOM["channels"], DOM["branch"]
    wbytes = sum(p.numel() for p in (blk.branch_conv1.weight, blk.branch_conv2.weight, blk.branch_conv3.weight)) * 4
    algo = nvox * (2 * c + 2 * b) * 2 + wbytes
    flops = 2.0 * nvox * (c * b + b * b * 27 + b * c)
    return launch, algo, flops


def dominant_kernel_roofline(dtype, dev, iters=50):
    import torch
    launch, algo, flops = dominant_setup(dev)
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    # the `iters` launches captured in a HIP graph, so the events time back-to-back kernels on
    # the replay stream (no host launch gaps)
    side = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            for _ in range(iters):
                launch()
    graph.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    graph.replay()
    e1.record(st)
    e1.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / iters
    achieved = algo / t / 1e9
    traffic = None
    if os.path.exists(PMC_FILE):
        try:
            pmc = json.load(open(PMC_FILE))
            if pmc.get("kernel") == DOM_NAME:
                traffic = pmc.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": DOM_NAME,
            "avg_launch_us": t * 1e6, "algorithmic_bytes": algo, "tflops": flops / t / 1e12}


def dist_graph_probe(dev, rank, world):
    """Capture + replay one RCCL all-reduce in a HIP graph; True when every rank got the right
    value (agreed through an eager all-reduce of the per-rank verdicts)."""
    import torch
    import torch.distributed as dist
    ok = 1.0
    try:
        t = torch.full((256,), float(rank + 1), device=dev)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                dist.all_reduce(t)
        torch.cuda.synchronize()
        t.fill_(float(rank + 1))
        g.replay()
        torch.cuda.synchronize()
        ok = 1.0 if abs(float(t[0]) - world * (world + 1) / 2) < 1e-3 else 0.0
    except Exception as e:  # capture unsupported: fall back to eager launches
        print(f"[bench] rank {rank}: graph capture of all_reduce failed ({e}); eager", file=sys.stderr)
        ok = 0.0
    v = torch.tensor([ok], device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MIN)
    return float(v) > 0.5


# ---------------------------------------------------------------------------------------------- CPU baseline
def cpu_baseline(mkw, size, sample=(256, 256, 64)):
    """The CPU oracle (oracle/vqvae_cpu.py, fp32 torch-CPU restatement of the reference step)
    timed on this host: one full training step of the same model on a smaller volume with
    `frac` of the voxels, scaled to volumes/s of the full 512x512x128 volume."""
    import torch

    from oracle import vqvae_cpu as O
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    import vq3d
    cfg = O.Config(**{k: v for k, v in mkw.items()})
    torch.manual_seed(0)
    ref = vq3d.VQVAE(vq3d.default_args(**mkw))
    sd = {k: v.detach().clone() for k, v in ref.state_dict().items()}
    x = torch.rand((1, 1) + tuple(sample), generator=torch.Generator().manual_seed(1234)) * 4.5 - 0.5
    st = {}
    O.train_step(cfg, sd, st, x, [sample[2]], 1e-4)  # warm-up (first-pass codebook init)
    t0 = time.perf_counter()
    O.train_step(cfg, sd, st, x, [sample[2]], 1e-4)
    dt = time.perf_counter() - t0
    frac = (sample[0] * sample[1] * sample[2]) / float(size[0] * size[1] * size[2])
    return {"value": frac / dt, "unit": "volumes/s", "cores": threads, "kind": "port",
            "sample": f"one oracle train step (fp32, same model) on a {sample[0]}x{sample[1]}x{sample[2]} "
                      f"volume = {frac:.4g} of the 512x512x128 voxels, {dt:.2f} s, scaled by voxel count"}


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
    from vq3d import ops
    ops.set_concurrent_wgrad(not a.serial_wgrad)
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
    # Capture one whole training step (forward, loss, backward, gradient all-reduce, Adam; ~3.7k
    # kernel launches) as a HIP graph after the eager warm-up (the Quantizer's first-pass init
    # happened there) and replay it per step: no Python / launch overhead on the timed path.
    # Every replay runs the full step on the resident input; Adam's step count lives on the
    # device.  N > 1: the RCCL collectives (EMA statistics in forward, gradient all-reduce) are
    # captured too, after a probe capture of one all-reduce succeeded on every rank; otherwise
    # (or with VQ3D_BENCH_DIST_GRAPH=0) the ranks run eagerly.
    graph = None
    use_graph = not a.eager and a.warmup >= 2
    if use_graph and world > 1:
        use_graph = os.environ.get("VQ3D_BENCH_DIST_GRAPH", "1") != "0" and dist_graph_probe(dev, rank, world)
    if use_graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step(a.warmup)  # allocator warm-up on the capture stream (one more untimed step)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            loss_static = step(a.warmup + 1)
        torch.cuda.synchronize()

        def step(i):  # noqa: F811
            graph.replay()
            return loss_static
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
    final_loss = float(loss.detach())
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
        "launch": "hip_graph" if graph is not None else "eager",
        "config": {"workload": f"vqvae_{a.config}_train_step", "volume": list(size), "batch_per_gpu": batch,
                   "global_batch": batch * world, "parallelism": f"dp{world}", "final_loss": final_loss},
    }
    if rank == 0 and not a.no_roofline:
        res["roofline"] = dominant_kernel_roofline(a.dtype, dev)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(mkw, size)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
