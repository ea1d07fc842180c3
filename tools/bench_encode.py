#!/usr/bin/env python3
"""Encode-only code extraction throughput (BASELINE.json configs[3]; extract_embeddings.py:16-23):
3-layer published model in eval mode, encoder + codebook search per 512x512x128 volume, bf16.

    python tools/bench_encode.py [--gpus N] [--steps K] [--warmup W]

One JSON line.  `value` = volumes/s with the volume resident in HBM (the encode captured as a
HIP graph and replayed); `extract_with_d2h` adds the copy of the three code arrays to pinned
host memory (what the reference pickles into LMDB).  N > 1 runs one independent replica per
GPU under torch.distributed.run (no collective on the data path: extraction is embarrassingly
parallel); the timing is the max over ranks.  `roofline` prices the whole
encoder forward against HBM: 3.39 GB of bf16 conv traffic per volume (per-layer
input + output + weights), i.e. 2,362 volumes/s at 8 TB/s.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

ENC_BYTES = 3.39e9  # cfg4 encoder-only fwd, 3L pub, bf16 per-layer bytes
HBM_PEAK_GBS = 8000.0


def cpu_baseline(mkw, threads=16, sample=(256, 256, 64)):
    """The oracle's eval-mode encode (fp32 torch-CPU) on a 1/8-voxel sample, scaled by voxels."""
    import torch

    import vq3d
    from oracle import vqvae_cpu as O
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    m = vq3d.VQVAE(vq3d.default_args(compute_dtype="fp32", **mkw))
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    for k in [k for k in sd if k.endswith("first_pass")]:
        sd[k].zero_()
    cfg = O.Config(**{k: v for k, v in mkw.items()})
    x = torch.rand((1, 1) + sample, generator=torch.Generator().manual_seed(1234)) * 4.5 - 0.5
    with torch.no_grad():
        t = time.perf_counter()
        O.encode(cfg, sd, x, train=False)
        dt = time.perf_counter() - t
    frac = sample[0] * sample[1] * sample[2] / (512 * 512 * 128)
    return {"value": frac / dt, "unit": "volumes/s", "cores": threads, "kind": "port",
            "sample": f"one oracle eval encode (fp32) of a {sample[0]}x{sample[1]}x{sample[2]} volume = "
                      f"{frac:.4g} of the voxels, {dt:.2f} s, scaled by voxel count"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="3l_pub", choices=sorted(bench.CONFIGS))
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    a = p.parse_args()
    import torch
    import torch.distributed as dist

    import vq3d
    from vq3d import parallel
    from vq3d.extract import extract_samples
    from vq3d.utils import synthetic_volume

    rank, world, local, dev = parallel.init_from_env()
    mkw, size, _ = bench.CONFIGS[a.config][:3]
    torch.manual_seed(0)
    model = vq3d.VQVAE(vq3d.default_args(compute_dtype=a.dtype, **mkw)).to(dev)
    for q in (m for m in model.modules() if isinstance(m, vq3d.Quantizer)):
        q.first_pass.zero_()  # a trained checkpoint's codebooks: no first-pass init in eval anyway
        q.first_pass_host = False
    x = synthetic_volume((1, 1) + size, rank).to(dev)
    for _ in range(a.warmup):
        idxs = next(extract_samples(model, [x]))
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        next(extract_samples(model, [x]))
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(graph):
        idxs = next(extract_samples(model, [x]))
    host = [torch.empty(i.shape, dtype=i.dtype, pin_memory=True) for i in idxs]

    def timed(d2h):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            graph.replay()
            if d2h:
                for h, i in zip(host, idxs):
                    h.copy_(i, non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t)
        return el

    graph.replay()
    torch.cuda.synchronize()
    el = timed(False)
    el_d2h = timed(True)
    vols = world * a.steps
    per_vol = el / a.steps
    res = {
        "metric": "volumes/sec (encode+VQ, eval, codes extraction) at 512x512x128",
        "value": vols / el, "unit": "volumes/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": 1000.0 * per_vol, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": a.dtype, "data": "synthetic (torch.rand*4.5-0.5 volume, reference init weights, seed 0)",
        "launch": "hip_graph",
        "config": {"workload": f"vqvae_{a.config}_encode_extract", "volume": list(size), "batch_per_gpu": 1,
                   "parallelism": f"replicas{world}", "code_shapes": [list(i.shape) for i in idxs]},
        "extract_with_d2h": {"value": vols / el_d2h, "unit": "volumes/s",
                             "note": "codes copied to pinned host memory each volume (PCIe-inclusive)"},
        "roofline": {"bound": "hbm", "achieved": ENC_BYTES / per_vol / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ENC_BYTES / per_vol / 1e9 / HBM_PEAK_GBS, "traffic": None,
                     "scope": "whole encoder forward, algorithmic bytes 3.39 GB/volume (SURVEY.md 8(d))"},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(mkw)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
