"""Host cost of an eager (non-graph) training step of bench.py's headline workload.

    python3 tools/eager_profile.py [--config 3l_pub] [--steps 5] [--top 40]

Prints per step: wall time (synchronised), host enqueue time (the Python / launch work, no sync),
the number of libvq3d C-ABI calls, then a cProfile of one step sorted by own time.  The gap
between the eager step and the graph replay is the part of the host cost the GPU does not hide.
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="3l_pub")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--top", type=int, default=40)
    a = p.parse_args()
    import torch

    import bench
    import vq3d
    from vq3d import _lib as L
    from vq3d import parallel
    from vq3d.utils import synthetic_volume
    dev = torch.device("cuda:0")
    mkw, size, batch, _ = bench.CONFIGS[a.config]
    torch.manual_seed(0)
    model = vq3d.VQVAE(vq3d.default_args(compute_dtype="bf16", base_lr=1e-4, **mkw)).to(dev)
    model.train()
    opt = model.configure_optimizers()
    red = parallel.GradientAllReduce(model)
    x = torch.cat([synthetic_volume((1, 1) + size, i) for i in range(batch)]).to(dev)
    nvs = torch.full((batch,), size[2], dtype=torch.int64, device=dev)

    def step():
        opt.zero_grad()
        loss = model.training_step((x, nvs), 0)
        loss.backward()
        red()
        opt.step()
        return loss

    calls = [0]
    orig = L.call

    def counting(name, *args):
        calls[0] += 1
        return orig(name, *args)
    L.call = counting
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    for i in range(a.steps):
        calls[0] = 0
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"step {i}: wall {1e3 * (t2 - t0):.2f} ms, host enqueue {1e3 * (t1 - t0):.2f} ms, "
              f"{calls[0]} C-ABI calls", flush=True)
    # graph replay of the same step for the comparison
    g, _ = bench.capture(lambda i: step(), 0)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g.replay()
    torch.cuda.synchronize()
    print(f"graph replay: {1e3 * (time.perf_counter() - t0) / a.steps:.2f} ms/step", flush=True)
    # the backward's Python runs on the autograd device thread unless multithreading is off: profile
    # one step with it off so every frame is seen
    pr = cProfile.Profile()
    with torch.autograd.set_multithreading_enabled(False):
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"single-threaded autograd: host enqueue {1e3 * (t1 - t0):.2f} ms", flush=True)
        pr.enable()
        step()
        pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr, stream=sys.stdout)
    st.sort_stats("tottime").print_stats(a.top)
    st.sort_stats("cumulative").print_stats(a.top)
    red.close()


if __name__ == "__main__":
    main()
