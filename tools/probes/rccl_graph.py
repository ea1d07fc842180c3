"""Probe: can an RCCL all-reduce be captured in a HIP graph and replayed (world size from env)?"""
import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    t = torch.full((1024,), float(rank + 1), device=dev)
    dist.all_reduce(t)  # warm-up (communicator init) outside capture
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            t.mul_(0.5)
            dist.all_reduce(t)
    torch.cuda.synchronize()
    t.fill_(float(rank + 1))
    g.replay()
    torch.cuda.synchronize()
    exp = 0.5 * sum(range(1, world + 1))
    print("rank", rank, "value", float(t[0]), "expected", exp, "ok", abs(float(t[0]) - exp) < 1e-6, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
