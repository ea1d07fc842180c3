"""Data parallelism: one process per GPU, whole volumes sharded across ranks (the reference's
PL 'ddp' accelerator, vqvae/train.py:26-27), RCCL over xGMI via torch.distributed 'nccl'.

Per step the only data-path exchange is the gradient all-reduce of the flat fp32 gradient
buffer (flat.py); the Quantizer's EMA statistics are all-reduced inside its forward exactly
where the reference does (layers.py:645-647, 670-676).  Replicas start identical (rank 0
broadcasts parameters and buffers once), so no per-step buffer broadcast is needed.
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env (RANK / WORLD_SIZE / ...).
    Returns (rank, world, local_rank, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        be = backend or ("nccl" if device.type == "cuda" else "gloo")
        kw = {"device_id": device} if be == "nccl" else {}
        dist.init_process_group(be, rank=rank, world_size=world, **kw)
    return rank, world, local, device


def shard_indices(step, rank, world, per_rank=1):
    """Volume indices of `rank` at `step` (DistributedSampler-style interleave, no overlap)."""
    base = (step * world + rank) * per_rank
    return list(range(base, base + per_rank))


class GradientAllReduce:
    """Average the model's flat gradient across ranks (one RCCL all-reduce; gloo in CPU tests)."""

    def __init__(self, model, group=None):
        self.flat = model.flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.world > 1:
            self.backend = dist.get_backend(group)
            # identical replicas: parameters and buffers from rank 0 (what DDP does at wrap time)
            dist.broadcast(self.flat.data, 0, group=group)
            for b in model.buffers():
                dist.broadcast(b, 0, group=group)

    def __call__(self):
        if self.world == 1:
            return
        from . import ops
        ops.join_side()
        if self.backend == "nccl":
            dist.all_reduce(self.flat.grad, op=dist.ReduceOp.AVG, group=self.group)
        else:  # gloo (CPU test transport): SUM then divide
            dist.all_reduce(self.flat.grad, group=self.group)
            self.flat.grad.div_(self.world)
