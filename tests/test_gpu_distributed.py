"""World-size-2 runs of the PRODUCT data-parallel path on one GPU: two processes on cuda:0
joined by a gloo group (gloo all-reduces device tensors; RCCL cannot put two ranks on one GPU).

* vq3d.Quantizer's distributed EMA (first-pass mean/std init, counts / dw SUM all-reduce,
  reference layers.py:645-647, 670-676) against the 2-rank golden the reference produced
  (tests/golden/ema_dist2.npz), both standalone and through the fused deferred statistics
  buffer that Encoder2 uses (one all-reduce for all levels).
* the bucketed gradient all-reduce overlapped with backward (vq3d.parallel) on a real VQVAE
  training step: the averaged gradient equals the mean of the two ranks' local gradients.
"""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch

from conftest import GOLDEN, PKG

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, PKG)


def _ema_worker(rank, world, port, out, deferred):
    import torch.distributed as dist
    _init(rank, world, port)
    from vq3d import functional as Fn
    from vq3d import layers as VL
    from vq3d.parallel import sum_allreduce
    dev = torch.device("cuda", 0)
    g = np.load(os.path.join(GOLDEN, "ema_dist2.npz"))
    q = VL.Quantizer(64, 4, commitment_cost=0.1).to(dev)
    with torch.no_grad():
        q.embed.copy_(torch.from_numpy(g[f"rank{rank}/embed0"]))
        q.embed_avg.copy_(torch.from_numpy(g[f"rank{rank}/embed0"]))
        q.cluster_size.zero_()
        q.first_pass.fill_(1)
    q.first_pass_host = True
    q.train()
    res = {}
    for step in range(2):
        x = torch.from_numpy(g[f"rank{rank}/step{step}/x"]).to(dev).contiguous(memory_format=torch.channels_last_3d)
        if deferred:  # the Encoder2 path: statistics into a fused slot, one all-reduce, then update
            stats = torch.empty(64 * 5, dtype=torch.float32, device=dev)
            q.ema_slot = stats
            loss, zst, idx = q(x)
            q.ema_slot = None
            sum_allreduce(stats)
            Fn.ema_update(q, stats)
        else:
            loss, zst, idx = q(x)
        torch.cuda.synchronize()
        res[f"step{step}/idx_eq"] = bool(np.array_equal(idx.cpu().numpy(), g[f"rank{rank}/step{step}/idx"]))
        for b in ("embed", "embed_avg", "cluster_size"):
            ref = g[f"rank{rank}/step{step}/{b}"]
            res[f"step{step}/{b}_err"] = float(np.abs(getattr(q, b).cpu().numpy() - ref).max() / (np.abs(ref).max() + 1e-12))
        res[f"step{step}/loss_err"] = abs(float(loss) - float(g[f"rank{rank}/step{step}/loss"]))
    torch.save(res, out + f".{rank}")
    dist.destroy_process_group()


@pytest.mark.parametrize("deferred", [False, True])
def test_quantizer_distributed_ema_two_ranks(deferred):
    import torch.multiprocessing as mp
    out = tempfile.mktemp()
    mp.spawn(_ema_worker, args=(2, _port(), out, deferred), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(out + f".{r}")
        for k, v in res.items():
            if k.endswith("idx_eq"):
                assert v, (r, k)
            else:  # EMA buffers: the reference sums dw in BLAS order (tolerance)
                assert v < 2e-5, (r, k, v)


def _ddp_worker(rank, world, port, out):
    import torch.distributed as dist
    _init(rank, world, port)
    import vq3d
    from vq3d import parallel
    from vq3d.utils import synthetic_volume
    dev = torch.device("cuda", 0)
    kw = dict(n_bottleneck_blocks=2, n_pre_quantization_blocks=1, n_post_quantization_blocks=1, compute_dtype="bf16")
    torch.manual_seed(0)
    a = vq3d.VQVAE(vq3d.default_args(**kw)).to(dev)   # bucketed all-reduce, overlapped
    torch.manual_seed(0)
    b = vq3d.VQVAE(vq3d.default_args(**kw)).to(dev)   # local gradient only
    for m in (a, b):
        m.train()
        with torch.no_grad():  # exercise conv3 / scale paths (zero-initialised by Fixup)
            gen = torch.Generator().manual_seed(1)
            m.flat.data.add_((torch.randn(m.flat.numel, generator=gen) * 0.02).to(dev))
    ar = parallel.GradientAllReduce(a, bucket_bytes=64 << 10)
    x = synthetic_volume((1, 1, 32, 32, 32), rank).to(dev)
    nvs = torch.tensor([32], device=dev)
    b.zero_grad()
    b.training_step((x, nvs), 0).backward()
    vq3d.ops.join_side()
    local = b.flat.grad.clone()
    allg = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(allg, local)
    expect = sum(allg) / world
    a.zero_grad()
    a.training_step((x, nvs), 0).backward()
    issued_during_backward = sum(ar.issued)
    ar()
    torch.cuda.synchronize()
    err = float((a.flat.grad - expect).abs().max() / expect.abs().max())
    other = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(other, a.flat.grad)
    same = bool(torch.equal(other[0], other[1]))
    ar.close()
    torch.save({"err": err, "same": same, "issued": issued_during_backward, "nb": len(ar.buckets)}, out + f".{rank}")
    dist.destroy_process_group()


def test_bucketed_gradient_allreduce_two_ranks():
    import torch.multiprocessing as mp
    out = tempfile.mktemp()
    mp.spawn(_ddp_worker, args=(2, _port(), out), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(out + f".{r}")
        assert res["same"], res                      # replicas hold identical averaged gradients
        assert res["err"] < 1e-5, res                # = mean of the local gradients (fp32 atomics order)
        assert res["nb"] >= 3 and res["issued"] >= 2, res  # buckets went out while backward ran
