"""CPU, world_size 2 over gloo: the data-parallel plumbing (vq3d.parallel) and the
distributed codebook EMA semantics (reference layers.py:645-647, 670-676) pinned by the
2-rank golden generated from the reference (tests/golden/ema_dist2.npz)."""
import os
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _ema_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import vqvae_cpu as O
    _init(rank, world, port)
    g = np.load(os.path.join(GOLDEN, "ema_dist2.npz"))
    sd = {"q.embed": torch.from_numpy(g[f"rank{rank}/embed0"].copy()),
          "q.embed_avg": torch.from_numpy(g[f"rank{rank}/embed0"].copy()),
          "q.cluster_size": torch.zeros(64), "q.first_pass": torch.as_tensor(1)}

    def allreduce(t):
        t = t.clone()
        dist.all_reduce(t)
        return t
    ok = True
    for step in range(2):
        x = torch.from_numpy(g[f"rank{rank}/step{step}/x"])
        loss, qst, idx = O.quantize(sd, "q.", x, True, allreduce=allreduce, world=world)
        ok &= np.array_equal(idx.numpy(), g[f"rank{rank}/step{step}/idx"])
        for b in ("embed", "embed_avg", "cluster_size"):
            ok &= np.allclose(sd["q." + b].numpy(), g[f"rank{rank}/step{step}/{b}"], rtol=1e-5, atol=1e-6)
    torch.save(torch.tensor(bool(ok)), out + f".{rank}")
    dist.destroy_process_group()


def test_distributed_ema_matches_reference_two_ranks():
    out = tempfile.mktemp()
    mp.spawn(_ema_worker, args=(2, free_port(), out), nprocs=2, join=True)
    assert all(bool(torch.load(out + f".{r}")) for r in range(2))


class _FakeFlat:
    def __init__(self, n, seed):
        g = torch.Generator().manual_seed(seed)
        self.data = torch.randn(n, generator=g)
        self.grad = torch.randn(n, generator=g)


class _FakeModel:
    def __init__(self, rank):
        self.flat = _FakeFlat(1000, 10 + rank)
        self._buf = torch.full((4,), float(rank))

    def buffers(self):
        return [self._buf]


def _allreduce_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3d-vq-vae-2_amd"))
    from vq3d import parallel
    _init(rank, world, port)
    m = _FakeModel(rank)
    grads = [_FakeFlat(1000, 10 + r).grad for r in range(world)]
    ar = parallel.GradientAllReduce(m)
    ar()
    ok = torch.allclose(m.flat.grad, sum(grads) / world, atol=1e-6)
    ok &= torch.equal(m.flat.data, _FakeFlat(1000, 10).data)  # rank 0's replica everywhere
    ok &= torch.equal(m._buf, torch.zeros(4))
    shards = [parallel.shard_indices(s, rank, world, 2) for s in range(3)]
    torch.save({"ok": torch.tensor(bool(ok)), "shards": shards}, out + f".{rank}")
    dist.destroy_process_group()


def test_gradient_allreduce_and_sharding_two_ranks():
    out = tempfile.mktemp()
    mp.spawn(_allreduce_worker, args=(2, free_port(), out), nprocs=2, join=True)
    res = [torch.load(out + f".{r}", weights_only=False) for r in range(2)]
    assert all(bool(r["ok"]) for r in res)
    seen = [i for r in res for s in r["shards"] for i in s]
    assert len(seen) == len(set(seen)) == 12  # disjoint volumes, every index once
