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


class _FakeQuantizer(torch.nn.Module):
    """Carries the first_pass buffer + host mirror (vq3d.layers.Quantizer) whose agreement
    across ranks GradientAllReduce must establish."""

    def __init__(self, rank):
        super().__init__()
        self.register_buffer("first_pass", torch.as_tensor(1 - rank))
        self.first_pass_host = bool(1 - rank)


class _FakeModel(torch.nn.Module):
    """Parameters in one flat buffer (vq3d.flat.FlatParams on the CPU) + a Quantizer-like buffer."""

    def __init__(self, rank):
        super().__init__()
        from vq3d.flat import FlatParams
        g = torch.Generator().manual_seed(10 + rank)
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(n, generator=g)) for n in (300, 1000, 7, 64, 2000)])
        self.q = _FakeQuantizer(rank)
        self.flat = FlatParams(self.ps, "cpu")
        for p in self.ps:
            p.grad.copy_(torch.randn(p.shape, generator=g))


def _allreduce_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3d-vq-vae-2_amd"))
    from vq3d import parallel
    _init(rank, world, port)
    models = [_FakeModel(r) for r in range(world)]
    m = models[rank]
    expect = sum(mm.flat.grad for mm in models) / world
    # 2 KB buckets: several buckets over the 3,371 parameters (+ alignment padding)
    ar = parallel.GradientAllReduce(m, bucket_bytes=2048)
    ok = len(ar.buckets) >= 3
    # buckets tile the flat buffer, highest offsets first
    ok &= ar.buckets[0][1] == m.flat.numel and ar.buckets[-1][0] == 0
    ok &= all(a[0] == b[1] for a, b in zip(ar.buckets, ar.buckets[1:]))
    # backward reports parameters in reverse order: buckets go out as they complete
    ps = list(m.ps)
    parallel.grads_ready(ps[4:])
    ok &= ar.issued[0] and not all(ar.issued)
    parallel.grads_ready(ps[:4])
    ok &= all(ar.issued)
    ar()
    ok &= torch.allclose(m.flat.grad, expect, atol=1e-6)
    ok &= torch.equal(m.flat.data, models[0].flat.data)  # rank 0's replica everywhere
    ok &= int(m.q.first_pass) == 1 and m.q.first_pass_host  # buffer and host mirror follow rank 0
    # a second step: the bucket state was reset; unreported buckets are issued by __call__
    for p in m.ps:
        p.grad.fill_(float(rank + 1))
    parallel.grads_ready(ps[4:])
    ar()
    ok &= torch.allclose(m.flat.grad[m.flat.offsets[0]:m.flat.offsets[0] + 300], torch.full((300,), 1.5))
    # an abandoned step (backward reported everything, the reducer was never called): the next
    # forward's step_begin drains it, so the new step's buckets are all issued and averaged
    parallel.grads_ready(ps)
    ok &= all(ar.issued)
    parallel.step_begin()
    ok &= not any(ar.issued) and not ar.works
    for p in m.ps:
        p.grad.fill_(float(2 * rank + 1))
    parallel.grads_ready(ps[4:])
    ar()
    ok &= all(torch.allclose(p.grad, torch.full_like(p.grad, 2.0)) for p in m.ps)  # (1 + 3) / 2
    # a backward that died after reporting PART of a multi-parameter bucket (nothing issued): the
    # next forward's step_begin must refill every pending set, or that bucket would be issued
    # before the parameters already struck off have this step's gradients
    bi = next(i for i, (_, _, ids) in enumerate(ar.buckets) if len(ids) > 1)
    p0 = next(p for p in ps if id(p) == ar.buckets[bi][2][0])
    parallel.grads_ready([p0])
    ok &= not any(ar.issued) and len(ar.pending[bi]) == len(ar.buckets[bi][2]) - 1
    parallel.step_begin()
    ok &= all(len(s) == len(ids) for s, (_, _, ids) in zip(ar.pending, ar.buckets))
    ar()  # the reducer issues every bucket of the (fresh) step
    # a replacement reducer (e.g. after a resume) closes the old one: only the new one reports
    ar2 = parallel.GradientAllReduce(m, bucket_bytes=2048)
    ok &= parallel._active[0] is ar2
    ar2.close()
    ar.close()
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


def _order_worker(rank, world, port, out):
    """Backward reports parameters in a rank-dependent order (the decoder's level chains run on
    their own streams, so which bucket completes first can differ between ranks); the reducer must
    still issue its collectives in bucket order on every rank -- gloo would otherwise pair
    different buckets (different sizes) across the ranks."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3d-vq-vae-2_amd"))
    from vq3d import parallel
    _init(rank, world, port)
    models = [_FakeModel(r) for r in range(world)]
    m = models[rank]
    expect = sum(mm.flat.grad for mm in models) / world
    ar = parallel.GradientAllReduce(m, bucket_bytes=2048)
    log = []
    issue = ar._issue

    def logged(bi):
        log.append(bi)
        issue(bi)
    ar._issue = logged
    ps = list(m.ps)
    order = ps if rank == 1 else ps[::-1]  # rank 1: the LAST bucket's parameters first
    for i, p in enumerate(order):
        parallel.grads_ready([p])
        if rank == 1 and i < len(order) - 1:
            ok_early = not ar.issued[0]  # bucket 0 (highest offsets) not complete yet: nothing issued
            if not ok_early:
                break
    ar()
    ok = log == sorted(log) and len(log) == len(ar.buckets)
    ok &= torch.allclose(m.flat.grad, expect, atol=1e-6)
    ar.close()
    torch.save({"ok": torch.tensor(bool(ok)), "log": log}, out + f".{rank}")
    dist.destroy_process_group()


def test_gradient_allreduce_issues_buckets_in_order_two_ranks():
    out = tempfile.mktemp()
    mp.spawn(_order_worker, args=(2, free_port(), out), nprocs=2, join=True)
    res = [torch.load(out + f".{r}", weights_only=False) for r in range(2)]
    assert all(bool(r["ok"]) for r in res), [r["log"] for r in res]
    assert res[0]["log"] == res[1]["log"]
