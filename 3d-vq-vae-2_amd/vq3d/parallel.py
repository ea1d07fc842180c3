"""Data parallelism: one process per GPU, whole volumes sharded across ranks (the reference's
PL 'ddp' accelerator, vqvae/train.py:26-27), RCCL over xGMI via torch.distributed 'nccl'.

Per step the data-path exchanges are:
  * the gradient average of the flat fp32 gradient buffer (flat.py), cut into buckets of
    contiguous parameters in reverse registration order (the order backward finishes them).
    Every autograd Function of the path reports its parameters once their gradient kernels are
    enqueued (`grads_ready`); when a bucket's last parameter is in, its all-reduce is issued
    on a communication stream that waits for the main and the weight-gradient side stream, so
    the RCCL ring runs while backward continues (what PL DDP's bucketing gives the reference,
    train.py:27).  `GradientAllReduce.__call__` issues what is left and joins before Adam.
  * the Quantizers' EMA statistics: ONE fused SUM all-reduce per forward (layers.Encoder2,
    reference layers.py:645-647 does two per level), plus the first-step mean/std (C3).
Replicas start identical (rank 0 broadcasts parameters and buffers once), so the reference's
per-forward buffer broadcast (DDP broadcast_buffers) is not needed.
"""
import os

import torch
import torch.distributed as dist

_active = [None]  # the GradientAllReduce whose buckets the autograd Functions report to


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env (RANK / WORLD_SIZE / ...).
    Returns (rank, world, local_rank, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of N ranks on a one-GPU box: every rank on device 0, collectives over gloo (RCCL
    # refuses two ranks on one device); never set for a real multi-GPU run
    share = os.environ.get("VQ3D_RANKS_SHARE_GPU") == "1"
    if torch.cuda.is_available():
        dev_index = 0 if share else local
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
        if share:
            backend = backend or "gloo"
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


def world_size(group=None):
    return dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1


def sum_allreduce(t, group=None):
    """In-place SUM all-reduce over the data-parallel ranks (no-op at world 1); returns world."""
    w = world_size(group)
    if w > 1:
        dist.all_reduce(t, group=group)
    return w


def grads_ready(params):
    """Called by the autograd Functions once the gradient kernels of `params` are enqueued."""
    r = _active[0]
    if r is not None:
        r.ready(params)


def step_begin():
    """Called at the start of every gradient-recording forward (VQVAE.forward): a reducer whose
    previous backward was not followed by its __call__ (an exception, a skipped step, a second
    backward) drains those collectives and starts the new step from fresh bucket state, so a
    stale `issued` flag can never make this step skip its gradient average."""
    r = _active[0]
    if r is not None:
        r.begin_step()


def graph_collectives_ok(dev, why=None):
    """Capture + replay the step's collective pattern in a HIP graph on every rank -- a bucket
    all-reduce issued asynchronously on a side communication stream and joined back (as
    GradientAllReduce does), plus a plain all-reduce (the fused EMA statistics) -- and report
    whether every rank got the right values (a collective; call on all ranks).  `why`: a list that
    receives this rank's reason (the exception, or the wrong values) when the probe fails."""
    rank, world = dist.get_rank(), dist.get_world_size()
    ok = 1.0
    why = why if why is not None else []
    try:
        t = torch.full((256,), float(rank + 1), device=dev)
        u = torch.full((64,), float(rank + 1), device=dev)
        side, comm = torch.cuda.Stream(), torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                dist.all_reduce(u)
                comm.wait_stream(side)
                with torch.cuda.stream(comm):
                    w = dist.all_reduce(t, op=dist.ReduceOp.AVG, async_op=True)
                w.wait()
                side.wait_stream(comm)
        torch.cuda.synchronize()
        t.fill_(float(rank + 1))
        u.fill_(float(rank + 1))
        g.replay()
        torch.cuda.synchronize()
        ok = 1.0 if (abs(float(t[0]) - (world + 1) / 2) < 1e-3 and abs(float(u[0]) - world * (world + 1) / 2) < 1e-3) \
            else 0.0
        if not ok:
            why.append(f"rank {rank}: replayed collectives gave {float(t[0])} / {float(u[0])}, expected "
                       f"{(world + 1) / 2} / {world * (world + 1) / 2}")
    except Exception as e:  # capture unsupported here: the callers fall back to eager launches
        ok = 0.0
        why.append(f"rank {rank}: {type(e).__name__}: {e}"[:300])
    v = torch.tensor([ok], device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MIN)
    if float(v) <= 0.5 and not why:
        why.append(f"rank {rank}: another rank's probe failed")
    return float(v) > 0.5


class GradientAllReduce:
    """Average the model's flat gradient across ranks in buckets overlapped with backward (one
    RCCL all-reduce per bucket; gloo SUM + divide in CPU tests).

    bucket_bytes: target bucket size.  A bucket is a contiguous slice of the flat gradient (the
    parameters are laid out in registration order, backward finishes them roughly in reverse)."""

    def __init__(self, model, group=None, bucket_bytes=8 << 20, overlap=True):
        self.flat = model.flat
        self.group = group
        self.world = world_size(group)
        self.works = []
        if self.world > 1:
            self.backend = dist.get_backend(group)
            # identical replicas: parameters and buffers from rank 0 (what DDP does at wrap time)
            dist.broadcast(self.flat.data, 0, group=group)
            for b in model.buffers():
                dist.broadcast(b, 0, group=group)
            # host mirrors of broadcast buffers follow rank 0 (Quantizer.first_pass_host gates a
            # collective, so every rank must agree on it)
            for m in model.modules():
                if hasattr(m, "first_pass_host"):
                    m.first_pass_host = bool(int(m.first_pass))
        self._build_buckets(bucket_bytes)
        self.overlap = overlap and self.world > 1
        self._comm = None
        if self.overlap:
            if _active[0] is not None and _active[0] is not self:
                _active[0].close()  # one reducer reports per process: the newest replaces the old
            _active[0] = self
        self._reset()

    def _build_buckets(self, bucket_bytes):
        f = self.flat
        order = sorted(range(len(f.params)), key=lambda i: -f.offsets[i])  # reverse registration
        self.buckets = []  # (lo, hi, [param ids])
        cur, lo, hi = [], None, None
        for i in order:
            p, off = f.params[i], f.offsets[i]
            end = off + p.numel()
            if not cur:
                hi = f.numel if not self.buckets else self.buckets[-1][0]
            cur.append(id(p))
            lo = off
            if (hi - lo) * 4 >= bucket_bytes:
                self.buckets.append((lo, hi, cur))
                cur = []
        if cur:
            self.buckets.append((0, hi, cur))
        elif self.buckets:
            lo0, hi0, ids0 = self.buckets[-1]
            self.buckets[-1] = (0, hi0, ids0)
        self.bucket_of = {pid: bi for bi, (_, _, ids) in enumerate(self.buckets) for pid in ids}

    def begin_step(self):
        # unconditional: a backward that died after reporting part of a bucket leaves that
        # bucket's pending set partly drained, which would issue its all-reduce early next step
        for work, _ in self.works:
            work.wait()
        self._reset()

    def _reset(self):
        self.pending = [set(ids) for _, _, ids in self.buckets]
        self.issued = [False] * len(self.buckets)
        self.next_issue = 0
        self.works = []

    def _stream(self):
        if self._comm is None and self.flat.data.is_cuda:
            self._comm = torch.cuda.Stream(device=self.flat.data.device)
        return self._comm

    def _issue(self, bi):
        lo, hi, _ = self.buckets[bi]
        view = self.flat.grad[lo:hi]
        self.issued[bi] = True
        if not view.is_cuda:
            self.works.append((dist.all_reduce(view, group=self.group, async_op=True), view))
            return
        from . import ops
        comm = self._stream()
        comm.wait_stream(torch.cuda.current_stream())
        for s in ops.side_streams():
            comm.wait_stream(s)
        with torch.cuda.stream(comm):
            op = dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM
            self.works.append((dist.all_reduce(view, op=op, group=self.group, async_op=True), view))

    def ready(self, params):
        """Strike `params` off their buckets' pending sets and issue, IN BUCKET ORDER, every bucket
        that is complete and whose predecessors are issued.  Collectives must be issued in the
        same order on every rank; the order in which backward reports parameters may differ (the
        decoder's level chains run on their own streams), so a bucket that completes early waits
        for the buckets before it."""
        for p in params:
            if p is None:
                continue
            bi = self.bucket_of.get(id(p))
            if bi is None or self.issued[bi]:
                continue
            self.pending[bi].discard(id(p))
        while self.next_issue < len(self.buckets) and not self.pending[self.next_issue]:
            if not self.issued[self.next_issue]:
                self._issue(self.next_issue)
            self.next_issue += 1

    def __call__(self):
        """Issue the buckets still pending, then make the current stream wait for every
        all-reduce (the optimizer follows on it)."""
        if self.world == 1:
            return
        from . import ops
        ops.join_side()
        for bi in range(len(self.buckets)):  # in bucket order, as ready() issues them
            if not self.issued[bi]:
                self._issue(bi)
        for work, view in self.works:
            work.wait()
            if self.backend != "nccl":
                view.div_(self.world)
        if self._comm is not None:
            torch.cuda.current_stream().wait_stream(self._comm)
        self._reset()

    def close(self):
        """Detach from the autograd Functions (drains any issued collectives first)."""
        for work, _ in self.works:
            work.wait()
        self.works = []
        if _active[0] is self:
            _active[0] = None
