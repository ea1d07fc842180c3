"""Replaying a whole training step as a HIP graph.

A step of the published model is ~1,300 kernel launches; issued from Python each step they cost
the host more than the GPU needs for the short ones (the tiny-grid levels).  StepGraph captures
the step once per input shape -- forward, loss, backward, the gradient all-reduce and Adam --
and replays it: inputs are copied into static device buffers, every launch inside reads fixed
addresses (the caching allocator's graph pool), and nothing in the step reads a host value that
changes between steps (Adam's step count lives on the device, the Quantizers' first-pass
flag is consumed by the eager warm-up steps).  bench.py and vq3d.train both use it.
"""
import torch


class StepGraph:
    """step_fn(*inputs) -> loss (a device scalar), captured per input signature after `warmup`
    eager calls of that signature.  enabled=False: always eager."""

    def __init__(self, step_fn, warmup=2, enabled=True):
        self.step_fn = step_fn
        self.warmup = max(1, int(warmup))
        self.enabled = enabled
        self.seen = {}
        self.graphs = {}

    @staticmethod
    def _key(inputs):
        return tuple((tuple(t.shape), t.dtype, t.device) for t in inputs)

    def __call__(self, *inputs):
        if not self.enabled:
            return self.step_fn(*inputs)
        key = self._key(inputs)
        ent = self.graphs.get(key)
        if ent is not None:
            graph, static, loss = ent
            for s, t in zip(static, inputs):
                s.copy_(t, non_blocking=True)
            graph.replay()
            return loss
        n = self.seen.get(key, 0)
        self.seen[key] = n + 1
        if n < self.warmup:
            return self.step_fn(*inputs)
        return self._capture(key, inputs)

    def _capture(self, key, inputs):
        # no extra warm-up step here (it would be one more optimizer update on this batch): the
        # eager steps of this signature have initialised every lazy state the step touches
        static = [t.clone() for t in inputs]
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        # thread_local: a DataLoader's pin-memory thread (and its worker hand-offs) may keep
        # calling into HIP while the training thread captures; the default global mode would make
        # those calls invalidate the capture
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            loss = self.step_fn(*static)
        self.graphs[key] = (graph, static, loss)
        # the capture ran nothing: replay once so this call's step happens
        for s, t in zip(static, inputs):
            s.copy_(t, non_blocking=True)
        graph.replay()
        return loss
