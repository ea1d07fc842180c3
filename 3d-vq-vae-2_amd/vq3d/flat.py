"""One flat fp32 buffer for all parameters and one for their gradients.

Every nn.Parameter becomes a view into `data` and its .grad a view into `grad`, so the
kernels accumulate weight gradients in place, the optimizer is one fused launch and the
data-parallel gradient all-reduce is one (bucketable) RCCL call over contiguous memory.
"""
import torch

from . import ops

ALIGN = 64  # elements: 256-byte aligned views
# bumped whenever a parameter or gradient view is (re)attached, so pointer tables built from the
# views (functional.StackPlan) know when to rebuild without walking every parameter per launch
VERSION = [0]


class FlatParams:
    def __init__(self, params, device):
        self.params = [p for p in params]
        offs, total = [], 0
        for p in self.params:
            offs.append(total)
            total += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.offsets = offs
        self.numel = total
        self.data = torch.zeros(total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(total, dtype=torch.float32, device=device)
        for p, off in zip(self.params, offs):
            if p.dtype != torch.float32:
                raise TypeError("parameters must be fp32 masters")
            v = self.data[off:off + p.numel()].view(p.shape)
            v.copy_(p.data)
            p.data = v
            p.grad = self.grad[off:off + p.numel()].view(p.shape)
        self.device = torch.device(device)
        VERSION[0] += 1

    def owns(self, p):
        return p.data.untyped_storage().data_ptr() == self.data.untyped_storage().data_ptr()

    def zero_grad(self):
        ops.zero_(self.grad)
        base = self.grad.data_ptr()
        for p, off in zip(self.params, self.offsets):  # re-attach any .grad a caller replaced
            g = p.grad
            if g is None or g.data_ptr() != base + 4 * off:
                p.grad = self.grad[off:off + p.numel()].view(p.shape)
                VERSION[0] += 1
