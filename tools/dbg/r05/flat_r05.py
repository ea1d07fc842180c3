"""One flat fp32 buffer for all parameters and one for their gradients.

Every nn.Parameter becomes a view into `data` and its .grad a view into `grad`, so the
kernels accumulate weight gradients in place, the optimizer is one fused launch and the
data-parallel gradient all-reduce is one (bucketable) RCCL call over contiguous memory.
"""
import weakref

import torch

from . import ops

ALIGN = 64  # elements: 256-byte aligned views
# bumped whenever a parameter or gradient view is (re)attached, so pointer tables built from the
# views (functional.StackPlan) know when to rebuild without walking every parameter per launch
VERSION = [0]
# live FlatParams by the address of their data buffer (flat_of)
_BY_DATA = weakref.WeakValueDictionary()


def flat_of(p):
    """the FlatParams whose data buffer holds parameter p, or None"""
    if not p.is_cuda:
        return None
    return _BY_DATA.get(p.untyped_storage().data_ptr())


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
        self._shadow = {}
        _BY_DATA[self.data.untyped_storage().data_ptr()] = self
        VERSION[0] += 1

    def refresh_shadow(self, dtype):
        """a 16-bit copy of every parameter in one launch (torch's round-to-nearest-even cast, as
        p.to(dtype)): the GEMM operands of a forward / backward read their weights from it instead
        of casting each weight per call.  Call it after the parameters change (once per forward)."""
        sh = self._shadow.get(dtype)
        if sh is None:
            sh = self._shadow[dtype] = torch.empty(self.numel, dtype=dtype, device=self.device)
        sh.copy_(self.data)
        return sh

    def shadow_view(self, p, dtype):
        """p's slice of the 16-bit shadow (refresh_shadow must have run since p last changed)"""
        off = (p.data_ptr() - self.data.data_ptr()) // 4
        return self._shadow[dtype][off:off + p.numel()].view(p.shape)

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
