"""CPU: the torch.library operators (vq3d/library.py) are traceable -- every vq3d::* operator has a
fake (meta) implementation, the inference forms propagate shapes / dtypes / channels-last strides
under FakeTensorMode without touching a GPU, and torch.export captures a PreActFixupResBlock
operator (the kernels never run here; tests/test_gpu_library.py replays the exported program)."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import vq3d.library as Lb
from vq3d import layers as VL

CL = torch.channels_last_3d


def test_every_operator_has_a_fake():
    from torch._library.simple_registry import singleton
    for name in Lb.OPS:
        entry = singleton.find(f"vq3d::{name}")
        assert entry.fake_impl.kernel is not None, name


def _params(blk):
    return list(blk._fn_params)


@pytest.mark.parametrize("cin,cout,mode,shape,out", [
    (18, 18, "same", (1, 18, 16, 16, 32), (1, 18, 16, 16, 32)),
    (4, 8, "down", (2, 4, 32, 32, 16), (2, 8, 16, 16, 8)),
    (8, 4, "up", (1, 8, 8, 8, 8), (1, 4, 16, 16, 16)),
])
def test_fake_shapes(cin, cout, mode, shape, out):
    torch.manual_seed(0)
    blk = VL.PreActFixupResBlock(cin, cout, mode=mode)
    with FakeTensorMode(allow_non_fake_inputs=True):
        x = torch.empty(shape, dtype=torch.bfloat16, device="cuda").contiguous(memory_format=CL)
        ps = [torch.empty_like(p, device="cuda") for p in _params(blk)]
        y, meta = torch.ops.vq3d.preact_block(x, ps, mode, False)
        assert tuple(y.shape) == out and y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=CL)
        assert meta.dtype == torch.int64
        with pytest.raises(NotImplementedError):
            torch.ops.vq3d.preact_block(x, ps, mode, True)
        r, _ = torch.ops.vq3d.preact_run(x, ps, "small", True, False)
        assert r.dtype == torch.float32 and r.shape == x.shape
        u = torch.ops.vq3d.upsample2x(x)
        assert tuple(u.shape[2:]) == tuple(2 * n for n in shape[2:])
        z = torch.empty((1, 8, 4, 4, 2), device="cuda").contiguous(memory_format=CL)
        loss, zst, idx = torch.ops.vq3d.vq_nearest(z, torch.empty((16, 8), device="cuda"), 0.1, torch.bfloat16)
        assert loss.shape == () and zst.dtype == torch.bfloat16 and tuple(idx.shape) == (1, 4, 4, 2)
        y2, _ = torch.ops.vq3d.conv3d(x, None, None, torch.empty((5, cin, 4, 4, 4), device="cuda"), None, None, None,
                                      [], [4, 2, 1, 1], False, False, False)
        assert tuple(y2.shape) == (shape[0], 5) + tuple(n // 2 for n in shape[2:])


def test_export_captures_a_block_operator():
    class Block(torch.nn.Module):
        def __init__(self, blk):
            super().__init__()
            self.blk = blk

        def forward(self, x):
            return torch.ops.vq3d.preact_block(x, list(self.blk._fn_params), self.blk.mode, False)[0]

    torch.manual_seed(0)
    m = Block(VL.PreActFixupResBlock(18, 18, mode="same")).eval()
    x = torch.randn(1, 18, 16, 16, 32).to(torch.bfloat16).contiguous(memory_format=CL)
    with torch.no_grad():
        ep = torch.export.export(m, (x,))
    calls = [n for n in ep.graph.nodes if n.op == "call_function" and "vq3d" in str(n.target)]
    assert len(calls) == 1 and "preact_block" in str(calls[0].target)
