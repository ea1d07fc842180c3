"""The 9 -> 9 3x3x3 circular conv weight gradient routed through the mid block's windowed W2
kernel (csrc/preact_mid.hip mid_w2grad: the up blocks' branch conv2, layers.py:124-132, 164-171)
against a float64 torch restatement of the same conv on the same bf16 inputs.  Tolerance: 1e-3
of the gradient's max magnitude (fp32 accumulation order only); bit-identical run to run."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
CL = torch.channels_last_3d


@pytest.mark.parametrize("shape", [(1, 9, 16, 16, 8), (2, 9, 32, 16, 16), (1, 9, 64, 64, 64), (1, 9, 32, 32, 128)])
def test_windowed_9x9_wgrad_vs_float64(gpu, shape):
    from vq3d import ops
    g_ = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(shape, generator=g_).bfloat16()
    gy = torch.randn(shape, generator=g_).bfloat16()
    w = torch.randn((9, 9, 3, 3, 3), generator=g_) * 0.2
    # reference: d/dW of sum(conv(pad_circ(x), W) * gy) in float64
    wr = w.double().requires_grad_(True)
    y = F.conv3d(F.pad(x.double(), (1,) * 6, mode="circular"), wr)
    (y * gy.double()).sum().backward()
    ref = wr.grad
    geom = ops.ConvGeom(3, 1, 1, True)
    xd, gd, wd = (x.to(gpu).contiguous(memory_format=CL), gy.to(gpu).contiguous(memory_format=CL), w.to(gpu))
    outs = []
    for _ in range(2):
        dw = torch.zeros_like(wd)
        ops.conv_bwd(gd, xd, wd, geom, want_gx=False, dw=dw)
        torch.cuda.synchronize()
        outs.append(dw.double().cpu())
    assert torch.equal(outs[0], outs[1])
    err = float((outs[0] - ref).abs().max()) / float(ref.abs().max())
    assert err <= 1e-3, err
