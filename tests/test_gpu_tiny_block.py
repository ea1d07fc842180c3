"""One-workgroup PreActFixupResBlock kernels (csrc/tiny_block.hip) against a torch fp64 CPU
autograd restatement of the block (vqvae/layers.py:176-195) and against the per-conv engine
path of the same block.  Tolerances: fp32 2e-4 relative to each tensor's max magnitude; bf16
3e-2 (inputs / outputs bf16-rounded, internals fp32)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last_3d

# (batch, channels, h, w, d) -- branch = channels // 2 (bottleneck_divisor 2)
SHAPES = [(1, 32, 8, 8, 2), (2, 16, 4, 4, 4), (1, 8, 4, 4, 2), (1, 32, 4, 4, 4), (1, 24, 2, 4, 2)]


def _block(c, seed):
    from vq3d import layers as VL
    torch.manual_seed(seed)
    blk = VL.PreActFixupResBlock(c, c, mode="same")
    with torch.no_grad():
        rng = np.random.default_rng(seed)
        for n, p in blk.named_parameters():
            if p.numel() == 1:
                p.fill_(float(rng.normal(0, 0.3)))
            else:
                p.normal_(0, 0.3)
        blk.scale.fill_(0.8)
    return blk


def _ref(blk, x, gy):
    """fp64 CPU restatement of PreActFixupResBlock.forward, circular 3x3x3 branch conv."""
    P = {n: p.detach().double().cpu().clone().requires_grad_(True) for n, p in blk.named_parameters()}
    x = x.detach().double().cpu().clone().requires_grad_(True)
    h = F.elu(x + P["bias1a"])
    h = F.conv3d(h + P["bias1b"], P["branch_conv1.weight"])
    h = F.elu(h + P["bias2a"])
    h = F.conv3d(F.pad(h + P["bias2b"], (1, 1, 1, 1, 1, 1), mode="circular"), P["branch_conv2.weight"])
    h = F.elu(h + P["bias3a"])
    h = F.conv3d(h + P["bias3b"], P["branch_conv3.weight"])
    out = h * P["scale"] + P["bias4"] + x
    out.backward(gy.detach().double().cpu())
    return out.detach(), x.grad, {n: p.grad for n, p in P.items()}


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-12))


def _run(blk, x, gy, dev, tdt, tiny):
    from vq3d import ops
    from vq3d.flat import FlatParams
    ops.set_tiny_blocks(tiny)
    try:
        m = blk.to(dev)
        for p in m.parameters():
            p.grad = None
        FlatParams(m.parameters(), dev)
        xg = x.to(dev).to(tdt).contiguous(memory_format=CL).requires_grad_(True)
        y = m(xg)
        y.backward(gy.to(dev).to(tdt).contiguous(memory_format=CL))
        torch.cuda.synchronize()
        return y.detach().float().cpu(), xg.grad.float().cpu(), {n: p.grad.cpu().clone()
                                                                  for n, p in m.named_parameters()}
    finally:
        ops.set_tiny_blocks(True)


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("shape", SHAPES)
def test_tiny_block_vs_reference(gpu, shape, dtype):
    from vq3d import ops
    b, c, h, w, d = shape
    assert ops.preact_tiny_supported(shape, c // 2)
    blk = _block(c, seed=c + h)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(shape, generator=g)
    gy = torch.randn(shape, generator=g)
    tdt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    if dtype != "fp32":  # compare against the reference on the same rounded inputs
        x, gy = x.to(tdt).float(), gy.to(tdt).float()
    ry, rgx, rgp = _ref(blk, x, gy)
    y, gx, gp = _run(blk, x, gy, gpu, tdt, tiny=True)
    tol = 2e-4 if dtype == "fp32" else 3e-2
    errs = {"y": rel(y, ry), "gx": rel(gx, rgx)}
    errs.update({"grad/" + n: rel(gp[n], rgp[n]) for n in rgp})
    bad = {k: v for k, v in errs.items() if not v <= tol}
    assert not bad, bad


def test_tiny_block_matches_engine_path(gpu):
    """Same block through the fused kernel and through the per-conv engines (fp32)."""
    shape = (1, 32, 8, 8, 2)
    blk = _block(32, seed=3)
    g = torch.Generator().manual_seed(9)
    x, gy = torch.randn(shape, generator=g), torch.randn(shape, generator=g)
    y0, gx0, gp0 = _run(blk, x, gy, gpu, torch.float32, tiny=False)
    y1, gx1, gp1 = _run(blk, x, gy, gpu, torch.float32, tiny=True)
    assert rel(y1, y0) < 1e-5 and rel(gx1, gx0) < 1e-5
    for n in gp0:
        assert rel(gp1[n], gp0[n]) < 1e-4, n


def test_tiny_block_rejects_out_of_range(gpu):
    from vq3d import ops
    assert not ops.preact_tiny_supported((1, 64, 8, 8, 2), 32)   # channels > 32
    assert not ops.preact_tiny_supported((1, 32, 16, 16, 4), 16)  # > 256 voxels
    assert not ops.preact_tiny_supported((1, 18, 4, 4, 4), 9)     # not a multiple of 4
