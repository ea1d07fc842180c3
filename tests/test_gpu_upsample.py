"""GPU: the trilinear x2 upsample (ResizeConv3D, vqvae/layers.py:591-597) and its adjoint in bf16
(the LDS-tiled forward for 9 channels, the 4-channel adjoint's run forms, the per-voxel kernels
otherwise) against the per-voxel fp32
kernels on the same bf16-representable inputs.  All compute every value with the same fp32
operations in the same order (no FP contraction in upsample.hip; the tiled kernel reads a halo of
clamped copies with the per-voxel kernel's weights), so the bf16 results must equal the fp32
results rounded to bf16 BIT FOR BIT -- forward (with a prologue) and adjoint (with the activation
derivative, the addend and the prologue-scalar partial sums, those within fp32 summation order).  The fp32 per-voxel kernels are pinned by the reference goldens
(tests/test_gpu_parity.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CL = torch.channels_last_3d
SHAPES = [(1, 4, 8, 16, 32), (2, 8, 8, 8, 16), (1, 9, 4, 8, 16), (2, 9, 8, 16, 32), (1, 9, 6, 8, 16),
          (1, 16, 4, 4, 16), (1, 4, 64, 64, 32), (1, 4, 4, 4, 4), (2, 4, 6, 2, 8),
          # grids large enough for the run forms of the 4-channel adjoint (upsample.hip
          # launch_up2_bwd): 2 x 2 source lines (even H, W; >= 4M source voxels), runs of 4 along D
          (1, 4, 256, 256, 64), (1, 4, 130, 128, 64)]


def rnd(shape, dev, g, scale=1.0):
    return (torch.randn(shape, device=dev, generator=g) * scale).to(torch.bfloat16).float()


@pytest.mark.parametrize("shape", SHAPES)
def test_upsample_tiled_bitwise(gpu, shape):
    from vq3d import ops
    g = torch.Generator(device=gpu).manual_seed(sum(shape))
    b, c, h, w, d = shape
    x = rnd(shape, gpu, g).contiguous(memory_format=CL)
    pa, pb = rnd((1,), gpu, g, 0.3), rnd((1,), gpu, g, 0.3)
    y32 = ops.upsample2x(x, pro=(pa, pb))
    y16 = ops.upsample2x(x.bfloat16(), pro=(pa, pb))
    assert torch.equal(y16, y32.bfloat16())
    gy = rnd((b, c, 2 * h, 2 * w, 2 * d), gpu, g).contiguous(memory_format=CL)
    aux = rnd(shape, gpu, g).contiguous(memory_format=CL)
    add = rnd(shape, gpu, g).contiguous(memory_format=CL)
    ab = rnd((1,), gpu, g, 0.3)
    outs = []
    for dt in (torch.float32, torch.bfloat16):
        pre, post = torch.zeros(1, device=gpu), torch.zeros(1, device=gpu)
        gx = ops.upsample2x_bwd(gy.to(dt), shape, aux=aux.to(dt), aux_b=ab, addend=add.to(dt), dpro_pre=pre,
                                dpro_post=post)
        outs.append((gx, pre, post))
    (g32, pre32, post32), (g16, pre16, post16) = outs
    assert torch.equal(g16, g32.bfloat16())
    scale = float(gy.abs().sum())
    assert abs(float(pre16) - float(pre32)) <= 1e-5 * scale + 1e-4
    assert abs(float(post16) - float(post32)) <= 1e-5 * scale + 1e-4
