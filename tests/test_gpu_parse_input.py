"""Encoder2.parse_input (vqvae/layers.py:535, Conv3d(1 -> 4, k = 1, bias)) on the bf16 path reads the
fp32 input volume directly (vq3d_parse_input_*; the reference's autocast hands this conv an fp16
copy, a bf16 copy would lose 3 more bits): against a float64 restatement, output rounded once to
bf16 (within 1 bf16 ulp: 2^-8 of the value), weight / bias gradients from bf16 g and the fp32
volume (1e-4 relative: fp32 vs float64 sums over 2^20 voxels), deterministic run to run."""
import pytest
import torch

pytestmark = pytest.mark.gpu
CL = torch.channels_last_3d


@pytest.mark.parametrize("c,shape", [(4, (1, 1, 64, 64, 32)), (2, (2, 1, 32, 32, 16)), (8, (1, 1, 16, 16, 16))])
@pytest.mark.parametrize("half", [torch.bfloat16, torch.float16])
def test_parse_input_matches_float64(gpu, c, shape, half):
    from vq3d import functional as Fn
    from vq3d.flat import FlatParams
    torch.manual_seed(c)
    conv = torch.nn.Conv3d(1, c, kernel_size=1).to(gpu)
    FlatParams(conv.parameters(), gpu)
    gen = torch.Generator().manual_seed(3)
    x = torch.rand(shape, generator=gen) * 4.5 - 0.5
    g = torch.randn(shape[:1] + (c,) + shape[2:], generator=gen).to(half)
    xd = x.to(gpu)
    assert Fn.parse_input_fused(xd, conv, half)
    outs = []
    for _ in range(2):
        conv.weight.grad.zero_()
        conv.bias.grad.zero_()
        y = Fn.ParseInputFn.apply(xd, conv.weight, conv.bias, half)
        assert y.dtype == half and y.is_contiguous(memory_format=CL)
        y.backward(g.to(gpu).contiguous(memory_format=CL))
        torch.cuda.synchronize()
        outs.append((y.float().cpu(), conv.weight.grad.cpu().clone(), conv.bias.grad.cpu().clone()))
    assert all(torch.equal(a, b) for a, b in zip(*outs))  # fixed-order reductions
    y, dw, db = outs[0]
    w = conv.weight.detach().double().cpu().reshape(c)
    b = conv.bias.detach().double().cpu()
    ref = x.double() * w.view(1, c, 1, 1, 1) + b.view(1, c, 1, 1, 1)
    assert float(((y.double() - ref).abs() / ref.abs().clamp_min(1e-3)).max()) <= 2.0 ** -8
    gd = g.double()
    rdw = (gd * x.double()).sum(dim=(0, 2, 3, 4))
    rdb = gd.sum(dim=(0, 2, 3, 4))
    assert float((dw.double().reshape(c) - rdw).abs().max() / rdw.abs().max()) <= 1e-4
    assert float((db.double() - rdb).abs().max() / rdb.abs().max()) <= 1e-4


def test_quantizer_fp32_z_bf16_straight_through(gpu):
    """An fp32 z (the encoder's fp32-stream pre-quantize runs) gives the same codes as the C oracle,
    the straight-through value fl(x + fl(q - x)) (layers.py:720) rounded to bf16 for the bf16
    consumers, and an fp32 gradient back into the run (vq3d_vq_bwd with bf16 g)."""
    import vq3d
    from oracle import vq_oracle
    from vq3d import layers as VL
    q = VL.Quantizer(128, 2, 0.1).to(gpu)
    q.zst_dtype = torch.bfloat16
    q.train()
    gen = torch.Generator().manual_seed(5)
    z = (torch.randn((1, 2, 16, 16, 8), generator=gen)).to(gpu).contiguous(memory_format=CL).requires_grad_(True)
    emb = q.embed.detach().cpu().clone()
    q.first_pass_host = False
    q.first_pass.zero_()
    loss, zst, idx = q(z)
    assert zst.dtype == torch.bfloat16
    flat = z.detach().permute(0, 2, 3, 4, 1).reshape(-1, 2).cpu().numpy()
    ridx, _, _ = vq_oracle.nearest(flat, emb.numpy())
    assert (idx.reshape(-1).cpu().numpy() == ridx).all()
    zf = z.detach().permute(0, 2, 3, 4, 1).reshape(-1, 2).cpu()
    qv = emb[torch.from_numpy(ridx)]
    st = (zf + (qv - zf)).bfloat16()
    assert torch.equal(zst.detach().permute(0, 2, 3, 4, 1).reshape(-1, 2).cpu(), st)
    (zst.float().sum() + loss).backward()
    assert z.grad.dtype == torch.float32 and torch.isfinite(z.grad).all()
    vq3d.ops.join_side()
