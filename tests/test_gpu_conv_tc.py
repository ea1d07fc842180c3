"""GPU: the tiny-channel 3x3x3 engine (csrc/conv_tc.hip: 1 / 2 / 4 channels, VALU over a staged
halo) against a float64 torch CPU restatement of nn.Conv3d (+ F.pad 'circular') with the fused
prologue / epilogue: forward, backward-data (with the activation-derivative epilogue and the
prologue-scalar sums) and the weight / scale / bias gradients.  Tolerances: fp32 1e-4, bf16
1.5e-2 of each tensor's max magnitude (bf16: inputs rounded the same way on both sides)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last_3d

CASES = [
    # (cin, cout, (h, w, d), circular)
    (2, 2, (16, 8, 32), True),
    (2, 1, (8, 16, 64), True),
    (1, 1, (8, 8, 32), True),
    (1, 4, (8, 8, 32), True),
    (1, 2, (16, 16, 32), False),
    (2, 1, (8, 8, 64), False),
]


def _conv(u, w, circ):
    if circ:
        return F.conv3d(F.pad(u, (1,) * 6, mode="circular"), w)
    return F.conv3d(u, w, padding=1)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("case", CASES)
def test_tiny_channel_conv_vs_torch(gpu, case, dt):
    from vq3d import ops
    cin, cout, (h, w, d), circ = case
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    tol = 1e-4 if dt == "fp32" else 1.5e-2
    g = torch.Generator().manual_seed(cin * 10 + cout + h)

    def rnd(*shape, scale=1.0):
        return (torch.randn(shape, generator=g) * scale).to(tdt).double()

    def dev(t):
        return t.to(gpu).to(tdt).contiguous(memory_format=CL)

    geom = ops.ConvGeom(3, 1, 1, circ)
    x = rnd(1, cin, h, w, d)
    res = rnd(1, cout, h, w, d)
    wt = (torch.randn((cout, cin, 3, 3, 3), generator=g) * 0.3).double()
    a, b = torch.tensor([0.15], dtype=torch.float64), torch.tensor([-0.2], dtype=torch.float64)
    sc = torch.tensor([0.7], dtype=torch.float64)
    af, bf, scf = a.float().to(gpu), b.float().to(gpu), sc.float().to(gpu)
    wf = wt.float().to(gpu)

    # forward: y = elu(scale * conv(elu(x + a) + b) + b + res) + a    (bias b, act (b, a))
    ref = F.elu(sc * _conv(F.elu(x + a) + b, wt, circ) + b + res + b) + a
    y = ops.conv_fwd(dev(x), wf, geom, pro=(af, bf), scale=scf, bias=bf, residual=dev(res), act=(bf, af))
    assert rel(y.float(), ref) < tol, ("fwd", rel(y.float(), ref))

    # backward-data with the derivative of the prologue, an addend and the scalar sums
    gy = rnd(1, cout, h, w, d)
    add = rnd(1, cin, h, w, d)
    u = torch.zeros_like(x, requires_grad=True)
    _conv(u, wt, circ).backward(gy)
    pre_t = u.grad * sc
    post_t = pre_t * torch.where(x + a > 0, torch.ones_like(x), torch.exp(x + a))
    gx_ref = post_t + add
    dpre = torch.zeros(1, device=gpu)
    dpost = torch.zeros(1, device=gpu)
    gx, _ = ops.conv_bwd(dev(gy), dev(x), wf, geom, pro=(af, bf), gscale=scf, aux=dev(x), addend=dev(add),
                         dpro_pre=dpre, dpro_post=dpost)
    assert rel(gx.float(), gx_ref) < tol, ("dgrad", rel(gx.float(), gx_ref))
    scale = float(pre_t.abs().sum())
    assert abs(float(dpre) - float(pre_t.sum())) <= tol * scale
    assert abs(float(dpost) - float(post_t.sum())) <= tol * scale

    # weight gradient (+ escale, dscale, scalar-bias and conv-bias gradients)
    wv = wt.clone().requires_grad_(True)
    _conv(F.elu(x + a) + b, wv, circ).backward(gy)
    gw = wv.grad
    dw = torch.zeros_like(wf)
    dscale = torch.zeros(1, device=gpu)
    dbias = torch.zeros(1, device=gpu)
    dcb = torch.zeros(cout, device=gpu)
    ops.conv_bwd(dev(gy), dev(x), wf, geom, pro=(af, bf), want_gx=False, dw=dw, dscale=dscale, dbias=dbias,
                 dcbias=dcb, escale=scf)
    assert rel(dw, gw * sc) < tol, ("dw", rel(dw, gw * sc))
    assert abs(float(dscale) - float((wt * gw).sum())) <= tol * float((wt * gw).abs().sum()) + 1e-4
    assert rel(dcb, gy.sum(dim=(0, 2, 3, 4))) < tol
    assert abs(float(dbias) - float(gy.sum())) <= tol * float(gy.abs().sum())
