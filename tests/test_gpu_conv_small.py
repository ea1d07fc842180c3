"""GPU: the small-grid / many-channel conv engine (csrc/conv_small.hip: reduction channels split
over workgroups, fixed-order partial sums) against a float64 torch CPU restatement of
nn.Conv3d (+ F.pad 'circular') with the fused prologue / epilogue, forward and
backward-data.  Tolerances: fp32 1e-4, bf16 1.5e-2 of the output's max magnitude.  bf16
runs the matrix-core form (k_small_mma) where the channel counts are multiples of 32 / 16."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last_3d

CASES = [
    # (cin, cout, (h, w, d), k, s, p, circular, cin2)
    (128, 128, (8, 8, 2), 3, 1, 1, True, 0),
    (128, 128, (16, 16, 4), 4, 2, 1, True, 0),  # dgrad (grid 1024) runs on the stride-2 engine
    (64, 64, (8, 8, 4), 3, 1, 1, True, 0),
    (36, 36, (8, 4, 4), 3, 1, 1, False, 36),
    (40, 20, (6, 5, 3), 3, 1, 1, True, 0),
    (33, 17, (4, 4, 2), 3, 1, 1, True, 0),
    (128, 64, (4, 4, 2), 2, 2, 0, False, 0),
    (32, 96, (8, 4, 4), 4, 2, 1, False, 0),
    # 16-bit: the matrix-core form (32-channel chunks x tap groups) incl. a dual input split at 64
    (64, 64, (8, 8, 2), 3, 1, 1, True, 64),
    (64, 32, (8, 8, 8), 3, 1, 1, False, 0),
]


def _conv_ref(u, w, k, s, p, circ):
    if circ and p:
        u = F.pad(u, (p,) * 6, mode="circular")
        return F.conv3d(u, w, stride=s)
    return F.conv3d(u, w, stride=s, padding=p)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("case", CASES)
def test_small_grid_conv_vs_torch(gpu, case, dt):
    from vq3d import ops
    from vq3d import _lib as L
    cin, cout, (h, w, d), k, s, p, circ, cin2 = case
    desc, _ = ops.conv_desc(torch.float32, 1, cin, cin2, cout, h, w, d, ops.ConvGeom(k, s, p, circ), 0)
    assert L.query("vq3d_conv3d_workspace_size", ctypes.byref(desc), L.PASS_FWD) > 0, "small-grid engine not selected"
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    tol = 1e-4 if dt == "fp32" else 1.5e-2
    g = torch.Generator().manual_seed(cin * 7 + cout)

    def rnd(*shape, scale=1.0):
        return (torch.randn(shape, generator=g) * scale).to(tdt).double()

    geom = ops.ConvGeom(k, s, p, circ)
    x = rnd(1, cin, h, w, d)
    x2 = rnd(1, cin2, h, w, d) if cin2 else None
    wt = (torch.randn((cout, cin + cin2, k, k, k), generator=g) * 0.2).double()
    a, b = torch.tensor([0.15], dtype=torch.float64), torch.tensor([-0.2], dtype=torch.float64)
    # forward: y = elu(conv(elu(x + a) + b) + b) + a
    xin = torch.cat([x, x2], 1) if cin2 else x
    ref = F.elu(_conv_ref(F.elu(xin + a) + b, wt, k, s, p, circ) + b) + a

    def dev(t):
        return t.to(gpu).to(tdt).contiguous(memory_format=CL)

    af, bf = a.float().to(gpu), b.float().to(gpu)
    wf = wt.float().to(gpu)
    y = ops.conv_fwd(dev(x), wf, geom, pro=(af, bf), x2=dev(x2) if cin2 else None, act=(bf, af))
    assert rel(y.float(), ref) < tol, ("fwd", rel(y.float(), ref))
    if cin2:
        return
    # backward-data: gx = addend + elu'(x + a) * gscale * W^T g ; dpre / dpost sums
    oh, ow, od = geom.out(h), geom.out(w), geom.out(d)
    gy = rnd(1, cout, oh, ow, od)
    add = rnd(1, cin, h, w, d)
    gsc = torch.tensor([0.7], dtype=torch.float64)
    u = torch.zeros_like(x, requires_grad=True)
    _conv_ref(u, wt, k, s, p, circ).backward(gy)
    pre_t = u.grad * gsc
    post_t = pre_t * torch.where(x + a > 0, torch.ones_like(x), torch.exp(x + a))
    gx_ref = post_t + add
    dpre = torch.zeros(1, device=gpu)
    dpost = torch.zeros(1, device=gpu)
    gx, _ = ops.conv_bwd(dev(gy), dev(x), wf, geom, pro=(af, bf), gscale=gsc.float().to(gpu), aux=dev(x),
                         addend=dev(add), dpro_pre=dpre, dpro_post=dpost)
    assert rel(gx.float(), gx_ref) < tol, ("dgrad", rel(gx.float(), gx_ref))
    scale = float(pre_t.abs().sum())
    assert abs(float(dpre) - float(pre_t.sum())) <= tol * scale
    assert abs(float(dpost) - float(post_t.sum())) <= tol * scale


def test_small_grid_misaligned_input_fits_workspace(gpu):
    """A 16-bit input that is not 16-byte aligned makes the matrix-core plan fall back to the VALU
    kernel with its own (larger) split: the queried workspace must cover that split.  The launch
    gets exactly the queried bytes followed by a canary region, which must stay untouched."""
    from vq3d import ops
    from vq3d import _lib as L
    cin = cout = 64
    h, w, d = 8, 8, 2
    geom = ops.ConvGeom(3, 1, 1, True)
    desc, _ = ops.conv_desc(torch.bfloat16, 1, cin, 0, cout, h, w, d, geom, L.PRO_NONE)
    nws = int(L.query("vq3d_conv3d_workspace_size", ctypes.byref(desc), L.PASS_FWD))
    assert nws > 0
    g = torch.Generator().manual_seed(11)
    x = (torch.randn((1, cin, h, w, d), generator=g)).to(torch.bfloat16)
    wt = torch.randn((cout, cin, 3, 3, 3), generator=g) * 0.05
    n = x.numel()
    buf = torch.empty(n + 4, dtype=torch.bfloat16, device=gpu)
    xm = buf[4:].view(1, h, w, d, cin).permute(0, 4, 1, 2, 3)  # channels-last, 8 bytes off 16-B alignment
    xm.copy_(x.to(gpu))
    assert xm.data_ptr() % 16 == 8 and xm.is_contiguous(memory_format=CL)
    canary = 1 << 20
    ws = torch.full((nws + canary,), 0x5A, dtype=torch.uint8, device=gpu)
    y = torch.empty_like(xm, memory_format=CL)
    epi = L.ConvEpilogue(scale=None, bias=None, cbias=None, residual=None, residual_up2=0, act=L.ACT_NONE,
                         act_a=None, act_b=None)
    wf = wt.to(gpu)
    L.call("vq3d_conv3d_fwd", ctypes.byref(desc), L.ptr(xm), None, L.ptr(wf), None, None, ctypes.byref(epi),
           L.ptr(y), ws.data_ptr(), nws, L.stream())
    torch.cuda.synchronize()
    assert bool((ws[nws:] == 0x5A).all()), "the launch wrote past the queried workspace"
    ref = _conv_ref(x.double(), wt.double(), 3, 1, 1, True)
    assert rel(y.float(), ref) < 1.5e-2
