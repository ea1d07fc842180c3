"""GPU: the bf16 MFMA implicit-GEMM conv engine against the fp32 VALU engine on the same
bf16-representable inputs, over the geometries / channel counts the model uses (including
tiny, odd and wrap-heavy grids).  Tolerance: 1.5e-2 of the output's max magnitude (bf16
weights and outputs in the MFMA path, fp32 in the reference engine)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CL = torch.channels_last_3d

CASES = [
    # (cin, cout, (h, w, d), k, s, p, circular)
    (9, 9, (16, 16, 8), 3, 1, 1, True),
    (4, 4, (8, 8, 32), 3, 1, 1, True),
    (1, 1, (8, 8, 8), 3, 1, 1, True),
    (2, 2, (6, 5, 3), 3, 1, 1, True),
    (16, 16, (8, 8, 2), 3, 1, 1, True),
    (36, 36, (8, 8, 4), 3, 1, 1, True),
    (72, 72, (4, 4, 2), 3, 1, 1, True),
    (128, 64, (4, 4, 2), 3, 1, 1, True),
    (18, 9, (4, 4, 4), 3, 1, 1, False),
    (4, 4, (8, 8, 8), 4, 2, 1, True),
    (8, 8, (4, 4, 2), 4, 2, 1, True),
    (16, 16, (8, 8, 4), 4, 2, 1, False),
    (4, 8, (8, 8, 8), 2, 2, 0, False),
    (3, 5, (3, 3, 3), 3, 1, 1, True),
    (1, 4, (2, 2, 1), 3, 1, 1, True),
    (18, 9, (8, 8, 8), 1, 1, 0, False),
    (9, 2, (8, 8, 5), 1, 1, 0, False),
    (64, 128, (4, 4, 2), 1, 1, 0, False),
    # channel counts that are not multiples of 4 (lines weight gradient, vector-run staging)
    (9, 9, (16, 16, 32), 3, 1, 1, True),
    (1, 1, (16, 8, 32), 3, 1, 1, True),
    (2, 2, (8, 8, 40), 3, 1, 1, True),
    (9, 9, (8, 8, 8), 3, 1, 1, False),
    (3, 6, (6, 6, 8), 4, 2, 1, True),
    # 4 / 8 output channels: 4 / 2 output voxels along D per MFMA row (lines engine D-shifts),
    # incl. a brick overhanging the grid in D, zero padding, stride 2 and a depth that falls back
    (4, 4, (16, 16, 64), 3, 1, 1, True),
    (8, 8, (8, 8, 32), 3, 1, 1, True),
    (4, 8, (8, 16, 16), 3, 1, 1, False),
    (8, 4, (8, 8, 12), 3, 1, 1, True),
    (9, 4, (8, 8, 24), 3, 1, 1, True),
    (4, 9, (8, 8, 16), 3, 1, 1, True),
    (4, 4, (16, 16, 32), 4, 2, 1, True),
    (8, 8, (16, 16, 16), 4, 2, 1, False),
    (4, 4, (8, 8, 6), 3, 1, 1, True),
]


HALF = [torch.bfloat16, torch.float16]  # the two 16-bit builds of the kernels
_H = [torch.bfloat16]  # the 16-bit format of the test being run (set per test)


@pytest.fixture(autouse=True)
def _bf16_by_default():
    """Tests that do not pick a format run bf16 (a parametrized fp16 test must not leak its choice)."""
    _H[0] = torch.bfloat16
    yield


def rnd(shape, dev, g, scale=1.0):
    return (torch.randn(shape, device=dev, generator=g) * scale).to(_H[0]).float()


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("half", HALF)
def test_mfma_forward_and_dgrad_match_valu(gpu, case, half):
    _H[0] = half
    from vq3d import ops
    cin, cout, (h, w, d), k, s, p, circ = case
    g = torch.Generator(device=gpu).manual_seed(hash(case) % 1000)
    geom = ops.ConvGeom(k, s, p, circ)
    x = rnd((2, cin, h, w, d), gpu, g).contiguous(memory_format=CL)
    wt = rnd((cout, cin, k, k, k), gpu, g, 0.3)
    a = rnd((1,), gpu, g, 0.1)
    b = rnd((1,), gpu, g, 0.1)
    ref = ops.conv_fwd(x, wt, geom, pro=(a, b), act=(b, a))
    out = ops.conv_fwd(x.to(_H[0]), wt, geom, pro=(a, b), act=(b, a))
    assert rel(out.float(), ref) < 1.5e-2, ("fwd", case, rel(out.float(), ref))
    if s != 1:
        return
    oh, ow, od = geom.out(h), geom.out(w), geom.out(d)
    gy = rnd((2, cout, oh, ow, od), gpu, g).contiguous(memory_format=CL)
    add = rnd((2, cin, h, w, d), gpu, g).contiguous(memory_format=CL)
    dpre_r = torch.zeros(1, device=gpu)
    dpost_r = torch.zeros(1, device=gpu)
    dpre = torch.zeros(1, device=gpu)
    dpost = torch.zeros(1, device=gpu)
    gscale = rnd((1,), gpu, g)
    gr, _ = ops.conv_bwd(gy, x, wt, geom, pro=(a, b), gscale=gscale, aux=x, addend=add, dpro_pre=dpre_r,
                         dpro_post=dpost_r)
    gm, _ = ops.conv_bwd(gy.to(_H[0]), x.to(_H[0]), wt, geom, pro=(a, b), gscale=gscale,
                         aux=x.to(_H[0]), addend=add.to(_H[0]), dpro_pre=dpre, dpro_post=dpost)
    assert rel(gm.float(), gr) < 1.5e-2, ("dgrad", case, rel(gm.float(), gr))
    assert abs(float(dpre) - float(dpre_r)) <= 2e-2 * float(gr.abs().sum()) / gr.numel() * gr.numel() ** 0.5 + 1e-3


@pytest.mark.parametrize("half", HALF)
def test_mfma_dual_input_and_residual(gpu, half):
    _H[0] = half
    from vq3d import ops
    g = torch.Generator(device=gpu).manual_seed(3)
    x1 = rnd((1, 8, 8, 8, 4), gpu, g).contiguous(memory_format=CL)
    x2 = rnd((1, 2, 8, 8, 4), gpu, g).contiguous(memory_format=CL)
    wt = rnd((6, 10, 3, 3, 3), gpu, g, 0.3)
    res = rnd((1, 6, 4, 4, 2), gpu, g).contiguous(memory_format=CL)
    sc = rnd((1,), gpu, g)
    bi = rnd((1,), gpu, g)
    geom = ops.ConvGeom(3, 1, 1, True)
    ref = ops.conv_fwd(x1, wt, geom, x2=x2, scale=sc, bias=bi, residual=res, residual_up2=True)
    out = ops.conv_fwd(x1.to(_H[0]), wt, geom, x2=x2.to(_H[0]), scale=sc, bias=bi, residual=res.to(_H[0]),
                       residual_up2=True)
    assert rel(out.float(), ref) < 1.5e-2


# more than 64 output channels: the MFMA weight gradient in 64-channel chunks (the top level's
# stride-2 down convs and 128-channel branch convs), incl. a partial last chunk
WGRAD_WIDE = [
    (64, 128, (8, 8, 4), 4, 2, 1, True),
    (128, 128, (8, 8, 4), 4, 2, 1, True),
    (16, 96, (8, 8, 4), 3, 1, 1, True),
    (32, 72, (6, 6, 4), 4, 2, 1, False),
    (128, 256, (8, 8, 4), 2, 2, 0, False),
]


@pytest.mark.parametrize("case", CASES + WGRAD_WIDE)
@pytest.mark.parametrize("half", HALF)
def test_tiled_wgrad_matches_valu(gpu, case, half):
    """bf16 MFMA / LDS-tiled weight gradient (+ epilogue scalar / conv-bias gradients) vs the fp32 engine."""
    _H[0] = half
    from vq3d import ops
    cin, cout, (h, w, d), k, s, p, circ = case
    g = torch.Generator(device=gpu).manual_seed(1 + hash(case) % 1000)
    geom = ops.ConvGeom(k, s, p, circ)
    x = rnd((2, cin, h, w, d), gpu, g).contiguous(memory_format=CL)
    wt = rnd((cout, cin, k, k, k), gpu, g, 0.3)
    a = rnd((1,), gpu, g, 0.1)
    b = rnd((1,), gpu, g, 0.1)
    sc = rnd((1,), gpu, g)
    oh, ow, od = geom.out(h), geom.out(w), geom.out(d)
    gy = rnd((2, cout, oh, ow, od), gpu, g).contiguous(memory_format=CL)
    outs = []
    for dt in (torch.float32, _H[0]):
        dw = torch.zeros_like(wt)
        dscale = torch.zeros(1, device=gpu)
        dbias = torch.zeros(1, device=gpu)
        dcb = torch.zeros(cout, device=gpu)
        ops.conv_bwd(gy.to(dt), x.to(dt), wt, geom, pro=(a, b), want_gx=False, dw=dw, dscale=dscale, dbias=dbias,
                     dcbias=dcb, escale=sc)
        outs.append((dw, dscale, dbias, dcb))
    (rw, rs, rb, rc), (mw, ms, mb, mc) = outs
    assert rel(mw, rw) < 1.5e-2, ("dw", case, rel(mw, rw))
    assert rel(mc, rc) < 1.5e-2, ("dcbias", case)
    assert abs(float(mb) - float(rb)) <= 1e-2 * float(rc.abs().sum()) + 1e-3
    assert abs(float(ms) - float(rs)) <= 2e-2 * (float((wt * rw).abs().sum()) / max(abs(float(sc)), 1e-3)) + 1e-3


S2_DGRAD_CASES = [
    # (cin, cout, (h, w, d) input, aux + addend + gscale): 4x4x4 stride-2 circular backward-data
    # (k_dgrad_s2_pair: parity-class rows, the down blocks' branch conv), incl. a 2-deep grid that
    # wraps inside one tile
    (4, 4, (8, 8, 16), True), (4, 8, (8, 8, 16), False), (8, 4, (8, 16, 8), True), (8, 8, (4, 4, 2), True),
    (8, 8, (16, 8, 32), False), (4, 4, (2, 4, 4), True),
    # 16+ input channels (k_dgrad_s2_mma: one GEMM per parity class on the matrix cores): the down
    # blocks' 4x4x4 branch convs and 2x2x2 zero-padded skip convs (k, p, circular), incl. channel
    # tiles spread over workgroups (48), 8-channel g rows and a single-tap K of 32; more than 512
    # input voxels (fewer go to the small-grid engine)
    (16, 16, (16, 16, 8), True, 4, 1, True), (32, 32, (8, 8, 8), True, 4, 1, True),
    (64, 64, (16, 8, 4), False, 4, 1, True), (128, 128, (8, 8, 8), True, 4, 1, True),
    (48, 24, (12, 8, 6), True, 4, 1, True), (16, 8, (8, 8, 8), True, 4, 1, True),
    (16, 32, (16, 8, 8), True, 2, 0, False), (64, 128, (8, 8, 8), True, 2, 0, False),
    (128, 256, (8, 8, 8), False, 2, 0, False),
    # the zero-padded 2x2x2 skip convs of the few-channel levels (pair kernel: no tap leaves the grid)
    (4, 8, (8, 8, 16), True, 2, 0, False), (8, 4, (16, 8, 8), True, 2, 0, False), (8, 8, (8, 8, 8), False, 2, 0, False),
    (8, 16, (16, 8, 8), True, 2, 0, False),
]


@pytest.mark.parametrize("case", S2_DGRAD_CASES)
@pytest.mark.parametrize("half", HALF)
def test_dgrad_s2_matches_valu(gpu, case, half):
    """bf16 stride-2 backward-data (+ the activated-aux derivative, the addend, the gradient scale and
    the prologue-scalar partial sums) vs the fp32 engine on the same bf16-representable inputs."""
    _H[0] = half
    from vq3d import ops
    cin, cout, (h, w, d), epi = case[:4]
    k, p, circ = case[4:] if len(case) > 4 else (4, 1, True)
    g = torch.Generator(device=gpu).manual_seed(11 + h + cin)
    geom = ops.ConvGeom(k, 2, p, circ)
    x = rnd((2, cin, h, w, d), gpu, g).contiguous(memory_format=CL)
    wt = rnd((cout, cin, k, k, k), gpu, g, 0.3)
    gy = rnd((2, cout, geom.out(h), geom.out(w), geom.out(d)), gpu, g).contiguous(memory_format=CL)
    add = rnd((2, cin, h, w, d), gpu, g).contiguous(memory_format=CL)
    ab, gs = rnd((1,), gpu, g, 0.3), rnd((1,), gpu, g)
    outs = []
    for dt in (torch.float32, _H[0]):
        pre, post = torch.zeros(1, device=gpu), torch.zeros(1, device=gpu)
        kw = dict(gscale=gs, aux=x.to(dt), aux_b=ab, addend=add.to(dt), dpro_pre=pre, dpro_post=post) if epi else {}
        gx, _ = ops.conv_bwd(gy.to(dt), x.to(dt), wt, geom, **kw)
        outs.append((gx.float(), pre, post))
    (r, rp, rq), (m, mp, mq) = outs
    assert rel(m, r) < 1.5e-2, rel(m, r)
    if epi:
        tol = 2e-2 * float(r.abs().sum()) / r.numel() ** 0.5 + 1e-3
        assert abs(float(mp) - float(rp)) <= tol and abs(float(mq) - float(rq)) <= tol


WGRAD_DS_CASES = [
    # (batch, cin, cout, (h, w, d) input, k, s, p, circular, prologue + bias gradient)
    (2, 4, 4, (8, 8, 128), 3, 1, 1, True, False),    # up-block ResizeConv branch conv (D-shifted kernel)
    (1, 4, 4, (4, 12, 128), 3, 1, 1, True, False),
    (1, 4, 4, (8, 8, 128), 4, 2, 1, True, False),    # down-block branch convs
    (2, 8, 8, (4, 8, 64), 4, 2, 1, True, False),
    (1, 16, 16, (8, 8, 32), 4, 2, 1, True, False),
    (1, 4, 8, (8, 8, 128), 2, 2, 0, False, True),    # down-block skip convs (+ bias1c, bias1d)
    (2, 8, 16, (4, 8, 64), 2, 2, 0, False, True),
    (1, 4, 4, (8, 8, 64), 3, 1, 1, True, False),     # depth without an instance: generic engine
]


@pytest.mark.parametrize("case", WGRAD_DS_CASES)
@pytest.mark.parametrize("half", HALF)
def test_wgrad_dshift(gpu, case, half):
    """Few-channel weight gradients without scale / conv-bias epilogue parameters (wgrad_ds.hip: the
    full-resolution up / down block convs, D-shifted MFMA over whole D-lines), bf16, accumulated
    into dW (and, for the skip convs, the bias gradient sum(g) and the prologue x + b), vs the fp32
    VALU engine on the same bf16-representable inputs: only the summation order differs."""
    _H[0] = half
    from vq3d import ops
    bsz, cin, cout, (h, w, d), k, s, p, circ, pro = case
    g = torch.Generator(device=gpu).manual_seed(5 + h + cin)
    geom = ops.ConvGeom(k, s, p, circ)
    x = rnd((bsz, cin, h, w, d), gpu, g).contiguous(memory_format=CL)
    gy = rnd((bsz, cout, geom.out(h), geom.out(w), geom.out(d)), gpu, g).contiguous(memory_format=CL)
    wt = rnd((cout, cin, k, k, k), gpu, g, 0.3)
    base = rnd((cout, cin, k, k, k), gpu, g)
    b1c = rnd((1,), gpu, g, 0.1)
    outs = []
    for dt in (torch.float32, _H[0]):
        dw = base.clone()
        db = torch.full((1,), 0.5, device=gpu)
        ops.conv_bwd(gy.to(dt), x.to(dt), wt, geom, want_gx=False, dw=dw, pro=(b1c,) if pro else None,
                     dbias=db if pro else None)
        outs.append((dw - base, db - 0.5))
    assert rel(outs[1][0], outs[0][0]) < 1e-3, rel(outs[1][0], outs[0][0])
    if pro:
        assert abs(float(outs[1][1]) - float(outs[0][1])) <= 1e-3 * float(gy.abs().sum()) ** 0.5 + 1e-3


PW_CASES = [
    # (cin, cin2, cout, (h, w, d))
    (9, 0, 18, (16, 16, 8)),
    (18, 0, 9, (8, 8, 8)),
    (4, 0, 2, (32, 16, 64)),
    (2, 0, 4, (8, 8, 8)),
    (1, 0, 2, (5, 7, 3)),
    (16, 2, 18, (8, 8, 4)),
    (64, 8, 72, (4, 4, 2)),
    (256, 0, 32, (4, 4, 2)),
    (72, 0, 36, (8, 8, 8)),
    # bf16 matrix-core path (k_pw_wgrad_mma): the step's shapes, odd channel counts (slab-staged),
    # a concatenated second input, ragged voxel counts, 255 + 1 columns, 8 co tiles
    (16, 0, 8, (64, 64, 32)),
    (32, 0, 16, (32, 32, 16)),
    (128, 0, 64, (16, 16, 4)),
    (64, 0, 128, (16, 16, 4)),
    (9, 0, 8, (32, 32, 16)),
    (18, 0, 18, (16, 16, 8)),
    (8, 8, 16, (16, 16, 8)),
    (16, 0, 8, (7, 9, 5)),
    (3, 5, 7, (9, 9, 9)),
    (255, 0, 16, (8, 8, 4)),
    (32, 0, 48, (8, 8, 8)),
]


@pytest.mark.parametrize("case", PW_CASES)
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
def test_pointwise_wgrad_vs_torch(gpu, case, dt):
    """1x1x1 weight / conv-bias / scalar gradients vs a plain torch fp32 einsum of the same
    (bf16-representable) inputs, with the ELU-affine prologue and a concatenated second input."""
    _H[0] = dt if dt != torch.float32 else torch.bfloat16  # inputs representable in the tested format
    from vq3d import ops
    cin, cin2, cout, (h, w, d) = case
    g = torch.Generator(device=gpu).manual_seed(7 + cin * 31 + cout)
    x = rnd((2, cin, h, w, d), gpu, g).contiguous(memory_format=CL)
    x2 = rnd((2, cin2, h, w, d), gpu, g).contiguous(memory_format=CL) if cin2 else None
    wt = rnd((cout, cin + cin2, 1, 1, 1), gpu, g, 0.3)
    a, b, sc = rnd((1,), gpu, g, 0.1), rnd((1,), gpu, g, 0.1), rnd((1,), gpu, g)
    gy = rnd((2, cout, h, w, d), gpu, g).contiguous(memory_format=CL)
    xs = x if x2 is None else torch.cat([x, x2], 1)
    xp = torch.nn.functional.elu(xs.float() + a) + b
    G = torch.einsum("bchwd,bohwd->oc", xp.double(), gy.double())
    dw = torch.zeros_like(wt)
    dscale, dbias, dcb = torch.zeros(1, device=gpu), torch.zeros(1, device=gpu), torch.zeros(cout, device=gpu)
    ops.conv_bwd(gy.to(dt), x.to(dt), wt, ops.ConvGeom(1), pro=(a, b), x2=None if x2 is None else x2.to(dt),
                 want_gx=False, dw=dw, dscale=dscale, dbias=dbias, dcbias=dcb, escale=sc)
    tol = 1e-4 if dt == torch.float32 else 1.5e-2
    assert rel(dw.view(cout, -1), (G * sc.double()).float()) < tol
    assert rel(dcb, gy.double().sum((0, 2, 3, 4)).float()) < tol
    assert abs(float(dbias) - float(gy.double().sum())) <= tol * float(gy.abs().sum()) + 1e-4
    ref_s = float((wt.view(cout, -1).double() * G).sum())
    assert abs(float(dscale) - ref_s) <= tol * float((wt.view(cout, -1).double() * G).abs().sum()) + 1e-4


PW_MMA_CASES = [
    # (batch, cin, cin2, cout, (h, w, d)): the up / down blocks' 1x1 convs on the mid grids, a
    # concatenated second input, a ragged voxel count, K < 32, 9 outputs, the largest K / N
    (1, 16, 0, 8, (64, 64, 32)),
    (1, 32, 0, 16, (32, 32, 16)),
    (2, 128, 0, 64, (8, 8, 4)),
    (1, 8, 0, 16, (32, 32, 32)),
    (1, 8, 8, 16, (16, 16, 8)),
    (2, 16, 0, 8, (5, 5, 5)),
    (1, 24, 0, 9, (8, 8, 8)),
    (1, 128, 128, 128, (8, 8, 4)),
    (2, 64, 32, 40, (8, 8, 8)),
]


@pytest.mark.parametrize("case", PW_MMA_CASES)
@pytest.mark.parametrize("half", HALF)
def test_pointwise_mma_matches_valu(gpu, case, half):
    """bf16 matrix-core 1x1 conv (k_pw_mma: bf16 operands, fp32 accumulation) vs the fp32 pointwise
    engine: forward with the ELU prologue and every epilogue term, backward-data with gscale, the
    prologue derivative, the addend, the split output and the prologue-scalar sums."""
    _H[0] = half
    from vq3d import ops
    bt, cin, cin2, cout, (h, w, d) = case
    g = torch.Generator(device=gpu).manual_seed(7 + cin + cout + h)
    geom = ops.ConvGeom(1, 1, 0, False)
    x = rnd((bt, cin, h, w, d), gpu, g).contiguous(memory_format=CL)
    x2 = rnd((bt, cin2, h, w, d), gpu, g).contiguous(memory_format=CL) if cin2 else None
    wt = rnd((cout, cin + cin2, 1, 1, 1), gpu, g, 0.3)
    a, b = rnd((1,), gpu, g, 0.1), rnd((1,), gpu, g, 0.1)
    sc, bi = rnd((1,), gpu, g), rnd((1,), gpu, g)
    cb = rnd((cout,), gpu, g)
    res = rnd((bt, cout, h, w, d), gpu, g).contiguous(memory_format=CL)
    bf = lambda t: None if t is None else t.to(_H[0])
    ref = ops.conv_fwd(x, wt, geom, pro=(a, b), x2=x2, scale=sc, bias=bi, cbias=cb, residual=res, act=(b, a))
    out = ops.conv_fwd(bf(x), wt, geom, pro=(a, b), x2=bf(x2), scale=sc, bias=bi, cbias=cb, residual=bf(res),
                       act=(b, a))
    assert torch.isfinite(out.float()).all()
    assert rel(out.float(), ref) < 1.5e-2, ("fwd", case, rel(out.float(), ref))
    gy = rnd((bt, cout, h, w, d), gpu, g).contiguous(memory_format=CL)
    add = rnd((bt, cin, h, w, d), gpu, g).contiguous(memory_format=CL)
    gscale = rnd((1,), gpu, g)
    res_ = []
    for cast in (lambda t: t, bf):
        pre, post = torch.zeros(1, device=gpu), torch.zeros(1, device=gpu)
        gx, gx2 = ops.conv_bwd(cast(gy), cast(x), wt, geom, pro=(a, b), x2=cast(x2), gscale=gscale, aux=cast(x),
                               addend=cast(add), dpro_pre=pre, dpro_post=post)
        res_.append((gx, gx2, pre, post))
    (gr, gr2, pre_r, post_r), (gm, gm2, pre_m, post_m) = res_
    assert rel(gm.float(), gr) < 1.5e-2, ("dgrad", case, rel(gm.float(), gr))
    if cin2:
        assert rel(gm2.float(), gr2) < 1.5e-2, ("dgrad x2", case, rel(gm2.float(), gr2))
    tol = 2e-2 * float((gr - add).abs().max()) * gr.numel() ** 0.5 + 1e-3
    assert abs(float(pre_m) - float(pre_r)) <= tol
    assert abs(float(post_m) - float(post_r)) <= tol


@pytest.mark.parametrize("case", [(4, 4, (16, 16, 32)), (2, 8, (8, 8, 8)), (4, 2, (6, 10, 4)), (8, 8, (4, 4, 4))])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
def test_pointwise_rows_residual_up2(gpu, case, dt):
    """Few-channel 1x1 conv with the ResizeConv skip's half-grid residual upsampled x2 on the fly
    (k_pw_rows; vqvae/layers.py:591-597) vs torch: conv * scale + bias + trilinear(res)."""
    _H[0] = dt if dt != torch.float32 else torch.bfloat16  # inputs representable in the tested format
    from vq3d import ops
    cin, cout, (h, w, d) = case
    g = torch.Generator(device=gpu).manual_seed(cin * 7 + cout + h)
    x = rnd((2, cin, h, w, d), gpu, g).contiguous(memory_format=CL)
    wt = rnd((cout, cin, 1, 1, 1), gpu, g, 0.3)
    res = rnd((2, cout, h // 2, w // 2, d // 2), gpu, g).contiguous(memory_format=CL)
    sc, bi = rnd((1,), gpu, g), rnd((1,), gpu, g)
    ref = (torch.nn.functional.conv3d(x.double(), wt.double()) * sc.double() + bi.double() +
           torch.nn.functional.interpolate(res.double(), scale_factor=2, mode="trilinear", align_corners=False))
    out = ops.conv_fwd(x.to(dt), wt, ops.ConvGeom(1), scale=sc, bias=bi, residual=res.to(dt), residual_up2=True)
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert rel(out.float(), ref.float()) < tol, rel(out.float(), ref.float())
