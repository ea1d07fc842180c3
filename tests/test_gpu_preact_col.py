"""Few-channel PreAct blocks on the big grids through the column kernels (csrc/preact_col.hip,
behind vq3d_preact_small_*: (C, branch) = (2, 1), (4, 2), (8, 4), H % 8 == W % 8 == 0,
D % 16 == 0) against a float64 restatement of the block (vqvae/layers.py:176-195) that rounds at
exactly the kernels' bf16 points: t2, t3, out, gz3, gz1, gx and the k^3 weights (matrix-core
operand) rounded to bf16, u1 rounded only as the W1-gradient operand, the 1x1 weights fp32.
What remains is fp32 vs float64 accumulation order and the bf16 ties it flips.

Tolerances: 1e-2 of each tensor's max magnitude for out, gx and every weight gradient; the 8
scalar-parameter gradients as one vector within 2e-2 relative L2 (single sums nearly cancel).
Also: bit-identical gradients run to run (fixed-order reduction), the production (2, 1) shape
at 128x128x32, and a 512x512x128 (4, 2) block checked through size-independent properties
(finite, deterministic, matches a float64 recompute on sampled voxels)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
CL = torch.channels_last_3d
SHAPES = [(1, 2, 16, 16, 32), (1, 4, 16, 8, 64), (1, 8, 8, 16, 32), (2, 4, 8, 8, 32), (1, 4, 8, 16, 16), (1, 2, 128, 128, 32)]


def _block(c, seed):
    from vq3d import layers as VL
    torch.manual_seed(seed)
    blk = VL.PreActFixupResBlock(c, c, mode="same")
    rng = np.random.default_rng(seed)
    with torch.no_grad():
        for n, p in blk.named_parameters():
            if p.numel() == 1:
                p.fill_(float(rng.normal(0, 0.3)))
            else:
                p.normal_(0, 0.3)
        blk.scale.fill_(0.8)
    return blk


HALF = [torch.bfloat16, torch.float16]  # the two 16-bit builds of the kernels
_H = [torch.bfloat16]  # the 16-bit format of the test being run (set per test)


@pytest.fixture(autouse=True)
def _bf16_by_default():
    """Tests that do not pick a format run bf16 (a parametrized fp16 test must not leak its choice)."""
    _H[0] = torch.bfloat16
    yield


def rb(t):
    return t.float().to(_H[0]).double()


def _pad(t):
    return F.pad(t, (1,) * 6, mode="circular")


def _ref_strict(blk, x, g, round_out=True, round_gx=True):
    P = {n: p.detach().double().cpu() for n, p in blk.named_parameters()}
    sc, b1a, b1b, b2a, b2b, b3a, b3b, b4 = (float(P[k]) for k in
                                             ("scale", "bias1a", "bias1b", "bias2a", "bias2b", "bias3a", "bias3b", "bias4"))
    w1, w2, w3 = P["branch_conv1.weight"], P["branch_conv2.weight"], P["branch_conv3.weight"]
    u1 = F.elu(x + b1a) + b1b
    t2 = rb(F.elu(F.conv3d(u1, w1) + b2a) + b2b)
    t3 = rb(F.elu(F.conv3d(_pad(t2), rb(w2)) + b3a) + b3b)
    out = x + sc * F.conv3d(t3, w3) + b4
    out = rb(out) if round_out else out
    acc3 = F.conv3d(g, w3.permute(1, 0, 2, 3, 4))
    gt3 = sc * acc3
    z3 = gt3 * torch.where(t3 - b3b > 0, torch.ones_like(t3), t3 - b3b + 1)
    z3r = rb(z3)
    t2v = t2.clone().requires_grad_(True)
    w2v = rb(w2).clone().requires_grad_(True)
    gt2 = torch.autograd.grad(F.conv3d(_pad(t2v), rb(w2)), t2v, z3r)[0]
    dw2 = torch.autograd.grad(F.conv3d(_pad(t2), w2v), w2v, z3r)[0]
    z1 = gt2 * torch.where(t2 - b2b > 0, torch.ones_like(t2), t2 - b2b + 1)
    z1r = rb(z1)
    gt1 = F.conv3d(z1r, w1.permute(1, 0, 2, 3, 4))
    e1 = torch.where(x + b1a > 0, torch.ones_like(x), torch.exp(x + b1a))
    gx = g + gt1 * e1
    gx = rb(gx) if round_gx else gx
    grads = {"branch_conv3.weight": (sc * torch.einsum("bchwd,bohwd->co", g, t3))[..., None, None, None],
             "scale": (acc3 * t3).sum(), "bias4": g.sum(), "bias3b": gt3.sum(), "bias3a": z3.sum(),
             "branch_conv2.weight": dw2, "bias2b": gt2.sum(), "bias2a": z1.sum(),
             "branch_conv1.weight": torch.einsum("bohwd,bchwd->oc", z1r, rb(u1))[..., None, None, None],
             "bias1b": gt1.sum(), "bias1a": (gt1 * e1).sum()}
    return out, gx, grads


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-12))


def _run(blk, x, gy, dev):
    from vq3d import _lib as L
    from vq3d import ops
    from vq3d.flat import FlatParams
    b, c, h, w, d = x.shape
    assert int(L.query("vq3d_preact_small_plan", b, c, c // 2, h, w, d)) == 2  # the column kernels
    m = blk.to(dev)
    FlatParams(m.parameters(), dev)
    xg = x.to(dev).to(_H[0]).contiguous(memory_format=CL).requires_grad_(True)
    assert ops.preact_small_supported(xg, c // 2) and ops.small_backward_fused(xg)
    y = m(xg)
    y.backward(gy.to(dev).to(_H[0]).contiguous(memory_format=CL))
    torch.cuda.synchronize()
    return m, y, xg


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("half", HALF)
def test_col_block_matches_float64(gpu, shape, half):
    _H[0] = half
    b, c, h, w, d = shape
    blk = _block(c, seed=h + d + c)
    gen = torch.Generator().manual_seed(7)
    x = rb(torch.randn(shape, generator=gen, dtype=torch.float64))
    gy = rb(torch.randn(shape, generator=gen, dtype=torch.float64))
    ry, rgx, rgp = _ref_strict(blk, x, gy)
    m, y, xg = _run(blk, x, gy, gpu)
    errs = {"y": rel(y, ry), "gx": rel(xg.grad, rgx)}
    gs, rs = [], []
    for n, p in m.named_parameters():
        if p.numel() > 1:
            errs["grad/" + n] = rel(p.grad, rgp[n].reshape(p.shape))
        else:
            gs.append(p.grad.double().cpu().reshape(-1))
            rs.append(rgp[n].double().reshape(-1))
    gv, rv = torch.cat(gs), torch.cat(rs)
    errs["scalars"] = float((gv - rv).norm() / rv.norm())
    print(shape, {k: f"{v:.1e}" for k, v in errs.items()})
    bad = {k: v for k, v in errs.items() if not v <= (2e-2 if k == "scalars" else 1e-2)}
    assert not bad, (shape, bad)


def test_col_block_deterministic(gpu):
    shape = (1, 4, 16, 8, 64)
    blk = _block(4, seed=3)
    gen = torch.Generator().manual_seed(1)
    x = rb(torch.randn(shape, generator=gen, dtype=torch.float64))
    gy = rb(torch.randn(shape, generator=gen, dtype=torch.float64))
    res = []
    for _ in range(2):
        m, y, xg = _run(_block(4, seed=3), x, gy, gpu)
        res.append([y.detach().clone(), xg.grad.clone()] + [p.grad.clone() for p in m.parameters()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("half", HALF)
def test_col_block_fullsize_sampled(gpu, half):
    """(4, 2) at 512x512x128 (the decoder's post-upscale blocks): finite, and out / gx on sampled
    voxels equal a float64 recompute of those voxels' 3x3x3 neighbourhoods."""
    _H[0] = half
    shape = (1, 4, 512, 512, 128)
    blk = _block(4, seed=11)
    gen = torch.Generator(device=gpu).manual_seed(5)
    x = torch.randn(shape, generator=gen, device=gpu).to(_H[0])
    gy = torch.randn(shape, generator=gen, device=gpu).to(_H[0])
    m, y, xg = _run(blk, x.float(), gy.float(), gpu)
    assert torch.isfinite(y.float()).all() and torch.isfinite(xg.grad.float()).all()
    for p in m.parameters():
        assert torch.isfinite(p.grad).all()
    # out at sampled voxels from a float64 recompute of a 5^3 window around each (forward only)
    rng = np.random.default_rng(0)
    P = {n: p.detach().double().cpu() for n, p in m.named_parameters()}
    sc, b1a, b1b, b2a, b2b, b3a, b3b, b4 = (float(P[k]) for k in
                                             ("scale", "bias1a", "bias1b", "bias2a", "bias2b", "bias3a", "bias3b", "bias4"))
    worst = 0.0
    for _ in range(8):
        hh, ww, dd = int(rng.integers(0, 512)), int(rng.integers(0, 512)), int(rng.integers(0, 128))
        ih = [(hh + k) % 512 for k in range(-1, 2)]
        iw = [(ww + k) % 512 for k in range(-1, 2)]
        idd = [(dd + k) % 128 for k in range(-1, 2)]
        xs = x.float().double().cpu()[0][:, ih][:, :, iw][:, :, :, idd]  # (4, 3, 3, 3)
        u1 = F.elu(xs + b1a) + b1b
        t2 = rb(F.elu(torch.einsum("oc,chwd->ohwd", P["branch_conv1.weight"][:, :, 0, 0, 0], u1) + b2a) + b2b)
        t3 = rb(F.elu((rb(P["branch_conv2.weight"]) * t2[None]).sum(dim=(1, 2, 3, 4)) + b3a) + b3b)
        o = rb(xs[:, 1, 1, 1] + sc * (P["branch_conv3.weight"][:, :, 0, 0, 0] @ t3) + b4)
        got = y.float().double().cpu()[0, :, hh, ww, dd]
        worst = max(worst, float((got - o).abs().max() / max(float(o.abs().max()), 1e-6)))
    assert worst <= 1e-2, worst


def _check_run_vs_per_block(gpu, shape, nblk):
    """A run of few-channel blocks through layers.BlockStack (Fn.PreActSmallRunFn: per-block fused
    kernels into slices of one run workspace, one reduction launch pair for the whole run; the
    (8, 4) 32x32x8 case takes the brick kernels' reduction) against the blocks run one by one:
    out, gx and every parameter gradient bit-identical (same kernels, same fixed-order sums).  The run
    is unchained here (test_small_run_chained_matches_unchained covers the links)."""
    from vq3d import functional as Fn
    from vq3d import layers as VL
    from vq3d import ops
    ops.set_small_chain(False)
    try:
        _run_vs_per_block(gpu, shape, nblk, Fn, VL)
    finally:
        ops.set_small_chain(True)


def _run_vs_per_block(gpu, shape, nblk, Fn, VL):
    c = shape[1]
    blocks = [_block(c, seed=40 + i) for i in range(nblk)]
    g = torch.Generator().manual_seed(41)
    x = torch.randn(shape, generator=g).bfloat16()
    gy = torch.randn(shape, generator=g).bfloat16()
    res = []
    for chained in (False, True):
        stack = VL.BlockStack(*blocks).to(gpu)
        for p in stack.parameters():
            p.grad = None
        xd = x.to(gpu).contiguous(memory_format=CL).requires_grad_(True)
        if chained:
            assert Fn.small_run_eligible(xd, blocks[0])
            out = stack(xd)
        else:
            out = xd
            for b in stack:
                out = Fn.PreActBlockFn.apply(out, b, *b._fn_params)
        out.backward(gy.to(gpu).contiguous(memory_format=CL))
        torch.cuda.synchronize()
        res.append((out.float().cpu(), xd.grad.float().cpu(),
                    {n: p.grad.cpu().clone() for n, p in stack.named_parameters()}))
    a, b = res
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    for n in a[2]:
        assert torch.equal(a[2][n], b[2][n]), (n, float((a[2][n] - b[2][n]).abs().max()))


@pytest.fixture
def bf16_stream():
    """runs carry a bf16 residual stream (the per-block path's numerics) for the duration of a test"""
    from vq3d import ops
    ops.set_fp32_stream(False)
    yield
    ops.set_fp32_stream(True)


@pytest.mark.parametrize("shape,nblk", [((1, 2, 128, 128, 32), 3), ((1, 4, 16, 8, 64), 2), ((1, 8, 32, 32, 8), 3)])
def test_small_run_bf16_stream_matches_per_block(gpu, shape, nblk, bf16_stream):
    _check_run_vs_per_block(gpu, shape, nblk)


@pytest.mark.parametrize("shape,nblk,out32", [((1, 2, 32, 32, 32), 3, True), ((1, 4, 16, 8, 64), 2, False),
                                              ((1, 8, 32, 32, 8), 3, True), ((1, 8, 16, 16, 32), 2, False),
                                              ((1, 2, 8, 8, 8), 3, False)])
def test_small_run_fp32_stream_matches_float64(gpu, shape, nblk, out32):
    """The residual stream of a run of few-channel blocks (column kernels, and the brick kernels for
    the 32x32x8 / 8x8x8 grids) in fp32 between the blocks, as the reference's autocast blocks return
    fp32 (vqvae/layers.py:187-193): against a float64 restatement that rounds only the conv operands
    (t2, t3, gz3, gz1, k^3 weights) and the run's own bf16 ends (its input, its output unless the
    run hands fp32 on -- out32, the encoder's pre-quantize runs into the Quantizer -- and gx of the
    input).  Tolerances as the single-block test; intermediate outs / gxs are unrounded here."""
    from vq3d import functional as Fn
    from vq3d import layers as VL
    from vq3d import ops
    assert ops.fp32_stream()
    c = shape[1]
    blocks = [_block(c, seed=60 + i) for i in range(nblk)]
    gen = torch.Generator().manual_seed(61)
    x = rb(torch.randn(shape, generator=gen, dtype=torch.float64))
    gy = rb(torch.randn(shape, generator=gen, dtype=torch.float64))
    # float64 reference of the chain
    xs = [x]
    for i, blk in enumerate(blocks):
        o, _, _ = _ref_strict(blk, xs[-1], torch.zeros_like(x), round_out=(i == nblk - 1 and not out32))
        xs.append(o)
    g = gy
    rgrads = [None] * nblk
    for i in reversed(range(nblk)):
        _, g, rgrads[i] = _ref_strict(blocks[i], xs[i], g, round_gx=(i == 0))
    stack = VL.BlockStack(*blocks).to(gpu)
    stack.out_fp32 = out32
    from vq3d.flat import FlatParams
    FlatParams(stack.parameters(), gpu)
    xd = x.float().to(gpu).bfloat16().contiguous(memory_format=CL).requires_grad_(True)
    assert Fn.small_run_eligible(xd, blocks[0])
    out = stack(xd)
    assert out.dtype == (torch.float32 if out32 else torch.bfloat16)
    gd = gy.to(gpu).to(out.dtype).contiguous(memory_format=CL)
    out.backward(gd)
    torch.cuda.synchronize()
    assert xd.grad.dtype == torch.bfloat16
    errs = {"y": rel(out, xs[-1]), "gx": rel(xd.grad, g)}
    for i, blk in enumerate(stack):
        gs, rs = [], []
        for n, p in blk.named_parameters():
            if p.numel() > 1:
                errs[f"{i}/{n}"] = rel(p.grad, rgrads[i][n].reshape(p.shape))
            else:
                gs.append(p.grad.double().cpu().reshape(-1))
                rs.append(rgrads[i][n].double().reshape(-1))
        gv, rv = torch.cat(gs), torch.cat(rs)
        errs[f"{i}/scalars"] = float((gv - rv).norm() / rv.norm())
    print(shape, nblk, out32, {k: f"{v:.1e}" for k, v in errs.items()})
    bad = {k: v for k, v in errs.items() if not v <= (2e-2 if k.endswith("scalars") else 1e-2)}
    assert not bad, (shape, bad)


@pytest.mark.parametrize("fmt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape,nblk", [((1, 4, 32, 16, 32), 3), ((2, 2, 16, 16, 32), 4), ((1, 8, 16, 16, 32), 2),
                                        ((1, 4, 8, 8, 16), 2)])
def test_small_run_chained_matches_unchained(gpu, shape, nblk, fmt):
    """Chained column-kernel runs (vq3d_preact_small_fwd_chain: each block's t2 formed in the previous
    block's epilogue) against the unchained run: out, gx and every parameter gradient bit-identical
    (same formulas, same order per voxel).  fp32 residual stream, both 16-bit formats."""
    from vq3d import layers as VL
    from vq3d import ops
    c = shape[1]
    blocks = [_block(c, seed=70 + i) for i in range(nblk)]
    g = torch.Generator().manual_seed(71)
    x = torch.randn(shape, generator=g).to(fmt)
    gy = torch.randn(shape, generator=g).to(fmt)
    res = []
    for chained in (False, True):
        ops.set_small_chain(chained)
        try:
            stack = VL.BlockStack(*blocks).to(gpu)
            for p in stack.parameters():
                p.grad = None
            xd = x.to(gpu).contiguous(memory_format=CL).requires_grad_(True)
            assert ops.small_chain_ok(xd, nblk) == chained
            out = stack(xd)
            out.backward(gy.to(gpu).contiguous(memory_format=CL))
            torch.cuda.synchronize()
            res.append((out.float().cpu(), xd.grad.float().cpu(),
                        {n: p.grad.cpu().clone() for n, p in stack.named_parameters()}))
        finally:
            ops.set_small_chain(True)
    a, b = res
    assert torch.equal(a[0], b[0]), float((a[0] - b[0]).abs().max())
    assert torch.equal(a[1], b[1]), float((a[1] - b[1]).abs().max())
    for n in a[2]:
        assert torch.equal(a[2][n], b[2][n]), (n, float((a[2][n] - b[2][n]).abs().max()))


def test_small_run_chain_saved_tensors(gpu):
    """The chained forward's saved t2 / t3 equal the unchained forward's, block by block."""
    from vq3d import ops
    c, shape, nblk = 4, (1, 4, 16, 16, 32), 3
    blocks = [_block(c, seed=80 + i).to(gpu) for i in range(nblk)]
    x = torch.randn(shape, generator=torch.Generator().manual_seed(81)).bfloat16().to(gpu).contiguous(
        memory_format=CL)
    odts = [torch.float32] * (nblk - 1) + [torch.bfloat16]
    out_c, saved_c = ops.preact_small_run_fwd(x, blocks, True, odts)
    xs, outs = x, []
    for i, blk in enumerate(blocks):
        o, t2, t3 = ops.preact_small_fwd(xs, blk, out_dtype=odts[i], fmt=torch.bfloat16)
        outs.append((t2, t3))
        xs = o
    torch.cuda.synchronize()
    assert torch.equal(out_c, xs)
    for (_, t2c, t3c), (t2, t3) in zip(saved_c, outs):
        assert torch.equal(t2c, t2) and torch.equal(t3c, t3)
