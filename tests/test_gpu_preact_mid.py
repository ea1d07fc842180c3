"""Fused PreAct block of the 18-channel level (csrc/preact_mid.hip: forward 2 launches, backward
3) against float64 torch-CPU restatements of vqvae/layers.py:176-195 and against the per-conv
engine path of the same block:

* strict: a float64 restatement that rounds to bf16 exactly where the kernels do (t2, t3, out;
  gz3, gz1, gx; the matrix-core weights W2 / W3, the backward's W1^T / W3^T operands and the
  W1-gradient operand u1) -- what remains is fp32-vs-float64 summation order.  Tolerances: every tensor within 1e-2 of its max
  magnitude, every scalar-parameter gradient within 2e-2 relative.
* loose: the plain float64 block (no rounding), 3e-2 of the max for output / gx / weight grads
  (bf16 activations).
Shapes include the production one (1 x 18 x 128 x 128 x 32, the published model's decoder
bottom level) and grids whose circular wrap lands inside the first / last tile.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last_3d
SHAPES = [(1, 18, 8, 8, 16), (2, 18, 16, 8, 16), (1, 18, 32, 16, 16), (1, 18, 16, 16, 64), (1, 18, 128, 128, 32)]


def _block(seed):
    from vq3d import layers as VL
    torch.manual_seed(seed)
    blk = VL.PreActFixupResBlock(18, 18, mode="same")
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
    """round float64 -> the 16-bit format -> float64 (round-to-nearest-even, torch's conversion)"""
    return t.float().to(_H[0]).double()


def rnd(t):
    return t.to(_H[0]).double()


def pad(t):
    return F.pad(t, (1,) * 6, mode="circular")


def _ref_strict(P, x, g):
    """float64 block fwd + bwd with the kernels' bf16 rounding points."""
    sc, b1a, b1b, b2a, b2b, b3a, b3b, b4 = (float(P[k]) for k in
                                             ("scale", "bias1a", "bias1b", "bias2a", "bias2b", "bias3a", "bias3b", "bias4"))
    w1, w2, w3 = P["branch_conv1.weight"], P["branch_conv2.weight"], P["branch_conv3.weight"]
    w2r, w3r = rb(w2), rb(w3)
    u1 = F.elu(x + b1a) + b1b
    t2 = rb(F.elu(F.conv3d(rb(u1), rb(w1)) + b2a) + b2b)
    t2v = t2.clone().requires_grad_(True)
    w2v = w2.clone().requires_grad_(True)
    h2 = F.conv3d(pad(t2v), w2v)
    t3 = rb(F.elu(F.conv3d(pad(t2), w2r) + b3a) + b3b)
    o3 = F.conv3d(t3, w3r)
    out = rb(o3 * sc + b4 + x)
    # backward
    G3 = torch.einsum("bchwd,bohwd->co", g, t3)
    gt3 = sc * F.conv3d(g, w3r.permute(1, 0, 2, 3, 4))
    d3 = torch.where(t3 - b3b > 0, torch.ones_like(t3), t3 - b3b + 1)
    z3 = gt3 * d3
    gz3 = rb(z3)
    gt2 = torch.autograd.grad(F.conv3d(pad(t2v), w2r), t2v, gz3)[0]
    dw2 = torch.autograd.grad(h2, w2v, gz3)[0]
    d2 = torch.where(t2 - b2b > 0, torch.ones_like(t2), t2 - b2b + 1)
    z1 = gt2 * d2
    gz1 = rb(z1)
    gt1 = F.conv3d(gz1, rb(w1).permute(1, 0, 2, 3, 4))
    e1 = torch.where(x + b1a > 0, torch.ones_like(x), torch.exp(x + b1a))
    gx = rb(g + gt1 * e1)
    grads = {
        "branch_conv3.weight": (sc * G3)[..., None, None, None], "scale": (w3r[..., 0, 0, 0] * G3).sum().reshape(1),
        "bias4": g.sum().reshape(1), "bias3b": gt3.sum().reshape(1), "bias3a": z3.sum().reshape(1),
        "branch_conv2.weight": dw2, "bias2b": gt2.sum().reshape(1), "bias2a": z1.sum().reshape(1),
        "branch_conv1.weight": torch.einsum("bohwd,bchwd->oc", gz1, rb(u1))[..., None, None, None],
        "bias1b": gt1.sum().reshape(1), "bias1a": (gt1 * e1).sum().reshape(1),
    }
    return out, gx, grads


def _ref_loose(P, x, g):
    P = {n: p.clone().requires_grad_(True) for n, p in P.items()}
    x = x.clone().requires_grad_(True)
    h = F.elu(x + P["bias1a"])
    h = F.conv3d(h + P["bias1b"], P["branch_conv1.weight"])
    h = F.elu(h + P["bias2a"])
    h = F.conv3d(pad(h + P["bias2b"]), P["branch_conv2.weight"])
    h = F.elu(h + P["bias3a"])
    h = F.conv3d(h + P["bias3b"], P["branch_conv3.weight"])
    out = h * P["scale"] + P["bias4"] + x
    out.backward(g)
    return out.detach(), x.grad, {n: p.grad for n, p in P.items()}


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-12))


def _run(blk, x, gy, dev, mid):
    from vq3d import ops
    from vq3d.flat import FlatParams
    ops.set_mid_blocks(mid)
    try:
        m = blk.to(dev)
        for p in m.parameters():
            p.grad = None
        FlatParams(m.parameters(), dev)
        xg = x.to(dev).to(_H[0]).contiguous(memory_format=CL).requires_grad_(True)
        y = m(xg)
        y.backward(gy.to(dev).to(_H[0]).contiguous(memory_format=CL))
        torch.cuda.synchronize()
        return y.detach().float().cpu(), xg.grad.float().cpu(), {n: p.grad.cpu().clone()
                                                                  for n, p in m.named_parameters()}
    finally:
        ops.set_mid_blocks(True)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("half", HALF)
def test_fused_mid_block(gpu, shape, half):
    _H[0] = half
    from vq3d import ops
    blk = _block(seed=shape[2] + shape[4])
    g = torch.Generator().manual_seed(11)
    x = rnd(torch.randn(shape, generator=g))
    gy = rnd(torch.randn(shape, generator=g))
    xg = x.to(gpu).to(_H[0]).contiguous(memory_format=CL)
    assert ops.preact_mid_supported(xg, 9)
    P = {n: p.detach().double().clone() for n, p in blk.named_parameters()}
    sy, sgx, sgp = _ref_strict(P, x, gy)
    y1, gx1, gp1 = _run(blk, x, gy, gpu, mid=True)
    errs = {"y": rel(y1, sy), "gx": rel(gx1, sgx)}
    for n in sgp:
        errs["grad/" + n] = rel(gp1[n], sgp[n].reshape(gp1[n].shape))
    scal = {"grad/" + n for n, p in blk.named_parameters() if p.numel() == 1}
    bad = {k: v for k, v in errs.items() if not v <= (2e-2 if k in scal else 1e-2)}
    print(shape, "strict", {k: f"{v:.2e}" for k, v in errs.items()})
    assert not bad, bad
    if shape[2] * shape[3] * shape[4] <= 16 * 16 * 16:
        ly, lgx, lgp = _ref_loose(P, x, gy)
        y0, gx0, gp0 = _run(blk, x, gy, gpu, mid=False)
        loose = {"y": rel(y1, ly), "gx": rel(gx1, lgx), "y_vs_engines": rel(y1, y0), "gx_vs_engines": rel(gx1, gx0)}
        for n in lgp:
            if n not in {k[5:] for k in scal}:
                loose["grad/" + n] = rel(gp1[n], lgp[n])
                loose["grad_vs_engines/" + n] = rel(gp1[n], gp0[n])
        bad = {k: v for k, v in loose.items() if not v <= 3e-2}
        assert not bad, bad


@pytest.mark.parametrize("half", HALF)
def test_fused_mid_block_deterministic(gpu, half):
    """Two backward passes give bit-identical gradients (fixed-order partial reductions)."""
    _H[0] = half
    blk = _block(seed=3)
    g = torch.Generator().manual_seed(5)
    shape = (1, 18, 32, 32, 16)
    x = rnd(torch.randn(shape, generator=g))
    gy = rnd(torch.randn(shape, generator=g))
    a = _run(blk, x, gy, gpu, mid=True)
    b = _run(blk, x, gy, gpu, mid=True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    for n in a[2]:
        assert torch.equal(a[2][n], b[2][n]), n


@pytest.mark.parametrize("shape", [(2, 18, 16, 8, 16), (1, 18, 128, 128, 32)])
@pytest.mark.parametrize("half", HALF)
def test_fused_mid_block_side_stream(gpu, shape, half):
    """Weight-gradient stages on the side stream (the product's concurrent mode) give the same
    bits as the single-stream backward."""
    _H[0] = half
    from vq3d import ops
    blk = _block(seed=9)
    g = torch.Generator().manual_seed(13)
    x = rnd(torch.randn(shape, generator=g))
    gy = rnd(torch.randn(shape, generator=g))
    a = _run(blk, x, gy, gpu, mid=True)
    ops.set_concurrent_wgrad(True)
    try:
        b = _run(blk, x, gy, gpu, mid=True)
    finally:
        ops.set_concurrent_wgrad(False)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    for n in a[2]:
        assert torch.equal(a[2][n], b[2][n]), n


def _poison():
    from vq3d import _lib as L
    L.call("vq3d_poison_lds", L.stream())


def _run_chain(blocks, x, gy, gpu, chained, concurrent=False, poison=False):
    """A run of blocks through layers.BlockStack (chained: Fn.PreActMidRunFn) or block by block
    (Fn.PreActBlockFn); returns out, gx and every parameter gradient, all as float64 on the CPU."""
    from vq3d import functional as Fn, ops
    from vq3d import layers as VL
    stack = VL.BlockStack(*[b for b in blocks]).to(gpu)
    for p in stack.parameters():
        p.grad = None
    xd = x.to(gpu).to(_H[0]).contiguous(memory_format=CL).requires_grad_(True)
    ops.set_concurrent_wgrad(concurrent)
    try:
        if poison:
            _poison()
        if chained:
            out = stack(xd)
        else:
            out = xd
            for b in stack:
                out = Fn.PreActBlockFn.apply(out, b, *b._fn_params)
        gyd = gy.to(gpu).to(_H[0]).contiguous(memory_format=CL)
        if poison:
            _poison()
        out.backward(gyd)
        ops.join_side()
    finally:
        ops.set_concurrent_wgrad(False)
    torch.cuda.synchronize()
    grads = {n: p.grad.double().cpu().clone() for n, p in stack.named_parameters()}
    return out.double().cpu(), xd.grad.double().cpu(), grads


@pytest.mark.parametrize("shape,nblk,concurrent", [((2, 18, 16, 8, 16), 4, False), ((1, 18, 32, 16, 16), 3, True),
                                                   ((1, 18, 128, 128, 32), 3, False)])
@pytest.mark.parametrize("half", HALF)
def test_mid_run_chain_matches_per_block(gpu, shape, nblk, concurrent, half):
    """The chained run (next block's t2 in the forward tile epilogue, previous block's gz3 in the
    backward tile epilogue) against the same blocks run one by one: out, gx and every gradient
    within 1e-2 of its max -- the chained t2 / gz3 are matrix-core sums of the same bf16 operands
    the per-block pointwise kernels sum on the VALU, so an odd bf16 rounding may land one ulp
    apart, and the run carries its stream in fp32 between the blocks where the one-by-one blocks
    round it to 16 bits.  The scalar biases / scales of a block compare as one vector (a lone
    scalar gradient is a sum of ~10^5 nearly cancelling terms: bias1b measured 1.1 % apart alone)."""
    _H[0] = half
    blocks = [_block(seed=20 + i) for i in range(nblk)]
    g = torch.Generator().manual_seed(21)
    x = rnd(torch.randn(shape, generator=g))
    gy = rnd(torch.randn(shape, generator=g))
    a = _run_chain(blocks, x, gy, gpu, chained=False)
    b = _run_chain(blocks, x, gy, gpu, chained=True, concurrent=concurrent)
    assert rel(b[0], a[0]) <= 1e-2, rel(b[0], a[0])
    assert rel(b[1], a[1]) <= 1e-2, rel(b[1], a[1])
    scal = {}
    for n in a[2]:
        if a[2][n].numel() > 1:
            assert rel(b[2][n], a[2][n]) <= 1e-2, (n, rel(b[2][n], a[2][n]))
        else:
            blk = n.split(".")[0]
            scal.setdefault(blk, ([], []))
            scal[blk][0].append(b[2][n].reshape(-1))
            scal[blk][1].append(a[2][n].reshape(-1))
    errs = {k: rel(torch.cat(u), torch.cat(v)) for k, (u, v) in scal.items()}
    print(shape, nblk, half, "scalar groups", {k: f"{e:.1e}" for k, e in errs.items()})
    assert max(errs.values()) <= 1e-2, errs


@pytest.mark.parametrize("shape", [(2, 18, 16, 8, 16), (1, 18, 128, 128, 32)])
@pytest.mark.parametrize("half", HALF)
def test_mid_run_chain_ignores_stale_lds(gpu, shape, half):
    """Regression: the chained forward's next-block t2 stage read K entries past a voxel's 18
    channels from LDS another wave had not written yet and multiplied them by zero weights; LDS
    left holding a NaN pattern by an earlier kernel turned into NaN activations (the 3-layer
    bench step went NaN after ~10 steps).  With every CU's LDS filled with NaN before the forward
    and before the backward the run must give the same bits as without."""
    _H[0] = half
    blocks = [_block(seed=40 + i) for i in range(3)]
    g = torch.Generator().manual_seed(41)
    x = rnd(torch.randn(shape, generator=g))
    gy = rnd(torch.randn(shape, generator=g))
    a = _run_chain(blocks, x, gy, gpu, chained=True)
    b = _run_chain(blocks, x, gy, gpu, chained=True, poison=True)
    assert torch.isfinite(b[0]).all() and torch.isfinite(b[1]).all()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    for n in a[2]:
        assert torch.equal(a[2][n], b[2][n]), n


@pytest.mark.parametrize("shape,nblk", [((2, 18, 16, 8, 16), 4), ((1, 18, 128, 128, 32), 5)])
@pytest.mark.parametrize("half", HALF)
def test_mid_run_batched_wgrad_bitwise(gpu, shape, nblk, half):
    """The run's weight gradients as one launch per kind after the data chain
    (vq3d_preact_mid_wgrad_run, the default) against the per-block stages 4 | 8 between the data
    kernels: the same workgroups and arithmetic per block, so out, gx and every gradient are equal
    bit for bit (the fixed-order reduction sums the same partial rows)."""
    from vq3d import ops
    _H[0] = half
    blocks = [_block(seed=60 + i) for i in range(nblk)]
    g = torch.Generator().manual_seed(61)
    x = rnd(torch.randn(shape, generator=g))
    gy = rnd(torch.randn(shape, generator=g))
    ops.set_batched_wgrad(False)
    try:
        a = _run_chain(blocks, x, gy, gpu, chained=True)
    finally:
        ops.set_batched_wgrad(True)
    b = _run_chain(blocks, x, gy, gpu, chained=True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    for n in a[2]:
        assert torch.equal(a[2][n], b[2][n]), n
