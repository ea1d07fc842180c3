"""The torch.library binding (vq3d.library, SURVEY.md 8(b) "Binding"): training steps of a 2-layer
and of the published 3-layer model through `torch.ops.vq3d.*` against the ctypes path -- loss,
codes, every parameter gradient, and after the Adam step every parameter and codebook / EMA
buffer.  Two steps each: the first runs the Quantizers' first-pass init (vq3d::vq_init), the second
the EMA path on initialised codebooks.  The 3-layer model at 128 x 128 x 64 exercises every fused
run engine (stack, wide, mid, small / column) through vq3d::preact_run and the single blocks / convs
of the down / up paths through vq3d::preact_block / vq3d::conv3d."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CFGS = {
    "2l": (dict(n_bottleneck_blocks=2, n_pre_quantization_blocks=2, n_post_quantization_blocks=2,
                n_post_upscale_blocks=2, n_post_downscale_blocks=2, num_embeddings=[128, 256]), (64, 64, 32)),
    "3l_pub": (dict(n_bottleneck_blocks=3, n_pre_quantization_blocks=50, n_post_quantization_blocks=50,
                    n_post_upscale_blocks=3, n_post_downscale_blocks=2, num_embeddings=[128, 256, 512]),
               (128, 128, 64)),
}


def _steps(gpu, binding, cfg, size, nsteps=2):
    import vq3d
    from vq3d import functional as Fn
    from vq3d import ops
    Fn.set_binding(binding)
    try:
        torch.manual_seed(0)
        m = vq3d.VQVAE(vq3d.default_args(base_lr=1e-4, **cfg))
        g = torch.Generator().manual_seed(1)
        with torch.no_grad():
            for _, p in sorted(m.named_parameters()):
                p.add_(0.02 * torch.randn(p.shape, generator=g))
        m = m.to(gpu)
        m.train()
        opt = m.configure_optimizers()
        x = (torch.rand((1, 1) + size, generator=torch.Generator().manual_seed(2)) * 4.5 - 0.5).to(gpu)
        rec = []
        for i in range(nsteps):
            opt.zero_grad()
            cap = {}
            fwd = m.forward

            def capture(data):
                cap["r"] = fwd(data)
                return cap["r"]
            m.forward = capture
            loss = m.training_step((x, torch.tensor([size[2]])), i)
            del m.forward
            loss.backward()
            ops.join_side()
            torch.cuda.synchronize()
            idxs = [t.cpu().clone() for t in cap["r"][1][2]]
            grads = {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}
            opt.step()
            torch.cuda.synchronize()
            state = {n: t.detach().cpu().clone() for n, t in m.state_dict().items()}
            rec.append((float(loss.detach()), idxs, grads, state))
        return rec
    finally:
        Fn.set_binding("ctypes")


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def _diff(ra, rb):
    """{name: relative max-abs difference} of the tensors of two step records that are not bitwise
    equal (loss and codes compare exactly: inf when they differ)"""
    out = {}
    for step, (x, y) in enumerate(zip(ra, rb)):
        if x[0] != y[0]:
            out[(step, "loss")] = float("inf")
        for i, (p, q) in enumerate(zip(x[1], y[1])):
            if not torch.equal(p, q):
                out[(step, "codes", i)] = float("inf")
        for k in (2, 3):
            for n in x[k]:
                if not torch.equal(x[k][n], y[k][n]):
                    out[(step, "grad" if k == 2 else "state", n)] = _rel(y[k][n], x[k][n])
    return out


@pytest.mark.parametrize("name", sorted(CFGS))
def test_library_step_matches_ctypes(gpu, name):
    """Every cross-workgroup sum of the step is a fixed-order reduction (no float atomics:
    tests/test_gpu_determinism.py), so the ctypes path reproduces itself bit for bit and the
    library binding -- the same kernels behind torch.ops.vq3d.* -- must equal it bit for bit: loss,
    codes, every gradient and every optimizer / Quantizer state tensor, on both steps."""
    import vq3d.library  # noqa: F401
    cfg, size = CFGS[name]
    a = _steps(gpu, "ctypes", cfg, size)
    a2 = _steps(gpu, "ctypes", cfg, size)
    b = _steps(gpu, "library", cfg, size)
    noise = _diff(a, a2)
    d = _diff(a, b)
    worst = max(d.items(), key=lambda kv: kv[1]) if d else None
    print(f"{name}: losses {[r[0] for r in a]}; ctypes run-to-run: {len(noise)} tensors differ; library vs "
          f"ctypes: {len(d)} differ, worst {worst}")
    assert not noise, sorted(noise.items())[:5]
    assert not d, worst


def test_library_ops_are_the_kernels(gpu):
    """A circular 3x3x3 conv through the library binding (lb.conv: the operator below the autograd
    key + its formula), and through torch.ops.vq3d.conv3d called directly under autograd (the
    register_autograd formula), against vq3d.functional.conv: output, input gradient and the weight / bias gradients bit for bit."""
    from vq3d import functional as Fn
    from vq3d import library as lb
    from vq3d.flat import FlatParams
    from vq3d.ops import ConvGeom
    torch.manual_seed(3)
    conv = torch.nn.Conv3d(8, 16, 3, padding=1, padding_mode="circular").to(gpu)
    FlatParams(conv.parameters(), gpu)
    x = torch.randn(1, 8, 16, 16, 16, device=gpu).bfloat16().contiguous(memory_format=torch.channels_last_3d)
    spec = Fn.ConvSpec(conv.weight, ConvGeom(3, 1, 1, True), cbias=conv.bias)
    def direct(xa, spec):  # the registered operator under autograd (torch.library.register_autograd)
        return torch.ops.vq3d.conv3d(xa, None, None, spec.w, None, None, spec.cbias, [], [3, 1, 1, 1], False, False,
                                     True)[0]
    out = []
    for path in (Fn.conv, lb.conv, direct):
        conv.weight.grad.zero_()
        conv.bias.grad.zero_()
        xa = x.clone().requires_grad_(True)
        y = path(xa, spec)
        y.float().square().sum().backward()
        torch.cuda.synchronize()
        out.append((y.detach().clone(), xa.grad.clone(), conv.weight.grad.clone(), conv.bias.grad.clone()))
    (ya, gxa, gwa, gba) = out[0]
    for yb, gxb, gwb, gbb in out[1:]:
        assert torch.equal(ya, yb)
        assert torch.equal(gxa, gxb)
        assert torch.equal(gwa, gwb) and torch.equal(gba, gbb), (_rel(gwb, gwa), _rel(gbb, gba))


def test_exported_block_operator_replays(gpu):
    """torch.export captures the vq3d::preact_block operator (its fake kernel propagates the
    shapes); the exported program, run on the GPU, gives the eager operator's output bit for bit."""
    from vq3d import layers as VL

    class Block(torch.nn.Module):
        def __init__(self, blk):
            super().__init__()
            self.blk = blk

        def forward(self, x):
            return torch.ops.vq3d.preact_block(x, list(self.blk._fn_params), self.blk.mode, False)[0]

    torch.manual_seed(0)
    blk = VL.PreActFixupResBlock(18, 18, mode="same")
    with torch.no_grad():
        for p in blk.parameters():
            p.add_(0.05 * torch.randn_like(p))
    m = Block(blk).to(gpu).eval()
    x = torch.randn(1, 18, 32, 32, 32, device=gpu).to(torch.bfloat16).contiguous(memory_format=torch.channels_last_3d)
    with torch.no_grad():
        ref = m(x).clone()
        ep = torch.export.export(m, (x,))
        got = ep.module()(x)
    torch.cuda.synchronize()
    calls = [n for n in ep.graph.nodes if n.op == "call_function" and "vq3d" in str(n.target)]
    assert len(calls) == 1 and "preact_block" in str(calls[0].target)
    assert torch.equal(got, ref)
