"""The torch.library binding (vq3d.library, SURVEY.md 8(b) "Binding"): training steps of a 2-layer
and of the published 3-layer model through `torch.ops.vq3d.*` equal the ctypes path's bit for bit --
loss, codes, every parameter gradient, and after the Adam step every parameter and codebook / EMA
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


@pytest.mark.parametrize("name", sorted(CFGS))
def test_library_step_bit_identical(gpu, name):
    import vq3d.library  # noqa: F401
    cfg, size = CFGS[name]
    a = _steps(gpu, "ctypes", cfg, size)
    b = _steps(gpu, "library", cfg, size)
    for step, (ra, rb) in enumerate(zip(a, b)):
        assert ra[0] == rb[0], (step, ra[0], rb[0])
        for ia, ib in zip(ra[1], rb[1]):
            assert torch.equal(ia, ib), step
        for n in ra[2]:
            assert torch.equal(ra[2][n], rb[2][n]), (step, "grad", n)
        for n in ra[3]:
            assert torch.equal(ra[3][n], rb[3][n]), (step, "state", n)
    print(name, "losses", [r[0] for r in a])


def test_library_ops_are_the_kernels(gpu):
    """A conv through torch.ops.vq3d.conv3d (+ its autograd backward) equals vq3d.functional.conv."""
    from vq3d import functional as Fn
    from vq3d import library as lb
    from vq3d.flat import FlatParams
    from vq3d.ops import ConvGeom
    torch.manual_seed(3)
    conv = torch.nn.Conv3d(8, 16, 3, padding=1, padding_mode="circular").to(gpu)
    FlatParams(conv.parameters(), gpu)
    x = torch.randn(1, 8, 16, 16, 16, device=gpu).bfloat16().contiguous(memory_format=torch.channels_last_3d)
    spec = Fn.ConvSpec(conv.weight, ConvGeom(3, 1, 1, True), cbias=conv.bias)
    out = []
    for path in (Fn.conv, lb.conv):
        conv.weight.grad.zero_()
        conv.bias.grad.zero_()
        xa = x.clone().requires_grad_(True)
        y = path(xa, spec)
        y.float().square().sum().backward()
        torch.cuda.synchronize()
        out.append((y.detach().clone(), xa.grad.clone(), conv.weight.grad.clone(), conv.bias.grad.clone()))
    for ta, tb in zip(*out):
        assert torch.equal(ta, tb)
