"""Run-to-run determinism of the training step: two identically initialised
(perturbed) models take one training step (forward, loss, backward; level streams and side streams as in
the bench step) on the same volume, and every parameter gradient, the loss and the codes must be
equal BIT FOR BIT.  Every cross-workgroup sum in the step is a fixed-order partial reduction
(common.h `finish_partials`, the engines' `*_reduce` kernels), never a float atomic, so the
order of workgroup completion -- which varies run to run -- cannot change a gradient bit.

The reference (PyTorch + cuDNN under PL) makes no such promise; this is a property of this
build, stated in DESIGN.md 4.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

PUB = dict(n_bottleneck_blocks=3, n_pre_quantization_blocks=50, n_post_quantization_blocks=50,
           n_post_upscale_blocks=3, n_post_downscale_blocks=2, num_embeddings=[128, 256, 512])
TWO = dict(n_bottleneck_blocks=2, n_pre_quantization_blocks=2, n_post_quantization_blocks=2,
           n_post_upscale_blocks=1, n_post_downscale_blocks=1, num_embeddings=[64, 32])


def _step(gpu, dt, size, mkw):
    import vq3d
    from vq3d.utils import synthetic_volume
    torch.manual_seed(0)
    m = vq3d.VQVAE(vq3d.default_args(compute_dtype=dt, base_lr=1e-4, **mkw))
    # perturbed away from the Fixup init (whose zero last-conv weights and unit scales make many
    # gradients trivially reproducible: the scale gradient is a sum of W3 * G3 terms)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for _, p in sorted(m.named_parameters()):
            p.add_(0.02 * torch.randn(p.shape, generator=g))
    m = m.to(gpu)
    m.train()
    opt = m.configure_optimizers()
    opt.zero_grad()
    x = synthetic_volume((1, 1) + size, 3).to(gpu)
    cap = {}
    fwd = m.forward

    def capture(data):
        cap["r"] = fwd(data)
        return cap["r"]
    m.forward = capture
    loss = m.training_step((x, torch.tensor([size[2]])), 0)
    del m.forward
    loss.backward()
    vq3d.ops.join_side()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    codes = [c.detach().clone() for c in cap["r"][1][2]]
    return float(loss.detach()), codes, grads


@pytest.mark.parametrize("dt,size,cfg", [("bf16", (512, 512, 128), "pub3"), ("fp16", (512, 512, 128), "pub3"),
                                         ("bf16", (128, 128, 64), "pub3"), ("bf16", (64, 64, 32), "two")])
def test_train_step_bitwise_reproducible(gpu, dt, size, cfg):
    mkw = PUB if cfg == "pub3" else TWO
    l0, c0, g0 = _step(gpu, dt, size, mkw)
    l1, c1, g1 = _step(gpu, dt, size, mkw)
    assert all(torch.equal(a, b) for a, b in zip(c0, c1))
    diff = []
    for n in g0:
        a, b = g0[n], g1[n]
        if not torch.equal(a, b):
            d = float((a - b).abs().max() / a.abs().max().clamp_min(1e-30))
            diff.append((n, int((a != b).sum()), d))
    print(f"{dt} {cfg} {size}: loss {l0!r} / {l1!r}; {len(diff)} of {len(g0)} gradient tensors differ")
    for n, k, d in diff[:40]:
        print(f"  {n}: {k} entries, max rel {d:.2e}")
    assert l0 == l1
    assert not diff, diff[:10]


@pytest.mark.parametrize("size", [(128, 128, 64)])
def test_captured_step_replays_bitwise(gpu, size):
    """The bench's HIP-graph form of the step: one capture of forward + loss + backward (level and
    side streams as in bench.py, the gradient zero fill inside the graph; codebook EMA decay 1 so the
    in-graph update rewrites the same codebook), replayed three times -- the loss, every code and
    every parameter gradient equal BIT FOR BIT across the replays.  (A graph
    whose zero fills were hipMemsetAsync memset nodes replayed with different gradients on this
    ROCm; libvq3d's zero / copy are kernels, vq3d_zero / vq3d_copy.)"""
    import vq3d
    from vq3d.utils import synthetic_volume
    torch.manual_seed(0)
    m = vq3d.VQVAE(vq3d.default_args(compute_dtype="bf16", base_lr=1e-4, **PUB))
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for _, p in sorted(m.named_parameters()):
            p.add_(0.02 * torch.randn(p.shape, generator=g))
    m = m.to(gpu)
    m.train()
    opt = m.configure_optimizers()
    x = synthetic_volume((1, 1) + size, 3).to(gpu)
    nvs = torch.tensor([size[2]], device=gpu)
    cap = {}
    fwd = m.forward

    def capture(data):
        cap["r"] = fwd(data)
        return cap["r"]
    m.forward = capture

    def step():
        opt.zero_grad()
        loss = m.training_step((x, nvs), 0)
        loss.backward()
        vq3d.ops.join_side()
        return loss
    for _ in range(2):  # eager warm-up (the codebooks' first-pass init happens here)
        step()
    # EMA decay 1 from here on: the codebook update inside the graph then rewrites the same codebook
    # every replay, so replays must agree (with 0.99 each replay moves the codebook)
    for q in m.encoder.quantize:
        q.decay = 1.0
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        static = step()
    runs = []
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        runs.append((float(static), [c.detach().clone() for c in cap["r"][1][2]],
                     [p.grad.detach().clone() for p in m.parameters()]))
    del m.forward
    names = [n for n, _ in m.named_parameters()]
    for r in runs[1:]:
        assert r[0] == runs[0][0]
        assert all(torch.equal(a, b) for a, b in zip(r[1], runs[0][1]))
        bad = [n for n, a, b in zip(names, r[2], runs[0][2]) if not torch.equal(a, b)]
        assert not bad, bad[:10]
