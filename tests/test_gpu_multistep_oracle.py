"""Three chained training steps of the published 3-layer model at 128 x 128 x 64 against the fp32 CPU
oracle (oracle/vqvae_cpu.train_step, pinned to the reference by the golden tests) from the same
perturbed weights and volume: forward, backward, Adam (amsgrad) and the codebooks' first-pass init +
EMA update all carry over from step to step.  The model's own trajectory is not smooth -- Adam's
first step on the Fixup-initialised stack sends the loss from 1.6 to ~134 before it falls back (the
oracle shows the same: 1.611, 133.91, 13.33) -- so agreement through the spike is a strict check of
the whole update path.  Stated tolerance: each step's loss within 0.5 % (bf16) / 0.2 % (fp16) relative
(measured <= 0.1 % / 0.03 %)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

PUB3 = dict(n_bottleneck_blocks=3, n_pre_quantization_blocks=50, n_post_quantization_blocks=50,
            n_post_upscale_blocks=3, n_post_downscale_blocks=2, num_embeddings=[128, 256, 512])
SIZE = (128, 128, 64)
NSTEPS = 3
_REF = {}


def _model(dt="bf16"):
    import vq3d
    torch.manual_seed(0)
    m = vq3d.VQVAE(vq3d.default_args(base_lr=1e-4, compute_dtype=dt, **PUB3))
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for _, q in sorted(m.named_parameters()):
            q.add_(0.02 * torch.randn(q.shape, generator=g))
    return m


@pytest.mark.parametrize("dt,tol", [("bf16", 5e-3), ("fp16", 2e-3)])
def test_three_steps_track_oracle(gpu, dt, tol):
    from oracle import vqvae_cpu as O
    from vq3d import ops
    from vq3d.optim import GradScaler
    x = torch.rand((1, 1) + SIZE, generator=torch.Generator().manual_seed(2)) * 4.5 - 0.5
    if "ref" not in _REF:
        m0 = _model()
        sd = {k: v.detach().clone() for k, v in m0.state_dict().items()}
        st = {}
        torch.set_num_threads(min(16, torch.get_num_threads()))
        _REF["ref"] = [float(O.train_step(O.Config(**PUB3), sd, st, x, [SIZE[2]], 1e-4)[0]) for _ in range(NSTEPS)]
    ref = _REF["ref"]
    m = _model(dt).to(gpu)
    m.train()
    opt = m.configure_optimizers()
    scaler = GradScaler(gpu, enabled=dt == "fp16")
    xd = x.to(gpu)
    got = []
    for i in range(NSTEPS):
        opt.zero_grad()
        loss = m.training_step((xd, torch.tensor([SIZE[2]])), i)
        scaler.scale(loss).backward()
        ops.join_side()
        scaler.step(opt)
        scaler.update()
        torch.cuda.synchronize()
        got.append(float(loss.detach()))
    rels = [abs(a - b) / abs(b) for a, b in zip(got, ref)]
    print(f"{dt}: gpu losses {got}; oracle {ref}; rel {[f'{r:.1e}' for r in rels]}")
    assert all(r <= tol for r in rels), rels
