"""The headline configuration itself (BASELINE.json configs[2] per GPU: 3-layer published model,
512 x 512 x 128, bf16) through size-independent properties, since the oracle cannot run a
whole step at this size in seconds:

* codebook search bit-exact at full size: every level's codes equal the C oracle's nearest
  codeword (oracle/vq_nearest.c, pinned by the reference's KATs) for the very z the HIP encoder
  produced (524,288 / 8,192 / 128 rows), and the commitment losses agree;
* one training step (forward, loss, backward, Adam) leaves a finite loss, finite gradients
  and finite parameters, and codes inside [0, K) with the reference's shapes.
"""
import numpy as np
import pytest
import torch

from oracle import vq_oracle

pytestmark = pytest.mark.gpu

PUB = dict(n_bottleneck_blocks=3, n_pre_quantization_blocks=50, n_post_quantization_blocks=50,
           n_post_upscale_blocks=3, n_post_downscale_blocks=2, num_embeddings=[128, 256, 512])
SHAPES = [(1, 128, 128, 32), (1, 32, 32, 8), (1, 8, 8, 2)]


def _model(dev):
    import vq3d
    torch.manual_seed(0)
    return vq3d.VQVAE(vq3d.default_args(compute_dtype="bf16", **PUB)).to(dev)


def test_fullsize_codes_bitexact_vs_oracle(gpu):
    from vq3d.extract import extract_samples
    from vq3d.utils import synthetic_volume
    m = _model(gpu)
    zs = {}
    hooks = [q.register_forward_pre_hook(lambda mod, inp, i=i: zs.__setitem__(i, inp[0].detach()))
             for i, q in enumerate(m.encoder.quantize)]
    losses = {}
    m.eval()
    x = synthetic_volume((1, 1, 512, 512, 128), 0).to(gpu)
    with torch.no_grad():
        for lvl, (c, _, _) in enumerate(m.encode(x)):
            losses[lvl] = float(c)
    idxs = next(extract_samples(m, [x]))
    for h in hooks:
        h.remove()
    for lvl, q in enumerate(m.encoder.quantize):
        ix = idxs[lvl]
        assert tuple(ix.shape) == SHAPES[lvl] and ix.dtype == torch.int64
        z = zs[lvl].float().permute(0, 2, 3, 4, 1).reshape(-1, q.embedding_dim).cpu().numpy()
        ref_idx, _, sq = vq_oracle.nearest(z, q.embed.cpu().numpy())
        assert np.array_equal(ix.reshape(-1).cpu().numpy(), ref_idx), lvl
        ref_loss = q.commitment_cost * sq / z.size
        assert abs(losses[lvl] - ref_loss) <= 1e-4 * abs(ref_loss) + 1e-12, (lvl, losses[lvl], ref_loss)


def test_fullsize_train_step_finite(gpu):
    from vq3d.utils import synthetic_volume
    m = _model(gpu)
    opt = m.configure_optimizers()
    x = synthetic_volume((1, 1, 512, 512, 128), 0).to(gpu)
    nvs = torch.tensor([128], device=gpu)
    m.train()
    cap = {}
    fwd = m.forward

    def capture(data):
        cap["r"] = fwd(data)
        return cap["r"]
    m.forward = capture
    loss = m.training_step((x, nvs), 0)
    del m.forward
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    assert np.isfinite(float(loss))
    assert torch.isfinite(m.flat.grad).all() and float(m.flat.grad.abs().max()) > 0
    assert torch.isfinite(m.flat.data).all()
    _, (_, _, idxs) = cap["r"]
    for lvl, (ix, k) in enumerate(zip(idxs, PUB["num_embeddings"])):
        assert tuple(ix.shape) == SHAPES[lvl]
        assert int(ix.min()) >= 0 and int(ix.max()) < k
    for q in m.encoder.quantize:  # first pass done: codebook initialised from the data statistics
        assert int(q.first_pass) == 0 and torch.isfinite(q.embed).all()


def test_fullsize_multistep_graph_replay(gpu):
    """25 training steps of the headline configuration the way bench.py runs them (2 eager steps,
    then one HIP graph of the whole step -- forward, loss, backward, Adam -- replayed): loss,
    gradients, parameters and codebooks finite after EVERY step, codes in range every step, and
    a falling loss over the window (least-squares slope < 0, last five below the first five).
    The round-3 NaN (stale LDS x zero weight) appeared only after ~10 replayed steps."""
    from vq3d.graph import StepGraph
    from vq3d.utils import synthetic_volume
    m = _model(gpu)
    opt = m.configure_optimizers()
    x = synthetic_volume((1, 1, 512, 512, 128), 0).to(gpu)
    nvs = torch.tensor([128], device=gpu)
    m.train()
    cap = {}
    fwd = m.forward

    def capture(data):
        cap["r"] = fwd(data)
        return cap["r"]
    m.forward = capture

    def step(xx, nn):
        opt.zero_grad()
        loss = m.training_step((xx, nn), 0)
        loss.backward()
        opt.step()
        return loss
    sg = StepGraph(step, warmup=2)
    losses = []
    for i in range(25):
        loss = sg(x, nvs)
        torch.cuda.synchronize()
        lv = float(loss)
        losses.append(lv)
        assert np.isfinite(lv), (i, losses)
        assert bool(torch.isfinite(m.flat.grad).all()), i
        assert bool(torch.isfinite(m.flat.data).all()), i
        _, (_, _, idxs) = cap["r"]
        for lvl, (ix, k) in enumerate(zip(idxs, PUB["num_embeddings"])):
            assert tuple(ix.shape) == SHAPES[lvl]
            assert int(ix.min()) >= 0 and int(ix.max()) < k, (i, lvl)
        for q in m.encoder.quantize:
            assert bool(torch.isfinite(q.embed).all()), i
    del m.forward
    assert len(sg.graphs) == 1  # steps 3.. were graph replays
    slope = np.polyfit(np.arange(len(losses)), np.array(losses), 1)[0]
    print("losses", [round(v, 5) for v in losses], "slope", slope)
    assert slope < 0, losses
    assert np.mean(losses[-5:]) < np.mean(losses[:5]), losses


# ---------------------------------------------------------------------------------------- cfg2
# BASELINE.json configs[1]: the 2-layer published model (150 pre-q / 150 post-q / 5 post-up /
# 5 post-down, K = 128 / 256; slurm-jobs/train_vqvae_3d_downscaled.job) on 256 x 256 x 128
# volumes, batch 2, bf16.
PUB2 = dict(n_bottleneck_blocks=2, n_pre_quantization_blocks=150, n_post_quantization_blocks=150,
            n_post_upscale_blocks=5, n_post_downscale_blocks=5, num_embeddings=[128, 256])
SHAPES2 = [(2, 64, 64, 32), (2, 16, 16, 8)]


def test_cfg2_train_step_and_codes_bitexact(gpu):
    """One batch-2 training step (finite loss / grads / params, in-range codes), then the eval
    encode of the same batch: every level's codes equal the C oracle's nearest codeword for
    the z the HIP encoder produced (bit-exact), commitment losses within 1e-4."""
    import vq3d
    from vq3d.utils import synthetic_volume
    torch.manual_seed(0)
    m = vq3d.VQVAE(vq3d.default_args(compute_dtype="bf16", **PUB2)).to(gpu)
    opt = m.configure_optimizers()
    x = torch.cat([synthetic_volume((1, 1, 256, 256, 128), i) for i in range(2)]).to(gpu)
    nvs = torch.tensor([128, 128], device=gpu)
    m.train()
    opt.zero_grad()
    loss = m.training_step((x, nvs), 0)
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    assert np.isfinite(float(loss))
    assert torch.isfinite(m.flat.grad).all() and float(m.flat.grad.abs().max()) > 0
    assert torch.isfinite(m.flat.data).all()
    zs = {}
    hooks = [q.register_forward_pre_hook(lambda mod, inp, i=i: zs.__setitem__(i, inp[0].detach()))
             for i, q in enumerate(m.encoder.quantize)]
    m.eval()
    with torch.no_grad():
        res = list(m.encode(x))
    for h in hooks:
        h.remove()
    for lvl, (q, (c, _, ix)) in enumerate(zip(m.encoder.quantize, res)):
        assert tuple(ix.shape) == SHAPES2[lvl] and ix.dtype == torch.int64
        assert int(ix.min()) >= 0 and int(ix.max()) < PUB2["num_embeddings"][lvl]
        z = zs[lvl].float().permute(0, 2, 3, 4, 1).reshape(-1, q.embedding_dim).cpu().numpy()
        ref_idx, _, sq = vq_oracle.nearest(z, q.embed.cpu().numpy())
        assert np.array_equal(ix.reshape(-1).cpu().numpy(), ref_idx), lvl
        ref_loss = q.commitment_cost * sq / z.size
        assert abs(float(c) - ref_loss) <= 1e-4 * abs(ref_loss) + 1e-12, (lvl, float(c), ref_loss)


def test_batched_encode_codes_equal_per_volume(gpu):
    """bench.py --encode-batch B: B volumes in one eval encode give every volume exactly the codes
    it gets alone (no op mixes volumes; the fused engines index the batch dimension)."""
    from vq3d.extract import extract_samples
    from vq3d.utils import synthetic_volume
    m = _model(gpu)
    m.eval()
    for q in m.encoder.quantize:
        q.first_pass.zero_()
        q.first_pass_host = False
    vols = [synthetic_volume((1, 1, 256, 256, 64), i).to(gpu) for i in range(3)]
    alone = [next(extract_samples(m, [v])) for v in vols]
    together = next(extract_samples(m, [torch.cat(vols)]))
    for lvl in range(3):
        for b in range(3):
            assert torch.equal(together[lvl][b], alone[b][lvl][0]), (lvl, b)
