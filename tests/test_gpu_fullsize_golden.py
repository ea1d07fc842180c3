"""The HEADLINE configuration pinned against the REFERENCE ITSELF at full size: one training
step of the published 3-layer model at 512 x 512 x 128 (vqvae/model.py:95-163;
slurm-jobs/train_vqvae_3d.job:76-86) on the GPU, bf16 (BASELINE's dtype) and fp16 (the
reference's own AMP format), against tests/golden/model_3l_pub_512.npz -- written by
tools/make_golden_fullsize.py, which imports /root/reference and runs the reference's own
VQVAE.training_step + backward in fp32 on this container's CPU from the same perturbed seed-0
weights (p += 0.02 randn, seed 1) and the same seed-1234 volume.

What the fixture holds and how it is compared (bounds below, stated with the measured values):
  * per-level code match, floored per dtype (bf16 >= 94 / 91 / 94 %, fp16 >= 99 / 99.5 / 100 %);
    codes are bit-exact given identical fp32 z (test_gpu_fullsize.py), so a mismatch is a z that
    16-bit rounding moved across a Voronoi boundary;
  * the loss and the three commitment losses (relative);
  * the decoded volume on the fixture's stride-8 lattice (relative MSE);
  * gradients: every parameter's norm (relative), the whole sampled gradient vector (relative L2
    and cosine), every weight tensor's sampled entries (relative L2 and cosine; tensors of more
    than 4,096 entries are represented by 512 seeded positions, so their error is an estimate),
    the scalar biases / scales per block stack as one vector;
  * fp32 (the north star's "code indices bit-exact vs reference"): the same forward in fp32 against
    the reference's codes, >= 99.9 % per level, and every differing row shown to be a Voronoi-boundary
    flip from the fixture's own Quantizer inputs z{lvl} and search codebooks cb{lvl} (measured r06:
    99.9994 / 100 / 100 %, 3 of 524,288 bottom rows, each within 0.55 of its z / codebook movement
    from the bisector; z within 7e-7 of the reference's, loss 7e-8 relative).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

PUB3 = dict(n_bottleneck_blocks=3, n_pre_quantization_blocks=50, n_post_quantization_blocks=50,
            n_post_upscale_blocks=3, n_post_downscale_blocks=2, num_embeddings=[128, 256, 512])
PATH = os.path.join(GOLDEN, "model_3l_pub_512.npz")
# per dtype: code floors (bottom, mid, top), (loss rel, commitment rel, decoded rel-MSE, sampled-
# gradient rel-L2 / cosine, per-tensor rel-L2 / cosine, scalar-group rel-L2, gradient-norm rel).
# Measured (r05): bf16 codes 94.70 / 92.00 / 95.31 %, loss 1.3e-3, decoded 7.7e-4, sampled gradient
# 2.46 % / 0.99976, worst tensor 0.387 / 0.990; fp16 codes 99.34 / 99.62 / 100 %, loss 2.8e-6, decoded
# 6.4e-6, sampled gradient 1.67 % / 0.99986, worst tensor 0.032 / 0.99995 (r06: libvq3d's zero fills as
# kernels; round 5, with hipMemsetAsync fills, 0.116 / 0.9956).  bf16's mid level sits
# below its 256^2 floor because 6 of the 128 top codes flip at this size and every mid voxel is
# conditioned on the top level's ST output through the UpBlock (two ResizeConvs + 3 + 3 blocks:
# a receptive field spanning most of the 32 x 32 x 8 mid grid); fp16 flips none.
BOUNDS = {"bf16": ((0.94, 0.91, 0.94), (1e-2, 5e-2, 1.5e-3, 0.04, 0.999, 0.5, 0.98, 0.1, 0.5)),
          "fp16": ((0.99, 0.995, 1.0), (2e-3, 1e-2, 2e-5, 0.025, 0.9998, 0.06, 0.999, 0.05, 0.06))}


def _perturb(m, seed=1, std=0.02):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for _, p in sorted(m.named_parameters()):
            p.add_(std * torch.randn(p.shape, generator=g))


@pytest.mark.parametrize("dt", ["bf16", "fp16"])
def test_published_model_fullsize_vs_reference(gpu, dt):
    import vq3d
    from vq3d.optim import GradScaler
    ref = np.load(PATH)
    size = tuple(int(v) for v in ref["size"])
    torch.manual_seed(0)
    m = vq3d.VQVAE(vq3d.default_args(compute_dtype=dt, base_lr=1e-4, **PUB3))
    _perturb(m)
    x = torch.rand((1, 1) + size, generator=torch.Generator().manual_seed(1234)) * 4.5 - 0.5
    m = m.to(gpu)
    m.train()
    opt = m.configure_optimizers()
    opt.zero_grad()
    cap = {}
    fwd = m.forward

    def capture(data):
        cap["r"] = fwd(data)
        return cap["r"]
    m.forward = capture
    loss = m.training_step((x.to(gpu), torch.tensor([size[2]])), 0)
    del m.forward
    scaler = GradScaler(gpu, init_scale=2.0 ** 16, enabled=dt == "fp16")
    scaler.scale(loss).backward()
    scaler.unscale_(opt)
    vq3d.ops.join_side()
    torch.cuda.synchronize()
    assert float(scaler.found_inf) == 0.0
    dec, (commit, _, idxs) = cap["r"]
    s = int(ref["dec_stride"])
    d_gpu = dec.detach()[0, 0, ::s, ::s, ::s].float().cpu().double()
    d_ref = torch.from_numpy(ref["dec"]).double()
    rmse = float(((d_gpu - d_ref) ** 2).sum() / (d_ref ** 2).sum())
    match = [float((a.cpu().numpy() == ref[f"idx{lvl}"]).mean()) for lvl, a in enumerate(idxs)]
    lr = abs(float(loss.detach()) - float(ref["loss"])) / abs(float(ref["loss"]))
    crel = max(abs(float(c) - float(ref[f"commit{lvl}"])) / abs(float(ref[f"commit{lvl}"]))
               for lvl, c in enumerate(commit))
    # gradients at the fixture's positions
    gs, rs, tensors, groups, norms = [], [], [], {}, []
    for n, p in m.named_parameters():
        g = p.grad.detach().reshape(-1).double().cpu()
        r = torch.from_numpy(ref[f"grad/{n}"]).double()
        rn = float(ref[f"gnorm/{n}"])
        if rn > 0 and g.numel() > 1:  # a lone scalar is a near-cancelling sum: no meaningful relative error
            norms.append((abs(float(g.norm()) - rn) / rn, n))
        if f"gpos/{n}" in ref:
            g = g[torch.from_numpy(ref[f"gpos/{n}"])]
        if float(r.norm()) == 0:
            continue
        gs.append(g)
        rs.append(r)
        if g.numel() > 1:
            tensors.append((float((g - r).norm() / r.norm()), float((g * r).sum() / (g.norm() * r.norm())), n))
        else:
            key = ".".join(n.split(".")[:3])
            groups.setdefault(key, ([], []))
            groups[key][0].append(g)
            groups[key][1].append(r)
    fg, fr = torch.cat(gs), torch.cat(rs)
    flat_rel = float((fg - fr).norm() / fr.norm())
    flat_cos = float((fg * fr).sum() / (fg.norm() * fr.norm()))
    # scalar groups of >= 2 entries (a lone scalar, e.g. decoder.out.bias, is a near-cancelling
    # sum over ~10^7 voxels: no meaningful relative error)
    scal = sorted(((float((torch.cat(a) - torch.cat(b)).norm() / torch.cat(b).norm()), k)
                   for k, (a, b) in groups.items() if len(a) > 1), reverse=True)
    worst_rel, worst_cos, worst_norm = max(tensors), min(tensors, key=lambda t: t[1]), max(norms)
    print(f"{dt} 3L-pub {size} vs the reference: loss gpu {float(loss):.6f} ref {float(ref['loss']):.6f} rel {lr:.2e}; "
          f"commitment worst rel {crel:.2e}; code match bottom/mid/top {match}; decoded rel-MSE (stride {s}) "
          f"{rmse:.2e}; sampled gradient rel-L2 {flat_rel:.3e} cosine {flat_cos:.6f}; worst tensor rel-L2 "
          f"{worst_rel[0]:.3f} ({worst_rel[2]}), worst cosine {worst_cos[1]:.4f} ({worst_cos[2]}); worst "
          f"gradient-norm rel {worst_norm[0]:.3f} ({worst_norm[1]}); worst scalar group {scal[0][0]:.3f} ({scal[0][1]})")
    floors, (b_loss, b_commit, b_mse, b_rel, b_cos, b_trel, b_tcos, b_scal, b_norm) = BOUNDS[dt]
    for lvl, (mm, fl) in enumerate(zip(match, floors)):
        assert mm >= fl, (lvl, mm)
    assert lr <= b_loss, lr
    assert crel <= b_commit, crel
    assert rmse <= b_mse, rmse
    assert flat_rel <= b_rel and flat_cos >= b_cos, (flat_rel, flat_cos)
    assert worst_rel[0] <= b_trel and worst_cos[1] >= b_tcos, (worst_rel, worst_cos)
    assert scal[0][0] <= b_scal, scal[0]
    assert worst_norm[0] <= b_norm, worst_norm


def _boundary_report(lvl, z_gpu, z_ref, cb_gpu, cb_ref, i_gpu, i_ref):
    """Every row whose code differs: the reference's z row's distance to the bisector of its own
    codeword and the GPU's (float64, |z - e_g|^2 - |z - e_r|^2 over 2 |e_r - e_g|) against how far
    the GPU's z row and codebook moved from the reference's.  A flip caused by summation order
    alone has boundary distance <= that movement; returns (rows, rows NOT explained, worst ratio)."""
    rows = np.nonzero(i_gpu != i_ref)[0]
    bad, worst = [], 0.0
    for r in rows:
        z, zg = z_ref[r].astype(np.float64), z_gpu[r].astype(np.float64)
        er, eg = cb_ref[i_ref[r]].astype(np.float64), cb_ref[i_gpu[r]].astype(np.float64)
        bdist = (((z - eg) ** 2).sum() - ((z - er) ** 2).sum()) / (2 * np.linalg.norm(er - eg))
        move = np.linalg.norm(zg - z) + max(np.linalg.norm(cb_gpu[i_ref[r]] - er), np.linalg.norm(cb_gpu[i_gpu[r]] - eg))
        ratio = bdist / max(move, 1e-30)
        worst = max(worst, ratio)
        if not bdist <= move:
            bad.append((int(r), float(bdist), float(move)))
    return len(rows), bad, worst


def test_published_model_fullsize_fp32_codes_vs_reference(gpu):
    """The north star's "code indices bit-exact vs reference" at the HEADLINE size, in fp32 (the
    only run where a code can differ by summation order alone): one training-mode forward of the
    published 3-layer model at 512 x 512 x 128 from the fixture's weights / volume.  Every level's
    codes match the reference's on >= 99.9 % of the rows, and EVERY differing row is a Voronoi
    boundary case: the reference's own z row lies closer to the bisector between its codeword and
    the GPU's than the GPU's z row and codebook (first-pass init from the GPU's z statistics)
    moved from the reference's (fixture rows z{lvl} / cb{lvl}: the reference's Quantizer inputs and
    search codebook).  The loss within 1e-4 relative."""
    import vq3d
    ref = np.load(PATH)
    size = tuple(int(v) for v in ref["size"])
    torch.manual_seed(0)
    m = vq3d.VQVAE(vq3d.default_args(compute_dtype="fp32", base_lr=1e-4, **PUB3))
    _perturb(m)
    x = torch.rand((1, 1) + size, generator=torch.Generator().manual_seed(1234)) * 4.5 - 0.5
    m = m.to(gpu)
    m.train()
    qs = list(m.encoder.quantize)
    embed0 = [q.embed.detach().clone().double().cpu() for q in qs]
    zcap = {}

    def hook(mod, inp):
        z = inp[0].detach()
        zcap[id(mod)] = z.float().permute(0, 2, 3, 4, 1).reshape(-1, z.shape[1]).cpu().numpy()
    hs = [q.register_forward_pre_hook(hook) for q in qs]
    cap = {}
    fwd = m.forward

    def capture(data):
        cap["r"] = fwd(data)
        return cap["r"]
    m.forward = capture
    try:
        with torch.no_grad():
            loss = m.training_step((x.to(gpu), torch.tensor([size[2]])), 0)
        torch.cuda.synchronize()
    finally:
        del m.forward
        for h in hs:
            h.remove()
    _, (_, _, idxs) = cap["r"]
    lr = abs(float(loss) - float(ref["loss"])) / abs(float(ref["loss"]))
    lines = []
    for lvl, (q, a) in enumerate(zip(qs, idxs)):
        i_gpu = a.reshape(-1).cpu().numpy()
        i_ref = ref[f"idx{lvl}"].reshape(-1).astype(np.int64)
        z_gpu, z_ref, cb_ref = zcap[id(q)], ref[f"z{lvl}"], ref[f"cb{lvl}"]
        zt = torch.from_numpy(z_gpu).double()
        cb_gpu = (embed0[lvl] * zt.std(0) + zt.mean(0)).numpy()
        match = float((i_gpu == i_ref).mean())
        zrel = float(np.abs(z_gpu - z_ref).max() / np.abs(z_ref).max())
        n, bad, worst = _boundary_report(lvl, z_gpu, z_ref, cb_gpu, cb_ref, i_gpu, i_ref)
        lines.append((lvl, match, n, bad, worst, zrel))
        print(f"fp32 level {lvl}: codes match {match * 100:.4f} % ({n} of {i_ref.size} rows differ, "
              f"{len(bad)} not explained by the z / codebook movement; worst boundary-distance / movement "
              f"{worst:.3g}); z max |gpu - ref| / max |ref| {zrel:.2e}")
    print(f"fp32 loss gpu {float(loss):.7f} ref {float(ref['loss']):.7f} rel {lr:.2e}")
    assert lr <= 1e-4, lr
    for lvl, match, n, bad, worst, zrel in lines:
        assert match >= 0.999, (lvl, match)
        assert not bad, (lvl, bad[:10])
