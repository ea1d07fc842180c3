#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by IMPORTING the reference.

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 \
    PYTHONPATH=tools/golden_stubs:/root/reference python tools/make_goldens.py

`tools/golden_stubs/` holds arithmetic-free stand-ins for pytorch_lightning /
monai / nrrd / lmdb (not installed offline); every number in
the fixtures comes from the reference's own modules running on this
container's CPU ATen (torch 2.10.0).  The fixtures are data only: inputs,
parameters and the reference's outputs / gradients, as .npz.
"""
import os
import sys
from argparse import Namespace

import numpy as np
import torch
import torch.nn.functional as F

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")

from vqvae import layers as L  # noqa: E402  (reference)
from vqvae import evonorm as EN  # noqa: E402  (reference)
from vqvae.model import VQVAE  # noqa: E402  (reference)

torch.set_num_threads(8)


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


def t2n(t):
    return t.detach().cpu().numpy()


def perturb_(module, seed=1, std=0.02):
    """p += std * randn so zero-initialised conv3 / gamma paths are exercised."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for _, p in sorted(module.named_parameters()):
            p.add_(std * torch.randn(p.shape, generator=g))


# ----------------------------------------------------------------------------------------
# A. VQ known-answer tests (Quantizer.forward in eval mode: cdist no-mm + argmin + ST + loss)
# ----------------------------------------------------------------------------------------

def f32_rule_dist(z, e):
    """numpy float32 restatement used ONLY to search for sqrt-rounding ties."""
    d = z.shape[-1]
    b = 4 * (d // 4)
    acc = np.zeros(np.broadcast(z[..., 0], e[..., 0]).shape, np.float32)
    for i in range(b):
        t = (z[..., i] - e[..., i]).astype(np.float32)
        acc = (acc + (t * t).astype(np.float32)).astype(np.float32)
    for i in range(b, d):
        t = (z[..., i] - e[..., i]).astype(np.float64)
        acc = (acc.astype(np.float64) + t * t).astype(np.float32)  # fma: exact product, one rounding
    return np.sqrt(acc, dtype=np.float32), acc


def ref_quantize_eval(z_nd, embed):
    """Run the reference Quantizer in eval mode on flat rows z (N, D)."""
    n, d = z_nd.shape
    k = embed.shape[0]
    q = L.Quantizer(num_embeddings=k, embedding_dim=d, commitment_cost=0.1)
    q.eval()
    with torch.no_grad():
        q.embed.copy_(torch.from_numpy(embed))
    # (1, D, N, 1, 1): channel-last flattening gives back rows in order
    inp = torch.from_numpy(z_nd.T.copy()).reshape(1, d, n, 1, 1).requires_grad_(True)
    loss, qst, idx = q(inp)
    gq = torch.from_numpy(np.random.default_rng(99).standard_normal(qst.shape).astype(np.float32))
    (loss * 1.7 + (qst * gq).sum()).backward()
    zst = t2n(qst).reshape(d, n).T
    gz = t2n(inp.grad).reshape(d, n).T
    dist = torch.cdist(torch.from_numpy(z_nd), torch.from_numpy(embed),
                       compute_mode='donot_use_mm_for_euclid_dist')
    return t2n(idx).reshape(n), zst, float(loss), t2n(gq).reshape(d, n).T, gz, t2n(dist)


def gen_vq_kats():
    rng = np.random.default_rng(1234)
    cases = {}
    # production (D, K) at reduced N
    for (d, k, n) in [(2, 128, 4096), (8, 256, 2048), (32, 512, 512)]:
        z = rng.standard_normal((n, d)).astype(np.float32) * 1.3
        e = rng.standard_normal((k, d)).astype(np.float32)
        cases[f"prod_d{d}_k{k}"] = (z, e)
    # odd embedding dims exercise the FMA tail (D mod 4)
    for d in [1, 3, 4, 5, 6, 7, 12, 13]:
        z = rng.standard_normal((512, d)).astype(np.float32)
        e = rng.standard_normal((64, d)).astype(np.float32)
        cases[f"dim_d{d}"] = (z, e)
    # value scales
    for s in [1e-3, 50.0]:
        z = (rng.standard_normal((1024, 8)) * s).astype(np.float32)
        e = (rng.standard_normal((128, 8)) * s).astype(np.float32)
        cases[f"scale_{s:g}"] = (z, e)
    # duplicate codewords + exact ties on a coarse grid
    e = (rng.integers(-3, 4, size=(64, 4)) * 0.5).astype(np.float32)
    e[10] = e[3]
    e[40] = e[3]
    e[63] = e[0]
    z = (rng.integers(-3, 4, size=(2048, 4)) * 0.25).astype(np.float32)
    z[:64] = e  # rows equal to (duplicated) codewords
    cases["ties_grid_d4"] = (z, e)
    e2 = (rng.integers(-2, 3, size=(32, 2)) * 1.0).astype(np.float32)
    z2 = (rng.integers(-4, 5, size=(2048, 2)) * 0.5).astype(np.float32)
    cases["ties_grid_d2"] = (z2, e2)
    # ties created only by sqrtf rounding: two codewords whose squared distances differ
    # in the last bit but round to the same sqrt
    found_z, found_e = [], []
    trials = 0
    while len(found_z) < 64 and trials < 200000:
        trials += 1
        d = 3
        z0 = rng.standard_normal(d).astype(np.float32)
        ea = (z0 + rng.standard_normal(d).astype(np.float32)).astype(np.float32)
        eb = ea.copy()
        j = rng.integers(0, d)
        eb[j] = np.nextafter(eb[j], np.float32(np.inf) if rng.random() < 0.5 else np.float32(-np.inf))
        (sa, aa) = f32_rule_dist(z0, ea)
        (sb, ab) = f32_rule_dist(z0, eb)
        if aa != ab and sa == sb:
            found_z.append(z0)
            found_e.append(np.stack([eb, ea] if ab > aa else [ea, eb]))
    zs = np.stack(found_z)
    # every row gets its own pair appended after a random background codebook
    bg = rng.standard_normal((16, 3)).astype(np.float32) * 4 + 8
    # place pairs as separate codebooks? keep one codebook: all pairs appended
    e_all = np.concatenate([bg] + [p for p in found_e], axis=0)
    cases["sqrt_ties_d3"] = (zs, e_all)
    print(f"sqrt-tie search: {len(found_z)} found in {trials} trials")

    out = {}
    for name, (z, e) in cases.items():
        idx, zst, loss, gq, gz, dist = ref_quantize_eval(z, e)
        out[f"{name}/z"] = z
        out[f"{name}/embed"] = e
        out[f"{name}/idx"] = idx.astype(np.int64)
        out[f"{name}/zst"] = zst
        out[f"{name}/loss"] = np.float32(loss)
        out[f"{name}/gq"] = gq
        out[f"{name}/gz"] = gz
        if name in ("dim_d1", "dim_d3", "dim_d5", "dim_d6", "sqrt_ties_d3", "ties_grid_d4"):
            out[f"{name}/dist"] = dist
    save("vq_kat", **out)


# ----------------------------------------------------------------------------------------
# B. Quantizer train mode: first pass (init EMA) + second pass (EMA update)
# ----------------------------------------------------------------------------------------

def gen_quantizer_train():
    out = {}
    for (k, d, shape) in [(128, 2, (2, 2, 16, 16, 8)), (256, 8, (1, 8, 8, 8, 4)), (512, 32, (1, 32, 4, 4, 2))]:
        torch.manual_seed(7 + k)
        q = L.Quantizer(num_embeddings=k, embedding_dim=d, commitment_cost=0.1)
        q.train()
        pre = f"k{k}_d{d}"
        out[f"{pre}/embed0"] = t2n(q.embed).copy()
        out[f"{pre}/embed_avg0"] = t2n(q.embed_avg).copy()
        out[f"{pre}/cluster_size0"] = t2n(q.cluster_size).copy()
        for step in range(2):
            g = torch.Generator().manual_seed(100 * step + k)
            x = (torch.randn(shape, generator=g) * (0.5 + step)).requires_grad_(True)
            loss, qst, idx = q(x)
            gq = torch.randn(qst.shape, generator=g)
            (loss * 2.0 + (qst * gq).sum()).backward()
            s = f"{pre}/step{step}"
            out[f"{s}/x"] = t2n(x)
            out[f"{s}/gq"] = t2n(gq)
            out[f"{s}/loss"] = np.float32(float(loss))
            out[f"{s}/qst"] = t2n(qst)
            out[f"{s}/idx"] = t2n(idx)
            out[f"{s}/gx"] = t2n(x.grad)
            out[f"{s}/embed"] = t2n(q.embed).copy()
            out[f"{s}/embed_avg"] = t2n(q.embed_avg).copy()
            out[f"{s}/cluster_size"] = t2n(q.cluster_size).copy()
            out[f"{s}/first_pass"] = t2n(q.first_pass).copy()
    save("quantizer_train", **out)


# ----------------------------------------------------------------------------------------
# C. Residual blocks / convs with perturbed weights: forward + all gradients
# ----------------------------------------------------------------------------------------

def run_module(name, module, x_shape, seed, out, extra_inputs=()):
    perturb_(module, seed=seed)
    g = torch.Generator().manual_seed(seed + 1000)
    x = torch.randn(x_shape, generator=g).requires_grad_(True)
    y = module(x)
    gy = torch.randn(y.shape, generator=g)
    (y * gy).sum().backward()
    out[f"{name}/x"] = t2n(x)
    out[f"{name}/y"] = t2n(y)
    out[f"{name}/gy"] = t2n(gy)
    out[f"{name}/gx"] = t2n(x.grad)
    for pn, p in module.named_parameters():
        out[f"{name}/param/{pn}"] = t2n(p)
        out[f"{name}/grad/{pn}"] = t2n(p.grad)


def gen_blocks():
    out = {}
    seed = 10
    # pre-activation Fixup blocks (the published block type)
    cfgs = [
        ("preact_same_4_4", L.PreActFixupResBlock, 4, 4, "same", (2, 4, 6, 8, 4)),
        ("preact_same_4_8", L.PreActFixupResBlock, 4, 8, "same", (1, 4, 6, 8, 4)),
        ("preact_same_2_2", L.PreActFixupResBlock, 2, 2, "same", (1, 2, 8, 8, 4)),
        ("preact_same_9_9_d2", L.PreActFixupResBlock, 9, 9, "same", (1, 9, 4, 4, 2)),
        ("preact_same_18_2", L.PreActFixupResBlock, 18, 2, "same", (1, 18, 4, 4, 4)),
        ("preact_out_4_1", L.PreActFixupResBlock, 4, 1, "out", (1, 4, 4, 4, 4)),
        ("preact_down_4_8", L.PreActFixupResBlock, 4, 8, "down", (2, 4, 8, 8, 4)),
        ("preact_down_8_16_d4", L.PreActFixupResBlock, 8, 16, "down", (1, 8, 8, 4, 4)),
        ("preact_up_8_4", L.PreActFixupResBlock, 8, 4, "up", (1, 8, 4, 4, 2)),
        ("preact_up_16_8", L.PreActFixupResBlock, 16, 8, "up", (2, 16, 2, 4, 2)),
        ("preact_up_2_1", L.PreActFixupResBlock, 2, 1, "up", (1, 2, 4, 4, 2)),
        # regular Fixup blocks (zero padding, post-activation)
        ("regular_same_4_4", L.FixupResBlock, 4, 4, "same", (2, 4, 6, 6, 4)),
        ("regular_down_4_8", L.FixupResBlock, 4, 8, "down", (1, 4, 8, 8, 4)),
        ("regular_up_8_4", L.FixupResBlock, 8, 4, "up", (1, 8, 4, 4, 2)),
        ("regular_out_4_2", L.FixupResBlock, 4, 2, "out", (1, 4, 4, 4, 4)),
        # EvoNorm-S0 blocks (batch 1 only)
        ("evonorm_same_8_8", L.EvonormResBlock, 8, 8, "same", (1, 8, 6, 6, 4)),
        ("evonorm_same_16_8", L.EvonormResBlock, 16, 8, "same", (1, 16, 4, 4, 4)),
        ("evonorm_down_8_16", L.EvonormResBlock, 8, 16, "down", (1, 8, 8, 8, 4)),
        ("evonorm_up_16_8", L.EvonormResBlock, 16, 8, "up", (1, 16, 4, 4, 2)),
    ]
    for name, cls, cin, cout, mode, xs in cfgs:
        torch.manual_seed(seed)
        m = cls(cin, cout, mode=mode)
        if hasattr(m, "initialize_weights") and cls is not L.EvonormResBlock:
            m.initialize_weights(num_layers=7)
        run_module(name, m, xs, seed, out)
        out[f"{name}/meta"] = np.array([cin, cout, ["down", "same", "up", "out"].index(mode)])
        seed += 1
    # single ops
    ops = [
        ("conv3_circ_5_3_d2", torch.nn.Conv3d(5, 3, 3, 1, 1, bias=False, padding_mode='circular'), (1, 5, 4, 3, 2)),
        ("conv4s2_circ_3_6", torch.nn.Conv3d(3, 6, 4, 2, 1, bias=False, padding_mode='circular'), (2, 3, 8, 4, 2)),
        ("conv2s2_4_8", torch.nn.Conv3d(4, 8, 2, 2, 0, bias=False), (1, 4, 6, 4, 8)),
        ("conv1_bias_3_5", torch.nn.Conv3d(3, 5, 1), (2, 3, 4, 5, 3)),
        ("resize3_circ_3_4", L.ResizeConv3D(3, 4, 3, 1, 1, bias=False, padding_mode='circular'), (1, 3, 3, 2, 2)),
        ("resize1_4_2", L.ResizeConv3D(4, 2, 1, 1, 0, bias=False), (2, 4, 2, 3, 2)),
        ("upsample_tri", torch.nn.Upsample(mode='trilinear', scale_factor=2, align_corners=False), (1, 3, 3, 4, 5)),
        ("conv3_zero_bias_4_4", torch.nn.Conv3d(4, 4, 3, 1, 1), (1, 4, 5, 4, 3)),
        ("conv4s2_zero_4_4", torch.nn.Conv3d(4, 4, 4, 2, 1), (1, 4, 8, 6, 4)),
    ]
    for name, m, xs in ops:
        torch.manual_seed(seed)
        m = m
        run_module(name, m, xs, seed, out)
        seed += 1
    # EvoNorm3DS0 alone (B = 1)
    torch.manual_seed(seed)
    en = EN.EvoNorm3DS0(16)
    run_module("evonorm_s0_16", en, (1, 16, 4, 6, 4), seed, out)
    save("blocks", **out)


# ----------------------------------------------------------------------------------------
# D. Reconstruction loss (VQVAE.huber -> loc_metric) on a fixed decoder output
# ----------------------------------------------------------------------------------------

def model_args(**kw):
    a = dict(input_channels=1, base_network_channels=4, n_bottleneck_blocks=2,
             n_downscales_per_bottleneck=2, n_pre_quantization_blocks=0,
             n_post_quantization_blocks=0, n_post_upscale_blocks=0, n_post_downscale_blocks=0,
             num_embeddings=[256], block_type='pre-activation', extract_center_cylinder=True,
             metric='huber', base_lr=1e-5, n_mix=2)
    a.update(kw)
    return Namespace(**a)


def gen_loss():
    out = {}
    for i, (shape, nvs, cyl) in enumerate([((2, 1, 12, 10, 6), [6, 4], True),
                                          ((1, 1, 16, 16, 8), [5], True),
                                          ((2, 1, 8, 8, 4), [4, 2], False)]):
        torch.manual_seed(50 + i)
        m = VQVAE(model_args(extract_center_cylinder=cyl))
        g = torch.Generator().manual_seed(60 + i)
        x = torch.rand(shape, generator=g) * 4.5 - 0.5
        dec = (torch.randn(shape, generator=g) * 1.5).requires_grad_(True)
        commit = [torch.tensor(0.25, requires_grad=True), torch.tensor(0.125, requires_grad=True)]
        m.forward = lambda data, dec=dec, commit=commit: (dec, (tuple(commit), None, None))
        loss, _ = m.huber((x, torch.tensor(nvs)), 0)
        loss.backward()
        p = f"case{i}"
        out[f"{p}/x"] = t2n(x)
        out[f"{p}/dec"] = t2n(dec)
        out[f"{p}/nvs"] = np.array(nvs, np.int64)
        out[f"{p}/cyl"] = np.int64(cyl)
        out[f"{p}/commit"] = np.array([0.25, 0.125], np.float32)
        out[f"{p}/loss"] = np.float32(float(loss))
        out[f"{p}/gdec"] = t2n(dec.grad)
    # the disc used by ExtractCenterCylinder at 512 x 512 (count pinned by SURVEY.md: 205,859)
    from utils import ExtractCenterCylinder
    out["mask512"] = np.packbits(t2n(ExtractCenterCylinder.create_cylinder_xy_mask((512, 512))))
    out["mask12x10"] = t2n(ExtractCenterCylinder.create_cylinder_xy_mask((12, 10)))
    save("loss", **out)


# ----------------------------------------------------------------------------------------
# E. Whole model: one training step (train-mode EMA incl. first pass) + Adam(amsgrad) step
# ----------------------------------------------------------------------------------------

def gen_model(name, args, x_shape, nvs, lr=1e-3, steps=2, keep_state=True, keep_grads=True,
              dec_stride=1):
    """Train-mode steps of the reference VQVAE: training_step + backward + Adam(amsgrad).

    Inputs are NOT stored: x_step = torch.rand(x_shape, generator=Generator().manual_seed(1234 + step))
    * 4.5 - 0.5 (torch's CPU generator is deterministic; tests regenerate it the same way).
    """
    torch.manual_seed(0)
    m = VQVAE(args)
    perturb_(m, seed=1)
    m.lr = lr
    opt = m.configure_optimizers()
    out = {"x_shape": np.array(x_shape), "nvs": np.array(nvs), "lr": np.float32(lr),
           "dec_stride": np.int64(dec_stride)}
    for pn, p in m.state_dict().items():
        out[f"init/{pn}"] = t2n(p).copy()
    for step in range(steps):
        g = torch.Generator().manual_seed(1234 + step)
        x = torch.rand(x_shape, generator=g) * 4.5 - 0.5
        m.train()
        opt.zero_grad()
        # wrap forward to capture decoded / codes of the same call training_step makes
        cap = {}
        fwd = m.forward

        def capture(data, fwd=fwd, cap=cap):
            r = fwd(data)
            cap["r"] = r
            return r
        m.forward = capture
        loss = m.training_step((x, torch.tensor(nvs)), step)
        m.forward = fwd
        dec, (commit, qst, idx) = cap["r"]
        s = dec_stride
        out[f"step{step}/dec"] = t2n(dec)[..., ::s, ::s, ::s]
        for lvl, ix in enumerate(idx):
            out[f"step{step}/idx{lvl}"] = t2n(ix).astype(np.int16)
        for lvl, c in enumerate(commit):
            out[f"step{step}/commit{lvl}"] = np.float32(float(c))
        loss.backward()
        out[f"step{step}/loss"] = np.float32(float(loss))
        if keep_grads and step == 0:
            for pn, p in m.named_parameters():
                out[f"step{step}/grad/{pn}"] = t2n(p.grad).copy()
        opt.step()
        for pn, p in m.state_dict().items():
            if keep_state and step == 0 or not p.dtype.is_floating_point or "quantize" in pn:
                out[f"step{step}/state/{pn}"] = t2n(p).copy()
    save(name, **out)


# ----------------------------------------------------------------------------------------
# F. 2-rank gloo: the Quantizer's distributed EMA (all_reduce sites layers.py:645-647,670-676)
# ----------------------------------------------------------------------------------------

def _ema_rank(rank, world, port, path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(3)  # identical codebook init on every rank
    q = L.Quantizer(num_embeddings=64, embedding_dim=4, commitment_cost=0.1)
    q.train()
    res = {"embed0": t2n(q.embed).copy()}
    for step in range(2):
        g = torch.Generator().manual_seed(500 + 10 * step + rank)
        x = torch.randn((1, 4, 8, 4, 4), generator=g) * (1.0 + rank)
        loss, qst, idx = q(x)
        res[f"step{step}/x"] = t2n(x)
        res[f"step{step}/idx"] = t2n(idx)
        res[f"step{step}/loss"] = np.float32(float(loss))
        for b in ("embed", "embed_avg", "cluster_size"):
            res[f"step{step}/{b}"] = t2n(getattr(q, b)).copy()
    np.savez(path + f".rank{rank}.npz", **res)
    dist.destroy_process_group()


def gen_ema_dist():
    import tempfile
    import torch.multiprocessing as mp
    tmp = tempfile.mkdtemp()
    path = os.path.join(tmp, "ema")
    mp.spawn(_ema_rank, args=(2, 29517, path), nprocs=2, join=True)
    out = {}
    for r in range(2):
        d = np.load(path + f".rank{r}.npz")
        for k in d.files:
            out[f"rank{r}/{k}"] = d[k]
    save("ema_dist2", **out)


# ----------------------------------------------------------------------------------------
# G. Encode-only extraction (extract_embeddings.py:16-23): eval mode, no_grad, batch 1,
#    codes per level bottom -> top, from a model whose codebooks went through one EMA step
# ----------------------------------------------------------------------------------------

def gen_encode(name, args, x_shape, n_samples=2):
    """State after one reference train step (first pass + EMA done), then model.eval() and
    `*_, idx = zip(*model.encode(x))` for n_samples volumes x_i = rand(seed 5000 + i) * 4.5 - 0.5."""
    torch.manual_seed(0)
    m = VQVAE(args)
    perturb_(m, seed=1)
    opt = m.configure_optimizers()
    g = torch.Generator().manual_seed(1234)
    x = torch.rand(x_shape, generator=g) * 4.5 - 0.5
    m.train()
    loss = m.training_step((x, torch.tensor([x_shape[-1]] * x_shape[0])), 0)
    loss.backward()
    opt.step()
    out = {"x_shape": np.array((1,) + tuple(x_shape[1:])), "n_samples": np.int64(n_samples)}
    for pn, p in m.state_dict().items():
        out[f"state/{pn}"] = t2n(p).copy()
    m.eval()
    with torch.no_grad():
        for i in range(n_samples):
            gi = torch.Generator().manual_seed(5000 + i)
            xi = torch.rand((1,) + tuple(x_shape[1:]), generator=gi) * 4.5 - 0.5
            losses, qsts, idxs = zip(*m.encode(xi))
            for lvl, (c, q, ix) in enumerate(zip(losses, qsts, idxs)):
                out[f"sample{i}/idx{lvl}"] = t2n(ix).astype(np.int16)
                out[f"sample{i}/commit{lvl}"] = np.float32(float(c))
                if lvl == 0:
                    out[f"sample{i}/qst{lvl}"] = t2n(q)
            # decode_embeddings.py:35-45 (without autocast: CPU fp32): codes -> embed_code ->
            # decode -> elu -> HU = rint(x * 1000 - 1000)
            embs = [qz.embed_code(ix).permute(0, 4, 1, 2, 3) for ix, qz in zip(idxs, m.encoder.quantize)]
            res = F.elu(m.decode(embs)).squeeze().numpy() * 1000 - 1000
            out[f"sample{i}/hu"] = np.rint(res).astype(np.int32)
    save(name, **out)


def main():
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1:] or ["vq", "qtrain", "blocks", "loss", "ema", "models", "encode"]
    if "ema" in which:
        gen_ema_dist()
    if "vq" in which:
        gen_vq_kats()
    if "qtrain" in which:
        gen_quantizer_train()
    if "blocks" in which:
        gen_blocks()
    if "loss" in which:
        gen_loss()
    if "models" in which:
        # cfg1: 2-layer CLI defaults at 32^3, batch 1 (BASELINE.json configs[0])
        gen_model("model_2l_dflt_32", model_args(), (1, 1, 32, 32, 32), [32])
        # 2-layer with every block list non-empty, K per level, batch 2, padded slices
        gen_model("model_2l_blocks_32", model_args(n_pre_quantization_blocks=1, n_post_quantization_blocks=1,
                                                   n_post_upscale_blocks=1, n_post_downscale_blocks=1,
                                                   num_embeddings=[64, 32]),
                  (2, 1, 32, 32, 16), [16, 11], keep_state=False)
        # 3-layer CLI defaults at 64 x 64 x 64 (top level 1 x 1 x 1)
        # 3-layer (base 2 channels to keep the fixture small) at 64^3: top level is 1 x 1 x 1
        gen_model("model_3l_b2_64", model_args(n_bottleneck_blocks=3, base_network_channels=2,
                                               num_embeddings=[128, 256, 512]),
                  (2, 1, 64, 64, 64), [64, 40], steps=1, keep_state=False, keep_grads=False, dec_stride=2)
        gen_model("model_2l_regular_32", model_args(block_type='regular', base_network_channels=2),
                  (1, 1, 32, 32, 16), [16], steps=1, keep_state=False)
        gen_model("model_2l_evonorm_32", model_args(block_type='evonorm'), (1, 1, 32, 32, 16), [16],
                  steps=1, keep_state=False)
    if "encode" in which:
        gen_encode("encode_2l_blocks_32", model_args(n_pre_quantization_blocks=1, n_post_quantization_blocks=1,
                                                     n_post_upscale_blocks=1, n_post_downscale_blocks=1,
                                                     num_embeddings=[64, 32]), (1, 1, 32, 32, 32))
        gen_encode("encode_3l_b2_64", model_args(n_bottleneck_blocks=3, base_network_channels=2,
                                                 num_embeddings=[128, 256, 512]), (2, 1, 64, 64, 64))


if __name__ == "__main__":
    main()
