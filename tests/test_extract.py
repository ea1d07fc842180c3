"""Encode-only code extraction (extract_embeddings.py:16-76, load_lmdb_dataset.py:54-109).

CPU: the oracle's eval-mode encode against the reference goldens (tools/make_goldens.py
gen_encode), and the code store / dataset semantics.  GPU: `vq3d.extract.extract_samples` on the
HIP path against the same goldens, buffers untouched in eval mode, codes through the store.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import vqvae_cpu as O

ENC_CFGS = {
    "encode_2l_blocks_32": dict(n_bottleneck_blocks=2, n_pre_quantization_blocks=1, n_post_quantization_blocks=1,
                                n_post_upscale_blocks=1, n_post_downscale_blocks=1, num_embeddings=[64, 32]),
    "encode_3l_b2_64": dict(n_bottleneck_blocks=3, base_network_channels=2, num_embeddings=[128, 256, 512]),
}


def sample(d, i):
    xs = tuple(int(v) for v in d["x_shape"])
    return torch.rand(xs, generator=torch.Generator().manual_seed(5000 + i)) * 4.5 - 0.5


@pytest.mark.parametrize("name", sorted(ENC_CFGS))
def test_oracle_encode_eval_vs_reference(name):
    """Oracle restatement of the eval-mode encode: codes bit-exact, commitment losses 1e-5 rel."""
    torch.set_num_threads(4)
    d = golden(name)
    cfg = O.Config(**ENC_CFGS[name])
    sd = {k[6:]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith("state/")}
    before = {k: v.clone() for k, v in sd.items() if "quantize." in k}
    for i in range(int(d["n_samples"])):
        with torch.no_grad():
            res = O.encode(cfg, sd, sample(d, i), train=False)
        for lvl, (c, q, ix) in enumerate(res):
            assert np.array_equal(ix.numpy(), d[f"sample{i}/idx{lvl}"]), (name, i, lvl)
            r = float(d[f"sample{i}/commit{lvl}"])
            assert abs(float(c) - r) <= 1e-5 * abs(r), (name, i, lvl)
        ref = d[f"sample{i}/qst0"]
        assert np.abs(res[0][1].numpy() - ref).max() <= 1e-5 * max(np.abs(ref).max(), 1.0)
    for k, v in before.items():  # eval mode leaves the codebook state alone
        assert torch.equal(sd[k], v), k


def test_code_store_roundtrip_and_dataset_semantics(tmp_path):
    from vq3d.extract import CodesDataset, CodeStore
    rng = np.random.default_rng(0)
    shapes = [(1, 8, 8, 2), (1, 2, 2, 1), (1, 1, 1, 1)]
    ks = [128, 256, 512]
    codes = [[rng.integers(0, k, size=s, dtype=np.int64) for s, k in zip(shapes, ks)] for _ in range(5)]
    root = str(tmp_path / "codes")
    with CodeStore(root, ks, len(codes)) as st:
        for i in (3, 0, 4, 1, 2):  # any order, as the reference's shuffled loader writes
            st.put(i, [torch.from_numpy(c) for c in codes[i]])
        with pytest.raises(ValueError):
            st.put(0, codes[0][:2])
        with pytest.raises(IndexError):
            st.put(5, codes[0])
    ds = CodesDataset(root)
    assert len(ds) == 5 and ds.n_enc == 3 and ds.num_embeddings == ks
    for i in range(5):
        got = ds[i]
        assert len(got) == 3
        for g, r in zip(got, codes[i]):
            assert g.dtype == np.int64 and np.array_equal(g, r)
    # embedding_id selects a level and the one above it (load_lmdb_dataset.py:84-89)
    ds0 = CodesDataset(root, embedding_id=0)
    assert ds0.num_embeddings == [128, 256] and [a.shape for a in ds0[2]] == shapes[:2]
    ds2 = CodesDataset(root, embedding_id=2)
    assert ds2.num_embeddings == [512, 0] and len(ds2[1]) == 1
    with pytest.raises(AssertionError):
        CodesDataset(root, embedding_id=3)
    with pytest.raises(IndexError):
        ds[5]


def test_write_lmdb_needs_python_lmdb():
    """python-lmdb is absent in this image: the reference-format writer says so instead of
    writing something else."""
    from vq3d.extract import write_lmdb
    try:
        import lmdb  # noqa: F401
        pytest.skip("lmdb installed")
    except ImportError:
        pass
    with pytest.raises(ImportError):
        write_lmdb("/nonexistent", None, [], 0)


def _load(name, dev, dtype):
    import vq3d
    d = golden(name)
    m = vq3d.VQVAE(vq3d.default_args(compute_dtype=dtype, **ENC_CFGS[name]))
    m.load_state_dict({k[6:]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith("state/")})
    return m.to(dev), d


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(ENC_CFGS))
def test_gpu_extract_fp32_vs_reference(gpu, name, tmp_path):
    """HIP encode in eval mode: codes >= 99.9 % equal to the reference's (conv summation order
    differs; the codebook search itself is bit-exact, test_gpu_parity KATs), commitment losses
    within 2e-4 relative, q_st within 5e-4 of its max; EMA buffers untouched; store round trip."""
    from vq3d.extract import CodesDataset, extract_samples, write_codes
    m, d = _load(name, gpu, "fp32")
    n = int(d["n_samples"])
    before = {k: v.clone() for k, v in m.state_dict().items() if "quantize." in k}
    vols = [sample(d, i) for i in range(n)]
    outs = []
    for i, idxs in enumerate(extract_samples(m, vols)):
        assert len(idxs) == m.n_bottleneck_blocks
        for lvl, ix in enumerate(idxs):
            ref = d[f"sample{i}/idx{lvl}"]
            got = ix.cpu().numpy()
            assert got.shape == ref.shape and ix.dtype == torch.int64
            assert (got == ref).mean() >= 0.999, (name, i, lvl, (got == ref).mean())
        outs.append([ix.cpu().numpy() for ix in idxs])
    m.eval()
    with torch.no_grad():
        for i in range(n):
            res = list(m.encode(vols[i].to(gpu)))
            for lvl, (c, q, ix) in enumerate(res):
                r = float(d[f"sample{i}/commit{lvl}"])
                assert abs(float(c) - r) <= 2e-4 * abs(r), (name, i, lvl, float(c), r)
            ref = d[f"sample{i}/qst0"]
            assert np.abs(res[0][1].float().cpu().numpy() - ref).max() <= 5e-4 * max(np.abs(ref).max(), 1.0)
    for k, v in before.items():
        assert torch.equal(m.state_dict()[k], v), k
    root = str(tmp_path / "codes")
    write_codes(root, m, vols, n)
    ds = CodesDataset(root)
    for i in range(n):
        for g, r in zip(ds[i], outs[i]):
            assert np.array_equal(g, r)


@pytest.mark.gpu
def test_gpu_extract_bf16_codes(gpu):
    """bf16 activations (the production dtype): codes mostly equal to the reference's."""
    from vq3d.extract import extract_samples
    m, d = _load("encode_2l_blocks_32", gpu, "bf16")
    for i, idxs in enumerate(extract_samples(m, [sample(d, i) for i in range(int(d["n_samples"]))])):
        for lvl, ix in enumerate(idxs):
            match = (ix.cpu().numpy() == d[f"sample{i}/idx{lvl}"]).mean()
            assert match >= 0.9, (i, lvl, match)


# ------------------------------------------------------------------------- decode path (§8(f) row 3)
def test_nrrd_roundtrip(tmp_path):
    from vq3d.decode import read_nrrd, write_nrrd
    rng = np.random.default_rng(1)
    for dt in (np.int64, np.int16, np.float32):
        a = (rng.standard_normal((5, 4, 3)) * 1000).astype(dt)
        p = str(tmp_path / f"v_{np.dtype(dt).name}.nrrd")
        write_nrrd(p, a)
        b, hdr = read_nrrd(p)
        assert b.dtype == a.dtype and np.array_equal(a, b)
        assert hdr["sizes"] == "5 4 3" and hdr["spacings"].split() == ["0.976", "0.976", "3.0"]


@pytest.mark.parametrize("name", sorted(ENC_CFGS))
def test_oracle_decode_codes_vs_reference(name):
    """Oracle decode of the reference's codes: HU volume (rint(elu(dec) * 1000 - 1000)) within
    1 HU of the reference (fp32 summation order; rint boundaries)."""
    torch.set_num_threads(4)
    d = golden(name)
    cfg = O.Config(**ENC_CFGS[name])
    sd = {k[6:]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith("state/")}
    for i in range(int(d["n_samples"])):
        qs = [sd[f"encoder.quantize.{lvl}.embed"][torch.from_numpy(d[f"sample{i}/idx{lvl}"].astype(np.int64))]
              .permute(0, 4, 1, 2, 3) for lvl in range(cfg.n_bottleneck_blocks)]
        with torch.no_grad():
            hu = np.rint(torch.nn.functional.elu(O.decode(cfg, sd, qs)).squeeze().numpy() * 1000 - 1000)
        assert np.abs(hu - d[f"sample{i}/hu"]).max() <= 1, name


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(ENC_CFGS))
def test_gpu_decode_codes_vs_reference(gpu, name, tmp_path):
    """HIP decode of the reference's codes (fp32): HU within 1 + 5e-4 of the volume's max |HU|;
    written to NRRD and read back unchanged."""
    from vq3d.decode import decode_codes, read_nrrd, write_nrrd
    m, d = _load(name, gpu, "fp32")
    for i in range(int(d["n_samples"])):
        codes = [d[f"sample{i}/idx{lvl}"].astype(np.int64) for lvl in range(m.n_bottleneck_blocks)]
        hu = decode_codes(m, codes).cpu().numpy()
        ref = d[f"sample{i}/hu"]
        assert hu.shape == ref.shape and hu.dtype == np.int64
        assert np.abs(hu - ref).max() <= 1 + 5e-4 * np.abs(ref).max(), (name, i, np.abs(hu - ref).max())
        p = str(tmp_path / f"s{i}.nrrd")
        write_nrrd(p, hu)
        back, _ = read_nrrd(p)
        assert np.array_equal(back, hu)
    with pytest.raises(IndexError):
        decode_codes(m, [np.full_like(codes[0], 10 ** 6)] + codes[1:])
