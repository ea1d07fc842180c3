"""CT data module (vq3d/data.py; reference utils/load_nrrd_dataset.py:16-175).  monai and
pynrrd are absent, so the transform is checked against its closed form (HU clip to
[-1500, 3000], / 1000, + 1, zero depth padding to 128 with the valid-slice label) and the NRRD
reader against files written here (raw and gzip, pynrrd's header fields): parity unpinned by a
reference run."""
import gzip
import random

import numpy as np
import torch

from vq3d import data as D


def _write(path, arr, spacing=(0.976, 0.976, 3.0), encoding="gzip", typ="short"):
    body = np.asfortranarray(arr).tobytes(order="F")
    if encoding == "gzip":
        body = gzip.compress(body)
    sd = " ".join(f"({spacing[0] if i == 0 else 0},{spacing[1] if i == 1 else 0},{spacing[2] if i == 2 else 0})"
                  for i in range(3))
    hdr = (f"NRRD0004\n# Complete NRRD file format specification at:\ntype: {typ}\ndimension: 3\n"
           f"space: left-posterior-superior\nsizes: {' '.join(map(str, arr.shape))}\nspace directions: {sd}\n"
           f"kinds: domain domain domain\nendian: little\nencoding: {encoding}\n"
           f"space origin: (-250,-250,-100)\n\n")
    with open(path, "wb") as f:
        f.write(hdr.encode("ascii") + body)


def test_normalize_and_depth_pad_crop():
    rng = np.random.default_rng(0)
    hu = rng.integers(-3000, 5000, size=(8, 6, 100)).astype(np.float32)
    hu[0, 0, :4] = [-1500, 3000, 2999, -1499]
    x, nvs = D.CTTransform(output_depth=128)(hu)
    ref = np.clip(hu, -1500, 3000) / 1000 + 1
    assert x.shape == (1, 8, 6, 128) and nvs == 100
    assert np.allclose(x[0, ..., :100].numpy(), ref, rtol=0, atol=1e-6)
    assert torch.all(x[..., 100:] == 0)
    assert float(x.min()) >= -0.5 - 1e-6 and float(x.max()) <= 4.0 + 1e-6  # x * (1 + (-1 + 1/1000)) in fp32
    x2, nvs2 = D.CTTransform(output_depth=128)(rng.normal(size=(4, 4, 150)).astype(np.float32) * 500)
    assert x2.shape == (1, 4, 4, 128) and nvs2 == 128  # deeper scans keep the first 128 slices
    # the reference draws a crop centre from Python's RNG (and ignores it): one draw per call
    random.seed(3)
    D.DepthPadAndCrop(128)(torch.zeros(1, 2, 2, 90))
    a = random.random()
    random.seed(3)
    random.randint(64, 64)
    assert random.random() == a


def test_area_rescale_keeps_label():
    hu = np.full((16, 16, 64), 1000, np.float32)
    x, nvs = D.CTTransform(128, rescale_input=(8, 8, 64))(hu)
    assert x.shape == (1, 8, 8, 64) and nvs == 64
    assert torch.allclose(x[..., :32], torch.full((1, 8, 8, 32), 2.0))
    assert torch.allclose(x[..., 32:], torch.zeros(1, 8, 8, 32))


def test_nrrd_reader_raw_and_gzip(tmp_path):
    rng = np.random.default_rng(1)
    a = rng.integers(-2000, 3000, size=(5, 4, 3)).astype(np.int16)
    for enc in ("raw", "gzip"):
        p = str(tmp_path / f"v_{enc}.nrrd")
        _write(p, a, encoding=enc)
        b, hdr = D.read_nrrd_volume(p)
        assert np.array_equal(a, b) and hdr["sizes"] == [5, 4, 3]
        assert np.allclose(np.diag(hdr["space directions"]), (0.976, 0.976, 3.0))


def test_ct_dataset_filters_and_datamodule(tmp_path):
    rng = np.random.default_rng(2)
    good = [rng.integers(-1500, 3000, size=(16, 16, d)).astype(np.int16) for d in (20, 40, 24, 30)]
    for i, g in enumerate(good):
        (tmp_path / f"p{i}").mkdir()
        _write(str(tmp_path / f"p{i}" / "scan.nrrd"), g)
    _write(str(tmp_path / "wrong_size.nrrd"), good[0][:8])
    _write(str(tmp_path / "wrong_spacing.nrrd"), good[0], spacing=(0.7, 0.7, 2.5))
    ds = D.CTScanDataset(str(tmp_path), transform=D.CTTransform(128), size=(16, 16, None), spacing=(0.976, 0.976, 3))
    assert len(ds) == 4
    depths = sorted(int(ds[i][1]) for i in range(len(ds)))
    assert depths == [20, 24, 30, 40]
    dm = D.CTDataModule(str(tmp_path), batch_size=2, train_frac=0.5, num_workers=0)
    dm.setup()
    # CTDataModule's default size filter is the reference's (512, 512, None): these scans are 16 x 16
    assert dm.train_len == 0 and dm.val_len == 0
