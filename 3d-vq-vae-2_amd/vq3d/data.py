"""CT volume data module (reference utils/load_nrrd_dataset.py:16-175).

The reference's loader is host-side (DataLoader workers) and so is this one; the volume it yields
is what `training_step` / `extract_samples` move to the GPU.  monai 0.8.0 and pynrrd are not
installed in this image, so the transform chain is restated from their published semantics
(parity unpinned by a reference run; pinned by the closed forms in tests/test_data.py):

  AddChannel                               x[None]
  ThresholdIntensity(3000, above=False)    where(x < 3000, x, 3000)     (HU clip, top)
  ThresholdIntensity(-1500, above=True)    where(x > -1500, x, -1500)   (HU clip, bottom)
  ScaleIntensity(factor=-1 + 1/1000)       x * (1 + factor) = x / 1000
  ShiftIntensity(1)                        x + 1                        -> [-0.5, 4.0]
  DepthPadAndCrop(128)                     zero-pad depth to 128, keep [..., :128]; label =
                                           number of valid slices (load_nrrd_dataset.py:16-42)
  Interpolate(size, mode='area')           optional rescale of the volume (not of the label)
"""
import gzip
import zlib
from pathlib import Path
from random import randint
from typing import Optional, Sequence, Tuple, Union

import numpy as np
import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader, Dataset, random_split

from .decode import _NRRD_DTYPES

MIN_VAL, MAX_VAL, SCALE_VAL = -1500, 3000, 1000  # load_nrrd_dataset.py:72

# NRRD type spellings -> the canonical names of vq3d.decode's table
_TYPE_ALIASES = {
    "signed char": "int8", "int8_t": "int8", "int8": "int8", "uchar": "uint8", "unsigned char": "uint8",
    "uint8_t": "uint8", "uint8": "uint8", "short": "short", "short int": "short", "signed short": "short",
    "signed short int": "short", "int16": "short", "int16_t": "short", "ushort": "ushort",
    "unsigned short": "ushort", "unsigned short int": "ushort", "uint16": "ushort", "uint16_t": "ushort",
    "int": "int", "signed int": "int", "int32": "int", "int32_t": "int", "uint": "uint", "unsigned int": "uint",
    "uint32": "uint", "uint32_t": "uint", "longlong": "longlong", "long long": "longlong", "int64": "longlong",
    "int64_t": "longlong", "ulonglong": "ulonglong", "unsigned long long": "ulonglong", "uint64": "ulonglong",
    "uint64_t": "ulonglong", "float": "float", "double": "double",
}


class DepthPadAndCrop(torch.nn.Module):
    """load_nrrd_dataset.py:16-42: pad the depth axis with `pad_value` up to `output_depth`, keep
    the first `output_depth` slices, return (x, num_valid_slices).  The reference draws (or
    checks) a crop centre but slices from 0 regardless; that behaviour is kept."""

    def __init__(self, output_depth, pad_value=0, center=None):
        super().__init__()
        self.output_depth = output_depth
        self.pad_value = pad_value
        self.center = center

    def forward(self, x):
        d = x.shape[-1]
        pad_size = max(0, self.output_depth - d)
        radius = self.output_depth // 2
        low, high = radius, (d + pad_size) - radius
        if self.center is not None:
            assert self.center in range(low, high + 1)
        else:
            randint(low, high)  # the reference consumes one draw of Python's RNG here
        num_valid_slices = self.output_depth - pad_size
        return F.pad(x, (0, pad_size, 0, 0, 0, 0))[..., :self.output_depth], num_valid_slices


def normalize_hu(x):
    """HU volume (H, W, D) -> (1, H, W, D) fp32 in [-0.5, 4.0] (load_nrrd_dataset.py:74-80)."""
    x = torch.as_tensor(np.asarray(x, dtype=np.float32))[None]
    x = torch.where(x < MAX_VAL, x, torch.tensor(float(MAX_VAL)))
    x = torch.where(x > MIN_VAL, x, torch.tensor(float(MIN_VAL)))
    x = x * (1 + (-1 + 1 / SCALE_VAL))
    return x + 1


class CTTransform:
    """The reference's Compose chain (load_nrrd_dataset.py:72-85): volume -> (x, num_valid_slices)."""

    def __init__(self, output_depth=128, rescale_input: Optional[Tuple[int, int, int]] = None):
        self.crop = DepthPadAndCrop(output_depth=output_depth)
        self.rescale_input = tuple(rescale_input) if rescale_input else None

    def __call__(self, data):
        x, nvs = self.crop(normalize_hu(data))
        if self.rescale_input:
            x = F.interpolate(x.unsqueeze(0), size=self.rescale_input, mode="area").squeeze(0)
        return x, nvs


# ------------------------------------------------------------------------------------------ NRRD
def read_nrrd_header(path):
    """The header fields of an NRRD file (text up to the blank line)."""
    hdr = {}
    with open(path, "rb") as f:
        magic = f.readline().decode("ascii").strip()
        if not magic.startswith("NRRD"):
            raise ValueError(f"{path}: not an NRRD file")
        for raw in f:
            ln = raw.decode("ascii").rstrip("\n")
            if ln == "":
                break
            if ln.startswith("#") or ":" not in ln:
                continue
            k, v = ln.split(":", 1)
            hdr[k.strip()] = v.strip().lstrip("=").strip()
    hdr["sizes"] = [int(s) for s in hdr["sizes"].split()]
    if "space directions" in hdr:
        vecs = []
        for tok in hdr["space directions"].replace(" ", "").split(")("):
            tok = tok.strip("()")
            vecs.append([float(v) for v in tok.split(",")] if tok != "none" else None)
        hdr["space directions"] = np.array([v for v in vecs if v is not None])
    return hdr


def read_nrrd_volume(path):
    """(array in the file's axis order, header) for raw or gzip NRRD (pynrrd's default writes gzip)."""
    with open(path, "rb") as f:
        blob = f.read()
    head, _, body = blob.partition(b"\n\n")
    hdr = read_nrrd_header(path)
    enc = hdr.get("encoding", "raw")
    if enc in ("gzip", "gz"):
        try:
            body = gzip.decompress(body)
        except OSError:
            body = zlib.decompress(body)
    elif enc != "raw":
        raise NotImplementedError(f"NRRD encoding {enc}")
    dt = _NRRD_DTYPES[_TYPE_ALIASES[hdr["type"]]]
    dt = dt.newbyteorder("<" if hdr.get("endian", "little") == "little" else ">")
    sizes = tuple(hdr["sizes"])
    return np.frombuffer(body, dtype=dt, count=int(np.prod(sizes))).reshape(sizes, order="F"), hdr


class CTScanDataset(Dataset):
    """load_nrrd_dataset.py:112-175: every `*.nrrd` below root whose sizes match `size` (None =
    any) and whose diagonal voxel spacing matches `spacing` (atol 1e-3); items are the
    transform of the fp32 volume."""

    def __init__(self, root: str, transform=None,
                 size: Tuple[Union[int, None], Union[int, None], Union[int, None]] = (512, 512, None),
                 spacing: Union[Tuple[float, float, float], None] = None, ext: str = ".nrrd"):
        self.transform = transform
        scans = sorted(str(p) for p in Path(root).glob(f"**/*{ext}"))
        keep = []
        for s in scans:
            hdr = read_nrrd_header(s)
            if any(want is not None and have != want for have, want in zip(hdr["sizes"], size)):
                continue
            if spacing is not None:
                sd = hdr.get("space directions")
                if sd is None or not np.isclose(np.diag(sd), spacing, atol=1e-3).all():
                    continue
            keep.append(s)
        self.scans = np.array(keep)

    def __len__(self) -> int:
        return self.scans.shape[0]

    def get_scan(self, scan_index: int):
        data, metadata = read_nrrd_volume(self.scans[scan_index])
        return data.astype(np.float32), metadata

    def __getitem__(self, index: int):
        data, _ = self.get_scan(index)
        return self.transform(data) if self.transform is not None else data


class CTDataModule:
    """load_nrrd_dataset.py:56-109 (LightningDataModule surface: setup / train_dataloader /
    val_dataloader)."""

    def __init__(self, path, batch_size=64, train_frac=0.95, num_workers=6,
                 rescale_input: Optional[Sequence[int]] = ()):
        assert 0 <= train_frac <= 1
        self.path = path
        self.train_frac = train_frac
        self.num_workers = num_workers
        self.batch_size = batch_size
        self.rescale_input = rescale_input

    def setup(self, stage=None):
        dataset = CTScanDataset(self.path, transform=CTTransform(128, self.rescale_input or None),
                                spacing=(0.976, 0.976, 3))
        train_len = int(len(dataset) * self.train_frac)
        val_len = len(dataset) - train_len
        self.train_dataset, self.val_dataset = random_split(dataset, [train_len, val_len])
        self.train_len, self.val_len = train_len, val_len

    def train_dataloader(self):
        return DataLoader(self.train_dataset, batch_size=self.batch_size, num_workers=self.num_workers,
                          pin_memory=torch.cuda.is_available(), shuffle=True, drop_last=True)

    def val_dataloader(self):
        return DataLoader(self.val_dataset, batch_size=self.batch_size, num_workers=self.num_workers,
                          pin_memory=torch.cuda.is_available(), shuffle=False, drop_last=True)
