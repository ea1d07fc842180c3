"""Encode-only code extraction (BASELINE config 4).

Mirrors `vqvae/extract_embeddings.py` and `utils/load_lmdb_dataset.py`:

* `extract_samples(model, volumes)` — eval mode, no autograd, one volume per call, yields the
  per-level code tensors bottom -> top exactly as `*_, idx = zip(*model.encode(x))`
  (extract_embeddings.py:16-23).  The encoder and the codebook search are the same HIP
  launches as in training (Quantizer in eval mode: no EMA update, no first-pass init,
  layers.py:695-707).
* `CodeStore` — the code database: one sub-database per level named "0" .. "n-1" (0 = bottom),
  key `str(i)`, value an int64 array (1, h, w, d); root entries `num_dbs`, `length`,
  `num_embeddings` (extract_embeddings.py:62-72).  python-lmdb is not installed in this image,
  so the store is a directory: `meta.json` for the root entries and one memory-mapped
  `level{j}.npy` of shape (length, 1, h, w, d) int64 per level; sample i of level j is row i.
  When `lmdb` is importable, `write_lmdb` writes the reference's exact LMDB layout instead.
* `CodesDataset(root, embedding_id=-1)` — `LMDBDataset` semantics over a `CodeStore`
  (load_lmdb_dataset.py:54-109): `embedding_id == -1` returns every level, otherwise level
  `embedding_id` and the one above it (conditioning), `num_embeddings` padded with 0 when only
  one level is returned.
"""
import json
import os
from typing import Iterable, List

import numpy as np
import torch


def extract_samples(model, volumes: Iterable[torch.Tensor], device=None):
    """Yield the tuple of code tensors (bottom -> top) of each volume (extract_embeddings.py:16-23).

    `volumes` yields fp32 (1, 1, H, W, D) tensors on the host or the device.  The codes stay on
    the device; `.cpu()` them (as the reference does before pickling) when they are consumed.
    """
    model.eval()
    dev = device if device is not None else next(model.parameters()).device
    with torch.no_grad():
        for sample in volumes:
            sample = sample.to(dev, non_blocking=True)
            *_, encoding_idx = zip(*model.encode(sample))
            yield encoding_idx


class CodeStore:
    """Writer of the code database (directory form of the reference's LMDB, see module doc)."""

    def __init__(self, root: str, num_embeddings, length: int):
        self.root = root
        self.num_embeddings = [int(k) for k in num_embeddings]
        self.num_dbs = len(self.num_embeddings)
        self.length = int(length)
        self._levels = None
        os.makedirs(root, exist_ok=True)

    def put(self, i: int, encodings) -> None:
        """Store sample i's per-level codes (tensors or arrays of shape (1, h, w, d))."""
        if not 0 <= i < self.length:
            raise IndexError(f"sample {i} outside [0, {self.length})")
        if len(encodings) != self.num_dbs:
            raise ValueError(f"{len(encodings)} levels given, the store has {self.num_dbs}")
        arrs = [e.cpu().numpy() if torch.is_tensor(e) else np.asarray(e) for e in encodings]
        if self._levels is None:
            self._levels = [np.lib.format.open_memmap(os.path.join(self.root, f"level{j}.npy"), mode="w+",
                                                      dtype=np.int64, shape=(self.length,) + a.shape)
                            for j, a in enumerate(arrs)]
        for lv, a in zip(self._levels, arrs):
            if a.shape != lv.shape[1:]:
                raise ValueError(f"code shape {a.shape} differs from the store's {lv.shape[1:]}")
            lv[i] = a

    def close(self) -> None:
        if self._levels is not None:
            for lv in self._levels:
                lv.flush()
        self._levels = None
        with open(os.path.join(self.root, "meta.json"), "w") as f:
            json.dump({"num_dbs": self.num_dbs, "length": self.length,
                       "num_embeddings": self.num_embeddings}, f)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_codes(root: str, model, volumes, length: int) -> None:
    """extract_embeddings.main without the data module: encode `length` volumes into a CodeStore."""
    with CodeStore(root, _num_embeddings(model), length) as store:
        for i, enc in enumerate(extract_samples(model, volumes)):
            store.put(i, enc)


def write_lmdb(path: str, model, volumes, length: int) -> None:
    """The reference's LMDB layout byte for byte (extract_embeddings.py:56-74); needs python-lmdb."""
    import pickle

    import lmdb  # not installed in this image: ImportError is the documented behaviour
    n = model.n_bottleneck_blocks
    db = lmdb.open(path, map_size=int(1e12), max_dbs=n)
    sub_dbs = [db.open_db(str(i).encode()) for i in range(n)]
    with db.begin(write=True) as txn:
        txn.put(b"num_dbs", str(n).encode())
        txn.put(b"length", str(length).encode())
        txn.put(b"num_embeddings", pickle.dumps(np.asarray(model.num_embeddings)))
        for i, enc in enumerate(extract_samples(model, volumes)):
            for sub_db, e in zip(sub_dbs, enc):
                txn.put(str(i).encode(), pickle.dumps(e.cpu().numpy()), db=sub_db)
    db.close()


def _num_embeddings(model) -> List[int]:
    k = model.num_embeddings
    return list(k) if isinstance(k, (list, tuple)) else [int(k)] * model.n_bottleneck_blocks


class CodesDataset(torch.utils.data.Dataset):
    """`LMDBDataset` (load_lmdb_dataset.py:54-109) over a CodeStore directory."""

    def __init__(self, root: str, embedding_id: int = -1, transform=None):
        with open(os.path.join(root, "meta.json")) as f:
            meta = json.load(f)
        self.length = int(meta["length"])
        self.n_enc = int(meta["num_dbs"])
        num_embeddings = meta["num_embeddings"]
        assert embedding_id < self.n_enc
        assert self.n_enc >= 1
        self.embedding_id = embedding_id
        self.levels = [np.load(os.path.join(root, f"level{j}.npy"), mmap_mode="r") for j in range(self.n_enc)]
        self.transform = transform
        get_embeddings = 2  # a level is conditioned on the one above it
        self._idx = range(self.n_enc) if embedding_id == -1 else range(embedding_id, self.n_enc)[:get_embeddings]
        self.num_embeddings = [num_embeddings[j] for j in self._idx]
        if len(self.num_embeddings) == 1:
            self.num_embeddings.append(0)

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, index: int) -> List[np.ndarray]:
        if not 0 <= index < self.length:
            raise IndexError(index)
        embeddings = [np.array(self.levels[j][index]) for j in self._idx]
        if self.transform is not None:
            embeddings = [t(e) for t, e in zip((self.transform[j] for j in self._idx), embeddings)]
        return embeddings
