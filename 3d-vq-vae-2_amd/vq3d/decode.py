"""Decode path: codes -> volume -> NRRD (vqvae/decode_embeddings.py:17-50).

`decode_codes(model, codes)` runs `quantizer.embed_code(idx).permute(0, 4, 1, 2, 3)` per level
(bottom -> top), the HIP decoder in eval mode without autograd, `elu`, and the reference's
Hounsfield mapping `rint(x * 1000 - 1000)` (decode_embeddings.py:19, 46-48), returning an
int64 volume on the device.  `write_nrrd` / `read_nrrd` cover the NRRD subset the reference
writes through pynrrd (not installed here): a 3-D little-endian raw array with `spacings`.
"""
import numpy as np
import torch
import torch.nn.functional as F

MIN_VAL, MAX_VAL, SCALE_VAL = -1500, 3000, 1000  # decode_embeddings.py:19
SPACINGS = (0.976, 0.976, 3)                      # decode_embeddings.py:50


@torch.no_grad()
def decode_codes(model, codes):
    """codes: per-level int64 (1, h, w, d) tensors / arrays, bottom -> top; returns the HU volume
    (H, W, D) int64 on the model's device."""
    model.eval()
    dev = next(model.parameters()).device
    quantizers = model.encoder.quantize
    if len(codes) > len(quantizers):
        raise ValueError(f"{len(codes)} code levels for a {len(quantizers)}-level model")
    embeddings = []
    for c, q in zip(codes, quantizers):
        idx = torch.as_tensor(c).to(dev, torch.int64)
        if idx.dim() == 3:
            idx = idx.unsqueeze(0)
        if int(idx.min()) < 0 or int(idx.max()) >= q.num_embeddings:
            raise IndexError(f"code outside [0, {q.num_embeddings})")
        embeddings.append(q.embed_code(idx).permute(0, 4, 1, 2, 3))
    res = F.elu(model.decode(embeddings).float())
    return torch.round(res.squeeze() * SCALE_VAL - SCALE_VAL).to(torch.int64)


_NRRD_TYPES = {np.dtype("int8"): "int8", np.dtype("uint8"): "uint8", np.dtype("int16"): "short",
               np.dtype("uint16"): "ushort", np.dtype("int32"): "int", np.dtype("uint32"): "uint",
               np.dtype("int64"): "longlong", np.dtype("uint64"): "ulonglong", np.dtype("float32"): "float",
               np.dtype("float64"): "double"}
_NRRD_DTYPES = {v: k for k, v in _NRRD_TYPES.items()}


def write_nrrd(path, data, spacings=SPACINGS):
    """NRRD0004, raw little-endian, Fortran (first axis fastest) order as pynrrd writes by default."""
    a = np.asarray(data)
    if a.dtype not in _NRRD_TYPES:
        raise TypeError(f"no NRRD type for {a.dtype}")
    header = ["NRRD0004", f"type: {_NRRD_TYPES[a.dtype]}", f"dimension: {a.ndim}",
              "sizes: " + " ".join(str(s) for s in a.shape)]
    if spacings is not None:
        header.append("spacings: " + " ".join(repr(float(s)) for s in spacings))
    header += ["endian: little", "encoding: raw"]
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n\n").encode("ascii"))
        f.write(np.asfortranarray(a.astype(a.dtype.newbyteorder("<"), copy=False)).tobytes(order="F"))


def read_nrrd(path):
    """(array, header dict) of a raw NRRD written by write_nrrd (or pynrrd with raw encoding)."""
    with open(path, "rb") as f:
        blob = f.read()
    head, _, body = blob.partition(b"\n\n")
    lines = head.decode("ascii").split("\n")
    if not lines[0].startswith("NRRD"):
        raise ValueError("not an NRRD file")
    hdr = {}
    for ln in lines[1:]:
        if ln.startswith("#") or ":" not in ln:
            continue
        k, v = ln.split(":", 1)
        hdr[k.strip()] = v.strip()
    if hdr.get("encoding", "raw") != "raw":
        raise NotImplementedError("only raw NRRD encoding")
    dt = _NRRD_DTYPES[hdr["type"]].newbyteorder("<" if hdr.get("endian", "little") == "little" else ">")
    sizes = tuple(int(s) for s in hdr["sizes"].split())
    arr = np.frombuffer(body, dtype=dt, count=int(np.prod(sizes))).reshape(sizes, order="F")
    return arr, hdr
