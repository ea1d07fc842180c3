"""ORACLE (test infrastructure only) — ctypes binding of oracle/vq_nearest.c.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
See vq_nearest.c for the exact arithmetic and the reference lines it restates
(vqvae/layers.py:700-703,716,720).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libvqoracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.vq_oracle_nearest.restype = ctypes.c_double
        _lib.vq_oracle_nearest.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p]
        _lib.vq_oracle_cdist.restype = None
        _lib.vq_oracle_cdist.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    return _lib


def nearest(z, embed):
    """z (N, D) float32, embed (K, D) float32 -> (idx int64 (N,), zst float32 (N, D), sum sq err)."""
    z = np.ascontiguousarray(z, dtype=np.float32)
    embed = np.ascontiguousarray(embed, dtype=np.float32)
    n, d = z.shape
    k = embed.shape[0]
    assert embed.shape[1] == d
    idx = np.empty(n, np.int64)
    zst = np.empty_like(z)
    sq = lib().vq_oracle_nearest(z.ctypes.data, n, d, embed.ctypes.data, k, idx.ctypes.data,
                                 zst.ctypes.data)
    return idx, zst, sq


def cdist(z, embed):
    z = np.ascontiguousarray(z, dtype=np.float32)
    embed = np.ascontiguousarray(embed, dtype=np.float32)
    out = np.empty((z.shape[0], embed.shape[0]), np.float32)
    lib().vq_oracle_cdist(z.ctypes.data, z.shape[0], z.shape[1], embed.ctypes.data,
                          embed.shape[0], out.ctypes.data)
    return out
