"""Criteo featurisation bindings (csrc/da/criteo.cpp).

``featurize_lines(bytes) -> (ids [n, 39] int32 padded with -1, labels [n])``
reproduces ``_get_next_input`` of the reference
(``cerebro_gpdb/preprocessing/criteo/preprocessing_criteo.py:75-110``):
13 bucketised continuous features + 26 murmur3-hashed categorical features
-> active columns of the 7306-wide one-hot vector.
"""

import ctypes

import numpy as np

from ..config import catalog as cat
from .da import lib as _da_lib

FIELDS = 39
_BOUND = False


def _lib():
    global _BOUND
    L = _da_lib()
    if not _BOUND:
        L.cer_murmur3_32.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_uint32]
        L.cer_murmur3_32.restype = ctypes.c_uint32
        L.cer_criteo_bucket.argtypes = [ctypes.c_double]
        L.cer_criteo_bucket.restype = ctypes.c_int
        L.cer_criteo_featurize.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
        L.cer_criteo_featurize.restype = ctypes.c_int64
        _BOUND = True
    return L


def murmur3_32(data, seed=0, signed=True):
    """MurmurHash3_x86_32; ``signed`` matches ``mmh3.hash``."""
    if isinstance(data, str):
        data = data.encode("utf-8")
    h = int(_lib().cer_murmur3_32(data, len(data), seed))
    return h - (1 << 32) if signed and h >= (1 << 31) else h


def bucket(v):
    return int(_lib().cer_criteo_bucket(float(v)))


def featurize_lines(buf, nthreads=8):
    """bytes of '\\n'-separated TSV rows -> (ids int32 [n, 39] (-1 pad), labels int32 [n])."""
    n = buf.count(b"\n") + (0 if buf.endswith(b"\n") or not buf else 1)
    ids = np.empty((max(n, 1), FIELDS), np.int32)
    labels = np.empty(max(n, 1), np.int32)
    rows = _lib().cer_criteo_featurize(buf, len(buf), ids.ctypes.data, labels.ctypes.data, n,
                                       nthreads)
    return ids[:rows], labels[:rows]


def ids_to_dense(ids, labels):
    """Compact ids -> the reference's dense f32 [n, 7306 + 1] rows (label last)."""
    n = ids.shape[0]
    dense = np.zeros((n, cat.INPUT_SHAPE_CRITEO[0] + 1), np.float32)
    r, c = np.nonzero(ids >= 0)
    dense[r, ids[r, c]] = 1.0
    dense[:, -1] = labels
    return dense
