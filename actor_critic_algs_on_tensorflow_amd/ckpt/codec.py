"""Python face of the C++ TF-bundle codec (``csrc/tfbundle``, built into ``_C/_tfbundle*.so``).

Maps TF ``DataType`` enums to numpy dtypes and offers ``read(prefix) -> {name: ndarray}`` /
``write(prefix, {name: ndarray})``. No TensorFlow is needed (or installed): the codec writes the exact byte
layout TensorFlow's ``Saver`` V2 writes (see ``tests/test_ckpt.py``: the reference demo checkpoint re-serialises
byte-identically).
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os

import numpy as np

_C_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C")
_mod = None

DT_TO_NP = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
            10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
NP_TO_DT = {np.dtype(v): k for k, v in DT_TO_NP.items()}
DT_BFLOAT16 = 14


def load():
    """Imports the compiled codec module (raises ImportError with a build hint if it is missing)."""
    global _mod
    if _mod is None:
        for suffix in importlib.machinery.EXTENSION_SUFFIXES:
            path = os.path.join(_C_DIR, "_tfbundle" + suffix)
            if os.path.exists(path):
                spec = importlib.util.spec_from_file_location("_tfbundle", path)
                m = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(m)
                _mod = m
                break
        if _mod is None:
            raise ImportError(f"_tfbundle extension not built in {_C_DIR}; run `python build.py`")
    return _mod


def read(prefix, verify_crc=True):
    """-> dict name -> numpy array (insertion order = sorted key order)."""
    out = {}
    for key, dt, shape, data in load().read_bundle(prefix, verify_crc):
        if dt == DT_BFLOAT16:
            a = np.frombuffer(data, dtype=np.uint16).reshape(shape)
        else:
            a = np.frombuffer(data, dtype=DT_TO_NP[dt]).reshape(shape)
        out[key] = a
    return out


def write(prefix, tensors):
    """``tensors``: dict name -> numpy array (C-contiguous little-endian); writes <prefix>.index/.data-*."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    items = []
    for k, v in tensors.items():
        a = np.asarray(v, order="C")
        dt = NP_TO_DT[a.dtype]
        items.append((k, dt, list(a.shape), a.tobytes()))
    load().write_bundle(prefix, items)


def parse_index(index_bytes):
    return load().parse_index(index_bytes)


def build_index(entries, num_shards=1, producer=1):
    return load().build_index(entries, num_shards, producer)


def masked_crc32c(b):
    return load().masked_crc32c(b)


def crc32c(b):
    return load().crc32c(b)
