"""Loader for the native library (HIP kernels for gfx950 + C++ runtime pieces).

The shared object ``_C/libacamd.so`` is built in-tree by ``build.py`` (``hipcc --offload-arch=gfx950`` for the
``csrc/kernels/*.hip`` sources, ``g++`` for the torch-op bindings and the TF-bundle checkpoint codec). It
registers its ops under ``torch.ops.acamd``.

Policy: on a GPU the HIP path is mandatory -- :func:`require` raises if the library is missing, so no test or
benchmark silently falls back to an eager PyTorch implementation. CPU tensors use the pure-PyTorch reference
implementations (the oracles the kernels are tested against) or the C++ CPU ops.
"""
from __future__ import annotations

import os
import threading

import torch

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_C")
# (ACAMD_LIB: an alternative in-tree build of the same library, for A/B runs of kernel variants)
LIB_PATH = os.environ.get("ACAMD_LIB") or os.path.join(_LIB_DIR, "libacamd.so")

_lock = threading.Lock()
_loaded = None
_error = None


def load(raise_on_error=False):
    """Loads the native library once; returns True on success."""
    global _loaded, _error
    with _lock:
        if _loaded is None:
            if not os.path.exists(LIB_PATH):
                _loaded, _error = False, FileNotFoundError(
                    f"{LIB_PATH} not built; run `python build.py` (or __graft_entry__.build())")
            else:
                try:
                    torch.ops.load_library(LIB_PATH)
                    _loaded = True
                except Exception as e:  # pragma: no cover - depends on the build
                    _loaded, _error = False, e
    if not _loaded and raise_on_error:
        raise RuntimeError(f"native library unavailable: {_error}")
    return _loaded


def available():
    return load(False)


def require():
    """Raises unless the native library is loaded. Called by every GPU op wrapper."""
    load(True)
    return torch.ops.acamd


def force_reference():
    """``ACAMD_FORCE_REFERENCE=1`` routes GPU tensors through the PyTorch reference ops (A/B + debugging)."""
    return os.environ.get("ACAMD_FORCE_REFERENCE", "0") == "1"


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU and the native kernels must be used."""
    return t.is_cuda and not force_reference()
