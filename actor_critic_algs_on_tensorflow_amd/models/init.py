"""Parameter initialisers that reproduce the reference's distributions.

* ``xavier_uniform_``: TF ``xavier_initializer()`` / ``glorot_uniform``: U(-l, l), l = sqrt(6 / (fan_in + fan_out))
  (``Basic_AC/policies.py:7``; also the TF1 default for ``tf.layers.dense`` kernels).
* ``scaled_xavier_``: ``xav`` = 0.1 * Xavier (``Basic_AC/policies.py:3-6``).
* ``normalized_column_``: N(0, 1) then every column (output unit) rescaled to L2 norm 0.1
  (``A3C/policies.py:29-32``).
* ``orthogonal_``: the conventional Atari A2C/PPO init (gain sqrt(2) trunk, 0.01 policy, 1 value).

Kernels are stored ``[in, out]`` (TF dense layout), so "column" means output unit.
"""
from __future__ import annotations

import math

import torch


def xavier_uniform_(w: torch.Tensor, gain=1.0, generator=None):
    fan_in, fan_out = _fans(w)
    lim = gain * math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        return w.uniform_(-lim, lim, generator=generator)


def scaled_xavier_(w, scale=0.1, generator=None):
    return xavier_uniform_(w, gain=scale, generator=generator)


def normalized_column_(w, norm=0.1, generator=None):
    with torch.no_grad():
        u = torch.randn(w.shape, generator=generator, dtype=torch.float32)
        scale = torch.sqrt((u * u).sum(0, keepdim=True)) / norm
        w.copy_(u / scale)
    return w


def orthogonal_(w, gain=1.0, generator=None):
    """Orthogonal init on the matrix view ``[fan_in, fan_out]``-compatible with the storage layout."""
    with torch.no_grad():
        shape = w.shape
        rows = shape[0] if w.dim() == 2 else shape[0]
        cols = w.numel() // rows
        a = torch.randn(rows, cols, generator=generator)
        transpose = rows < cols
        if transpose:
            a = a.t()
        q, r = torch.linalg.qr(a)
        q = q * torch.sign(torch.diagonal(r)).unsqueeze(0)
        if transpose:
            q = q.t()
        w.copy_((gain * q).reshape(shape))
    return w


def _fans(w):
    if w.dim() == 2:           # dense [in, out]
        return w.shape[0], w.shape[1]
    if w.dim() == 4:           # conv [out, in, kh, kw]
        rf = w.shape[2] * w.shape[3]
        return w.shape[1] * rf, w.shape[0] * rf
    n = w.numel()
    return n, n
