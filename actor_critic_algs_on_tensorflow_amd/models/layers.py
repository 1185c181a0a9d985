"""Layers with TF-compatible parameter layout.

``Dense`` stores ``kernel [in, out]`` and ``bias [out]`` -- the layout of ``tf.layers.dense`` and therefore of
the reference checkpoint -- so checkpoints round-trip without transposes and the GEMM kernels
consume ``X[B, in] @ W[in, out]`` directly. ``Conv`` stores ``weight [out, in, kh, kw]``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import init as I


def lrelu(x, alpha=0.2):
    """``(1 - alpha) relu(x) + alpha x`` (``Basic_AC/policies.py:20-21``)."""
    return (1 - alpha) * F.relu(x) + alpha * x


ACTIVATIONS = {
    "lrelu": lrelu,
    "relu": F.relu,
    "tanh": torch.tanh,
    "none": lambda x: x,
    None: lambda x: x,
}


class Dense(nn.Module):
    def __init__(self, in_features, out_features, activation=None, kernel_init="xavier", bias_init=0.0,
                 generator=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.activation = activation
        self.kernel = nn.Parameter(torch.empty(in_features, out_features))
        self.bias = nn.Parameter(torch.full((out_features,), float(bias_init)))
        self.reset_kernel(kernel_init, generator)

    def reset_kernel(self, kernel_init, generator=None):
        if callable(kernel_init):
            kernel_init(self.kernel)
        elif kernel_init == "xavier":
            I.xavier_uniform_(self.kernel, generator=generator)
        elif kernel_init == "xav":
            I.scaled_xavier_(self.kernel, 0.1, generator=generator)
        elif kernel_init == "normc":
            I.normalized_column_(self.kernel, 0.1, generator=generator)
        elif isinstance(kernel_init, tuple) and kernel_init[0] == "orthogonal":
            I.orthogonal_(self.kernel, kernel_init[1], generator=generator)
        else:
            raise ValueError(kernel_init)

    def forward(self, x):
        y = torch.addmm(self.bias, x, self.kernel) if x.dim() == 2 else x @ self.kernel + self.bias
        return ACTIVATIONS[self.activation](y)


class Conv(nn.Module):
    """VALID convolution with a selectable weight layout.

    ``layout="oihw"``: ``weight [out, in, kh, kw]`` (PyTorch order; the im2col k index is (c, i, j)) -- used for
    the first Atari conv, whose input is the uint8 frame stack with frames as channels.
    ``layout="ohwi"``: ``weight [out, kh, kw, in]`` (k index (i, j, c)) -- used for convs over NHWC activations,
    where 8 consecutive k are 8 consecutive channels and the engine's im2col is a 16-byte copy.
    The forward here is the fp32 PyTorch reference of the engine's conv (``F.conv2d`` on NCHW tensors).
    """

    def __init__(self, cin, cout, k, stride, activation="relu", gain=2 ** 0.5, generator=None, layout="oihw"):
        super().__init__()
        self.cin, self.cout, self.k, self.stride = cin, cout, k, stride
        self.activation = activation
        self.layout = layout
        shape = (cout, cin, k, k) if layout == "oihw" else (cout, k, k, cin)
        self.weight = nn.Parameter(torch.empty(shape))
        self.bias = nn.Parameter(torch.zeros(cout))
        with torch.no_grad():
            flat = torch.empty(cout, cin * k * k)
            I.orthogonal_(flat, gain, generator=generator)
            w = flat.view(cout, cin, k, k)
            self.weight.copy_(w if layout == "oihw" else w.permute(0, 2, 3, 1))

    def weight_oihw(self):
        return self.weight if self.layout == "oihw" else self.weight.permute(0, 3, 1, 2)

    def out_hw(self, h):
        return (h - self.k) // self.stride + 1

    def forward(self, x):
        return ACTIVATIONS[self.activation](F.conv2d(x, self.weight_oihw(), self.bias, stride=self.stride))
