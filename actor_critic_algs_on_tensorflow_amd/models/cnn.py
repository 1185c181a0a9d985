"""Nature-CNN shared trunk for Atari-shaped observations (BASELINE configs 2-4; not in the reference, which
supports only vector observations -- SURVEY §0 fact 5).

::

    obs uint8 [B, 4, 84, 84] / 255
    conv1 4->32, 8x8 stride 4, relu  -> [B, 32, 20, 20]     weight [32, 4, 8, 8]   (OIHW)
    conv2 32->64, 4x4 stride 2, relu -> [B, 64, 9, 9]       weight [64, 4, 4, 32]  (OHWI)
    conv3 64->64, 3x3 stride 1, relu -> [B, 64, 7, 7]       weight [64, 3, 3, 64]  (OHWI)
    flatten in NHWC order (h, w, c)  -> [B, 3136]
    fc    3136->512 relu                                     kernel [3136, 512] ([in, out], TF dense layout)
    heads 512->A+1: columns 0..A-1 policy logits, column A the value

The weight layouts and the NHWC flatten are the ones the GPU engine (:mod:`..algos.engine`) computes in: every
activation there is an NHWC bf16 matrix ``[B*H*W, C]`` produced by one MFMA GEMM (``csrc/kernels/gemm.hip``)
from an im2col image (``csrc/kernels/conv.hip``), so this fp32 module is the exact reference of that engine.
Parameters are fp32 masters; the engine reads a bf16 shadow written by the fused optimiser.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .layers import Conv, Dense


class NatureCNN(nn.Module):
    def __init__(self, in_ch=4, hidden=512, generator=None):
        super().__init__()
        g = 2 ** 0.5
        self.conv1 = Conv(in_ch, 32, 8, 4, "relu", gain=g, generator=generator, layout="oihw")
        self.conv2 = Conv(32, 64, 4, 2, "relu", gain=g, generator=generator, layout="ohwi")
        self.conv3 = Conv(64, 64, 3, 1, "relu", gain=g, generator=generator, layout="ohwi")
        self.fc = Dense(64 * 7 * 7, hidden, "relu", kernel_init=("orthogonal", g), generator=generator)
        self.out_dim = hidden

    def forward(self, obs):
        x = obs.float() * (1.0 / 255.0)
        x = self.conv3(self.conv2(self.conv1(x)))
        return self.fc(x.permute(0, 2, 3, 1).flatten(1))


class CNNActorCriticNet(nn.Module):
    """Shared trunk + one fused head: logits (orthogonal init, gain 0.01) and value (gain 1.0) columns."""

    def __init__(self, num_actions, in_ch=4, hidden=512, generator=None):
        super().__init__()
        self.num_actions = num_actions
        self.trunk = NatureCNN(in_ch, hidden, generator)
        self.heads = Dense(hidden, num_actions + 1, None, kernel_init=("orthogonal", 0.01), generator=generator)
        with torch.no_grad():
            v = torch.empty(hidden, 1)
            from .init import orthogonal_
            orthogonal_(v, 1.0, generator=generator)
            self.heads.kernel[:, num_actions:].copy_(v)

    def forward(self, obs):
        z = self.heads(self.trunk(obs))
        return z[:, :self.num_actions], z[:, self.num_actions]
