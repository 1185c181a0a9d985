"""Nature-CNN shared trunk for Atari-shaped observations (BASELINE configs 2-4; not in the reference, which
supports only vector observations -- SURVEY §0 fact 5).

::

    obs uint8 [B, 4, 84, 84] / 255
    conv1 4->32, 8x8 stride 4, relu  -> [B, 32, 20, 20]
    conv2 32->64, 4x4 stride 2, relu -> [B, 64, 9, 9]
    conv3 64->64, 3x3 stride 1, relu -> [B, 64, 7, 7]
    fc    3136->512 relu
    heads: policy logits 512->A, value 512->1

Parameters are fp32 masters; the GPU engine (:mod:`..algos.engine`) runs the GEMMs in bf16 on MFMA with fp32
accumulation through hand-written implicit-GEMM kernels (``csrc/kernels/conv_gemm.hip``).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .layers import Conv, Dense


class NatureCNN(nn.Module):
    def __init__(self, in_ch=4, hidden=512, generator=None):
        super().__init__()
        g = 2 ** 0.5
        self.conv1 = Conv(in_ch, 32, 8, 4, "relu", gain=g, generator=generator)
        self.conv2 = Conv(32, 64, 4, 2, "relu", gain=g, generator=generator)
        self.conv3 = Conv(64, 64, 3, 1, "relu", gain=g, generator=generator)
        self.fc = Dense(64 * 7 * 7, hidden, "relu", kernel_init=("orthogonal", g), generator=generator)
        self.out_dim = hidden

    def forward(self, obs):
        x = obs.float() * (1.0 / 255.0)
        x = self.conv3(self.conv2(self.conv1(x)))
        return self.fc(x.flatten(1))


class CNNActorCriticNet(nn.Module):
    """Shared trunk + categorical policy head + value head."""

    def __init__(self, num_actions, in_ch=4, hidden=512, generator=None):
        super().__init__()
        self.trunk = NatureCNN(in_ch, hidden, generator)
        self.pi = Dense(hidden, num_actions, None, kernel_init=("orthogonal", 0.01), generator=generator)
        self.v = Dense(hidden, 1, None, kernel_init=("orthogonal", 1.0), generator=generator)

    def forward(self, obs):
        h = self.trunk(obs)
        return self.pi(h), self.v(h).view(-1)
