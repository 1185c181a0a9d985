"""The reference's MLP actor and critic, with TF-compatible variable names.

Actor (``Basic_AC/policies.py:33-89``, ``A3C/policies.py:34-104``)::

    first_layer  D->128 lrelu(0.2) -> second_layer 128->128 lrelu -> third_layer 128->64 lrelu
    continuous: mu_layer 64->A, tanh * ac_scale;  log_std [A] (init 0, clipped to [-2.5, 2.5] in forward)
    discrete:   logits 64->A

Critic (``Basic_AC/policies.py:123-149``, ``A3C/policies.py:137-170``)::

    first_layer D->256 relu -> second_layer 256->128 relu -> third_layer 128->128 relu -> value 128->1

``variant`` selects the documented divergences:
  * ``"basic"``: mu kernel init 0.1*Xavier, logits default Xavier, critic value reads the *second* layer
    (the third layer is built but unused -- bug #4, kept so checkpoints carry the same variables).
  * ``"a3c"``: mu kernel default Xavier, logits column-normalised (0.1), critic value reads the third layer.

On GPU the whole actor / critic forward can run as ONE fused kernel with the weights resident in LDS
(``ops.mlp.fused_mlp_forward``; the actor's 99 KiB of fp32 weights fit a CU's 160 KiB LDS).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .layers import Dense


class MLPActor(nn.Module):
    def __init__(self, ob_dim, ac_dim, discrete=False, ac_scale=2.0, variant="basic", generator=None):
        super().__init__()
        self.ob_dim, self.ac_dim, self.discrete, self.variant = ob_dim, ac_dim, discrete, variant
        self.first_layer = Dense(ob_dim, 128, "lrelu", generator=generator)
        self.second_layer = Dense(128, 128, "lrelu", generator=generator)
        self.third_layer = Dense(128, 64, "lrelu", generator=generator)
        if discrete:
            self.logits = Dense(64, ac_dim, None, kernel_init="xavier" if variant == "basic" else "normc",
                                generator=generator)
        else:
            self.mu_layer = Dense(64, ac_dim, "tanh", kernel_init="xav" if variant == "basic" else "xavier",
                                  generator=generator)
            self.log_std = nn.Parameter(torch.zeros(ac_dim))
            scale = np.broadcast_to(np.asarray(ac_scale if ac_scale is not None else 1.0, dtype=np.float32),
                                    (ac_dim,)).copy()
            self.register_buffer("ac_scale", torch.as_tensor(scale))

    def trunk(self, ob):
        return self.third_layer(self.second_layer(self.first_layer(ob)))

    def forward(self, ob):
        """-> logits ``[B, A]`` (discrete) or mu ``[B, A]`` (continuous)."""
        h = self.trunk(ob.float())
        if self.discrete:
            return self.logits(h)
        return self.mu_layer(h) * self.ac_scale


class MLPCritic(nn.Module):
    def __init__(self, ob_dim, variant="basic", ob_scale=1.0, generator=None):
        super().__init__()
        self.variant = variant
        self.ob_scale = ob_scale
        self.first_layer = Dense(ob_dim, 256, "relu", generator=generator)
        self.second_layer = Dense(256, 128, "relu", generator=generator)
        # basic: built with the TF default (glorot) initialiser and unused by the value path
        self.third_layer = Dense(128, 128, "relu", generator=generator)
        self.value = Dense(128, 1, None, generator=generator)

    def forward(self, ob):
        x1 = self.second_layer(self.first_layer(ob.float() * self.ob_scale))
        if self.variant == "a3c":
            x1 = self.third_layer(x1)
        return self.value(x1).view(-1)
