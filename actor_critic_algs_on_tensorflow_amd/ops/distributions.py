"""Policy heads: categorical and diagonal-Gaussian (kernels K04 / K05 of SURVEY §2.4).

Reference semantics (``Basic_AC/policies.py:47-69``, ``A3C/policies.py:49-72``):
  * categorical: ``logp = log_softmax(logits + 1e-8)[a]`` (the +1e-8 shift is a no-op),
    ``H = -sum softmax * log_softmax``; sampling ``tf.multinomial``.
  * Gaussian: ``mu = tanh(z) * ac_scale`` (applied by the model), ``sigma = exp(clip(log_std, -2.5, 2.5))``,
    ``logp = sum_i log N(a_i; mu_i, sigma_i)``, ``H = sum_i (1/2 + 1/2 log 2 pi + log sigma_i)``; actions are not
    clipped to the bounds -- envs clip.

Sampling is counter-based: row ``b`` draws with key ``(seed, keys[b], stream)`` through the same hash as the env
bank (:mod:`..envs.rng`), Gumbel-max for categorical and Box-Muller for Gaussian. On GPU one fused HIP launch
(``csrc/kernels/heads.hip``) produces action, log-prob and entropy per row; the functions named ``*_ref`` are
the PyTorch oracles.
"""
from __future__ import annotations

import math

import torch

from .. import _native
from ..envs import rng

LOG_STD_MIN, LOG_STD_MAX = -2.5, 2.5
HALF_LOG_2PI = 0.5 * math.log(2 * math.pi)


def _u_open(seed, keys, stream):
    """Uniform in (0, 1): ((h >> 8) + 0.5) / 2^24, h = hash(seed, key_lo32, key_hi32, stream)."""
    keys = torch.as_tensor(keys, dtype=torch.int64)
    h = rng.hash_u32(seed, keys & rng.M32, (keys >> 32) & rng.M32, stream)
    return ((h >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)


# ------------------------------------------------------------------ categorical
def categorical_logp_entropy(logits, actions):
    lp = torch.log_softmax(logits.float(), dim=-1)
    logp = lp.gather(-1, actions.long().view(-1, 1)).squeeze(-1)
    ent = -(lp.exp() * lp).sum(-1)
    return logp, ent


def categorical_sample_ref(logits, keys, seed):
    B, A = logits.shape
    k = keys.view(B, 1).to(torch.int64)
    streams = torch.arange(A, device=logits.device, dtype=torch.int64).view(1, A)
    u = _u_open(seed, k, streams)
    g = -torch.log(-torch.log(u))
    act = torch.argmax(logits.float() + g, dim=-1).to(torch.int32)
    logp, ent = categorical_logp_entropy(logits, act)
    return act, logp, ent


def categorical_sample(logits, keys, seed=0):
    """-> (actions int32 [B], logp fp32 [B], entropy fp32 [B])."""
    if _native.use_native(logits):
        B = logits.shape[0]
        act = torch.empty(B, dtype=torch.int32, device=logits.device)
        logp = torch.empty(B, dtype=torch.float32, device=logits.device)
        ent = torch.empty_like(logp)
        _native.require().categorical_sample(logits.contiguous(), keys.to(torch.int64).contiguous(), int(seed),
                                             act, logp, ent)
        return act, logp, ent
    return categorical_sample_ref(logits, keys, seed)


# ------------------------------------------------------------------ gaussian
def gaussian_logp_entropy(mu, log_std, actions):
    ls = torch.clamp(log_std.float(), LOG_STD_MIN, LOG_STD_MAX).expand_as(mu)
    z = (actions.float() - mu.float()) * torch.exp(-ls)
    logp = (-0.5 * z * z - ls - HALF_LOG_2PI).sum(-1)
    ent = (0.5 + HALF_LOG_2PI + ls).sum(-1)
    return logp, ent


def gaussian_sample_ref(mu, log_std, keys, seed):
    B, A = mu.shape
    k = keys.view(B, 1).to(torch.int64)
    j = torch.arange(A, device=mu.device, dtype=torch.int64).view(1, A)
    u1 = _u_open(seed, k, 2 * j)
    u2 = _u_open(seed, k, 2 * j + 1)
    eps = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2 * math.pi * u2)
    ls = torch.clamp(log_std.float(), LOG_STD_MIN, LOG_STD_MAX).view(1, A)
    act = mu.float() + torch.exp(ls) * eps
    logp, ent = gaussian_logp_entropy(mu, log_std, act)
    return act, logp, ent


def gaussian_sample(mu, log_std, keys, seed=0):
    """-> (actions fp32 [B, A], logp [B], entropy [B])."""
    if _native.use_native(mu):
        B, A = mu.shape
        act = torch.empty(B, A, dtype=torch.float32, device=mu.device)
        logp = torch.empty(B, dtype=torch.float32, device=mu.device)
        ent = torch.empty_like(logp)
        _native.require().gaussian_sample(mu.float().contiguous(), log_std.float().contiguous(),
                                          keys.to(torch.int64).contiguous(), int(seed), act, logp, ent)
        return act, logp, ent
    return gaussian_sample_ref(mu, log_std, keys, seed)
