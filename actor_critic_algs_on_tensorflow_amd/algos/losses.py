"""Actor-critic losses (kernels K07 / K08 of SURVEY §2.4).

Actor loss of the reference (``Basic_AC/policies.py:72-78``)::

    L_actor = -mean(A_hat * logp(a)) + beta * mean((logp_old - logp(a))^2) - c_ent * mean(H)

(``beta`` is the "KL" coefficient of a squared log-prob-drift *proxy*; ``c_ent`` is called
``gamma`` in the reference). Critic loss ``mean((V - R)^2)`` (``Basic_AC/policies.py:138``).

PPO-clip (extension): ``-mean(min(r A, clip(r, 1-eps, 1+eps) A))`` with ``r = exp(logp - logp_old)``, optional
clipped value loss.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class LossOut:
    total: torch.Tensor
    actor: torch.Tensor
    critic: torch.Tensor
    pg: torch.Tensor
    kl: torch.Tensor
    entropy: torch.Tensor
    clipfrac: torch.Tensor | None = None


def actor_loss(logp, logp_old, adv, entropy, beta, ent_coef):
    pg = -(adv * logp).mean()
    kl = ((logp_old - logp) ** 2).mean()
    ent = entropy.mean()
    return pg + beta * kl - ent_coef * ent, pg, kl, ent


def ppo_actor_loss(logp, logp_old, adv, entropy, clip_eps, ent_coef, beta=0.0):
    ratio = torch.exp(logp - logp_old)
    s1 = ratio * adv
    s2 = torch.clamp(ratio, 1.0 - clip_eps, 1.0 + clip_eps) * adv
    pg = -torch.min(s1, s2).mean()
    kl = ((logp_old - logp) ** 2).mean()
    ent = entropy.mean()
    clipfrac = ((ratio - 1.0).abs() > clip_eps).float().mean()
    return pg + beta * kl - ent_coef * ent, pg, kl, ent, clipfrac


def value_loss(v, returns, v_old=None, clip_eps=None):
    if v_old is not None and clip_eps is not None:
        v_clip = v_old + torch.clamp(v - v_old, -clip_eps, clip_eps)
        return torch.max((v - returns) ** 2, (v_clip - returns) ** 2).mean()
    return ((v - returns) ** 2).mean()
