"""Policy+value model families behind one interface used by every trainer.

``ActorCritic`` API (all batched; ``obs`` is ``[B, ...]``):
  * ``pi_params(obs)``    -> logits ``[B, A]`` or mu ``[B, A]``
  * ``value(obs)``        -> ``[B]``
  * ``forward(obs)``      -> (pi_params, value)
  * ``act(obs, keys)``    -> (action, logp, entropy, value)     (counter-based sampling, see ops.distributions)
  * ``evaluate(obs, a)``  -> (logp, entropy, value)
  * ``param_groups()``    -> {"actor": [...], "critic": [...]} (separate nets, reference) or {"shared": [...]}

Families:
  * :class:`MLPActorCritic` -- the reference's separate actor + critic MLPs, discrete or
    continuous. Used by the reference-parity trainer, CartPole/Pendulum configs and MuJoCo-shape PPO.
  * :class:`CNNActorCritic` -- Nature-CNN shared trunk with categorical head (Atari-shaped configs).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import distributions as D
from .cnn import CNNActorCriticNet
from .mlp import MLPActor, MLPCritic


class ActorCritic(nn.Module):
    discrete = True

    def pi_params(self, obs):
        raise NotImplementedError

    def value(self, obs):
        raise NotImplementedError

    def forward(self, obs):
        return self.pi_params(obs), self.value(obs)

    def log_std_param(self):
        return None

    def dist_logp_entropy(self, pi, actions):
        if self.discrete:
            return D.categorical_logp_entropy(pi, actions)
        return D.gaussian_logp_entropy(pi, self.log_std_param(), actions)

    def sample(self, pi, keys, seed=0):
        if self.discrete:
            return D.categorical_sample(pi, keys, seed)
        return D.gaussian_sample(pi, self.log_std_param(), keys, seed)

    @torch.no_grad()
    def act(self, obs, keys=None, seed=0, deterministic=False):
        pi, v = self.forward(obs)
        if deterministic:
            a = pi.argmax(-1).to(torch.int32) if self.discrete else pi.float()
            logp, ent = self.dist_logp_entropy(pi, a)
            return a, logp, ent, v
        if keys is None:
            keys = torch.randint(0, 2 ** 62, (obs.shape[0],), device=obs.device, dtype=torch.int64)
        a, logp, ent = self.sample(pi, keys, seed)
        return a, logp, ent, v

    def evaluate(self, obs, actions):
        pi, v = self.forward(obs)
        logp, ent = self.dist_logp_entropy(pi, actions)
        return logp, ent, v

    def param_groups(self):
        return {"shared": list(self.parameters())}


class MLPActorCritic(ActorCritic):
    def __init__(self, ob_dim, ac_dim, discrete, ac_scale=None, variant="basic", generator=None):
        super().__init__()
        self.discrete = discrete
        # the reference builds the critic first (Basic_AC/run_AC.py:197-198)
        self.critic = MLPCritic(ob_dim, variant=variant, generator=generator)
        self.actor = MLPActor(ob_dim, ac_dim, discrete, ac_scale if ac_scale is not None else 1.0, variant,
                              generator=generator)

    def pi_params(self, obs):
        return self.actor(obs)

    def value(self, obs):
        return self.critic(obs)

    def log_std_param(self):
        return self.actor.log_std

    def param_groups(self):
        return {"actor": list(self.actor.parameters()), "critic": list(self.critic.parameters())}


class CNNActorCritic(ActorCritic):
    discrete = True

    def __init__(self, num_actions, in_ch=4, hidden=512, generator=None):
        super().__init__()
        self.net = CNNActorCriticNet(num_actions, in_ch, hidden, generator)

    def forward(self, obs):
        return self.net(obs)

    def pi_params(self, obs):
        return self.net(obs)[0]

    def value(self, obs):
        return self.net(obs)[1]

    def param_groups(self):
        """One group; the fc weight LAST in the flat slab. Data parallelism all-reduces the gradient in two buckets:
        the fc weight (95 % of the bytes, final right after the fc-layer backward) overlapped with the conv backward,
        then everything else -- the conv layers and the small head / fc-bias gradients, which the native head
        launches leave as partial planes that only the backward's last (finaliser) launch sums -- so both buckets
        are contiguous ranges and no extra launch is needed before the first all-reduce (algos/engine.py
        tail_bucket)."""
        fck = self.net.trunk.fc.kernel
        return {"shared": [p for p in self.parameters() if p is not fck] + [fck]}


def build_model(env, family="auto", variant="basic", seed=0, hidden=512):
    """Builds the model family for an env bank (``family``: auto | mlp | cnn)."""
    g = torch.Generator().manual_seed(int(seed))
    obs_shape = env.obs_shape
    if family == "auto":
        family = "cnn" if len(obs_shape) == 3 else "mlp"
    if family == "cnn":
        return CNNActorCritic(env.action_space.n, in_ch=obs_shape[0], hidden=hidden, generator=g)
    if env.is_discrete:
        return MLPActorCritic(obs_shape[0], env.action_space.n, True, None, variant, generator=g)
    import numpy as np
    sp = env.action_space
    ac_scale = np.maximum(sp.high, np.abs(sp.low))
    return MLPActorCritic(obs_shape[0], sp.shape[0], False, ac_scale, variant, generator=g)
