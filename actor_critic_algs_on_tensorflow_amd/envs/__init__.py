"""Env registry: ``make(env_id, num_envs, device, seed)`` -> a device-resident :class:`VecEnv` bank.

Ids follow gym so reference command lines (``--env Pendulum-v0``, ``--env CartPole-v0``) keep working.
``get_roll_params`` reproduces the reference's per-env rollout sizing (``Basic_AC/run_AC.py:124-136``,
``A3C/process.py:100-109``).
"""
from __future__ import annotations

from .atari import BreakoutShapeVecEnv, PongVecEnv
from .base import VecEnv
from .classic import CartPoleV0VecEnv, CartPoleVecEnv, PendulumVecEnv
from .mujoco import MujocoShapeVecEnv
from .spaces import Box, Discrete, EnvSpec

REGISTRY = {
    "CartPole-v0": CartPoleV0VecEnv,
    "CartPole-v1": CartPoleVecEnv,
    "Pendulum-v0": PendulumVecEnv,
    "Pendulum-v1": PendulumVecEnv,
    "PongNoFrameskip-v4": PongVecEnv,
    "Pong": PongVecEnv,
    "BreakoutNoFrameskip-v4": BreakoutShapeVecEnv,
    "Breakout": BreakoutShapeVecEnv,
    "HalfCheetahShape-v0": MujocoShapeVecEnv,
    "MujocoShape": MujocoShapeVecEnv,
}


def make(env_id, num_envs=1, device="cpu", seed=0, **kw) -> VecEnv:
    try:
        cls = REGISTRY[env_id]
    except KeyError:
        raise KeyError(f"unknown env {env_id!r}; known: {sorted(REGISTRY)}") from None
    return cls(num_envs, device=device, seed=seed, **kw)


def get_roll_params(env_id, variant="basic"):
    """Returns ``(max_path_length, ep_length_stop)``.

    ``variant="basic"``: defaults (1200, 3000); Pendulum-v0 -> (400, 1400); else if the env has a time limit L,
    (L, min(4L, 3000)). ``variant="a3c"``: (L, min(6L, 3000)) with no Pendulum special case.
    """
    cls = REGISTRY[env_id]
    max_steps = cls.default_max_steps
    if variant == "basic":
        if env_id == "Pendulum-v0":
            return 400, 1400
        if max_steps is not None:
            return max_steps, min(max_steps * 4, 3000)
        return 1200, 3000
    if max_steps is not None:
        return max_steps, min(max_steps * 6, 3000)
    return 1200, 3000


__all__ = ["make", "get_roll_params", "REGISTRY", "VecEnv", "Box", "Discrete", "EnvSpec", "PongVecEnv",
           "CartPoleVecEnv", "PendulumVecEnv", "MujocoShapeVecEnv", "BreakoutShapeVecEnv", "CartPoleV0VecEnv"]
