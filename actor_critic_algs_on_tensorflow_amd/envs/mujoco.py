"""MuJoCo-shaped continuous-control env (BASELINE config 5: "MuJoCo-shape obs PPO, diagonal-Gaussian").

MuJoCo is not available; this env reproduces the *shapes* of HalfCheetah-v2 (17-d observation, 6-d action in
[-1, 1], 1000-step episodes, no termination) with a stable linear-Gaussian system::

    s' = A s + B a + noise,   r = s'[8] - 0.1 |a|^2

``A`` (a damped rotation, spectral radius 0.97) and ``B`` are generated deterministically from ``dyn_seed`` and
passed to the HIP kernel as buffers, so the kernel and this oracle run identical dynamics. Reward 0.1-scaled
forward "velocity" (state 8) makes it learnable: the optimal policy pushes s[8] up through B.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native
from . import rng
from .base import VecEnv
from .spaces import Box

OBS_DIM, ACT_DIM = 17, 6


def make_dynamics(dyn_seed=1234):
    g = np.random.default_rng(dyn_seed)
    q, _ = np.linalg.qr(g.standard_normal((OBS_DIM, OBS_DIM)))
    A = 0.97 * q
    B = 0.3 * g.standard_normal((OBS_DIM, ACT_DIM)) / np.sqrt(ACT_DIM)
    return A.astype(np.float32), B.astype(np.float32)


class MujocoShapeVecEnv(VecEnv):
    env_id = "HalfCheetahShape-v0"
    state_dim = OBS_DIM
    default_max_steps = 1000
    observation_space = Box(low=np.full(OBS_DIM, -np.inf), high=np.full(OBS_DIM, np.inf))
    action_space = Box(low=-np.ones(ACT_DIM), high=np.ones(ACT_DIM))

    def __init__(self, num_envs, device="cpu", seed=0, max_episode_steps=None, env_offset=0, frame_stack=1,
                 dyn_seed=1234):
        super().__init__(num_envs, device, seed, max_episode_steps, env_offset, frame_stack)
        A, B = make_dynamics(dyn_seed)
        self.A = torch.as_tensor(A, device=self.device)   # [17, 17]
        self.B = torch.as_tensor(B, device=self.device)   # [17, 6]

    @property
    def frame_shape(self):
        return (OBS_DIM,)

    def _reset_state(self, mask):
        ids = self.env_ids
        for j in range(OBS_DIM):
            u = rng.uniform(self.seed, ids, self.tg, 100 + j)
            self.state[:, j] = torch.where(mask, (u - 0.5) * 0.2, self.state[:, j])

    def _dynamics(self, actions):
        a = torch.clamp(actions.reshape(self.num_envs, ACT_DIM).float(), -1.0, 1.0)
        ids = self.env_ids
        noise = torch.stack([rng.uniform(self.seed, ids, self.tg, 300 + j) for j in range(OBS_DIM)], 1)
        s = self.state @ self.A.t() + a @ self.B.t() + (noise - 0.5) * 0.02
        self.state.copy_(s)
        rew = s[:, 8] - 0.1 * (a * a).sum(1)
        return rew, torch.zeros_like(rew, dtype=torch.bool)

    def _frame(self):
        return self.state.clone()

    native_final_obs = True   # the kernel can write the terminal observation (time-limit bootstrap)

    def _native_step(self, actions, prev, out, rew, done, trunc, final_out=None):
        _native.require().env_step_linear(
            self.state, self.t, self.tg, self.ep_ret, self.ep_stats, self.env_ids,
            actions.reshape(self.num_envs, ACT_DIM).float().contiguous(), self.A, self.B,
            prev, out, rew, done, trunc, self.seed, self.max_episode_steps, self.frame_stack,
            final_out)
