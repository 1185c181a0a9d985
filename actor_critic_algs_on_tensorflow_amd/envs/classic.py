"""Classic-control envs with the exact gym equations (gym itself is not installed -- SURVEY §7.5 item 8).

* ``CartPole-v0`` / ``CartPole-v1``: gym ``CartPoleEnv`` (Euler integrator, 12 deg / 2.4 thresholds, reward 1
  per step including the terminating one); TimeLimit 200 / 500.
* ``Pendulum-v0``: gym ``PendulumEnv`` v0 (``thdot += (-3g/(2l) sin(th+pi) + 3/(ml^2) u) dt`` ...);
  reward ``-(angle_normalize(th)^2 + .1 thdot^2 + .001 u^2)``; TimeLimit 200; no termination.

These are the envs the reference trains on (``README.md``, ``Basic_AC/run_AC.py:13``). Random resets use the
counter-based hash RNG (:mod:`.rng`) so the HIP kernels (``csrc/kernels/env_classic.hip``) reproduce them.
"""
from __future__ import annotations

import math

import torch

from .. import _native
from . import rng
from .base import VecEnv
from .spaces import Box, Discrete


class CartPoleVecEnv(VecEnv):
    env_id = "CartPole-v1"
    state_dim = 4
    default_max_steps = 500
    observation_space = Box(low=[-4.8, -3.4e38, -0.419, -3.4e38], high=[4.8, 3.4e38, 0.419, 3.4e38])
    action_space = Discrete(2)

    GRAVITY, MASSCART, MASSPOLE, LENGTH, FORCE_MAG, TAU = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
    THETA_LIMIT = 12 * 2 * math.pi / 360
    X_LIMIT = 2.4

    @property
    def frame_shape(self):
        return (4,)

    def _reset_state(self, mask):
        ids = self.env_ids
        for j in range(4):
            u = rng.uniform(self.seed, ids, self.tg, 100 + j)
            self.state[:, j] = torch.where(mask, u * 0.1 - 0.05, self.state[:, j])

    def _dynamics(self, actions):
        x, x_dot, th, th_dot = self.state.unbind(1)
        total_mass = self.MASSPOLE + self.MASSCART
        pml = self.MASSPOLE * self.LENGTH
        force = torch.where(actions.view(-1).long() == 1, torch.full_like(x, self.FORCE_MAG),
                            torch.full_like(x, -self.FORCE_MAG))
        c, s = torch.cos(th), torch.sin(th)
        temp = (force + pml * th_dot * th_dot * s) / total_mass
        thacc = (self.GRAVITY * s - c * temp) / (self.LENGTH * (4.0 / 3.0 - self.MASSPOLE * c * c / total_mass))
        xacc = temp - pml * thacc * c / total_mass
        x = x + self.TAU * x_dot
        x_dot = x_dot + self.TAU * xacc
        th = th + self.TAU * th_dot
        th_dot = th_dot + self.TAU * thacc
        self.state.copy_(torch.stack([x, x_dot, th, th_dot], 1))
        term = (x < -self.X_LIMIT) | (x > self.X_LIMIT) | (th < -self.THETA_LIMIT) | (th > self.THETA_LIMIT)
        return torch.ones_like(x), term

    def _frame(self):
        return self.state.clone()

    native_final_obs = True   # the kernel can write the terminal observation (time-limit bootstrap)

    def _native_step(self, actions, prev, out, rew, done, trunc, final_out=None):
        _native.require().env_step_cartpole(
            self.state, self.t, self.tg, self.ep_ret, self.ep_stats, self.env_ids, actions.to(torch.int32),
            prev, out, rew, done, trunc, self.seed, self.max_episode_steps, self.frame_stack,
            final_out)


class CartPoleV0VecEnv(CartPoleVecEnv):
    env_id = "CartPole-v0"
    default_max_steps = 200


def angle_normalize(x):
    return torch.remainder(x + math.pi, 2 * math.pi) - math.pi


class PendulumVecEnv(VecEnv):
    env_id = "Pendulum-v0"
    state_dim = 2
    default_max_steps = 200
    observation_space = Box(low=[-1.0, -1.0, -8.0], high=[1.0, 1.0, 8.0])
    action_space = Box(low=[-2.0], high=[2.0])

    MAX_SPEED, MAX_TORQUE, DT, G, M, L = 8.0, 2.0, 0.05, 10.0, 1.0, 1.0

    @property
    def frame_shape(self):
        return (3,)

    def _reset_state(self, mask):
        ids = self.env_ids
        th = rng.uniform(self.seed, ids, self.tg, 100) * (2 * math.pi) - math.pi
        thd = rng.uniform(self.seed, ids, self.tg, 101) * 2.0 - 1.0
        self.state[:, 0] = torch.where(mask, th, self.state[:, 0])
        self.state[:, 1] = torch.where(mask, thd, self.state[:, 1])

    def _dynamics(self, actions):
        th, thdot = self.state.unbind(1)
        u = torch.clamp(actions.reshape(self.num_envs, -1)[:, 0].float(), -self.MAX_TORQUE, self.MAX_TORQUE)
        costs = angle_normalize(th) ** 2 + 0.1 * thdot ** 2 + 0.001 * (u ** 2)
        newthdot = thdot + (-3 * self.G / (2 * self.L) * torch.sin(th + math.pi)
                            + 3.0 / (self.M * self.L ** 2) * u) * self.DT
        newth = th + newthdot * self.DT
        newthdot = torch.clamp(newthdot, -self.MAX_SPEED, self.MAX_SPEED)
        self.state.copy_(torch.stack([newth, newthdot], 1))
        return -costs, torch.zeros_like(th, dtype=torch.bool)

    def _frame(self):
        th, thdot = self.state.unbind(1)
        return torch.stack([torch.cos(th), torch.sin(th), thdot], 1)

    native_final_obs = True   # the kernel can write the terminal observation (time-limit bootstrap)

    def _native_step(self, actions, prev, out, rew, done, trunc, final_out=None):
        _native.require().env_step_pendulum(
            self.state, self.t, self.tg, self.ep_ret, self.ep_stats, self.env_ids,
            actions.reshape(self.num_envs, -1).float().contiguous(),
            prev, out, rew, done, trunc, self.seed, self.max_episode_steps, self.frame_stack,
            final_out)
