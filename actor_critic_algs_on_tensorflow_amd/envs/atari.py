"""Atari-shaped synthetic env: a Pong-like game rendered straight to 84x84 uint8 frames.

BASELINE.json's headline config is "Atari-Pong A2C, 32 synthetic 84x84x4 vec-envs". ALE is not available, so
this env is *shape-faithful* (84x84 grayscale uint8 frames, 4-frame stack, frameskip 4, 6 Pong actions, +-1
rewards, games to 21 points) and also genuinely learnable: the agent's paddle (right) must intercept a ball
against a rate-limited opponent (left).

Per env step the bank runs 4 physics sub-steps, renders one frame and pushes it into the ``[N, 4, 84, 84]``
stack (new episodes get 4 copies of their first frame -- the ``Framer`` padding rule of
``Basic_AC/run_AC.py:37-40``). On GPU this whole step is ONE launch of ``env_step_pong``
(``csrc/kernels/env_atari.hip``): one workgroup per env renders its frame with 16-byte stores while lane 0
advanced the physics. The oracle below is the specification that kernel is tested against.

Action map (ALE Pong minimal set): 0 NOOP, 1 FIRE, 2 RIGHT(up), 3 LEFT(down), 4 RIGHTFIRE(up), 5 LEFTFIRE(down).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native
from . import rng
from .base import VecEnv
from .spaces import Box, Discrete

H = W = 84
FIELD_TOP, FIELD_BOT = 10.0, 74.0
BALL = 2.0
PADDLE_H, PADDLE_W = 8.0, 2.0
AGENT_X, OPP_X = 74.0, 8.0          # left column of each paddle
AGENT_SPEED, OPP_SPEED = 2.0, 1.25
BALL_VX = 1.5
SUBSTEPS = 4
WIN_SCORE = 21.0
BG, WALL, OPP_C, AGENT_C, BALL_C = 87, 236, 130, 200, 255


class PongVecEnv(VecEnv):
    env_id = "PongNoFrameskip-v4"
    state_dim = 8   # bx, by, vx, vy, pa, po, score_agent, score_opp
    default_max_steps = 10000
    obs_dtype = torch.uint8
    observation_space = Box(low=np.zeros((4, H, W)), high=np.full((4, H, W), 255.0))
    action_space = Discrete(6)

    def __init__(self, num_envs, device="cpu", seed=0, max_episode_steps=None, env_offset=0, frame_stack=4):
        super().__init__(num_envs, device, seed, max_episode_steps, env_offset, frame_stack)
        ys = torch.arange(H, device=self.device, dtype=torch.float32).view(1, H, 1)
        xs = torch.arange(W, device=self.device, dtype=torch.float32).view(1, 1, W)
        self._ys, self._xs = ys, xs

    @property
    def frame_shape(self):
        return (H, W)

    # -- dynamics --------------------------------------------------------------------------------------------
    def _serve(self, mask, stream0):
        ids = self.env_ids
        u0 = rng.uniform(self.seed, ids, self.tg, stream0)
        u1 = rng.uniform(self.seed, ids, self.tg, stream0 + 1)
        u2 = rng.uniform(self.seed, ids, self.tg, stream0 + 2)
        s = self.state
        s[:, 0] = torch.where(mask, torch.full_like(u0, 41.0), s[:, 0])
        s[:, 1] = torch.where(mask, 30.0 + u0 * 24.0, s[:, 1])
        s[:, 2] = torch.where(mask, torch.where(u1 < 0.5, torch.full_like(u1, BALL_VX),
                                                 torch.full_like(u1, -BALL_VX)), s[:, 2])
        s[:, 3] = torch.where(mask, (u2 - 0.5) * 2.0, s[:, 3])

    def _reset_state(self, mask):
        s = self.state
        mid = 0.5 * (FIELD_TOP + FIELD_BOT)
        for j, v in ((4, mid), (5, mid), (6, 0.0), (7, 0.0)):
            s[:, j] = torch.where(mask, torch.full_like(s[:, j], v), s[:, j])
        self._serve(mask, 100)

    def _dynamics(self, actions):
        a = actions.view(-1).long()
        dirn = torch.zeros(self.num_envs, device=self.device)
        dirn = torch.where((a == 2) | (a == 4), torch.full_like(dirn, -1.0), dirn)
        dirn = torch.where((a == 3) | (a == 5), torch.full_like(dirn, 1.0), dirn)
        rew = torch.zeros(self.num_envs, device=self.device)
        lo, hi = FIELD_TOP + PADDLE_H / 2, FIELD_BOT - PADDLE_H / 2
        for sub in range(SUBSTEPS):
            bx, by, vx, vy, pa, po, sa, so = [c.clone() for c in self.state.unbind(1)]
            pa = torch.clamp(pa + dirn * AGENT_SPEED, lo, hi)
            po = torch.clamp(po + torch.clamp(by + 1.0 - po, -OPP_SPEED, OPP_SPEED), lo, hi)
            bx = bx + vx
            by = by + vy
            top = by < FIELD_TOP
            by = torch.where(top, 2 * FIELD_TOP - by, by)
            vy = torch.where(top, -vy, vy)
            bot = by > FIELD_BOT - BALL
            by = torch.where(bot, 2 * (FIELD_BOT - BALL) - by, by)
            vy = torch.where(bot, -vy, vy)
            hit_a = (vx > 0) & (bx + BALL >= AGENT_X) & (bx + BALL - vx < AGENT_X) & \
                    (torch.abs(by + 1.0 - pa) <= PADDLE_H / 2 + 1.0)
            vy = torch.where(hit_a, torch.clamp(vy + 0.25 * (by + 1.0 - pa), -2.0, 2.0), vy)
            bx = torch.where(hit_a, torch.full_like(bx, AGENT_X - BALL), bx)
            vx = torch.where(hit_a, -vx, vx)
            edge = OPP_X + PADDLE_W
            hit_o = (vx < 0) & (bx <= edge) & (bx - vx > edge) & (torch.abs(by + 1.0 - po) <= PADDLE_H / 2 + 1.0)
            vy = torch.where(hit_o, torch.clamp(vy + 0.25 * (by + 1.0 - po), -2.0, 2.0), vy)
            bx = torch.where(hit_o, torch.full_like(bx, edge), bx)
            vx = torch.where(hit_o, -vx, vx)
            miss_a = bx > float(W)
            miss_o = bx < -BALL
            rew = rew + miss_o.float() - miss_a.float()
            sa = sa + miss_o.float()
            so = so + miss_a.float()
            self.state.copy_(torch.stack([bx, by, vx, vy, pa, po, sa, so], 1))
            self._serve(miss_a | miss_o, 200 + 4 * sub)
        term = (self.state[:, 6] >= WIN_SCORE) | (self.state[:, 7] >= WIN_SCORE)
        return rew, term

    def _frame(self):
        s = self.state
        ys, xs = self._ys, self._xs
        img = torch.full((self.num_envs, H, W), BG, dtype=torch.uint8, device=self.device)
        wall = (ys < FIELD_TOP) | (ys >= FIELD_BOT)
        img = torch.where(wall.expand_as(img), torch.full_like(img, WALL), img)
        pa0 = torch.floor(s[:, 4] - PADDLE_H / 2).view(-1, 1, 1)
        po0 = torch.floor(s[:, 5] - PADDLE_H / 2).view(-1, 1, 1)
        agent = (xs >= AGENT_X) & (xs < AGENT_X + PADDLE_W) & (ys >= pa0) & (ys < pa0 + PADDLE_H)
        opp = (xs >= OPP_X) & (xs < OPP_X + PADDLE_W) & (ys >= po0) & (ys < po0 + PADDLE_H)
        img = torch.where(agent, torch.full_like(img, AGENT_C), img)
        img = torch.where(opp, torch.full_like(img, OPP_C), img)
        bx0 = torch.floor(s[:, 0]).view(-1, 1, 1)
        by0 = torch.floor(s[:, 1]).view(-1, 1, 1)
        ball = (xs >= bx0) & (xs < bx0 + BALL) & (ys >= by0) & (ys < by0 + BALL)
        img = torch.where(ball, torch.full_like(img, BALL_C), img)
        return img

    def _native_step(self, actions, prev, out, rew, done, trunc):
        _native.require().env_step_pong(
            self.state, self.t, self.tg, self.ep_ret, self.ep_stats, self.env_ids, actions.to(torch.int32),
            prev, out, rew, done, trunc, self.seed, self.max_episode_steps, self.frame_stack)


class BreakoutShapeVecEnv(PongVecEnv):
    """Breakout-shape alias (BASELINE config 3): same 84x84x4 uint8 observation pipeline, 4 actions.

    The dynamics are the Pong game with Breakout's action-set size (NOOP, FIRE, RIGHT, LEFT); what the
    benchmark measures (CNN, PPO, GAE over 128 envs) depends only on the shapes.
    """

    env_id = "BreakoutNoFrameskip-v4"
    action_space = Discrete(4)
