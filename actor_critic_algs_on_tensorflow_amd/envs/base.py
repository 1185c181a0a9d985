"""Vectorised, device-resident environment bank.

The reference steps ONE gym env per process at batch 1 (``Basic_AC/run_AC.py:82-107``). Here each GPU owns a
bank of ``N`` envs whose state lives in HBM; one ``step`` is one kernel launch for the whole bank (the
``csrc/kernels/env_*.hip`` kernels) that also auto-resets finished envs, applies the frame-stack shift and
accumulates episode statistics on device, so a rollout step never synchronises with the host and can be
captured into a hipGraph.

Every env has a pure-PyTorch implementation of the same dynamics (the oracle, used on CPU and in tests) and,
on GPU, a HIP kernel that must match it (``tests/test_envs.py``).

Conventions
  * ``step(actions)`` returns ``(obs, reward, done, info)``; ``done = terminated | truncated``; when an env is
    done the returned observation is already the first observation of its next episode (gym VectorEnv rule).
  * time-limit truncation is reported separately in ``info['truncated']``; the reference treats it as terminal
     and the trainers do the same unless ``bootstrap_on_timeout`` is set.
  * episode statistics: ``ep_stats`` = device tensor ``[3]`` (sum of finished-episode returns, count, sum of
    lengths) that the trainer drains when it logs.
"""
from __future__ import annotations

import torch

from .. import _native
from .spaces import Box, Discrete, EnvSpec


def _slot_property(name):
    def get(self):
        return self._sbuf[name][self.parity]

    def set(self, value):   # in-place operators re-assign the same view; anything else is copied in
        cur = self._sbuf[name][self.parity]
        if value is not cur:
            cur.copy_(value)
    return property(get, set)


class VecEnv:
    env_id = "base"
    observation_space = None
    action_space = None
    obs_dtype = torch.float32
    state_dim = 0

    state = _slot_property("state")
    t = _slot_property("t")
    tg = _slot_property("tg")
    ep_ret = _slot_property("ep_ret")

    def __init__(self, num_envs, device="cpu", seed=0, max_episode_steps=None, env_offset=0, frame_stack=1):
        self.num_envs = int(num_envs)
        self.device = torch.device(device)
        self.seed = int(seed) & 0xFFFFFFFF
        self.max_episode_steps = max_episode_steps if max_episode_steps is not None else self.default_max_steps
        self.env_offset = int(env_offset)
        self.frame_stack = int(frame_stack)
        N, dev = self.num_envs, self.device
        # per-env state, double-buffered: ``state`` / ``t`` / ``tg`` / ``ep_ret`` are views of slot ``parity``. Kernels
        # that read the state in several workgroups while one of them commits the step (the fused rollout step of
        # the CNN engine) read the current slot and write the other; :meth:`flip` then makes it current.
        self._sbuf = {
            "state": torch.zeros(2, N, self.state_dim, dtype=torch.float32, device=dev),
            "t": torch.zeros(2, N, dtype=torch.int32, device=dev),        # steps in the current episode
            "tg": torch.zeros(2, N, dtype=torch.int64, device=dev),       # global step counter (RNG key)
            "ep_ret": torch.zeros(2, N, dtype=torch.float32, device=dev),  # running episode return
        }
        self.parity = 0
        self.ep_stats = torch.zeros(3, dtype=torch.float32, device=dev)  # [sum_ret, count, sum_len]
        self.env_ids = torch.arange(N, dtype=torch.int64, device=dev) + self.env_offset
        self.obs = torch.zeros((N,) + self.obs_shape, dtype=self.obs_dtype, device=dev)
        self.reward = torch.zeros(N, dtype=torch.float32, device=dev)
        self.done = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.truncated = torch.zeros(N, dtype=torch.uint8, device=dev)
        # gym-style single-env adapters need the terminal observation the auto-reset overwrites (oracle path only)
        self.keep_final_obs = False
        self.final_obs = None

    def next_state(self):
        """(state, t, tg, ep_ret) views of the non-current parity slot."""
        q = 1 - self.parity
        return tuple(self._sbuf[k][q] for k in ("state", "t", "tg", "ep_ret"))

    def flip(self):
        """The other parity slot becomes current (after a kernel committed the step into it)."""
        self.parity ^= 1

    # -- shape info -------------------------------------------------------------------------------------------
    default_max_steps = 1000

    @property
    def frame_shape(self):
        raise NotImplementedError

    @property
    def obs_shape(self):
        fs = self.frame_shape
        if self.frame_stack == 1 and self.obs_dtype != torch.uint8:
            return fs
        if self.obs_dtype == torch.uint8:          # image: [k, H, W]
            return (self.frame_stack,) + tuple(fs[-2:])
        return (fs[0] * self.frame_stack,)          # vector: concat (Framer semantics)

    @property
    def spec(self):
        return EnvSpec(self.env_id, self.max_episode_steps)

    @property
    def is_discrete(self):
        return isinstance(self.action_space, Discrete)

    # -- dynamics (oracle) ---------------------------------------------------------------------------------------
    def _reset_state(self, mask):
        """Re-initialise ``self.state`` rows where ``mask``; must use only ``rng.uniform`` keyed on ``tg``."""
        raise NotImplementedError

    def _dynamics(self, actions):
        """Advance ``self.state`` one env step; returns (reward, terminated) float32/bool tensors."""
        raise NotImplementedError

    def _frame(self):
        """Current single frame / observation vector for every env, shape ``[N, *frame_shape]``."""
        raise NotImplementedError

    # -- public API ------------------------------------------------------------------------------------------
    def reset(self, out=None):
        allm = torch.ones(self.num_envs, dtype=torch.bool, device=self.device)
        self._reset_state(allm)
        self.t.zero_()
        self.ep_ret.zero_()
        f = self._frame()
        self._stack_reset(f, self.obs, allm)
        if out is not None:
            out.copy_(self.obs)
            return out
        return self.obs

    def _stack_reset(self, frame, obs, mask):
        k = self.frame_stack
        if self.obs_dtype == torch.uint8:
            st = frame.unsqueeze(1).expand(-1, k, -1, -1)
        else:
            st = frame.repeat(1, k)
        m = mask.view(-1, *([1] * (obs.dim() - 1)))
        obs.copy_(torch.where(m, st.to(obs.dtype), obs))

    def _stack_push(self, frame, prev, out):
        k = self.frame_stack
        if k == 1:
            out.copy_(frame.to(out.dtype))
            return
        if self.obs_dtype == torch.uint8:
            new = torch.cat([prev[:, 1:], frame.unsqueeze(1).to(out.dtype)], dim=1)
        else:
            d = frame.shape[1]
            new = torch.cat([prev[:, d:], frame.to(out.dtype)], dim=1)
        out.copy_(new)

    native_final_obs = False   # env kernel writes the terminal observation (subclasses with that support)

    def step(self, actions, prev_obs=None, obs_out=None, reward_out=None, done_out=None, trunc_out=None,
             final_out=None):
        """One env step for the whole bank.

        ``prev_obs`` / ``obs_out`` let a rollout read the stack from slot ``t`` and write slot ``t+1`` of its
        buffer directly, and ``reward_out`` / ``done_out`` / ``trunc_out`` receive the transition's reward, done and
        truncation flags (static addresses => hipGraph-capturable; on GPU the env kernel writes them in place, no
        copies). Defaults: the bank's own buffers. With ``keep_final_obs`` the stack holding the transition's new
        frame before any auto-reset (the terminal observation of finished episodes) goes to ``final_out`` (default
        ``self.final_obs``).
        """
        prev = self.obs if prev_obs is None else prev_obs
        out = self.obs if obs_out is None else obs_out
        rew = self.reward if reward_out is None else reward_out
        done = self.done if done_out is None else done_out
        trunc = self.truncated if trunc_out is None else trunc_out
        if prev.data_ptr() == out.data_ptr():
            prev = prev.clone()   # the kernels read the old stack while writing the new one
        native = _native.use_native(self.state) and (not self.keep_final_obs or self.native_final_obs)
        if native and self.keep_final_obs:
            if final_out is None:
                if self.final_obs is None:
                    self.final_obs = torch.empty_like(out)
                final_out = self.final_obs
            self._native_step(actions, prev, out, rew, done, trunc, final_out)
        elif native:
            self._native_step(actions, prev, out, rew, done, trunc)
        else:
            self._torch_step(actions, prev, out)
            if self.keep_final_obs and final_out is not None:
                final_out.copy_(self.final_obs)
            for src, dst in ((self.reward, rew), (self.done, done), (self.truncated, trunc)):
                if dst.data_ptr() != src.data_ptr():
                    dst.copy_(src)
        info = {"truncated": trunc, "ep_stats": self.ep_stats}
        return out, rew, done, info

    @torch.no_grad()
    def _torch_step(self, actions, prev, out):
        self.tg += 1
        rew, term = self._dynamics(actions)
        self.t += 1
        trunc = (self.t >= self.max_episode_steps) & ~term
        done = term | trunc
        self.ep_ret += rew
        fin_ret = torch.where(done, self.ep_ret, torch.zeros_like(self.ep_ret))
        self.ep_stats[0] += fin_ret.sum()
        self.ep_stats[1] += done.float().sum()
        self.ep_stats[2] += torch.where(done, self.t.float(), torch.zeros_like(rew)).sum()
        self.reward.copy_(rew)
        self.done.copy_(done.to(torch.uint8))
        self.truncated.copy_(trunc.to(torch.uint8))
        if self.keep_final_obs:
            if self.final_obs is None:
                self.final_obs = torch.empty_like(out)
            self._stack_push(self._frame(), prev, self.final_obs)
        # auto-reset (on the host, skipped when no env finished: the counter RNG consumes no state)
        if done.device.type != "cpu" or bool(done.any()):
            self._reset_state(done)
        self.t.masked_fill_(done, 0)
        self.ep_ret.masked_fill_(done, 0.0)
        f = self._frame()
        self._stack_push(f, prev, out)
        self._stack_reset(f, out, done)

    def _native_step(self, actions, prev, out, rew, done, trunc):
        raise NotImplementedError(f"{type(self).__name__} has no native kernel")

    def drain_episode_stats(self):
        """Host read of (mean finished return, episodes, mean length) since the last drain (syncs)."""
        s = self.ep_stats.detach().cpu().clone()
        self.ep_stats.zero_()
        n = float(s[1])
        return (float(s[0]) / n if n else float("nan")), int(n), (float(s[2]) / n if n else float("nan"))

    def sample_actions(self, generator=None):
        if self.is_discrete:
            return torch.randint(0, self.action_space.n, (self.num_envs,), device=self.device,
                                 dtype=torch.int32, generator=generator)
        lo = torch.as_tensor(self.action_space.low, device=self.device)
        hi = torch.as_tensor(self.action_space.high, device=self.device)
        u = torch.rand((self.num_envs,) + tuple(self.action_space.shape), device=self.device, generator=generator)
        return lo + (hi - lo) * u
