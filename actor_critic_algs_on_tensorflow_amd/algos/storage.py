"""Preallocated ``[T, N]`` rollout storage living on the device.

The reference accumulates Python lists per episode (``Basic_AC/run_AC.py:209-236``). Here a rollout of T steps
over N envs writes into fixed slabs (static addresses, so the rollout can be hipGraph-captured)::

    obs      [T+1, N, *obs_shape]   (uint8 frames for Atari: 32 envs x 6 slots x 28 KiB = 5.4 MB)
    actions  [T, N] int32 | [T, N, A] fp32
    logp, entropy, rewards, dones, truncated   [T, N]
    values   [T+1, N]                           (values[T] = bootstrap value of the last observation)

Sizing for 288 GB HBM: even 8192 envs x 128 steps of Atari frames is ~7.4 GB, so N and T are pure
throughput knobs.
"""
from __future__ import annotations

import torch


class RolloutStorage:
    def __init__(self, T, N, obs_shape, obs_dtype, action_shape, action_dtype, device):
        self.T, self.N = T, N
        dev = torch.device(device)
        self.obs = torch.zeros((T + 1, N) + tuple(obs_shape), dtype=obs_dtype, device=dev)
        self.actions = torch.zeros((T, N) + tuple(action_shape), dtype=action_dtype, device=dev)
        self.logp = torch.zeros(T, N, dtype=torch.float32, device=dev)
        self.entropy = torch.zeros(T, N, dtype=torch.float32, device=dev)
        self.rewards = torch.zeros(T, N, dtype=torch.float32, device=dev)
        self.dones = torch.zeros(T, N, dtype=torch.uint8, device=dev)
        self.truncated = torch.zeros(T, N, dtype=torch.uint8, device=dev)
        self.values = torch.zeros(T + 1, N, dtype=torch.float32, device=dev)
        self.keys = torch.zeros(T, N, dtype=torch.int64, device=dev)

    def flat(self, name):
        x = getattr(self, name)
        if name in ("obs", "values"):
            x = x[:self.T]
        return x.reshape((self.T * self.N,) + tuple(x.shape[2:]))

    def roll_over(self):
        """The last observation becomes the first of the next rollout."""
        self.obs[0].copy_(self.obs[self.T])

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in (self.obs, self.actions, self.logp, self.entropy,
                                                          self.rewards, self.dones, self.values, self.keys))
