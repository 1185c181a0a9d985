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


class _ObsRing:
    """``obs[t]`` of a ring of 2T observation slots: rollout k uses slots ``phase*T .. phase*T + T`` (mod 2T), so
    the last observation of one rollout IS the first of the next -- the rollover is a phase flip, not a copy of
    the whole frame stack (903 KB for the bench's 32 Atari envs: a copy launch + a kernel boundary per update)."""

    def __init__(self, st):
        self.st = st

    def __getitem__(self, t):
        st = self.st
        if not isinstance(t, int) or not 0 <= t <= st.T:
            raise IndexError("ring observation slots take an int in [0, T]")
        return st.slots[(st.phase * st.T + t) % (2 * st.T)]

    def __len__(self):
        return self.st.T + 1

    @property
    def dtype(self):
        return self.st.slots.dtype

    @property
    def device(self):
        return self.st.slots.device


class RolloutStorage:
    def __init__(self, T, N, obs_shape, obs_dtype, action_shape, action_dtype, device, ring=False):
        self.T, self.N = T, N
        dev = torch.device(device)
        self.ring = bool(ring)
        self.phase = 0
        if self.ring:
            self.slots = torch.zeros((2 * T, N) + tuple(obs_shape), dtype=obs_dtype, device=dev)
            self.obs = _ObsRing(self)
        else:
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
        if name == "obs" and self.ring:   # this rollout's T slots are contiguous in the ring
            x = self.slots[self.phase * self.T:(self.phase + 1) * self.T]
            return x.reshape((self.T * self.N,) + tuple(x.shape[2:]))
        x = getattr(self, name)
        if name in ("obs", "values"):
            x = x[:self.T]
        return x.reshape((self.T * self.N,) + tuple(x.shape[2:]))

    def roll_over(self):
        """The last observation becomes the first of the next rollout (ring: flip the phase, no copy)."""
        if self.ring:
            self.phase ^= 1
        else:
            self.obs[0].copy_(self.obs[self.T])

    def nbytes(self):
        obs = self.slots if self.ring else self.obs
        return sum(t.numel() * t.element_size() for t in (obs, self.actions, self.logp, self.entropy,
                                                          self.rewards, self.dones, self.values, self.keys))
