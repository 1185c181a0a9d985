"""Frame stacking.

``Framer`` reproduces ``Basic_AC/run_AC.py:24-53`` (dup ``A3C/process.py:14-43``): observations are
left-padded with ``k-1`` copies of ``obs[0]``; ``last(obs)`` concatenates the last ``k`` padded observations,
``full(obs)[t]`` the padded observations ``t .. t+k-1`` (one feature per input observation).

:class:`FrameStack` is the batched, device-resident form used by the vectorised env bank: a ``[N, k, ...]``
stack per env that shifts in the newest frame and, at reset, fills every slot with the first frame (the same
left-padding rule). On GPU the Atari env-step kernel performs this shift in the same launch as the env step.
"""
from __future__ import annotations

import numpy as np
import torch


class Framer:
    def __init__(self, frame_num):
        self.frame_num = frame_num

    def _extend(self, obs):
        obs = list(obs)
        return [obs[0]] * (self.frame_num - 1) + obs

    def last(self, obs):
        obs = self._extend(obs)
        return np.concatenate([np.asarray(obs[i]) for i in range(-self.frame_num, 0)])

    def full(self, obs):
        obs = self._extend(obs)
        k = self.frame_num
        return [np.concatenate([np.asarray(obs[i + j]) for j in range(k)]) for i in range(len(obs) - k + 1)]

    def full_array(self, obs):
        """Vectorised ``full``: ``[T, D] -> [T, k*D]`` without Python loops over T."""
        obs = np.asarray(obs)
        k = self.frame_num
        pad = np.repeat(obs[:1], k - 1, axis=0)
        ext = np.concatenate([pad, obs], axis=0)
        T = obs.shape[0]
        return np.concatenate([ext[j:j + T] for j in range(k)], axis=1)


class FrameStack:
    """Batched frame stack ``[N, k, *frame_shape]`` (channel-major, as the CNN consumes it)."""

    def __init__(self, num_envs, k, frame_shape, dtype, device):
        self.k = k
        self.buf = torch.zeros((num_envs, k) + tuple(frame_shape), dtype=dtype, device=device)

    def reset(self, frames, mask=None):
        """Fill every slot with ``frames`` (all envs, or only where ``mask``)."""
        if mask is None:
            self.buf.copy_(frames.unsqueeze(1).expand_as(self.buf))
        else:
            m = mask.view(-1, *([1] * (self.buf.dim() - 1)))
            self.buf.copy_(torch.where(m, frames.unsqueeze(1).expand_as(self.buf), self.buf))
        return self.buf

    def push(self, frames, reset_mask=None):
        """Shift in the newest frame; envs in ``reset_mask`` get a stack of copies of their new first frame."""
        self.buf[:, :-1] = self.buf[:, 1:].clone()
        self.buf[:, -1] = frames
        if reset_mask is not None:
            self.reset(frames, reset_mask)
        return self.buf
