"""Return / advantage estimators over ``[T, N]`` rollouts (kernel K06 + K09 of SURVEY §2.4).

* :func:`path_adv` -- verbatim-behaviour ``PathAdv.__call__`` for one episode (``Basic_AC/run_AC.py:55-80``):
  L-step truncated discounted return plus bootstrap, advantage = target - V. numpy, used by the parity trainer.
* :func:`nstep_returns` -- the same estimator generalised to a ``[T, N]`` rollout with episode boundaries
  (``dones[t]`` = the transition at t ended its episode): for each (t, n) the window [t, min(t+L, end)) is summed
  with discount, and ``gamma^(h-t) V[h]`` is added unless the window stops at a terminal transition. With
  ``L >= T`` this is the classic A2C n-step return.
* :func:`gae` -- GAE(lambda): ``A_t = delta_t + gamma lambda (1-d_t) A_{t+1}``, ``R_t = A_t + V_t``.
* :func:`normalize_advantages` -- ``(A - mean) / (1e-8 + std)`` with the population std
  (``Basic_AC/run_AC.py:241``).

On GPU each function is one HIP launch (``csrc/kernels/returns.hip``): one thread per env column runs the
reverse scan for GAE; n-step runs one thread per (t, n) with an O(L) window. The PyTorch code below is the
oracle those kernels are tested against.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native


def path_adv(rews, vals, terminal, gamma=0.98, look_ahead=30):
    """``PathAdv(gamma, look_ahead)(rews, vals, terminal)`` -> (targets, advs) as lists."""
    rews = np.asarray(rews, dtype=np.float64)
    vals = np.asarray(vals, dtype=np.float64)
    T = len(rews)
    assert len(vals) == T + 1
    kern = np.power(gamma, np.arange(look_ahead))
    action_val = np.convolve(rews[::-1], kern)[T - 1::-1].copy()
    assert len(action_val) == T
    advs = np.zeros(T)
    for i in range(T):
        h = min(i + look_ahead, T)
        if not terminal or h != T:
            action_val[i] += np.power(gamma, h - i) * vals[h]
        advs[i] = action_val[i] - vals[i]
    return list(action_val), list(advs)


class PathAdv:
    """Callable object with the reference interface (``__call__``, ``reset``)."""

    def __init__(self, gamma=0.98, look_ahead=30):
        self.reset(gamma, look_ahead)

    def __call__(self, rews, vals, terminal):
        return path_adv(rews, vals, terminal, self.gamma, self.look_ahead)

    def reset(self, gamma, look_ahead):
        self.gamma = gamma
        self.look_ahead = look_ahead
        self.kern = [np.power(gamma, k) for k in range(look_ahead)]


def _check(rews, vals, dones):
    T, N = rews.shape
    assert vals.shape == (T + 1, N), (vals.shape, rews.shape)
    assert dones.shape == (T, N)


def nstep_returns_ref(rews, vals, dones, gamma, look_ahead):
    """PyTorch oracle. rews/dones ``[T, N]``, vals ``[T+1, N]`` -> (targets, advs) fp32 ``[T, N]``."""
    _check(rews, vals, dones)
    T, N = rews.shape
    r = rews.double()
    v = vals.double()
    d = dones.to(torch.bool)
    tgt = torch.zeros(T, N, dtype=torch.float64, device=rews.device)
    for t in range(T):
        acc = torch.zeros(N, dtype=torch.float64, device=rews.device)
        alive = torch.ones(N, dtype=torch.bool, device=rews.device)
        disc = 1.0
        h_end = min(t + look_ahead, T)
        for k in range(t, h_end):
            acc = acc + torch.where(alive, disc * r[k], torch.zeros_like(acc))
            alive = alive & ~d[k]
            disc *= gamma
        # bootstrap with V[h_end] only if no terminal transition inside the window
        acc = acc + torch.where(alive, (gamma ** (h_end - t)) * v[h_end], torch.zeros_like(acc))
        tgt[t] = acc
    adv = tgt - v[:T]
    return tgt.float(), adv.float()


def gae_ref(rews, vals, dones, gamma, lam):
    _check(rews, vals, dones)
    T, N = rews.shape
    r, v = rews.double(), vals.double()
    nd = 1.0 - dones.double()
    adv = torch.zeros(T, N, dtype=torch.float64, device=rews.device)
    last = torch.zeros(N, dtype=torch.float64, device=rews.device)
    for t in reversed(range(T)):
        delta = r[t] + gamma * v[t + 1] * nd[t] - v[t]
        last = delta + gamma * lam * nd[t] * last
        adv[t] = last
    ret = adv + v[:T]
    return ret.float(), adv.float()


def nstep_returns(rews, vals, dones, gamma=0.99, look_ahead=None):
    """L-step truncated returns with bootstrap (``look_ahead=None`` -> whole rollout, classic A2C)."""
    L = rews.shape[0] if look_ahead is None else int(look_ahead)
    if _native.use_native(rews):
        tgt = torch.empty_like(rews, dtype=torch.float32)
        adv = torch.empty_like(tgt)
        _native.require().nstep_returns(rews.float().contiguous(), vals.float().contiguous(),
                                        dones.to(torch.uint8).contiguous(), tgt, adv, float(gamma), L)
        return tgt, adv
    return nstep_returns_ref(rews, vals, dones, gamma, L)


def gae(rews, vals, dones, gamma=0.99, lam=0.95):
    """GAE(lambda) -> (returns, advantages)."""
    if _native.use_native(rews):
        ret = torch.empty_like(rews, dtype=torch.float32)
        adv = torch.empty_like(ret)
        _native.require().gae(rews.float().contiguous(), vals.float().contiguous(),
                              dones.to(torch.uint8).contiguous(), ret, adv, float(gamma), float(lam))
        return ret, adv
    return gae_ref(rews, vals, dones, gamma, lam)


def normalize_advantages(adv, eps=1e-8):
    """Population-std normalisation (numpy ddof=0), as ``Basic_AC/run_AC.py:241``."""
    a = adv.float()
    return (a - a.mean()) / (eps + a.std(unbiased=False))
