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

On GPU the trainers use :func:`returns_scan`: ONE HIP launch (``returns_scan_kernel`` in
``csrc/kernels/returns.hip``) computes either estimator as a chunked associative reverse scan over (time chunk x
env) -- both are affine recurrences ``x_t = a_t + c_t x_{t+1}`` -- together with the EV-before correlation, the
moments a data-parallel run all-reduces, and (optionally) the in-place advantage normalisation. The truncated
n-step window (``L < T``) uses its prefix-sum form (scan of the un-bootstrapped return + next-terminal index). The
simple per-column kernels (:func:`gae`, :func:`nstep_returns`) stay as the small-T building blocks. The PyTorch
code below is the oracle all of them are tested against.
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
    if int(look_ahead) < 1:
        # L = 0 would make every target the bootstrap V(s_t) itself (advantage 0); no entry point supports it
        raise ValueError(f"look_ahead must be >= 1, got {look_ahead}")
    r = rews.double()
    v = vals.double()
    d = dones.to(torch.bool)
    L = min(int(look_ahead), T)
    # every start t at once, one window offset j per pass (L passes instead of T * L): the same per-t summation
    # order and the same Python-float discount products as a per-t loop, so the values are bitwise those of it
    acc = torch.zeros(T, N, dtype=torch.float64, device=rews.device)
    alive = torch.ones(T, N, dtype=torch.bool, device=rews.device)
    zero = torch.zeros((), dtype=torch.float64, device=rews.device)
    disc = 1.0
    for j in range(L):
        n = T - j                     # starts t < T - j still have step t + j inside the rollout
        acc[:n] = acc[:n] + torch.where(alive[:n], disc * r[j:], zero)
        alive[:n] = alive[:n] & ~d[j:]
        disc *= gamma
    # bootstrap with V[h_end], h_end = min(t + L, T), only if no terminal transition inside the window
    t_idx = torch.arange(T, device=rews.device)
    h_end = torch.clamp(t_idx + L, max=T)
    pw = torch.tensor([gamma ** e for e in range(L + 1)], dtype=torch.float64, device=rews.device)
    boot = pw[h_end - t_idx][:, None] * v[h_end]
    tgt = acc + torch.where(alive, boot, zero)
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
    if L < 1:
        raise ValueError(f"look_ahead must be >= 1 (or None for the whole rollout), got {look_ahead}")
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


class ScanWorkspace:
    """Device workspace of :func:`returns_scan` / the many-workgroup EV: per-workgroup fp64 partial moments, the
    self-cleaning last-arriver ticket, the fp64 totals ``mom`` (``[count, sum adv, sum adv^2, sum ret, sum ret^2,
    sum V, sum V^2, sum ret*V]``) and the truncated-window scratch. Create once, outside any graph capture."""

    def __init__(self, device, T=0, N=0):
        self.device = torch.device(device)
        self.part = torch.zeros(256 * 8, dtype=torch.float64, device=self.device)
        self.ticket = torch.zeros(4, dtype=torch.int32, device=self.device)
        self.ev_ticket = torch.zeros(4, dtype=torch.int32, device=self.device)
        self.ev_part = torch.zeros(64 * 8, dtype=torch.float64, device=self.device)
        # [0:8] the moments; [8:10] a slot the trainer packs into the same all-reduce (its deferred KL)
        self.mom = torch.zeros(10, dtype=torch.float64, device=self.device)
        self.gz = torch.zeros(max(T * N, 1), dtype=torch.float64, device=self.device)

    def fit(self, T, N):
        blocks = _native.require().returns_scan_geometry(T, N)[3]
        if self.part.numel() < blocks * 8:
            self.part = torch.zeros(blocks * 8, dtype=torch.float64, device=self.device)
        if self.gz.numel() < T * N:
            self.gz = torch.zeros(T * N, dtype=torch.float64, device=self.device)
        return self


def returns_scan(rews, vals, dones, mode="gae", gamma=0.99, lam=0.95, look_ahead=None, norm=False, eps=1e-8,
                 ws: ScanWorkspace | None = None, ev_out=None, ret_out=None, adv_out=None):
    """Fused returns + statistics. ``mode`` "gae" or "nstep" (``look_ahead`` None -> whole rollout).

    Returns ``(ret, adv, mom)``: ``adv`` normalised (population std) when ``norm``; ``mom`` the fp64 totals
    (``[count, sum adv, sum adv^2, sum ret, sum ret^2, sum V, sum V^2, sum ret*V]``, pre-normalisation) and, if
    ``ev_out`` is given, ``ev_out[0]`` = EV correlation of (ret, V[:T]) (``Basic_AC/util.py:4-12``)."""
    T, N = rews.shape
    L = T if look_ahead is None else int(look_ahead)
    if not _native.use_native(rews):
        ret, adv = gae_ref(rews, vals, dones, gamma, lam) if mode == "gae" else \
            nstep_returns_ref(rews, vals, dones, gamma, L)
        v = vals[:T].double()
        a, r = adv.double(), ret.double()
        mom = torch.stack([torch.tensor(float(T * N), dtype=torch.float64, device=rews.device), a.sum(),
                           (a * a).sum(), r.sum(), (r * r).sum(), v.sum(), (v * v).sum(), (r * v).sum()])
        if ev_out is not None:
            from ..utils.stats import var_accounted_for_tensor
            ev_out.view(-1)[0] = var_accounted_for_tensor(ret.reshape(-1), vals[:T].reshape(-1))
        if norm:
            adv = normalize_advantages(adv, eps)
        if ret_out is not None:
            ret_out.view(T, N).copy_(ret)
            ret = ret_out.view(T, N)
        if adv_out is not None:
            adv_out.view(T, N).copy_(adv)
            adv = adv_out.view(T, N)
        return ret, adv, mom
    ws = (ws or ScanWorkspace(rews.device)).fit(T, N)
    ret = ret_out.view(T, N) if ret_out is not None else torch.empty(T, N, device=rews.device)
    adv = adv_out.view(T, N) if adv_out is not None else torch.empty(T, N, device=rews.device)
    _native.require().returns_scan(rews.float().contiguous(), vals.float().contiguous(),
                                   dones.to(torch.uint8).contiguous(), ret, adv, 2 if mode == "gae" else 1,
                                   float(gamma), float(lam), L, bool(norm), float(eps), ws.part, ws.ticket, ws.mom,
                                   ev_out, ws.gz)
    return ret, adv, ws.mom
