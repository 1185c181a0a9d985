"""Hyper-parameter schedules and the KL-adaptive learning-rate controller.

Behavioural parity targets:
  * ``LinearSchedule`` -- ``Basic_AC/util.py:15-41`` (identical in ``A3C/util.py:16-42``).
  * ``KLAdaptiveLR``   -- the inline controller of ``Basic_AC/run_AC.py:257-266`` and
    ``A3C/process.py:262-270``: after the update, ``kl < d/4`` multiplies the actor lr by 1.5 (capped),
    ``kl > 4d`` divides it by 1.5 (floored).
  * ``RegularizerSchedule`` -- the log10 entropy / KL coefficient annealing of
    ``Basic_AC/run_AC.py:181-182,268-275``.

The device variant (:class:`DeviceKLAdaptiveLR`) keeps lr on the GPU so the learner step can run inside a
captured hipGraph without a host sync; it applies the exact same rule with ``torch.where``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch


class LinearSchedule:
    """Piecewise-linear interpolation between ``(init_t, init_val)`` and ``(end_t, end_val)``.

    ``val(t)`` is ``init_val`` before ``init_t``, ``end_val`` after ``end_t`` and the linear blend in
    between; ``update_time(t)`` is the periodic trigger ``t % update_every_t == 0`` (true at t=0).
    """

    def __init__(self, init_t, end_t, init_val, end_val, update_every_t):
        self.init_t = init_t
        self.end_t = end_t
        self.init_val = init_val
        self.end_val = end_val
        self.update_every_t = update_every_t

    def val(self, t):
        if t < self.init_t:
            return self.init_val
        if t > self.end_t:
            return self.end_val
        return ((t - self.init_t) * self.end_val + (self.end_t - t) * self.init_val) / float(self.end_t - self.init_t)

    def update_time(self, t):
        return t % self.update_every_t == 0


class KLAdaptiveLR:
    """Host-side KL-adaptive learning-rate rule (reference parity).

    Basic_AC bounds are ``[1e-6, 1.0]`` (``run_AC.py:178``); A3C uses ``[1e-6, 0.1]`` (``process.py:12``).
    """

    def __init__(self, desired_kl=0.002, min_lr=1e-6, max_lr=1.0, factor=1.5):
        self.desired_kl = desired_kl
        self.min_lr = min_lr
        self.max_lr = max_lr
        self.factor = factor

    def __call__(self, lr, kl):
        if kl < self.desired_kl / 4:
            return min(self.max_lr, lr * self.factor)
        if kl > self.desired_kl * 4:
            return max(self.min_lr, lr / self.factor)
        return lr


class DeviceKLAdaptiveLR(KLAdaptiveLR):
    """Same rule on device scalars: ``lr`` and ``kl`` are 0-d tensors, ``lr`` is updated in place.

    Graph-capturable (no ``.item()``); used by the fused learner so the adaptive lr never forces a sync.
    """

    @torch.no_grad()
    def update_(self, lr: torch.Tensor, kl: torch.Tensor, valid: torch.Tensor | None = None) -> torch.Tensor:
        """``valid`` (0-d bool tensor): apply the rule only where it is true (a deferred KL that may be absent)."""
        up = torch.clamp(lr * self.factor, max=self.max_lr)
        down = torch.clamp(lr / self.factor, min=self.min_lr)
        new = torch.where(kl < self.desired_kl / 4, up, torch.where(kl > self.desired_kl * 4, down, lr))
        if valid is not None:
            new = torch.where(valid, new, lr)
        lr.copy_(new)
        return lr


@dataclass
class RegularizerSchedule:
    """log10 annealing of the entropy coefficient ("gamma") and KL coefficient ("beta").

    Defaults reproduce ``Basic_AC/run_AC.py:181-182``: entropy 10^(-2 -> -8), KL 10^(0 -> -4), linear in
    iterations 100..3000, applied every 100 iterations (including iteration 0).
    """

    init_t: int = 100
    end_t: int = 3000
    log_ent_init: float = -2.0
    log_ent_end: float = -8.0
    log_kl_init: float = 0.0
    log_kl_end: float = -4.0
    every: int = 100

    def __post_init__(self):
        self.ent = LinearSchedule(self.init_t, self.end_t, self.log_ent_init, self.log_ent_end, self.every)
        self.kl = LinearSchedule(self.init_t, self.end_t, self.log_kl_init, self.log_kl_end, self.every)

    def entropy_coef(self, it):
        """Returns the new entropy coefficient at iteration ``it`` or ``None`` when it is not an update step."""
        return math.pow(10.0, self.ent.val(it)) if self.ent.update_time(it) else None

    def kl_coef(self, it):
        return math.pow(10.0, self.kl.val(it)) if self.kl.update_time(it) else None
