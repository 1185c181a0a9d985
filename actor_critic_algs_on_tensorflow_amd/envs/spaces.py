"""Minimal gym-shaped action/observation spaces (gym is not a dependency)."""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class Discrete:
    n: int

    @property
    def shape(self):
        return ()


@dataclass
class Box:
    low: np.ndarray
    high: np.ndarray
    shape: tuple = field(default=None)
    dtype: str = "float32"

    def __post_init__(self):
        self.low = np.asarray(self.low, dtype=np.float32)
        self.high = np.asarray(self.high, dtype=np.float32)
        if self.shape is None:
            self.shape = tuple(self.low.shape)


@dataclass
class EnvSpec:
    """What ``gym.make(id).spec`` exposes that the trainers need (``Basic_AC/run_AC.py:124-136``)."""

    id: str
    max_episode_steps: int | None
    reward_threshold: float | None = None
