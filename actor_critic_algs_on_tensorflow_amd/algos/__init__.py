"""Algorithms: synchronous A2C / PPO-clip trainers, the reference-parity episode-batched trainer, A3C."""
from .storage import RolloutStorage
from .trainer import ActorCriticTrainer

__all__ = ["RolloutStorage", "ActorCriticTrainer"]
