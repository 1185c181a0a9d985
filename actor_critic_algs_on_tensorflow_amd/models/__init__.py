"""Model families: the reference MLP actor/critic and the Nature-CNN shared-trunk actor-critic."""
from .cnn import CNNActorCriticNet, NatureCNN
from .layers import Conv, Dense, lrelu
from .mlp import MLPActor, MLPCritic
from .policy import ActorCritic, CNNActorCritic, MLPActorCritic, build_model

__all__ = ["NatureCNN", "CNNActorCriticNet", "Dense", "Conv", "lrelu", "MLPActor", "MLPCritic", "ActorCritic",
           "CNNActorCritic", "MLPActorCritic", "build_model"]
