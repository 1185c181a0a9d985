"""MI355X-native actor-critic RL framework (capabilities of renly/Actor-Critic-Algs-on-Tensorflow).

Public API::

    import actor_critic_algs_on_tensorflow_amd as aca
    cfg = aca.preset("pong_a2c", total_updates=1000)
    result = aca.train(cfg)                      # -> TrainResult
    agent = aca.Agent.from_checkpoint(path)      # TF-bundle checkpoints (reference-compatible)
    action, logp, entropy = agent.act(obs)       # batched act()
"""
from . import _native
from .config import PRESETS, TrainConfig, preset

__version__ = "0.1.0"

__all__ = ["TrainConfig", "preset", "PRESETS", "train", "Agent", "_native"]


def __getattr__(name):
    if name in ("train", "Agent", "TrainResult"):
        from . import api
        return getattr(api, name)
    raise AttributeError(name)
