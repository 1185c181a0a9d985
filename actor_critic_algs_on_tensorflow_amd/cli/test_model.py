"""Evaluation CLI (``Basic_AC/test_model.py``, ``A3C/test_model.py``): restore a TF-bundle checkpoint and run
episodes, printing the reference's per-episode report. Accepts both reference spellings of the no-render flag
(``--no_animation`` Basic, ``--animate_not`` A3C).

    python -m actor_critic_algs_on_tensorflow_amd.cli.test_model Pendulum-v0 tests/fixtures/model-Pendulum_a3c
"""
from __future__ import annotations

import argparse


def main(argv=None):
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("env")
    p.add_argument("model_path")
    p.add_argument("--no_animation", default=False, action="store_true")
    p.add_argument("--animate_not", default=False, action="store_true")
    p.add_argument("--seed", default=12321, type=int)
    p.add_argument("--frames", default=1, type=int)
    p.add_argument("--num_episodes", default=3, type=int)
    a = p.parse_args(argv)
    from ..api import evaluate
    from .. import ckpt
    path = a.model_path
    if not path.endswith(".index") and ckpt.latest_checkpoint(path):
        path = ckpt.latest_checkpoint(path)
    path = path[:-len(".index")] if path.endswith(".index") else path
    print("\n************Test Mode**********\nUsing model path {}\n\n".format(path))
    return evaluate(path, a.env, num_episodes=a.num_episodes, seed=a.seed, frames=a.frames,
                    animate=not (a.no_animation or a.animate_not))


if __name__ == "__main__":
    main()
