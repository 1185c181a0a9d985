"""Single-process trainer CLI, flag-compatible with ``Basic_AC/run_AC.py`` (``Basic_AC/run_AC.py:11-22``).

    python -m actor_critic_algs_on_tensorflow_amd.cli.run_ac --env CartPole-v0 --seed 12321 --frames 1

Default ``--algo basic_ac`` is the reference's episode-batched loop (batch-1 inference, PathAdv targets,
KL-adaptive lr, log10 regulariser schedules, reference log format). ``--algo a2c|ppo`` (with ``--preset``)
switches to the vectorised GPU-native trainers with the same flags where they apply.
"""
from __future__ import annotations

import argparse
import os


def build_parser():
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("--animate", default=False, action="store_true")
    p.add_argument("--env", default="Pendulum-v0")
    p.add_argument("--seed", default=12321, type=int)
    p.add_argument("--tboard", default=False, action="store_true")
    p.add_argument("--save_every", default=600, type=int)
    p.add_argument("--outdir", default="log.txt")
    p.add_argument("--checkpoint_dir", default=os.path.join("tmp", "checkpoints"))
    p.add_argument("--frames", default=1, type=int)
    p.add_argument("--mode", choices=["train", "debug"], default="train")
    p.add_argument("--desired_kl", default=0.002, type=float)
    # extensions
    p.add_argument("--algo", default="basic_ac", choices=["basic_ac", "a2c", "ppo"])
    p.add_argument("--preset", default=None, help="start from a named preset (config.PRESETS)")
    p.add_argument("--iters", default=5000000, type=int, help="ITER of the reference")
    p.add_argument("--device", default=None)
    p.add_argument("--num_envs", default=None, type=int)
    p.add_argument("--metrics", default=None, help="JSONL metrics sidecar path")
    p.add_argument("--quiet", action="store_true")
    return p


def main(argv=None):
    a = build_parser().parse_args(argv)
    from ..api import train
    from ..config import preset
    name = a.preset or ("basic_ac" if a.algo == "basic_ac" else ("breakout_ppo" if a.algo == "ppo" else "cartpole_cpu"))
    kw = dict(env=a.env, seed=a.seed, save_every=a.save_every, outdir=a.outdir, checkpoint_dir=a.checkpoint_dir,
              frames=a.frames, mode=a.mode, desired_kl=a.desired_kl, total_updates=a.iters, tboard=a.tboard,
              metrics_path=a.metrics, quiet=a.quiet)
    if a.algo != "basic_ac":
        kw["algo"] = a.algo
    if a.device:
        kw["device"] = a.device
    if a.num_envs:
        kw["num_envs"] = a.num_envs
    cfg = preset(name, **kw)
    res = train(cfg)
    print("done: %d iterations, %d env steps, %.1f env-steps/s" % (res.iterations, res.env_steps,
                                                                    res.env_steps_per_sec))
    return res


if __name__ == "__main__":
    main()
