#!/usr/bin/env python3
"""Learning curve of the reference's Basic AC (``Basic_AC/run_AC.py:208-284``, README.md:13-16 runs it on
CartPole-v0) with the reference defaults: whole-episode batches (<= 7 episodes, >= 4 x 200 steps), PathAdv L = 40,
gamma 0.98, advantage normalisation, one critic + one actor Adam step per batch (actor clip +-1, lr 0.005 under the
KL-adaptive controller, desired_kl 0.002, cap 1.0), log10 entropy / KL schedules. CPU, faithful batch-1 loop.

    python scripts/learn_basic_ac.py [--env CartPole-v0] [--iters 100] [--seed 12321] [--out profiles/...]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="CartPole-v0")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--seed", type=int, default=12321)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.basic_ac import BasicACTrainer
    cfg = preset("basic_ac", env=a.env, seed=a.seed, outdir=None, quiet=True, save_every=0, stdout_freq=0)
    tr = BasicACTrainer(cfg)
    lines = [f"# Basic AC (reference defaults) on {a.env}, seed {a.seed}: iteration, episodes, mean episode return, "
             "actor lr, KL proxy, EV before / after, env steps, wall s"]
    t0 = time.time()
    for i in range(a.iters):
        s = tr.step()
        lines.append(f"{i:4d} {s['episodes']:2d} {s['avg_rew']:8.2f} {s['act_lr']:.5f} {s['kl']:.6f} "
                     f"{s['ev_before']:7.4f} {s['ev_after']:7.4f} {tr.env_steps:7d} {time.time() - t0:7.1f}")
        print(lines[-1], flush=True)
    rets = [h["avg_rew"] for h in tr.history]
    first = next((i for i in range(4, len(rets)) if sum(rets[i - 4:i + 1]) / 5 >= 195), None)
    lines.append(f"# first iteration with a 5-iteration mean return >= 195: {first}; mean of the last 20: "
                 f"{sum(rets[-20:]) / len(rets[-20:]):.1f}")
    print(lines[-1])
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
