"""Learning curve of the Breakout-shape PPO config (Pong-shaped 84x84x4 bank, 128 envs x 128 steps, 4 epochs x 4
minibatches of 4096, native CNN engine, hipGraph): fraction of points won per report window.
Usage (GPU box): python scripts/learn_breakout_ppo.py [--updates 300] [--report 25] [--out file.json]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--updates", type=int, default=300)
    ap.add_argument("--report", type=int, default=25)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tr = ActorCriticTrainer(preset("breakout_ppo", device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                                   save_every=0, seed=a.seed))
    if tr.cfg.cuda_graph:
        tr.capture(warmup=1)
    won = torch.zeros((), device=tr.device)
    lost = torch.zeros((), device=tr.device)
    rows = []
    for u in range(1, a.updates + 1):
        tr.step()
        r = tr.storage.rewards
        won += (r > 0).sum()
        lost += (r < 0).sum()
        if u % a.report == 0:
            w, l = float(won), float(lost)
            rows.append(dict(u=u, env_steps=u * tr.cfg.num_envs * tr.cfg.n_steps, win=round(w / max(w + l, 1.0), 4)))
            print(json.dumps(rows[-1]), flush=True)
            won.zero_()
            lost.zero_()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f)


if __name__ == "__main__":
    main()
