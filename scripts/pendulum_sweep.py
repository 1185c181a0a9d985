"""Pendulum-v0 learning sweep on one GPU (native MLP engine, hipGraph-captured updates).

Each config is the reference actor/critic (``model_variant="a3c"``) trained by the vectorised
trainer with the reference losses (PathAdv n-step returns gamma 0.98 / L 40, normalised advantages, entropy +
KL-proxy regularisers with the log10 schedules, element-clipped Adam, KL-adaptive actor lr) plus per-config
overrides. Prints one JSON line per report: (updates, env steps, mean finished-episode return, actor lr, KL).

    python scripts/pendulum_sweep.py --configs cap01,cap001 --updates 20000 --out gpurun_out/pend
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    # the reference A3C hyper-parameters verbatim (lr cap 0.1)
    "cap01": dict(),
    "cap001": dict(max_lr=0.01),
    "cap001_torch": dict(max_lr=0.01, engine="torch"),
    "cap0003": dict(max_lr=0.003),
    "cap001_n64": dict(max_lr=0.01, num_envs=64),
    "cap001_n128": dict(max_lr=0.01, num_envs=128),
    "cap001_t40": dict(max_lr=0.01, n_steps=40),
    "cap001_ep": dict(max_lr=0.01, num_envs=16, n_steps=200),
    "fixed3e4_n64": dict(kl_adaptive_lr=False, lr=3e-4, num_envs=64),
    "basic_n64": dict(max_lr=0.01, clip_value=1.0, num_envs=64),
    "noanneal_n64": dict(max_lr=0.01, anneal_regularizers=False, num_envs=64),
    "ppo_ref": dict(algo="ppo", returns="gae", gae_lambda=0.95, num_envs=64, n_steps=200, ppo_epochs=10,
                    ppo_minibatches=8, ppo_clip=0.2, kl_adaptive_lr=False, kl_coef=0.0, lr=3e-4,
                    anneal_regularizers=False, ent_coef=0.0, clip_value=None, max_grad_norm=0.5,
                    _updates_div=30),
}


def run_one(name, over, updates, reports, device, seed, save_dir=None):
    import torch
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    kw = dict(algo="a2c", num_envs=32, n_steps=16, outdir=None, quiet=True, stdout_freq=0, save_every=0,
              device=device, cuda_graph=True, seed=seed)
    over = dict(over)
    updates = max(1, updates // over.pop("_updates_div", 1))
    kw.update(over)
    cfg = preset("a3c", **kw)
    tr = ActorCriticTrainer(cfg)
    tr.capture(warmup=2)
    t0 = time.time()
    every = max(1, updates // reports)
    rows = []
    for u in range(1, updates + 1):
        tr.step()
        if u % every == 0:
            ret, n_ep, _ = tr.env.drain_episode_stats()
            row = dict(config=name, updates=u, env_steps=tr.env_steps, ret=round(ret, 1) if n_ep else None,
                       episodes=n_ep, lr=float(tr.actor_opt.lr), kl=float(tr.stats["kl"]),
                       wall_s=round(time.time() - t0, 2))
            rows.append(row)
            print(json.dumps(row), flush=True)
    path = None
    if save_dir:
        path = tr.save_checkpoint(os.path.join(save_dir, f"model-Pendulum-{name}"))
    return rows, path


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default=",".join(CONFIGS))
    p.add_argument("--updates", type=int, default=20000)
    p.add_argument("--reports", type=int, default=20)
    p.add_argument("--seed", type=int, default=12321)
    p.add_argument("--device", default="cuda:0")
    p.add_argument("--out", default=None)
    a = p.parse_args()
    if a.out:
        os.makedirs(a.out, exist_ok=True)
    for name in a.configs.split(","):
        rows, path = run_one(name, CONFIGS[name], a.updates, a.reports, a.device, a.seed, save_dir=a.out)
        tail = [r["ret"] for r in rows[-max(1, len(rows) // 4):] if r["ret"] is not None]
        summ = dict(config=name, summary=True, last_quarter_mean=(sum(tail) / len(tail)) if tail else math.nan,
                    best=max((r["ret"] for r in rows if r["ret"] is not None), default=None), checkpoint=path)
        print(json.dumps(summ), flush=True)


if __name__ == "__main__":
    main()
