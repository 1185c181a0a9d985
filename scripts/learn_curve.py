#!/usr/bin/env python3
"""Learning curve of a preset on the device engines (the reference's correctness signal is its training curve,
Basic_AC/run_AC.py:277-280). Prints one JSON line per report: updates, env steps, wall seconds, the fraction of
points won since the last report (reward-sign games such as Pong: +1 / -1 per point) and the mean finished-episode
return (ep_stats of the env bank).

    python scripts/learn_curve.py --preset pong_a2c --updates 20000 --report 2000 [--engine native|torch] [k=v ...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def parse_kv(items):
    out = {}
    for it in items:
        k, v = it.split("=", 1)
        for cast in (int, float):
            try:
                v = cast(v)
                break
            except ValueError:
                pass
        else:
            v = {"true": True, "false": False}.get(v.lower(), v)
        out[k] = v
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="pong_a2c")
    ap.add_argument("--updates", type=int, default=20000)
    ap.add_argument("--report", type=int, default=2000)
    ap.add_argument("--engine", default="auto")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("overrides", nargs="*")
    a = ap.parse_args()
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    kw = dict(outdir=None, quiet=True, stdout_freq=0, save_every=0, engine=a.engine, seed=a.seed)
    kw.update(parse_kv(a.overrides))
    cfg = preset(a.preset, **kw)
    tr = ActorCriticTrainer(cfg)
    if cfg.cuda_graph and tr.device.type == "cuda":
        tr.capture(warmup=1)
    dev = tr.device
    won = torch.zeros((), device=dev)
    lost = torch.zeros((), device=dev)
    t0 = time.time()
    for u in range(1, a.updates + 1):
        tr.step()
        r = tr.storage.rewards
        won += (r > 0).sum()
        lost += (r < 0).sum()
        if u % a.report == 0:
            w, l = float(won), float(lost)
            ret, n_ep, ep_len = tr.env.drain_episode_stats()
            print(json.dumps({"updates": u, "env_steps": tr.env_steps, "wall_s": round(time.time() - t0, 2),
                              "points": int(w + l), "win_frac": (w / (w + l)) if w + l else None,
                              "ep_return": ret, "episodes": n_ep, "ep_len": ep_len}), flush=True)
            won.zero_()
            lost.zero_()


if __name__ == "__main__":
    main()
