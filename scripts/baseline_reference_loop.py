#!/usr/bin/env python3
"""Measured "reference-style" baseline: the reference's own architecture -- ONE env per process,
batch-1 policy inference every env step, the learner on the CPU -- run with this repo's code on this container's
CPU, labelled as such. The reference publishes no number and TF 1.3 / gym are not installable here.

Two loops, one JSON line each (written to profiles/r4_reference_style_baseline.jsonl by default):
  * ``pong_a2c_1env_cpu``: the headline config's model and algorithm (Nature-CNN A2C, n-step 5, RMSprop) with 1 env
    and batch-1 inference on the CPU (torch autograd engine) -- the denominator of ``bench.py``'s ``vs_baseline``;
  * ``basic_ac_cartpole_cpu``: the faithful Basic AC loop (Basic_AC/run_AC.py:208-284: whole episodes, batch-1
    inference, PathAdv L = 40, one critic + one actor Adam step per batch) on CartPole-v0.

    python scripts/baseline_reference_loop.py [--updates 200] [--iters 20] [--out PATH]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def pong_loop(updates):
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    cfg = preset("pong_a2c", num_envs=1, device="cpu", outdir=None, quiet=True, stdout_freq=0, save_every=0,
                 engine="torch", cuda_graph=False)
    tr = ActorCriticTrainer(cfg)
    for _ in range(5):
        tr.step()
    t0 = time.perf_counter()
    for _ in range(updates):
        tr.step()
    dt = time.perf_counter() - t0
    return {"loop": "pong_a2c_1env_cpu", "env_steps_per_s": round(cfg.n_steps * updates / dt, 2),
            "ms_per_update": round(1e3 * dt / updates, 3), "updates": updates,
            "what": "reference-style loop, this repo's code: Nature-CNN A2C (pong_a2c preset), 1 env, batch-1 "
                    "inference, torch autograd learner, CPU"}


def basic_ac_loop(iters):
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.basic_ac import BasicACTrainer
    cfg = preset("basic_ac", env="CartPole-v0", outdir=None, quiet=True, save_every=0, stdout_freq=0)
    tr = BasicACTrainer(cfg)
    tr.step()
    s0 = tr.env_steps
    t0 = time.perf_counter()
    for _ in range(iters):
        tr.step()
    dt = time.perf_counter() - t0
    return {"loop": "basic_ac_cartpole_cpu", "env_steps_per_s": round((tr.env_steps - s0) / dt, 2),
            "ms_per_iteration": round(1e3 * dt / iters, 3), "iterations": iters,
            "what": "the faithful Basic AC loop (algos/basic_ac.py), CartPole-v0, reference defaults, CPU"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--updates", type=int, default=200)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r4_reference_style_baseline.jsonl"))
    a = ap.parse_args()
    env = {"cpu_threads": torch.get_num_threads(), "cpus": os.cpu_count(), "machine": platform.processor() or
           platform.machine(), "torch": torch.__version__}
    rows = [dict(pong_loop(a.updates), **env), dict(basic_ac_loop(a.iters), **env)]
    with open(a.out, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
