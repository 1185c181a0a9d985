#!/usr/bin/env python3
"""Throughput of every BASELINE.json config on one device (env-steps/s, ms per update), one JSON line per config.

    python scripts/bench_configs.py [--configs pong_a2c,breakout_ppo,mujoco_ppo_dp8,cartpole_cpu] [--updates K]
                                    [--warmup W] [--engine auto|torch] [--device cuda:0] [--engine-opts JSON]

Each config runs with its preset (config.py PRESETS): same model, env bank, rollout length, optimiser and PPO
epochs/minibatches as BASELINE.json names; synthetic envs and random-init weights. The update is captured as a
hipGraph where the trainer supports it (single device). The 8-GPU configs (a2c_dp8, mujoco_ppo_dp8) are measured
here per device; their multi-GPU runs go through torch.distributed.run like bench.py.
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


def run(name, updates, warmup, engine, device, dp_world1=False, engine_opts=None):
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    dev = device if name != "cartpole_cpu" or device == "cpu" else device
    cfg = preset(name, device=dev, outdir=None, quiet=True, stdout_freq=0, save_every=0, engine=engine,
                 cuda_graph=dev.startswith("cuda"))
    if engine_opts:
        import dataclasses
        cfg.engine_opts = dataclasses.replace(cfg.engine_opts, **engine_opts)
    dp = None
    if dp_world1:
        # the data-parallel update at world size 1 (RCCL on a GPU): every collective of the DP schedule is issued
        # (recorded in the update's graph), so the trace shows what the collectives cost on top of the compute
        import torch.distributed as dist
        from actor_critic_algs_on_tensorflow_amd.parallel import dp as DP
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29531")
            kw = dict(device_id=torch.device(dev)) if dev.startswith("cuda") else {}
            dist.init_process_group("nccl" if dev.startswith("cuda") else "gloo", rank=0, world_size=1, **kw)
        dp = DP.DataParallel()
    tr = ActorCriticTrainer(cfg, dp=dp)
    cuda = dev.startswith("cuda")
    if cuda:
        tr.capture(warmup=2)
    for _ in range(warmup):
        tr.step()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(updates):
        tr.step()
    if cuda:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = cfg.n_steps * tr.env.num_envs * updates
    return {"config": name, "env_steps_per_s": round(steps / dt, 1), "ms_per_update": round(1e3 * dt / updates, 4),
            "updates": updates, "envs": tr.env.num_envs, "n_steps": cfg.n_steps, "algo": cfg.algo,
            "engine": "native-cnn" if tr.engine is not None else ("native-mlp" if tr.mlp is not None else "torch"),
            "hipgraph": bool(tr.graph), "device": dev, "dp_world1": bool(dp_world1),
            "engine_opts": engine_opts or {},
            "ppo": {"epochs": cfg.ppo_epochs, "minibatches": cfg.ppo_minibatches} if cfg.algo == "ppo" else None}


def main():
    # one JSON line per config on stdout: native libraries (RCCL's banner / warnings) write to fd 1 -> stderr
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="pong_a2c,breakout_ppo,mujoco_ppo_dp8,cartpole_cpu")
    ap.add_argument("--updates", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--engine", default="auto")
    ap.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--dp-world1", action="store_true", help="run the data-parallel schedule at world size 1")
    ap.add_argument("--engine-opts", default="", help='JSON EngineOpts overrides, e.g. \'{"ppo_head": false}\'')
    args = ap.parse_args()
    opts = json.loads(args.engine_opts) if args.engine_opts else None
    for name in args.configs.split(","):
        res = run(name, args.updates, args.warmup, args.engine, args.device, args.dp_world1, opts)
        os.write(out_fd, (json.dumps(res) + "\n").encode())


if __name__ == "__main__":
    main()
