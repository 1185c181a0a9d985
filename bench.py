#!/usr/bin/env python3
"""Headline benchmark: env-steps/sec (whole node) of synchronous A2C on the Atari-shaped CNN, 32 vec-envs per GPU.

BASELINE.json metric "env-steps/sec (whole node) A2C Atari-CNN 32 vec-envs/GPU at 1/2/4/8 MI355X", config
"Atari-Pong A2C, 32 synthetic 84x84x4 vec-envs, CNN+MLP bf16" (preset ``pong_a2c``: n_steps 5, RMSprop 7e-4,
global-norm clip 0.5, entropy 0.01, value coef 0.5). One timed step = one full A2C update: 5 rollout steps of the
32-env bank (CNN inference + categorical sampling + env physics + frame rendering/stacking) plus the bootstrap
value, n-step returns, the learner forward/loss/backward over the 160-sample batch and the fused RMSprop update
(and, for N > 1, the RCCL all-reduce of the flat gradient slab). Weak scaling: 32 envs per GPU.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]; N > 1 under torch.distributed.run (one rank per GPU).
Synthetic data (the Pong-shaped env bank renders its own frames), random-init weights.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

METRIC = "env-steps/sec (whole node) A2C Atari-CNN 32 vec-envs/GPU at 1/2/4/8 MI355X"
# The reference publishes no number. vs_baseline is taken against the MEASURED reference-style loop
# (SURVEY §6.3): the same model and algorithm in the reference's architecture -- one env per process, batch-1
# inference every step, CPU learner -- run with this repo's code (scripts/baseline_reference_loop.py,
# profiles/r4_reference_style_baseline.jsonl, BASELINE.md "Measured reference-style baseline").
BASELINE_VALUE = 63.08
BASELINE_WHAT = "reference-style loop (1 env, batch-1 inference, CPU; this repo's code), 63.08 env-steps/s"


def _json_stdout():
    """stdout carries exactly ONE JSON line: native libraries (RCCL's version banner and warnings) write to fd 1, so
    fd 1 is pointed at stderr for the whole run and the result goes to the saved original stdout."""
    sys.stdout.flush()
    out = os.dup(1)
    os.dup2(2, 1)
    return out


def main():
    out_fd = _json_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=32)
    ap.add_argument("--engine", default="auto")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--overlap", default="strict", choices=["strict", "lag1"],
                    help="DP schedule: strict = exact sync A2C, fc/head gradient bucket all-reduced under the conv "
                         "backward; lag1 = all-reduce overlapped with the next rollout, gradient applied one update "
                         "late")
    ap.add_argument("--bucket-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="dtype of the all-reduced gradient buckets (bf16 halves the xGMI bytes)")
    ap.add_argument("--engine-opts", default="",
                    help="JSON dict of EngineOpts overrides (A/B runs; the defaults are the measured fastest)")
    ap.add_argument("--dp-world1", action="store_true",
                    help="one process: run the data-parallel schedule (--overlap, --bucket-dtype) on a 1-rank RCCL "
                         "group, so its collectives and buckets are issued exactly as at N >= 2 (the step from N = 1 "
                         "to N = 2 of a scaling curve, without the second GPU)")
    args = ap.parse_args()

    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    from actor_critic_algs_on_tensorflow_amd.parallel import dp as DP

    rank, world, local = DP.init_from_env("nccl")
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    if args.dp_world1 and world == 1 and not torch.distributed.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
    dp = DP.DataParallel() if (world > 1 or args.dp_world1) else None
    cfg = preset("pong_a2c", num_envs=args.envs, device=f"cuda:{local}", outdir=None, quiet=True,
                 stdout_freq=0, save_every=0, engine=args.engine, cuda_graph=not args.no_graph,
                 overlap=args.overlap, grad_bucket_dtype=args.bucket_dtype,
                 engine_opts=json.loads(args.engine_opts) if args.engine_opts else None)
    tr = ActorCriticTrainer(cfg, dp=dp)
    if cfg.cuda_graph:
        tr.capture(warmup=2)
    for _ in range(args.warmup):
        tr.step()
    torch.cuda.synchronize()
    if dp is not None:
        dp.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.step()
    torch.cuda.synchronize()
    if dp is not None:
        dp.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dp is not None:
        t = torch.tensor([dt], device=f"cuda:{local}", dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    steps_per_update = cfg.n_steps * args.envs * world
    value = steps_per_update * args.steps / dt
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_VALUE, 1) if BASELINE_VALUE else None,
            "baseline": BASELINE_WHAT,
            "dtype": "bf16",
            "data": "synthetic (Pong-shaped 84x84x4 uint8 env bank, random-init weights)",
            "config": {"model": "Nature-CNN actor-critic (3 conv + fc512, 1.69M params)",
                       "global_batch": steps_per_update, "seq_len": cfg.n_steps, "envs_per_gpu": args.envs,
                       "algo": "A2C (RMSprop 7e-4, n-step returns, grad-norm 0.5)",
                       "parallelism": f"dp{world}", "engine": "native" if tr.engine is not None else "torch",
                       "hipgraph": bool(tr.graph), "dp_schedule": tr.graph[0] if tr.graph else "eager",
                       "grad_bucket_dtype": args.bucket_dtype, "dp_world1": bool(args.dp_world1)},
        }
        os.write(out_fd, (json.dumps(out) + "\n").encode())
        if os.environ.get("ACA_BENCH_SAVE_PLANS"):   # record the GEMM plans this run tuned (scripts/plan_search.sh)
            from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
            G.save_plans(os.environ["ACA_BENCH_SAVE_PLANS"])
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
