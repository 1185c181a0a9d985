#!/usr/bin/env python3
"""GPU-native async PS run on one device (1 PS + W workers sharing it over gloo), printing each worker's
episode-return curve: python scripts/a3c_gpu_curve.py --workers 2 --updates 3000 [--env Pendulum-v0] [k=v ...]"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _proc(rank, world, port, out, kw, updates, report, staleness):
    import torch.distributed as dist
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos import a3c_gpu
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    base = dict(num_envs=32, n_steps=16, total_updates=updates, outdir=None, quiet=True, stdout_freq=0,
                save_every=0, device="cuda:0", cuda_graph=True)
    base.update(kw)
    cfg = preset("a3c", **base)
    res = a3c_gpu.run(cfg, data_backend="gloo", max_staleness=staleness, device="cuda:0", report_every=report)
    res.pop("params", None)
    res.pop("log", None)
    torch.save(res, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--updates", type=int, default=3000)
    ap.add_argument("--report", type=int, default=100)
    ap.add_argument("--staleness", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/a3c_curve")
    ap.add_argument("overrides", nargs="*")
    a = ap.parse_args()
    from learn_curve import parse_kv
    kw = parse_kv(a.overrides)
    os.makedirs(a.out, exist_ok=True)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 1 + a.workers
    mp.spawn(_proc, args=(world, port, a.out, kw, a.updates, a.report, a.staleness), nprocs=world, join=True)
    for r in range(world):
        res = torch.load(os.path.join(a.out, f"r{r}.pt"), weights_only=False)
        print(json.dumps({k: v for k, v in res.items() if k not in ("history",)}, default=str), flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
