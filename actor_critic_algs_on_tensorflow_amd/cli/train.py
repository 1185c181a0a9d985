"""A3C per-process CLI, flag-compatible with ``A3C/train.py`` (``python train.py {ps,worker} TASK [...]``).

The reference builds a localhost TF ClusterSpec on ports ``initport + i`` (``A3C/train.py:29-38``). Here every
process joins one ``torch.distributed`` gloo group: rendezvous at ``127.0.0.1:initport``, world size
``ps_num + worker_num``, rank ``task`` for PS tasks and ``ps_num + task`` for workers. Worker logs go to
``<outdir>/worker_<task>.log``; the chief (worker 0) writes ``<checkpoint_dir>/model-<EnvPrefix>-<global_step>``.

Also usable under torchrun (``--job auto``: the rank decides the role).

``--device cuda`` (or ``cuda:K``; ``cuda`` alone maps each rank to GPU ``rank % device_count``) selects the
GPU-native mode (:mod:`..algos.a3c_gpu`): workers own ``--num_envs`` device envs and the device engines, PS tasks
keep their shard and Adam moments on the device; ``--data_plane nccl`` moves the payloads over RCCL (one GPU per
rank), ``gloo`` stages them through host memory. ``--max_staleness s`` bounds gradient staleness (-1: unbounded,
as the reference).
"""
from __future__ import annotations

import argparse
import datetime
import os


def build_parser():
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("job", choices=["ps", "worker", "auto"])
    p.add_argument("task", type=int, nargs="?", default=0)
    p.add_argument("--animate", default=False, action="store_true")
    p.add_argument("--env", default="Pendulum-v0")
    p.add_argument("--seed", default=12321, type=int)
    p.add_argument("--tboard", default=False)
    p.add_argument("--worker_num", default=4, type=int)
    p.add_argument("--ps_num", default=2, type=int)
    p.add_argument("--initport", default=2849, type=int)
    p.add_argument("--stdout_freq", default=20, type=int)
    p.add_argument("--save_every", default=600, type=int)
    p.add_argument("--outdir", default=os.path.join("tmp", "logs"))
    p.add_argument("--checkpoint_dir", default=os.path.join("tmp", "checkpoints"))
    p.add_argument("--frames", default=1, type=int)
    p.add_argument("--mode", choices=["train", "debug-light", "debug-full"], default="train")
    p.add_argument("--desired_kl", default=0.002, type=float)
    p.add_argument("--max_iters", default=int(1e7), type=int, help="stop at this many global steps (MAX_ITERS)")
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--device", default="cpu", help="cpu (reference-shaped episode workers) | cuda[:K] (GPU-native)")
    p.add_argument("--num_envs", default=16, type=int, help="GPU mode: device envs per worker")
    p.add_argument("--n_steps", default=16, type=int, help="GPU mode: rollout length per update")
    p.add_argument("--data_plane", default="gloo", choices=["gloo", "nccl"])
    p.add_argument("--max_staleness", default=-1, type=int)
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    import torch.distributed as dist
    from ..algos import a3c
    from ..config import preset
    world = args.ps_num + args.worker_num
    if args.job == "auto":
        rank = int(os.environ.get("RANK", "0"))
    else:
        rank = args.task if args.job == "ps" else args.ps_num + args.task
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(args.initport))
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
    cfg = preset("a3c", env=args.env, seed=args.seed, frames=args.frames, desired_kl=args.desired_kl,
                 stdout_freq=args.stdout_freq, save_every=args.save_every, checkpoint_dir=args.checkpoint_dir,
                 total_updates=args.max_iters, ps_num=args.ps_num, mode=args.mode, quiet=args.quiet)
    role = "ps" if rank < args.ps_num else "worker"
    task = rank if role == "ps" else rank - args.ps_num
    log = os.path.join(args.outdir, "worker_{}.log".format(task)) if role == "worker" else "N/A"
    print("Starting {} {} with log at {}".format(role, task, log), flush=True)
    if args.device.startswith("cuda"):
        import torch
        from ..algos import a3c_gpu
        dev = args.device if ":" in args.device else f"cuda:{rank % max(1, torch.cuda.device_count())}"
        cfg = cfg.replace(device=dev, num_envs=args.num_envs, n_steps=args.n_steps, cuda_graph=True, outdir=None)
        out = a3c_gpu.run(cfg, rank=rank, world=world, ps_num=args.ps_num, data_backend=args.data_plane,
                          max_staleness=args.max_staleness, device=dev, log_dir=args.outdir)
    else:
        out = a3c.run(cfg, rank=rank, world=world, ps_num=args.ps_num, log_dir=args.outdir)
    dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
