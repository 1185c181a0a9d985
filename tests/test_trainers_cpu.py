"""Algorithm smoke / learning tests and multi-process distributed tests on CPU (gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from actor_critic_algs_on_tensorflow_amd import preset
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _quiet(**kw):
    base = dict(outdir=None, quiet=True, stdout_freq=0, save_every=0)
    base.update(kw)
    return base


def _mean_return(tr, updates):
    tr.env.ep_stats.zero_()
    for _ in range(updates):
        tr.step()
    s = tr.env.ep_stats
    return float(s[0] / max(float(s[1]), 1.0))


def test_cartpole_a2c_learns():
    """BASELINE config 1 (CartPole A2C on CPU) improves well beyond a random policy (~22)."""
    torch.manual_seed(0)
    tr = ActorCriticTrainer(preset("cartpole_cpu", **_quiet(num_envs=16, n_steps=8, seed=3)))
    first = _mean_return(tr, 60)
    for _ in range(300):
        tr.step()
    last = _mean_return(tr, 60)
    assert last > max(60.0, 2 * first), (first, last)


def test_ppo_and_gaussian_paths_run():
    for name, kw in (("breakout_ppo", dict(num_envs=4, n_steps=8, ppo_minibatches=2, ppo_epochs=2)),
                     ("mujoco_ppo_dp8", dict(num_envs=4, n_steps=16, ppo_minibatches=2, ppo_epochs=2))):
        tr = ActorCriticTrainer(preset(name, **_quiet(device="cpu", cuda_graph=False, **kw)))
        p0 = tr.flat.data.clone()
        for _ in range(2):
            tr.step()
        assert torch.isfinite(tr.flat.data).all() and (tr.flat.data != p0).any()
        assert 0.0 <= float(tr.stats["clipfrac"]) <= 1.0


def test_reference_regularisers_and_adaptive_lr():
    cfg = preset("basic_ac", **_quiet(algo="a2c", env="CartPole-v0", n_steps=16, num_envs=2, anneal_regularizers=True))
    tr = ActorCriticTrainer(cfg)
    lr0 = tr.actor_opt.get_lr()
    tr.step()
    assert abs(float(tr.ent_coef) - 1e-2) < 1e-9 and abs(float(tr.kl_coef) - 1.0) < 1e-9
    assert tr.actor_opt.get_lr() in (pytest.approx(lr0 * 1.5), pytest.approx(lr0 / 1.5), pytest.approx(lr0))
    assert float(tr.stats["kl"]) >= 0 and np.isfinite(float(tr.stats["ev_after"]))


def test_basic_ac_parity_trainer(tmp_path):
    from actor_critic_algs_on_tensorflow_amd.api import train
    log = tmp_path / "log.txt"
    r = train("basic_ac", env="CartPole-v0", total_updates=3, outdir=str(log), quiet=True, save_every=2,
              checkpoint_dir=str(tmp_path / "ck"), ep_length_stop=300)
    assert r.iterations == 3 and r.env_steps >= 3 * 7 * 8   # each batch: >= 300 steps or MAX_ROLLS = 7 episodes
    assert (tmp_path / "ck-CartPole-0.index").exists()
    from actor_critic_algs_on_tensorflow_amd.ckpt import codec
    t = codec.read(str(tmp_path / "ck-CartPole-0"))
    # Basic_AC names: discrete actor has no log-std variable; beta, gamma, lr are Variable, _1, _2; Adam slots saved
    assert "Actor/logits/kernel" in t and "Actor/Variable_2" in t and "Critic/Variable" in t
    assert "Actor/first_layer/kernel/Adam" in t and "Critic/beta1_power" in t


# ------------------------------------------------------------------------------------------------ distributed
def _dp_worker(rank, world, port, out_dir, n_envs=4, extra=None, updates=3, kl_defer=True):
    import torch.distributed as dist
    from actor_critic_algs_on_tensorflow_amd.parallel.dp import DataParallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = preset("cartpole_cpu", **_quiet(num_envs=n_envs, n_steps=5, seed=11, optimizer="adam", max_grad_norm=0.5,
                                          **(extra or {})))
    tr = ActorCriticTrainer(cfg, dp=DataParallel())
    tr._kl_defer_on = kl_defer
    lrs = []
    for _ in range(updates):
        tr.step()
        lrs.append(float(tr.actor_opt.get_lr()))
    issued = tr.dp.issued
    tr.flush_kl()   # a deferred KL (DP + norm_adv) is settled here, as at a checkpoint / the end of train()
    torch.save({"p": tr.flat.data.clone(), "kl": float(tr.stats["kl"]), "lr": float(tr.actor_opt.get_lr()),
                "lrs": lrs, "issued": issued}, os.path.join(out_dir, f"dp{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_gloo_equals_single_process_union_batch(tmp_path, world):
    """Sync DP over W ranks x 8/W envs == one process over the same 8 envs (grad all-reduce + global adv norm via
    the packed moments all-reduce)."""
    mp.spawn(_dp_worker, args=(world, _free_port(), str(tmp_path), 8 // world), nprocs=world, join=True)
    ps = [torch.load(tmp_path / f"dp{r}.pt", weights_only=True)["p"] for r in range(world)]
    for p in ps[1:]:
        assert torch.equal(p, ps[0]), "ranks diverged"
    cfg = preset("cartpole_cpu", **_quiet(num_envs=8, n_steps=5, seed=11, optimizer="adam", max_grad_norm=0.5))
    single = ActorCriticTrainer(cfg)
    for _ in range(3):
        single.step()
    assert torch.allclose(ps[0], single.flat.data, rtol=1e-4, atol=1e-6)


def test_dp_gloo_world4_ppo_kl_lr_and_bf16_buckets(tmp_path):
    """World-4 PPO (minibatch all-reduce per optimiser step, global adv norm, KL proxy all-reduced for the adaptive
    lr): ranks stay bit-identical; bf16 gradient buckets track the fp32 run."""
    extra = dict(algo="ppo", ppo_epochs=2, ppo_minibatches=2, kl_adaptive_lr=True, kl_coef=0.1)
    mp.spawn(_dp_worker, args=(4, _free_port(), str(tmp_path), 2, extra), nprocs=4, join=True)
    fp = [torch.load(tmp_path / f"dp{r}.pt", weights_only=True) for r in range(4)]
    for d in fp[1:]:
        assert torch.equal(d["p"], fp[0]["p"]) and d["kl"] == fp[0]["kl"]
    (tmp_path / "b").mkdir()
    mp.spawn(_dp_worker, args=(4, _free_port(), str(tmp_path / "b"), 2, dict(extra, grad_bucket_dtype="bf16")),
             nprocs=4, join=True)
    bf = [torch.load(tmp_path / "b" / f"dp{r}.pt", weights_only=True)["p"] for r in range(4)]
    for p in bf[1:]:
        assert torch.equal(p, bf[0])
    cfg = preset("cartpole_cpu", **_quiet(num_envs=2, n_steps=5, seed=11, optimizer="adam", max_grad_norm=0.5))
    p0 = ActorCriticTrainer(cfg).flat.data
    d_fp, d_bf = fp[0]["p"] - p0, bf[0] - p0
    cos = float(torch.nn.functional.cosine_similarity(d_fp.double(), d_bf.double(), dim=0))
    assert cos > 0.97, cos


def test_dp_gloo_kl_rides_in_moments_allreduce(tmp_path):
    """DP + global adv norm + KL-adaptive lr: the post-update KL is packed into the next update's moments
    all-reduce (one non-gradient collective per update instead of two). Same parameters, lr sequence (shifted by
    one update: applied before the next optimiser step instead of after this one) and settled KL as the
    standalone-collective schedule."""
    extra = dict(algo="ppo", ppo_epochs=2, ppo_minibatches=2, kl_adaptive_lr=True, desired_kl=1e-4, lr=3e-3)
    out = {}
    for defer in (True, False):
        d = tmp_path / str(defer)
        d.mkdir()
        mp.spawn(_dp_worker, args=(2, _free_port(), str(d), 2, extra, 6, defer), nprocs=2, join=True)
        out[defer] = [torch.load(d / f"dp{r}.pt", weights_only=True) for r in range(2)]
    a, b = out[True][0], out[False][0]
    assert torch.equal(a["p"], b["p"]) and a["lr"] == b["lr"] and a["kl"] == pytest.approx(b["kl"], rel=1e-6)
    assert a["lrs"][1:] == b["lrs"][:-1], (a["lrs"], b["lrs"])
    assert len(set(b["lrs"])) > 1, "the lr rule never fired: the comparison is vacuous"
    assert b["issued"] - a["issued"] == 6, (a["issued"], b["issued"])   # one KL collective per update saved
    assert torch.equal(out[True][1]["p"], a["p"]) and out[True][1]["kl"] == a["kl"]


def _dp_union_worker(rank, world, port, out_dir, name, kw):
    import torch.distributed as dist
    from actor_critic_algs_on_tensorflow_amd.parallel.dp import DataParallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = ActorCriticTrainer(preset(name, **_quiet(device="cpu", cuda_graph=False, **kw)), dp=DataParallel())
    for _ in range(3):
        tr.step()
    torch.save({"p": tr.flat.data.clone(), "env": tr.env.num_envs}, os.path.join(out_dir, f"u{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,kw,exact", [
    # MLP PPO (BASELINE config 5 shape, Gaussian head): one minibatch per epoch, so the union-batch step is the same
    ("mujoco_ppo_dp8", dict(n_steps=8, ppo_epochs=2, ppo_minibatches=1), True),
    # CNN PPO (BASELINE config 3 shape, Nature CNN on the autograd engine): Adam turns the fp32 summation-order noise
    # of near-zero gradients (dead ReLU units) into lr-sized steps, so the update is compared by direction and size
    ("breakout_ppo", dict(n_steps=4, ppo_epochs=2, ppo_minibatches=1), False),
])
def test_dp_gloo_world8_ppo_equals_union_batch(tmp_path, name, kw, exact):
    """World-8 data parallelism (the BASELINE node: 8 ranks, one env bank per rank): PPO with the
    minibatch gradient all-reduce and the global advantage moments == one process stepping the union batch of 8
    env banks (every rank's envs are its own: env ids offset by rank * N, so the union is the same 8 envs); ranks
    bit-identical."""
    world = 8
    mp.spawn(_dp_union_worker, args=(world, _free_port(), str(tmp_path), name, dict(kw, num_envs=1, seed=5)),
             nprocs=world, join=True)
    ps = [torch.load(tmp_path / f"u{r}.pt", weights_only=True)["p"] for r in range(world)]
    for p in ps[1:]:
        assert torch.equal(p, ps[0]), "ranks diverged"
    torch.set_num_threads(4)
    single = ActorCriticTrainer(preset(name, **_quiet(device="cpu", cuda_graph=False, **dict(kw, num_envs=world,
                                                                                              seed=5))))
    p0 = single.flat.data.clone()
    for _ in range(3):
        single.step()
    d8, d1 = ps[0] - p0, single.flat.data - p0
    assert d1.abs().max() > 0
    if exact:
        assert torch.allclose(ps[0], single.flat.data, rtol=1e-4, atol=1e-6), float((d8 - d1).abs().max())
    cos = float(torch.nn.functional.cosine_similarity(d8.double(), d1.double(), dim=0))
    assert cos > 0.999 and abs(float(d8.norm() / d1.norm()) - 1) < 1e-2, (cos, float(d8.norm() / d1.norm()))


def _a3c_proc(rank, world, port, d, ps=1, iters=6):
    from actor_critic_algs_on_tensorflow_amd.cli import train
    torch.set_num_threads(1)
    job = "ps" if rank < ps else "worker"
    task = rank if rank < ps else rank - ps
    out = train.main([job, str(task), "--env", "CartPole-v0", "--ps_num", str(ps), "--worker_num", str(world - ps),
                      "--initport", str(port), "--outdir", d + "/logs", "--checkpoint_dir", d + "/ck",
                      "--max_iters", str(iters), "--save_every", "3", "--quiet"])
    torch.save({"gstep": out["global_step"], "role": out["role"],
                "steps": [h["gstep"] for h in out.get("history", [])]}, f"{d}/r{rank}.pt")


def test_a3c_async_parameter_server(tmp_path):
    d = str(tmp_path)
    mp.spawn(_a3c_proc, args=(3, _free_port(), d), nprocs=3, join=True)
    ps = torch.load(f"{d}/r0.pt", weights_only=True)
    w0 = torch.load(f"{d}/r1.pt", weights_only=True)
    w1 = torch.load(f"{d}/r2.pt", weights_only=True)
    assert ps["role"] == "ps" and ps["gstep"] >= 6
    steps = sorted(w0["steps"] + w1["steps"])
    assert steps == list(range(1, len(steps) + 1)), "PS serialises applies: every global step taken once"
    assert os.path.exists(f"{d}/logs/worker_0.log") and os.path.exists(f"{d}/logs/worker_1.log")
    from actor_critic_algs_on_tensorflow_amd import ckpt
    latest = ckpt.latest_checkpoint(f"{d}/ck")
    t = ckpt.load_tensors(latest)
    assert "global_actor/logits/kernel" in t and "global_critic/Variable_1" in t


def test_a3c_eight_process_cluster_two_ps_six_workers(tmp_path):
    """An 8-process A3C cluster (2 parameter-server shards + 6 workers; the reference's default is 2 ps + 4 workers,
    A3C/train.py:15-16): the shards split the variables (greedy_ps_strategy), every push is applied once under one
    serialised global step, each worker's steps are increasing, and the chief's checkpoint holds every reference
    variable."""
    d = str(tmp_path)
    mp.spawn(_a3c_proc, args=(8, _free_port(), d, 2, 4), nprocs=8, join=True)
    roles = [torch.load(f"{d}/r{r}.pt", weights_only=True) for r in range(8)]
    assert [r["role"] for r in roles] == ["ps", "ps"] + ["worker"] * 6
    steps = sorted(s for r in roles[2:] for s in r["steps"])
    assert steps == list(range(1, len(steps) + 1)), "every global step taken exactly once across 6 workers"
    for r in roles[2:]:
        assert r["steps"] == sorted(r["steps"]) and len(r["steps"]) >= 1
    assert all(r["gstep"] >= 4 for r in roles[:2])
    for w in range(6):
        assert os.path.exists(f"{d}/logs/worker_{w}.log")
    from actor_critic_algs_on_tensorflow_amd import ckpt
    t = ckpt.load_tensors(ckpt.latest_checkpoint(f"{d}/ck"))
    assert "global_actor/logits/kernel" in t and "global_critic/value/bias" in t


def test_pendulum_ppo_solves_on_cpu_and_test_model_scores_checkpoint(tmp_path):
    """VERDICT r2 item 1 on the reference's own device (CPU, torch engine): preset pendulum_ppo -- the reference
    A3C actor / critic, gamma 0.98 -- swings Pendulum-v0 up (mean return > -400, the bar the shipped demo policy
    meets) within 55 updates (176k env steps; measured -160..-190 at 50-60 updates for seeds 1 and 7,
    profiles/r3_pendulum_learning.txt), and the reference-named checkpoint it saves scores > -400 in the
    evaluation CLI (cli/test_model.py)."""
    import numpy as np
    import torch
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    from actor_critic_algs_on_tensorflow_amd.cli import test_model
    nt = torch.get_num_threads()
    torch.set_num_threads(4)
    try:
        tr = ActorCriticTrainer(preset("pendulum_ppo", device="cpu", cuda_graph=False, outdir=None, quiet=True,
                                       stdout_freq=0, save_every=0, seed=1))
        rets = []
        for u in range(1, 56):
            tr.step()
            if u % 5 == 0:
                rets.append(tr.env.drain_episode_stats()[0])
    finally:
        torch.set_num_threads(nt)
    assert rets[0] < -900, rets
    assert np.mean(rets[-2:]) > -400, rets
    path = tr.save_checkpoint(str(tmp_path / "model-Pendulum-55"))
    rewards = test_model.main(["Pendulum-v0", path, "--num_episodes", "5", "--no_animation"])
    assert np.mean(rewards) > -400, rewards
