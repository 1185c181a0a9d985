"""GPU-native async parameter-server mode (algos/a3c_gpu.py; reference A3C/process.py:156-288): vectorised device
workers push gradients / pull parameters, the PS applies them serially with the fused Adam kernel and per-worker
step counts. CPU runs (gloo, world 3 and 4) check the protocol; the GPU run shares cuda:0 between three ranks
(gloo data plane staged through host memory -- RCCL needs one GPU per rank)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from actor_critic_algs_on_tensorflow_amd import preset


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(device, total, **kw):
    base = dict(num_envs=4, n_steps=8, total_updates=total, outdir=None, quiet=True, stdout_freq=0, save_every=0,
                device=device, cuda_graph=device.startswith("cuda"), seed=7)
    base.update(kw)
    return preset("a3c", **base)


def _proc(rank, world, port, out, device, total, ps_num, staleness, kw, report=0):
    import datetime
    import torch.distributed as dist
    from actor_critic_algs_on_tensorflow_amd.algos import a3c_gpu
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if device.startswith("cuda"):
        torch.cuda.set_device(0)
    kw = dict(kw)
    log_dir = kw.pop("_log_dir", None)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=kw.get("dist_timeout_s", 300)))
    try:
        res = a3c_gpu.run(_cfg(device, total, **kw), ps_num=ps_num, data_backend="gloo", max_staleness=staleness,
                          device=device, report_every=report, log_dir=log_dir)
        torch.save(res, os.path.join(out, f"r{rank}.pt"))
        if not kw.get("fault_inject"):
            dist.barrier()
    except RuntimeError as e:   # a surviving worker of a job whose PS aborted
        torch.save({"role": "worker", "error": repr(e)}, os.path.join(out, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _run(tmp_path, world, device="cpu", total=12, ps_num=1, staleness=1, report=0, **kw):
    mp.spawn(_proc, args=(world, _free_port(), str(tmp_path), device, total, ps_num, staleness, kw, report),
             nprocs=world, join=True)
    return [torch.load(tmp_path / f"r{r}.pt", weights_only=False) for r in range(world)]


def _check(res, ps_num, staleness, total):
    ps, workers = res[:ps_num], res[ps_num:]
    W = len(workers)
    for p in ps:
        assert p["role"] == "ps"
        log = p["log"]
        # serialised global steps: every apply takes exactly the next step
        assert [g for _, _, g in log] == list(range(len(log)))
        assert p["global_step"] == len(log) >= total
        # bounded staleness (stale-synchronous bound s on the apply counts): while a worker computes, each other
        # worker can catch up from s + 1 behind and run s + 1 ahead, so no gradient is older than 2 (W - 1)(s + 1)
        # global steps (a round-end GPU run logged w2: version 1 applied at step 4 after w1's steps 1-3, W = 2, s = 1)
        if staleness >= 0:
            assert max(g - v for _, v, g in log) <= 2 * (W - 1) * (staleness + 1), log
        # per-worker Adam step counts == that worker's applies
        for key, t in p["adam_t"].items():
            w = int(key.split(":")[1])
            assert t == p["n_applies"][w], (key, t, p["n_applies"])
        assert torch.isfinite(p["params"]).all()
    for w in workers:
        assert w["role"] == "worker" and w["updates"] >= 1
    assert sum(ps[0]["n_applies"].values()) == ps[0]["global_step"]


def test_a3c_gpu_mode_protocol_cpu(tmp_path):
    res = _run(tmp_path, 3, staleness=1)
    _check(res, 1, 1, 12)


def test_a3c_gpu_mode_two_ps_shards_three_workers_cpu(tmp_path):
    res = _run(tmp_path, 5, ps_num=2, staleness=0, total=9)
    _check(res, 2, 0, 9)
    n = [r["params"].numel() for r in res[:2]]
    assert all(k > 0 for k in n)


@pytest.mark.gpu
def test_a3c_gpu_workers_on_device(cuda, tmp_path):
    """Workers run the device engines (env bank + hipGraph-captured segments on cuda:0); the PS holds its slab and
    Adam moments on the device and applies with the native fused Adam kernel."""
    res = _run(tmp_path, 3, device="cuda:0", staleness=1, total=30)
    _check(res, 1, 1, 30)


@pytest.mark.gpu
def test_a3c_gpu_worker_learns_cartpole(cuda, tmp_path):
    """The reference's own update (preset a3c: one element-clipped Adam step per batch with the KL-adaptive actor
    lr, capped at the reference's 0.1, A3C/process.py:12) trained THROUGH the device parameter server: CartPole-v0
    (the reference's other env, its discrete head), 32 envs x 16 steps per worker update. One worker makes the run
    deterministic (serial applies, deterministic kernels). The mean episode length (= return; random play lasts
    about 20 steps) must reach 140.

    Pendulum with this update at the reference geometry is seed-dependent in the reference's own algorithm: an
    independent plain-PyTorch oracle of the worker update (scripts/exp/a3c_oracle.py) reaches -121 / -185 on two of
    four seeds and stalls on the other two, and this framework's update equals the oracle's to 1e-6 per update
    (tests/test_a3c_update_parity_cpu.py; profiles/r4_a3c_parity_and_seeds.txt has the per-seed curves). The
    framework's reliable Pendulum solve is test_gpu_learning.py::test_pendulum_ppo_solves_and_checkpoint_evaluates
    (PPO on the reference networks)."""
    res = _run(tmp_path, 2, device="cuda:0", staleness=-1, total=2000, report=400, num_envs=32, n_steps=16,
               seed=12321, max_lr=0.1, env="CartPole-v0")
    _check(res, 1, -1, 2000)
    rets = [r[2] for r in res[1]["returns"]]
    assert len(rets) >= 4, rets
    assert max(rets[-2:]) > 140 and max(rets[-2:]) > rets[0] + 40, rets


def test_a3c_gpu_mode_chief_checkpoints_and_worker_logs_cpu(tmp_path):
    """A3C/process.py:211-214,280-283: the chief writes the GLOBAL actor/critic under the reference names every
    save_every global steps (evaluable by cli/test_model.py), every worker keeps a reference-format log file."""
    from actor_critic_algs_on_tensorflow_amd import ckpt
    from actor_critic_algs_on_tensorflow_amd.api import evaluate
    ck = tmp_path / "ck"
    res = _run(tmp_path, 3, staleness=-1, total=9, save_every=4, checkpoint_dir=str(ck), stdout_freq=1,
               flush_every=2, _log_dir=str(tmp_path / "logs"))
    ps, w0, w1 = res
    assert ps["status"] == "ok"
    latest = ckpt.latest_checkpoint(str(ck))
    assert latest is not None and latest.endswith("-%d" % w0["global_step"]), (latest, w0["global_step"])
    t = ckpt.load_tensors(latest)
    assert "global_actor/first_layer/kernel" in t and "global_critic/value/bias" in t
    # the chief's final checkpoint holds the PS parameters (its last pull)
    assert len(w0["checkpoints"]) >= 2 and not w1["checkpoints"]
    rewards = evaluate(latest, "Pendulum-v0", num_episodes=1, verbose=False, max_path_length=20)
    assert len(rewards) == 1
    for task in (0, 1):
        rows = open(tmp_path / "logs" / f"worker_{task}.log").read().splitlines()
        assert rows[0].split()[:3] == ["step", "avg_rew", "ev_before"] and len(rows) > 1


def test_a3c_gpu_mode_worker_death_aborts_cleanly_cpu(tmp_path):
    """a worker dying mid-run (no DONE message) makes the PS return "aborted" instead of serving
    forever, and the surviving worker's next exchange fails -- every process ends, nothing hangs."""
    import multiprocessing
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import FAULT_EXIT_CODE
    ctx = multiprocessing.get_context("spawn")
    port = _free_port()
    # rank 2 (worker 1) dies when it reaches its 3rd iteration
    args = (3, port, str(tmp_path), "cpu", 40, 1, -1, dict(fault_inject="2:3", dist_timeout_s=30))
    procs = [ctx.Process(target=_proc, args=(r,) + args) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(150)
    alive = [p.is_alive() for p in procs]
    for p in procs:   # the exact child objects, never a pattern
        if p.is_alive():
            p.kill()
    assert not any(alive), "a process of the job hung after a worker died"
    assert procs[2].exitcode == FAULT_EXIT_CODE
    ps = torch.load(tmp_path / "r0.pt", weights_only=False)
    assert ps["role"] == "ps" and ps["status"] == "aborted", ps.get("status")
    # the dead worker's applies stop at its fault; the survivor either finished the job through the PS or got an
    # error from its exchange -- both are clean ends
    assert ps["n_applies"][2] <= 3
    w0 = torch.load(tmp_path / "r1.pt", weights_only=False)
    assert "error" in w0 or w0["global_step"] >= 40


@pytest.mark.parametrize("where", ["push", "reply"])
def test_a3c_gpu_mode_worker_death_mid_exchange_cpu(tmp_path, where):
    """a worker that dies INSIDE an exchange -- after its push header but before the payload ("push"),
    or after the push while the PS is about to reply ("reply") -- ends the PS with status "aborted" (its payload
    receive / reply send fails), never with an exception escaping serve() and never with a hang. One worker, no
    staleness bound: the PS's next peer I/O is with the dead worker."""
    import multiprocessing
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import FAULT_EXIT_CODE
    ctx = multiprocessing.get_context("spawn")
    port = _free_port()
    args = (2, port, str(tmp_path), "cpu", 40, 1, -1, dict(fault_inject=f"1:2:{where}", dist_timeout_s=30))
    procs = [ctx.Process(target=_proc, args=(r,) + args) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(150)
    alive = [p.is_alive() for p in procs]
    for p in procs:   # the exact child objects, never a pattern
        if p.is_alive():
            p.kill()
    assert not any(alive), "a process of the job hung after a worker died mid-exchange"
    assert procs[1].exitcode == FAULT_EXIT_CODE
    assert procs[0].exitcode == 0, "the PS must end cleanly (no escaped exception)"
    ps = torch.load(tmp_path / "r0.pt", weights_only=False)
    assert ps["role"] == "ps" and ps["status"] == "aborted", ps.get("status")
    # iterations 0, 1 applied; "reply": iteration 2's payload arrived and was applied before the reply failed
    assert ps["n_applies"][1] == (3 if where == "reply" else 2), ps["n_applies"]


def _pf_proc(rank, port, d):
    from actor_critic_algs_on_tensorflow_amd.compat import reference as ref
    cluster = {"ps": [f"localhost:{port}"], "worker": [f"localhost:{port + 1}", f"localhost:{port + 2}"]}
    job, task = ("ps", 0) if rank == 0 else ("worker", rank - 1)
    logger = ref.Logger(f"{d}/w{task}.log", quiet=True) if job == "worker" else None
    out = ref.process_fn(cluster, task, job, "CartPole-v0", logger, f"{d}/ck", 0, random_seed=5, save_every=2,
                         checkpoint_basename="model-CartPole", max_iters=4)
    if logger is not None:
        logger.close()
    torch.save({"role": out["role"], "gstep": out["global_step"]}, f"{d}/pf{rank}.pt")


def test_process_fn_reference_signature(tmp_path):
    """compat.reference.process_fn(cluster, task_id, job, env_id, logger, save_path, ...) runs the async job."""
    d = str(tmp_path)
    mp.spawn(_pf_proc, args=(_free_port(), d), nprocs=3, join=True)
    ps = torch.load(f"{d}/pf0.pt", weights_only=True)
    assert ps["role"] == "ps" and ps["gstep"] >= 4
    assert any(n.startswith("model-CartPole-") for n in os.listdir(f"{d}/ck"))
    assert os.path.exists(f"{d}/w0.log")


def test_cpu_ps_per_worker_adam_step_count():
    """the CPU PS's Adam bias correction uses the SENDER's own step count (reference workers each own an
    Adam whose beta powers advance only with their applies): worker B's first apply after two of worker A's uses
    t = 1, i.e. the TF formula lr * sqrt(1 - b2) / (1 - b1) * m / (sqrt(v) + eps)."""
    import numpy as np
    from actor_critic_algs_on_tensorflow_amd.algos.a3c import ParameterServer

    class _Shard:
        sizes, is_actor = [4], [False]
        shard_vars, shard_numel = [[0]], [4]

    ps = ParameterServer(_Shard(), 0, torch.zeros(4), [1, 2], critic_lr=0.01)
    g = torch.tensor([1.0, -2.0, 0.5, 0.0])
    ps.apply(g, 0.0, src=1)
    ps.apply(g, 0.0, src=1)
    m_prev, v_prev = ps.adam.m.clone(), ps.adam.v.clone()
    p_prev = ps.params.detach().clone()
    ps.apply(g, 0.0, src=2)
    b1, b2, eps = ps.adam.b1, ps.adam.b2, ps.adam.eps
    m = b1 * m_prev + (1 - b1) * g
    v = b2 * v_prev + (1 - b2) * g * g
    lr_t = 0.01 * np.sqrt(1 - b2) / (1 - b1)   # t = 1 for worker 2
    torch.testing.assert_close(ps.params.detach(), p_prev - lr_t * m / (torch.sqrt(v) + eps))
    assert ps.worker_t == {1: 2, 2: 1} and ps.global_step == 3
