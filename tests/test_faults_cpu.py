"""Failure handling: a data-parallel rank killed by fault injection aborts the job cleanly (the
surviving rank's collective raises instead of hanging), and the job resumed from the newest checkpoint -- every
rank's env bank gathered into it -- finishes bit-identical to an uninterrupted run. gloo, 2 ranks, CPU."""
import os
import socket

import torch
import torch.multiprocessing as mp

from actor_critic_algs_on_tensorflow_amd.algos.trainer import FAULT_EXIT_CODE


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job(rank, world, port, d, ck, tag, total, fault, resume):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.api import train
    cfg = preset("cartpole_cpu", num_envs=4, n_steps=5, seed=11, outdir=None, quiet=True, stdout_freq=0,
                 save_every=2, checkpoint_dir=ck, total_updates=total, fault_inject=fault, resume=resume,
                 dist_backend="gloo", dist_timeout_s=60)
    try:
        res = train(cfg)
    except Exception as e:   # the surviving rank of a crashed job
        with open(os.path.join(d, f"{tag}_r{rank}.err"), "w") as f:
            f.write(repr(e))
        os._exit(3)
    if rank == 0:
        torch.save({"p": res.trainer.flat.data.clone(), "it": res.iterations}, os.path.join(d, f"{tag}.pt"))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def _run(world, *args, timeout=240):
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_job, args=(r, world, _free_port_for(args)) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    codes = [p.exitcode for p in procs]
    for p in procs:   # the exact child objects, never a pattern
        if p.is_alive():
            p.kill()
    return codes


_PORTS = {}


def _free_port_for(args):
    key = args[2]   # one rendezvous port per job tag
    if key not in _PORTS:
        _PORTS[key] = _free_port()
    return _PORTS[key]


def test_rank_failure_aborts_and_resume_is_exact(tmp_path):
    d = str(tmp_path)
    # uninterrupted reference: 6 updates
    assert _run(2, d, os.path.join(d, "ck_ref"), "ref", 6, None, None) == [0, 0]
    # rank 1 dies when it reaches iteration 3 (checkpoints were written after iterations 0 and 2)
    ck = os.path.join(d, "ck_crash")
    codes = _run(2, d, ck, "crash", 6, "1:3", None)
    assert codes[1] == FAULT_EXIT_CODE, codes
    assert codes[0] == 3 and os.path.exists(os.path.join(d, "crash_r0.err")), codes
    from actor_critic_algs_on_tensorflow_amd import ckpt
    latest = ckpt.latest_checkpoint(ck)
    assert latest.endswith("-3")
    t = ckpt.load_tensors(latest)
    assert "_acamd/env/rank1/state" in t and int(t["_acamd/world_size"]) == 2
    # resume from the newest checkpoint and finish the remaining 3 updates
    assert _run(2, d, ck, "resume", 6, None, "auto") == [0, 0]
    ref = torch.load(os.path.join(d, "ref.pt"), weights_only=True)
    res = torch.load(os.path.join(d, "resume.pt"), weights_only=True)
    assert ref["it"] == res["it"] == 6
    assert torch.equal(ref["p"], res["p"]), "resumed DP run must match the uninterrupted run bit for bit"


def test_sync_trainer_rejects_ps_exchange_fault_points():
    """'rank:iteration:push|reply' names a fault point inside the async PS worker's exchange; the synchronous trainer
    refuses it instead of silently never injecting the fault."""
    import pytest
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    cfg = preset("cartpole_cpu", outdir=None, quiet=True, stdout_freq=0, save_every=0, fault_inject="0:1:push",
                 total_updates=2)
    tr = ActorCriticTrainer(cfg)
    with pytest.raises(ValueError, match="parameter-server"):
        tr.train()
