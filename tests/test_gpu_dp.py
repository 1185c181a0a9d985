"""Data-parallel schedules of the native engine on a real GPU (2 ranks sharing cuda:0 over gloo).

RCCL needs one GPU per rank, and the GPU box has one GPU, so these tests drive the SAME captured segments and
host-side collective schedule as the RCCL run (``ActorCriticTrainer._replay``) with the gloo backend (which
all-reduces CUDA tensors through host memory). What is checked:

* ``overlap="strict"`` (bucketed: fc/head gradients all-reduced while the conv backward runs, then the conv bucket):
  2 ranks x N envs == one rank x 2N envs (the env banks and the sampling keys are keyed by the global env id, so
  the union batch is the same data) -- and world-1 DP == the single-graph non-DP update;
* ``overlap="lag1"`` (all-reduce of update k overlapped with the rollout of k+1, applied one update late): the same
  2-rank == union equivalence, ranks bit-identical, and the delayed-gradient semantics (the first update applies
  nothing).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from actor_critic_algs_on_tensorflow_amd import preset

pytestmark = pytest.mark.gpu

UPDATES = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(num_envs, overlap):
    return preset("pong_a2c", num_envs=num_envs, n_steps=3, device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                  save_every=0, overlap=overlap, seed=5)


def _run(dp, num_envs, overlap, updates=UPDATES):
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    tr = ActorCriticTrainer(_cfg(num_envs, overlap), dp=dp)
    assert tr.engine is not None
    p0 = tr.flat.data.clone()
    tr.capture(warmup=1)
    assert tr.graph is not None
    kind = tr.graph[0]
    snaps = []
    for _ in range(updates):
        tr.step()
        torch.cuda.synchronize()
        snaps.append(tr.flat.data.clone())
    # the warm-up update before the capture moved the parameters too: report deltas from the post-capture start
    return p0, tr, kind, snaps


def _worker(rank, world, port, out_dir, num_envs, overlap):
    import torch.distributed as dist
    from actor_critic_algs_on_tensorflow_amd.parallel.dp import DataParallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, tr, kind, snaps = _run(DataParallel(), num_envs, overlap)
        torch.save({"snaps": [s.cpu() for s in snaps], "kind": kind},
                   os.path.join(out_dir, f"{overlap}_w{world}_r{rank}.pt"))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _spawn(tmp_path, world, num_envs, overlap):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), num_envs, overlap), nprocs=world, join=True)
    return [torch.load(tmp_path / f"{overlap}_w{world}_r{r}.pt", weights_only=True) for r in range(world)]


def _cos(a, b):
    return float(torch.nn.functional.cosine_similarity(a.double().flatten(), b.double().flatten(), dim=0))


@pytest.mark.parametrize("overlap", ["strict", "lag1"])
def test_dp_segments_union_equivalence(cuda, tmp_path, overlap):
    two = _spawn(tmp_path, 2, 8, overlap)
    one = _spawn(tmp_path, 1, 16, overlap)
    assert two[0]["kind"] == overlap and one[0]["kind"] == overlap
    for a, b in zip(two[0]["snaps"], two[1]["snaps"]):
        assert torch.equal(a, b), "ranks diverged"
    # per-update parameter deltas of the 2-rank run follow the 1-rank union run (bf16 MFMA, split-K atomics:
    # summation order differs, so compare directions and magnitudes, not bits)
    s2, s1 = two[0]["snaps"], one[0]["snaps"]
    for k in range(1, UPDATES):
        d2, d1 = s2[k] - s2[k - 1], s1[k] - s1[k - 1]
        assert d1.abs().max() > 0
        assert _cos(d2, d1) > 0.98, (k, _cos(d2, d1))
        assert abs(float(d2.norm() / d1.norm()) - 1.0) < 0.05


def test_dp_world1_strict_equals_single_graph(cuda, tmp_path):
    """The 3-segment bucketed update with a world-1 group == the one-graph update without DP."""
    one = _spawn(tmp_path, 1, 16, "strict")
    _, _, kind, snaps = _run(None, 16, "strict")
    assert kind == "single"
    for k in range(1, UPDATES):
        d_dp = one[0]["snaps"][k] - one[0]["snaps"][k - 1]
        d_sg = snaps[k].cpu() - snaps[k - 1].cpu()
        assert _cos(d_dp, d_sg) > 0.99, (k, _cos(d_dp, d_sg))
