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


def _cfg(num_envs, overlap, name="pong_a2c", **kw):
    base = dict(n_steps=3) if name == "pong_a2c" else {}
    base.update(kw)
    return preset(name, num_envs=num_envs, device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                  save_every=0, overlap=overlap, seed=5, **base)


def _run(dp, num_envs, overlap, updates=UPDATES, name="pong_a2c", capture=True, **kw):
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    tr = ActorCriticTrainer(_cfg(num_envs, overlap, name, **kw), dp=dp)
    assert tr.engine is not None or tr.mlp is not None
    p0 = tr.flat.data.clone()
    kind = "eager"
    if capture:
        tr.capture(warmup=1)
        assert tr.graph is not None, "DP update fell back to eager execution"
        kind = tr.graph[0]
    else:
        tr.step()   # the same one warm-up update the capture runs
    snaps = []
    for _ in range(updates):
        tr.step()
        torch.cuda.synchronize()
        snaps.append(tr.flat.data.clone())
    # the warm-up update before the capture moved the parameters too: report deltas from the post-capture start
    return p0, tr, kind, snaps


def _worker(rank, world, port, out_dir, num_envs, overlap, opts=None):
    import torch.distributed as dist
    from actor_critic_algs_on_tensorflow_amd.parallel.dp import DataParallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    opts = dict(opts or {})
    tag = opts.pop("tag", overlap)
    try:
        _, tr, kind, snaps = _run(DataParallel(), num_envs, overlap, **opts)
        n_graphs = tr.graph[1].n_graphs if kind == "segments" else None
        torch.save({"snaps": [s.cpu() for s in snaps], "kind": kind, "n_graphs": n_graphs},
                   os.path.join(out_dir, f"{tag}_w{world}_r{rank}.pt"))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _spawn(tmp_path, world, num_envs, overlap, **opts):
    tag = opts.get("tag", overlap)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), num_envs, overlap, opts), nprocs=world, join=True)
    return [torch.load(tmp_path / f"{tag}_w{world}_r{r}.pt", weights_only=True) for r in range(world)]


def _cos(a, b):
    return float(torch.nn.functional.cosine_similarity(a.double().flatten(), b.double().flatten(), dim=0))


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("overlap", ["strict", "lag1"])
def test_dp_segments_union_equivalence(cuda, tmp_path, overlap, world):
    two = _spawn(tmp_path, world, 16 // world, overlap)
    one = _spawn(tmp_path, 1, 16, overlap)
    assert two[0]["kind"] == overlap and one[0]["kind"] == overlap
    for r in range(1, world):
        for a, b in zip(two[0]["snaps"], two[r]["snaps"]):
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


def _deltas(snaps):
    return [snaps[k] - snaps[k - 1] for k in range(1, len(snaps))]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_ppo_captured_as_segments_equals_eager(cuda, tmp_path, world, monkeypatch):
    """Breakout-shaped PPO under DP (minibatch gradient all-reduces, global advantage normalisation via the packed
    fp64 moments, which also carry the KL proxy for the adaptive lr) is captured as a segment chain -- no eager
    fallback -- and its
    replay is BITWISE equal to the eager DP run (deterministic PPO backward: split-K planes + ordered finaliser,
    ordered bias sums; fixed GEMM plans so both processes run the same kernels); ranks stay bit-identical."""
    monkeypatch.setenv("ACAMD_GEMM_TUNE", "0")
    kw = dict(name="breakout_ppo", n_steps=8, ppo_epochs=2, ppo_minibatches=2, kl_adaptive_lr=True, kl_coef=0.05)
    cap = _spawn(tmp_path, world, 4, "strict", tag="ppo_cap", **kw)
    eag = _spawn(tmp_path, world, 4, "strict", tag="ppo_eager", capture=False, **kw)
    assert cap[0]["kind"] == "segments"
    # 4 gradient all-reduces + 1 packed all-reduce of the advantage moments and the previous update's KL -> 6 graphs
    assert cap[0]["n_graphs"] == 6, cap[0]["n_graphs"]
    for r in range(1, world):
        for a, b in zip(cap[0]["snaps"], cap[r]["snaps"]):
            assert torch.equal(a, b), "ranks diverged"
    for k, (a, b) in enumerate(zip(cap[0]["snaps"], eag[0]["snaps"])):
        assert torch.equal(a, b), (k, _cos(a, b))


@pytest.mark.parametrize("world", [2, 8])
def test_dp_mlp_ppo_captured_as_segments(cuda, tmp_path, world):
    """MuJoCo-shaped PPO on the MLP engine under DP (world 2, and the BASELINE node's 8 ranks): captured (segments),
    ranks identical, replay follows eager."""
    kw = dict(name="mujoco_ppo_dp8", n_steps=16, ppo_epochs=2, ppo_minibatches=4)
    cap = _spawn(tmp_path, world, 16 // world, "strict", tag="mlp_cap", **kw)
    eag = _spawn(tmp_path, world, 16 // world, "strict", tag="mlp_eager", capture=False, **kw)
    assert cap[0]["kind"] == "segments"
    for r in range(1, world):
        for a, b in zip(cap[0]["snaps"], cap[r]["snaps"]):
            assert torch.equal(a, b), "ranks diverged"
    for d_c, d_e in zip(_deltas(cap[0]["snaps"]), _deltas(eag[0]["snaps"])):
        assert _cos(d_c, d_e) > 0.99, _cos(d_c, d_e)


@pytest.mark.parametrize("overlap", ["strict", "lag1"])
def test_dp_bf16_buckets_track_fp32(cuda, tmp_path, overlap):
    """bf16 gradient buckets (half the all-reduce bytes): ranks identical, updates follow the fp32-bucket run."""
    b16 = _spawn(tmp_path, 2, 8, overlap, tag=f"{overlap}_b16", grad_bucket_dtype="bf16")
    f32 = _spawn(tmp_path, 2, 8, overlap, tag=f"{overlap}_f32")
    assert b16[0]["kind"] == overlap
    for a, b in zip(b16[0]["snaps"], b16[1]["snaps"]):
        assert torch.equal(a, b), "ranks diverged"
    for d_b, d_f in zip(_deltas(b16[0]["snaps"]), _deltas(f32[0]["snaps"])):
        assert _cos(d_b, d_f) > 0.97, _cos(d_b, d_f)


# ---------------------------------------------------------------------------------------------- RCCL, in-graph
def _rccl_worker(_idx, port, out_dir, name, kw, modes, overlap="strict"):
    """One process, an RCCL ("nccl") group of world 1 on cuda:0: the same DP update captured with the collectives
    INSIDE one hipGraph (``dp_capture="auto"``) and as the host-cut segment chain (``"segments"``)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ACAMD_GEMM_TUNE="0")
    import torch.distributed as dist
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    from actor_critic_algs_on_tensorflow_amd.parallel.dp import DataParallel
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        res = {}
        for mode in modes:
            dp = DataParallel()
            assert dp.backend == "nccl"
            tr = ActorCriticTrainer(_cfg(kw_envs(name), overlap, name, dp_capture=mode, **kw), dp=dp)
            tr.capture(warmup=1)
            kind = tr.graph[0]
            n_graphs = (tr.graph[1].n_graphs if kind == "segments" else
                        len(tr.graph) - 1 if kind in ("strict", "lag1") else 1)
            issued = dp.issued
            snaps = []
            for _ in range(UPDATES):
                tr.step()
                torch.cuda.synchronize()
                snaps.append(tr.flat.data.cpu().clone())
            res[mode] = {"kind": kind, "n_graphs": n_graphs, "host_collectives": dp.issued - issued,
                         "snaps": snaps}
        torch.save(res, os.path.join(out_dir, f"rccl_{name}_{overlap}.pt"))
    finally:
        dist.destroy_process_group()


def kw_envs(name):
    return {"pong_a2c": 16, "breakout_ppo": 4, "mujoco_ppo_dp8": 8}[name]


@pytest.mark.parametrize("name,kw", [
    ("pong_a2c", {}),
    ("breakout_ppo", dict(n_steps=8, ppo_epochs=2, ppo_minibatches=2, kl_adaptive_lr=True, kl_coef=0.05)),
    ("mujoco_ppo_dp8", dict(n_steps=16, ppo_epochs=2, ppo_minibatches=4, kl_adaptive_lr=True, kl_coef=0.05)),
])
def test_rccl_dp_update_is_one_graph(cuda, tmp_path, name, kw):
    """RCCL data parallelism (world 1 here; the driver's node runs 2-8): the whole DP update -- per-minibatch
    gradient all-reduces (CNN: fc/head bucket overlapped with the conv backward), the advantage moments, the KL
    scalar -- is ONE captured hipGraph whose replay issues zero collectives from the host, and it is BITWISE equal
    to the segment-chain capture of the same update (host-issued collectives between graphs)."""
    mp.spawn(_rccl_worker, args=(_free_port(), str(tmp_path), name, dict(kw), ["auto", "segments"]), nprocs=1,
             join=True)
    res = torch.load(tmp_path / f"rccl_{name}_strict.pt", weights_only=True)
    one, seg = res["auto"], res["segments"]
    assert one["kind"] == "single", one["kind"]
    assert one["host_collectives"] == 0, one["host_collectives"]
    assert seg["host_collectives"] > 0 and seg["n_graphs"] > 1
    for k, (a, b) in enumerate(zip(one["snaps"], seg["snaps"])):
        assert torch.equal(a, b), (k, _cos(a, b))
    assert not torch.equal(one["snaps"][0], one["snaps"][-1])


def test_rccl_lag1_one_graph_with_adam_equals_segments(cuda, tmp_path):
    """RCCL lag-1 A2C as one graph per update, with Adam: the first replay holds no gradient in the
    all-reduced copy C, so the gated optimiser launches apply nothing -- no moment decay, no step count -- exactly as
    the segmented lag-1 schedule, which skips its first optimiser graph on the host. Bitwise equal, every update."""
    mp.spawn(_rccl_worker, args=(_free_port(), str(tmp_path), "pong_a2c", dict(optimizer="adam"),
                                 ["auto", "segments"], "lag1"), nprocs=1, join=True)
    res = torch.load(tmp_path / "rccl_pong_a2c_lag1.pt", weights_only=True)
    one, seg = res["auto"], res["segments"]
    assert one["kind"] == "single" and seg["kind"] == "lag1", (one["kind"], seg["kind"])
    for k, (a, b) in enumerate(zip(one["snaps"], seg["snaps"])):
        assert torch.equal(a, b), (k, _cos(a, b))
    assert not torch.equal(one["snaps"][0], one["snaps"][-1])


def test_dp_world1_mlp_ppo_tracks_single_process(cuda, tmp_path):
    """MuJoCo-shaped PPO under DP at world 1 (the gradient all-reduce is the identity) follows the non-DP update: the
    global norm of the all-reduced gradient (a sum-of-squares launch) differs from the engine's per-tile partials
    only in summation order."""
    kw = dict(name="mujoco_ppo_dp8", n_steps=16, ppo_epochs=2, ppo_minibatches=4)
    one = _spawn(tmp_path, 1, 8, "strict", tag="mlp_w1", **kw)
    _, tr, _, snaps = _run(None, 8, "strict", **kw)
    for k, (d_dp, d_sg) in enumerate(zip(_deltas(one[0]["snaps"]), _deltas([s.cpu() for s in snaps]))):
        rel = float((d_dp - d_sg).norm() / d_sg.norm())
        assert rel < 1e-3, (k, rel)
