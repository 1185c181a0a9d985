"""GPU tests of the round-2 kernels (row-split trunk, ...) against the kernels / fp32 oracles they replace."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trunk_inputs(cuda, B, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    W1 = (torch.randn(32, 256, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    W2 = (torch.randn(64, 512, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    W3 = (torch.randn(64, 576, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    b1, b2, b3 = ((torch.rand(n, generator=g) * 0.1 - 0.02).to(cuda) for n in (32, 64, 64))
    return obs, W1, b1, W2, b2, W3, b3


@pytest.mark.parametrize("B", [1, 7, 32, 37])
def test_trunk_rows_bitwise_equals_per_env_trunk(cuda, B):
    """7 row workgroups per env (receptive fields recomputed, each output row stored by its owner; modes 1 / 2) == the
    one workgroup per env kernel (mode 3, bf16-staged), bit for bit, including the frame-stack shift; copy_out == the
    observation."""
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    obs, W1, b1, W2, b2, W3, b3 = _trunk_inputs(cuda, B)
    outs = []
    for mode in (3, 1, 2):
        ys = [torch.full((B * r, c), float("nan"), dtype=torch.bfloat16, device=cuda)
              for r, c in ((400, 32), (81, 64), (49, 64))]
        sh = torch.full_like(obs, 7)
        cp = torch.full_like(obs, 9) if mode in (1, 2) else None
        G.cnn_trunk_fwd(obs, W1, b1, W2, b2, W3, b3, *ys, shift_out=sh, mode=mode, copy_out=cp)
        torch.cuda.synchronize()
        outs.append((ys, sh, cp))
    (y0, s0, _) = outs[0]
    for (y1, s1, c1) in outs[1:]:
        for a, b in zip(y0, y1):
            assert not torch.isnan(b.float()).any(), "row-split trunk left an activation row unwritten"
            assert torch.equal(a.view(torch.int16), b.view(torch.int16))
        assert torch.equal(s0[:, :3], s1[:, :3]) and torch.equal(s1[:, :3], obs[:, 1:])
        assert (s1[:, 3] == 7).all(), "the newest frame slot is the env kernel's to render"
        if c1 is not None:
            assert torch.equal(c1, obs)


@pytest.mark.parametrize("B", [1, 5, 160])
def test_trunk_bwd_matches_conv_transpose(cuda, B):
    """Fused per-sample data-gradient chain vs fp32 torch conv_transpose2d on the same bf16 inputs: dy2 = tconv(dy3,
    W3) * (y2 > 0), dy1 = tconv(dy2_bf16, W2) * (y1 > 0), and the per-sample bias-gradient partials."""
    import torch.nn.functional as F
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(3)
    dy3 = (torch.randn(B, 7, 7, 64, generator=g) * (torch.rand(B, 7, 7, 64, generator=g) > 0.4)).to(torch.bfloat16)
    W3 = (torch.randn(64, 3, 3, 64, generator=g) * 0.05).to(torch.bfloat16)        # OHWI
    W2 = (torch.randn(64, 4, 4, 32, generator=g) * 0.05).to(torch.bfloat16)
    y2 = (torch.rand(B, 9, 9, 64, generator=g) - 0.3).clamp(min=0).to(torch.bfloat16)
    y1 = (torch.rand(B, 20, 20, 32, generator=g) - 0.3).clamp(min=0).to(torch.bfloat16)
    dev = [t.to(cuda) for t in (dy3, W3, y2, W2, y1)]
    dy2 = torch.full((B * 81, 64), float("nan"), dtype=torch.bfloat16, device=cuda)
    dy1 = torch.full((B * 400, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
    bp = torch.full((B, 160), float("nan"), device=cuda)
    ops.cnn_trunk_bwd(dev[0].reshape(B * 49, 64), dev[1].reshape(64, 576), dev[2].reshape(B * 81, 64),
                      dev[3].reshape(64, 512), dev[4].reshape(B * 400, 32), dy2, dy1, bp)
    torch.cuda.synchronize()
    r2 = F.conv_transpose2d(dy3.float().permute(0, 3, 1, 2), W3.float().permute(0, 3, 1, 2), stride=1)
    r2 = r2.permute(0, 2, 3, 1) * (y2.float() > 0)                                     # [B, 9, 9, 64]
    got2 = dy2.float().cpu().view(B, 9, 9, 64)
    assert torch.allclose(got2, r2, rtol=2e-2, atol=2e-2), (got2 - r2).abs().max()
    # dy1 from the kernel's own bf16 dy2 (the chain's rounding point)
    r1 = F.conv_transpose2d(got2.permute(0, 3, 1, 2), W2.float().permute(0, 3, 1, 2), stride=2)
    r1 = r1.permute(0, 2, 3, 1) * (y1.float() > 0)                                     # [B, 20, 20, 32]
    got1 = dy1.float().cpu().view(B, 20, 20, 32)
    assert torch.allclose(got1, r1, rtol=2e-2, atol=2e-2), (got1 - r1).abs().max()
    bpc = bp.cpu()
    assert torch.allclose(bpc[:, :64], dy3.float().sum((1, 2)), rtol=1e-4, atol=1e-4)
    assert torch.allclose(bpc[:, 64:128], got2.sum((1, 2)), rtol=1e-4, atol=1e-3)
    assert torch.allclose(bpc[:, 128:], got1.sum((1, 2)), rtol=1e-4, atol=1e-3)
    # bitwise reproducible
    dy1b, bpb = dy1.clone(), bp.clone()
    ops.cnn_trunk_bwd(dev[0].reshape(B * 49, 64), dev[1].reshape(64, 576), dev[2].reshape(B * 81, 64),
                      dev[3].reshape(64, 512), dev[4].reshape(B * 400, 32), dy2, dy1, bp)
    torch.cuda.synchronize()
    assert torch.equal(dy1b.view(torch.int16), dy1.view(torch.int16)) and torch.equal(bpb, bp)
    # the persistent form (weights staged once, workgroups walking the samples) is bit-identical
    dy2b = dy2.clone()
    for persist in (3, 256):
        dy2.fill_(float("nan")), dy1.fill_(float("nan")), bp.fill_(float("nan"))
        ops.cnn_trunk_bwd(dev[0].reshape(B * 49, 64), dev[1].reshape(64, 576), dev[2].reshape(B * 81, 64),
                          dev[3].reshape(64, 512), dev[4].reshape(B * 400, 32), dy2, dy1, bp, None, persist)
        torch.cuda.synchronize()
        assert torch.equal(dy2b.view(torch.int16), dy2.view(torch.int16)), persist
        assert torch.equal(dy1b.view(torch.int16), dy1.view(torch.int16)), persist
        assert torch.equal(bpb, bp), persist


def _one_update(fused, algo="pong_a2c", head=True, **kw):
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    cfg = preset(algo, num_envs=8, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0,
                 cuda_graph=False, optimizer="adam", **kw)
    tr = ActorCriticTrainer(cfg)
    tr.engine.fused_bwd = fused
    tr.engine.fused_head = head
    p0 = tr.flat.data.clone()
    tr.step()
    torch.cuda.synchronize()
    return tr.flat.data - p0, tr.stats_buf.clone()


@pytest.mark.parametrize("algo,kw", [("pong_a2c", {}), ("breakout_ppo", dict(n_steps=16, ppo_minibatches=2,
                                                                              ppo_epochs=1))])
def test_fused_backward_update_matches_gemm_backward(cuda, algo, kw):
    """One optimiser step with the fused data-gradient kernel + finaliser == the transposed-conv GEMM backward
    (same loss statistics, same parameter update up to bf16 rounding order)."""
    d1, s1 = _one_update(True, algo, **kw)
    d0, s0 = _one_update(False, algo, **kw)
    assert torch.allclose(s0, s1, rtol=1e-3, atol=1e-5)
    assert (d0 - d1).norm() / d0.norm() < 2e-2, float((d0 - d1).norm() / d0.norm())


def test_grad_finalize_planes_and_norm(cuda):
    """grad_finalize: plane sums in fixed order into dst, read-only segments untouched, sum-of-squares partials of
    the final gradient over both kinds of segment."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(0)
    slab = torch.randn(70001, generator=g).to(cuda)
    planes = torch.randn(7, 1003, generator=g).to(cuda)     # 7 planes of a 1003-element gradient (stride 1003)
    rows = torch.randn(33, 160, generator=g).to(cuda)       # per-sample rows, columns 64..127 -> a 64-element bias
    dA, dB = slab[10:1013], slab[2000:2064]
    ro = slab[3000:70001]
    from actor_critic_algs_on_tensorflow_amd.ops.optim import finalize_jobs
    words = finalize_jobs([(dA.data_ptr(), planes.data_ptr(), 1003, 1003, 7),
                           (dB.data_ptr(), rows.data_ptr() + 64 * 4, 64, 160, 33),
                           (ro.data_ptr(), 0, ro.numel(), 0, 0)], cuda)
    keep = ro.clone()
    parts = torch.full((256,), float("nan"), device=cuda)
    ops.grad_finalize(words, parts)
    torch.cuda.synchronize()
    assert torch.allclose(dA, planes.sum(0), atol=1e-5)
    assert torch.allclose(dB, rows[:, 64:128].sum(0), atol=1e-5)
    assert torch.equal(ro, keep)
    tot = float(parts.double().sum())
    ref = float(dA.double().pow(2).sum() + dB.double().pow(2).sum() + ro.double().pow(2).sum())
    assert abs(tot - ref) <= 1e-4 * ref


@pytest.mark.parametrize("norm_adv,returns", [(False, "nstep"), (True, "gae")])
def test_fused_head_matches_loss_plus_head_gemms(cuda, norm_adv, returns):
    """head_bwd (loss + dz + dh + dWh + dbh + dbfc in one launch) == ac_loss + the dh / dWh GEMMs + colsums: same
    statistics, same update up to summation order."""
    d1, s1 = _one_update(True, head=True, norm_adv=norm_adv, returns=returns)
    d0, s0 = _one_update(True, head=False, norm_adv=norm_adv, returns=returns)
    assert torch.allclose(s0[:8], s1[:8], rtol=1e-4, atol=1e-6), (s0[:8], s1[:8])
    assert (d0 - d1).norm() / d0.norm() < 1e-2, float((d0 - d1).norm() / d0.norm())


def test_a2c_update_is_bitwise_deterministic(cuda):
    """Two identical native A2C runs (graph-captured, 5 updates) end bit-identical."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    outs = []
    for _ in range(2):
        cfg = preset("pong_a2c", num_envs=16, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0)
        tr = ActorCriticTrainer(cfg)
        tr.capture(warmup=1)
        for _ in range(5):
            tr.step()
        torch.cuda.synchronize()
        outs.append((tr.flat.data.clone(), tr.stats_buf.clone()))
    assert torch.equal(outs[0][0], outs[1][0]), "parameters differ between identical runs"
    assert torch.equal(outs[0][1], outs[1][1])


def test_mb_gather_equals_index_select_of_keyed_permutation(cuda):
    """PPO minibatch gather (one launch: keyed epoch permutation evaluated in the kernel + every row copied) ==
    index_select with the oracle permutation (envs/rng.py prp), bit for bit."""
    from actor_critic_algs_on_tensorflow_amd import _native
    from actor_critic_algs_on_tensorflow_amd.envs import rng
    ops = _native.require()
    n, mb, seed = 1000, 250, 12345
    g = torch.Generator(device="cpu").manual_seed(3)
    obs = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    act = torch.randint(0, 6, (n,), dtype=torch.int32, generator=g).to(cuda)
    fl = [torch.randn(n, generator=g).to(cuda) for _ in range(4)]
    uc = torch.tensor([7], dtype=torch.int64, device=cuda)
    for ep, k in ((0, 0), (2, 3)):
        outs = [torch.empty(mb, 4, 84, 84, dtype=torch.uint8, device=cuda),
                torch.empty(mb, dtype=torch.int32, device=cuda)] + [torch.empty(mb, device=cuda) for _ in range(4)]
        ops.mb_gather(obs, act, *fl, *outs, seed, uc, ep, k * mb)
        key = rng.minibatch_key(seed, torch.tensor(7), ep)
        sel = rng.prp(torch.arange(k * mb, (k + 1) * mb, dtype=torch.int64), n, key).to(cuda)
        for src, out in zip([obs, act] + fl, outs):
            assert torch.equal(torch.index_select(src, 0, sel), out)
        # deferred advantage normalisation (fp64 totals [count, sum, sum of squares] of the whole batch)
        adv = fl[1].double()
        mom = torch.stack([torch.tensor(float(n), dtype=torch.float64, device=cuda), adv.sum(), (adv * adv).sum()])
        o_adv = torch.empty(mb, device=cuda)
        ops.mb_gather(obs, act, *fl, outs[0], outs[1], outs[2], o_adv, outs[4], outs[5], seed, uc, ep, k * mb, mom,
                      1e-8)
        ref = (fl[1] - fl[1].mean()) / (1e-8 + fl[1].std(unbiased=False))
        torch.testing.assert_close(o_adv, torch.index_select(ref, 0, sel), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name", ["breakout_ppo", "mujoco_ppo_dp8"])
def test_ppo_graph_replay_bitwise_equals_eager(cuda, name, monkeypatch):
    """Single-device PPO: the captured update replays bit-for-bit what the eager update computes (same kernels,
    deterministic reductions), over several updates with the keyed minibatch permutation and adv normalisation."""
    monkeypatch.setattr("actor_critic_algs_on_tensorflow_amd.ops.gemm.TUNE", False)
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    kw = dict(num_envs=8, n_steps=16, ppo_epochs=2, ppo_minibatches=4, device="cuda:0", outdir=None, quiet=True,
              stdout_freq=0, save_every=0, seed=3)
    if name == "breakout_ppo":
        kw.update(kl_adaptive_lr=True, kl_coef=0.05)
    runs = []
    for capture in (True, False):
        tr = ActorCriticTrainer(preset(name, **kw))
        if capture:
            tr.capture(warmup=1)
            assert tr.graph is not None and tr.graph[0] == "single"
        else:
            tr.step()
        snaps = []
        uc0 = int(tr.update_counter)
        for _ in range(3):
            tr.step()
            snaps.append(tr.flat.data.clone())
        torch.cuda.synchronize()
        assert int(tr.update_counter) == uc0 + 3   # advanced in-kernel by the last minibatch of each update
        runs.append(snaps)
    for k, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), k


@pytest.mark.parametrize("env_id", ["PongNoFrameskip-v4", "CartPole-v1", "Pendulum-v0"])
def test_agent_act_runs_native_engine(cuda, env_id):
    """Public Agent.act on a GPU runs the HIP engines (CNN trunk/head + sampling kernel; fused MLP towers +
    sampling) and draws the same actions as the PyTorch modules from the same counter-based keys."""
    import numpy as np
    from actor_critic_algs_on_tensorflow_amd import Agent
    from actor_critic_algs_on_tensorflow_amd import envs as E
    nat = Agent.for_env(env_id, device="cuda:0", seed=4)
    ref = Agent.for_env(env_id, device="cuda:0", seed=4)
    ref.engine_kind = "torch"
    env = E.make(env_id, 64, device="cpu", seed=2, frame_stack=4 if "Pong" in env_id else 1)
    obs = torch.zeros((64,) + tuple(env.obs_shape), dtype=env.obs_dtype)
    env.reset(out=obs)
    a1, lp1, e1 = nat.act(obs.numpy())
    a2, lp2, e2 = ref.act(obs.numpy())
    assert nat._eng is not None and ref._eng is None
    if "Pong" in env_id:   # bf16 engine vs fp32 modules: near-ties may flip a few draws
        assert np.mean(a1 == a2) > 0.9
        assert np.abs(lp1 - lp2)[a1 == a2].max() < 0.05
    else:
        np.testing.assert_allclose(a1, a2, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(lp1, lp2, rtol=1e-3, atol=1e-3)
        np.testing.assert_allclose(e1, e2, rtol=1e-3, atol=1e-3)


def test_grouped_gemm_launch_equals_separate_launches(cuda):
    """{dWfc, dy3} and {dW3, dW2, dW1} as ONE grouped launch each == the same products launched one by one, bit for
    bit (same tile plans), and the grouped kernel really ran (not the per-product fallback)."""
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    B = 160
    g = torch.Generator(device="cpu").manual_seed(9)

    def bf(*shape):
        return (torch.randn(*shape, generator=g) * 0.1).to(torch.bfloat16).to(cuda)

    y3, dh, Wfc = bf(B * 49, 64), bf(B, 512), bf(3136, 512)
    dy3m = bf(B, 3136)
    dy2, dy1, y2, y1 = bf(B * 81, 64), bf(B * 400, 32), bf(B * 81, 64), bf(B * 400, 32)
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    dy3 = bf(B * 49, 64)

    def run(grouped):
        outs = [torch.zeros(3136 * 512, device=cuda), torch.zeros(B * 3136, dtype=torch.bfloat16, device=cuda),
                torch.zeros(32 * 64 * 576, device=cuda), torch.zeros(32 * 64 * 512, device=cuda),
                torch.zeros(32 * 32 * 256, device=cuda)]
        ws1, ws2 = G.GemmWorkspace(cuda), G.GemmWorkspace(cuda)
        before = dict(G.GROUP_STATS)

        def first():
            G.gemm(y3, 3136, False, dh, 512, False, outs[0], 512, 0, 3136, 512, B, workspace=ws2, tile=4, bk=64,
                   splits=1)
            G.gemm(dh, 512, True, Wfc, 512, True, outs[1], 3136, 1, B, 3136, 512, mask=dy3m, ldm=3136, workspace=ws1,
                   tile=4, bk=64, splits=1)

        def second():
            G.gemm(dy3, 64, False, y2, 0, False, outs[2], 576, 3, 64, 576, B * 49, gb=[2, B, 64, 9, 9, 3, 3, 1],
                   tile=2, bk=64, splits=32, max_planes=32)
            G.gemm(dy2, 64, False, y1, 0, False, outs[3], 512, 3, 64, 512, B * 81, gb=[2, B, 32, 20, 20, 4, 4, 2],
                   tile=2, bk=64, splits=32, max_planes=32)
            G.gemm(dy1, 32, False, obs, 0, False, outs[4], 256, 3, 32, 256, B * 400, gb=[1, B, 4, 84, 84, 8, 8, 4],
                   gb_scale=1.0 / 255.0, tile=4, bk=256, splits=32, max_planes=32)

        for fn in (first, second):
            if grouped:
                with G.group():
                    fn()
            else:
                fn()
        torch.cuda.synchronize()
        ran = G.GROUP_STATS["grouped"] - before["grouped"]
        return outs, ran

    sep, _ = run(False)
    grp, ran = run(True)
    assert ran == 2
    for a, b in zip(sep, grp):
        assert torch.equal(a, b)


@pytest.mark.parametrize("capture", [True, False])
def test_fused_rollout_step_equals_separate_policy_and_trunk(cuda, capture, monkeypatch):
    """The rollout step fused with the next observation's row-split trunk (pong_fused_step, env state in two parity
    slots) reproduces the separate trunk + policy/env launches bit for bit: parameters, rollout tensors and env
    state over several updates with episode truncations, an odd rollout length (parity flips on graph replay) and
    graph capture or eager steps."""
    monkeypatch.setattr("actor_critic_algs_on_tensorflow_amd.ops.gemm.TUNE", False)
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    runs = []
    for fused in ("1", "0"):
        tr = ActorCriticTrainer(preset("pong_a2c", num_envs=16, n_steps=5, device="cuda:0", outdir=None, quiet=True,
                                       stdout_freq=0, save_every=0, seed=5, engine_opts=dict(fused_step=fused == "1")))
        tr.env.max_episode_steps = 7
        if capture:
            tr.capture(warmup=1)
        else:
            tr.step()
        snaps = []
        for _ in range(4):
            tr.step()
            st = tr.storage
            snaps.append([tr.flat.data.clone(), st.actions[:].clone(), st.rewards[:].clone(),
                          st.values[:].clone(), st.obs[st.T].clone(), tr.env.state.clone(), tr.env.t.clone(),
                          tr.env.tg.clone(), tr.env.ep_ret.clone(), tr.env.ep_stats.clone()])
        torch.cuda.synchronize()
        assert (getattr(tr, "_env_flips", 0) == 5) == (fused == "1")
        runs.append(snaps)
    for k, (a, b) in enumerate(zip(*runs)):
        for j, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x, y), (k, j)


@pytest.mark.parametrize("B,P", [(7, 4), (160, 64), (1024, 64), (1100, 256)])
def test_conv1_wgrad_planes_match_autograd(cuda, B, P):
    """Per-sample conv1 weight gradient (conv_wgrad.hip conv1_wgrad2_kernel, all channels per workgroup): the
    plane sum == the fp32 autograd conv weight gradient of obs/255 and dy1, every plane holds exactly its sample
    range, and two runs are bit-identical."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(B)
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    dy1 = (torch.randn(B * 400, 32, generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    planes = torch.full((max(64, P) * 32 * 256,), float("nan"), device=cuda)
    ops.conv1_wgrad(obs, dy1, planes, P, 1.0 / 255.0, None)
    got = planes[:P * 8192].view(P, 32, 256)
    # fp32 references on the CPU (a MIOpen weight-gradient solver is not a reliable reference, test_gpu_r3.py)
    go = dy1.float().cpu().view(B, 20, 20, 32).permute(0, 3, 1, 2)
    obs_c = obs.cpu()
    ref = torch.nn.grad.conv2d_weight(obs_c.float() / 255.0, (32, 4, 8, 8), go, stride=4).reshape(32, 256).to(cuda)
    tot = got.sum(0)
    assert ((tot - ref).norm() / ref.norm()).item() < 1e-4
    # plane 0 = samples [0, B // P)
    n0 = B // P
    if n0:
        r0 = torch.nn.grad.conv2d_weight(obs_c[:n0].float() / 255.0, (32, 4, 8, 8), go[:n0],
                                         stride=4).reshape(32, 256).to(cuda)
        torch.testing.assert_close(got[0], r0, rtol=1e-4, atol=1e-4)
    again = torch.zeros_like(planes)
    ops.conv1_wgrad(obs, dy1, again, P, 1.0 / 255.0, None)
    assert torch.equal(again[:P * 8192], planes[:P * 8192])
    # frames gathered through an index (PPO minibatch rows of a larger observation buffer)
    perm = torch.randperm(B, generator=g).to(cuda)
    by_idx = torch.zeros_like(planes)
    ops.conv1_wgrad(obs[perm.argsort()].contiguous(), dy1, by_idx, P, 1.0 / 255.0, perm.argsort().argsort())
    assert torch.equal(by_idx[:P * 8192], planes[:P * 8192])
