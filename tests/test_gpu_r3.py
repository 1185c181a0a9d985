"""Round-3 HIP kernels vs fp32 PyTorch references of the same op.

* ``conv_wgrad_gemm`` (conv_wgrad.hip conv_wgrad_gemm_kernel): the batched-position MFMA 32x32x16 weight gradient
  of conv2 / conv3 -- every plane == the fp32 autograd weight gradient of its sample range, planes bit-identical
  across runs, empty sample ranges written as zeros;
* the A2C head launch (``a2c_head``), the per-env lean-LDS trunk forward, PPO minibatches gathered by index.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _wgrad_ref(layer, img, dy):
    # fp32 reference on the CPU: a MIOpen weight-gradient solver once returned a wrong plane on a fresh box
    # (448 elements off by up to 0.75), so the GPU library is not a reference here
    H, C, KS, S, OH = (20, 32, 4, 2, 9) if layer == 2 else (9, 64, 3, 1, 7)
    ref = torch.nn.grad.conv2d_weight(img.float().cpu().permute(0, 3, 1, 2), (64, C, KS, KS),
                                      dy.float().cpu().permute(0, 3, 1, 2), stride=S)
    return ref.permute(0, 2, 3, 1).reshape(64, KS * KS * C).to(img.device)


@pytest.mark.parametrize("layer,B,P", [(2, 5, 3), (2, 7, 8), (2, 300, 64), (3, 9, 4), (3, 301, 64), (3, 4096, 256)])
def test_conv_wgrad_gemm_planes_match_autograd(cuda, layer, B, P):
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    H, C, KS, OH = (20, 32, 4, 9) if layer == 2 else (9, 64, 3, 7)
    n = KS * KS * C
    g = torch.Generator(device="cpu").manual_seed(B * 7 + layer)
    img = torch.rand(B, H, H, C, generator=g).to(torch.bfloat16).to(cuda)
    dy = (torch.randn(B, OH, OH, 64, generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    planes = torch.full((P * 64 * n,), float("nan"), device=cuda)
    ops.conv_wgrad_gemm(layer, img.view(B * H * H, C), dy.view(B * OH * OH, 64), planes, P)
    torch.cuda.synchronize()
    pl = planes.view(P, 64, n)
    assert torch.isfinite(pl).all()
    # every plane is the gradient of its own sample range [g B / P, (g + 1) B / P)
    for gi in sorted({0, P // 2, P - 1}):
        b0, b1 = gi * B // P, (gi + 1) * B // P
        if b1 == b0:
            assert (pl[gi] == 0).all()
            continue
        r = _wgrad_ref(layer, img[b0:b1], dy[b0:b1])
        torch.testing.assert_close(pl[gi], r, rtol=1e-4, atol=1e-4)
    tot = pl.sum(0)
    ref = _wgrad_ref(layer, img, dy)
    assert ((tot - ref).norm() / ref.norm()).item() < 1e-4
    again = torch.zeros_like(planes)
    ops.conv_wgrad_gemm(layer, img.view(B * H * H, C), dy.view(B * OH * OH, 64), again, P)
    assert torch.equal(again, planes)


def test_native_mlp_time_limit_bootstrap_matches_oracle(cuda):
    """time-limit bootstrapping on the native engines. The env kernel writes the terminal
    observation of every transition (before the auto-reset), one critic launch values them after the rollout, and
    the truncated steps' rewards carry gamma * V(terminal observation) -- the CPU oracle of
    test_semantics_cpu.py::test_bootstrap_on_timeout_cuts_episode_and_bootstraps_terminal_value, on the GPU."""
    from actor_critic_algs_on_tensorflow_amd import envs as E
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    gamma = 0.9
    env = E.make("Pendulum-v0", 3, seed=5, max_episode_steps=3, device=cuda)
    cfg = preset("basic_ac", algo="a2c", num_envs=3, n_steps=7, gamma=gamma, look_ahead=None, returns="nstep",
                 bootstrap_on_timeout=True, norm_adv=False, kl_adaptive_lr=False, anneal_regularizers=False,
                 device="cuda:0", cuda_graph=False, outdir=None, quiet=True, stdout_freq=0, save_every=0)
    tr = ActorCriticTrainer(cfg, env=env)
    assert tr.mlp is not None, "the native MLP engine must run with bootstrap_on_timeout"
    st = tr.storage
    tr.collect()
    torch.cuda.synchronize()
    twin = E.make("Pendulum-v0", 3, seed=5, max_episode_steps=3, device=cuda)
    twin.keep_final_obs = True
    twin.reset()
    with torch.no_grad():
        for t in range(7):
            prev = twin.obs.clone()
            _, r, d, info = twin.step(st.actions[t], prev_obs=prev)
            boot = gamma * tr.model.value(twin.final_obs) * info["truncated"].float()
            assert torch.equal(d, st.dones[t])
            torch.testing.assert_close(st.rewards[t], r + boot, rtol=1e-5, atol=1e-5)
    assert st.truncated[2].all() and st.dones[2].all() and st.truncated[5].all()
    # the terminal stacks are the pre-reset observations: never equal to the reset observation that follows
    assert not torch.equal(tr._final_obs[2], st.obs[3])


def test_trunk_fwd_per_env_is_batch_invariant(cuda):
    """The per-env trunk forward (cnn_fused.hip cnn_trunk_fwd_s16_kernel, mode 3: one workgroup per sample, the
    observation converted once into a bf16 LDS image) gives every sample the same bits whatever batch it is launched
    in: a 1283-sample launch == two launches of 700 and 583 samples."""
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    torch.manual_seed(4)
    B = 1283
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    W1 = (torch.randn(32, 256, device=cuda) * 0.05).to(torch.bfloat16)
    W2 = (torch.randn(64, 512, device=cuda) * 0.05).to(torch.bfloat16)
    W3 = (torch.randn(64, 576, device=cuda) * 0.05).to(torch.bfloat16)
    b1, b2, b3 = (torch.rand(n, device=cuda) * 0.1 - 0.02 for n in (32, 64, 64))

    def run(o):
        n = o.shape[0]
        y1 = torch.full((n * 400, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
        y2 = torch.full((n * 81, 64), float("nan"), dtype=torch.bfloat16, device=cuda)
        y3 = torch.full((n * 49, 64), float("nan"), dtype=torch.bfloat16, device=cuda)
        G.cnn_trunk_fwd(o, W1, b1, W2, b2, W3, b3, y1, y2, y3, mode=3)
        return y1, y2, y3

    big = run(obs)
    parts = [run(obs[i:i + 700]) for i in (0, 700)]
    torch.cuda.synchronize()
    for k in range(3):
        ref = torch.cat([p[k] for p in parts])
        assert torch.equal(big[k], ref), k


@pytest.mark.parametrize("T,N,mode,norm_adv", [(5, 32, 1, False), (5, 32, 2, True), (5, 64, 1, True),
                                               (16, 24, 2, False)])
def test_a2c_head_equals_fc_value_plus_head_bwd(cuda, T, N, mode, norm_adv):
    """a2c_head (bootstrap value from the fc partial planes + returns + loss + head backward, ONE launch of 32
    workgroups meeting at a grid barrier) == fc_value + head_bwd (round 2's two launches): V(s_T) bit-identical
    (shared plane reduction and dot-product tree); given the same V(s_T): dh, dz-derived
    statistics, targets / advantages and dbh bit-identical for B <= 256 (same per-element arithmetic and reduction
    trees; above, a thread holds two rows and the fp64 moments may round differently), dWh /
    dbfc equal up to the summation order over rows; the barrier words are back to zero after every launch."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    A, A1, B, S = 6, 7, T * N, 13
    g = torch.Generator(device="cpu").manual_seed(T * 100 + N)
    z = torch.randn(B, A1, generator=g).to(cuda)
    act = torch.randint(0, A, (B,), dtype=torch.int32, generator=g).to(cuda)
    lpo = (-torch.rand(B, generator=g) * 2).to(cuda)
    rew = torch.randn(T, N, generator=g).to(cuda)
    dones = (torch.rand(T, N, generator=g) < 0.1).to(torch.uint8).to(cuda)
    h = torch.relu(torch.randn(B, 512, generator=g)).to(torch.bfloat16).to(cuda)
    Wh = (0.05 * torch.randn(512, A1, generator=g)).to(torch.bfloat16).to(cuda)
    hpart = (0.1 * torch.randn(32, N, 512, generator=g)).to(cuda)
    bfc = (0.1 * torch.randn(512, generator=g)).to(cuda)
    bh = torch.randn(A1, generator=g).to(cuda)
    ent, kl = torch.tensor([0.01], device=cuda), torch.tensor([0.3], device=cuda)
    val0 = torch.randn(T + 1, N, generator=g).to(cuda)

    def outs():
        return dict(ret=torch.zeros(B, device=cuda), adv=torch.zeros(B, device=cuda),
                    dh=torch.zeros(B, 512, dtype=torch.bfloat16, device=cuda), gWh=torch.zeros(512 * A1, device=cuda),
                    gbh=torch.zeros(A1, device=cuda), gbfc=torch.zeros(512, device=cuda),
                    stats=torch.zeros(8, device=cuda))

    ref, new = outs(), outs()
    vref = val0.clone()
    ops.fc_value(hpart, S, bfc, Wh, bh, vref[T], None)
    bar = torch.zeros(4, dtype=torch.int32, device=cuda)
    vfirst = None
    for rep in range(3):   # repeated launches: the barrier resets itself
        vnew = val0.clone()
        vnew[T] = float("nan")
        ops.a2c_head(z, act, lpo, ent, kl, 0.5, rew, vnew, dones, 5, mode, norm_adv, 0.99, 0.95, new["ret"],
                     new["adv"], h, Wh, new["dh"], new["gWh"], new["gbh"], new["gbfc"], new["stats"], hpart, S, bfc, bh,
                     bar)
        torch.cuda.synchronize()
        assert bar.tolist() == [0, 0, 0, 0], bar
        # V(s_T): fc_value and the bootstrap phase share the plane reduction and the dot product's reduction tree
        assert torch.equal(vnew, vref)
        if vfirst is None:
            vfirst = vnew.clone()
            # the reference head_bwd, fed the same bootstrap values
            ops.head_bwd(z, act, lpo, ent, kl, 0.5, rew, vfirst, dones, 5, mode, norm_adv, 0.99, 0.95, ref["ret"],
                         ref["adv"], h, Wh, ref["dh"], ref["gWh"], ref["gbh"], ref["gbfc"], ref["stats"])
        assert torch.equal(vnew, vfirst)
        for k in ("ret", "adv", "dh", "gbh", "stats"):
            if B <= 256 or k in ("ret", "adv"):   # one row per thread in both kernels: identical fp64 moment trees
                assert torch.equal(new[k], ref[k]), (k, new[k], ref[k])
            else:
                torch.testing.assert_close(new[k].float(), ref[k].float(), rtol=1e-2, atol=1e-5)
        torch.testing.assert_close(new["gWh"], ref["gWh"], rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(new["gbfc"], ref["gbfc"], rtol=1e-5, atol=1e-7)
    # without planes the kernel reads V(s_T) from val (no barrier)
    new2 = outs()
    ops.a2c_head(z, act, lpo, ent, kl, 0.5, rew, vfirst, dones, 5, mode, norm_adv, 0.99, 0.95, new2["ret"], new2["adv"],
                 h, Wh, new2["dh"], new2["gWh"], new2["gbh"], new2["gbfc"], new2["stats"], None, 0, None, None, None)
    for k in ("ret", "adv", "dh", "gbh", "stats", "gWh", "gbfc"):
        assert torch.equal(new2[k], new[k]), k


def test_a2c_update_with_fused_bootstrap_head_matches_round2_head(cuda):
    """Native Pong A2C, 3 graph-captured updates: the a2c_head path (no fc_value launch) tracks the round-2
    fc_value + head_bwd path (same statistics; parameters equal up to the dWh / dbfc summation order)."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    res = {}
    for knob in ("1", "0"):
        cfg = preset("pong_a2c", num_envs=32, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0,
                     engine_opts=dict(a2c_head=knob == "1"))
        tr = ActorCriticTrainer(cfg)
        assert tr.engine.a2c_head == (knob == "1")
        tr.capture(warmup=1)
        p0 = tr.flat.data.clone()
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
        assert (getattr(tr, "_boot", None) is None)
        res[knob] = (tr.flat.data - p0, tr.stats_buf.clone(), tr.storage.values.clone())
    d1, s1, v1 = res["1"]
    d0, s0, v0 = res["0"]
    assert torch.allclose(s0[:8], s1[:8], rtol=1e-3, atol=1e-5), (s0[:8], s1[:8])
    assert (d0 - d1).norm() / d0.norm() < 1e-2, float((d0 - d1).norm() / d0.norm())


def test_ppo_minibatch_by_index_is_bitwise_the_copied_minibatch(cuda, monkeypatch):
    """PPO on the CNN engine with minibatches gathered BY INDEX (mb_gather index mode: the trunk forward and the
    conv1 weight gradient read obs[idx[r]] in place, no 28 KB copy per row) == the copied minibatches, bit for bit:
    parameters and statistics over 2 graph-replayed updates (16 envs x 128 steps, 2 minibatches of 1024)."""
    monkeypatch.setattr("actor_critic_algs_on_tensorflow_amd.ops.gemm.TUNE", False)
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    runs = []
    for knob in ("1", "0"):
        tr = ActorCriticTrainer(preset("breakout_ppo", num_envs=16, n_steps=128, ppo_epochs=2, ppo_minibatches=2,
                                       device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0, seed=9,
                                       engine_opts=dict(mb_index=knob == "1")))
        assert tr.engine.obs_index_ok(1024) == (knob == "1")
        tr.capture(warmup=1)
        for _ in range(2):
            tr.step()
        torch.cuda.synchronize()
        runs.append((tr.flat.data.clone(), tr.stats_buf.clone()))
    assert torch.equal(runs[0][0], runs[1][0])
    assert torch.equal(runs[0][1], runs[1][1])


def test_mb_gather_index_mode_equals_copy_mode(cuda):
    """mb_gather index mode writes the same keyed-permutation rows the copy mode copies, and the same scalars."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    n, mb, seed = 700, 300, 4242
    g = torch.Generator(device="cpu").manual_seed(5)
    obs = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    act = torch.randint(0, 6, (n,), dtype=torch.int32, generator=g).to(cuda)
    fl = [torch.randn(n, generator=g).to(cuda) for _ in range(4)]
    uc = torch.tensor([3], dtype=torch.int64, device=cuda)
    outs_c = [torch.empty(mb, 4, 84, 84, dtype=torch.uint8, device=cuda), torch.empty(mb, dtype=torch.int32,
                                                                                      device=cuda)]
    outs_c += [torch.empty(mb, device=cuda) for _ in range(4)]
    outs_i = [torch.empty(mb, dtype=torch.int32, device=cuda)] + [torch.empty(mb, device=cuda) for _ in range(4)]
    idx = torch.empty(mb, dtype=torch.int64, device=cuda)
    ops.mb_gather(obs, act, *fl, *outs_c, seed, uc, 1, 400)
    ops.mb_gather(obs, act, *fl, None, *outs_i, seed, uc, 1, 400, None, 1e-8, None, idx)
    assert torch.equal(obs[idx], outs_c[0])
    for a, b in zip(outs_c[1:], outs_i):
        assert torch.equal(a, b)


def test_a2c_head_timeout_is_raised_not_trained_on(cuda):
    """a timed-out a2c_head hand-off (sticky word 2 of its barrier block) surfaces as an error at the next
    health check (log / checkpoint / end of train) instead of silently training on a stale V(s_T)."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    tr = ActorCriticTrainer(preset("pong_a2c", num_envs=32, device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                                   save_every=0, cuda_graph=False, engine_opts=dict(a2c_head_env=False)))
    tr.step()
    torch.cuda.synchronize()
    assert tr.engine._a2c_bar is not None and not tr.engine.a2c_head_timed_out()
    tr.check_health()
    tr.engine._a2c_bar[2] = 1
    with pytest.raises(RuntimeError, match="a2c_head"):
        tr.check_health()
