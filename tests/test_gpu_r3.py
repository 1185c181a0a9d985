"""Round-3 HIP kernels vs fp32 PyTorch references of the same op.

* ``conv_wgrad_gemm`` (conv_wgrad.hip conv_wgrad_gemm_kernel): the batched-position MFMA 32x32x16 weight gradient
  of conv2 / conv3 -- every plane == the fp32 autograd weight gradient of its sample range, planes bit-identical
  across runs, empty sample ranges written as zeros;
* ``grad_finalize_opt`` (optim.hip grad_finalize_opt_kernel): the finaliser + RMSprop / Adam update in one launch
  == the finaliser launch followed by the optimiser launch, and the gradient slab is left zero.
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


@pytest.mark.parametrize("adam", [False, True])
def test_grad_finalize_opt_equals_two_launches(cuda, adam):
    """One launch of finaliser + optimiser (grid barrier between the phases) == grad_finalize then the optimiser
    step reading the finalised slab: same parameters / moments / bf16 shadow (RMSprop bitwise), and the slab is
    zero."""
    from actor_critic_algs_on_tensorflow_amd import _native
    from actor_critic_algs_on_tensorflow_amd.ops.optim import (FlatParams, FusedAdam, FusedRMSprop,
                                                               finalize_jobs)
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(3 + adam)
    shapes = [(4099,), (64, 513), (33,), (257, 129)]
    runs = []
    for fused in (False, True):
        torch.manual_seed(0)
        params = [torch.nn.Parameter(torch.randn(s, generator=torch.Generator().manual_seed(i)))
                  for i, s in enumerate(shapes)]
        flat = FlatParams({"shared": params}, cuda)
        shadow = torch.zeros(flat.numel, dtype=torch.bfloat16, device=cuda)
        cls = FusedAdam if adam else FusedRMSprop
        opt = cls(flat, "shared", 1e-3, max_grad_norm=0.5, bf16_shadow=shadow)
        opt.zero_grad_after = True
        # plane sources for params 1 and 3 (7 planes each); params 0 and 2 are final in the slab (read-only jobs)
        gen = torch.Generator(device="cpu").manual_seed(11)
        planes = {}
        for i in (1, 3):
            planes[i] = torch.randn(7 * params[i].numel(), generator=gen).to(cuda)
        for step in range(3):
            for i in (0, 2):
                off = flat.offsets[i]
                flat.grad[off:off + params[i].numel()] = torch.randn(params[i].numel(), generator=gen).to(cuda)
            segs = []
            for i, p in enumerate(params):
                off = flat.offsets[i]
                dst = flat.grad[off:off + p.numel()].data_ptr()
                if i in planes:
                    segs.append((dst, planes[i].data_ptr(), p.numel(), p.numel(), 7))
                else:
                    segs.append((dst, 0, p.numel(), 0, 0))
            words, maxn = finalize_jobs(segs, cuda, return_max=True)
            parts = torch.zeros(256, device=cuda)
            if fused:
                assert opt.step_finalize(words, maxn, parts)
            else:
                ops.grad_finalize(words, parts)
                opt.ext_parts = parts
                opt.step()
            torch.cuda.synchronize()
        st = {"p": flat.data.clone(), "v": opt.v.clone(), "shadow": shadow.clone(), "grad": flat.grad.clone()}
        if adam:
            st.update(m=opt.m.clone(), t=opt.t.clone())
        if fused:
            assert int(opt._fin_state[2]) == 0, "grid barrier timed out"
        runs.append(st)
    a, b = runs
    for k in a:
        if k == "grad":
            continue
        if adam and k in ("p", "m", "v", "shadow"):
            # the Adam update compiles with different fp contractions in the two kernels (fma placement in the
            # moment / step expressions): the same maths to the last ulp or two; RMSprop comes out bitwise
            torch.testing.assert_close(a[k].float(), b[k].float(), rtol=1e-6, atol=1e-7)
        else:
            assert torch.equal(a[k], b[k]), k
    assert (b["grad"] == 0).all() and (a["grad"] == 0).all()


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K,out_mode,epi", [
    (4096, 512, 3136, 1, "bias_relu"),     # PPO fc forward
    (4096, 3136, 512, 1, "mask"),          # dy3 = dh Wfc^T * (y3 > 0)
    (3136, 512, 4096, 0, None),            # dWfc (fp32 store)
    (1000, 136, 1024, 3, None),            # partial tiles, split-K planes
])
def test_gemm_mfma32_matches_fp32_reference(cuda, a_k, b_k, M, N, K, out_mode, epi):
    """The 32x32x16-MFMA GEMM (gemm_mfma32.hip) == the fp32 oracle of the same product (bf16 operands in every
    storage orientation, bias / relu / mask epilogues, fp32 / bf16 stores, split-K partial planes)."""
    from actor_critic_algs_on_tensorflow_amd import _native
    from actor_critic_algs_on_tensorflow_amd.ops.gemm import gemm_ref
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + 2 * a_k + b_k)
    lda = K if a_k else M
    ldb = K if b_k else N
    A = (torch.randn((M if a_k else K) * lda, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    B = (torch.randn((N if b_k else K) * ldb, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda) if epi == "bias_relu" else None
    mask = torch.randn(M * N, generator=g).to(torch.bfloat16).to(cuda) if epi == "mask" else None
    splits = 4 if out_mode == 3 else 1
    dt = torch.bfloat16 if out_mode == 1 else torch.float32
    C = torch.full((splits * M * N,), float("nan"), dtype=dt, device=cuda)
    ok = ops.gemm_mfma32(A, lda, a_k, B, ldb, b_k, C, N, out_mode, M, N, K, 1.0, bias, epi == "bias_relu", mask,
                         N if mask is not None else 0, splits)
    assert ok
    torch.cuda.synchronize()
    ref = gemm_ref(A, lda, a_k, B, ldb, b_k, M, N, K, 1.0, bias, epi == "bias_relu", mask, N if mask is not None else 0)
    got = C.view(splits, M, N).float().sum(0) if out_mode == 3 else C.view(M, N).float()
    tol = 2e-2 if out_mode == 1 else 1e-3
    err = ((got - ref).norm() / ref.norm()).item()
    assert err < tol, err
    assert torch.isfinite(got).all()


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


def test_trunk_fwd_persistent_equals_per_env_kernel(cuda):
    """The persistent trunk forward (cnn_fused.hip cnn_trunk_fwd_persist_kernel: one workgroup per CU walking
    samples, W2 / W3 fragments resident in registers, the next observation copied global -> LDS by LDS-DMA as uint8)
    is BITWISE equal to the per-env kernel (taken for batches below ACA_TRUNK_FWD_PERSIST_MIN_B = 1024): same bf16
    integer pixels, same MFMA order. 1283 samples: the walk ends unevenly over the 256 workgroups."""
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
        G.cnn_trunk_fwd(o, W1, b1, W2, b2, W3, b3, y1, y2, y3, mode=0)
        return y1, y2, y3

    big = run(obs)                                   # persistent walk (B >= 1024)
    parts = [run(obs[i:i + 700]) for i in (0, 700)]  # per-env kernel (B < 1024)
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


def test_a2c_update_with_fused_bootstrap_head_matches_round2_head(cuda, monkeypatch):
    """Native Pong A2C, 3 graph-captured updates: the a2c_head path (no fc_value launch) tracks the round-2
    fc_value + head_bwd path (same statistics; parameters equal up to the dWh / dbfc summation order)."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    res = {}
    for knob in ("1", "0"):
        monkeypatch.setenv("ACA_A2C_HEAD", knob)
        cfg = preset("pong_a2c", num_envs=32, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0)
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


@pytest.mark.parametrize("N", [16, 32])
def test_fc_fold_planes_match_fp32_product(cuda, N):
    """fc fold (cnn_fused.hip FcFold): the row-split trunk launch also computes the fc product as 7 partial planes
    (plane r = conv3 row r of every env x the matching 448 rows of Wfc, 16 helper workgroups per row meeting the row's
    other workgroups at a counter). y1 / y2 / y3 stay bit-identical to the unfolded launch, every plane matches the
    fp32 product of the same bf16 operands, repeated launches give identical planes (no races), and the counter words
    are back to zero with no helper timeout."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(N)
    obs = torch.randint(0, 256, (N, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    W1 = (0.05 * torch.randn(32, 256, generator=g)).to(torch.bfloat16).to(cuda)
    W2 = (0.05 * torch.randn(64, 512, generator=g)).to(torch.bfloat16).to(cuda)
    W3 = (0.05 * torch.randn(64, 576, generator=g)).to(torch.bfloat16).to(cuda)
    b1, b2, b3 = [(0.1 * torch.randn(n, generator=g)).to(cuda) for n in (32, 64, 64)]
    Wfc = (0.02 * torch.randn(3136, 512, generator=g)).to(torch.bfloat16).to(cuda)

    def acts():
        return (torch.zeros(N * 400 * 32, dtype=torch.bfloat16, device=cuda),
                torch.zeros(N * 81 * 64, dtype=torch.bfloat16, device=cuda),
                torch.zeros(N * 49 * 64, dtype=torch.bfloat16, device=cuda))

    ref = acts()
    ops.cnn_trunk_fwd(obs, W1, b1, W2, b2, W3, b3, *ref, 1.0 / 255.0, None, None, 2, None)
    cnt = torch.zeros(16, dtype=torch.int32, device=cuda)
    planes = torch.full((32 * N * 512,), float("nan"), device=cuda)
    got = acts()
    first = None
    for rep in range(5):
        ops.cnn_trunk_fwd(obs, W1, b1, W2, b2, W3, b3, *got, 1.0 / 255.0, None, None, 2, None, Wfc, planes, cnt)
        torch.cuda.synchronize()
        assert cnt.tolist() == [0] * 16, cnt
        for x, y in zip(got, ref):
            assert torch.equal(x, y)
        p = planes[:7 * N * 512].view(7, N, 512).clone()
        if first is None:
            first = p
        assert torch.equal(p, first), rep
    y3 = ref[2].float().view(N, 7, 448)
    for r in range(7):
        want = y3[:, r] @ Wfc[r * 448:(r + 1) * 448].float()
        torch.testing.assert_close(first[r], want, rtol=1e-4, atol=1e-4)
    h = first.sum(0)
    torch.testing.assert_close(h, ref[2].float().view(N, 3136) @ Wfc.float(), rtol=1e-4, atol=1e-3)


def test_a2c_with_fc_fold_tracks_gemm_fc(cuda, monkeypatch):
    """Native Pong A2C (32 envs, graph-captured): the folded fc product (no fc GEMM launches) tracks the split-K GEMM
    path over 3 updates (same loss statistics within rounding; the plane sums differ in order only), and the helpers
    never timed out."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    res = {}
    for knob in ("1", "0"):
        monkeypatch.setenv("ACA_FC_FOLD", knob)
        cfg = preset("pong_a2c", num_envs=32, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0)
        tr = ActorCriticTrainer(cfg)
        assert tr.engine.fold_ok(32) == (knob == "1")
        tr.capture(warmup=1)
        p0 = tr.flat.data.clone()
        tr.step()
        torch.cuda.synchronize()
        assert not tr.engine.fold_timed_out()
        res[knob] = (tr.flat.data - p0, tr.stats_buf.clone())
    (d1, s1), (d0, s0) = res["1"], res["0"]
    # losses / entropy / ratio agree to rounding; EV-before (stats[7]) of a random-init critic is ~1e-3 noise
    assert torch.allclose(s0[:7], s1[:7], rtol=1e-2, atol=1e-3), (s0[:8], s1[:8])
    assert (d0 - d1).norm() / d0.norm() < 5e-2, float((d0 - d1).norm() / d0.norm())


@pytest.mark.parametrize("name,kw", [("mujoco_ppo_dp8", dict(num_envs=16, n_steps=64, ppo_epochs=2, ppo_minibatches=4)),
                                     ("cartpole_cpu", dict(num_envs=64, n_steps=5, device="cuda:0", cuda_graph=True))])
def test_mlp_wgrad_with_fused_adam_is_bitwise_the_two_launch_update(cuda, name, kw, monkeypatch):
    """MLP engine: Adam folded into the weight-gradient launch (mlp_wgrad_adam_kernel: grid barrier on the sum-of-
    squares slots, each tile workgroup updating its own tile + transposed shadow) == weight-gradient launch +
    opt_multi: Adam step counts and the untouched gradient slab exactly, parameters / moments / global norms / the
    transposed shadows to float rounding (same operation order; the compiler's fp contraction differs between the two
    kernels), over several graph-replayed updates (PPO with the Gaussian head and log-std, A2C with the categorical
    head). Each path alone is bitwise deterministic (test_ppo_graph_replay_bitwise_equals_eager)."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    runs = []
    for knob in ("1", "0"):
        monkeypatch.setenv("ACA_MLP_FUSED_OPT", knob)
        base = dict(outdir=None, quiet=True, stdout_freq=0, save_every=0, seed=4)
        base.update(kw)
        tr = ActorCriticTrainer(preset(name, **base))
        assert tr.mlp is not None
        tr.capture(warmup=1)
        assert (tr._mlp_fused_opt() is not None) == (knob == "1")
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
        if knob == "1":
            assert not tr.mlp.fused_opt_timed_out()
        o = tr.opts
        runs.append([tr.flat.data.clone(), tr.flat.grad.clone()] +
                    [x.clone() for g in ("actor", "critic") for x in (o[g].m, o[g].v, o[g].t, o[g].gnorm)] +
                    [tr.mlp.wt[id(lay)].clone() for tw in tr.mlp.towers for lay in tw])
    exact = {1, 4, 8}   # gradient slab, actor / critic step counts
    for j, (x, y) in enumerate(zip(*runs)):
        if j in exact:
            assert torch.equal(x, y), j
        else:
            torch.testing.assert_close(x, y, rtol=2e-4, atol=1e-6, msg=lambda m: f"item {j}: {m}")


def test_ppo_minibatch_by_index_is_bitwise_the_copied_minibatch(cuda, monkeypatch):
    """PPO on the CNN engine with minibatches gathered BY INDEX (mb_gather index mode: the trunk forward and the
    conv1 weight gradient read obs[idx[r]] in place, no 28 KB copy per row) == the copied minibatches, bit for bit:
    parameters and statistics over 2 graph-replayed updates (16 envs x 128 steps, 2 minibatches of 1024)."""
    monkeypatch.setattr("actor_critic_algs_on_tensorflow_amd.ops.gemm.TUNE", False)
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    runs = []
    for knob in ("1", "0"):
        monkeypatch.setenv("ACA_MB_INDEX", knob)
        tr = ActorCriticTrainer(preset("breakout_ppo", num_envs=16, n_steps=128, ppo_epochs=2, ppo_minibatches=2,
                                       device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0, seed=9))
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


def test_trunk_fwd_8wave_equals_4wave_kernel(cuda):
    """The per-env lean-LDS trunk forward's opt-in 8-wave form (batches up to ACA_TRUNK_FWD_WIDE_MAX_B) and its
    4-wave form share the per-tile MFMA order: the first 200 samples of a 300-sample launch equal a 200-sample launch
    bit for bit (whichever form the process's knob selects for each; the GPU job sets 256 to cover both)."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(11)
    obs = torch.randint(0, 256, (300, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    W1 = (0.05 * torch.randn(32, 256, generator=g)).to(torch.bfloat16).to(cuda)
    W2 = (0.05 * torch.randn(64, 512, generator=g)).to(torch.bfloat16).to(cuda)
    W3 = (0.05 * torch.randn(64, 576, generator=g)).to(torch.bfloat16).to(cuda)
    b1, b2, b3 = [(0.1 * torch.randn(n, generator=g)).to(cuda) for n in (32, 64, 64)]

    def run(B):
        y = (torch.zeros(B * 400 * 32, dtype=torch.bfloat16, device=cuda),
             torch.zeros(B * 81 * 64, dtype=torch.bfloat16, device=cuda),
             torch.zeros(B * 49 * 64, dtype=torch.bfloat16, device=cuda))
        ops.cnn_trunk_fwd(obs[:B], W1, b1, W2, b2, W3, b3, *y, 1.0 / 255.0, None, None, 0, None)
        torch.cuda.synchronize()
        return y

    wide, narrow = run(200), run(300)
    for a, b in zip(wide, narrow):
        assert torch.equal(a, b[:a.numel()])


@pytest.mark.parametrize("B,A1", [(1, 2), (33, 5), (4096, 5), (1000, 7), (64, 8)])
def test_head_fwd_matches_fp32(cuda, B, A1):
    """heads.hip head_fwd (large-batch policy/value head, 8 lanes per row, Wh staged in LDS) == the fp32 product of
    the same bf16 operands, and repeat launches are bit-identical."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(B + A1)
    h = torch.relu(torch.randn(B, 512, generator=g)).to(torch.bfloat16).to(cuda)
    Wh = (0.05 * torch.randn(512, A1, generator=g)).to(torch.bfloat16).to(cuda)
    bh = torch.randn(A1, generator=g).to(cuda)
    z = torch.full((B, A1), float("nan"), device=cuda)
    ops.head_fwd(h, Wh, bh, z)
    z2 = torch.empty_like(z)
    ops.head_fwd(h, Wh, bh, z2)
    torch.cuda.synchronize()
    ref = h.double() @ Wh.double() + bh.double()
    torch.testing.assert_close(z.double(), ref, rtol=1e-5, atol=1e-4)
    assert torch.equal(z, z2)


def test_ppo_learner_forward_head_fwd_equals_gemm_path(cuda, monkeypatch):
    """The CNN engine's large-batch head (head_fwd) and the GEMM path give the same logits / values to fp32
    rounding on a PPO-sized batch."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    tr = ActorCriticTrainer(preset("breakout_ppo", num_envs=16, n_steps=64, device="cuda:0", outdir=None, quiet=True,
                                   stdout_freq=0, save_every=0, cuda_graph=False))
    eng = tr.engine
    obs = torch.randint(0, 256, (1024, 4, 84, 84), dtype=torch.uint8, device=cuda)
    b = eng.bufs(1024)
    eng.head_fwd_min_b = 512   # opt-in (ACA_HEAD_FWD_MIN_B)
    assert eng.head_fwd_ok(1024)
    z_new = eng.forward(obs, b).clone()
    eng.head_fwd_min_b = 1 << 62
    assert not eng.head_fwd_ok(1024)
    z_gemm = eng.forward(obs, b).clone()
    torch.cuda.synchronize()
    torch.testing.assert_close(z_new, z_gemm, rtol=1e-4, atol=1e-4)
