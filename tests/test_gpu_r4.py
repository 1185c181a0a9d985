"""Round-4 HIP kernels vs fp32 PyTorch references of the same op.

* ``ppo_head`` (ppo_head.hip): the large-batch learner head in one launch -- z = h Wh + bh, the PPO-clip / A2C
  actor loss + KL proxy + entropy + (clipped) value loss, dz, dh = (h > 0) dz Wh^T and per-workgroup partial planes
  of dWh / dbh / dbfc -- against autograd of the same loss in fp32 (float64 for the statistics), and the PPO update
  through it against the generic loss + GEMM head path.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ppo_head_ref(h, Wh, bh, act, lpo, adv, ret, v_old, c_ent, beta, vf, clip, v_clip):
    hf = h.float().cpu().double()
    W = Wh.float().cpu().double().requires_grad_(False)
    z = (hf @ W + bh.cpu().double()).requires_grad_(True)
    A = z.shape[1] - 1
    logp = torch.log_softmax(z[:, :A], 1)
    lpa = logp.gather(1, act.long().cpu().view(-1, 1)).view(-1)
    H = -(logp.exp() * logp).sum(1)
    adv_, lpo_, ret_ = adv.cpu().double(), lpo.cpu().double(), ret.cpu().double()
    if clip > 0:
        ratio = torch.exp(lpa - lpo_)
        pg = -torch.min(ratio * adv_, torch.clamp(ratio, 1 - clip, 1 + clip) * adv_)
        cf = ((ratio - 1).abs() > clip).double()
    else:
        ratio = torch.ones_like(lpa)
        pg = -adv_ * lpa
        cf = torch.zeros_like(lpa)
    kl = (lpo_ - lpa) ** 2
    v = z[:, A]
    vl = (v - ret_) ** 2
    if v_clip > 0:
        vo = v_old.cpu().double()
        vc = vo + torch.clamp(v - vo, -v_clip, v_clip)
        vl = torch.max(vl, (vc - ret_) ** 2)
    loss = pg.mean() + beta * kl.mean() - c_ent * H.mean() + vf * vl.mean()
    loss.backward()
    dz = z.grad
    dh = (dz @ W.t()) * (hf > 0)
    stats = [pg.mean(), kl.mean(), H.mean(), vl.mean(), cf.mean(), pg.mean() + beta * kl.mean() - c_ent * H.mean(),
             ratio.mean()]
    return dict(z=z.detach(), dh=dh, dWh=hf.t() @ dz, dbh=dz.sum(0), dbfc=dh.sum(0),
                stats=torch.stack([s.detach() for s in stats]))


@pytest.mark.parametrize("B,A1,clip,v_clip", [(4096, 5, 0.1, 0.0), (37, 7, 0.2, 0.3), (1000, 3, 0.0, 0.0),
                                              (4096, 8, 0.1, 0.2)])
def test_ppo_head_matches_fp32_autograd(cuda, B, A1, clip, v_clip):
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(B + A1)
    h = torch.relu(torch.randn(B, 512, generator=g)).to(torch.bfloat16).to(cuda)
    Wh = (0.05 * torch.randn(512, A1, generator=g)).to(torch.bfloat16).to(cuda)
    bh = (0.1 * torch.randn(A1, generator=g)).to(cuda)
    act = torch.randint(0, A1 - 1, (B,), dtype=torch.int32, generator=g).to(cuda)
    lpo = (-torch.rand(B, generator=g) * 2).to(cuda)
    adv = torch.randn(B, generator=g).to(cuda)
    ret = torch.randn(B, generator=g).to(cuda)
    v_old = torch.randn(B, generator=g).to(cuda)
    ent, kl = torch.tensor([0.01], device=cuda), torch.tensor([0.3], device=cuda)
    P = int(ops.ppo_head_planes(B))
    assert P == (B + 15) // 16
    out = dict(dh=torch.full((B, 512), float("nan"), dtype=torch.bfloat16, device=cuda),
               z=torch.full((B, A1), float("nan"), device=cuda), pWh=torch.full((P * 512 * A1,), float("nan"), device=cuda),
               pbh=torch.full((P * A1,), float("nan"), device=cuda), pbfc=torch.full((P * 512,), float("nan"), device=cuda),
               st=torch.zeros(P * 6, dtype=torch.float64, device=cuda), stats=torch.zeros(8, device=cuda))
    ticket = torch.zeros(1, dtype=torch.int32, device=cuda)
    runs = []
    for _ in range(2):
        ops.ppo_head(h, Wh, bh, act, lpo, adv, ret, v_old if v_clip else None, ent, kl, 0.5, clip, v_clip,
                     out["dh"], out["z"], out["pWh"], out["pbh"], out["pbfc"], out["st"], ticket, out["stats"])
        torch.cuda.synchronize()
        assert int(ticket) == 0
        runs.append({k: v.clone() for k, v in out.items()})
    for k in runs[0]:   # deterministic: fixed-order sums everywhere
        assert torch.equal(runs[0][k], runs[1][k]), k
    ref = _ppo_head_ref(h, Wh, bh, act, lpo, adv, ret, v_old, 0.01, 0.3, 0.5, clip, v_clip)
    torch.testing.assert_close(out["z"].cpu().double(), ref["z"], rtol=1e-5, atol=1e-5)
    # dh is stored in bf16
    torch.testing.assert_close(out["dh"].float().cpu().double(), ref["dh"], rtol=1e-2, atol=1e-7)
    sums = dict(dWh=out["pWh"].view(P, -1).sum(0), dbh=out["pbh"].view(P, -1).sum(0),
                dbfc=out["pbfc"].view(P, -1).sum(0))
    for k, v in sums.items():
        r = ref[k].reshape(-1)
        assert ((v.cpu().double() - r).norm() / r.norm()).item() < 1e-5, k
    torch.testing.assert_close(out["stats"][:7].cpu().double(), ref["stats"], rtol=1e-5, atol=1e-6)
    # without the ticket (the engine's default): the statistics records are left for the gradient finaliser's duty,
    # which reduces them along with the head's planes -- the same statistics
    from actor_critic_algs_on_tensorflow_amd.ops.optim import finalize_jobs
    st2 = torch.zeros(8, device=cuda)
    ops.ppo_head(h, Wh, bh, act, lpo, adv, ret, v_old if v_clip else None, ent, kl, 0.5, clip, v_clip,
                 out["dh"], out["z"], out["pWh"], out["pbh"], out["pbfc"], out["st"], None, st2)
    dbh = torch.zeros(A1, device=cuda)
    jobs = finalize_jobs([(dbh.data_ptr(), out["pbh"].data_ptr(), A1, A1, P)], cuda)
    parts = torch.zeros(256, device=cuda)
    ops.grad_finalize(jobs, parts, out["st"].view(P, 6), B, ent, kl, st2)
    torch.cuda.synchronize()
    assert torch.equal(st2[7], torch.zeros((), device=cuda))
    torch.testing.assert_close(st2[:7], out["stats"][:7], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(dbh.cpu().double(), ref["dbh"], rtol=1e-4, atol=1e-6)


def test_ppo_update_through_ppo_head_tracks_generic_head(cuda, monkeypatch):
    """Breakout-shape PPO (16 envs x 128 steps, 2 epochs x 2 minibatches of 1024, graph-captured): the ppo_head path
    (fp32 dz, head gradient planes) tracks the generic loss + GEMM head path (bf16 dz) over 2 updates."""
    monkeypatch.setattr("actor_critic_algs_on_tensorflow_amd.ops.gemm.TUNE", False)
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    runs = []
    for on in (True, False):
        tr = ActorCriticTrainer(preset("breakout_ppo", num_envs=16, n_steps=128, ppo_epochs=2, ppo_minibatches=2,
                                       device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0, seed=9,
                                       engine_opts=dict(ppo_head=on)))
        assert tr.engine.ppo_head_ok(1024) == on
        p0 = tr.flat.data.clone()
        tr.capture(warmup=1)
        for _ in range(2):
            tr.step()
        torch.cuda.synchronize()
        runs.append((tr.flat.data - p0, tr.stats_buf.clone()))
    (d1, s1), (d0, s0) = runs
    assert torch.isfinite(d1).all()
    assert torch.allclose(s0[:7], s1[:7], rtol=2e-2, atol=1e-4), (s0[:7], s1[:7])
    assert ((d1 - d0).norm() / d0.norm()).item() < 5e-2


@pytest.mark.parametrize("preset_name,capture", [("pong_a2c", True), ("breakout_ppo", False), ("breakout_ppo", True)])
def test_fused_env_step_equals_separate_trunk_and_policy(cuda, preset_name, capture, monkeypatch):
    """Large banks (72 envs > the row-split limit): the per-env fused rollout step (pong_fused_env_step: policy/env
    step t + render + shift + the trunk of obs t+1 in one launch) reproduces the separate per-env trunk + policy/env
    launches bit for bit -- parameters, rollout tensors and env state over several updates with episode
    truncations, A2C (learner reuses the rollout activations) and PPO, graph-captured or eager -- in both its forms:
    two workgroups per env (the conv rows split in halves, the env state alternating parity slots; T = 5 leaves the
    parity flipped at every update) and one."""
    monkeypatch.setattr("actor_critic_algs_on_tensorflow_amd.ops.gemm.TUNE", False)
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    runs = []
    for fused, split in ((True, True), (True, False), (False, False)):
        kw = dict(n_steps=5) if preset_name == "pong_a2c" else dict(n_steps=8, ppo_epochs=1, ppo_minibatches=2)
        tr = ActorCriticTrainer(preset(preset_name, num_envs=72, device="cuda:0", outdir=None, quiet=True,
                                       stdout_freq=0, save_every=0, seed=5,
                                       engine_opts=dict(fused_step=fused, fused_env_split=split), **kw))
        assert tr.engine.fused_env_step_ok(72) == fused
        tr.env.max_episode_steps = 7
        if capture:
            tr.capture(warmup=1)
        else:
            tr.step()
        snaps = []
        for _ in range(3):
            tr.step()
            st = tr.storage
            snaps.append([tr.flat.data.clone(), st.actions[:].clone(), st.rewards[:].clone(), st.dones[:].clone(),
                          st.values[:].clone(), st.logp[:].clone(), st.obs[st.T].clone(), tr.env.state.clone(),
                          tr.env.t.clone(), tr.env.tg.clone(), tr.env.ep_ret.clone(), tr.env.ep_stats.clone()])
        torch.cuda.synchronize()
        runs.append(snaps)
    for other in runs[1:]:
        for k, (a, b) in enumerate(zip(runs[0], other)):
            for j, (x, y) in enumerate(zip(a, b)):
                assert torch.equal(x, y), (k, j)


@pytest.mark.parametrize("a_k,b_k,M,N,K,out_mode,epi,splits", [
    (True, False, 4096, 512, 3136, 1, "bias_relu", 1),     # PPO fc forward: h = relu(y3 Wfc + bfc)
    (True, False, 4096, 512, 3072, 1, "bias_relu", 2),     # ... split-K slabs (3072 = 48 k-steps)
    (False, False, 3136, 512, 4096, 0, None, 2),           # dWfc = y3^T dh (fp32, partial M tile)
    (True, True, 4096, 3136, 512, 1, "mask", 1),           # dy3 = (dh Wfc^T) * (y3 > 0) (partial N tile)
    (False, True, 200, 136, 256, 0, None, 4),              # both partial tiles, 4 splits
])
def test_gemm_big_matches_fp32_reference(cuda, a_k, b_k, M, N, K, out_mode, epi, splits):
    """gemm_big.hip (128 x 128 tiles of the 32x32x16 MFMA, LDS-DMA 3-stage ring, swizzled images) == the fp32
    product of the same bf16 operands in every storage orientation; split-K slabs reduced by the last arriver; a
    second launch is bitwise identical (fixed split order)."""
    from actor_critic_algs_on_tensorflow_amd import _native
    from actor_critic_algs_on_tensorflow_amd.ops.gemm import gemm_ref
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + 2 * a_k + b_k + splits)
    lda = K if a_k else M
    ldb = K if b_k else N
    A = (torch.randn((M if a_k else K) * lda, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    B = (torch.randn((N if b_k else K) * ldb, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda) if epi == "bias_relu" else None
    mask = torch.randn(M * N, generator=g).to(torch.bfloat16).to(cuda) if epi == "mask" else None
    dt = torch.bfloat16 if out_mode == 1 else torch.float32
    ws = torch.zeros(max(1, int(ops.gemm_big_ws(M, N, splits))), device=cuda)
    tickets = torch.zeros(((M + 127) // 128) * ((N + 127) // 128), dtype=torch.int32, device=cuda)
    outs = []
    for _ in range(2):
        C = torch.full((M * N,), float("nan"), dtype=dt, device=cuda)
        ops.gemm_big(A, lda, a_k, B, ldb, b_k, C, N, out_mode, M, N, K, 1.0, bias, epi == "bias_relu", mask,
                     N if mask is not None else 0, splits, ws, tickets)
        torch.cuda.synchronize()
        outs.append(C)
    assert torch.equal(outs[0], outs[1])
    assert (tickets == 0).all()
    ref = gemm_ref(A, lda, a_k, B, ldb, b_k, M, N, K, 1.0, bias, epi == "bias_relu", mask, N if mask is not None else 0)
    got = outs[0].view(M, N).float()
    assert torch.isfinite(got).all()
    err = ((got - ref).norm() / ref.norm()).item()
    assert err < (1e-2 if out_mode == 1 else 1e-5), err


@pytest.mark.parametrize("a_k,b_k,M,N,K", [(True, False, 4096, 512, 3136), (False, False, 3136, 512, 4096),
                                           (False, True, 200, 136, 256)])
def test_gemm_big_partial_planes_sum_to_the_slab_reduction(cuda, a_k, b_k, M, N, K):
    """out_mode 3: each split stores its fp32 tile into its own plane (no slab, no ticket); summing the planes in
    split order reproduces the last-arriver slab reduction bit for bit."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(M + K)
    lda, ldb = (K if a_k else M), (K if b_k else N)
    A = (torch.randn((M if a_k else K) * lda, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    B = (torch.randn((N if b_k else K) * ldb, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    ws = torch.zeros(int(ops.gemm_big_ws(M, N, 2)), device=cuda)
    tickets = torch.zeros(((M + 127) // 128) * ((N + 127) // 128), dtype=torch.int32, device=cuda)
    C = torch.full((M * N,), float("nan"), device=cuda)
    ops.gemm_big(A, lda, a_k, B, ldb, b_k, C, N, 0, M, N, K, 1.0, None, False, None, 0, 2, ws, tickets)
    P = torch.full((2 * M * N,), float("nan"), device=cuda)
    ops.gemm_big(A, lda, a_k, B, ldb, b_k, P, N, 3, M, N, K, 1.0, None, False, None, 0, 2, None, None)
    torch.cuda.synchronize()
    p = P.view(2, M * N)
    assert torch.isfinite(p).all()
    assert torch.equal(p[0] + p[1], C)


def test_ppo_head_from_fc_planes_equals_stored_h(cuda):
    """The learner head fed the fc product's two split-K planes (sum + bias + ReLU + bf16 inside the head launch)
    == the head fed h stored by the fc product's own epilogue: every output bitwise."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    B, A1 = 4096, 5
    g = torch.Generator(device="cpu").manual_seed(11)
    y3 = torch.relu(torch.randn(B * 3136, generator=g)).to(torch.bfloat16).to(cuda)
    Wfc = (0.02 * torch.randn(3136 * 512, generator=g)).to(torch.bfloat16).to(cuda)
    bfc = (0.1 * torch.randn(512, generator=g)).to(cuda)
    Wh = (0.05 * torch.randn(512, A1, generator=g)).to(torch.bfloat16).to(cuda)
    bh = (0.1 * torch.randn(A1, generator=g)).to(cuda)
    act = torch.randint(0, A1 - 1, (B,), dtype=torch.int32, generator=g).to(cuda)
    lpo = (-torch.rand(B, generator=g) * 2).to(cuda)
    adv, ret = torch.randn(B, generator=g).to(cuda), torch.randn(B, generator=g).to(cuda)
    ent, kl = torch.tensor([0.01], device=cuda), torch.tensor([0.3], device=cuda)
    h = torch.empty(B, 512, dtype=torch.bfloat16, device=cuda)
    ws = torch.zeros(int(ops.gemm_big_ws(B, 512, 2)), device=cuda)
    tickets = torch.zeros((B // 128) * 4, dtype=torch.int32, device=cuda)
    ops.gemm_big(y3, 3136, True, Wfc, 512, False, h, 512, 1, B, 512, 3136, 1.0, bfc, True, None, 0, 2, ws, tickets)
    hp = torch.empty(2 * B * 512, device=cuda)
    ops.gemm_big(y3, 3136, True, Wfc, 512, False, hp, 512, 3, B, 512, 3136, 1.0, None, False, None, 0, 2, None, None)
    P = int(ops.ppo_head_planes(B))
    outs = []
    for planes in (False, True):
        o = dict(dh=torch.empty(B, 512, dtype=torch.bfloat16, device=cuda), z=torch.empty(B, A1, device=cuda),
                 pWh=torch.empty(P * 512 * A1, device=cuda), pbh=torch.empty(P * A1, device=cuda),
                 pbfc=torch.empty(P * 512, device=cuda), st=torch.zeros(P * 6, dtype=torch.float64, device=cuda),
                 stats=torch.zeros(8, device=cuda))
        ticket = torch.zeros(1, dtype=torch.int32, device=cuda)
        hin = torch.full_like(h, float("nan")) if planes else h   # the planes path must not read h
        ops.ppo_head(hin, Wh, bh, act, lpo, adv, ret, None, ent, kl, 0.5, 0.1, 0.0, o["dh"], o["z"], o["pWh"],
                     o["pbh"], o["pbfc"], o["st"], ticket, o["stats"], hp if planes else None, 2 if planes else 0,
                     bfc if planes else None)
        torch.cuda.synchronize()
        outs.append(o)
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k


def test_sumsq_multi_equals_separate_launches(cuda):
    """One launch for several groups' sums of squares (data-parallel multi-group optimiser step): per group the same
    total as one sumsq launch (its own workgroup split, 2 float4 per thread: the partials are not the same set), unused
    slots zero, bitwise reproducible."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(4)
    xs = [torch.randn(n, generator=g).to(cuda) for n in (37, 25347, 50561, 4 * 1024 * 1024 + 3)]
    P = int(ops.sumsq_parts()) if hasattr(ops, "sumsq_parts") else 256
    sep = [torch.full((P,), float("nan"), device=cuda) for _ in xs]
    mul = [torch.full((P,), float("nan"), device=cuda) for _ in xs]
    for x, p in zip(xs, sep):
        ops.sumsq(x, p)
    ops.sumsq_multi(xs, mul)
    again = [torch.full((P,), float("nan"), device=cuda) for _ in xs]
    ops.sumsq_multi(xs, again)
    torch.cuda.synchronize()
    for a, b, c, x in zip(sep, mul, again, xs):
        assert torch.equal(b, c) and not torch.isnan(b).any()
        assert abs(float(a.double().sum()) - float(b.double().sum())) <= 1e-5 * float(a.double().sum())
        assert abs(float(b.double().sum()) - float((x.double() ** 2).sum())) <= 1e-4 * float((x.double() ** 2).sum())


def test_trunk_fwd_bf16_staged_by_index_equals_lean_form(cuda):
    """cnn_trunk_fwd mode 3 (cnn_trunk_fwd_s16_kernel: bytes converted once into a bf16 image, y1/y2/y3 out through
    LDS as 16-byte rows) reading a PPO minibatch through an index == mode 5 (the same kernel on fragment-ordered
    weight copies) bit for bit, and both match the fp32 torch convolutions of the same bf16 operands."""
    import torch.nn.functional as F
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    g = torch.Generator(device="cpu").manual_seed(11)
    R, B = 300, 257
    obs = torch.randint(0, 256, (R, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    idx = torch.randint(0, R, (B,), generator=g).to(cuda)
    W1 = (torch.randn(32, 256, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    W2 = (torch.randn(64, 512, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    W3 = (torch.randn(64, 576, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    b1, b2, b3 = ((torch.rand(n, generator=g) * 0.1 - 0.02).to(cuda) for n in (32, 64, 64))
    from actor_critic_algs_on_tensorflow_amd.ops.optim import frag_order
    F1, F2, F3 = (frag_order(W, *W.shape) for W in (W1, W2, W3))
    outs = []
    for mode in (3, 5):   # 5: the staged kernel reading the fragment-ordered weight copies
        ys = [torch.full((B * r, c), float("nan"), dtype=torch.bfloat16, device=cuda)
              for r, c in ((400, 32), (81, 64), (49, 64))]
        w = (F1, F2, F3) if mode == 5 else (W1, W2, W3)
        G.cnn_trunk_fwd(obs, w[0], b1, w[1], b2, w[2], b3, *ys, mode=mode, obs_idx=idx)
        outs.append(ys)
    torch.cuda.synchronize()
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    x = obs[idx].float() / 255.0
    w1 = W1.float().view(32, 4, 8, 8)
    y1 = F.relu(F.conv2d(x, w1, b1, stride=4)).to(torch.bfloat16)
    w2 = W2.float().view(64, 4, 4, 32).permute(0, 3, 1, 2)
    y2 = F.relu(F.conv2d(y1.float(), w2, b2, stride=2)).to(torch.bfloat16)
    w3 = W3.float().view(64, 3, 3, 64).permute(0, 3, 1, 2)
    y3 = F.relu(F.conv2d(y2.float(), w3, b3, stride=1))
    got = outs[1][2].float().view(B, 7, 7, 64).permute(0, 3, 1, 2)
    assert torch.allclose(got, y3, rtol=2e-2, atol=2e-2), (got - y3).abs().max()


def test_register_move_wave_reductions_are_bit_identical_to_bpermute(cuda):
    """common.h wave_sum / wave_max (permlane32/16 swaps, DPP row_ror:8, row_shl/shr:4, quad permutes) == the
    ds_bpermute xor butterflies bit for bit in every lane, on random data with signed zeros and infinities mixed in."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(4096, 64, generator=g) * torch.exp(torch.randn(4096, 64, generator=g) * 4)
    x[::7, ::5] = -0.0
    x[::11, 3] = float("inf")
    x[::13, 9] = float("-inf")
    x = x.to(cuda)
    out = torch.empty(4096, 4, 64, device=cuda)
    ops.wave_reduce_check(x, out)
    torch.cuda.synchronize()
    a = out.view(torch.int32)
    assert torch.equal(a[:, 0], a[:, 1]), "wave_sum"
    assert torch.equal(a[:, 2], a[:, 3]), "wave_max"
    fin = torch.isfinite(out[:, 1]).all(dim=1)
    ref = x.double().sum(dim=1)
    assert torch.allclose(out[fin, 1, 0].double(), ref[fin], rtol=1e-4, atol=1e-3 * x.abs().max().item())


def test_mlp_ppo_adam_step_offsets_equal_ticket(cuda):
    """MuJoCo-shape PPO (MLP engine, separate actor / critic Adam in one opt_multi launch per minibatch): the grouped
    Adam launches taking their step from the minibatch index (no per-launch step ticket, counters advanced once per
    update) == the ticket form bit for bit -- parameters, Adam moments and step counters over captured updates."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    runs = []
    for offsets in (True, False):
        tr = ActorCriticTrainer(preset("mujoco_ppo_dp8", num_envs=16, n_steps=32, ppo_epochs=2, ppo_minibatches=4,
                                       device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0, seed=2,
                                       engine_opts=dict(adam_step_offsets=offsets)))
        tr.capture(warmup=1)
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
        state = [tr.flat.data.clone()]
        for o in tr.opts.values():
            state += [o.m.clone(), o.v.clone(), o.t.clone()]
        runs.append(state)
        t = float(list(tr.opts.values())[0].t)
        assert t >= 3 * 8 and t % 8 == 0, t   # whole updates of 2 x 4 minibatch steps
    for k, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), k


@pytest.mark.parametrize("preset_name,envs", [("pong_a2c", 32), ("breakout_ppo", 72)])
def test_fragment_ordered_weights_equal_row_major(cuda, preset_name, envs, monkeypatch):
    """EngineOpts.frag_weights: the conv weights' fragment-ordered bf16 copies, rewritten by the optimiser step itself
    (RMSprop for A2C, Adam for PPO) and read by the rollout step kernels (row-split at 32 envs, per-env split at 72)
    and the learner's staged trunk forward, give the same training bit for bit as the row-major weights -- and after
    the updates the copies equal frag_order(bf16 shadow) exactly (no stale copy)."""
    monkeypatch.setattr("actor_critic_algs_on_tensorflow_amd.ops.gemm.TUNE", False)
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    from actor_critic_algs_on_tensorflow_amd.ops.optim import frag_order
    runs = []
    for on in (True, False):
        kw = dict(n_steps=5) if preset_name == "pong_a2c" else dict(n_steps=8, ppo_epochs=2, ppo_minibatches=2)
        tr = ActorCriticTrainer(preset(preset_name, num_envs=envs, device="cuda:0", outdir=None, quiet=True,
                                       stdout_freq=0, save_every=0, seed=3, engine_opts=dict(frag_weights=on), **kw))
        eng = tr.engine
        assert (eng.frag is not None) == on
        tr.capture(warmup=1)
        snaps = []
        for _ in range(3):
            tr.step()
            st = tr.storage
            snaps.append([tr.flat.data.clone(), st.actions[:].clone(), st.values[:].clone(), st.logp[:].clone()])
        torch.cuda.synchronize()
        if on:
            for S, (K, N), F in zip((eng.sW1, eng.sW2, eng.sW3), eng._FRAG_SHAPES, eng.frag):
                assert torch.equal(F.view(torch.int16), frag_order(S, K, N).view(torch.int16))
        runs.append(snaps)
    for k, (a, b) in enumerate(zip(*runs)):
        for j, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x, y), (k, j)


def test_row_split_trunk_on_fragment_ordered_weights_is_bitwise(cuda):
    """cnn_trunk_fwd modes 6 / 7 (the row-split trunk reading fragment-ordered conv2 / conv3 weights) == modes 1 / 2
    bit for bit, shifted frames included."""
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    from actor_critic_algs_on_tensorflow_amd.ops.optim import frag_order
    g = torch.Generator(device="cpu").manual_seed(21)
    B = 37
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    W1 = (torch.randn(32, 256, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    W2 = (torch.randn(64, 512, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    W3 = (torch.randn(64, 576, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    b1, b2, b3 = ((torch.rand(n, generator=g) * 0.1 - 0.02).to(cuda) for n in (32, 64, 64))
    F2, F3 = frag_order(W2, 64, 512), frag_order(W3, 64, 576)
    for base in (1, 2):
        outs = []
        for mode in (base, base + 5):
            ys = [torch.full((B * r, c), float("nan"), dtype=torch.bfloat16, device=cuda)
                  for r, c in ((400, 32), (81, 64), (49, 64))]
            sh = torch.zeros_like(obs)
            w2, w3 = (F2, F3) if mode > 5 else (W2, W3)
            G.cnn_trunk_fwd(obs, W1, b1, w2, b2, w3, b3, *ys, shift_out=sh, mode=mode)
            outs.append(ys + [sh])
        torch.cuda.synchronize()
        for a, b in zip(*outs):
            assert torch.equal(a.view(torch.uint8) if a.dtype == torch.uint8 else a.view(torch.int16),
                               b.view(torch.uint8) if b.dtype == torch.uint8 else b.view(torch.int16)), base


@pytest.mark.parametrize("n,off", [(1, 0), (3, 1), (1024, 0), (1000003, 0), (4097, 1), (65536, 2)])
def test_cast_bf16_matches_torch_rounding(cuda, n, off):
    """The comm-buffer cast of bf16 DP buckets (vector path when both ends are aligned, scalar path otherwise) rounds
    exactly as torch's fp32 -> bf16 conversion."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(n + off)
    x = (torch.randn(n + off + 3, generator=g) * 1e3).to(cuda)
    x[::7] *= 1e-30
    y = torch.zeros(n + off, dtype=torch.bfloat16, device=cuda)
    ops.cast_bf16(x[off:off + n], y[off:])
    torch.cuda.synchronize()
    assert torch.equal(y[off:], x[off:off + n].to(torch.bfloat16))
