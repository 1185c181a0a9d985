"""Numerics of every hand-written HIP kernel against its fp32 PyTorch reference (run on an MI355X).

Each test calls the ``torch.ops.acamd`` op directly (the native path is required: the ``cuda`` fixture refuses to
run without the extension) and compares with the oracle in ``ops/*`` / ``envs/*`` evaluated on the same inputs.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(x):
    return x.to(torch.bfloat16)


# ------------------------------------------------------------------------------------------------------ GEMM
def _tile_bk():
    from actor_critic_algs_on_tensorflow_amd.ops.gemm import BKS   # every supported (tile, k-step) pair
    return [(t, bk) for t in sorted(BKS) for bk in BKS[t]]


TILE_BK = _tile_bk()


@pytest.mark.parametrize("a_k", [True, False])
@pytest.mark.parametrize("b_k", [True, False])
@pytest.mark.parametrize("tile,bk", TILE_BK)
def test_gemm_layouts_tiles(cuda, a_k, b_k, tile, bk):
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    g = torch.Generator(device="cpu").manual_seed(tile * 7 + a_k * 2 + b_k + bk)
    for (M, N, K) in [(70, 45, 100), (256, 128, 320), (33, 7, 512), (513, 96, 64)]:
        lda = (K if a_k else M) + 8
        ldb = (K if b_k else N) + 8
        A = _bf(torch.randn((M if a_k else K) * lda, generator=g)).to(cuda)
        B = _bf(torch.randn((N if b_k else K) * ldb, generator=g)).to(cuda)
        bias = torch.randn(N, generator=g).to(cuda)
        mask = _bf(torch.randn(M * N, generator=g)).to(cuda)
        ref = G.gemm_ref(A, lda, a_k, B, ldb, b_k, M, N, K, alpha=0.5, bias=bias, relu=True, mask=mask, ldm=N)
        C = torch.full((M * N,), float("nan"), device=cuda)
        colsum = torch.zeros(N, device=cuda)
        G.gemm(A, lda, a_k, B, ldb, b_k, C, N, 0, M, N, K, alpha=0.5, bias=bias, relu=True, mask=mask, ldm=N,
               colsum=colsum, tile=tile, splits=1, bk=bk)
        scale = ref.abs().max().item() + 1e-3
        assert (C.view(M, N) - ref).abs().max().item() <= 2e-3 * scale * math.sqrt(K / 64), (M, N, K)
        assert torch.allclose(colsum, ref.sum(0), rtol=1e-3, atol=1e-2 * scale)
        # bf16 output, slab split-K (deterministic last-arriver reduction)
        ws = G.GemmWorkspace(cuda)
        Cb = torch.empty(M * N, dtype=torch.bfloat16, device=cuda)
        G.gemm(A, lda, a_k, B, ldb, b_k, Cb, N, 1, M, N, K, alpha=0.5, bias=bias, relu=True, mask=mask, ldm=N,
               tile=tile, splits=4, workspace=ws, bk=bk)
        assert (Cb.view(M, N).float() - ref).abs().max().item() <= 1e-2 * scale
        assert int(ws.tickets.abs().sum()) == 0  # tickets are self-cleaning
        # atomic split-K (weight-gradient mode)
        Ca = torch.zeros(M * N, device=cuda)
        G.gemm(A, lda, a_k, B, ldb, b_k, Ca, N, 2, M, N, K, alpha=0.5, tile=tile, splits=3, bk=bk)
        ref2 = G.gemm_ref(A, lda, a_k, B, ldb, b_k, M, N, K, alpha=0.5)
        assert (Ca.view(M, N) - ref2).abs().max().item() <= 2e-3 * (ref2.abs().max().item() + 1e-3) * math.sqrt(K / 64)


def test_gemm_identity_asymmetric(cuda):
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    n = 64
    A = _bf(torch.eye(n)).to(cuda).reshape(-1)
    Bm = torch.arange(n * n, dtype=torch.float32).view(n, n) % 17 - 8
    for b_k in (True, False):
        B = _bf(Bm.t().contiguous() if b_k else Bm).to(cuda).reshape(-1)
        C = torch.zeros(n * n, device=cuda)
        G.gemm(A, n, True, B, n, b_k, C, n, 0, n, n, n, tile=0, splits=1, bk=64)
        assert torch.equal(C.view(n, n).cpu(), Bm)


@pytest.mark.parametrize("tile,bk", TILE_BK)
def test_gemm_implicit_im2col_matches_explicit(cuda, tile, bk):
    """The gathered (implicit-im2col) operands give bit-identical products to explicit im2col + plain GEMM."""
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    B = 3
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    y1 = _bf(torch.randn(B * 400, 32)).to(cuda)
    W1 = _bf(torch.randn(32, 256)).to(cuda)
    W2 = _bf(torch.randn(64, 512)).to(cuda)
    col1 = torch.empty(B * 400, 256, dtype=torch.bfloat16, device=cuda)
    G.im2col_u8(x, col1, 8, 8, 4)
    col2 = torch.empty(B * 81, 512, dtype=torch.bfloat16, device=cuda)
    G.im2col_nhwc(y1, col2, B, 20, 20, 32, 4, 4, 2)
    for src, ga, scale, col, W, M, N, K in [(x, [1, B, 4, 84, 84, 8, 8, 4], 1 / 255, col1, W1, B * 400, 32, 256),
                                            (y1, [2, B, 32, 20, 20, 4, 4, 2], 1.0, col2, W2, B * 81, 64, 512)]:
        C0 = torch.empty(M, N, device=cuda)
        C1 = torch.empty(M, N, device=cuda)
        G.gemm(col, K, True, W, K, True, C0, N, 0, M, N, K, tile=tile, bk=bk, splits=1)
        G.gemm(src, 0, True, W, K, True, C1, N, 0, M, N, K, tile=tile, bk=bk, splits=1, ga=ga, ga_scale=scale)
        assert torch.equal(C0, C1)
        # weight-gradient form: dW[n_out, k] = dY^T col, B gathered
        dY = _bf(torch.randn(M, N)).to(cuda)
        D0 = torch.zeros(N, K, device=cuda)
        D1 = torch.zeros(N, K, device=cuda)
        G.gemm(dY, N, False, col, K, False, D0, K, 2, N, K, M, tile=tile, bk=bk, splits=1)
        G.gemm(dY, N, False, src, 0, False, D1, K, 2, N, K, M, tile=tile, bk=bk, splits=1, gb=ga, gb_scale=scale)
        assert torch.equal(D0, D1)


# ------------------------------------------------------------------------------------------------------ conv lowering
def test_im2col_col2im(cuda):
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    B = 3
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    col = torch.empty(B * 400, 256, dtype=torch.bfloat16, device=cuda)
    G.im2col_u8(x, col, 8, 8, 4)
    ref = G.im2col_u8_ref(x.cpu(), 8, 8, 4).to(torch.bfloat16)
    assert torch.equal(col.cpu(), ref)
    y = _bf(torch.randn(B * 20 * 20, 32)).to(cuda)
    col2 = torch.empty(B * 81, 512, dtype=torch.bfloat16, device=cuda)
    G.im2col_nhwc(y, col2, B, 20, 20, 32, 4, 4, 2)
    assert torch.equal(col2.cpu().float(), G.im2col_nhwc_ref(y.cpu(), B, 20, 20, 32, 4, 4, 2))
    # col2im is the adjoint of im2col (with the ReLU mask)
    for (H, C, k, s) in [(20, 32, 4, 2), (9, 64, 3, 1)]:
        OH = (H - k) // s + 1
        dcol = _bf(torch.randn(B * OH * OH, k * k * C)).to(cuda)
        ym = _bf(torch.randn(B * H * H, C)).to(cuda)
        dx = torch.empty(B * H * H, C, dtype=torch.bfloat16, device=cuda)
        cs = torch.zeros(C, device=cuda)
        G.col2im_nhwc(dcol, ym, dx, cs, B, H, H, C, k, k, s)
        ref = G.col2im_nhwc_ref(dcol.cpu(), ym.cpu(), B, H, H, C, k, k, s)
        assert (dx.cpu().float() - ref).abs().max().item() < 0.05
        assert torch.allclose(cs.cpu(), dx.cpu().float().sum(0), rtol=1e-3, atol=1e-2)


# ------------------------------------------------------------------------------------------------------ env banks
@pytest.mark.parametrize("env_id", ["PongNoFrameskip-v4", "CartPole-v1", "Pendulum-v0", "HalfCheetahShape-v0"])
def test_env_bank_matches_oracle(cuda, env_id):
    from actor_critic_algs_on_tensorflow_amd import envs as E
    N = 16
    gpu = E.make(env_id, N, device=cuda, seed=5)
    cpu = E.make(env_id, N, device="cpu", seed=5)
    gpu.reset()
    cpu.reset()
    gpu.state.copy_(cpu.state)
    gpu.obs.copy_(cpu.obs)
    g = torch.Generator().manual_seed(1)
    steps = 300 if env_id.startswith("Pong") else 60
    for t in range(steps):
        a = cpu.sample_actions(generator=g)
        prev_c, prev_g = cpu.obs.clone(), gpu.obs.clone()
        oc, rc, dc, _ = cpu.step(a, prev_obs=prev_c, obs_out=cpu.obs)
        og, rg, dg, _ = gpu.step(a.to(cuda), prev_obs=prev_g, obs_out=gpu.obs)
        assert torch.equal(dc, dg.cpu()), (env_id, t)
        if env_id.startswith("Pong"):
            assert torch.equal(rc, rg.cpu()), t
            assert torch.equal(oc, og.cpu()), t
            assert torch.equal(cpu.state, gpu.state.cpu()), t
        else:
            assert torch.allclose(rc, rg.cpu(), rtol=1e-4, atol=1e-4), (env_id, t)
            assert torch.allclose(oc, og.cpu(), rtol=1e-4, atol=1e-4), (env_id, t)
            gpu.state.copy_(cpu.state)  # keep chaotic dynamics from drifting apart by ulps
            gpu.obs.copy_(cpu.obs)
    assert torch.allclose(cpu.ep_stats, gpu.ep_stats.cpu(), rtol=1e-4, atol=1e-3)


# ------------------------------------------------------------------------------------------------------ heads / returns
def test_categorical_and_gaussian_heads(cuda):
    from actor_critic_algs_on_tensorflow_amd.ops import distributions as D
    B, A = 2048, 6
    logits = torch.randn(B, A) * 2
    keys = torch.arange(B, dtype=torch.int64) * 7919 + (3 << 33)
    a_r, lp_r, e_r = D.categorical_sample_ref(logits, keys, 11)
    a_g, lp_g, e_g = D.categorical_sample(logits.to(cuda), keys.to(cuda), 11)
    assert (a_r == a_g.cpu()).float().mean() > 0.999
    same = a_r == a_g.cpu()
    assert torch.allclose(lp_r[same], lp_g.cpu()[same], atol=1e-5)
    assert torch.allclose(e_r, e_g.cpu(), atol=1e-5)
    # empirical distribution of Gumbel-max sampling matches softmax
    lg = torch.tensor([[0.0, 1.0, 2.0, -1.0]]).repeat(200000, 1)
    k = torch.arange(200000, dtype=torch.int64)
    a, _, _ = D.categorical_sample(lg.to(cuda), k.to(cuda), 3)
    freq = torch.bincount(a.cpu().long(), minlength=4).float() / 200000
    assert torch.allclose(freq, torch.softmax(lg[0], 0), atol=5e-3)
    mu = torch.randn(B, 3)
    ls = torch.tensor([0.3, -3.0, 1.0])
    r = D.gaussian_sample_ref(mu, ls, keys, 5)
    gq = D.gaussian_sample(mu.to(cuda), ls.to(cuda), keys.to(cuda), 5)
    for x, y in zip(r, gq):
        assert torch.allclose(x, y.cpu(), rtol=1e-4, atol=1e-4)


def test_returns_kernels(cuda):
    from actor_critic_algs_on_tensorflow_amd.ops import returns as R
    T, N = 37, 19
    g = torch.Generator().manual_seed(0)
    r = torch.randn(T, N, generator=g)
    v = torch.randn(T + 1, N, generator=g)
    d = (torch.rand(T, N, generator=g) < 0.1).to(torch.uint8)
    for L in (1, 5, 40):
        a = R.nstep_returns_ref(r, v, d, 0.98, L)
        b = R.nstep_returns(r.to(cuda), v.to(cuda), d.to(cuda), 0.98, L)
        for x, y in zip(a, b):
            assert torch.allclose(x, y.cpu(), atol=1e-4)
    a = R.gae_ref(r, v, d, 0.99, 0.95)
    b = R.gae(r.to(cuda), v.to(cuda), d.to(cuda), 0.99, 0.95)
    for x, y in zip(a, b):
        assert torch.allclose(x, y.cpu(), atol=1e-4)
    adv = torch.randn(5000, generator=g) * 3 + 1
    out = torch.empty(5000, device=cuda)
    from actor_critic_algs_on_tensorflow_amd import _native
    _native.require().normalize(adv.to(cuda), out, 1e-8)
    assert torch.allclose(out.cpu(), R.normalize_advantages(adv), atol=1e-5)


# ------------------------------------------------------------------------------------------------------ optimisers
@pytest.mark.parametrize("name", ["adam", "rmsprop"])
@pytest.mark.parametrize("clip,max_norm", [(None, None), (0.1, None), (None, 0.5), (1.0, 0.5)])
def test_fused_optimizers(cuda, name, clip, max_norm):
    from actor_critic_algs_on_tensorflow_amd.ops.optim import FlatParams, make_optimizer
    n = 100003
    p0 = torch.randn(n)
    res = {}
    for dev in ("cpu", cuda):
        p = torch.nn.Parameter(p0.clone())
        flat = FlatParams({"shared": [p]}, torch.device(dev))
        sh = torch.empty(flat.numel, dtype=torch.bfloat16, device=dev)
        opt = make_optimizer(name, flat, "shared", 1e-3, clip, max_norm, bf16_shadow=sh)
        g = torch.Generator().manual_seed(4)
        for _ in range(5):
            flat.grad.copy_((torch.randn(n, generator=g) * 0.3).to(dev))
            opt.step()
        res[str(dev)] = (flat.data.cpu(), sh.cpu(), float(opt.t))
    a, b = res["cpu"], res[str(cuda)]
    assert torch.allclose(a[0], b[0], rtol=1e-5, atol=1e-6)
    assert torch.allclose(b[1].float(), b[0], rtol=1e-2, atol=1e-3)
    if name == "adam":
        assert a[2] == b[2] == 5.0


# ------------------------------------------------------------------------------------------------------ loss
@pytest.mark.parametrize("ppo", [False, True])
def test_ac_loss_kernel_matches_autograd(cuda, ppo):
    from actor_critic_algs_on_tensorflow_amd import _native
    from actor_critic_algs_on_tensorflow_amd.algos import losses as L
    from actor_critic_algs_on_tensorflow_amd.ops import distributions as D
    B, A = 300, 6
    g = torch.Generator().manual_seed(2)
    z = torch.randn(B, A + 1, generator=g)
    act = torch.randint(0, A, (B,), generator=g, dtype=torch.int32)
    lpo = D.categorical_logp_entropy(z[:, :A], act)[0] + 0.1 * torch.randn(B, generator=g)
    adv = torch.randn(B, generator=g)
    ret = torch.randn(B, generator=g)
    ent_c, kl_c, vf = 0.01, 0.3, 0.5
    zz = z.clone().requires_grad_(True)
    logp, ent = D.categorical_logp_entropy(zz[:, :A], act)
    if ppo:
        al, pg, kl, em, cf = L.ppo_actor_loss(logp, lpo, adv, ent, 0.2, ent_c, kl_c)
    else:
        al, pg, kl, em = L.actor_loss(logp, lpo, adv, ent, kl_c, ent_c)
    vl = L.value_loss(zz[:, A], ret)
    (al + vf * vl).backward()
    zc = z.to(cuda)
    dz = torch.empty(B, A + 1, dtype=torch.bfloat16, device=cuda)
    stats = torch.zeros(8, device=cuda)
    _native.require().ac_loss(zc, A + 1, zc[:, A:], A + 1, act.to(cuda), None, None, lpo.to(cuda), adv.to(cuda),
                              ret.to(cuda), None, torch.tensor(ent_c, device=cuda), torch.tensor(kl_c, device=cuda),
                              vf, 0.2 if ppo else 0.0, 0.0, dz, A + 1, dz[:, A:], A + 1, None, stats, B, A, False)
    assert torch.allclose(dz.cpu().float(), zz.grad, rtol=2e-2, atol=2e-5)
    s = stats.cpu()
    assert abs(s[5] - al.item()) < 1e-4 and abs(s[3] - vl.item()) < 1e-4 and abs(s[1] - kl.item()) < 1e-5


# ------------------------------------------------------------------------------------------------------ engine
@pytest.mark.parametrize("implicit,fused,tconv", [(True, True, True), (True, False, False), (False, False, False)])
def test_cnn_engine_matches_autograd(cuda, implicit, fused, tconv):
    """Full native forward + loss + backward of the Atari CNN vs fp32 autograd on the same parameters."""
    from actor_critic_algs_on_tensorflow_amd.algos import losses as L
    from actor_critic_algs_on_tensorflow_amd.algos.engine import CNNEngine
    from actor_critic_algs_on_tensorflow_amd.models.policy import CNNActorCritic
    from actor_critic_algs_on_tensorflow_amd.ops import distributions as D
    from actor_critic_algs_on_tensorflow_amd.ops.optim import FlatParams
    torch.manual_seed(0)
    A, B = 6, 24
    model = CNNActorCritic(A, generator=torch.Generator().manual_seed(3)).to(cuda)
    with torch.no_grad():  # make the tiny head weights large enough to test the head gradient path well
        model.net.heads.kernel.mul_(20)
        for m in (model.net.trunk.conv1, model.net.trunk.conv2, model.net.trunk.conv3):
            m.bias.uniform_(-0.05, 0.1)
    flat = FlatParams(model.param_groups(), cuda)
    shadow = flat.data.to(torch.bfloat16)
    eng = CNNEngine(model, flat, shadow, implicit=implicit, fused_trunk_max_b=None if fused else 0, tconv_dgrad=tconv)
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    b = eng.bufs(B, with_grad=True)
    z = eng.forward(obs, b).clone()
    # fp32 reference on the bf16-rounded parameters
    ref_model = CNNActorCritic(A).to(cuda)
    with torch.no_grad():
        for pr, p in zip(ref_model.parameters(), model.parameters()):
            pr.copy_(p.to(torch.bfloat16).float())
    logits, v = ref_model(obs)
    zr = torch.cat([logits, v[:, None]], 1)
    assert (z - zr).abs().max().item() < 3e-2 * (zr.abs().max().item() + 1e-2)
    act = torch.randint(0, A, (B,), device=cuda, dtype=torch.int32)
    lpo = D.categorical_logp_entropy(zr[:, :A].detach(), act)[0]
    adv = torch.randn(B, device=cuda)
    ret = torch.randn(B, device=cuda)
    ec, kc = torch.tensor(0.01, device=cuda), torch.tensor(0.0, device=cuda)
    flat.zero_grad()
    eng.loss(b, act, lpo, adv, ret, None, ec, kc, 0.5, 0.0, 0.0)
    eng.backward(b)
    logp, ent = D.categorical_logp_entropy(logits, act)
    al, *_ = L.actor_loss(logp, lpo, adv, ent, 0.0, 0.01)
    (al + 0.5 * L.value_loss(v, ret)).backward()
    for (name, p), pr in zip(model.named_parameters(), ref_model.parameters()):
        i = [id(q) for q in flat.params].index(id(p))
        off = flat.offsets[i]
        g = flat.grad[off:off + p.numel()].view_as(p)
        err = (g - pr.grad).norm() / (pr.grad.norm() + 1e-12)
        assert err < 0.05, (name, float(err))


def test_cnn_trunk_fused_matches_layers(cuda):
    """Fused conv1..conv3 kernel vs an fp32 PyTorch conv stack fed the same bf16-rounded inputs per layer."""
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    import torch.nn.functional as F
    torch.manual_seed(1)
    B = 37
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    W1 = (torch.randn(32, 4, 8, 8, device=cuda) * 0.05).to(torch.bfloat16)          # OIHW
    W2 = (torch.randn(64, 4, 4, 32, device=cuda) * 0.05).to(torch.bfloat16)         # OHWI
    W3 = (torch.randn(64, 3, 3, 64, device=cuda) * 0.05).to(torch.bfloat16)
    b1, b2, b3 = (torch.rand(n, device=cuda) * 0.1 - 0.02 for n in (32, 64, 64))
    y1 = torch.empty(B * 400, 32, dtype=torch.bfloat16, device=cuda)
    y2 = torch.empty(B * 81, 64, dtype=torch.bfloat16, device=cuda)
    y3 = torch.empty(B * 49, 64, dtype=torch.bfloat16, device=cuda)
    G.cnn_trunk_fwd(obs, W1.reshape(32, 256), b1, W2.reshape(64, 512), b2, W3.reshape(64, 576), b3, y1, y2, y3)
    x = (obs.float() / 255.0).to(torch.bfloat16).float()
    r1 = F.relu(F.conv2d(x, W1.float(), b1, stride=4))                                 # [B, 32, 20, 20]
    assert torch.allclose(y1.float().view(B, 20, 20, 32).permute(0, 3, 1, 2), r1, rtol=1e-2, atol=1e-2)
    x2 = y1.float().view(B, 20, 20, 32).permute(0, 3, 1, 2)
    r2 = F.relu(F.conv2d(x2, W2.float().permute(0, 3, 1, 2), b2, stride=2))
    assert torch.allclose(y2.float().view(B, 9, 9, 64).permute(0, 3, 1, 2), r2, rtol=1e-2, atol=1e-2)
    x3 = y2.float().view(B, 9, 9, 64).permute(0, 3, 1, 2)
    r3 = F.relu(F.conv2d(x3, W3.float().permute(0, 3, 1, 2), b3, stride=1))
    assert torch.allclose(y3.float().view(B, 7, 7, 64).permute(0, 3, 1, 2), r3, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("k,s,H,Cout,Cin,B,subpixel", [(3, 1, 9, 64, 64, 5, False), (4, 2, 20, 64, 32, 3, False),
                                                        (8, 4, 84, 32, 8, 2, False), (4, 2, 20, 64, 32, 160, True),
                                                        (8, 4, 84, 32, 8, 32, True), (4, 2, 20, 64, 32, 16, True)])
def test_gemm_transposed_conv_dgrad(cuda, k, s, H, Cout, Cin, B, subpixel):
    """Data-gradient GEMM (A gathered from dy on the stride grid, B = OHWI weight read transposed) vs
    torch conv_transpose2d, with the ReLU mask and bias-gradient column sums of the epilogue."""
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    import torch.nn.functional as F
    torch.manual_seed(2)
    OH = (H - k) // s + 1
    dy = torch.randn(B, OH, OH, Cout, device=cuda).to(torch.bfloat16)
    W = (torch.randn(Cout, k, k, Cin, device=cuda) * 0.1).to(torch.bfloat16)        # OHWI
    ymask = (torch.rand(B * H * H, Cin, device=cuda) > 0.3).to(torch.bfloat16)
    out = torch.empty(B * H * H, Cin, dtype=torch.bfloat16, device=cuda)
    cs = torch.zeros(Cin, device=cuda)
    ran = 0
    for tile, bk in ((4, 64), (2, 128), (0, 64)):
        cs.zero_()
        if subpixel:   # rows per phase B*(H/s)^2 must be a multiple of the tile height
            if (B * (H // s) ** 2) % G.TILES[tile][0]:
                continue
            G._native.require().gemm(dy, 0, True, W, 0, False, out, Cin, 1, B * H * H, Cin, (k // s) ** 2 * Cout, 1.0,
                                     None, False, ymask, Cin, cs, 0, tile, bk, 1, None, None,
                                     [5, B, Cout, H, H, k, k, s], 1.0, [6, 1, Cout, 1, Cin, k, k, s], 1.0)
        else:
            G._native.require().gemm(dy, 0, True, W, 0, False, out, Cin, 1, B * H * H, Cin, k * k * Cout, 1.0, None,
                                     False, ymask, Cin, cs, 0, tile, bk, 1, None, None, [3, B, Cout, H, H, k, k, s],
                                     1.0, [4, 1, Cout, 1, Cin, k, k, 1], 1.0)
        ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), W.float().permute(0, 3, 1, 2), stride=s)
        ref = ref[:, :, :H, :H].permute(0, 2, 3, 1).reshape(B * H * H, Cin) * ymask.float()
        assert torch.allclose(out.float(), ref, rtol=2e-2, atol=2e-2), (tile, bk, (out.float() - ref).abs().max())
        # column sums are taken from the fp32 values before the bf16 store
        err = (cs - ref.sum(0)).abs()
        assert (err <= 1e-2 * ref.abs().sum(0) + 1e-2).all(), (tile, bk, err.max())
        ran += 1
    assert ran > 0


def test_trainer_native_graph_updates(cuda):
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    for algo in ("pong_a2c", "breakout_ppo"):
        kw = dict(num_envs=8, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0)
        if algo == "breakout_ppo":
            kw.update(n_steps=16, ppo_minibatches=2, ppo_epochs=2)
        tr = ActorCriticTrainer(preset(algo, **kw))
        assert tr.engine is not None
        tr.capture(warmup=1)
        p0 = tr.flat.data.clone()
        for _ in range(5):
            tr.step()
        torch.cuda.synchronize()
        assert torch.isfinite(tr.flat.data).all()
        assert (tr.flat.data - p0).abs().max() > 0
        assert torch.isfinite(torch.stack(list(tr.stats.values()))).all()


def test_a2c_activation_reuse_is_exact(cuda):
    """Learner on the rollout's stored activations == learner that recomputes its forward (same params)."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    res = []
    for reuse in (True, False):
        cfg = preset("pong_a2c", num_envs=8, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0,
                     cuda_graph=False, reuse_rollout_acts=reuse, optimizer="adam", max_grad_norm=None)
        tr = ActorCriticTrainer(cfg)
        p0 = tr.flat.data.clone()
        tr.step()
        torch.cuda.synchronize()
        res.append((tr.flat.data - p0, tr.storage.actions.clone(), tr.stats_buf.clone()))
    assert torch.equal(res[0][1], res[1][1])
    # same loss statistics; same update up to bf16 rounding of activations recomputed with another tile plan
    assert torch.allclose(res[0][2], res[1][2], rtol=1e-3, atol=1e-5)
    d0, d1 = res[0][0], res[1][0]
    assert (d0 - d1).norm() / d0.norm() < 0.05


def test_fused_policy_env_step_matches_separate_kernels(cuda):
    """env_policy_step_pong == head GEMM + categorical_sample_env + env_step_pong on the same inputs."""
    from actor_critic_algs_on_tensorflow_amd import _native
    from actor_critic_algs_on_tensorflow_amd import envs as E
    ops = _native.require()
    N, A = 16, 6
    g = torch.Generator().manual_seed(5)
    h = torch.relu(torch.randn(N, 512, generator=g)).to(torch.bfloat16).to(cuda)
    Wh = (torch.randn(512 * (A + 1), generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    bh = torch.randn(A + 1, generator=g).to(cuda)
    outs = []
    for fused in (True, False, "pre_shifted"):
        env = E.make("PongNoFrameskip-v4", N, device=cuda, seed=3)
        o0 = env.reset().clone()
        o1 = torch.empty_like(o0)
        act = torch.empty(N, dtype=torch.int32, device=cuda)
        lp, en, val = (torch.empty(N, device=cuda) for _ in range(3))
        z = torch.empty(N, A + 1, device=cuda)
        rew = torch.empty(N, device=cuda)
        dn, tr = (torch.empty(N, dtype=torch.uint8, device=cuda) for _ in range(2))
        if fused == "pre_shifted":
            # the fused trunk writes the shifted stack into o1, the env kernel then only renders the newest frame
            W = [(torch.randn(n, generator=g) * 0.05).to(torch.bfloat16).to(cuda) for n in (8192, 32768, 36864)]
            bb = [torch.zeros(n, device=cuda) for n in (32, 64, 64)]
            ys = [torch.empty(N * r, c, dtype=torch.bfloat16, device=cuda) for r, c in ((400, 32), (81, 64), (49, 64))]
            ops.cnn_trunk_fwd(o0, W[0], bb[0], W[1], bb[1], W[2], bb[2], ys[0], ys[1], ys[2], 1.0 / 255.0, o1)
            ops.env_policy_step_pong(h, Wh, bh, z, act, lp, en, val, 20, 77, env.state, env.t, env.tg, env.ep_ret,
                                     env.ep_stats, env.env_ids, o0, o1, rew, dn, tr, env.seed,
                                     env.max_episode_steps, 4, True)
        elif fused:
            ops.env_policy_step_pong(h, Wh, bh, z, act, lp, en, val, 20, 77, env.state, env.t, env.tg, env.ep_ret,
                                     env.ep_stats, env.env_ids, o0, o1, rew, dn, tr, env.seed,
                                     env.max_episode_steps, 4)
        else:
            z = (h.float() @ Wh.float().view(512, A + 1)) + bh
            ops.categorical_sample_env(z[:, :A].contiguous(), env.tg, env.env_ids, 20, 77, act, lp, en, None)
            val = z[:, A].clone()
            env.step(act, prev_obs=o0, obs_out=o1, reward_out=rew, done_out=dn, trunc_out=tr)
        outs.append((act.clone(), lp.clone(), en.clone(), val.clone(), o1.clone(), z.clone()))
    (a0, l0, e0, v0, f0, z0), (a1, l1, e1, v1, f1, z1), (a2, l2, e2, v2, f2, z2) = outs
    assert torch.equal(a0, a2) and torch.equal(f0, f2) and torch.equal(z0, z2) and torch.equal(l0, l2)
    assert torch.allclose(z0, z1, atol=2e-3)
    same = a0 == a1
    assert same.float().mean() >= 0.9
    assert torch.allclose(l0[same], l1[same], atol=2e-3) and torch.allclose(e0, e1, atol=2e-3)
    assert torch.allclose(v0, v1, atol=2e-3)
    assert torch.equal(f0[same], f1[same])


def test_fc_partial_planes_and_consumers(cuda):
    """GEMM out_mode 3 (split-K partial planes) + its consumers: fc_value and the fused policy step reducing the
    planes themselves (bias + ReLU + bf16 like the GEMM epilogue) == the finished-h path."""
    from actor_critic_algs_on_tensorflow_amd import _native
    from actor_critic_algs_on_tensorflow_amd import envs as E
    from actor_critic_algs_on_tensorflow_amd.ops import gemm as G
    ops = _native.require()
    g = torch.Generator().manual_seed(11)
    N, A = 32, 6
    y3 = torch.relu(torch.randn(N, 3136, generator=g)).to(torch.bfloat16).to(cuda)
    Wfc = (torch.randn(3136, 512, generator=g) * 0.02).to(torch.bfloat16).to(cuda)
    bfc = (torch.randn(512, generator=g) * 0.1).to(cuda)
    Wh = (torch.randn(512 * (A + 1), generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    bh = torch.randn(A + 1, generator=g).to(cuda)
    ref = torch.relu(y3.float() @ Wfc.float() + bfc)
    for tile, bk, splits in ((1, 64, 4), (4, 256, 8), (0, 128, 1), (4, 64, 32), (1, 64, 16)):
        hp = torch.full((32 * N * 512,), float("nan"), device=cuda)   # unused planes must never be read as data
        S = G.gemm(y3, 3136, True, Wfc, 512, False, hp, 512, 3, N, 512, 3136, tile=tile, bk=bk, splits=splits,
                   max_planes=32)
        assert S == G.effective_splits(3136, bk, splits)
        h_sum = torch.relu(hp.view(32, N, 512)[:S].sum(0) + bfc)
        assert torch.allclose(h_sum, ref, rtol=1e-3, atol=1e-3)
        val = torch.empty(N, device=cuda)
        hout = torch.empty(N, 512, dtype=torch.bfloat16, device=cuda)
        ops.fc_value(hp, S, bfc, Wh, bh, val, hout)
        assert torch.allclose(hout.float(), ref, rtol=1e-2, atol=1e-2)
        vref = hout.float() @ Wh.float().view(512, A + 1)[:, A] + bh[A]
        assert torch.allclose(val, vref, rtol=1e-4, atol=1e-4)
        outs = []
        for parts in (True, False):
            env = E.make("PongNoFrameskip-v4", N, device=cuda, seed=3)
            o0 = env.reset().clone()
            o1 = torch.empty_like(o0)
            act = torch.empty(N, dtype=torch.int32, device=cuda)
            lp, en, v = (torch.empty(N, device=cuda) for _ in range(3))
            z = torch.empty(N, A + 1, device=cuda)
            rew = torch.empty(N, device=cuda)
            dn, tr = (torch.empty(N, dtype=torch.uint8, device=cuda) for _ in range(2))
            h = torch.empty(N, 512, dtype=torch.bfloat16, device=cuda) if parts else hout.clone()
            ops.env_policy_step_pong(h, Wh, bh, z, act, lp, en, v, 20, 77, env.state, env.t, env.tg, env.ep_ret,
                                     env.ep_stats, env.env_ids, o0, o1, rew, dn, tr, env.seed,
                                     env.max_episode_steps, 4, False, hp if parts else None, S if parts else 0,
                                     bfc if parts else None)
            outs.append((h.clone(), z.clone(), act.clone(), v.clone(), o1.clone()))
        for a, b in zip(outs[0], outs[1]):
            assert torch.equal(a, b)
        assert torch.allclose(outs[0][3], val, atol=1e-5)
