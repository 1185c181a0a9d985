"""Round-5 HIP kernels vs fp32 / fp64 PyTorch references of the same op.

* ``a2c_head_env`` (loss.hip): the A2C learner head as one workgroup per env -- V(s_T) from the rollout's last fc
  partial planes, returns, loss, dz, dh and per-env partial planes of dWh / dbfc / dbh + fp64 statistics rows --
  against the 32-workgroup ``a2c_head`` (which itself is pinned to fc_value + head_bwd and to autograd in
  test_gpu_r3 / test_gpu_learning), and the whole headline update through it against the ``a2c_head`` path.
* ``fc_rollout`` (fc_rollout.hip): the rollout fc product on the fragment-ordered Wfc copy vs an fp64 product of the
  same bf16 operands, every variant.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,N,mode", [(5, 32, 1), (5, 32, 2), (16, 24, 2), (5, 7, 1), (40, 3, 1)])
def test_a2c_head_env_matches_a2c_head(cuda, T, N, mode):
    """Per-env head == the grid-barrier head: V(s_T), targets / advantages and dh bit-identical (same plane
    reduction and dot-product tree, same per-row arithmetic); dWh / dbfc / dbh (per-env planes summed over envs) and
    the statistics (per-env fp64 rows combined by the finaliser duty) equal up to the summation order over rows."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    A, A1, B, S = 6, 7, T * N, 13
    g = torch.Generator(device="cpu").manual_seed(T * 100 + N + mode)
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
    L = 5

    def outs():
        return dict(ret=torch.zeros(B, device=cuda), adv=torch.zeros(B, device=cuda),
                    dh=torch.zeros(B, 512, dtype=torch.bfloat16, device=cuda), gWh=torch.zeros(512 * A1, device=cuda),
                    gbh=torch.zeros(A1, device=cuda), gbfc=torch.zeros(512, device=cuda),
                    stats=torch.zeros(8, device=cuda))

    ref, new = outs(), outs()
    vref = val0.clone()
    bar = torch.zeros(4, dtype=torch.int32, device=cuda)
    ops.a2c_head(z, act, lpo, ent, kl, 0.5, rew, vref, dones, L, mode, False, 0.99, 0.95, ref["ret"], ref["adv"], h,
                 Wh, ref["dh"], ref["gWh"], ref["gbh"], ref["gbfc"], ref["stats"], hpart, S, bfc, bh, bar)
    vnew = val0.clone()
    vnew[T] = float("nan")
    pWh, pbfc, pbh = (torch.full((N * n,), float("nan"), device=cuda) for n in (512 * A1, 512, A1))
    spart = torch.full((N, 10), float("nan"), dtype=torch.float64, device=cuda)
    ops.a2c_head_env(z, act, lpo, ent, kl, 0.5, rew, vnew, dones, L, mode, 0.99, 0.95, new["ret"], new["adv"], h, Wh,
                     new["dh"], hpart, S, bfc, bh, pWh, pbfc, pbh, spart)
    # the finaliser's statistics duty (no jobs but the duty's extra workgroup: one empty job)
    jobs = torch.zeros(1, 8, dtype=torch.int64, device=cuda)
    dummy = torch.zeros(4, device=cuda)
    jobs[0, 0] = dummy.data_ptr()
    jobs[0, 2] = 4
    parts = torch.zeros(256, device=cuda)
    ops.grad_finalize(jobs, parts, spart, B, ent, kl, new["stats"])
    torch.cuda.synchronize()
    assert torch.equal(vnew, vref)
    for k in ("ret", "adv", "dh"):
        assert torch.equal(new[k], ref[k]), k
    torch.testing.assert_close(pWh.view(N, -1).sum(0), ref["gWh"], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(pbfc.view(N, -1).sum(0), ref["gbfc"], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(pbh.view(N, -1).sum(0), ref["gbh"], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(new["stats"], ref["stats"], rtol=1e-4, atol=1e-6)
    # without planes the kernel reads V(s_T) from val
    new2 = outs()
    pWh2 = torch.zeros_like(pWh)
    ops.a2c_head_env(z, act, lpo, ent, kl, 0.5, rew, vnew, dones, L, mode, 0.99, 0.95, new2["ret"], new2["adv"], h,
                     Wh, new2["dh"], None, 0, None, None, pWh2, torch.zeros_like(pbfc), torch.zeros_like(pbh),
                     torch.zeros_like(spart))
    torch.cuda.synchronize()
    for k in ("ret", "adv", "dh"):
        assert torch.equal(new2[k], new[k]), k
    assert torch.equal(pWh2, pWh)


def test_a2c_update_with_per_env_head_matches_a2c_head(cuda):
    """Native Pong A2C, 3 graph-captured updates: the per-env head (head gradients as per-env planes summed by the
    finaliser, statistics by its duty workgroup) tracks the a2c_head path: statistics close, parameters equal up to
    the summation order of dWh / dbfc / dbh; and the update stays bitwise deterministic."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    res = {}
    for knob in (True, False, True):
        cfg = preset("pong_a2c", num_envs=32, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0,
                     engine_opts=dict(a2c_head_env=knob))
        tr = ActorCriticTrainer(cfg)
        tr.capture(warmup=1)
        p0 = tr.flat.data.clone()
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
        assert bool(tr.engine._ae) == knob
        out = (tr.flat.data - p0, tr.stats_buf.clone(), tr.storage.values.clone())
        if knob in res:
            assert all(torch.equal(a, b) for a, b in zip(out, res[knob])), "per-env head update not deterministic"
        res[knob] = out
    d1, s1, _ = res[True]
    d0, s0, _ = res[False]
    assert torch.allclose(s0[:8], s1[:8], rtol=1e-3, atol=1e-5), (s0[:8], s1[:8])
    assert (d0 - d1).norm() / d0.norm() < 1e-2, float((d0 - d1).norm() / d0.norm())


@pytest.mark.parametrize("M", [32, 7, 1, 128, 70])
def test_fc_rollout_matches_fp64_product(cuda, M):
    """fc_rollout's planes summed in plane order == X @ W in fp64 (same bf16 operands) for every variant; the
    fragment-ordered copy is frag_order_kc of the row-major weight."""
    from actor_critic_algs_on_tensorflow_amd import _native
    from actor_critic_algs_on_tensorflow_amd.ops.optim import frag_order_kc
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(M)
    X = (torch.randn(M, 3136, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    W = (torch.randn(3136, 512, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    Wf = frag_order_kc(W.float(), 3136, 512)
    # the layout itself: element (k, n) at ((k/16 * 16 + n/32) * 64 + (k/8 % 2) * 32 + n % 32) * 8 + k % 8
    k, n = 1234, 345
    assert torch.equal(Wf[((k // 16 * 16 + n // 32) * 64 + (k // 8 % 2) * 32 + n % 32) * 8 + k % 8], W[k, n])
    ref = X.double() @ W.double()
    for v in range(10):
        if v == 9 and M > 64:
            continue   # rejected by the launcher (would spill)
        hp = torch.full((32 * M * 512,), float("nan"), device=cuda)
        S = ops.fc_rollout(X, Wf, hp, v)
        got = hp.view(32, M, 512)[:S].double().sum(0)
        assert float((got - ref).abs().max() / ref.abs().max()) < 1e-5, v


@pytest.mark.parametrize("cls_name", ["rmsprop", "adam"])
def test_optimiser_writes_the_kc_fragment_copy(cuda, cls_name):
    """The native optimiser's k-contiguous fragment region (optim.hip opt_body wave items, layout -2): parameters,
    moments and the row-major bf16 shadow bit-identical to the same update without the region (the per-element
    arithmetic is shared), and the copy == frag_order_kc of the updated shadow, over 3 steps; a conv-layout copy in
    the same segment stays current too."""
    from actor_critic_algs_on_tensorflow_amd.ops.optim import (FlatParams, FusedAdam, FusedRMSprop, frag_order,
                                                               frag_order_kc)
    cls = FusedRMSprop if cls_name == "rmsprop" else FusedAdam
    runs = []
    for with_kc in (True, False):
        g = torch.Generator(device="cpu").manual_seed(11)
        Wc = torch.nn.Parameter(torch.randn(64, 512, generator=g).to(cuda))
        Wa = torch.nn.Parameter(torch.randn(37, generator=g).to(cuda))
        Wk = torch.nn.Parameter(torch.randn(3136, 512, generator=g).to(cuda))
        flat = FlatParams({"shared": [Wc, Wa, Wk]}, cuda)
        sh = torch.empty(flat.numel, dtype=torch.bfloat16, device=cuda)
        sh.copy_(flat.data)
        opt = cls(flat, "shared", lr=1e-2, max_grad_norm=0.5, bf16_shadow=sh)
        Fc = torch.empty(64 * 512, dtype=torch.bfloat16, device=cuda)
        Fk = torch.full((3136 * 512,), float("nan"), dtype=torch.bfloat16, device=cuda)
        vc = flat.data[flat.offsets[0]:flat.offsets[0] + Wc.numel()]
        ok, nk = flat.offsets[2], Wk.numel()
        ent = [(vc, 64, 512, Fc)] + ([(flat.data[ok:ok + nk], 3136, 512, Fk, -2)] if with_kc else [])
        opt.set_frag(ent)
        for _ in range(3):
            flat.grad.copy_(torch.randn(flat.numel, generator=g).to(cuda))
            from actor_critic_algs_on_tensorflow_amd import _native
            ops = _native.require()
            ops.sumsq(flat.grad, opt._partial)
            opt.ext_parts = opt._partial
            opt.step()
        torch.cuda.synchronize()
        assert torch.equal(Fc, frag_order(sh[flat.offsets[0]:flat.offsets[0] + Wc.numel()].float(), 64, 512))
        if with_kc:
            assert torch.equal(Fk, frag_order_kc(sh[ok:ok + nk].float(), 3136, 512))
        runs.append((flat.data.clone(), opt.v.clone(), sh.clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [160, 7, 256, 33, 1])
def test_fc_bwd_matches_fp64(cuda, B):
    """fc_bwd.hip: dWfc = y3^T dh (fp32, every element stored), its per-(tile, wave) sums of squares (the finaliser's
    presummed norm partials) and dy3 = (dh Wfc^T) * (y3 > 0) (bf16) against fp64 products of the same bf16
    operands."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(B)
    dh = (torch.randn(B, 512, generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    W = (torch.randn(3136, 512, generator=g) * 0.05).to(torch.bfloat16).to(cuda)
    y3 = torch.relu(torch.randn(B, 3136, generator=g)).to(torch.bfloat16).to(cuda)
    dy3 = torch.full((B, 3136), float("nan"), dtype=torch.bfloat16, device=cuda)
    dW = torch.full((3136, 512), float("nan"), device=cuda)
    sq = torch.full((392 * 4,), float("nan"), device=cuda)
    ops.fc_bwd(dh, W, y3, dy3, dW, None, sq)
    torch.cuda.synchronize()
    # per (64 x 64 tile, wave quadrant) sums of squares: tile t = kf block t // 8, n block t % 8 in XCD order is a
    # permutation, so compare per-tile sets and the total
    q = dW.double().view(49, 2, 32, 8, 2, 32).pow(2).sum((2, 5))          # [kf blk, mq, n blk, nq]
    ref_sq = q.permute(0, 2, 1, 3).reshape(392 * 4)                       # tile (i, j) -> wave 2 mq + nq
    assert float((sq.double() - ref_sq).abs().max() / ref_sq.abs().max()) < 1e-5
    ref_w = y3.double().t() @ dh.double()
    assert float((dW.double() - ref_w).abs().max() / ref_w.abs().max()) < 1e-5
    ref_d = (dh.double() @ W.double().t()) * (y3.double() > 0)
    err = (dy3.double() - ref_d).abs()
    assert bool((err <= ref_d.abs() * 2.0 ** -8 + 1e-6).all()), float(err.max())
    assert bool((dy3[y3 == 0] == 0).all())


@pytest.mark.parametrize("B,persist", [(1100, 256), (300, 7)])
def test_trunk_bwd_persist_bias_rows_accumulated_per_workgroup(cuda, B, persist):
    """cnn_trunk_bwd_persist with bias_acc: dy2 / dy1 bit-identical to the per-sample-row form, and row w of biasp ==
    the fp32 sum, in walk order (samples w, w + grid, ...), of the per-sample rows the plain form writes."""
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(B)
    dy3 = (torch.randn(B, 7, 7, 64, generator=g) * (torch.rand(B, 7, 7, 64, generator=g) > 0.4)).to(torch.bfloat16)
    W3 = (torch.randn(64, 3, 3, 64, generator=g) * 0.05).to(torch.bfloat16)
    W2 = (torch.randn(64, 4, 4, 32, generator=g) * 0.05).to(torch.bfloat16)
    y2 = (torch.rand(B, 9, 9, 64, generator=g) - 0.3).clamp(min=0).to(torch.bfloat16)
    y1 = (torch.rand(B, 20, 20, 32, generator=g) - 0.3).clamp(min=0).to(torch.bfloat16)
    dev = [t.to(cuda) for t in (dy3, W3, y2, W2, y1)]
    args = (dev[0].reshape(B * 49, 64), dev[1].reshape(64, 576), dev[2].reshape(B * 81, 64), dev[3].reshape(64, 512),
            dev[4].reshape(B * 400, 32))
    res = []
    for acc in (False, True):
        dy2 = torch.full((B * 81, 64), float("nan"), dtype=torch.bfloat16, device=cuda)
        dy1 = torch.full((B * 400, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
        bp = torch.full((B, 160), float("nan"), device=cuda)
        ops.cnn_trunk_bwd(*args, dy2, dy1, bp, None, persist, None, None, None, 1.0, acc)
        torch.cuda.synchronize()
        res.append((dy2.view(torch.int16).clone(), dy1.view(torch.int16).clone(), bp.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    rows, got = res[0][2], res[1][2]
    grid = min(persist, B)
    for w in range(grid):
        ref = torch.zeros(160)
        for b in range(w, B, grid):
            ref = ref + rows[b]
        assert torch.equal(got[w], ref), w
    assert torch.isnan(got[grid:]).all(), "rows past the grid are not written"


@pytest.mark.parametrize("B,persist,idx", [(1100, 256, True), (300, 7, False)])
def test_persistent_trunk_bwd_conv1_fold_matches_fp64(cuda, B, persist, idx):
    """The persistent trunk backward with the conv1 weight gradient folded in: dy2 and the bias rows bit-identical to
    the plain persistent kernel, dy1 not stored (skip_dy1), and plane w == scale * sum over the workgroup's samples
    (w, w + grid, ...) of dy1_b^T unfold(obs_b), in fp64, using the dy1 the plain kernel writes."""
    import torch.nn.functional as F
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    g = torch.Generator(device="cpu").manual_seed(B + persist)
    dy3 = (torch.randn(B, 7, 7, 64, generator=g) * (torch.rand(B, 7, 7, 64, generator=g) > 0.4)).to(torch.bfloat16)
    W3 = (torch.randn(64, 3, 3, 64, generator=g) * 0.05).to(torch.bfloat16)
    W2 = (torch.randn(64, 4, 4, 32, generator=g) * 0.05).to(torch.bfloat16)
    y2 = (torch.rand(B, 9, 9, 64, generator=g) - 0.3).clamp(min=0).to(torch.bfloat16)
    y1 = (torch.rand(B, 20, 20, 32, generator=g) - 0.3).clamp(min=0).to(torch.bfloat16)
    R = B + 17 if idx else B
    obs = torch.randint(0, 256, (R, 4, 84, 84), dtype=torch.uint8, generator=g)
    oi = torch.randperm(R, generator=g)[:B] if idx else None
    dev = [t.to(cuda) for t in (dy3, W3, y2, W2, y1)]
    args = (dev[0].reshape(B * 49, 64), dev[1].reshape(64, 576), dev[2].reshape(B * 81, 64), dev[3].reshape(64, 512),
            dev[4].reshape(B * 400, 32))
    grid = min(persist, B)
    planes = torch.full((grid, 32, 256), float("nan"), device=cuda)
    res = []
    for fold in (False, True):
        dy2 = torch.full((B * 81, 64), float("nan"), dtype=torch.bfloat16, device=cuda)
        dy1 = torch.full((B * 400, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
        bp = torch.full((B, 160), float("nan"), device=cuda)
        if fold:
            ops.cnn_trunk_bwd(*args, dy2, dy1, bp, None, persist, obs.to(cuda), oi.to(cuda) if idx else None, planes,
                              1.0 / 255.0, True, True)
        else:
            ops.cnn_trunk_bwd(*args, dy2, dy1, bp, None, persist, None, None, None, 1.0, True)
        torch.cuda.synchronize()
        res.append((dy2.view(torch.int16).clone(), dy1.clone(), bp.clone()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][2][:grid], res[1][2][:grid])
    assert torch.isnan(res[1][1].float()).all(), "skip_dy1: dy1 must not be written"
    d1 = res[0][1].cpu().double().view(B, 400, 32)
    fr = obs[oi] if idx else obs
    cols = F.unfold(fr.double(), 8, stride=4)
    per = torch.einsum("bpo,bcp->boc", d1, cols) / 255.0                # [B, 32, 256]
    ref = torch.stack([per[w::grid].sum(0) for w in range(grid)])
    got = planes.cpu().double()
    err = float((got - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err
