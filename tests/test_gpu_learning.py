"""The native GPU engines learn, at production shapes (the reference's correctness signal is
its training curve, Basic_AC/run_AC.py:277-280 / Basic_AC/util.py:64-106).

* native Pong A2C (bf16 CNN engine, the headline config, graph-captured): the fraction of points won rises from
  the random policy's level by a fixed margin within a bounded number of updates;
* CartPole on the fused MLP engine and on the torch/autograd engine: both reach the 500-step cap and stay there;
* MuJoCo-shape PPO on the MLP engine learns and holds >= 0.9 of its peak over the last third of 300 updates;
* engine-vs-autograd gradients at the production batch sizes (B = 160 A2C learner, B = 4096 PPO minibatch) with
  the autotuned GEMM plans.
Thresholds come from measured curves (scripts/learn_curve.py on an MI355X; profiles/r2_learning_curves.txt)."""
import pytest
import torch

from actor_critic_algs_on_tensorflow_amd import preset

pytestmark = pytest.mark.gpu


def _curve(name, updates, report, **kw):
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    base = dict(outdir=None, quiet=True, stdout_freq=0, save_every=0, seed=1)
    base.update(kw)
    tr = ActorCriticTrainer(preset(name, **base))
    if tr.cfg.cuda_graph:
        tr.capture(warmup=1)
    won = torch.zeros((), device=tr.device)
    lost = torch.zeros((), device=tr.device)
    rows = []
    for u in range(1, updates + 1):
        tr.step()
        r = tr.storage.rewards
        won += (r > 0).sum()
        lost += (r < 0).sum()
        if u % report == 0:
            w, l = float(won), float(lost)
            ret, n_ep, _ = tr.env.drain_episode_stats()
            rows.append(dict(u=u, win=w / max(w + l, 1.0), ret=ret, n_ep=n_ep))
            won.zero_()
            lost.zero_()
    return tr, rows


def test_native_pong_a2c_learns(cuda):
    tr, rows = _curve("pong_a2c", 24000, 2000)
    assert tr.engine is not None and tr.graph is not None
    first, last = rows[0]["win"], rows[-1]["win"]
    # measured: 0.08 -> 0.55 over 24k updates (3.8M env steps); random play wins ~8% of the points
    assert last > 0.35 and last > first + 0.2, rows


def test_cartpole_native_mlp_and_torch_engines_learn_alike(cuda):
    """A2C on CartPole-v1 (64 envs x 5 steps) reaches the 500-step cap and STAYS there on both engines. With the
    preset's lr (1e-3 actor / 5e-3 critic) the policy solves and collapses again (one seed fell to 9-step episodes,
    profiles/r3_learning_stability.txt); actor 3e-4 / critic 1e-3 with linear lr decay over the run stayed at 500 on
    all 3 measured seeds x 2 engines. Bar: the mean of the last 3 reports (the final 1200 updates) > 400."""
    finals = {}
    for eng in ("native", "torch"):
        tr, rows = _curve("cartpole_cpu", 4000, 400, device="cuda:0", num_envs=64, cuda_graph=True, engine=eng,
                          lr=3e-4, critic_lr=1e-3, lr_schedule="linear", total_updates=4000)
        assert (tr.mlp is not None) == (eng == "native")
        finals[eng] = sum(r["ret"] for r in rows[-3:]) / 3
        assert rows[0]["ret"] < 100 and finals[eng] > 400, (eng, rows)
    assert abs(finals["native"] - finals["torch"]) < 100, finals


def test_pendulum_ppo_solves_and_checkpoint_evaluates(cuda, tmp_path):
    """the framework solves the reference's flagship task. Pendulum-v0 swing-up with the
    reference A3C actor / critic on the native MLP engine (preset pendulum_ppo: gamma 0.98, PPO-clip, one 200-step
    episode per env per rollout): the mean finished-episode return rises from random play (about -1200) above -400
    -- the bar the reference's own shipped demo policy meets (tests/test_ckpt_cpu.py) -- within 100 updates (320k env
    steps); the trained policy is saved as a TF bundle under the reference names (global_actor/..., A3C/process.py's
    Saver) and the evaluation CLI (cli/test_model.py, README.md:33-37) scores it above -400 too."""
    import numpy as np
    from actor_critic_algs_on_tensorflow_amd import ckpt
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    from actor_critic_algs_on_tensorflow_amd.cli import test_model
    tr = ActorCriticTrainer(preset("pendulum_ppo", device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                                   save_every=0, seed=3))
    assert tr.mlp is not None and tr.cfg.model_variant == "a3c"
    tr.capture(warmup=1)
    rets = []
    for u in range(1, 101):
        tr.step()
        if u % 10 == 0:
            rets.append(tr.env.drain_episode_stats()[0])
    assert rets[0] < -600, rets               # random-level start (the first 10 updates)
    assert np.mean(rets[-3:]) > -400, rets    # solved: the demo checkpoint's bar
    path = tr.save_checkpoint(str(tmp_path / "model-Pendulum-ppo-100"))
    names = ckpt.load_tensors(path)
    assert "global_actor/mu_layer/kernel" in names and "global_critic/value/bias" in names
    rewards = test_model.main(["Pendulum-v0", path, "--num_episodes", "10", "--animate_not", "--seed", "77"])
    assert np.mean(rewards) > -400, rewards


def test_mujoco_ppo_mlp_engine_learns_and_does_not_decay(cuda):
    """MuJoCo-shape PPO on the MLP engine (64 envs x 256 steps, 10 epochs x 32 minibatches) over 300 updates, seeds 1
    and 2: the return rises from its start and the last third of the run holds >= 0.9 of the peak on average over the
    two seeds (>= 0.85 each). The preset's constant 3e-4 peaks near update 90 and then decays (462 -> 338 by update
    300, profiles/r2_learning_curves.txt); actor 1e-4 with linear lr decay holds: last third / peak 0.97-0.99 on 3
    seeds in round 3 (profiles/r3_learning_stability.txt), 0.89-0.98 on seeds 1-5 with the round-6 kernels (seeds 1
    and 5 at 0.89: fp32 summation order alone moves a seed across the band; profiles/r6_mujoco_learning_seeds.txt)."""
    ratios = []
    for seed in (1, 2):
        tr, rows = _curve("mujoco_ppo_dp8", 300, 30, lr=1e-4, critic_lr=1e-3, lr_schedule="linear", total_updates=300,
                          seed=seed)
        assert tr.mlp is not None
        rets = [r["ret"] for r in rows]
        peak = max(rets)
        assert peak > rets[0] + 150, rets
        last_third = rets[-(len(rets) // 3):]
        ratios.append(sum(last_third) / len(last_third) / peak)
        assert ratios[-1] >= 0.85, (seed, rets)
    assert sum(ratios) / len(ratios) >= 0.9, ratios


def test_breakout_ppo_learns_on_the_large_batch_kernels_and_tracks_torch(cuda):
    """BASELINE config 3 (Breakout-shape PPO: 128 envs x 128 steps, GAE 0.95, 4 epochs x 4 minibatches of 4096) with
    the default EngineOpts -- the per-env split fused rollout step, the large-batch head (ppo_head), gemm_big fc
    products and the persistent trunk backward, all asserted taken -- LEARNS: the fraction of points won rises from
    random play (~0.10) past 0.45 within 300 updates (4.9M env steps; measured 0.10 -> 0.77 / 0.63 on seeds 1 / 2),
    and the torch/autograd engine on the same seed follows it within a band at 200 updates (measured native 0.44 /
    torch 0.45 on seed 1, 0.26 / 0.28 on seed 2; profiles/r5_breakout_learning.txt)."""
    tr, rows = _curve("breakout_ppo", 300, 25, device="cuda:0", seed=1)
    eng = tr.engine
    assert eng is not None and tr.graph is not None
    mb = tr.cfg.num_envs * tr.cfg.n_steps // tr.cfg.ppo_minibatches
    assert eng.fused_env_step_ok(tr.cfg.num_envs) and eng.opts.fused_env_split
    assert eng.ppo_head_ok(mb) and eng.big_gemm_ok(mb) and mb >= eng.large_b
    win = [r["win"] for r in rows]
    assert win[0] < 0.15 and win[-1] > 0.45 and win[-1] > win[0] + 0.3, win
    trt, rows_t = _curve("breakout_ppo", 200, 25, device="cuda:0", seed=1, engine="torch")
    assert trt.engine is None
    win_t = [r["win"] for r in rows_t]
    assert win_t[-1] > win_t[0] + 0.15, win_t
    assert abs(win_t[-1] - win[7]) < 0.15, (win[7], win_t[-1])


@pytest.mark.parametrize("B,ppo", [(160, False), (4096, True)])
def test_cnn_engine_matches_autograd_at_production_batch(cuda, B, ppo):
    """Native forward + fused loss + backward (trunk rows / per-env trunk, fused data-gradient kernel, split-K
    plane weight gradients + finaliser, autotuned plans) vs fp32 autograd on the same bf16-rounded parameters."""
    from actor_critic_algs_on_tensorflow_amd.algos import losses as L
    from actor_critic_algs_on_tensorflow_amd.algos.engine import CNNEngine
    from actor_critic_algs_on_tensorflow_amd.models.policy import CNNActorCritic
    from actor_critic_algs_on_tensorflow_amd.ops import distributions as D
    from actor_critic_algs_on_tensorflow_amd.ops.optim import FlatParams
    A = 6
    g = torch.Generator().manual_seed(B)
    model = CNNActorCritic(A, generator=g).to(cuda)
    with torch.no_grad():
        model.net.heads.kernel.mul_(20)
        for m in (model.net.trunk.conv1, model.net.trunk.conv2, model.net.trunk.conv3):
            m.bias.uniform_(-0.05, 0.1)
    flat = FlatParams(model.param_groups(), cuda)
    shadow = flat.data.to(torch.bfloat16)
    eng = CNNEngine(model, flat, shadow)
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, generator=g).to(cuda)
    b = eng.bufs(B, with_grad=True)
    eng.forward(obs, b)
    ref = CNNActorCritic(A).to(cuda)
    with torch.no_grad():
        for pr, p in zip(ref.parameters(), model.parameters()):
            pr.copy_(p.to(torch.bfloat16).float())
    logits, v = ref(obs)
    act = torch.randint(0, A, (B,), dtype=torch.int32, generator=g).to(cuda)
    lpo = (D.categorical_logp_entropy(logits.detach(), act)[0] + 0.05 * torch.randn(B, generator=g).to(cuda))
    adv = torch.randn(B, generator=g).to(cuda)
    ret = torch.randn(B, generator=g).to(cuda)
    v_old = v.detach() + 0.1 * torch.randn(B, generator=g).to(cuda)
    ec, kc = torch.tensor(0.01, device=cuda), torch.tensor(0.0, device=cuda)
    flat.zero_grad()
    eng.loss(b, act, lpo, adv, ret, v_old if ppo else None, ec, kc, 0.5, 0.1 if ppo else 0.0, 0.0)
    eng.backward(b)
    torch.cuda.synchronize()
    logp, ent = D.categorical_logp_entropy(logits, act)
    if ppo:
        al, *_ = L.ppo_actor_loss(logp, lpo, adv, ent, 0.1, ec, kc)
    else:
        al, *_ = L.actor_loss(logp, lpo, adv, ent, 0.0, 0.01)
    (al + 0.5 * L.value_loss(v, ret)).backward()
    errs = {}
    for (name, p), pr in zip(model.named_parameters(), ref.parameters()):
        i = [id(q) for q in flat.params].index(id(p))
        off = flat.offsets[i]
        gn = flat.grad[off:off + p.numel()].view_as(p)
        errs[name] = float((gn - pr.grad).norm() / (pr.grad.norm() + 1e-12))
    print("relative gradient errors", B, errs)
    # bf16 operands, fp32 accumulation: measured max 1.28 % (B = 160, conv1) and 0.17 % (B = 4096) per parameter
    # (profiles/r5_breakout_learning.txt); the bars keep ~1.5-3x of headroom
    bar = 0.02 if B <= 256 else 0.005
    for name, err in errs.items():
        assert err < bar, (name, err, bar)


def test_default_headline_update_matches_fp32_torch_update(cuda):
    """Direct fp32 pin of the DEFAULT headline update (BASELINE config 2, pong_a2c, default EngineOpts, one captured
    graph replay: fused rollout steps -> per-env A2C head -> fc_bwd -> grouped conv weight gradients -> finaliser ->
    RMSprop with the 0.5 global-norm clip) against the reference semantics in fp32 (``Basic_AC/policies.py:72-82``:
    loss, clip, optimiser step) computed by the torch engine: the same rollout (observations, actions, rewards,
    dones of the replayed update), the same bf16-rounded parameters, the same optimiser state, n-step returns from
    fp32 values, autograd of the trainer's torch loss, FusedRMSprop's plain-torch step. Every parameter tensor's
    update must match: relative error ||dp_native - dp_torch|| / ||dp_torch|| below the bar (bf16 operands with
    fp32 accumulation in the native engine; measured 0.1 % (heads) .. 2.7 % (conv1 bias), so 5 % keeps ~1.9x)."""
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    from actor_critic_algs_on_tensorflow_amd.ops import returns as R
    kw = dict(device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0, seed=7)
    tr = ActorCriticTrainer(preset("pong_a2c", **kw))
    assert tr.engine is not None and tr.engine.opts == type(tr.engine.opts)()
    tr.capture(warmup=1)
    assert tr.graph is not None
    st = tr.storage
    T, N = st.T, tr.env.num_envs
    p0 = tr.flat.data.clone()
    v0 = {g: o.v.clone() for g, o in tr.opts.items()}
    phase0 = st.phase
    tr.step()
    torch.cuda.synchronize()
    d_nat = tr.flat.data - p0
    ph = st.phase
    st.phase = phase0   # the replayed rollout's observation slots
    obs = torch.stack([st.obs[t] for t in range(T + 1)]).clone()
    st.phase = ph
    act, rew, dn = st.actions.clone(), st.rewards.clone(), st.dones.clone()
    lpo = st.logp.clone()
    stats_nat = tr.stats_buf.clone()

    ref = ActorCriticTrainer(preset("pong_a2c", engine="torch", dtype="fp32", cuda_graph=False, **kw))
    assert ref.engine is None and ref.flat.data.numel() == p0.numel() and list(ref.opts) == list(tr.opts)
    pb = p0.to(torch.bfloat16).float()
    with torch.no_grad():
        ref.flat.data.copy_(pb)
        for g, o in ref.opts.items():
            o.v.copy_(v0[g])
            o.lr.copy_(tr.opts[g].lr)
        _, v_all = ref.model(obs.view((T + 1) * N, *obs.shape[2:]))
        ret, adv = R.nstep_returns_ref(rew, v_all.view(T + 1, N).float(), dn, tr.cfg.gamma, T)
    ref.flat.zero_grad()
    total, a_loss, c_loss, kl, ent, _ = ref._loss(obs[:T].reshape(T * N, *obs.shape[2:]), act.reshape(-1),
                                                  lpo.reshape(-1), adv.reshape(-1).float(), ret.reshape(-1).float())
    total.backward()
    for o in ref.opts.values():
        o._torch_step()
    torch.cuda.synchronize()
    d_ref = ref.flat.data - pb
    errs = {}
    for name, p in ref.model.named_parameters():
        i = [id(q) for q in ref.flat.params].index(id(p))
        off, n = ref.flat.offsets[i], p.numel()
        a, b = d_nat[off:off + n], d_ref[off:off + n]
        errs[name] = float((a - b).norm() / (b.norm() + 1e-20))
    print("relative update errors", errs)
    print("native stats", stats_nat[:8].tolist(), "torch", [float(a_loss), float(c_loss), float(ent)])
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import STAT_KEYS
    assert float(stats_nat[STAT_KEYS.index("entropy")]) == pytest.approx(float(ent), rel=2e-2)
    for name, err in errs.items():
        assert err < 0.05, (name, err)
