"""CPU oracle tests against the reference behaviour spec."""
import math

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from actor_critic_algs_on_tensorflow_amd.envs import rng
from actor_critic_algs_on_tensorflow_amd.models import init as I
from actor_critic_algs_on_tensorflow_amd.models.mlp import MLPActor, MLPCritic
from actor_critic_algs_on_tensorflow_amd.ops import distributions as D
from actor_critic_algs_on_tensorflow_amd.ops import returns as R
from actor_critic_algs_on_tensorflow_amd.utils import framer as F
from actor_critic_algs_on_tensorflow_amd.utils import logger as LG
from actor_critic_algs_on_tensorflow_amd.utils import schedule as S
from actor_critic_algs_on_tensorflow_amd.utils import stats as ST


# ------------------------------------------------------------------------------------------------ Framer (A.2)
def test_framer_spec_example():
    fr = F.Framer(3)
    obs = [np.array([t, 10 + t]) for t in range(5)]
    full = fr.full(obs)
    assert len(full) == len(obs)
    assert list(full[0]) == [0, 10, 0, 10, 0, 10]
    assert list(full[3]) == [1, 11, 2, 12, 3, 13]
    assert list(fr.last(obs)) == [2, 12, 3, 13, 4, 14]
    assert list(fr.last(obs[:1])) == [0, 10, 0, 10, 0, 10]
    assert np.array_equal(np.stack(full), fr.full_array(np.stack(obs)))


def test_framestack_reset_and_push():
    fs = F.FrameStack(2, 3, (2,), torch.float32, "cpu")
    f0 = torch.tensor([[1.0, 2.0], [3.0, 4.0]])
    fs.reset(f0)
    assert torch.equal(fs.buf[0], f0[0].expand(3, 2))
    f1 = torch.tensor([[5.0, 6.0], [7.0, 8.0]])
    fs.push(f1, reset_mask=torch.tensor([False, True]))
    assert torch.equal(fs.buf[0, -1], f1[0]) and torch.equal(fs.buf[0, 0], f0[0])
    assert torch.equal(fs.buf[1], f1[1].expand(3, 2))


# ------------------------------------------------------------------------------------------------ PathAdv (A.3)
def _closed_form(r, v, terminal, g, L):
    T = len(r)
    tgt = np.zeros(T)
    for i in range(T):
        h = min(i + L, T)
        tgt[i] = sum(g ** (k - i) * r[k] for k in range(i, h))
        if not (terminal and h == T):
            tgt[i] += g ** (h - i) * v[h]
    return tgt, tgt - np.asarray(v[:T])


@pytest.mark.parametrize("T,L,term", [(10, 4, False), (10, 4, True), (3, 40, True), (50, 40, False), (200, 40, True)])
def test_pathadv_closed_form(T, L, term):
    g = np.random.default_rng(T + L)
    r, v = g.normal(size=T), g.normal(size=T + 1)
    tgt, adv = R.PathAdv(0.98, L)(r, v, term)
    et, ea = _closed_form(r, v, term, 0.98, L)
    assert np.allclose(tgt, et) and np.allclose(adv, ea)


@settings(max_examples=40, deadline=None)
@given(T=st.integers(1, 60), L=st.integers(1, 70), term=st.booleans(), seed=st.integers(0, 10 ** 6))
def test_nstep_tensor_matches_pathadv(T, L, term, seed):
    """The [T, N] n-step estimator reproduces PathAdv on a single episode column."""
    g = np.random.default_rng(seed)
    r, v = g.normal(size=T), g.normal(size=T + 1)
    d = np.zeros(T, dtype=np.uint8)
    d[-1] = term
    tgt, adv = R.nstep_returns_ref(torch.tensor(r).view(T, 1).float(), torch.tensor(v).view(T + 1, 1).float(),
                                   torch.tensor(d).view(T, 1), 0.98, L)
    et, ea = R.path_adv(r, v, term, 0.98, L)
    assert np.allclose(tgt[:, 0].numpy(), et, atol=1e-4) and np.allclose(adv[:, 0].numpy(), ea, atol=1e-4)


def test_nstep_episode_boundaries_and_gae():
    T, N = 6, 2
    r = torch.ones(T, N)
    v = torch.zeros(T + 1, N) + 10.0
    d = torch.zeros(T, N, dtype=torch.uint8)
    d[2, 0] = 1
    tgt, _ = R.nstep_returns_ref(r, v, d, 0.5, T)
    # env 0: t=0 window stops at the terminal at t=2 -> 1 + .5 + .25, no bootstrap
    assert abs(tgt[0, 0] - 1.75) < 1e-6
    # t=3 starts a new episode: 1 + .5 + .25 + bootstrap .125 * 10
    assert abs(tgt[3, 0] - (1.75 + 1.25)) < 1e-6
    ret, adv = R.gae_ref(r, v, d, 0.9, 1.0)
    # lambda = 1 GAE == full discounted return with bootstrap
    t2, _ = R.nstep_returns_ref(r, v, d, 0.9, T)
    assert torch.allclose(ret, t2, atol=1e-5)
    ret0, _ = R.gae_ref(r, v, d, 0.9, 0.0)
    assert torch.allclose(ret0[0, 1], torch.tensor(1.0 + 0.9 * 10.0))


def test_normalize_population_std():
    a = torch.tensor([1.0, 2.0, 3.0, 6.0])
    n = R.normalize_advantages(a)
    ref = (a.numpy() - a.numpy().mean()) / (1e-8 + a.numpy().std())
    assert np.allclose(n.numpy(), ref)


# ------------------------------------------------------------------------------------------------ schedules (A.1)
def test_linear_schedule():
    s = S.LinearSchedule(100, 3000, -2, -8, 100)
    assert s.val(0) == -2 and s.val(99) == -2 and s.val(3001) == -8
    assert math.isclose(s.val(1550), -5.0)
    assert s.update_time(0) and s.update_time(200) and not s.update_time(150)
    r = S.RegularizerSchedule()
    assert math.isclose(r.entropy_coef(0), 1e-2) and r.entropy_coef(1) is None
    assert math.isclose(r.kl_coef(3000), 1e-4) and math.isclose(r.entropy_coef(3100), 1e-8)


def test_kl_adaptive_lr_host_and_device():
    c = S.KLAdaptiveLR(0.002, 1e-6, 1.0)
    assert math.isclose(c(0.01, 0.0001), 0.015)
    assert math.isclose(c(0.01, 0.01), 0.01 / 1.5)
    assert c(0.01, 0.002) == 0.01
    assert c(0.9, 0.0) == 1.0 and c(1e-6, 1.0) == 1e-6
    d = S.DeviceKLAdaptiveLR(0.002, 1e-6, 0.1)
    lr = torch.tensor(0.08)
    d.update_(lr, torch.tensor(0.0))
    assert math.isclose(float(lr), 0.1, rel_tol=1e-6)
    d.update_(lr, torch.tensor(1.0))
    assert math.isclose(float(lr), 0.1 / 1.5, rel_tol=1e-6)


# ------------------------------------------------------------------------------------------------ logger (A.6)
def test_logger_format_and_legacy_index(tmp_path, capsys):
    for legacy in (False, True):
        p = tmp_path / f"log{legacy}.txt"
        lg = LG.Logger(str(p), legacy_step_index=legacy)
        for flush in range(3):
            for i in range(2):
                lg(i, act_loss=0.5, circ_loss=1.25, kl_dist=0.001, avg_rew=-3.0, print_tog=(i == 0), act_lr=0.005,
                   avg_ent=1.4, ev_before=0.1, ev_after=0.2)
            lg.flush()
        lg.close()
        lines = p.read_text().splitlines()
        assert lines[0] == "step avg_rew ev_before ev_after act_loss crit_loss kl_dist avg_ent"
        assert lines[1] == "0 -3.0000 0.1000  0.2000 0.5000  1.2500 0.0010 1.4000"
        steps = [int(x.split()[0]) for x in lines[1:]]
        # bug #8 (Basic_AC/util.py:106): last_write = +n -> the third flush restarts at 2 instead of 4
        assert steps == ([0, 1, 2, 3, 2, 3] if legacy else [0, 1, 2, 3, 4, 5])
    out = capsys.readouterr().out
    assert "Iteration 0" in out and "EpRewMean -3.0000" in out and "Performed by worker 0" in out


# ------------------------------------------------------------------------------------------------ stats / init
def test_var_accounted_for():
    g = np.random.default_rng(0)
    x = g.normal(size=500)
    y = 2 * x + g.normal(size=500) * 0.1
    assert abs(ST.var_accounted_for(x, y) - np.corrcoef(x, y)[0, 1]) < 1e-9
    assert abs(float(ST.var_accounted_for_tensor(torch.tensor(x), torch.tensor(y))) - np.corrcoef(x, y)[0, 1]) < 1e-5


def test_initialisers():
    g = torch.Generator().manual_seed(0)
    w = torch.empty(300, 200)
    I.xavier_uniform_(w, generator=g)
    lim = math.sqrt(6 / 500)
    assert w.abs().max() <= lim and w.abs().max() > 0.95 * lim
    I.scaled_xavier_(w, 0.1, generator=g)
    assert w.abs().max() <= 0.1 * lim
    I.normalized_column_(w, 0.1, generator=g)
    assert torch.allclose(w.norm(dim=0), torch.full((200,), 0.1), atol=1e-5)
    I.orthogonal_(w, 2.0, generator=g)
    assert torch.allclose(w.t() @ w, 4 * torch.eye(200), atol=1e-4)


def test_reference_param_counts():
    a = MLPActor(3, 1, discrete=False, ac_scale=2.0, variant="a3c")
    c = MLPCritic(3, variant="a3c")
    assert sum(p.numel() for p in a.parameters()) == 25346
    assert sum(p.numel() for p in c.parameters()) == 50561


def test_lrelu():
    from actor_critic_algs_on_tensorflow_amd.models.layers import lrelu
    x = torch.tensor([-1.0, 2.0])
    assert torch.allclose(lrelu(x), torch.tensor([-0.2, 2.0]))


def test_basic_critic_dead_layer_and_a3c_third_layer():
    x = torch.randn(4, 3)
    cb = MLPCritic(3, variant="basic")
    with torch.no_grad():
        v0 = cb(x)
        cb.third_layer.kernel.add_(1.0)
        assert torch.equal(cb(x), v0)   # bug #4: value reads the second layer
    ca = MLPCritic(3, variant="a3c")
    with torch.no_grad():
        v0 = ca(x)
        ca.third_layer.kernel.add_(1.0)
        assert not torch.equal(ca(x), v0)


# ------------------------------------------------------------------------------------------------ RNG + heads
def test_hash_vectors_pinned():
    # identical to csrc/kernels/common.h; GPU tests compare the kernels against these oracles
    assert rng.hash_u32_py(0, 0, 0, 0) == 1106484830
    assert rng.hash_u32_py(12321, 5, 77, 3) == 4030581239
    assert rng.hash_u32_py(0xFFFFFFFF, 123456, 2 ** 31, 200) == 3159308600
    assert int(rng.hash_u32(12321, torch.tensor([5]), torch.tensor([77]), 3)) == 4030581239


def test_heads_match_torch_distributions():
    logits = torch.randn(50, 6)
    a = torch.randint(0, 6, (50,))
    lp, ent = D.categorical_logp_entropy(logits, a)
    cd = torch.distributions.Categorical(logits=logits)
    assert torch.allclose(lp, cd.log_prob(a), atol=1e-5) and torch.allclose(ent, cd.entropy(), atol=1e-5)
    mu = torch.randn(50, 3)
    ls = torch.tensor([0.2, -3.0, 3.1])
    act = torch.randn(50, 3)
    lp, ent = D.gaussian_logp_entropy(mu, ls, act)
    nd = torch.distributions.Normal(mu, torch.exp(ls.clamp(-2.5, 2.5)))
    assert torch.allclose(lp, nd.log_prob(act).sum(1), atol=1e-4)
    assert torch.allclose(ent, nd.entropy().sum(1), atol=1e-5)


def test_sampling_distributions():
    keys = torch.arange(100000, dtype=torch.int64)
    lg = torch.tensor([[0.0, 1.0, -1.0]]).repeat(100000, 1)
    a, _, _ = D.categorical_sample_ref(lg, keys, 7)
    f = torch.bincount(a.long(), minlength=3).float() / 1e5
    assert torch.allclose(f, torch.softmax(lg[0], 0), atol=6e-3)
    mu = torch.zeros(100000, 1)
    act, _, _ = D.gaussian_sample_ref(mu, torch.tensor([math.log(2.0)]), keys, 7)
    assert abs(act.mean()) < 0.03 and abs(act.std() - 2.0) < 0.03


def test_reference_helper_names():
    """C13/C14 helpers under their reference names: lrelu, xav/xavier bounds, column-normalised init, fancy_clip."""
    import torch
    from actor_critic_algs_on_tensorflow_amd.compat import reference as R
    x = torch.tensor([-2.0, 0.0, 3.0])
    assert torch.allclose(R.lrelu(x), torch.tensor([-0.4, 0.0, 3.0]))
    assert R.ID_FN(x) is x and R.SCALE == 0.1
    g = torch.Generator().manual_seed(0)
    w = R.xavier((64, 128), generator=g)
    lim = (6.0 / (64 + 128)) ** 0.5
    assert w.abs().max() <= lim and w.abs().max() > 0.9 * lim
    assert R.xav((64, 128), generator=g).abs().max() <= 0.1 * lim
    c = R.normalized_column_initializer(0.1)((32, 8), generator=g)
    assert torch.allclose(c.norm(dim=0), torch.full((8,), 0.1), atol=1e-6)
    assert R.fancy_clip(None, -1, 1) is None
    assert torch.equal(R.fancy_clip(torch.tensor([-3.0, 0.5, 2.0]), -1.0, 1.0), torch.tensor([-1.0, 0.5, 1.0]))
