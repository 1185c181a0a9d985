"""Synthetic env banks: gym dynamics, time limits, auto-reset, frame stacking, episode statistics (CPU oracles)."""
import math

import numpy as np
import pytest
import torch

from actor_critic_algs_on_tensorflow_amd import envs as E
from actor_critic_algs_on_tensorflow_amd.compat.reference import GymEnv


def test_registry_and_roll_params():
    assert E.get_roll_params("Pendulum-v0", "basic") == (400, 1400)
    assert E.get_roll_params("Pendulum-v0", "a3c") == (200, 1200)
    assert E.get_roll_params("CartPole-v0", "basic") == (200, 800)
    assert E.get_roll_params("CartPole-v1", "a3c") == (500, 3000)
    with pytest.raises(KeyError):
        E.make("NoSuchEnv-v0")


def test_cartpole_matches_gym_equations():
    env = E.make("CartPole-v1", 1, seed=1)
    env.reset()
    s = env.state[0].double().numpy().copy()
    env.step(torch.tensor([1], dtype=torch.int32), prev_obs=env.obs.clone())
    x, xd, th, thd = s
    g, mc, mp, l, f, tau = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
    tm, pml = mc + mp, mp * l
    temp = (f + pml * thd ** 2 * math.sin(th)) / tm
    tha = (g * math.sin(th) - math.cos(th) * temp) / (l * (4 / 3 - mp * math.cos(th) ** 2 / tm))
    xa = temp - pml * tha * math.cos(th) / tm
    exp = [x + tau * xd, xd + tau * xa, th + tau * thd, thd + tau * tha]
    assert np.allclose(env.state[0].numpy(), exp, atol=1e-6)
    assert env.reward[0] == 1.0


def test_pendulum_matches_gym_equations():
    env = E.make("Pendulum-v0", 1, seed=2)
    env.reset()
    th, thd = env.state[0].double().numpy()
    u = 1.3
    env.step(torch.tensor([[u]]), prev_obs=env.obs.clone())
    an = ((th + math.pi) % (2 * math.pi)) - math.pi
    cost = an ** 2 + 0.1 * thd ** 2 + 0.001 * u ** 2
    nthd = thd + (-3 * 10 / 2 * math.sin(th + math.pi) + 3.0 * u) * 0.05
    nth = th + nthd * 0.05
    assert abs(env.reward[0] + cost) < 1e-5
    assert np.allclose(env.state[0].numpy(), [nth, np.clip(nthd, -8, 8)], atol=1e-5)
    assert np.allclose(env.obs[0].numpy(), [math.cos(nth), math.sin(nth), nthd], atol=1e-5)


@pytest.mark.parametrize("env_id,limit", [("Pendulum-v0", 200), ("CartPole-v0", 200), ("CartPole-v1", 500)])
def test_time_limits_and_autoreset(env_id, limit):
    env = E.make(env_id, 3, seed=0)
    env.reset()
    lengths = []
    t = torch.zeros(3, dtype=torch.int64)
    for _ in range(limit + 5):
        a = torch.zeros(3, dtype=torch.int32) if env.is_discrete else torch.zeros(3, 1)
        _, _, d, info = env.step(a, prev_obs=env.obs.clone())
        t += 1
        for i in range(3):
            if d[i]:
                lengths.append(int(t[i]))
                t[i] = 0
    assert all(1 <= L <= limit for L in lengths)
    if env_id.startswith("Pendulum"):
        assert lengths[:3] == [limit] * 3
    s = env.ep_stats
    assert int(s[1]) == len(lengths) and abs(float(s[2]) - sum(lengths)) < 1e-3


def test_frame_stack_vector():
    env = E.make("CartPole-v1", 2, seed=0, frame_stack=3)
    o0 = env.reset().clone()
    assert o0.shape == (2, 12) and torch.equal(o0[:, 0:4], o0[:, 8:12])
    o1, _, d, _ = env.step(torch.ones(2, dtype=torch.int32), prev_obs=o0)
    assert torch.equal(o1[:, 0:8], o0[:, 4:12])
    assert torch.allclose(o1[:, 8:12], env.state)


def test_pong_frames_and_rewards():
    env = E.make("PongNoFrameskip-v4", 4, seed=0)
    o = env.reset().clone()
    assert o.shape == (4, 4, 84, 84) and o.dtype == torch.uint8
    assert torch.equal(o[:, 0], o[:, 3])
    assert (o[0, 0, 0] == 236).all() and (o[0, 0, 40, 20] == 87)
    rews, dones = [], []
    prev = o
    for t in range(600):
        out, r, d, _ = env.step(torch.zeros(4, dtype=torch.int32), prev_obs=prev)
        if t == 0:
            assert torch.equal(out[:, :3], o[:, 1:]) or d.any()
        prev = out.clone()
        rews.append(r.clone())
        dones.append(d.clone())
    rr = torch.stack(rews)
    assert set(rr.unique().tolist()) <= {-1.0, 0.0, 1.0} and (rr != 0).any()


def test_mujoco_shape_env():
    env = E.make("HalfCheetahShape-v0", 2, seed=0)
    o = env.reset()
    assert o.shape == (2, 17) and env.action_space.shape == (6,)
    _, r, d, _ = env.step(torch.zeros(2, 6), prev_obs=o.clone())
    assert r.shape == (2,) and not d.any()


def test_env_partitioning_is_rank_invariant():
    """Counter-based RNG keyed by global env id: a 2-rank split reproduces the 1-rank bank (DP invariance)."""
    full = E.make("CartPole-v1", 4, seed=9)
    a = E.make("CartPole-v1", 2, seed=9, env_offset=0)
    b = E.make("CartPole-v1", 2, seed=9, env_offset=2)
    for e in (full, a, b):
        e.reset()
    assert torch.equal(full.state[:2], a.state) and torch.equal(full.state[2:], b.state)


def test_gym_adapter_terminal_obs():
    env = GymEnv("CartPole-v1", seed=0)
    ob = env.reset()
    done, n = False, 0
    while not done:
        ob2, r, done, _ = env.step(1)
        n += 1
    assert n < 100 and abs(ob2[2]) > 0.2   # pushed right until the pole falls: terminal angle > 12 degrees
