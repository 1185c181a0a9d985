"""Reference-semantics regressions on CPU: env time limits vs the rollout bound, time-limit bootstrapping, and the
order of the regulariser schedules (Basic_AC/run_AC.py:95,130-131,268-275)."""
import numpy as np
import torch

from actor_critic_algs_on_tensorflow_amd import envs as E
from actor_critic_algs_on_tensorflow_amd import preset
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
from actor_critic_algs_on_tensorflow_amd.ops import returns as R


def _quiet(**kw):
    base = dict(outdir=None, quiet=True, stdout_freq=0, save_every=0)
    base.update(kw)
    return base


def test_basic_pendulum_batch_is_seven_200_step_episodes():
    """Basic_AC's Pendulum max_path_length 400 only bounds the rollout loop; gym's TimeLimit still ends every
    episode at 200, so one iteration collects MAX_ROLLS = 7 episodes of 200 steps (1400 < EP_LENGTH_STOP ends it
    at the 7th roll, not earlier)."""
    from actor_critic_algs_on_tensorflow_amd.algos.basic_ac import BasicACTrainer
    tr = BasicACTrainer(preset("basic_ac", **_quiet()))
    assert tr.max_path_length == 400 and tr.ep_length_stop == 1400
    assert tr.env.spec.max_episode_steps == 200
    s = tr.step()
    assert s["episodes"] == 7 and tr.env_steps == 7 * 200


def test_reference_get_roll_params_keeps_env_time_limit():
    from actor_critic_algs_on_tensorflow_amd.compat import reference as ref
    env, mpl, stop = ref.get_roll_params("Pendulum-v0", "basic")
    assert (mpl, stop) == (400, 1400) and env.spec.max_episode_steps == 200
    env.reset()
    n = 0
    done = False
    while not done:
        _, _, done, _ = env.step(np.zeros(1, dtype=np.float32))
        n += 1
    assert n == 200


def test_bootstrap_on_timeout_cuts_episode_and_bootstraps_terminal_value():
    """Time limit (3) shorter than the rollout (T = 7): the truncated step keeps done = 1 (no reward or value of the
    next episode leaks into its target) and its reward carries gamma * V(terminal observation)."""
    gamma = 0.9
    env = E.make("Pendulum-v0", 2, seed=5, max_episode_steps=3)
    cfg = preset("basic_ac", **_quiet(algo="a2c", num_envs=2, n_steps=7, gamma=gamma, look_ahead=None,
                                      returns="nstep", bootstrap_on_timeout=True, norm_adv=False,
                                      kl_adaptive_lr=False, anneal_regularizers=False))
    tr = ActorCriticTrainer(cfg, env=env)
    st = tr.storage
    tr.collect()
    # replay the same actions on a twin bank that keeps the terminal observations
    twin = E.make("Pendulum-v0", 2, seed=5, max_episode_steps=3)
    twin.keep_final_obs = True
    twin.reset()
    raw = torch.zeros(7, 2)
    with torch.no_grad():
        for t in range(7):
            prev = twin.obs.clone()
            _, r, d, info = twin.step(st.actions[t], prev_obs=prev)
            raw[t] = r
            boot = gamma * tr.model.value(twin.final_obs) * info["truncated"].float()
            assert torch.equal(d, st.dones[t])
            assert torch.allclose(st.rewards[t], r + boot, atol=1e-6)
    assert st.truncated[2].all() and st.dones[2].all() and st.truncated[5].all()
    ret, adv = tr.compute_returns()
    ret = ret.view(7, 2)
    # target of the truncated step = its (bootstrapped) reward only: nothing from the next episode
    assert torch.allclose(ret[2], st.rewards[2], atol=1e-6)
    assert torch.allclose(ret[1], st.rewards[1] + gamma * st.rewards[2], atol=1e-5)
    ref_ret, _ = R.nstep_returns(st.rewards, st.values, st.dones, gamma, None)
    assert torch.allclose(ret, ref_ret, atol=1e-6)


def test_regularizer_schedule_applies_after_the_update():
    cfg = preset("basic_ac", **_quiet(algo="a2c", env="CartPole-v0", n_steps=4, num_envs=2, ent_coef=0.05,
                                      kl_coef=0.5, anneal_regularizers=True))
    tr = ActorCriticTrainer(cfg)
    assert abs(float(tr.ent_coef) - 0.05) < 1e-7 and abs(float(tr.kl_coef) - 0.5) < 1e-7
    seen = []
    orig = tr.update_body

    def body():
        seen.append((float(tr.ent_coef), float(tr.kl_coef)))
        orig()
    tr.update_body = body
    tr.step()
    tr.step()
    assert np.allclose(seen[0], (0.05, 0.5))             # iteration 0 runs with the configured coefficients
    assert abs(seen[1][0] - 1e-2) < 1e-9 and abs(seen[1][1] - 1.0) < 1e-9   # the i = 0 schedule acts from i = 1
