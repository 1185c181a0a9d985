"""Reference-shaped API (``Basic_AC/policies.py``, ``Basic_AC/run_AC.py``, ``A3C/policies.py``, ``A3C/process.py``)
on this framework's modules, so code written against the TensorFlow reference ports 1:1 (``sess`` arguments are
accepted and ignored).

* :class:`Actor`  -- ``act`` / ``optimize`` / ``get_kl`` / ``set_opt_param`` / ``get_opt_param`` / ``printoo`` /
  ``sync_w_global`` (``Basic_AC/policies.py:33-120``; A3C variant ``A3C/policies.py:34-134``).
* :class:`Critic` -- ``value`` / ``optimize`` / ``set_opt_param`` (a no-op, as in the reference: bug #6 of
  SURVEY §2.9) / ``printoo`` / ``sync_w_global`` (``Basic_AC/policies.py:123-162``).
* :func:`process_fn` -- one PS / worker process of the async job (``A3C/process.py:156-158`` signature).
* :func:`rollout`, :func:`train_ciritic`, :func:`train_actor`, :func:`get_roll_params`, :func:`test_process`,
  :class:`GymEnv` (a one-env gym-style adapter over the env bank), plus re-exports of ``Framer``, ``PathAdv``,
  ``LinearSchedule``, ``Logger``, ``var_accounted_for``, ``make_np``.

Each Actor/Critic owns its parameters in a flat fp32 slab with a fused TF-semantics Adam (element-wise clip +-1
Basic / +-0.1 A3C on the actor, none on the critic), i.e. the same optimiser kernels as the vectorised trainers.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import envs as E
from ..models.mlp import MLPActor, MLPCritic
from ..ops import distributions as D
from ..ops.optim import FlatParams, FusedAdam
from ..ops.returns import PathAdv
from ..utils.framer import Framer
from ..utils.logger import Logger
from ..utils.schedule import LinearSchedule
from ..utils.stats import make_np, var_accounted_for


class GymEnv:
    """gym-style single env (``reset() -> ob``, ``step(ac) -> (ob, rew, done, info)``) over a 1-env bank.

    ``done`` includes time-limit truncation, exactly like gym's TimeLimit wrapper the reference relies on
    (SURVEY §2.9 item 3).
    """

    def __init__(self, env_id, seed=0, max_episode_steps=None):
        self.bank = E.make(env_id, 1, device="cpu", seed=seed, max_episode_steps=max_episode_steps)
        self.bank.keep_final_obs = True
        self.env_id = env_id
        self.observation_space = self.bank.observation_space
        self.action_space = self.bank.action_space
        self.spec = self.bank.spec
        self._done = True

    def seed(self, s):
        self.bank.seed = int(s) & 0xFFFFFFFF

    def reset(self):
        self._done = False
        return self.bank.reset()[0].numpy().copy()

    def step(self, ac):
        if self.bank.is_discrete:
            a = torch.as_tensor(np.asarray(ac), dtype=torch.int32).reshape(1)
        else:
            a = torch.as_tensor(np.asarray(ac, dtype=np.float32)).reshape(1, -1)
        prev = self.bank.obs.clone()
        ob, r, d, info = self.bank.step(a, prev_obs=prev)
        done = bool(d[0])
        if done:
            ob = self.bank.final_obs  # the bank auto-resets; a gym env returns the terminal observation
        return ob[0].numpy().copy(), float(r[0]), done, {}

    def render(self, mode="human"):
        return None


def get_roll_params(env_id, variant="basic", seed=0):
    """-> (env, max_path_length, ep_length_stop) (``Basic_AC/run_AC.py:124-136``, ``A3C/process.py:100-109``)."""
    mpl, stop = E.get_roll_params(env_id, variant)
    env = GymEnv(env_id, seed=seed)   # env time limit kept; mpl only bounds the rollout loop
    print('\nMAX PATH LENGTH, EP LENGTH STEP: {}, {}\n'.format(mpl, stop))
    return env, mpl, stop


def _clip_scale(action_space):
    return np.maximum(action_space.high, np.abs(action_space.low))


class Actor:
    def __init__(self, num_ob_feat, ac_dim=None, act_type="cont", init_lr=0.005, init_beta=1.0, init_gamma=0.01,
                 ac_scale=2.0, variant="basic", name=None, num_ac=None, global_actor=None, seed=0, device="cpu"):
        ac_dim = ac_dim if ac_dim is not None else num_ac
        self.variant = variant
        self.discrete = act_type != "cont"
        g = torch.Generator().manual_seed(seed)
        self.net = MLPActor(num_ob_feat, ac_dim, self.discrete, ac_scale if ac_scale is not None else 1.0, variant,
                            generator=g).to(device)
        self.flat = FlatParams({"actor": list(self.net.parameters())}, torch.device(device))
        clip = 1.0 if variant == "basic" else 0.1   # Basic_AC/policies.py:81 / A3C/policies.py:85
        self.adam = FusedAdam(self.flat, "actor", init_lr, clip_value=clip)
        self.beta = float(init_beta)
        self.gamma = float(init_gamma)
        self.global_actor = global_actor
        self.name = name
        self._ctr = 0
        self.seed = seed

    # -- acting ---------------------------------------------------------------------------------------------
    @torch.no_grad()
    def act(self, ob, sess=None):
        ob = np.array(ob, dtype=np.float32)
        if ob.ndim != 2:
            ob = ob[None]
        o = torch.as_tensor(ob, device=self.flat.data.device)
        pi = self.net(o)
        keys = torch.arange(o.shape[0], dtype=torch.int64, device=o.device) + (self._ctr << 20)
        self._ctr += 1
        if self.discrete:
            a, logp, ent = D.categorical_sample(pi, keys, self.seed)
        else:
            a, logp, ent = D.gaussian_sample(pi, self.net.log_std, keys, self.seed)
        return a[0].cpu().numpy(), float(logp[0]), float(ent[0])

    def _logp(self, obs, acs):
        o = torch.as_tensor(np.asarray(obs, dtype=np.float32), device=self.flat.data.device)
        pi = self.net(o)
        if self.discrete:
            a = torch.as_tensor(np.asarray(acs), device=o.device).long().view(-1)
            return D.categorical_logp_entropy(pi, a)
        a = torch.as_tensor(np.asarray(acs, dtype=np.float32), device=o.device).view(pi.shape)
        return D.gaussian_logp_entropy(pi, self.net.log_std, a)

    # -- learning -------------------------------------------------------------------------------------------
    def loss(self, acs, obs, advs, logps):
        logp, ent = self._logp(obs, acs)
        adv = torch.as_tensor(np.asarray(advs, dtype=np.float32), device=logp.device).view(-1)
        lpo = torch.as_tensor(np.asarray(logps, dtype=np.float32), device=logp.device).view(-1)
        return -(adv * logp).mean() + self.beta * ((lpo - logp) ** 2).mean() - self.gamma * ent.mean()

    def compute_grads(self, acs, obs, advs, logps):
        self.flat.zero_grad()
        loss = self.loss(acs, obs, advs, logps)
        loss.backward()
        return float(loss.detach())

    def optimize(self, acs, obs, advs, logps, sess=None):
        loss = self.compute_grads(acs, obs, advs, logps)
        if self.global_actor is not None:
            # A3C: the local gradients (clipped +-0.1 in the global apply) update the global parameters
            self.global_actor.flat.grad.copy_(self.flat.grad)
            self.global_actor.adam.lr.copy_(self.adam.lr)
            self.global_actor.adam.step()
        else:
            self.adam.step()
        return loss, None

    @torch.no_grad()
    def get_kl(self, sess=None, logp_feeds=None, obs=None, acs=None):
        logp, _ = self._logp(obs, acs)
        lpo = torch.as_tensor(np.asarray(logp_feeds, dtype=np.float32), device=logp.device).view(-1)
        return float(((lpo - logp) ** 2).mean())

    def set_opt_param(self, sess=None, new_lr=None, new_beta=None, new_gamma=None):
        if new_lr is not None:
            self.adam.set_lr(new_lr)
        if new_beta is not None:
            self.beta = float(new_beta)
        if new_gamma is not None:
            self.gamma = float(new_gamma)
        return self.get_opt_param(sess)

    def get_opt_param(self, sess=None):
        return [self.adam.get_lr(), self.beta, self.gamma]

    @torch.no_grad()
    def printoo(self, obs, sess=None):
        o = torch.as_tensor(np.asarray(obs, dtype=np.float32), device=self.flat.data.device)
        x = self.net.first_layer(o)
        x1 = self.net.second_layer(x)
        mu = self.net(o)
        print("Actor layer data", float(x.mean()), float(x1.mean()), float(mu.mean()))
        print("Actor Variable data", [float(p.mean()) for p in self.net.parameters()])

    def sync_w_global(self, sess=None):
        if self.global_actor is not None:
            self.flat.data.copy_(self.global_actor.flat.data)


class Critic:
    def __init__(self, num_ob_feat, init_lr=0.001, ob_scale=1.0, variant="basic", name=None, global_critic=None,
                 seed=0, device="cpu"):
        g = torch.Generator().manual_seed(seed + 1)
        self.net = MLPCritic(num_ob_feat, variant=variant, ob_scale=ob_scale, generator=g).to(device)
        self.flat = FlatParams({"critic": list(self.net.parameters())}, torch.device(device))
        self.adam = FusedAdam(self.flat, "critic", init_lr)
        self.global_critic = global_critic

    @torch.no_grad()
    def value(self, obs, sess=None):
        o = torch.as_tensor(np.asarray(obs, dtype=np.float32), device=self.flat.data.device)
        return self.net(o).cpu().numpy()

    def compute_grads(self, obs, targets):
        self.flat.zero_grad()
        o = torch.as_tensor(np.asarray(obs, dtype=np.float32), device=self.flat.data.device)
        t = torch.as_tensor(np.asarray(targets, dtype=np.float32), device=o.device).view(-1)
        loss = ((self.net(o) - t) ** 2).mean()
        loss.backward()
        return float(loss.detach())

    def optimize(self, obs, targets, sess=None):
        loss = self.compute_grads(obs, targets)
        if self.global_critic is not None:
            self.global_critic.flat.grad.copy_(self.flat.grad)
            self.global_critic.adam.step()
        else:
            self.adam.step()
        return loss, None

    def set_opt_param(self, new_lr, sess=None):
        """Reference parity: ``sess.run(self.lr, feed_dict={self.lr: new_lr})`` only *reads* the variable
        (``Basic_AC/policies.py:158-159``), so the critic lr never changes. Returns the new value fed."""
        return new_lr

    @torch.no_grad()
    def printoo(self, obs, sess=None):
        o = torch.as_tensor(np.asarray(obs, dtype=np.float32), device=self.flat.data.device)
        x = torch.relu(self.net.first_layer(o))
        print("Critic data", float(x.mean()), float(self.net(o).mean()))

    def sync_w_global(self, sess=None):
        if self.global_critic is not None:
            self.flat.data.copy_(self.global_critic.flat.data)


def rollout(env, sess, policy, framer, max_path_length=100, render=False):
    """One episode (``Basic_AC/run_AC.py:82-107``): per step ``policy(framer.last(obs))`` then ``env.step``."""
    t = 0
    ob = env.reset()
    obs = [ob]
    logps, rews, acs = [], [], []
    sum_ents = 0.0
    done = False
    while t < max_path_length and not done:
        if render:
            env.render()
        t += 1
        ac, logp, ent = policy(framer.last(obs), sess=sess)
        ob, rew, done, _ = env.step(ac)
        obs.append(ob)
        rews.append(rew)
        acs.append(ac)
        sum_ents += ent
        logps.append(logp)
    return {"rews": rews, "obs": obs, "acs": acs, "terminated": done, "logps": logps, "entropy": sum_ents}


def train_ciritic(critic, sess, obs, targets):
    """Critic fit with EV before/after (``Basic_AC/run_AC.py:109-116``; the reference's spelling)."""
    assert len(obs) == len(targets)
    pre = critic.value(obs, sess=sess)
    ev_before = var_accounted_for(targets, pre)
    loss, _ = critic.optimize(obs=obs, targets=targets, sess=sess)
    post = critic.value(obs, sess=sess)
    ev_after = var_accounted_for(targets, post)
    return loss, ev_before, ev_after


train_critic = train_ciritic


def train_actor(actor, sess, obs, advs, logps, acs):
    assert len(obs) == len(advs)
    assert len(advs) == len(acs)
    loss, _ = actor.optimize(sess=sess, obs=obs, acs=acs, advs=advs, logps=logps)
    return loss


def make_actor_critic(env, frames=1, variant="basic", seed=0, device="cpu"):
    """Builds (Actor, Critic) for an env exactly as the reference mains do (``Basic_AC/run_AC.py:188-198``)."""
    ob_dim = env.observation_space.shape[0] * frames
    if isinstance(env.action_space, E.Discrete):
        act_type, ac_dim, ac_scale = "disc", env.action_space.n, None
    else:
        act_type, ac_dim, ac_scale = "cont", env.action_space.shape[0], _clip_scale(env.action_space)
    critic = Critic(ob_dim, variant=variant, seed=seed, device=device)   # built first, as in the reference
    actor = Actor(ob_dim, ac_dim, act_type, ac_scale=ac_scale, variant=variant, seed=seed, device=device)
    return actor, critic


def test_process(env_id, random_seed, stack_frames, model_path, num_episodes, animate=True):
    """``A3C/process.py:125-153`` / ``Basic_AC/run_AC.py:139-163``: restore a checkpoint and run episodes."""
    from ..api import evaluate
    return evaluate(model_path, env_id, num_episodes=num_episodes, seed=random_seed, frames=stack_frames,
                    animate=animate)


def process_fn(cluster, task_id, job, env_id, logger, save_path, stdout_freq, random_seed=12321, gamma=0.98,
               look_ahead=40, stack_frames=3, animate=False, save_every=600, desired_kl=0.002, TB_log=False,
               run_mode="train", checkpoint_basename="model", device="cpu", num_envs=16, n_steps=16,
               data_plane="gloo", max_staleness=-1, max_iters=int(1e7)):
    """``A3C/process.py:156-158``: one process of the async job, by (job, task_id) in the cluster dict
    ``{"ps": ["host:port", ...], "worker": [...]}``. All processes join one gloo group rendezvousing at the first
    PS address (PS tasks are ranks 0..P-1, workers P..). ``device="cpu"`` runs the reference-shaped episode
    workers (:mod:`..algos.a3c`); ``device="cuda[:K]"`` the GPU-native mode (:mod:`..algos.a3c_gpu`: vectorised
    device workers, device-resident PS shards, RCCL or gloo data plane). ``logger`` is the worker's Logger (None
    for PS tasks), ``save_path`` the checkpoint directory, ``checkpoint_basename`` the file prefix. Returns the
    role's summary dict (the reference returns nothing; a PS task returns when every worker has finished instead
    of joining forever)."""
    import datetime
    import os

    import torch.distributed as dist

    from ..config import preset
    num_ps, num_workers = len(cluster["ps"]), len(cluster["worker"])
    rank = task_id if job == "ps" else num_ps + task_id
    world = num_ps + num_workers
    host, port = cluster["ps"][0].rsplit(":", 1)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1" if host in ("localhost", "") else host)
    os.environ.setdefault("MASTER_PORT", port)
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
    cfg = preset("a3c", env=env_id, seed=random_seed, gamma=gamma, look_ahead=look_ahead, frames=stack_frames,
                 save_every=save_every, desired_kl=desired_kl, tboard=bool(TB_log), mode=run_mode,
                 checkpoint_dir=save_path, stdout_freq=stdout_freq, ps_num=num_ps, total_updates=int(max_iters))
    if str(device).startswith("cuda"):
        from ..algos import a3c_gpu
        cfg = cfg.replace(device=device, num_envs=num_envs, n_steps=n_steps, cuda_graph=True, outdir=None)
        # worker rows go to the caller's Logger, the chief writes checkpoints into save_path (A3C/process.py:211-214)
        return a3c_gpu.run(cfg, rank=rank, world=world, ps_num=num_ps, data_backend=data_plane,
                           max_staleness=max_staleness, device=device, logger=logger,
                           checkpoint_basename=checkpoint_basename)
    from ..algos import a3c
    return a3c.run(cfg, rank=rank, world=world, ps_num=num_ps, logger=logger, checkpoint_basename=checkpoint_basename)


# ---- reference helper names, as plain tensor functions -------------------------------------
SCALE = 0.1   # Basic_AC/policies.py:4


def ID_FN(x):   # Basic_AC/policies.py:5 -- identity observation scaler
    return x


def lrelu(x, alpha=0.2):   # Basic_AC/policies.py:28-31: (1 - a) relu(x) + a x
    from ..models.layers import lrelu as _lrelu
    return _lrelu(x, alpha)


def xavier(shape, generator=None):   # TF Xavier-uniform for a [in, out] kernel
    from ..models.init import xavier_uniform_
    return xavier_uniform_(torch.empty(*shape), generator=generator)


def xav(shape, generator=None):   # Basic_AC/policies.py:6-7: SCALE * Xavier-uniform
    from ..models.init import scaled_xavier_
    return scaled_xavier_(torch.empty(*shape), scale=SCALE, generator=generator)


def normalized_column_initializer(std=SCALE):   # A3C/policies.py:3-10: N(0,1) columns rescaled to L2 norm ``std``
    from ..models.init import normalized_column_

    def _init(shape, generator=None):
        return normalized_column_(torch.empty(*shape), norm=std, generator=generator)
    return _init


def fancy_clip(grad, clip_value_min, clip_value_max):   # Basic_AC/policies.py:23-26: clip that passes None through
    if grad is None:
        return None
    return torch.clamp(grad, clip_value_min, clip_value_max)


__all__ = ["Actor", "Critic", "GymEnv", "rollout", "train_ciritic", "train_critic", "train_actor", "get_roll_params",
           "test_process", "make_actor_critic", "Framer", "PathAdv", "LinearSchedule", "Logger",
           "var_accounted_for", "make_np", "SCALE", "ID_FN", "lrelu", "xavier", "xav",
           "normalized_column_initializer", "fancy_clip"]
