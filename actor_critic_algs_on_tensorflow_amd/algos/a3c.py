"""A3C-style asynchronous parameter-server training (``A3C/process.py:156-288``, ``A3C/train.py``).

Reference semantics: ``ps_num`` parameter-server tasks hold the global actor/critic (and
the shared Adam moment slots, because every worker's optimiser creates its slots under the same global names --
but each worker's own beta-power step count, kept per source rank on the PS); each of
``worker_num`` workers collects whole episodes with its LOCAL copy until >= ``ep_length_stop`` steps, computes
actor (clip +-0.1) and critic gradients locally, applies them to the GLOBAL variables with its own learning rate,
then copies the global variables back (``sync_w_global``). The actor apply increments ``global_step``; the chief
(worker 0) checkpoints every ``save_every`` global steps; training stops at ``total_updates`` global steps.

Transport: ``torch.distributed`` point-to-point with the gloo backend (TCP; the messages are a few hundred KB of
fp32 per update -- 296.5 KiB each way for Pendulum). A PS serves whichever worker's request arrives
first (``recv`` from any source), so applies are serialised: the reference's lock-free Hogwild races on the PS
variables cannot happen, while staleness stays bounded by the number of workers. Variables are
placed on PS tasks round-robin in creation order (critic first, then actor), the placement TF used
because ``greedy_ps_strategy`` returns ``None`` (``A3C/util.py:51-53``). Deviations from the reference, both
fixes: every worker pulls the global parameters before its first rollout (bug #12) and only rank 0 initialises
them (bug #11); PS processes exit once every worker has finished.

Rank layout: ranks ``0 .. ps_num-1`` are PS tasks, ranks ``ps_num .. ps_num+worker_num-1`` are workers 0..W-1.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.distributed as dist

from .. import ckpt as C
from ..compat import reference as ref
from ..ops.optim import FlatParams, FusedAdam
from ..utils.schedule import LinearSchedule

CMD_PULL, CMD_APPLY, CMD_DONE = 1, 2, 3
ACTOR_CLIP = 0.1   # A3C/policies.py:85


def _param_list(critic_net, actor_net):
    """(name, tensor) of trainable variables in TF creation order: global_critic first, then global_actor."""
    t = C.reference_tensors(actor_net, critic_net, "a3c")
    crit = [(k, p) for k, p in t.items() if k.startswith("global_critic/") and isinstance(p, torch.nn.Parameter)]
    act = [(k, p) for k, p in t.items() if k.startswith("global_actor/") and isinstance(p, torch.nn.Parameter)]
    return crit + act


class ShardMap:
    """Round-robin variable -> PS placement and the flat offsets of each shard."""

    def __init__(self, params, ps_num):
        self.ps_num = ps_num
        self.names = [k for k, _ in params]
        self.sizes = [p.numel() for _, p in params]
        self.is_actor = [k.startswith("global_actor/") for k in self.names]
        self.owner = [i % ps_num for i in range(len(params))]
        self.shard_vars = [[i for i in range(len(params)) if self.owner[i] == s] for s in range(ps_num)]
        self.shard_numel = [sum(self.sizes[i] for i in v) for v in self.shard_vars]


def _flatten(tensors, idx):
    return torch.cat([tensors[i].detach().reshape(-1) for i in idx]) if idx else torch.zeros(0)


def _unflatten_into(flat, tensors, idx):
    off = 0
    for i in idx:
        n = tensors[i].numel()
        tensors[i].data.copy_(flat[off:off + n].view_as(tensors[i]))
        off += n


# ------------------------------------------------------------------------------------------------ parameter server
class ParameterServer:
    """Holds one shard of the global variables + their (shared) Adam slots; serves pull/apply requests."""

    def __init__(self, shard, shard_id, init_values, worker_ranks, critic_lr):
        self.shard = shard
        self.sid = shard_id
        idx = shard.shard_vars[shard_id]
        self.idx = idx
        n = shard.shard_numel[shard_id]
        self.params = torch.nn.Parameter(init_values.clone() if n else torch.zeros(0))
        self.flat = FlatParams({"shard": [self.params]}, torch.device("cpu"))
        # separate Adam views for the actor variables (clipped) and the critic variables (unclipped) of the shard
        mask = torch.cat([torch.full((shard.sizes[i],), shard.is_actor[i], dtype=torch.bool) for i in idx]) \
            if idx else torch.zeros(0, dtype=torch.bool)
        self.actor_mask = mask
        self.adam = FusedAdam(self.flat, "shard", 1e-3)
        self.critic_lr = critic_lr
        self.global_step = 0
        self.workers = set(worker_ranks)
        self.worker_t = {}   # per-worker Adam step counts (bias correction)

    def apply(self, grad, actor_lr, src=None):
        """One worker's update: critic vars with the critic lr, actor vars clipped +-0.1 with the worker's lr.
        The moments are shared (one set of global slot variables), but the bias-correction step count is the
        sender's own: each reference worker builds its own Adam whose beta1/beta2 powers advance only with its
        applies (A3C/policies.py:83-98)."""
        a = self.actor_mask
        g = grad.clone()
        g[a] = torch.clamp(g[a], -ACTOR_CLIP, ACTOR_CLIP)
        ad = self.adam
        t = self.worker_t.get(src, 0) + 1
        self.worker_t[src] = t
        ad.t.fill_(float(t))
        ad.m.mul_(ad.b1).add_(g, alpha=1 - ad.b1)
        ad.v.mul_(ad.b2).addcmul_(g, g, value=1 - ad.b2)
        corr = np.sqrt(1 - ad.b2 ** float(t)) / (1 - ad.b1 ** float(t))
        lr = torch.where(a, torch.tensor(float(actor_lr)), torch.tensor(float(self.critic_lr)))
        self.params.data.sub_(lr * corr * ad.m / (torch.sqrt(ad.v) + ad.eps))
        self.global_step += 1

    def serve(self):
        hdr = torch.zeros(4, dtype=torch.int64)
        n = self.params.numel()
        while self.workers:
            src = dist.recv(hdr)
            cmd = int(hdr[0])
            if cmd == CMD_DONE:
                self.workers.discard(src)
                continue
            if cmd == CMD_APPLY:
                buf = torch.empty(n + 1)
                dist.recv(buf, src=src)
                self.apply(buf[:n], float(buf[n]), src)
            out = torch.cat([self.params.data, torch.tensor([float(self.global_step)])])
            dist.send(out, dst=src)


# ------------------------------------------------------------------------------------------------ worker
class A3CWorker:
    def __init__(self, cfg, task, shard, ps_ranks, logfile=None, logger=None, checkpoint_basename=None):
        self.cfg = cfg
        self.task = task
        self.is_chief = task == 0
        # A3C/process.py:175
        self.debug = cfg.mode == "debug-full" or (cfg.mode == "debug-light" and self.is_chief)
        self.shard = shard
        self.ps_ranks = ps_ranks
        seed = cfg.seed + task
        np.random.seed(seed)
        torch.manual_seed(seed)
        mpl, stop = ref.E.get_roll_params(cfg.env, "a3c")
        self.max_path_length = cfg.max_path_length or mpl
        self.ep_length_stop = cfg.ep_length_stop or stop
        self.env = ref.GymEnv(cfg.env, seed=seed)   # env time limit kept; max_path_length bounds the loop
        self.framer = ref.Framer(cfg.frames)
        self.actor, self.critic = ref.make_actor_critic(self.env, cfg.frames, "a3c", seed=seed)
        self.actor.set_opt_param(new_lr=cfg.lr, new_beta=cfg.kl_coef, new_gamma=cfg.ent_coef)
        self.path_adv = ref.PathAdv(gamma=cfg.gamma, look_ahead=cfg.look_ahead or 40)
        self.log_gamma = LinearSchedule(100, 3000, -2, -8, 100)
        self.log_beta = LinearSchedule(100, 3000, 0, -4, 100)
        self.params = [p for _, p in _param_list(self.critic.net, self.actor.net)]
        self.logger = logger if logger is not None else (ref.Logger(logfile, quiet=cfg.quiet) if logfile else None)
        self.ckpt_base = checkpoint_basename or ("model-" + C.env_prefix(cfg.env))
        self.gstep = 0
        self.history = []

    # -- PS protocol -------------------------------------------------------------------------------------------
    def _exchange(self, grads=None):
        """Apply (if grads) and pull every shard; returns the global step."""
        cmd = CMD_APPLY if grads is not None else CMD_PULL
        lr = self.actor.adam.get_lr()
        for s, r in enumerate(self.ps_ranks):
            idx = self.shard.shard_vars[s]
            dist.send(torch.tensor([cmd, self.task, self.shard.shard_numel[s], 0], dtype=torch.int64), dst=r)
            if grads is not None:
                dist.send(torch.cat([_flatten(grads, idx), torch.tensor([lr])]), dst=r)
        gstep = 0
        for s, r in enumerate(self.ps_ranks):
            idx = self.shard.shard_vars[s]
            buf = torch.empty(self.shard.shard_numel[s] + 1)
            dist.recv(buf, src=r)
            _unflatten_into(buf[:-1], self.params, idx)
            if s == 0:
                gstep = int(buf[-1])
        return gstep

    def done(self):
        for r in self.ps_ranks:
            dist.send(torch.tensor([CMD_DONE, self.task, 0, 0], dtype=torch.int64), dst=r)

    # -- loop --------------------------------------------------------------------------------------------------
    def run(self):
        cfg = self.cfg
        actor, critic, framer = self.actor, self.critic, self.framer
        self.gstep = self._exchange()   # initial sync_w_global (fixes reference bug #12)
        i = 0
        last_save = -1
        while self.gstep < cfg.total_updates:
            ep_obs, ep_advs, ep_logps, ep_targets, ep_acs, ep_rews = [], [], [], [], [], []
            tot_rews, tot_ent, rolls = 0.0, 0.0, 0
            while len(ep_rews) < self.ep_length_stop:
                path = ref.rollout(self.env, None, actor.act, framer, self.max_path_length)
                obs_aug = framer.full(path["obs"])
                ep_obs += obs_aug[:-1]
                ep_logps += path["logps"]
                ep_acs += path["acs"]
                vals = critic.value(obs_aug).reshape(-1)
                tv, advs = self.path_adv(rews=path["rews"], vals=vals, terminal=path["terminated"])
                ep_targets += list(tv)
                ep_advs += list(advs)
                ep_rews += path["rews"]
                tot_rews += sum(path["rews"])
                tot_ent += path["entropy"]
                if rolls == 0 and i % 50 == 0 and not cfg.quiet:
                    print("Total Steps %d" % self.gstep)
                    print("Path length %d" % len(path["rews"]))
                    print("Terminated {}".format(path["terminated"]))
                rolls += 1
            avg_rew = tot_rews / rolls
            ep_obs, ep_advs, ep_logps, ep_targets, ep_acs = ref.make_np(ep_obs, ep_advs, ep_logps, ep_targets, ep_acs)
            ep_advs = (ep_advs - np.mean(ep_advs)) / (1e-8 + np.std(ep_advs))
            avg_ent = tot_ent / float(len(ep_logps))
            if self.debug and i % 50 == 13:   # A3C/process.py:250-256
                perm = np.random.choice(len(ep_advs), size=20)
                print("Some preds", critic.value(ep_obs[perm]))
                print("Some target vals", ep_targets[perm])
                print("Some logps", ep_logps[perm])
                actor.printoo(ep_obs)
                critic.printoo(ep_obs)
            ev_before = ref.var_accounted_for(ep_targets, critic.value(ep_obs))
            cir_loss = critic.compute_grads(ep_obs, ep_targets)
            act_loss = actor.compute_grads(ep_acs, ep_obs, ep_advs, ep_logps)
            grads = [p.grad for p in self.params]
            self.gstep = self._exchange(grads)          # apply to the global vars + sync_w_global
            ev_after = ref.var_accounted_for(ep_targets, critic.value(ep_obs))
            kl = actor.get_kl(None, ep_logps, ep_obs, ep_acs)
            act_lr, cur_beta, cur_gamma = actor.get_opt_param()
            if kl < cfg.desired_kl / 4:
                actor.set_opt_param(new_lr=min(cfg.max_lr, act_lr * 1.5))
            elif kl > cfg.desired_kl * 4:
                actor.set_opt_param(new_lr=max(cfg.min_lr, act_lr / 1.5))
            if cfg.anneal_regularizers:
                if self.log_gamma.update_time(i):
                    actor.set_opt_param(new_gamma=float(np.power(10.0, self.log_gamma.val(i))))
                if self.log_beta.update_time(i):
                    actor.set_opt_param(new_beta=float(np.power(10.0, self.log_beta.val(i))))
            if self.logger is not None:
                self.logger(i, act_loss=act_loss, worker_id=self.task, act_lr=act_lr, kl_dist=kl,
                            circ_loss=np.sqrt(cir_loss), avg_rew=avg_rew, ev_before=ev_before, ev_after=ev_after,
                            print_tog=(cfg.stdout_freq and i % cfg.stdout_freq == 0) and not cfg.quiet,
                            avg_ent=avg_ent)
                if cfg.flush_every and i % cfg.flush_every == cfg.flush_every // 2:
                    self.logger.flush()
            self.history.append(dict(iteration=i, gstep=self.gstep, avg_rew=avg_rew, kl=kl, act_lr=act_lr,
                                     ev_before=ev_before, ev_after=ev_after))
            if self.is_chief and cfg.save_every and cfg.checkpoint_dir:
                mark = self.gstep // cfg.save_every
                if mark != last_save:
                    self.save(self.gstep)
                    last_save = mark
            i += 1
        self.done()
        if self.logger is not None:
            self.logger.close()
        return self.history

    def save(self, gstep):
        os.makedirs(self.cfg.checkpoint_dir, exist_ok=True)
        base = self.ckpt_base
        path = os.path.join(self.cfg.checkpoint_dir, f"{base}-{gstep}")
        t = C.reference_tensors(self.actor.net, self.critic.net, "a3c", actor_lr=self.cfg.lr,
                                ent_coef=self.cfg.ent_coef, kl_coef=self.cfg.kl_coef, critic_lr=self.cfg.critic_lr)
        C.save_tensors(path, t)   # global vars only, no Adam slots / global_step -- as the reference
        kept = C._prune(self.cfg.checkpoint_dir, base, self.cfg.keep_checkpoints)
        C._write_state_file(self.cfg.checkpoint_dir, path, kept or [path])
        return path


def run(cfg, rank=None, world=None, ps_num=None, log_dir=None, logger=None, checkpoint_basename=None):
    """Entry point of one process of the A3C job (PS or worker by rank); the process group must be initialised
    (gloo) or is initialised here from the torchrun environment."""
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    rank = dist.get_rank() if rank is None else rank
    world = dist.get_world_size() if world is None else world
    ps_num = cfg.ps_num if ps_num is None else ps_num
    n_workers = world - ps_num
    assert n_workers >= 1, "need at least one worker rank"
    # every rank builds the same variable list (deterministic shapes); rank 0's initial values are the global init
    env = ref.GymEnv(cfg.env, seed=cfg.seed)
    actor, critic = ref.make_actor_critic(env, cfg.frames, "a3c", seed=cfg.seed)
    params = _param_list(critic.net, actor.net)
    shard = ShardMap(params, ps_num)
    tensors = [p for _, p in params]
    if rank < ps_num:
        init = _flatten(tensors, shard.shard_vars[rank])
        ps = ParameterServer(shard, rank, init, range(ps_num, world), cfg.critic_lr)
        ps.serve()
        return {"role": "ps", "global_step": ps.global_step}
    task = rank - ps_num
    log_dir = log_dir if log_dir is not None else (cfg.outdir if cfg.outdir else None)
    logfile = os.path.join(log_dir, f"worker_{task}.log") if log_dir else None
    if logfile:
        os.makedirs(log_dir, exist_ok=True)
    w = A3CWorker(cfg, task, shard, list(range(ps_num)), None if logger is not None else logfile, logger=logger,
                  checkpoint_basename=checkpoint_basename)
    hist = w.run()
    return {"role": "worker", "task": task, "history": hist, "global_step": w.gstep}
