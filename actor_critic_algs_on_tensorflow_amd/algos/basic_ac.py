"""Reference-parity episode-batched actor-critic trainer (``Basic_AC/run_AC.py:166-286``).

Per iteration:
  * collect whole episodes with batch-1 inference until >= ``ep_length_stop`` steps or ``max_rolls`` (7) episodes;
  * per episode: ``Framer.full`` features, critic values of every observation, ``PathAdv`` L-step targets and
    advantages (gamma 0.98, L 40);
  * normalise advantages over the batch, one critic Adam step (EV before/after), one actor Adam step (clip +-1);
  * KL proxy on the updated actor -> KL-adaptive lr (x1.5 / /1.5 in [1e-6, 1]), log10 schedules of the entropy and
    KL coefficients every 100 iterations, reference Logger (report every 20, flush at i % 100 == 50), checkpoint
    every ``save_every`` iterations named ``<checkpoint_dir>-<EnvPrefix>-<total episodes>``.

This is the slow, faithful loop (one env, batch-1 inference on the CPU, as the reference); the vectorised
GPU-native trainers of :mod:`.trainer` are the fast path with the same losses and schedules.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from .. import ckpt as C
from ..compat import reference as ref
from ..utils.schedule import LinearSchedule


class BasicACTrainer:
    def __init__(self, cfg):
        self.cfg = cfg
        self.variant = cfg.model_variant if cfg.model_variant in ("basic", "a3c") else "basic"
        torch.manual_seed(cfg.seed)
        np.random.seed(cfg.seed)
        mpl, stop = ref.E.get_roll_params(cfg.env, "basic")
        self.max_path_length = cfg.max_path_length or mpl
        self.ep_length_stop = cfg.ep_length_stop or stop
        # the env keeps its own time limit (gym TimeLimit: 200 for Pendulum-v0); max_path_length only bounds the
        # rollout loop (Basic_AC/run_AC.py:95,130-131), so a Basic Pendulum batch is 7 episodes of 200 steps
        self.env = ref.GymEnv(cfg.env, seed=cfg.seed)
        self.framer = ref.Framer(cfg.frames)
        self.actor, self.critic = ref.make_actor_critic(self.env, cfg.frames, self.variant, seed=cfg.seed)
        self.actor.set_opt_param(new_lr=cfg.lr, new_beta=cfg.kl_coef, new_gamma=cfg.ent_coef)
        self.critic.adam.set_lr(cfg.critic_lr)
        self.path_adv = ref.PathAdv(gamma=cfg.gamma, look_ahead=cfg.look_ahead or 40)
        self.log_gamma = LinearSchedule(100, 3000, -2, -8, 100)
        self.log_beta = LinearSchedule(100, 3000, 0, -4, 100)
        self.logger = ref.Logger(cfg.outdir, legacy_step_index=cfg.legacy_step_index, metrics_path=cfg.metrics_path,
                                 quiet=cfg.quiet) if cfg.outdir else None
        self.iteration = 0
        self.env_steps = 0
        self.tot_rolls = 0
        self.rank = 0
        self.history = []
        self.model = self._model_view()
        self.tb = None
        if cfg.tboard:   # Basic_AC/run_AC.py:201-202: summaries/<outdir stem>.data
            from ..utils import tensorboard as TB
            self.tb = TB.VariableSummaries(TB.SummaryWriter(TB.summaries_dir(cfg.outdir or "run", cfg.tb_root)),
                                           TB.reference_summary_scopes(self.actor.net, self.critic.net))

    def _model_view(self):
        from ..models.policy import MLPActorCritic
        m = MLPActorCritic.__new__(MLPActorCritic)
        torch.nn.Module.__init__(m)
        m.discrete = self.actor.discrete
        m.critic = self.critic.net
        m.actor = self.actor.net
        return m

    def iterate(self, i):
        cfg = self.cfg
        actor, critic, framer = self.actor, self.critic, self.framer
        ep_obs, ep_advs, ep_logps, ep_targets, ep_acs, ep_rews = [], [], [], [], [], []
        tot_rews, tot_ent, rolls = 0.0, 0.0, 0
        while len(ep_rews) < self.ep_length_stop and rolls < cfg.max_rolls:
            path = ref.rollout(self.env, None, actor.act, framer, self.max_path_length,
                               render=False)
            obs_aug = framer.full(path["obs"])
            ep_obs += obs_aug[:-1]
            ep_logps += path["logps"]
            ep_acs += path["acs"]
            tot_ent += path["entropy"]
            vals = critic.value(obs_aug).reshape(-1)
            tv, advs = self.path_adv(rews=path["rews"], vals=vals, terminal=path["terminated"])
            ep_targets += list(tv)
            ep_advs += list(advs)
            ep_rews += path["rews"]
            tot_rews += sum(path["rews"])
            if rolls == 0 and i % 10 == 0 and cfg.mode == "debug":
                actor.printoo(ep_obs)
                critic.printoo(ep_obs)
                print("Path length %d" % len(path["rews"]))
                print("Terminated {}".format(path["terminated"]))
            rolls += 1
        avg_rew = tot_rews / rolls
        avg_ent = tot_ent / float(len(ep_logps))
        ep_obs, ep_advs, ep_logps, ep_targets, ep_acs = ref.make_np(ep_obs, ep_advs, ep_logps, ep_targets, ep_acs)
        if cfg.norm_adv:
            ep_advs = (ep_advs - np.mean(ep_advs)) / (1e-8 + np.std(ep_advs))
        if i % 50 == 13 and cfg.mode == "debug":   # Basic_AC/run_AC.py:243-247
            perm = np.random.choice(len(ep_advs), size=20)
            print("Some targets", ep_targets[perm])
            print("Some preds", critic.value(ep_obs[perm]))
            print("Some logps", ep_logps[perm])
        cir_loss, ev_before, ev_after = ref.train_ciritic(critic, None, ep_obs, ep_targets)
        act_loss = ref.train_actor(actor, None, ep_obs, ep_advs, ep_logps, ep_acs)
        if self.tb is not None:   # every iteration, after both updates (Basic_AC/run_AC.py:253-255)
            self.tb.write(i)
        act_lr, cur_beta, cur_gamma = actor.get_opt_param()
        kl = actor.get_kl(None, ep_logps, ep_obs, ep_acs)
        if cfg.kl_adaptive_lr:
            if kl < cfg.desired_kl / 4:
                actor.set_opt_param(new_lr=min(cfg.max_lr, act_lr * 1.5))
            elif kl > cfg.desired_kl * 4:
                actor.set_opt_param(new_lr=max(cfg.min_lr, act_lr / 1.5))
        if cfg.anneal_regularizers:
            if self.log_gamma.update_time(i):
                ng = float(np.power(10.0, self.log_gamma.val(i)))
                actor.set_opt_param(new_gamma=ng)
                if not cfg.quiet:
                    print("\nUpdated gamma from %.4f to %.4f." % (cur_gamma, ng))
            if self.log_beta.update_time(i):
                nb = float(np.power(10.0, self.log_beta.val(i)))
                actor.set_opt_param(new_beta=nb)
                if not cfg.quiet:
                    print("Updated beta from %.4f to %.4f." % (cur_beta, nb))
        stats = dict(act_loss=act_loss, crit_loss=cir_loss, kl=kl, entropy=avg_ent, ev_before=ev_before,
                     ev_after=ev_after, avg_rew=avg_rew, episodes=rolls, act_lr=act_lr)
        if self.logger is not None:
            self.logger(i, act_loss=act_loss, circ_loss=np.sqrt(cir_loss), avg_rew=avg_rew, ev_before=ev_before,
                        ev_after=ev_after, act_lr=act_lr, print_tog=(cfg.stdout_freq and i % cfg.stdout_freq == 0)
                        and not cfg.quiet, kl_dist=kl, avg_ent=avg_ent)
            if cfg.flush_every and i % cfg.flush_every == cfg.flush_every // 2:
                self.logger.flush()
        if cfg.save_every and i % cfg.save_every == 0 and cfg.checkpoint_dir:
            self.save_checkpoint()
        self.tot_rolls += rolls
        self.env_steps += len(ep_rews)
        return stats

    def step(self):
        s = self.iterate(self.iteration)
        self.history.append(dict(iteration=self.iteration, **s))
        self.iteration += 1
        return s

    def train(self, num_updates=None):
        n = self.cfg.total_updates if num_updates is None else num_updates
        for _ in range(n):
            self.step()
        return self.history

    def checkpoint_path(self):
        return f"{self.cfg.checkpoint_dir}-{C.env_prefix(self.cfg.env)}-{self.tot_rolls}"

    def save_checkpoint(self, path=None):
        path = path or self.checkpoint_path()
        t = C.reference_tensors(self.actor.net, self.critic.net, self.variant, actor_lr=self.actor.adam.get_lr(),
                                ent_coef=self.actor.gamma, kl_coef=self.actor.beta,
                                critic_lr=self.critic.adam.get_lr())
        # the Basic_AC Saver is built after the optimisers, so Adam slots are part of the checkpoint
        for scope, net, opt in (("Actor" if self.variant == "basic" else "global_actor", self.actor.net,
                                 self.actor.adam),
                                ("Critic" if self.variant == "basic" else "global_critic", self.critic.net,
                                 self.critic.adam)):
            names = {id(p): k for k, p in t.items() if isinstance(p, torch.nn.Parameter)}
            off = 0
            for p in net.parameters():
                n = p.numel()
                k = names.get(id(p))
                if k is not None:
                    t[k + "/Adam"] = opt.m[off:off + n].view(p.shape)
                    t[k + "/Adam_1"] = opt.v[off:off + n].view(p.shape)
                off += n
            step = float(opt.t)
            t[f"{scope}/beta1_power"] = torch.tensor(opt.b1 ** (step + 1))
            t[f"{scope}/beta2_power"] = torch.tensor(opt.b2 ** (step + 1))
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        C.save_tensors(path, t)
        base = os.path.basename(path).rsplit("-", 1)[0]
        kept = C._prune(d or ".", base, self.cfg.keep_checkpoints)
        C._write_state_file(d or ".", path, kept or [path])
        return path

    def close(self):
        if self.logger is not None:
            self.logger.close()
        if self.tb is not None:
            self.tb.close()
