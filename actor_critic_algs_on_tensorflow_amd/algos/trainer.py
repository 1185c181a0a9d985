"""Synchronous actor-critic trainers: A2C and PPO-clip over a device-resident env bank.

One *update* = collect a ``[T, N]`` rollout (batched policy inference + one env-bank kernel per step), estimate
returns/advantages (n-step or GAE), then learn:
  * ``a2c``: one full-batch gradient step (as the reference: ``Basic_AC/run_AC.py:250-251``);
  * ``ppo``: ``ppo_epochs`` x ``ppo_minibatches`` clipped-surrogate steps.

Reference features kept: KL-proxy + entropy regularised actor loss (``Basic_AC/policies.py:72-78``), per-batch
advantage normalisation (``Basic_AC/run_AC.py:241``), element-wise gradient clipping, TF-semantics Adam,
KL-adaptive actor lr (``Basic_AC/run_AC.py:257-266``, device-side), log10 annealing of the entropy/KL coefficients
(``Basic_AC/run_AC.py:181-182,268-275``), the reference Logger format, EV before/after.

Two execution engines share this driver:
  * ``native`` (CNN family on GPU, the default there): the hand-written HIP engine of :mod:`.engine` -- explicit
    MFMA forward/backward, fused loss/head-gradient kernel, env kernels writing straight into the rollout slabs,
    sampling kernel deriving its RNG keys from the env counters, optimiser zeroing the gradient slab after use.
  * ``torch`` (everything else, and the CPU oracle): the same maths through autograd over the same flat slabs.
Nothing in ``collect``/``learn`` reads back to the host, so on a GPU the update is captured as hipGraph(s) and
replayed (see ``capture``). Data parallelism (sync DP over RCCL, :mod:`..parallel.dp`) all-reduces the flat
gradient slab between backward and the optimiser step.
"""
from __future__ import annotations

import math
import os
import sys
import time

import torch

from .. import _native
from .. import envs as E
from ..config import TrainConfig
from ..models.policy import build_model
from ..ops import distributions as D
from ..ops import returns as R
from ..ops.optim import FlatParams, make_optimizer
from ..utils.logger import Logger
from ..utils.schedule import DeviceKLAdaptiveLR, RegularizerSchedule
from ..utils.stats import var_accounted_for_tensor
from ..utils.trace import PhaseTimer
from . import losses as L
from .storage import RolloutStorage

KEY_ENV_BITS = 20
# Graph capture is thread-local: RCCL's watchdog thread polls the events of earlier (uncaptured) collectives while
# the trainer captures an update whose collectives are recorded in the graph; in the default global mode that poll
# is a forbidden call during capture and kills the process group (seen on MI355X: hipErrorStreamCaptureUnsupported
# from ProcessGroupNCCL's watchdog).
CAPTURE_MODE = "thread_local"
FAULT_EXIT_CODE = 43   # exit status of a rank killed by ``fault_inject`` (SURVEY §5.3 test hook)


def parse_fault(spec):
    """``"rank:iteration"`` -> (rank, iteration); ``"rank:iteration:where"`` -> (rank, iteration, where) for the
    async PS worker's mid-exchange fault points (``where`` = ``"push"``: die after the push header, before the
    payload; ``"reply"``: die after the push, before the PS's reply); None for no fault."""
    if not spec:
        return None
    parts = str(spec).split(":")
    if len(parts) == 3:
        if parts[2] not in ("push", "reply"):
            raise ValueError(f"fault_inject {spec!r}: the fault point must be 'push' or 'reply'")
        return int(parts[0]), int(parts[1]), parts[2]
    r, it = parts
    return int(r), int(it)

# layout of the device statistics buffer; slots 0..6 are written directly by the fused loss kernel
STAT_KEYS = ("pg", "kl", "entropy", "crit_loss", "clipfrac", "act_loss", "ratio", "ev_before", "ev_after")
LOG_KEYS = ("act_loss", "crit_loss", "kl", "entropy", "ev_before", "ev_after", "clipfrac")


class SegmentRecorder:
    """Captures one update as a chain of hipGraphs cut at the host-issued collectives.

    Trainer code routes every collective through :meth:`ActorCriticTrainer._comm`; while recording, that ends the
    current graph, stores the collective (a closure over persistent buffers, written in place) and opens the next
    graph, so ``replay`` = graph 0, collective 0, graph 1, ... All graphs share one memory pool and always replay in
    capture order (the condition under which pool sharing is safe). Collectives are stream-ordered, not host-
    blocking: the host only walks the list."""

    def __init__(self):
        self.items = []
        self.pool = torch.cuda.graph_pool_handle()
        self._g = None
        self._ctx = None

    def start(self):
        self._g = torch.cuda.CUDAGraph()
        self._ctx = torch.cuda.graph(self._g, pool=self.pool, capture_error_mode=CAPTURE_MODE)
        self._ctx.__enter__()

    def cut(self, fn):
        self._ctx.__exit__(None, None, None)
        self.items.append(("graph", self._g))
        self.items.append(("host", fn))
        self.start()

    def finish(self):
        self._ctx.__exit__(None, None, None)
        self.items.append(("graph", self._g))
        self._g = self._ctx = None

    def abort(self):
        if self._ctx is not None:
            try:
                self._ctx.__exit__(None, None, None)
            except Exception:   # pragma: no cover - capture already invalid
                pass
            self._g = self._ctx = None

    @property
    def n_graphs(self):
        return sum(1 for k, _ in self.items if k == "graph")

    def replay(self):
        for kind, obj in self.items:
            if kind == "graph":
                obj.replay()
            else:
                obj()


class ActorCriticTrainer:
    def __init__(self, cfg: TrainConfig, env=None, model=None, dp=None):
        self.cfg = cfg
        self.device = torch.device(cfg.device)
        self.dp = dp
        self.rank = dp.rank if dp is not None else 0
        self.worker_id = self.rank   # Logger rows' worker column (an async PS worker sets its task id)
        self.world = dp.world_size if dp is not None else 1
        fs = 4 if ("Pong" in cfg.env or "Breakout" in cfg.env) else cfg.frames
        self.env = env if env is not None else E.make(
            cfg.env, cfg.num_envs, device=self.device, seed=cfg.seed, env_offset=self.rank * cfg.num_envs,
            frame_stack=fs)
        self.model = (model if model is not None else
                      build_model(self.env, cfg.model, cfg.model_variant, seed=cfg.seed)).to(self.device)
        self.flat = FlatParams(self.model.param_groups(), self.device)
        if dp is not None:
            dp.broadcast_params(self.flat)
            if cfg.grad_bucket_dtype == "bf16" and dp.compress is None:
                dp.compress = "bf16"
            dp.prepare(self.flat.grad)
        self.engine = None
        self.mlp = None
        self.shadow = None
        if self._want_native_mlp():
            from ..ops.mlp import MLPEngine
            self.mlp = MLPEngine(self.model, self.flat)
        elif self._want_native():
            from .engine import CNNEngine
            self.shadow = torch.empty(self.flat.numel, dtype=torch.bfloat16, device=self.device)
            self.shadow.copy_(self.flat.data)
            self.engine = CNNEngine(self.model, self.flat, self.shadow, opts=cfg.engine_opts)
        self.opts = {}
        for g in self.flat.groups:
            s, e = self.flat.groups[g]
            sh = self.shadow[s:e] if self.shadow is not None else None
            if g == "critic":
                opt = make_optimizer(cfg.optimizer, self.flat, g, cfg.critic_lr, cfg.critic_clip_value,
                                     cfg.max_grad_norm, bf16_shadow=sh)
            else:
                opt = make_optimizer(cfg.optimizer, self.flat, g, cfg.lr, cfg.clip_value, cfg.max_grad_norm,
                                     bf16_shadow=sh)
            opt.zero_grad_after = self.engine is not None or self.mlp is not None
            if dp is not None:
                opt.grad_mul = dp.grad_mul   # the all-reduce leaves the sum; the update kernel averages on read
            self.opts[g] = opt
        if self.engine is not None and self.engine.frag_entries():
            # the group holding the conv (and fc) weights also rewrites their fragment-ordered copies in its update
            ent = self.engine.frag_entries()
            owner = [o for o in self.opts.values()
                     if all(0 <= e[0].data_ptr() - o.p.data_ptr() < o.p.numel() * 4 for e in ent)]
            assert len(owner) == 1, "the conv / fc weights must live in one optimiser group"
            owner[0].set_frag(ent)
        self.actor_opt = self.opts.get("actor", self.opts.get("shared"))
        if (dp is not None and dp.compress == "bf16" and self.engine is not None and len(self.opts) == 1
                and all(o.clip_value is None for o in self.opts.values()) and _native.use_native(self.flat.data)):
            # bf16 buckets: the optimiser (and its sum of squares) read the all-reduced bf16 comm buffer itself -- no
            # cast back into the fp32 slab (one launch and ~10 MB of traffic less per update)
            dp.prepare(self.flat.grad)
            for o in self.opts.values():
                o.bind_grad16(dp.comm_view(self.flat.grad))
            dp.direct_read = True
        if (self.engine is not None and dp is None and len(self.opts) == 1
                and all(o.clip_value is None for o in self.opts.values())):
            # the engine's gradient finaliser writes the global-norm partials: no separate sum-of-squares pass
            self.engine.want_parts = True
            for o in self.opts.values():
                o.ext_parts = self.engine.fin_parts
        T, N = cfg.n_steps, self.env.num_envs
        act_shape = () if self.env.is_discrete else tuple(self.env.action_space.shape)
        act_dtype = torch.int32 if self.env.is_discrete else torch.float32
        self.storage = RolloutStorage(T, N, self.env.obs_shape, self.env.obs_dtype, act_shape, act_dtype,
                                      self.device, ring=self.engine is not None)
        if cfg.bootstrap_on_timeout:
            self.env.keep_final_obs = True   # the torch env step keeps the pre-reset observation (envs/base.py)
        self.env.reset(out=self.storage.obs[0])
        dev = self.device
        self.ent_coef = torch.tensor(cfg.ent_coef, device=dev)
        self.kl_coef = torch.tensor(cfg.kl_coef, device=dev)
        self.lr_ctrl = DeviceKLAdaptiveLR(cfg.desired_kl, cfg.min_lr, cfg.max_lr) if cfg.kl_adaptive_lr else None
        self.reg_sched = RegularizerSchedule() if cfg.anneal_regularizers else None
        self.policy_seed = (cfg.seed * 7919 + 17) & 0xFFFFFFFF
        self.update_counter = torch.zeros((), dtype=torch.int64, device=dev)
        self.stats_buf = torch.zeros(16, dtype=torch.float32, device=dev)
        self.stats = {k: self.stats_buf[i] for i, k in enumerate(STAT_KEYS)}
        self.adv_buf = torch.zeros(T * N, dtype=torch.float32, device=dev)
        self.iteration = 0
        self.env_steps = 0
        self.graph = None
        self._defer_allreduce = False
        self._bw_stage = "all"      # "tail" while capturing the first segment of the bucketed DP update
        self._bw_pending = None
        self._comm_grad = None      # lag-1 DP: the all-reduced copy of the previous update's gradient
        self._comm_work = None
        self._rec = None            # SegmentRecorder while capturing a segmented (DP) update
        self._grad_sink = None      # async PS worker: replaces all-reduce + optimiser (algos/a3c_gpu.py)
        self._kl_buf = torch.zeros(1, dtype=torch.float32, device=self.device) if dp is not None else None
        # deferred post-update KL [sum over ranks, ranks that wrote it] (_kl_deferred); re-pointed into the returns
        # scan's moment buffer once that exists, so it travels in the same all-reduce
        self._kl_tail = torch.zeros(2, dtype=torch.float64, device=self.device) if dp is not None else None
        self._kl_defer_on = True
        self.logger = None
        if self.rank == 0 and cfg.outdir:
            self.logger = Logger(cfg.outdir, legacy_step_index=cfg.legacy_step_index, metrics_path=cfg.metrics_path,
                                 quiet=cfg.quiet)
        self.tb = None
        if cfg.tboard and self.rank == 0:
            from ..utils import tensorboard as TB
            self.tb = TB.VariableSummaries(TB.SummaryWriter(TB.summaries_dir(cfg.outdir or "run", cfg.tb_root)),
                                           self._summary_scopes(), self.flat)
        self.timer = PhaseTimer(self.device, enabled=cfg.trace)
        self._fault = parse_fault(cfg.fault_inject)

    def _want_native(self):
        """The hand-written HIP engine runs the CNN family on GPU (``engine="auto"|"native"``)."""
        from ..models.policy import CNNActorCritic
        eng = self.cfg.engine
        if self.cfg.bootstrap_on_timeout and eng == "native":
            raise ValueError("bootstrap_on_timeout needs the terminal observation of truncated episodes, which the "
                             "native env/rollout kernels do not keep: use engine='torch'")
        if eng == "torch" or self.cfg.bootstrap_on_timeout or self.device.type != "cuda" or \
                not isinstance(self.model, CNNActorCritic):
            if eng == "native":
                raise ValueError("engine='native' needs a CNN model on a GPU")
            return False
        _native.require()
        return True

    def _want_native_mlp(self):
        """The fused MLP engine (``ops/mlp.py``) runs the reference's MLP actor/critic on GPU."""
        from ..models.policy import MLPActorCritic
        # time-limit bootstrapping needs the env kernel's terminal observation (classic / MuJoCo-shaped banks)
        boot_ok = not self.cfg.bootstrap_on_timeout or getattr(self.env, "native_final_obs", False)
        if self.cfg.engine == "torch" or not boot_ok or self.device.type != "cuda" or \
                not isinstance(self.model, MLPActorCritic):
            return False
        if self.model.actor.ac_dim > 16 or self.env.obs_dtype != torch.float32 or len(self.env.obs_shape) != 1:
            if self.cfg.engine == "native":
                raise ValueError("the native MLP engine needs fp32 vector observations and at most 16 actions")
            return False
        _native.require()
        return True

    # ------------------------------------------------------------------ rollout
    def _keys(self):
        return self.env.tg * (1 << KEY_ENV_BITS) + self.env.env_ids

    @torch.no_grad()
    def collect(self):
        if self.mlp is not None:
            return self._collect_mlp()
        if self.engine is not None:
            return self._collect_native()
        st, env, model = self.storage, self.env, self.model
        for t in range(st.T):
            obs_t = st.obs[t]
            pi, v = model(obs_t)
            a, logp, ent = model.sample(pi, self._keys(), self.policy_seed)
            st.actions[t].copy_(a.view_as(st.actions[t]))
            st.logp[t].copy_(logp)
            st.entropy[t].copy_(ent)
            st.values[t].copy_(v)
            env.step(a, prev_obs=obs_t, obs_out=st.obs[t + 1], reward_out=st.rewards[t], done_out=st.dones[t],
                     trunc_out=st.truncated[t])
            if self.cfg.bootstrap_on_timeout:
                # a time-limit cut stays an episode boundary (done = 1: nothing leaks into the next episode, whose
                # reset observation already sits in obs[t+1]); the truncated step's reward gets gamma * V(terminal
                # observation) -- the observation the auto-reset overwrote, kept by the bank in final_obs
                vf = model.value(env.final_obs)
                st.rewards[t].add_(self.cfg.gamma * vf * st.truncated[t].to(vf.dtype))
        st.values[st.T].copy_(model.value(st.obs[st.T]))

    @torch.no_grad()
    def _collect_mlp(self):
        """MuJoCo-shaped bank: ONE persistent launch for the whole rollout + one critic launch (ops/mlp.py
        ``rollout_linear``). Otherwise one launch per step for the policy (both towers + sampling) and one for the
        env bank."""
        st, env, eng = self.storage, self.env, self.mlp
        boot = self.cfg.bootstrap_on_timeout
        if self.cfg.fused_rollout and eng.supports_fused_rollout(env) and not boot:
            eng.rollout_linear(env, st, KEY_ENV_BITS, self.policy_seed)
            return
        if boot and getattr(self, "_final_obs", None) is None:
            self._final_obs = torch.zeros((st.T,) + tuple(st.obs.shape[1:]), dtype=st.obs.dtype, device=self.device)
            self._final_v = torch.zeros(st.T * st.N, dtype=torch.float32, device=self.device)
        for t in range(st.T):
            eng.policy_step(st.obs[t], st.actions[t], st.logp[t], st.entropy[t], st.values[t], env.tg, env.env_ids,
                            KEY_ENV_BITS, self.policy_seed)
            env.step(st.actions[t], prev_obs=st.obs[t], obs_out=st.obs[t + 1], reward_out=st.rewards[t],
                     done_out=st.dones[t], trunc_out=st.truncated[t],
                     final_out=self._final_obs[t] if boot else None)
        eng.value(st.obs[st.T], st.values[st.T])
        if boot:
            # a time-limit cut stays an episode boundary (done = 1); the truncated step's reward gets
            # gamma * V(terminal observation): ONE critic launch over the T x N terminal stacks the env kernel wrote
            eng.value(self._final_obs.view(st.T * st.N, -1), self._final_v)
            st.rewards.addcmul_(self._final_v.view(st.T, st.N), st.truncated.to(torch.float32),
                                value=self.cfg.gamma)

    def _reuse_acts(self):
        """A2C takes one gradient step at the parameters that acted, so the rollout's forward activations ARE the
        learner's forward pass: each rollout step writes them into its rows of the learner buffers and the learner
        goes straight to loss + backward (exact; PPO re-evaluates after its first step and keeps the forward)."""
        return self.engine is not None and self.cfg.algo == "a2c" and self.cfg.reuse_rollout_acts

    @torch.no_grad()
    def _collect_native(self):
        st, env, eng = self.storage, self.env, self.engine
        A = eng.A
        N = env.num_envs
        b = eng.bufs(N)
        ops = _native.require()
        lb = eng.bufs(st.T * N, with_grad=True) if self._reuse_acts() else None
        fused = isinstance(env, E.PongVecEnv)
        if fused and env.frame_stack == 4 and eng.fused_step_ok(N):
            return self._collect_fused_steps(st, env, eng, lb, b, N)
        if fused and env.frame_stack == 4 and eng.fused_env_step_ok(N):
            return self._collect_fused_env_steps(st, env, eng, lb, b, N)
        for t in range(st.T):
            bt = lb.rows(t * N, N) if lb is not None else b
            if fused:
                # conv trunk + fc, then ONE launch: policy/value head + sampling + env step (+ frame render)
                # (the fused trunk also shifts the frame stack into obs[t + 1]; the env kernel renders the newest)
                # (and leaves the fc product as split-K planes that the env kernel reduces into bt.h)
                shifted = eng.forward(st.obs[t], bt, head=False, shift_out=st.obs[t + 1], fc_parts=eng.fc_parts)
                hp, S = eng.last_fc if eng.fc_parts else (None, 0)
                ops.env_policy_step_pong(bt.h, eng.sWh, eng.bh, bt.z, st.actions[t], st.logp[t], st.entropy[t],
                                         st.values[t], KEY_ENV_BITS, self.policy_seed, env.state, env.t, env.tg,
                                         env.ep_ret, env.ep_stats, env.env_ids, st.obs[t], st.obs[t + 1],
                                         st.rewards[t], st.dones[t], st.truncated[t], env.seed,
                                         env.max_episode_steps, env.frame_stack, shifted, hp, S,
                                         eng.bfc if hp is not None else None)
                continue
            z = eng.forward(st.obs[t], bt)
            # one launch: sample + logp + entropy + value copy, RNG keys from the env counters
            ops.categorical_sample_env(z[:, :A], env.tg, env.env_ids, KEY_ENV_BITS, self.policy_seed, st.actions[t],
                                       st.logp[t], st.entropy[t], st.values[t])
            env.step(st.actions[t], prev_obs=st.obs[t], obs_out=st.obs[t + 1], reward_out=st.rewards[t],
                     done_out=st.dones[t], trunc_out=st.truncated[t])
        eng.value(st.obs[st.T], b, st.values[st.T])

    def _collect_fused_steps(self, st, env, eng, lb, b, N):
        """Rollout as trunk(obs_0) + fc, then per step ONE launch of policy/env step t fused with the row-split trunk
        of obs_{t+1} (``pong_fused_step``) + the fc product of obs_{t+1}; the last step's trunk is the bootstrap
        observation's, whose value comes straight from the fc planes. The env state alternates between its two
        parity slots (the fused kernel reads one and commits into the other)."""
        ops = _native.require()
        T = st.T
        rows = (lambda t: lb.rows(t * N, N)) if lb is not None else (lambda t: b)
        _, W2, W3, frag = eng.trunk_w()   # conv2 / conv3 operands (fragment-ordered copies when kept)
        eng.forward(st.obs[0], rows(0), head=False, shift_out=st.obs[1], fc_parts=True)
        for t in range(T):
            hp, S = eng.last_fc
            cur = rows(t)
            nxt = rows(t + 1) if t + 1 < T else b
            sn, tn, tgn, ern = env.next_state()
            ops.pong_fused_step(cur.h, eng.sWh, eng.bh, cur.z, st.actions[t], st.logp[t], st.entropy[t],
                                st.values[t], KEY_ENV_BITS, self.policy_seed, env.state, env.t, env.tg, env.ep_ret,
                                sn, tn, tgn, ern, env.ep_stats, env.env_ids, st.obs[t], st.obs[t + 1],
                                st.rewards[t], st.dones[t], st.truncated[t], env.seed, env.max_episode_steps, hp, S,
                                eng.bfc, eng.sW1, eng.b1, W2, eng.b2, W3, eng.b3, nxt.y1, nxt.y2, nxt.y3,
                                1.0 / 255.0, st.obs[t + 2] if t + 2 <= T else None, None, frag)
            env.flip()
            nxt.obs = st.obs[t + 1]
            eng.fc_planes(nxt)
        hp, S = eng.last_fc
        self._env_flips = T
        if self._boot_in_head():
            # V(s_T) is computed by the learner's head launch straight from these planes (no fc_value launch)
            self._boot = (hp, S)
            return
        ops.fc_value(hp, S, eng.bfc, eng.sWh, eng.bh, st.values[T], None)

    def _collect_fused_env_steps(self, st, env, eng, lb, b, N):
        """Large banks (per-env trunk): trunk(obs_0) + fc, then per step ONE launch of policy/env step t fused with
        the per-env trunk of obs_{t+1} (``pong_fused_env_step``) + the fc product of obs_{t+1}; the last step's
        trunk is the bootstrap observation's, whose value comes straight from the fc planes. With
        ``EngineOpts.fused_env_split`` two workgroups per env share each step (the conv rows split in halves) and the
        env state alternates between its parity slots, as in the row-split step."""
        ops = _native.require()
        T = st.T
        split = eng.opts.fused_env_split
        _, W2, W3, frag = eng.trunk_w()
        rows = (lambda t: lb.rows(t * N, N)) if lb is not None else (lambda t: b)
        eng.forward(st.obs[0], rows(0), head=False, shift_out=st.obs[1], fc_parts=True)
        for t in range(T):
            hp, S = eng.last_fc
            cur = rows(t)
            nxt = rows(t + 1) if t + 1 < T else b
            ops.pong_fused_env_step(cur.h, eng.sWh, eng.bh, cur.z, st.actions[t], st.logp[t], st.entropy[t],
                                    st.values[t], KEY_ENV_BITS, self.policy_seed, env.state, env.t, env.tg,
                                    env.ep_ret, env.ep_stats, env.env_ids, st.obs[t + 1], st.rewards[t], st.dones[t],
                                    st.truncated[t], env.seed, env.max_episode_steps, hp, S, eng.bfc, eng.sW1,
                                    eng.b1, W2, eng.b2, W3, eng.b3, nxt.y1, nxt.y2, nxt.y3, 1.0 / 255.0,
                                    st.obs[t + 2] if t + 2 <= T else None,
                                    list(env.next_state()) if split else None, None, frag)
            if split:
                env.flip()
            nxt.obs = st.obs[t + 1]
            eng.fc_planes(nxt)
        self._env_flips = T if split else 0
        hp, S = eng.last_fc
        if self._boot_in_head():
            self._boot = (hp, S)
            return
        ops.fc_value(hp, S, eng.bfc, eng.sWh, eng.bh, st.values[T], None)

    def _boot_in_head(self):
        """The A2C head launch (``a2c_head``) also computes the bootstrap value V(s_T) from the last fc planes."""
        st = self.storage
        return (self._fused_returns() and self.engine.a2c_head and self.engine.head_ok(st.T * st.N, st.N))

    # ------------------------------------------------------------------ returns
    def _fused_returns(self):
        """Native A2C: returns, EV-before and advantage normalisation run inside the loss kernel."""
        return (self._reuse_acts() and (self.dp is None or not self.cfg.norm_adv)
                and not self.cfg.bootstrap_on_timeout and self.cfg.returns in ("nstep", "gae"))

    def compute_returns(self):
        if self._fused_returns():
            return None, None
        cfg, st = self.cfg, self.storage
        dones = st.dones   # bootstrap_on_timeout: the bootstrap is already in the truncated step's reward (collect)
        self._scanned = False
        if _native.use_native(st.rewards) and cfg.returns in ("gae", "nstep"):
            # ONE launch: chunked scan returns + EV-before + moments (+ in-place adv normalisation on one rank; under
            # DP the fp64 moments are all-reduced on the device and an elementwise kernel normalises)
            T, N = st.T, st.N
            if getattr(self, "_scan_ws", None) is None:
                self._scan_ws = R.ScanWorkspace(self.device, T, N)
                if self._kl_tail is not None:
                    self._kl_tail = self._scan_ws.mom[8:10]
                self._scan_ret = torch.empty(T * N, device=self.device)
                self._scan_adv = torch.empty(T * N, device=self.device)
            # native PPO: the minibatch gather normalises while it copies (no pass over the whole batch here)
            self._norm_mom = None
            defer = (cfg.norm_adv and self.engine is not None and cfg.algo == "ppo"
                     and st.actions.dtype == torch.int32)
            local_norm = cfg.norm_adv and self.dp is None and not defer
            ret, adv, mom = R.returns_scan(st.rewards, st.values, dones, cfg.returns, cfg.gamma, cfg.gae_lambda,
                                           cfg.look_ahead, norm=local_norm, ws=self._scan_ws,
                                           ev_out=self.stats["ev_before"].view(1), ret_out=self._scan_ret,
                                           adv_out=self._scan_adv)
            if cfg.norm_adv and self.dp is not None:
                dp = self.dp
                self._comm(lambda: dp.allreduce_sum_(mom))   # moments [0:8] + the deferred KL [8:10]
                self._settle_kl()
                if not defer:
                    _native.require().normalize_mom(self._scan_adv, self._scan_adv, mom, 1e-8)
            if defer:
                self._norm_mom = mom
            self._scanned = True
            return self._scan_ret, self._scan_adv
        if cfg.returns == "gae":
            ret, adv = R.gae(st.rewards, st.values, dones, cfg.gamma, cfg.gae_lambda)
        else:
            ret, adv = R.nstep_returns(st.rewards, st.values, dones, cfg.gamma, cfg.look_ahead)
        return ret.reshape(-1), adv.reshape(-1)

    def _normalize(self, adv):
        if self.dp is not None:
            out = self.dp.normalize_advantages(adv, extra=self._kl_tail if self._kl_deferred() else None)
            self._settle_kl()
            return out
        if _native.use_native(adv):
            _native.require().normalize(adv.contiguous(), self.adv_buf, 1e-8)
            return self.adv_buf
        return R.normalize_advantages(adv)

    def _pre_learn_stats(self, ret, adv, v_old):
        """EV-before and advantage normalisation, unless the fused returns scan already produced both."""
        if getattr(self, "_scanned", False):
            return adv
        self._ev(ret, v_old, "ev_before")
        return self._normalize(adv) if self.cfg.norm_adv else adv

    def _ev(self, target, pred, slot):
        if _native.use_native(target):
            ws = getattr(self, "_scan_ws", None)   # many-workgroup form when the scan workspace exists
            _native.require().ev(target.contiguous(), pred.contiguous(), self.stats[slot].view(1),
                                 ws.ev_part if ws is not None else None, ws.ev_ticket if ws is not None else None)
        else:
            self.stats[slot].copy_(var_accounted_for_tensor(target, pred))

    # ------------------------------------------------------------------ learning (autograd engine)
    def _loss(self, obs, actions, logp_old, adv, ret, v_old=None):
        cfg = self.cfg
        logp, ent, v = self.model.evaluate(obs, actions)
        if cfg.algo == "ppo":
            a_loss, pg, kl, entm, clipfrac = L.ppo_actor_loss(logp, logp_old, adv, ent, cfg.ppo_clip, self.ent_coef,
                                                              self.kl_coef)
        else:
            a_loss, pg, kl, entm = L.actor_loss(logp, logp_old, adv, ent, self.kl_coef, self.ent_coef)
            clipfrac = torch.zeros((), device=self.device)
        c_loss = L.value_loss(v, ret, v_old, cfg.ppo_value_clip if cfg.algo == "ppo" else None)
        shared = "shared" in self.flat.groups
        total = a_loss + (cfg.vf_coef * c_loss if shared else c_loss)
        return total, a_loss, c_loss, kl, entm, clipfrac

    def _after_pull(self):
        """Parameters were replaced from outside (PS pull): clear the gradient slab the optimiser would have
        zeroed and refresh the engines' low-precision / transposed weight shadows."""
        self.flat.grad.zero_()
        if self.shadow is not None:
            self.shadow.copy_(self.flat.data)
        if self.engine is not None:
            self.engine.sync_frag()
        if self.mlp is not None:
            self.mlp.sync_shadow()

    def _comm(self, fn):
        """Runs a collective now (eager) or, while a :class:`SegmentRecorder` is capturing, records it as a cut
        between two graphs. ``fn`` must work in place on buffers that outlive the capture."""
        if self._rec is None:
            fn()
        else:
            self._rec.cut(fn)

    def _inline_comm(self):
        """DP collectives are recorded inside the update's hipGraph (RCCL) instead of cutting it (gloo)."""
        return (self.dp is not None and self.dp.graph_capturable and self.cfg.dp_capture != "segments"
                and self._grad_sink is None)

    def _inline_dp_overlap(self):
        """RCCL DP on the CNN engine: the gradient all-reduce is split into the fc-weight bucket (all-reduced while
        the conv backward runs) and the conv bucket. (Also with ``dp_capture="segments"``, where both are host
        cuts, so the two capture modes run the same kernels and stay bitwise equal.)"""
        return (self.engine is not None and self.dp is not None and self.dp.graph_capturable
                and self._grad_sink is None and not self._defer_allreduce and self._bw_stage == "all")

    def _backward_allreduce_overlapped(self, b, head_bias_done, head_done=False):
        """Backward + gradient all-reduce + optimiser for RCCL data parallelism, as ONE stream-ordered sequence that
        a hipGraph records whole: the fc-layer backward makes the tail bucket (the fc weight, 95 % of the bytes) final;
        its all-reduce is issued on RCCL's stream (a forked branch of the graph) while the conv backward runs on the
        compute stream; then the conv bucket is all-reduced and the compute stream joins both before the optimiser.
        Nothing is issued from the host at replay time."""
        eng, dp, g = self.engine, self.dp, self.flat.grad
        eng.backward(b, head_bias_done=head_bias_done, stage="tail", head_done=head_done)
        s, e = eng.tail_bucket()
        dp.pack(g, s, e)
        inline = self._inline_comm()
        if inline:
            w_tail = dp.allreduce_async(dp.comm_view(g, s, e))
        else:
            self._comm(lambda: dp.allreduce_packed(g, s, e))
        eng.backward(b, head_bias_done=head_bias_done, stage="trunk")
        dp.pack(g, 0, s)
        self._comm(lambda: dp.allreduce_packed(g, 0, s))
        if inline:
            w_tail.wait()
        dp.unpack(g)
        self._run_optimizers()

    def _apply_grads(self):
        """All-reduce (DP) + optimiser step; inside a segmented capture the pre-graph stops before both."""
        if self._defer_allreduce:
            return
        if self._grad_sink is not None:   # async PS worker (a3c_gpu): push the gradient, pull the parameters
            self._comm(self._grad_sink)
            self._after_pull()
            return
        if self.dp is not None:
            dp, g = self.dp, self.flat.grad
            dp.pack(g)                                   # bf16 buckets: captured cast into the comm buffer
            self._comm(lambda: dp.allreduce_packed(g))
            dp.unpack(g)
        self._run_optimizers()

    def _run_optimizers(self):
        """Optimiser step(s). Several groups (the reference's separate actor / critic Adam) run as ONE launch, which
        also writes the MLP engine's weight fragment copies; otherwise one launch per group (+ a copy pass)."""
        opts = list(self.opts.values())
        if len(opts) > 1 and _native.use_native(self.flat.data):
            from ..ops.optim import FusedGroupStep
            if not hasattr(self, "_group_step"):
                self._group_step = None
                if FusedGroupStep.compatible(opts):
                    copies = None
                    if self.mlp is not None and list(self.opts) == ["actor", "critic"]:
                        copies = self.mlp.frag_copies()
                    self._group_step = FusedGroupStep(opts, copies)
            if self._group_step is not None:
                t_off = getattr(self, "_t_off", None)
                if (self.mlp is not None and self.dp is not None and self.cfg.overlap != "lag1"
                        and self._grad_sink is None):
                    # strict DP on the MLP engine: the weight-gradient launch stores every element and the all-reduce
                    # runs in place, so nothing accumulates into the slab -- no zeroing pass behind the update
                    for o in opts:
                        o.zero_grad_after = not getattr(self.mlp, "last_stores_all", False)
                self._group_step.step(t_off=t_off)
                if t_off is not None:
                    self._t_offs_used += 1
                if self.mlp is not None and self._group_step._items[0] is None:
                    self.mlp.sync_shadow()
                return
        # the CNN engine's grouped A2C backward STORES every gradient element (head launch, dWfc GEMM, finaliser of the
        # conv planes and bias rows), so the optimiser need not zero the slab behind itself: one 6.75 MB write pass
        # less per update. Every other backward (atomics, accumulating GEMM epilogues, DP buckets) keeps the zeroing.
        # (DP: the all-reduce / bf16 unpack overwrite the slab in place; lag-1's grad_move zeroes G itself)
        stores_all = (self.engine is not None and self._grad_sink is None
                      and getattr(self.engine, "last_bwd_stores_all", False))
        for opt in opts:
            if self.engine is not None:
                opt.zero_grad_after = not stores_all
            opt.step()
        if self.mlp is not None:
            self.mlp.sync_shadow()

    def _epoch_perm(self, B, ep):
        """Keyed pseudo-random permutation of the batch for PPO epoch ``ep`` (envs/rng.py ``prp``; one native launch
        on GPU, key derived on the device from the update counter -> graph-capturable)."""
        if _native.use_native(self.update_counter):
            if not hasattr(self, "_perm_buf") or self._perm_buf.numel() != B:
                self._perm_buf = torch.empty(B, dtype=torch.int64, device=self.device)
            # reused across epochs: the previous epoch's consumers are already queued on the stream
            _native.require().prp_perm(self._perm_buf, self.policy_seed, self.update_counter.view(1), ep)
            return self._perm_buf
        key = E.rng.minibatch_key(self.policy_seed, self.update_counter, ep)
        return E.rng.prp(torch.arange(B, device=self.device, dtype=torch.int64), B, key)

    def _minibatches(self, B):
        """PPO minibatch index sets: one keyed permutation of the batch per epoch, split into contiguous slices."""
        cfg = self.cfg
        mb = B // cfg.ppo_minibatches
        for ep in range(cfg.ppo_epochs):
            perm = self._epoch_perm(B, ep)
            for k in range(cfg.ppo_minibatches):
                yield perm[k * mb:(k + 1) * mb]

    def learn(self, ret, adv):
        if self.mlp is not None:
            return self._learn_mlp(ret, adv)
        if self.engine is not None:
            return self._learn_native_update(ret, adv)
        cfg, st = self.cfg, self.storage
        obs, actions, logp_old = st.flat("obs"), st.flat("actions"), st.flat("logp")
        v_old = st.flat("values")
        adv = self._pre_learn_stats(ret, adv, v_old)
        if cfg.algo == "ppo":
            for sel in self._minibatches(obs.shape[0]):
                self.flat.zero_grad()
                total, a_loss, c_loss, kl, ent, cf = self._loss(obs[sel], actions[sel], logp_old[sel], adv[sel],
                                                                ret[sel], v_old[sel])
                total.backward()
                self._apply_grads()
        else:
            self.flat.zero_grad()
            total, a_loss, c_loss, kl, ent, cf = self._loss(obs, actions, logp_old, adv, ret)
            total.backward()
            self._apply_grads()
        self.stats["act_loss"].copy_(a_loss.detach())
        self.stats["crit_loss"].copy_(c_loss.detach())
        self.stats["entropy"].copy_(ent.detach())
        self.stats["clipfrac"].copy_(cf.detach())
        self.stats["kl"].copy_(kl.detach())
        self.update_counter += 1
        if self.lr_ctrl is not None or cfg.kl_coef > 0:
            self._post_update_kl(obs, actions, logp_old, ret)

    @torch.no_grad()
    def _post_update_kl(self, obs, actions, logp_old, ret):
        """KL proxy and EV on the *updated* parameters (``Basic_AC/run_AC.py:257-258``), then the lr rule."""
        logp, _, v = self.model.evaluate(obs, actions)
        self._kl_and_lr(logp_old, logp, ret, v)

    def _kl_deferred(self):
        """DP with global advantage normalisation: the post-update KL proxy is not all-reduced on its own but rides
        in the NEXT update's advantage-moments all-reduce (one packed fp64 collective per update for both, SURVEY
        §5.8). The KL-adaptive lr rule then runs right after that all-reduce -- before the next update's first
        optimiser step, the first place the rule's result is used, so the lr sequence is unchanged. Until then
        ``stats["kl"]`` holds this rank's KL; :meth:`flush_kl` settles a pending KL (checkpoints, end of train)."""
        return (self.dp is not None and self.cfg.norm_adv and self._kl_defer_on and not self._fused_returns()
                and (self.lr_ctrl is not None or self.cfg.kl_coef > 0))

    def _settle_kl(self):
        """Consumes the all-reduced deferred KL slot (no-op on the device when nothing was pending)."""
        if not self._kl_deferred():
            return
        t = self._kl_tail
        valid = t[1] > 0
        kl = (t[0] / torch.clamp(t[1], min=1.0)).float()
        self.stats["kl"].copy_(torch.where(valid, kl, self.stats["kl"]))
        if self.lr_ctrl is not None:
            self.lr_ctrl.update_(self.actor_opt.lr, kl, valid)
        t.zero_()

    @torch.no_grad()
    def flush_kl(self):
        """Settles a KL still waiting for the next moments all-reduce: one standalone all-reduce of the 2-slot
        tail. Collective: every rank calls it at the same point (save_checkpoint and the end of train do)."""
        if not self._kl_deferred():
            return
        self.dp.allreduce_sum_(self._kl_tail)
        self._settle_kl()

    def _kl_and_lr(self, logp_old, logp, ret, v):
        kl = ((logp_old - logp) ** 2).mean()
        if self._kl_deferred():
            self._kl_tail.copy_(torch.stack([kl.double(), torch.ones((), dtype=torch.float64, device=kl.device)]))
            self.stats["kl"].copy_(kl)   # this rank's value until the next moments all-reduce
            self._ev(ret, v, "ev_after")
            return
        if self.dp is not None:   # in-place device all-reduce: capturable as a segment cut
            dp, buf = self.dp, self._kl_buf
            buf.copy_(kl.reshape(1))
            self._comm(lambda: dp.allreduce_sum_(buf))
            kl = (buf / self.world).reshape(())
        self.stats["kl"].copy_(kl)
        self._ev(ret, v, "ev_after")
        if self.lr_ctrl is not None:
            self.lr_ctrl.update_(self.actor_opt.lr, kl)

    # ------------------------------------------------------------------ learning (native MLP engine)
    def _mlp_step(self, eng, B, idx, obs, actions, logp_old, adv, ret, v_old, perm=None, bump=None):
        cfg = self.cfg
        ppo = cfg.algo == "ppo"
        used = eng.train(obs, actions, logp_old, adv, ret, self.ent_coef, self.kl_coef, B, idx=idx, perm=perm, bump=bump,
                         v_old=v_old if ppo else None, vf_coef=1.0, ppo=ppo, ppo_clip=cfg.ppo_clip if ppo else 0.0,
                         v_clip=(cfg.ppo_value_clip or 0.0) if ppo else 0.0, stats=self.stats_buf,
                         clips=(cfg.clip_value, cfg.critic_clip_value), want_parts=self.dp is None)
        for t, g in enumerate(("actor", "critic")):
            self.opts[g].ext_parts = eng.parts[t] if used else None
        self._apply_grads()

    def _epoch_buffers(self, obs, actions, B):
        """Persistent minibatch-order copies of one epoch's PPO inputs (fixed addresses: graph-capturable)."""
        key = (B, obs.shape[1], tuple(actions.shape[1:]), actions.dtype)
        if getattr(self, "_epoch_key", None) != key:
            dev = obs.device
            self._epoch_bufs = dict(obs=torch.empty(B, obs.shape[1], device=dev),
                                    act=torch.empty((B,) + tuple(actions.shape[1:]), dtype=actions.dtype, device=dev),
                                    **{k: torch.empty(B, device=dev) for k in ("logp", "adv", "ret", "v")})
            self._epoch_key = key
        return self._epoch_bufs

    @torch.no_grad()
    def _learn_mlp(self, ret, adv):
        cfg, st, eng = self.cfg, self.storage, self.mlp
        obs, actions, logp_old = st.flat("obs"), st.flat("actions"), st.flat("logp")
        v_old = st.flat("values")
        adv = self._pre_learn_stats(ret, adv, v_old)
        adv, ret = adv.contiguous(), ret.contiguous()
        B = obs.shape[0]
        if cfg.algo == "ppo":
            mb = B // cfg.ppo_minibatches
            uc = self.update_counter.view(1)
            # the grouped Adam launches of this update know their step (t + j + 1 for minibatch j): no per-launch
            # step ticket, the counters advance once after the loop
            offsets = self.cfg.engine_opts.adam_step_offsets
            self._t_offs_used = 0
            g = self._epoch_buffers(obs, actions, B)
            for ep in range(cfg.ppo_epochs):
                # the epoch's rows in minibatch order (the keyed permutation, one gather launch): the train launches
                # read contiguous rows, with no index or permutation round trip ahead of their input tiles
                _native.require().mlp_epoch_gather(obs, actions, logp_old, adv, ret, v_old, g["obs"], g["act"],
                                                   g["logp"], g["adv"], g["ret"], g["v"], uc, ep, self.policy_seed)
                for k in range(cfg.ppo_minibatches):
                    last = ep == cfg.ppo_epochs - 1 and k == cfg.ppo_minibatches - 1
                    self._t_off = ep * cfg.ppo_minibatches + k if offsets else None
                    sl = slice(k * mb, (k + 1) * mb)
                    # the last minibatch's weight-gradient launch advances the update counter (no extra launch)
                    self._mlp_step(eng, mb, None, g["obs"][sl], g["act"][sl], g["logp"][sl], g["adv"][sl],
                                   g["ret"][sl], g["v"][sl], bump=self.update_counter if last else None)
            self._t_off = None
            if self._t_offs_used:
                assert self._t_offs_used == cfg.ppo_epochs * cfg.ppo_minibatches
                self._group_step.advance(self._t_offs_used)
        else:
            self._mlp_step(eng, B, None, obs, actions, logp_old, adv, ret, v_old)
            self.update_counter += 1
        if self.lr_ctrl is not None or cfg.kl_coef > 0:
            if not hasattr(self, "_eval_buf"):
                self._eval_buf = (torch.empty(B, device=self.device), torch.empty(B, device=self.device))
            logp, v = self._eval_buf
            eng.evaluate(obs, actions, logp, None, v)
            self._kl_and_lr(logp_old, logp, ret, v)

    # ------------------------------------------------------------------ learning (native engine)
    def _learn_native(self, obs, actions, logp_old, adv, ret, v_old, forward=True, obs_idx=None):
        cfg, eng = self.cfg, self.engine
        b = eng.bufs(obs.shape[0] if obs_idx is None else obs_idx.numel(), with_grad=True)
        ppo = cfg.algo == "ppo"
        vf = cfg.vf_coef if "shared" in self.flat.groups else 1.0
        if (forward and self._grad_sink is None and self._bw_stage == "all"
                and actions.dtype == torch.int32 and eng.ppo_head_ok(b.B)):
            # ONE head launch (z, loss, dz, dh, head gradient planes); the backward starts at the fc layer (DP: the
            # head planes are summed by the finaliser at the end of the bucketed backward, before the 2nd bucket)
            planes = eng.big_gemm_ok(b.B)   # the fc product's split-K planes go straight to the head launch
            eng.forward(obs, b, head=False, obs_idx=obs_idx, fc_parts=planes)
            eng.ppo_head(b, actions, logp_old, adv, ret, v_old, self.ent_coef, self.kl_coef, vf,
                         cfg.ppo_clip if ppo else 0.0, (cfg.ppo_value_clip or 0.0) if ppo else 0.0, self.stats_buf,
                         fc=eng.last_fc if planes else None)
            self._bw_pending = (b, True)
            if self._inline_dp_overlap():
                return self._backward_allreduce_overlapped(b, True, head_done=True)
            eng.backward(b, head_bias_done=True, stage="all", head_done=True)
            self._apply_grads()
            return
        if forward:
            eng.forward(obs, b, obs_idx=obs_idx)
        else:
            b.obs = obs  # activations were written by the rollout; dW1 re-gathers the frames
        # the loss kernel writes its statistics straight into stats_buf[0:7]
        eng.loss(b, actions, logp_old, adv, ret, v_old if ppo else None, self.ent_coef, self.kl_coef, vf,
                 cfg.ppo_clip if ppo else 0.0, cfg.ppo_value_clip if ppo else 0.0, stats=self.stats_buf)
        self._bw_pending = (b, False)
        if self._inline_dp_overlap():
            return self._backward_allreduce_overlapped(b, False)
        eng.backward(b, stage=self._bw_stage)   # gradient slab is clean: the optimiser zeroed it after its last use
        self._apply_grads()

    @torch.no_grad()
    def _learn_native_fused(self):
        """A2C on the rollout's activations: ONE loss launch (returns + EV + adv-norm + loss + dz + head-bias grad),
        the backward, the optimiser."""
        cfg, st, eng = self.cfg, self.storage, self.engine
        obs, actions, logp_old = st.flat("obs"), st.flat("actions"), st.flat("logp")
        T, N = st.T, st.N
        b = eng.bufs(T * N, with_grad=True)
        b.obs = obs
        if not hasattr(self, "_ret_w"):
            self._ret_w = torch.zeros(T * N, device=self.device)
            self._adv_w = torch.zeros(T * N, device=self.device)
        vf = cfg.vf_coef if "shared" in self.flat.groups else 1.0
        rets = dict(mode=1 if cfg.returns == "nstep" else 2, rew=st.rewards, val=st.values, dones=st.dones,
                    L=T if cfg.look_ahead is None else cfg.look_ahead, gamma=cfg.gamma, lam=cfg.gae_lambda,
                    norm_adv=cfg.norm_adv, ret_w=self._ret_w, adv_w=self._adv_w)
        head_done = eng.head_ok(T * N, N)
        if head_done:
            # loss + dz + the head's backward (dh, dWh, dbh, dbfc) in one launch
            boot, self._boot = getattr(self, "_boot", None), None
            # the per-env head's gradient planes are summed by this backward's finaliser (under DP at the end of the
            # "trunk" stage: the head / fc-bias gradients belong to the second bucket, engine.tail_bucket)
            eng.head_backward(b, actions, logp_old, self.ent_coef, self.kl_coef, vf, self.stats_buf, rets, boot=boot,
                              planes_ok=self._bw_stage in ("all", "tail"))
        else:
            eng.loss(b, actions, logp_old, None, None, None, self.ent_coef, self.kl_coef, vf, 0.0, 0.0,
                     stats=self.stats_buf, returns=rets)
        self._bw_pending = (b, True)
        if self._inline_dp_overlap():
            self._backward_allreduce_overlapped(b, True, head_done)
        else:
            eng.backward(b, head_bias_done=True, stage=self._bw_stage, head_done=head_done)
            self._apply_grads()
        self._last = (obs, actions, logp_old, self._ret_w)
        if not self._defer_allreduce:
            self._finish_learn()

    @torch.no_grad()
    def _learn_native_update(self, ret, adv):
        if ret is None:
            return self._learn_native_fused()
        cfg, st = self.cfg, self.storage
        obs, actions, logp_old = st.flat("obs"), st.flat("actions"), st.flat("logp")
        v_old = st.flat("values")
        adv = self._pre_learn_stats(ret, adv, v_old)
        if cfg.algo == "ppo":
            B = obs.shape[0]
            mb = B // cfg.ppo_minibatches
            if not hasattr(self, "_mb"):
                dev = self.device
                self._mb = dict(obs=torch.empty((mb,) + tuple(obs.shape[1:]), dtype=obs.dtype, device=dev),
                                act=torch.empty(mb, dtype=actions.dtype, device=dev),
                                logp=torch.empty(mb, device=dev), adv=torch.empty(mb, device=dev),
                                ret=torch.empty(mb, device=dev), v=torch.empty(mb, device=dev))
            m = self._mb
            if actions.dtype == torch.int32:
                # one launch per minibatch: the keyed epoch permutation evaluated in place + every row gathered
                ops = _native.require()
                uc = self.update_counter.view(1)
                args = [t.contiguous() for t in (obs, actions, logp_old, adv, ret, v_old)]
                if not hasattr(self, "_uc_ticket"):
                    self._uc_ticket = torch.zeros(1, dtype=torch.int32, device=self.device)
                # index mode: the minibatch's observations are read in place through their row indices (no copy)
                by_index = self.engine.obs_index_ok(mb) and args[0].is_contiguous()
                if by_index and "idx" not in m:
                    m["idx"] = torch.empty(mb, dtype=torch.int64, device=self.device)
                for ep in range(cfg.ppo_epochs):
                    for k in range(cfg.ppo_minibatches):
                        last = ep == cfg.ppo_epochs - 1 and k == cfg.ppo_minibatches - 1
                        # the last gather also advances the update counter (its last workgroup; no extra launch)
                        ops.mb_gather(*args, None if by_index else m["obs"], m["act"], m["logp"], m["adv"], m["ret"],
                                      m["v"], self.policy_seed, uc, ep, k * mb, getattr(self, "_norm_mom", None), 1e-8,
                                      self._uc_ticket if last else None, m["idx"] if by_index else None)
                        if by_index:
                            self._learn_native(args[0], m["act"], m["logp"], m["adv"], m["ret"], m["v"],
                                               obs_idx=m["idx"])
                        else:
                            self._learn_native(m["obs"], m["act"], m["logp"], m["adv"], m["ret"], m["v"])
                self._uc_bumped = True
            else:
                for sel in self._minibatches(B):
                    for key, src in (("obs", obs), ("act", actions), ("logp", logp_old), ("adv", adv), ("ret", ret),
                                     ("v", v_old)):
                        torch.index_select(src, 0, sel, out=m[key])
                    self._learn_native(m["obs"], m["act"], m["logp"], m["adv"], m["ret"], m["v"])
        else:
            self._learn_native(obs, actions, logp_old, adv.contiguous(), ret.contiguous(), v_old,
                               forward=not self._reuse_acts())
        self._last = (obs, actions, logp_old, ret)
        if not self._defer_allreduce:
            self._finish_learn()

    def _finish_learn(self):
        """Post-update KL / EV / adaptive lr (after the optimiser step)."""
        if self.engine is None:
            return
        if self.cfg.algo == "ppo" and not getattr(self, "_uc_bumped", False):
            self.update_counter += 1   # keys the minibatch permutations
        if self.lr_ctrl is not None or self.cfg.kl_coef > 0:
            obs, actions, logp_old, ret = self._last
            eng = self.engine
            b = eng.bufs(obs.shape[0], with_grad=True)
            z = eng.forward(obs, b)
            logp, _ = D.categorical_logp_entropy(z[:, :eng.A], actions)
            self._kl_and_lr(logp_old, logp, ret, z[:, eng.A])

    # ------------------------------------------------------------------ driver
    # Without DP the whole update is ONE captured hipGraph. With RCCL data parallelism it is ONE graph too: every
    # collective is recorded in it (RCCL calls are stream-ordered and capturable); the CNN engine's gradient
    # all-reduce is split into the fc-weight bucket, issued on RCCL's stream (a forked graph branch) while the conv
    # backward runs, and the conv bucket (_backward_allreduce_overlapped). The host issues nothing per replay.
    # Host-side collectives (gloo) cannot be captured, so there the update is split into captured segments around
    # them, issued from the host between replays (async w.r.t. the host: the stream waits, the CPU does not); the
    # same segment schedules serve RCCL lag-1 A2C, whose all-reduce spans two updates:
    #   overlap="strict" (exact synchronous A2C, the default):
    #       pre   = rollout + returns + loss + backward of the head and fc layers        (graph 1)
    #       AR(fc-weight bucket, 95% of the bytes) on the RCCL stream    || mid = conv backward (graph 2)
    #       AR(conv + head bucket) ; the main stream waits for both ; post = optimiser + stats    (graph 3)
    #   overlap="lag1" (policy lag 1, BASELINE's "all-reduce overlapped with the next rollout"):
    #       pre   = rollout + returns + loss + full backward into the gradient slab G     (graph 1)
    #               || AR(C) of the PREVIOUS update's gradient, issued at the end of the previous step
    #       wait ; post = optimiser step reading C (the previous gradient) + move G -> C, G = 0   (graph 2)
    #       AR(C) issued, overlapping the next update's rollout.
    #     Every gradient is on-policy for its batch (computed at the parameters that acted) and applied one update
    #     late (delayed-gradient SGD with staleness 1).
    # Capture selection (_capture_set, in this order):
    #   * the gloo / lag-1 A2C segment schedules above (_segmented);
    #   * RCCL (_inline_comm), every other algorithm and engine (PPO minibatch steps, global advantage moments, the
    #     KL-adaptive lr / KL proxy, the MLP engine): ONE graph per update with every collective recorded in it;
    #   * gloo DP outside the A2C schedules, or a gradient sink (A3C worker): a SegmentRecorder -- one graph chain
    #     per update cut at each host-issued collective;
    #   * no DP: one graph.
    # No DP configuration runs eagerly.

    def _can_capture(self):
        return self.cfg.cuda_graph and self.device.type == "cuda"

    def _a2c_dp_schedule(self):
        """The strict / lag-1 A2C data-parallel schedules apply (no batch-wide statistic inside the update)."""
        cfg = self.cfg
        return (self.dp is not None and cfg.algo == "a2c" and self.engine is not None and not cfg.norm_adv
                and self.lr_ctrl is None and cfg.kl_coef == 0.0)

    def _segmented(self):
        """The A2C strict / lag-1 schedules with host-issued collectives between captured segments (gloo). Under
        RCCL both are ONE graph per update (see _capture_set; lag-1: _update_body_lag1)."""
        if self._inline_comm():
            return False
        return self._a2c_dp_schedule()

    def _update_body_lag1(self):
        """RCCL lag-1 A2C as ONE captured graph per update, on PING-PONG gradient slabs: the graph set of ring phase p
        has the engine write G[p] and the optimiser read G[1-p]. The all-reduce of G[1-p] -- the PREVIOUS update's
        gradient -- is forked onto RCCL's stream at the start, so it runs under this update's rollout, loss and
        backward (which write G[p]); then G[1-p] is applied and G[p] packed for the next replay's all-reduce. No
        C <- G copy, and with a backward that stores every element no zeroing either (the optimiser clears the slab
        it read otherwise: the next backward into it accumulates). The optimiser launches are gated on a device flag
        (``_lag1_gate``) set at the end of every replay: the first replay after capture and the first after
        :meth:`flush_pending` hold no gradient in G[1-p] and apply nothing -- parameters, moments and the Adam step
        count unchanged, exactly as the segmented schedule's first update."""
        dp, G = self.dp, self._lag1_slabs
        p = self.storage.phase
        prev = G[1 - p]
        w = dp.allreduce_async(dp.comm_view(prev))
        self._defer_allreduce = True
        try:
            self.collect()
            ret, adv = self.compute_returns()
            self.learn(ret, adv)
        finally:
            self._defer_allreduce = False
        w.wait()
        dp.unpack(prev)
        self._post_body()
        self._lag1_gate.fill_(1)   # from the next replay on, the slab it reads holds a gradient
        dp.pack(G[p])
        self.storage.roll_over()

    def _bind_lag1_phase(self, p):
        """Engine writes G[p], optimisers read G[1-p] (the bf16 comm buffer of G[1-p] with direct reads)."""
        G = self._lag1_slabs
        self.engine.use_grad_slab(G[p])
        for opt in self.opts.values():
            opt.bind_grad(G[1 - p])
            if self.dp.direct_read:
                opt.bind_grad16(self.dp.comm_view(G[1 - p]))

    def update_body(self):
        with self.timer.phase("rollout"):
            self.collect()
        with self.timer.phase("returns"):
            ret, adv = self.compute_returns()
        with self.timer.phase("learn"):
            self.learn(ret, adv)
        self.storage.roll_over()

    def _post_body(self):
        self._run_optimizers()
        self._finish_learn()

    def _lag1(self):
        return self.cfg.overlap == "lag1"

    def _grad_move(self):
        """lag-1: C <- G, G <- 0 (one launch) so the next backward accumulates into a clean slab while C is
        all-reduced and consumed by the next optimiser step; the one-graph schedule's gate opens in the same launch."""
        gate = getattr(self, "_lag1_gate", None)
        # G needs no clearing when the next backward stores every gradient element (the CNN engine's grouped
        # backward: head launch, fc_bwd, finaliser planes)
        zero = not (self.engine is not None and getattr(self.engine, "last_bwd_stores_all", False))
        if _native.use_native(self.flat.grad):
            _native.require().grad_move(self.flat.grad, self._comm_grad, gate, zero)
        else:
            self._comm_grad.copy_(self.flat.grad)
            if zero:
                self.flat.grad.zero_()
            if gate is not None:
                gate.fill_(1)

    def capture(self, warmup=2):
        """Capture the update as hipGraph(s) (see above). Warm-up updates run first (GEMM autotuning, allocator)."""
        if not self._can_capture():
            return None
        self.timer.suspended = True
        try:
            return self._capture(warmup)
        finally:
            self.timer.suspended = False

    def _bind_comm_grad(self):
        """lag-1: the optimisers read C, the all-reduced copy of the previous update's gradient."""
        if self._comm_grad is None:   # one buffer shared by both ring-phase graph sets
            self._comm_grad = torch.zeros_like(self.flat.grad)
            for opt in self.opts.values():
                opt.bind_grad(self._comm_grad)
                if self.dp.direct_read:   # bf16 buckets read in place: C's own comm buffer
                    opt.bind_grad16(self.dp.comm_view(self._comm_grad))
            self.dp.pack(self._comm_grad)

    def _capture(self, warmup):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(max(1, warmup)):
                self.update_body()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.check_health()
        st = self.storage
        if st.ring:
            # one graph set per ring phase (their slot addresses differ); capturing runs nothing, and each set
            # flips the host-side phase once, so after both captures host phase == device state again
            p0 = st.phase
            first = self._capture_set()
            second = self._capture_set()
            assert st.phase == p0
            self._graph_sets = {p0: first, 1 - p0: second}
            self.graph = first
            return self.graph
        self.graph = self._capture_set()
        return self.graph

    def _capture_set(self):
        if self._segmented():
            self._defer_allreduce = True
            try:
                if self._lag1():
                    self._bind_comm_grad()
                    g1 = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g1, capture_error_mode=CAPTURE_MODE):
                        self.update_body()
                    g2 = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g2, capture_error_mode=CAPTURE_MODE):
                        self.dp.unpack(self._comm_grad)     # bf16 buckets: the all-reduced sum back into C
                        self._post_body()
                        self._grad_move()
                        self.dp.pack(self._comm_grad)
                    graph = ("lag1", g1, g2)
                else:
                    self._bw_stage = "tail"
                    g1 = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g1, capture_error_mode=CAPTURE_MODE):
                        self.collect()
                        ret, adv = self.compute_returns()
                        self.learn(ret, adv)
                        self.dp.pack(self.flat.grad, *self.engine.tail_bucket())
                    self._bw_stage = "all"
                    b, hb = self._bw_pending
                    g2 = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g2, capture_error_mode=CAPTURE_MODE):
                        self.engine.backward(b, head_bias_done=hb, stage="trunk")
                        self.dp.pack(self.flat.grad, 0, self.engine.tail_bucket()[0])
                    g3 = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g3, capture_error_mode=CAPTURE_MODE):
                        self.dp.unpack(self.flat.grad)
                        self._post_body()
                        self.storage.roll_over()
                    graph = ("strict", g1, g2, g3)
            finally:
                self._defer_allreduce = False
                self._bw_stage = "all"
        elif self._inline_comm():
            # RCCL: every collective of the update (gradient buckets per optimiser step, the advantage moments, the
            # KL scalar; lag-1: the previous gradient's all-reduce) is recorded in the graph -- one replay per
            # update, zero host-issued collectives
            lag1 = self._lag1() and self._a2c_dp_schedule()
            if lag1:
                if getattr(self, "_lag1_slabs", None) is None:   # G[0] is the slab the engine was built on
                    self._lag1_slabs = [self.flat.grad, torch.zeros_like(self.flat.grad)]
                    for g in self._lag1_slabs:
                        self.dp.prepare(g)
                        self.dp.pack(g)
                if getattr(self, "_lag1_gate", None) is None:   # closed: no slab holds a gradient yet
                    self._lag1_gate = torch.zeros(1, dtype=torch.int32, device=self.device)
                    for opt in self.opts.values():
                        opt.set_gate(self._lag1_gate)
                self._bind_lag1_phase(self.storage.phase)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                if lag1:
                    self._update_body_lag1()
                else:
                    self.update_body()
            self._lag1_inline = lag1
            graph = ("single", g)
        elif self.dp is not None or self._grad_sink is not None:
            rec = SegmentRecorder()
            self._rec = rec
            try:
                rec.start()
                self.update_body()
                rec.finish()
            except BaseException:
                rec.abort()
                raise
            finally:
                self._rec = None
            graph = ("segments", rec)
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                self.update_body()
            graph = ("single", g)
        return graph

    def _replay(self):
        st = self.storage
        graph = self._graph_sets[st.phase] if st.ring else self.graph
        self._replay_set(graph)
        if st.ring:
            st.phase ^= 1   # the replayed update ended with its rollover
        if getattr(self, "_env_flips", 0) & 1:   # the fused rollout steps alternated the env's state slots
            self.env.flip()

    def _replay_set(self, graph):
        kind = graph[0]
        if kind == "single":
            graph[1].replay()
        elif kind == "segments":
            graph[1].replay()
        elif kind == "strict":
            _, g1, g2, g3 = graph
            s, e = self.engine.tail_bucket()
            g1.replay()
            w_tail = self.dp.allreduce_async(self.dp.comm_view(self.flat.grad, s, e))   # overlaps the conv backward
            g2.replay()
            w_trunk = self.dp.allreduce_async(self.dp.comm_view(self.flat.grad, 0, s))
            w_tail.wait()
            w_trunk.wait()
            g3.replay()
        else:   # lag1
            _, g1, g2 = graph
            g1.replay()                       # overlaps the all-reduce of the previous gradient
            if self._comm_work is None:       # first update: nothing to apply yet
                self._grad_move()
                self.dp.pack(self._comm_grad)
            else:
                self._comm_work.wait()
                g2.replay()
            self._comm_work = self.dp.allreduce_async(self.dp.comm_view(self._comm_grad))

    def step(self):
        """One update (graph replay when captured)."""
        if self.graph is not None:
            with self.timer.phase("update_graph"):
                self._replay()
        else:
            self.update_body()
        if self.cfg.lr_schedule == "linear":
            self._decay_lr(self.iteration + 1)
        if self.reg_sched is not None:
            # after update i, as the reference (Basic_AC/run_AC.py:268-275): a new coefficient acts from i + 1 on
            e, k = self.reg_sched.entropy_coef(self.iteration), self.reg_sched.kl_coef(self.iteration)
            if e is not None:
                self.ent_coef.fill_(e)
            if k is not None:
                self.kl_coef.fill_(k)
        self.iteration += 1
        self.env_steps += self.cfg.n_steps * self.env.num_envs * self.world

    def _decay_lr(self, it):
        """Linear lr decay (``lr_schedule="linear"``): update ``it`` runs with lr0 * (1 - it / total_updates). One
        device scalar write per optimiser between replays (the captured update reads lr from device memory)."""
        frac = max(0.0, 1.0 - it / max(1, self.cfg.total_updates))
        for g, opt in self.opts.items():
            if g == "critic" or self.lr_ctrl is None or opt is not self.actor_opt:
                base = self.cfg.critic_lr if g == "critic" else self.cfg.lr
                opt.lr.fill_(base * frac)

    def flush_pending(self):
        """lag-1 DP: apply the last all-reduced gradient (end of training / before a checkpoint)."""
        if self.graph is not None and getattr(self, "_lag1_inline", False):
            # the one-graph schedule leaves the last update's gradient packed in G[q] (its all-reduce would open the
            # next replay): all-reduce and apply it now (eagerly, the optimisers pointed at G[q]), then G[q] = 0 and
            # the gate closed (the next replay applies nothing twice)
            q = 1 - self.storage.phase   # the last replay's phase (its rollover flipped the ring)
            last = self._lag1_slabs[q]
            self.dp.allreduce_packed(last)
            self.dp.unpack(last)
            self._bind_lag1_phase(1 - q)   # optimisers read G[q]
            self._post_body()
            last.zero_()
            self._lag1_gate.zero_()   # the next replay's optimiser step has nothing to apply
            self.dp.pack(last)
            return
        if self.graph is not None and self.graph[0] == "lag1" and self._comm_work is not None:
            self._comm_work.wait()
            self.dp.unpack(self._comm_grad)
            self._post_body()
            self._comm_grad.zero_()
            self._comm_work = None

    def log(self, i, print_tog, ep_stats=None):
        """One Logger row. ``ep_stats`` = (mean return, episodes, mean length) already drained by the caller (the
        async worker shares one drain between its consumers); else the env bank's counters are drained here."""
        if self.logger is None:
            return None
        self.check_health()
        vals = self.stats_buf.detach().cpu().tolist()
        s = {k: vals[STAT_KEYS.index(k)] for k in LOG_KEYS}
        avg_rew, n_ep, ep_len = ep_stats if ep_stats is not None else self.env.drain_episode_stats()
        self.logger(i, act_loss=s["act_loss"], circ_loss=math.sqrt(max(s["crit_loss"], 0.0)), kl_dist=s["kl"],
                    avg_rew=avg_rew, print_tog=print_tog, act_lr=self.actor_opt.get_lr(), avg_ent=s["entropy"],
                    worker_id=self.worker_id, ev_before=s["ev_before"], ev_after=s["ev_after"])
        s.update(avg_rew=avg_rew, episodes=n_ep, ep_len=ep_len)
        if self._kl_deferred():
            # DP + global advantage normalisation: this row's kl is rank 0's local post-update KL and act_lr the value
            # before the KL-adaptive rule, which settles inside the NEXT update's moments all-reduce (_kl_deferred);
            # the lr sequence used for training is the single-GPU one, the logged columns lag it by one update
            s["kl_lr_presettle"] = 1
        return s

    def check_health(self, collective=False):
        """Raises if a native in-launch hand-off timed out (its outputs, and so this update's gradients, would be
        corrupt). One host read; called at log / checkpoint time, after the capture warm-up and at the end of
        ``train``. ``collective`` (DP, at points every rank reaches: checkpoints, end of train): the flag is
        max-all-reduced first, so every rank raises together instead of the healthy ones waiting in the next
        collective until ``dist_timeout_s``."""
        errs = self.engine.health_errors() if self.engine is not None else []
        if collective and self.dp is not None:
            flag = torch.tensor([1.0 if errs else 0.0], device=self.device)
            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MAX, group=self.dp.group)
            if float(flag) > 0 and not errs:
                errs = ["a peer rank's native hand-off"]
        if errs:
            raise RuntimeError("native engine hand-off timed out (" + ", ".join(errs) + "): the affected "
                               "updates trained on incomplete data")

    def train(self, num_updates=None, callback=None):
        cfg = self.cfg
        if self._fault is not None and len(self._fault) == 3:
            raise ValueError(f"fault_inject {cfg.fault_inject!r}: the 'push' / 'reply' fault points belong to the "
                             "async parameter-server worker (a3c_gpu); the synchronous trainer takes 'rank:iteration'")
        n = cfg.total_updates if num_updates is None else num_updates
        if self._can_capture() and self.graph is None:
            self.capture()
        t0 = time.time()
        history = []
        for _ in range(n):
            self._maybe_fault()
            self.step()
            it = self.iteration - 1
            if cfg.stdout_freq and it % cfg.stdout_freq == 0:
                s = self.log(it, print_tog=not cfg.quiet)
                if s is not None:
                    history.append(dict(iteration=it, **s))
                    el = time.time() - t0
                    extra = {"phase_ms": self.timer.summary()} if cfg.trace else {}
                    self.logger.log_metrics(iteration=it, env_steps=self.env_steps,
                                            env_steps_per_sec=self.env_steps / max(el, 1e-9), **extra, **s)
                if self.tb is not None:
                    self.tb.write(it, extra=self._tb_scalars(s))
                if cfg.mode.startswith("debug") and (cfg.mode != "debug-light" or self.rank == 0):
                    self._debug_print()
            if self.logger is not None and cfg.flush_every and it % cfg.flush_every == cfg.flush_every // 2:
                self.logger.flush()
            if cfg.save_every and it % cfg.save_every == 0 and cfg.checkpoint_dir and \
                    (self.rank == 0 or self.dp is not None):   # DP: every rank takes part (env-state gather)
                self.save_checkpoint()
            if callback is not None:
                callback(self, it)
        self.flush_pending()
        self.flush_kl()
        self.check_health(collective=True)
        return history

    # ------------------------------------------------------------------ checkpoints
    def save_checkpoint(self, path=None):
        # the collective flush first: a rank whose hand-off timed out raises only after its peers left the
        # all-reduce, so they reach their own check (or the next collective's error) instead of waiting out
        # dist_timeout_s in a collective this rank never joins
        self.flush_kl()
        self.check_health(collective=True)
        from ..ckpt import save_trainer
        return save_trainer(self, path)

    def load_checkpoint(self, path):
        from ..ckpt import load_trainer
        return load_trainer(self, path)

    def close(self):
        if self.logger is not None:
            self.logger.close()
        if self.tb is not None:
            self.tb.close()

    # ------------------------------------------------------------------ observability / failure hooks
    def _maybe_fault(self):
        """SURVEY §5.3 fault injection: ``fault_inject="rank:iteration"`` kills this process -- no cleanup, no
        collective goodbye, as a crashed host would -- when it is about to run that iteration. The surviving ranks'
        next collective raises (gloo: peer closed; RCCL: ``dist_timeout_s``), and ``resume="auto"`` restarts the job
        from the newest checkpoint."""
        if self._fault is not None and self._fault == (self.rank, self.iteration):
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(FAULT_EXIT_CODE)

    def _summary_scopes(self):
        """The reference's per-variable summary scopes (``Basic_AC/policies.py:83-85,146-149``) for the MLP family;
        one ``ActorCritic`` scope over every parameter otherwise."""
        from ..models.policy import MLPActorCritic
        from ..utils.tensorboard import reference_summary_scopes
        if isinstance(self.model, MLPActorCritic):
            return reference_summary_scopes(self.model.actor, self.model.critic)
        return [("ActorCritic", list(self.model.parameters()))]

    def _tb_scalars(self, s):
        if s is None:
            vals = self.stats_buf.detach().cpu().tolist()
            s = {k: vals[STAT_KEYS.index(k)] for k in LOG_KEYS}
        return {"train/" + k: float(v) for k, v in s.items() if isinstance(v, (int, float))}

    @torch.no_grad()
    def _debug_print(self):
        """``--mode debug`` (``debug-light``: rank 0 only, ``debug-full``: every rank): the reference's printer block
        (``Basic_AC/policies.py:87-89,144-145``; ``A3C/process.py:250-256``) -- per-variable means (one statistics
        launch over the parameter slab) and a strided sample of predicted values, log-probs and returns."""
        from ..ops.stats import param_segments, seg_stats
        params = list(self.model.parameters())
        means = seg_stats(self.flat.data, param_segments(self.flat, params))[:, 0].cpu().tolist()
        st = self.storage
        n = st.T * self.env.num_envs
        idx = torch.arange(20, device=st.values.device) * max(1, n // 20) % n
        print("[rank %d] Variable data" % self.rank, [round(m, 6) for m in means])
        print("[rank %d] Some preds" % self.rank, st.values[:st.T].reshape(-1)[idx].cpu().numpy())
        print("[rank %d] Some logps" % self.rank, st.logp.reshape(-1)[idx].cpu().numpy())
        print("[rank %d] Some rewards" % self.rank, st.rewards.reshape(-1)[idx].cpu().numpy(), flush=True)
