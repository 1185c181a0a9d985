"""GPU-native asynchronous parameter-server training (the reference's A3C, ``A3C/process.py:156-288``, redesigned
for MI355X: SURVEY §2.2 D03/D04/X04, §5.8).

Roles (ranks ``0 .. ps_num-1`` are parameter servers, the rest workers, as :mod:`.a3c`):

* **worker**: a vectorised trainer (:class:`.trainer.ActorCriticTrainer`, algo ``a2c``) that owns a device env bank
  (``num_envs`` envs, global env ids ``task * num_envs + i``) and the device engines (native MLP / CNN engine,
  hipGraph capture). One iteration = rollout ``[T, N]`` + returns + loss + backward exactly as the synchronous
  trainer, but the optimiser step is replaced by the **exchange**: the gradient slab (and the worker's own
  KL-adaptive actor lr) is pushed to every PS shard, the updated parameters and the global step are pulled back
  (the reference's ``apply_gradients`` on the global variables + ``sync_w_global``). Under capture the exchange is a
  segment cut (:class:`.trainer.SegmentRecorder`): rollout..backward and the post-pull work replay as graphs, the
  exchange runs between them.
* **parameter server**: holds a contiguous shard of the flat fp32 parameter slab and its Adam moments ON ITS
  DEVICE, and applies each request with the fused native Adam kernel (actor segment element-clipped +-clip_value
  with the sender's lr, critic segment with the critic lr), one request at a time -- applies are serialised, so the
  reference's Hogwild races on the PS variables cannot happen. Adam's bias-correction step count is
  kept PER WORKER (each reference worker builds its own Adam, whose beta powers advance only with its own applies).

Transport: a gloo **control plane** (int64 headers, ``recv`` from any source, so the PS serves whichever worker
asks first; the PS's reply header carries the global step, so a worker never reads the device to learn it) and a
**data plane** for the payloads: ``"nccl"`` = RCCL point-to-point ``send/recv`` of device tensors (over xGMI
between GPUs of a node; needs one GPU per rank), or ``"gloo"`` = the same messages staged through host memory (CPU
runs, several ranks sharing one GPU). A PS apply is ONE native launch (``opt_multi``: the shard's actor and critic
segments with their own lr / clip / per-worker step count; the actor lr is read straight from the payload slot the
worker filled). Bounded staleness (stale-synchronous parallel): with ``max_staleness = s`` a PS defers a worker's
apply while that worker is more than ``s`` applies ahead of the slowest live worker. While one worker computes a
gradient, another can first catch up (it may trail by up to ``s + 1`` applies) and then run ``s + 1`` applies
ahead, so a gradient is never older than ``2 (W - 1) (s + 1)`` global steps; ``s < 0`` disables the bound (the
reference's unbounded asynchrony). Every apply is logged as (worker, pulled version, global step).

Chief duties and logs (``A3C/process.py:211-214,280-283``, ``A3C/train.py:39``): worker 0 writes the global
actor/critic as a TF bundle ``<checkpoint_dir>/model-<Env>-<global step>`` every ``save_every`` global steps (the
reference's ``CheckpointSaverHook``; reference variable names, so ``cli/test_model.py`` evaluates it) and every
worker keeps a reference-format Logger file ``<log_dir>/worker_<task>.log``.

Failure handling: a worker that dies mid-run (``fault_inject="rank:iteration"`` at the start of an
iteration; ``"rank:iteration:push"`` after its push header, before the payload; ``"rank:iteration:reply"`` after the
push, before the PS's reply) makes the PS's next exchange with it fail -- gloo reports the closed peer, or the group
timeout expires -- and the PS returns an ``"aborted"`` summary instead of waiting forever or raising; the surviving
workers' exchange with the departed PS raises, so every process of the job ends.
"""
from __future__ import annotations

import os
import sys
import time

import torch
import torch.distributed as dist

from .. import envs as E
from ..ops.optim import make_optimizer

CMD_PULL, CMD_APPLY, CMD_DONE, CMD_REPLY = 1, 2, 3, 4
PAY_ALIGN = 8   # payload slots: the actor lr sits after the gradient, padded to a 32-byte boundary


def _pay_len(n):
    return (n + PAY_ALIGN - 1) // PAY_ALIGN * PAY_ALIGN + PAY_ALIGN


class _PeerLost(Exception):
    """A control-plane receive on the PS failed: a worker departed (closed peer or group timeout)."""


def shard_ranges(flat, ps_num):
    """Contiguous slab ranges, one per PS, cut at parameter boundaries and balanced by element count."""
    bounds = [off + p.numel() for p, off in zip(flat.params, flat.offsets)]
    total = flat.numel
    cuts = [0]
    for s in range(1, ps_num):
        target = total * s / ps_num
        c = min(bounds, key=lambda b: abs(b - target))
        cuts.append(max(c, cuts[-1]))
    cuts.append(total)
    return [(cuts[i], cuts[i + 1]) for i in range(ps_num)]


class _Planes:
    """Control plane (gloo, CPU headers) + data plane (RCCL device tensors, or gloo via host staging)."""

    def __init__(self, ctrl, data, data_backend, device):
        self.ctrl, self.data, self.backend, self.device = ctrl, data, data_backend, device

    def send_hdr(self, vals, dst):
        dist.send(torch.tensor(vals, dtype=torch.int64), dst=dst, group=self.ctrl)

    def recv_hdr(self, src=None):
        h = torch.zeros(4, dtype=torch.int64)
        s = dist.recv(h, src=src, group=self.ctrl)
        return s, [int(x) for x in h]

    def send(self, t, dst):
        if self.backend == "nccl":
            dist.send(t, dst=dst, group=self.data)
        else:
            dist.send(t.detach().to("cpu"), dst=dst, group=self.data)

    def recv(self, t, src):
        if self.backend == "nccl":
            dist.recv(t, src=src, group=self.data)
        else:
            h = torch.empty(t.shape, dtype=t.dtype)
            dist.recv(h, src=src, group=self.data)
            t.copy_(h)


def _build_flat(cfg, device):
    """Model + flat slab exactly as a worker's trainer builds them (same seed -> same initial values)."""
    from ..models.policy import build_model
    from ..ops.optim import FlatParams
    fs = 4 if ("Pong" in cfg.env or "Breakout" in cfg.env) else cfg.frames   # as ActorCriticTrainer
    env = E.make(cfg.env, 1, device=device, seed=cfg.seed, frame_stack=fs)
    model = build_model(env, cfg.model, cfg.model_variant, seed=cfg.seed).to(device)
    return FlatParams(model.param_groups(), device)


class DeviceParameterServer:
    def __init__(self, cfg, sid, rng_, worker_ranks, planes, device, max_staleness=-1):
        self.cfg, self.sid = cfg, sid
        self.s, self.e = rng_
        self.n = self.e - self.s
        self.device = torch.device(device)
        self.flat = _build_flat(cfg, self.device)
        self.planes = planes
        self.workers = list(worker_ranks)
        self.live = set(self.workers)
        self.max_staleness = max_staleness
        # optimiser segments = (group, start, end) of this shard, with their own Adam moments
        self.segs = []
        for g, (gs, ge) in list(self.flat.groups.items()):
            a, b = max(gs, self.s), min(ge, self.e)
            if a >= b:
                continue
            name = f"ps{sid}_{g}"
            self.flat.groups[name] = (a, b)
            actor = g != "critic"
            # element-wise clipping only (A3C/policies.py:85): a global-norm clip would be taken per shard here
            opt = make_optimizer("adam", self.flat, name, cfg.lr if actor else cfg.critic_lr,
                                 cfg.clip_value if actor else cfg.critic_clip_value, None)
            self.segs.append((opt, a - self.s, b - self.s, actor))
        # per-worker Adam step counts (bias correction advances with that worker's applies only)
        self.t = {(k, w): torch.zeros((), dtype=torch.float32, device=self.device)
                  for k in range(len(self.segs)) for w in self.workers}
        self.n_applies = {w: 0 for w in self.workers}
        self.global_step = 0
        self.log = []   # (worker rank, version the gradient was computed at, global step before the apply)
        self.status = "ok"
        self._pay = {w: torch.zeros(_pay_len(self.n), device=self.device) for w in self.workers}
        self._steppers = {w: self._stepper(w) for w in self.workers}

    def _stepper(self, w):
        """The apply of worker ``w``'s payload: per segment a shallow view of the shard optimiser whose gradient is
        the payload slice, whose step count is ``w``'s own and (actor segments) whose lr is the payload's lr slot --
        all segments in ONE ``opt_multi`` launch on a GPU (moments and parameters are the shared ones)."""
        import copy
        from .. import _native
        from ..ops.optim import FusedGroupStep
        buf = self._pay[w]
        lr_slot = buf[_pay_len(self.n) - PAY_ALIGN]
        views = []
        for k, (opt, a, b, actor) in enumerate(self.segs):
            o = copy.copy(opt)
            o.g = buf[a:b]
            o.t = self.t[(k, w)]
            if actor:
                o.lr = lr_slot
            views.append(o)
        if _native.use_native(self.flat.data):
            return FusedGroupStep(views).step   # opt_multi takes 1..OPT_MAXSEG segments
        return lambda: [o.step() for o in views]

    # -- one apply ------------------------------------------------------------------------------------------------
    @torch.no_grad()
    def apply(self, w, version):
        self._steppers[w]()
        if self.flat.data.is_cuda:
            # an asynchronous device fault of the optimiser launch surfaces HERE (outside the peer I/O), not inside
            # the reply's send, where it would be reported as a departed worker
            torch.cuda.current_stream(self.flat.data.device).synchronize()
        self.log.append((w, version, self.global_step))
        self.global_step += 1
        self.n_applies[w] += 1

    def reply(self, w):
        """Reply header (global step, on the control plane) + the shard's parameters (data plane)."""
        self.planes.send_hdr([CMD_REPLY, self.sid, self.global_step, 0], w)
        self.planes.send(self.flat.data[self.s:self.e], w)

    def _allowed(self, w):
        if self.max_staleness < 0 or len(self.live) <= 1:
            return True
        slowest = min(self.n_applies[v] for v in self.live)
        return self.n_applies[w] - slowest <= self.max_staleness

    def serve(self):
        """Serves until every worker said DONE. A failed exchange with a worker -- the control-plane header receive,
        the payload receive after a push header, or the reply (header + parameters) to a worker -- means the worker
        died (gloo reports the closed peer, or the group timeout expired) and ends the PS with ``status ==
        "aborted"`` instead of a hang or an exception. Only peer I/O is treated as a departure: a failure of the
        apply (optimiser launch) propagates, so a kernel error on the PS is never reported as a worker death."""
        try:
            self._serve()
        except _PeerLost as e:
            self.status = "aborted"
            self.error = repr(e.__cause__)

    @staticmethod
    def _peer_io(fn, *args):
        """One exchange with a worker; a transport error (gloo: peer closed / timeout -- DistBackendError is a
        RuntimeError) becomes :class:`_PeerLost`."""
        try:
            return fn(*args)
        except RuntimeError as e:
            raise _PeerLost() from e

    def _recv_hdr(self):
        return self._peer_io(self.planes.recv_hdr)

    def _reply(self, w):
        self._peer_io(self.reply, w)

    def _apply_and_reply(self, w, v):
        self.apply(w, v)      # not peer I/O: errors propagate
        self._reply(w)

    def _serve(self):
        pending = []   # deferred applies (stale-synchronous bound), served in arrival order once allowed
        while self.live or pending:
            if self.live:
                src, (cmd, _task, version, _) = self._recv_hdr()
                if cmd == CMD_DONE:
                    self.live.discard(src)
                elif cmd == CMD_PULL:
                    self._reply(src)
                else:
                    self._peer_io(self.planes.recv, self._pay[src], src)
                    pending.append((src, version))
            progressed = True
            while progressed:
                progressed = False
                for i, (w, v) in enumerate(pending):
                    if self._allowed(w) or not self.live - {w}:
                        pending.pop(i)
                        self._apply_and_reply(w, v)
                        progressed = True
                        break
            if not self.live and pending:   # every other worker finished: nothing left to wait for
                for w, v in pending:
                    self._apply_and_reply(w, v)
                pending = []


class GPUWorker:
    """A vectorised device trainer whose optimiser step is the PS exchange."""

    def __init__(self, cfg, task, ranges, ps_ranks, planes, device, log_dir=None, rank=None, logger=None,
                 checkpoint_basename=None):
        from .trainer import ActorCriticTrainer
        from ..utils.logger import Logger
        self.cfg, self.task = cfg, task
        self.rank = rank if rank is not None else task
        self.ranges, self.ps_ranks, self.planes = ranges, ps_ranks, planes
        self.device = torch.device(device)
        wcfg = cfg.replace(algo="a2c", device=str(self.device), outdir=None)
        fs = 4 if ("Pong" in cfg.env or "Breakout" in cfg.env) else cfg.frames
        env = E.make(cfg.env, cfg.num_envs, device=self.device, seed=cfg.seed, env_offset=task * cfg.num_envs,
                     frame_stack=fs)
        self.tr = ActorCriticTrainer(wcfg, env=env)
        self.tr._grad_sink = self._exchange
        self.tr.worker_id = task
        if logger is not None:   # the caller's Logger (compat.process_fn's ``logger`` argument)
            self.tr.logger = logger
        elif log_dir:   # A3C/train.py:39: tmp/logs/worker_<i>.log, one per worker
            self.tr.logger = Logger(os.path.join(log_dir, f"worker_{task}.log"), quiet=cfg.quiet)
        self.ckpt_base = checkpoint_basename
        self.version = 0
        self._die_at = None   # mid-exchange fault point armed by run() (fault_inject "rank:iter:push|reply")
        n = [e - s for s, e in ranges]
        self._pay = [torch.zeros(_pay_len(k), device=self.device) for k in n]
        self.saved = []

    @torch.no_grad()
    def _exchange(self, pull_only=False):
        """Push the gradient + this worker's actor lr to every shard, pull the parameters back. The global step
        comes in the PS's reply header (host memory), so nothing here reads the device."""
        tr = self.tr
        flat = tr.flat
        lr = tr.actor_opt.lr
        for sid, ((s, e), r) in enumerate(zip(self.ranges, self.ps_ranks)):
            self.planes.send_hdr([CMD_PULL if pull_only else CMD_APPLY, self.task, self.version, 0], r)
            if not pull_only and self._die_at == "push":   # fault point: the header is out, the payload never comes
                self._die()
            if not pull_only:
                p = self._pay[sid]
                p[:e - s].copy_(flat.grad[s:e])
                p[p.numel() - PAY_ALIGN:p.numel() - PAY_ALIGN + 1].copy_(lr.reshape(1))
                self.planes.send(p, r)
        if not pull_only and self._die_at == "reply":   # fault point: pushed, dies before the PS's reply
            self._die()
        version = 0
        for sid, ((s, e), r) in enumerate(zip(self.ranges, self.ps_ranks)):
            _, (cmd, _sid, gstep, _) = self.planes.recv_hdr(r)
            assert cmd == CMD_REPLY, cmd
            self.planes.recv(flat.data[s:e], r)
            if sid == 0:
                version = gstep   # global step of PS 0 (the shard that also counts the actor applies)
        self.version = version
        return version

    @staticmethod
    def _die():
        from .trainer import FAULT_EXIT_CODE
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(FAULT_EXIT_CODE)

    def run(self, total_updates, report_every=0):
        """Trains until the PS global step reaches ``total_updates``. Returns the global step after each of this
        worker's updates; with ``report_every`` also (update, global step, mean finished-episode return) rows in
        ``self.returns`` (a host read of the env bank's episode statistics every ``report_every`` updates). Worker
        0 (the chief) checkpoints every ``save_every`` global steps; each worker logs reference-format rows."""
        from .trainer import parse_fault
        cfg, tr = self.cfg, self.tr
        fault = parse_fault(cfg.fault_inject)
        self._exchange(pull_only=True)   # initial sync_w_global (reference bug #12 fixed)
        tr._after_pull()
        if tr._can_capture():
            tr.capture(warmup=1)
        hist = []
        self.returns = []
        last_mark = -1
        i = 0
        # the env bank's episode counters are drained ONCE per iteration in which any consumer reads them, into one
        # accumulator per consumer, so the `returns` rows and the worker log each see every finished episode
        acc = {"report": [0.0, 0, 0.0], "log": [0.0, 0, 0.0]}

        def take(key):
            s, n, ln = acc[key]
            acc[key] = [0.0, 0, 0.0]
            return (s / n if n else float("nan")), n, (ln / n if n else float("nan"))

        while self.version < total_updates:
            if fault is not None and fault[:2] == (self.rank, i):   # SURVEY §5.3 test hook: die without goodbye
                if len(fault) == 2:
                    self._die()
                self._die_at = fault[2]   # inside this iteration's exchange (parse_fault: "push" / "reply")
            tr.step()
            hist.append(self.version)
            rep_due = bool(report_every) and len(hist) % report_every == 0
            log_due = tr.logger is not None and bool(cfg.stdout_freq) and i % cfg.stdout_freq == 0
            if rep_due or log_due:
                ret, n_ep, ln = tr.env.drain_episode_stats()
                for a in acc.values():
                    if n_ep:
                        a[0] += ret * n_ep
                        a[1] += n_ep
                        a[2] += ln * n_ep
            if rep_due:
                ret, n_ep, _ = take("report")
                self.returns.append((len(hist), self.version, ret, n_ep))
            if log_due:
                tr.log(i, print_tog=not cfg.quiet, ep_stats=take("log"))   # A3C/process.py:280-283
            if tr.logger is not None and cfg.flush_every and i % cfg.flush_every == cfg.flush_every // 2:
                tr.logger.flush()
            if self.task == 0 and cfg.save_every and cfg.checkpoint_dir:
                mark = self.version // cfg.save_every   # CheckpointSaverHook(save_steps=save_every), chief only
                if mark != last_mark:
                    self.saved.append(self.save(self.version))
                    last_mark = mark
            i += 1
        if self.task == 0 and cfg.save_every and cfg.checkpoint_dir:
            self.saved.append(self.save(self.version))   # the final global parameters
        for r in self.ps_ranks:
            self.planes.send_hdr([CMD_DONE, self.task, self.version, 0], r)
        if tr.logger is not None:
            tr.logger.close()
        return hist

    def save(self, gstep):
        """The global actor/critic (this worker holds them right after its pull) under the reference names
        ``global_actor/...`` / ``global_critic/...``: no Adam slots and no global step, as the reference's Saver
        built before them."""
        from .. import ckpt as C
        from ..models.policy import MLPActorCritic
        cfg, m = self.cfg, self.tr.model
        d = cfg.checkpoint_dir
        os.makedirs(d, exist_ok=True)
        base = self.ckpt_base or ("model-" + C.env_prefix(cfg.env))
        path = os.path.join(d, f"{base}-{gstep}")
        if isinstance(m, MLPActorCritic):
            t = C.reference_tensors(m.actor, m.critic, "a3c", actor_lr=cfg.lr, ent_coef=cfg.ent_coef,
                                    kl_coef=cfg.kl_coef, critic_lr=cfg.critic_lr)
        else:
            t = C.generic_tensors(m)
        C.save_tensors(path, t)
        kept = C._prune(d, base, cfg.keep_checkpoints)
        C._write_state_file(d, path, kept or [path])
        return path


def run(cfg, rank=None, world=None, ps_num=None, data_backend="gloo", max_staleness=-1, device=None,
        report_every=0, log_dir=None, logger=None, checkpoint_basename=None):
    """Entry point of one process of the GPU-native async job. The default process group (gloo) must exist or is
    created from the torchrun environment; with ``data_backend="nccl"`` an RCCL group carries the payloads.
    ``log_dir``: per-worker Logger files ``worker_<task>.log`` (the reference's ``tmp/logs``)."""
    import datetime
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    rank = dist.get_rank() if rank is None else rank
    world = dist.get_world_size() if world is None else world
    ps_num = cfg.ps_num if ps_num is None else ps_num
    assert world - ps_num >= 1, "need at least one worker rank"
    if cfg.max_grad_norm is not None:
        raise ValueError("async PS mode clips element-wise only (A3C/policies.py:85); a global-norm clip "
                         f"(max_grad_norm={cfg.max_grad_norm}) would be computed per PS shard: set it to None")
    if cfg.lr_schedule != "constant":
        raise ValueError("async PS mode: the critic lr lives in the PS shard optimisers, which do not decay it; "
                         "lr_schedule must be 'constant'")
    device = torch.device(device or cfg.device)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    tmo = datetime.timedelta(seconds=cfg.dist_timeout_s)
    ctrl = dist.new_group(backend="gloo", timeout=tmo)
    data = dist.new_group(backend="nccl", timeout=tmo) if data_backend == "nccl" else ctrl
    planes = _Planes(ctrl, data, data_backend, device)
    flat = _build_flat(cfg, torch.device("cpu"))
    ranges = shard_ranges(flat, ps_num)
    t0 = time.time()
    if rank < ps_num:
        ps = DeviceParameterServer(cfg, rank, ranges[rank], range(ps_num, world), planes, device, max_staleness)
        ps.serve()
        return {"role": "ps", "status": ps.status, "error": getattr(ps, "error", None),
                "global_step": ps.global_step, "log": ps.log, "n_applies": ps.n_applies,
                "adam_t": {f"{k}:{w}": float(t) for (k, w), t in ps.t.items()}, "wall_s": time.time() - t0,
                "params": ps.flat.data[ps.s:ps.e].detach().cpu()}
    task = rank - ps_num
    w = GPUWorker(cfg, task, ranges, list(range(ps_num)), planes, device, log_dir=log_dir, rank=rank, logger=logger,
                  checkpoint_basename=checkpoint_basename)
    hist = w.run(cfg.total_updates, report_every)
    tr = w.tr
    ret, n_ep, _ = tr.env.drain_episode_stats()
    return {"role": "worker", "task": task, "global_step": w.version, "history": hist, "updates": len(hist),
            "env_steps": tr.env_steps, "wall_s": time.time() - t0, "ep_return": ret, "episodes": n_ep,
            "returns": w.returns, "checkpoints": w.saved}
