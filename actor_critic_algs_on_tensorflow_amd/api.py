"""Public API: ``train(cfg) -> TrainResult``, ``Agent`` (batched ``act``), ``evaluate`` (the reference's
``test_process``, ``A3C/process.py:125-153``).

    import actor_critic_algs_on_tensorflow_amd as aca
    res = aca.train(aca.preset("cartpole_cpu", total_updates=2000))
    agent = aca.Agent.from_checkpoint("tests/fixtures/model-Pendulum_a3c", "Pendulum-v0")
    a, logp, ent = agent.act(obs)          # obs [N, obs_dim] -> actions [N(, A)], logp [N], entropy [N]
    aca.evaluate("tests/fixtures/model-Pendulum_a3c", "Pendulum-v0", num_episodes=3)
"""
from __future__ import annotations

import dataclasses
import time

import numpy as np
import torch

from . import envs as E
from .config import TrainConfig, preset


@dataclasses.dataclass
class TrainResult:
    history: list
    iterations: int
    env_steps: int
    seconds: float
    checkpoint: str | None
    trainer: object = None

    @property
    def env_steps_per_sec(self):
        return self.env_steps / max(self.seconds, 1e-9)


def make_trainer(cfg: TrainConfig, dp=None):
    if cfg.algo == "basic_ac":
        from .algos.basic_ac import BasicACTrainer
        return BasicACTrainer(cfg)
    if cfg.algo == "a3c":
        raise ValueError("algo='a3c' runs as a multi-process job: use actor_critic_algs_on_tensorflow_amd.algos.a3c"
                         ".run(cfg) under torch.distributed (see cli/train.py)")
    from .algos.trainer import ActorCriticTrainer
    return ActorCriticTrainer(cfg, dp=dp)


def train(cfg: TrainConfig | str, **overrides) -> TrainResult:
    """Trains with a config (or preset name + overrides) on one process; returns the history and final state.

    Multi-GPU data parallelism: launch this under ``torch.distributed.run`` with ``dist_backend`` "nccl"/"gloo";
    the process group is initialised from the environment (one rank per GPU).
    """
    if isinstance(cfg, str):
        cfg = preset(cfg, **overrides)
    elif overrides:
        cfg = cfg.replace(**overrides)
    dp = None
    from .parallel import dp as DP
    rank, world, local = DP.init_from_env(cfg.dist_backend, timeout_s=cfg.dist_timeout_s)
    if world > 1:
        if cfg.device.startswith("cuda"):
            cfg = cfg.replace(device=f"cuda:{local}")
        dp = DP.DataParallel()
    tr = make_trainer(cfg, dp)
    n = None
    if cfg.resume:   # restart from the newest (or a given) checkpoint, run the remaining updates
        if cfg.algo == "basic_ac":
            raise ValueError("resume needs the vectorised trainers (the basic_ac parity loop keeps no resume state)")
        from . import ckpt
        path = ckpt.latest_checkpoint(cfg.checkpoint_dir) if cfg.resume == "auto" else cfg.resume
        if path is not None:
            tr.load_checkpoint(path)
        n = max(0, cfg.total_updates - tr.iteration)
    t0 = time.time()
    hist = tr.train(n) if n is not None else tr.train()
    if cfg.device.startswith("cuda"):
        torch.cuda.synchronize()
    dt = time.time() - t0
    ck = None
    if cfg.checkpoint_dir and cfg.save_every and (getattr(tr, "rank", 0) == 0 or getattr(tr, "dp", None) is not None):
        ck = tr.save_checkpoint()
    if hasattr(tr, "close"):
        tr.close()
    return TrainResult(hist, tr.iteration, tr.env_steps, dt, ck, tr)


class Agent:
    """A policy ready to act: wraps a model family and its device; ``act`` is batched over observations.

    On a GPU (``engine="auto"|"native"``) ``act`` runs the hand-written HIP engines the trainers use: the CNN family
    through :class:`.algos.engine.CNNEngine` (fused trunk + fc + head, bf16 MFMA) and the categorical sampling
    kernel; the MLP family through :class:`.ops.mlp.MLPEngine` (both towers + sampling in one launch). Sampling keys
    are ``(call counter << 20) + row``, so the native and the PyTorch paths draw the same actions from the same
    logits. ``engine="torch"`` (and every CPU agent) runs the PyTorch modules."""

    def __init__(self, model, env_id=None, device="cpu", seed=0, engine="auto"):
        self.model = model.to(device)
        self.model.eval()
        self.env_id = env_id
        self.device = torch.device(device)
        self.seed = seed
        self._ctr = 0
        self.engine_kind = engine
        self._eng = None

    def _engine(self):
        """Lazily builds the native engine over the model's parameters (None on CPU / engine="torch")."""
        if self._eng is not None or self.engine_kind == "torch" or self.device.type != "cuda":
            return self._eng
        from .models.policy import CNNActorCritic, MLPActorCritic
        from .ops.optim import FlatParams
        from . import _native
        _native.require()
        flat = FlatParams(self.model.param_groups(), self.device)   # re-homes the parameters into one slab
        if isinstance(self.model, CNNActorCritic):
            from .algos.engine import CNNEngine
            shadow = flat.data.to(torch.bfloat16)
            self._eng = ("cnn", CNNEngine(self.model, flat, shadow), flat)
        elif isinstance(self.model, MLPActorCritic) and self.model.actor.ac_dim <= 16:
            from .ops.mlp import MLPEngine
            self._eng = ("mlp", MLPEngine(self.model, flat), flat)
        elif self.engine_kind == "native":
            raise ValueError("no native engine for this model")
        return self._eng

    @torch.no_grad()
    def _act_native(self, o, keys_ctr, deterministic):
        from .ops import distributions as D
        kind, eng, _ = self._eng
        N = o.shape[0]
        if kind == "cnn":
            b = eng.bufs(N)
            z = eng.forward(o.to(torch.uint8).contiguous(), b)
            logits = z[:, :eng.A].contiguous()
            if deterministic:
                a = logits.argmax(-1).to(torch.int32)
                logp, ent = D.categorical_logp_entropy(logits, a)
                return a, logp, ent
            keys = torch.arange(N, dtype=torch.int64, device=self.device) + (keys_ctr << 20)
            return D.categorical_sample(logits, keys, self.seed)
        if deterministic:
            return None
        act = torch.empty((N,) if eng.discrete else (N, eng.A), dtype=torch.int32 if eng.discrete else torch.float32,
                          device=self.device)
        logp = torch.empty(N, device=self.device)
        ent = torch.empty(N, device=self.device)
        v = torch.empty(N, device=self.device)
        tg = torch.full((N,), keys_ctr, dtype=torch.int64, device=self.device)
        ids = torch.arange(N, dtype=torch.int64, device=self.device)
        eng.policy_step(o.float().contiguous(), act, logp, ent, v, tg, ids, 20, self.seed)
        return act, logp, ent

    @classmethod
    def for_env(cls, env_id, family="auto", variant="basic", frames=1, device="cpu", seed=0):
        from .models.policy import build_model
        env = E.make(env_id, 1, device="cpu", frame_stack=4 if ("Pong" in env_id or "Breakout" in env_id) else frames)
        return cls(build_model(env, family, variant, seed=seed), env_id, device, seed)

    @classmethod
    def from_checkpoint(cls, path, env_id, frames=1, device="cpu", variant=None):
        """Loads a TF-bundle checkpoint (reference names or this framework's)."""
        from . import ckpt
        t = ckpt.load_tensors(path)
        v = variant or ckpt.detect_variant(t.keys())
        fam = "mlp" if v in ("a3c", "basic") else "auto"
        agent = cls.for_env(env_id, family=fam, variant=v if v != "generic" else "basic", frames=frames,
                            device="cpu")
        ckpt.load_model(agent.model, t, v if v != "generic" else "basic", strict=True)
        agent.model.to(device)
        agent.device = torch.device(device)
        return agent

    @torch.no_grad()
    def act(self, obs, deterministic=False):
        """obs ``[N, ...]`` (or a single observation) -> (action, logp, entropy) as numpy arrays."""
        o = torch.as_tensor(np.asarray(obs))
        single = o.dim() == self._obs_rank()
        if single:
            o = o.unsqueeze(0)
        o = o.to(self.device)
        N = o.shape[0]
        ctr = self._ctr
        self._ctr += 1
        res = self._act_native(o, ctr, deterministic) if self._engine() is not None else None
        if res is not None:
            a, logp, ent = res
        else:
            keys = torch.arange(N, dtype=torch.int64, device=self.device) + (ctr << 20)
            a, logp, ent, _ = self.model.act(o, keys=keys, seed=self.seed, deterministic=deterministic)
        out = (a.cpu().numpy(), logp.cpu().numpy(), ent.cpu().numpy())
        return tuple(x[0] for x in out) if single else out

    def _obs_rank(self):
        from .models.policy import CNNActorCritic
        return 3 if isinstance(self.model, CNNActorCritic) else 1

    @torch.no_grad()
    def value(self, obs):
        o = torch.as_tensor(np.asarray(obs)).to(self.device)
        if o.dim() == self._obs_rank():
            o = o.unsqueeze(0)
        return self.model.value(o).cpu().numpy()


def evaluate(model_path, env_id, num_episodes=3, seed=12321, frames=1, animate=False, variant=None, verbose=True,
             max_path_length=None):
    """Runs ``num_episodes`` episodes of a saved policy, printing the reference's per-episode report."""
    agent = Agent.from_checkpoint(model_path, env_id, frames=frames, variant=variant)
    agent.seed = seed
    env = E.make(env_id, 1, device="cpu", seed=seed, frame_stack=frames)
    mpl, _ = E.get_roll_params(env_id, "a3c" if (variant or "a3c") == "a3c" else "basic")
    if max_path_length is not None:
        mpl = max_path_length
    rewards = []   # the env keeps its own time limit; mpl only bounds the loop (rollout(), run_AC.py:95)
    obs = env.reset().clone()
    for i in range(num_episodes):
        total, length = 0.0, 0
        while True:
            a, _, _ = agent.act(obs)
            a_t = torch.as_tensor(np.asarray(a)).reshape(1, *([-1] if not env.is_discrete else []))
            if env.is_discrete:
                a_t = a_t.to(torch.int32).reshape(1)
            obs_next, r, d, _ = env.step(a_t)
            total += float(r[0])
            length += 1
            obs = obs_next.clone()
            if bool(d[0]):
                break   # the bank auto-reset: obs already holds the next episode's first observation
            if length >= mpl:
                # cut by the loop bound without done: start the next episode fresh, as rollout() does with its
                # env.reset() per episode (Basic_AC/run_AC.py:88)
                obs = env.reset().clone()
                break
        rewards.append(total)
        if verbose:
            print("Iteration {}".format(i))
            print("Reward {}".format(total))
            print("Episode Length {}\n".format(length))
    avg = float(np.mean(rewards)) if rewards else float("nan")
    if verbose:
        print("Average reward over {} was {}".format(num_episodes, avg))
    return rewards
