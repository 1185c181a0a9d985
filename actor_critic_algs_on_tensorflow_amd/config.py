"""Typed training configuration + presets.

The reference configures itself with argparse flags and module constants (defaults table: SURVEY §2.6). Here
one dataclass carries everything; presets mirror the reference defaults (``basic_ac``, ``a3c``) and the
BASELINE.json configs (``cartpole_cpu``, ``pong_a2c``, ``breakout_ppo``, ``a2c_dp8``, ``mujoco_ppo_dp8``).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass
class EngineOpts:
    """Kernel selection of the native CNN engine (``algos/engine.py``). Every switch is a path that is the default of
    some BASELINE config or the oracle of a test (tests/test_config_cpu.py pins the list); the defaults are the
    fastest measured configuration on MI355X (A/B evidence in ``profiles/``). ``TrainConfig.engine_opts`` carries one;
    plain dicts are accepted and converted."""
    # -- rollout -------------------------------------------------------------------------------------------------
    fused_step: bool = True           # Pong bank: policy/env step t fused with the trunk of obs t+1 (off: oracle)
    trunk_rows_max_b: int = 64        # row-split trunk (7 workgroups per env) up to this many envs, per-env above
    fused_env_split: bool = True      # per-env fused step (banks above trunk_rows_max_b): two workgroups per env
    adam_step_offsets: bool = True    # MLP PPO: grouped Adam launches take their step from the minibatch index (no ticket)
    frag_weights: bool = True         # conv weights also kept fragment-ordered (written by the optimiser step): the
                                      # MFMA weight loads become one contiguous 1 KB read per wave
    fc_max_planes: int = 32           # split-K partial planes of the rollout fc product (consumer-reduced)
    fc_frag_big: int = 17             # ... for banks of 33..128 envs (+16: 32-row blocks split over workgroups)
    fc_frag: int = 5                  # rollout fc product (<= 32 envs) on a fragment-ordered Wfc copy (fc_rollout.hip
                                      # variant 0..9; -1: the general GEMM on the row-major shadow)
    # -- learner -------------------------------------------------------------------------------------------------
    a2c_head: bool = True             # A2C: V(s_T) + returns + loss + head backward in one launch (loss.hip a2c_head)
    a2c_head_env: bool = True         # ... as one workgroup per env without a grid-wide hand-off (A2C without
                                      # advantage normalisation; head gradients as per-env planes the finaliser sums)
    fused_head: bool = True           # A2C: loss + head backward in one launch (round-2 head_bwd) when a2c_head is off
    grouped: bool = True              # independent backward products as ONE grouped GEMM launch (no side stream)
    det_wgrad: bool = True            # weight gradients as split-K planes reduced in fixed order (bitwise determinism)
    fused_bwd: bool = True            # dy3 -> dy2 -> dy1 in one per-sample kernel (cnn_trunk_bwd)
    mb_index: bool = True             # PPO minibatches read their observations in place through a row index
    ppo_head: bool = True             # large-batch head: z, loss, dz, dh and dWh / dbh / dbfc planes in one launch
    fc_bwd: bool = True               # learner batches of <= 256 rows: dy3 and dWfc in one dedicated launch (fc_bwd.hip)
    large_batch_min_b: int = 1024     # learner batches from this many rows: the persistent trunk backward (with the
                                      # conv1 weight gradient folded in), the batched-position conv2 / conv3 weight
                                      # gradients, gemm_big fc products, the backward on one stream
    trunk_bwd_persist: int = 256      # workgroups of the persistent trunk backward
    wgrad_planes: int = 64            # split-K planes of the GEMM weight gradients
    conv1_v2_planes: int = 256        # planes of the conv1 weight gradient when it is not folded (one workgroup each)
    nhwc_planes: int = 256            # planes of the conv2 / conv3 weight-gradient kernels

    def replace(self, **kw):
        return dataclasses.replace(self, **kw)


# string-valued TrainConfig fields and the values they accept (validated in __post_init__)
CHOICES = {
    "algo": {"a2c", "ppo", "a3c", "basic_ac"},
    "model": {"auto", "mlp", "cnn"},
    "model_variant": {"basic", "a3c"},
    "returns": {"nstep", "gae"},
    "optimizer": {"adam", "rmsprop"},
    "lr_schedule": {"constant", "linear"},
    "dtype": {"bf16", "fp32"},
    "engine": {"auto", "native", "torch"},
    "dist_backend": {"auto", "nccl", "gloo"},
    "overlap": {"strict", "lag1"},
    "grad_bucket_dtype": {"fp32", "bf16"},
    "dp_capture": {"auto", "segments"},
    "mode": {"train", "debug", "debug-light", "debug-full"},
}


@dataclass
class TrainConfig:
    # -- problem ---------------------------------------------------------------------------------------------
    env: str = "Pendulum-v0"
    algo: str = "a2c"                 # a2c | ppo | a3c | basic_ac (reference-parity episode-batched trainer)
    num_envs: int = 1                 # envs per rank / GPU
    n_steps: int = 5                  # rollout length T
    frames: int = 1                   # frame stack for vector envs (Atari envs always stack 4)
    model: str = "auto"               # auto | mlp | cnn
    model_variant: str = "basic"      # basic | a3c (reference divergences)
    seed: int = 12321
    device: str = "cpu"
    # -- returns -----------------------------------------------------------------------------------------------
    gamma: float = 0.99
    returns: str = "nstep"            # nstep (PathAdv generalisation) | gae
    look_ahead: int | None = None     # n-step truncation L (reference: 40); None = whole rollout
    gae_lambda: float = 0.95
    norm_adv: bool = False
    bootstrap_on_timeout: bool = False
    # -- losses ------------------------------------------------------------------------------------------------
    ent_coef: float = 0.01            # reference "gamma" (Basic_AC/policies.py:38)
    kl_coef: float = 0.0              # reference "beta" (squared log-prob drift proxy)
    vf_coef: float = 0.5
    # -- optimiser ---------------------------------------------------------------------------------------------
    optimizer: str = "adam"           # adam | rmsprop
    lr: float = 7e-4                  # shared-model lr / actor lr
    critic_lr: float = 1e-3           # separate-critic lr (reference 0.001)
    clip_value: float | None = None   # element-wise grad clip (reference actor: 1.0 Basic / 0.1 A3C)
    critic_clip_value: float | None = None
    max_grad_norm: float | None = 0.5
    # -- reference regularisation machinery -----------------------------------------------------------------------
    kl_adaptive_lr: bool = False
    desired_kl: float = 0.002
    min_lr: float = 1e-6
    max_lr: float = 1.0
    anneal_regularizers: bool = False  # log10 schedules of ent/kl coefs (Basic_AC/run_AC.py:181-182)
    lr_schedule: str = "constant"     # constant | linear (every optimiser's lr decays linearly to 0 at total_updates;
                                      # not combined with the KL-adaptive lr, which owns the actor lr)
    # -- PPO ---------------------------------------------------------------------------------------------------
    ppo_epochs: int = 4
    ppo_minibatches: int = 4
    ppo_clip: float = 0.1
    ppo_value_clip: float | None = None
    # -- execution -----------------------------------------------------------------------------------------------
    dtype: str = "bf16"               # compute dtype of the GPU engine (fp32 masters always)
    engine: str = "auto"              # auto | native (hand-written HIP engine) | torch (autograd reference)
    cuda_graph: bool = True
    reuse_rollout_acts: bool = True   # native A2C: the rollout's activations are the learner's forward (exact)
    fused_rollout: bool = True        # native MLP engine + MuJoCo-shaped bank: the whole rollout in one launch
    engine_opts: EngineOpts = field(default_factory=EngineOpts)   # kernel selection of the native CNN engine
    total_updates: int = 1000
    # -- distributed -----------------------------------------------------------------------------------------------
    dist_backend: str = "auto"        # auto -> nccl (RCCL) on GPU, gloo on CPU
    overlap: str = "strict"           # strict | lag1 (all-reduce overlapped with next rollout, policy lag 1)
    grad_bucket_dtype: str = "fp32"   # fp32 | bf16 (all-reduce the gradient buckets as bf16: half the xGMI bytes)
    dp_capture: str = "auto"          # auto: RCCL collectives recorded INSIDE the update's hipGraph (one graph per
                                      # update); gloo (host-side collectives) -> a graph chain cut at each one |
                                      # segments: force the graph chain (A/B and equivalence tests)
    ps_num: int = 1                   # A3C parameter-server ranks
    # -- reference episode-batched trainer (basic_ac) -------------------------------------------------------------
    max_rolls: int = 7
    max_path_length: int | None = None
    ep_length_stop: int | None = None
    # -- logging / checkpoints ---------------------------------------------------------------------------------------
    outdir: str = "log.txt"
    metrics_path: str | None = None
    stdout_freq: int = 20
    flush_every: int = 100
    save_every: int = 600
    checkpoint_dir: str = "tmp/checkpoints"
    keep_checkpoints: int = 3
    quiet: bool = False
    legacy_step_index: bool = False
    tboard: bool = False              # TensorBoard event file under summaries_dir(outdir) (utils/tensorboard.py)
    tb_root: str = "summaries"
    mode: str = "train"               # train | debug | debug-light | debug-full
    trace: bool = False               # per-phase timers + ROCTx ranges (utils/trace.py), reported in the metrics stream
    # -- failure handling -------------------------------------------------------------------------------
    fault_inject: str | None = None   # "rank:iteration": that rank dies (os._exit) when it reaches that iteration
    resume: str | None = None         # "auto" = newest checkpoint in checkpoint_dir, or a checkpoint prefix
    dist_timeout_s: int = 300         # collective timeout: a dead peer surfaces as an exception, not a hang

    def __post_init__(self):
        for name, allowed in CHOICES.items():
            v = getattr(self, name)
            if v not in allowed:
                raise ValueError(f"TrainConfig.{name}={v!r}: expected one of {sorted(allowed)}")
        if self.lr_schedule == "linear" and self.kl_adaptive_lr:
            raise ValueError("lr_schedule='linear' with kl_adaptive_lr=True: the KL controller owns the actor lr, so "
                             "only the critic would decay; pick one")
        if not isinstance(self.engine_opts, EngineOpts):
            self.engine_opts = EngineOpts(**dict(self.engine_opts or {}))
        if self.look_ahead is not None and int(self.look_ahead) < 1:
            raise ValueError(f"TrainConfig.look_ahead={self.look_ahead}: must be >= 1 (None = the whole rollout)")

    def replace(self, **kw):
        return dataclasses.replace(self, **kw)

    def to_dict(self):
        return dataclasses.asdict(self)


PRESETS = {
    # Basic_AC/run_AC.py defaults
    "basic_ac": dict(algo="basic_ac", env="Pendulum-v0", gamma=0.98, look_ahead=40, norm_adv=True, ent_coef=0.01,
                     kl_coef=1.0, lr=0.005, critic_lr=0.001, clip_value=1.0, max_grad_norm=None,
                     kl_adaptive_lr=True, max_lr=1.0, anneal_regularizers=True, model_variant="basic",
                     optimizer="adam", device="cpu", cuda_graph=False),
    # A3C/process.py defaults
    "a3c": dict(algo="a3c", env="Pendulum-v0", gamma=0.98, look_ahead=40, norm_adv=True, ent_coef=0.01,
                kl_coef=1.0, lr=0.005, critic_lr=0.001, clip_value=0.1, max_grad_norm=None, kl_adaptive_lr=True,
                max_lr=0.1, anneal_regularizers=True, model_variant="a3c", optimizer="adam", device="cpu",
                cuda_graph=False),
    # The reference's flagship task (Pendulum-v0, README.md:18,33-37) solved by PPO-clip on the reference networks:
    # the A3C actor / critic (model_variant a3c), gamma 0.98 as the reference, one 200-step episode per
    # env per rollout (16 envs: 3200 steps, the scale of the reference's 1200-step batches), GAE(0.95), 10 epochs x
    # 8 minibatches, Adam 3e-4 with a 0.5 global-norm clip. Reaches a mean return above -200 within ~150k env steps
    # (profiles/r3_pendulum_learning.txt); the reference's own single-step KL-adaptive update is preset "a3c".
    "pendulum_ppo": dict(algo="ppo", env="Pendulum-v0", model="mlp", model_variant="a3c", num_envs=16, n_steps=200,
                         gamma=0.98, returns="gae", gae_lambda=0.95, norm_adv=True, ppo_epochs=10, ppo_minibatches=8,
                         ppo_clip=0.2, optimizer="adam", lr=3e-4, critic_lr=1e-3, ent_coef=0.0, kl_coef=0.0,
                         max_grad_norm=0.5, device="cuda", dtype="fp32"),
    # BASELINE config 1
    "cartpole_cpu": dict(algo="a2c", env="CartPole-v1", num_envs=1, n_steps=5, gamma=0.99, model="mlp",
                         lr=1e-3, critic_lr=5e-3, norm_adv=True, device="cpu", cuda_graph=False,
                         max_grad_norm=0.5),
    # BASELINE config 2 (headline metric)
    "pong_a2c": dict(algo="a2c", env="PongNoFrameskip-v4", num_envs=32, n_steps=5, gamma=0.99, model="cnn",
                     optimizer="rmsprop", lr=7e-4, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5,
                     device="cuda", dtype="bf16"),
    # BASELINE config 3
    "breakout_ppo": dict(algo="ppo", env="BreakoutNoFrameskip-v4", num_envs=128, n_steps=128, gamma=0.99,
                         returns="gae", gae_lambda=0.95, norm_adv=True, model="cnn", optimizer="adam", lr=2.5e-4,
                         ppo_epochs=4, ppo_minibatches=4, ppo_clip=0.1, ent_coef=0.01, vf_coef=0.5,
                         max_grad_norm=0.5, device="cuda", dtype="bf16"),
    # BASELINE config 4
    "a2c_dp8": dict(algo="a2c", env="PongNoFrameskip-v4", num_envs=32, n_steps=5, gamma=0.99, model="cnn",
                    optimizer="rmsprop", lr=7e-4, max_grad_norm=0.5, device="cuda", dtype="bf16"),
    # BASELINE config 5
    "mujoco_ppo_dp8": dict(algo="ppo", env="HalfCheetahShape-v0", num_envs=64, n_steps=256, gamma=0.99,
                           returns="gae", gae_lambda=0.95, norm_adv=True, model="mlp", optimizer="adam", lr=3e-4,
                           critic_lr=1e-3, ppo_epochs=10, ppo_minibatches=32, ppo_clip=0.2, ent_coef=0.0,
                           vf_coef=0.5, max_grad_norm=0.5, device="cuda", dtype="fp32"),
}


def preset(name, **overrides) -> TrainConfig:
    kw = dict(PRESETS[name])
    kw.update(overrides)
    return TrainConfig(**kw)
