"""Checkpoints in TensorFlow's tensor-bundle (Saver V2) format, with the reference's variable names.

The reference saves with ``tf.train.Saver`` (``Basic_AC/run_AC.py:199,282-284``; chief-only ``CheckpointSaverHook``
in ``A3C/process.py:197,211-214``) and restores for evaluation in ``test_process`` (``A3C/process.py:125-153``).
This module writes and reads the same files through the C++ codec (:mod:`.codec`, ``csrc/tfbundle``):

* reference MLP actor/critic -> the exact reference names:
    - ``variant="a3c"``:  ``global_actor/{first,second,third}_layer/{kernel,bias}``, ``global_actor/mu_layer/...`` or
      ``global_actor/logits/...``, ``global_actor/log_std``, ``global_actor/Variable{,_1,_2}`` = lr, entropy coef
      ("gamma"), KL coef ("beta") (``A3C/policies.py:77-79``); ``global_critic/...`` + ``global_critic/Variable{,_1}`` =
      the (duplicated, ``A3C/policies.py:151,154``) critic lr.
    - ``variant="basic"``: scopes ``Actor/`` / ``Critic/``; the unnamed log-std is ``Actor/Variable`` (continuous),
      then beta, gamma, lr (``Basic_AC/policies.py:49,75-77``); ``Critic/Variable`` = critic lr; Adam slots are
      written as ``<var>/Adam`` (m) and ``<var>/Adam_1`` (v) plus ``<scope>/beta{1,2}_power`` as TF's Saver does when
      it is built after the optimisers (the Basic_AC case).
  Kernels are stored ``[in, out]`` in both frameworks, so no transposes happen.
* any other model (the Atari CNN): ``acamd/<module path>`` names.
* native resume state (not in the reference, which cannot resume -- SURVEY §5.4) goes under ``_acamd/...`` keys:
  optimiser moments/step/lr per group, iteration and env-step counters, env-bank state. TF ignores unknown keys
  only if they are not requested, so reference tooling can still restore the model variables.

A ``checkpoint`` state file (``model_checkpoint_path: "..."``) is written next to the bundles and the newest
``keep`` checkpoints are retained (``max_to_keep=3`` in the reference).
"""
from __future__ import annotations

import glob
import os
import re

import numpy as np
import torch

from . import codec

# ------------------------------------------------------------------------------------------------ name maps


def _dense_names(prefix, module, layers):
    out = {}
    for lname in layers:
        layer = getattr(module, lname, None)
        if layer is None:
            continue
        out[f"{prefix}/{lname}/kernel"] = layer.kernel
        out[f"{prefix}/{lname}/bias"] = layer.bias
    return out


def reference_tensors(actor, critic, variant="a3c", actor_lr=0.005, ent_coef=0.01, kl_coef=1.0, critic_lr=0.001):
    """-> ordered dict name -> torch tensor (parameters are live views; scalars are fresh tensors)."""
    a_scope, c_scope = ("global_actor", "global_critic") if variant == "a3c" else ("Actor", "Critic")
    t = {}
    head = ["logits"] if actor.discrete else ["mu_layer"]
    t.update(_dense_names(a_scope, actor, ["first_layer", "second_layer", "third_layer"] + head))
    f = lambda v: torch.tensor(float(v), dtype=torch.float32)
    if variant == "a3c":
        if not actor.discrete:
            t[f"{a_scope}/log_std"] = actor.log_std
        t[f"{a_scope}/Variable"] = f(actor_lr)
        t[f"{a_scope}/Variable_1"] = f(ent_coef)
        t[f"{a_scope}/Variable_2"] = f(kl_coef)
        t.update(_dense_names(c_scope, critic, ["first_layer", "second_layer", "third_layer", "value"]))
        t[f"{c_scope}/Variable"] = f(critic_lr)
        t[f"{c_scope}/Variable_1"] = f(critic_lr)
    else:
        i = 0
        if not actor.discrete:
            t[f"{a_scope}/Variable"] = actor.log_std
            i = 1
        for val in (kl_coef, ent_coef, actor_lr):   # beta, gamma, lr (Basic_AC/policies.py:75-77)
            t[f"{a_scope}/Variable" + (f"_{i}" if i else "")] = f(val)
            i += 1
        t.update(_dense_names(c_scope, critic, ["first_layer", "second_layer", "third_layer", "value"]))
        t[f"{c_scope}/Variable"] = f(critic_lr)
    return t


def generic_tensors(model, prefix="acamd"):
    return {f"{prefix}/" + n.replace(".", "/"): p for n, p in model.named_parameters()}


def model_tensors(model, variant="basic", opts=None):
    """Name map for a model built by :func:`..models.policy.build_model`."""
    from ..models.policy import MLPActorCritic
    if isinstance(model, MLPActorCritic):
        lr = {}
        if opts:
            for g, o in opts.items():
                lr[g] = o.get_lr()
        return reference_tensors(model.actor, model.critic, variant,
                                 actor_lr=lr.get("actor", 0.005), critic_lr=lr.get("critic", 0.001))
    return generic_tensors(model)


# ------------------------------------------------------------------------------------------------ save / load
def _to_np(x):
    return x.detach().to("cpu", torch.float32).contiguous().numpy() if x.dtype.is_floating_point else \
        x.detach().cpu().contiguous().numpy()


def save_tensors(prefix, tensors):
    codec.write(prefix, {k: _to_np(v) if isinstance(v, torch.Tensor) else np.asarray(v) for k, v in tensors.items()})
    return prefix


def load_tensors(prefix, verify_crc=True):
    return codec.read(prefix, verify_crc)


def _write_state_file(directory, newest, all_paths):
    lines = ['model_checkpoint_path: "%s"' % os.path.basename(newest)]
    lines += ['all_model_checkpoint_paths: "%s"' % os.path.basename(p) for p in all_paths]
    with open(os.path.join(directory, "checkpoint"), "w") as f:
        f.write("\n".join(lines) + "\n")


def latest_checkpoint(directory):
    """TF ``tf.train.latest_checkpoint`` equivalent (reads the ``checkpoint`` state file)."""
    p = os.path.join(directory, "checkpoint")
    if not os.path.exists(p):
        return None
    m = re.search(r'model_checkpoint_path:\s*"([^"]+)"', open(p).read())
    return os.path.join(directory, m.group(1)) if m else None


def _prune(directory, base, keep):
    found = []
    for idx in glob.glob(os.path.join(directory, base + "-*.index")):
        m = re.match(r".*-(\d+)\.index$", idx)
        if m:
            found.append((int(m.group(1)), idx[:-len(".index")]))
    found.sort()
    for _, prefix in found[:-keep] if keep else []:
        for f in glob.glob(prefix + ".*"):
            os.remove(f)
    return [p for _, p in found[-keep:]] if keep else [p for _, p in found]


def env_prefix(env_id):
    return env_id.split("-")[0]


def _env_state(trainer):
    env = trainer.env
    st = {k: getattr(env, k) for k in ("state", "t", "tg", "ep_ret")}
    st["obs"] = trainer.storage.obs[0]
    return st


def _gather_env_states(trainer):
    """-> {rank: {name: tensor}} on rank 0, None on the other ranks. With data parallelism every rank simulates its
    own envs, so a resumable checkpoint needs all of them: one all_gather per tensor (identical shapes on every
    rank), called collectively by all ranks."""
    st = _env_state(trainer)
    dp = getattr(trainer, "dp", None)
    if dp is None or dp.world_size == 1:
        return {0: st}
    import torch.distributed as dist
    got = {r: {} for r in range(dp.world_size)}
    for k, v in st.items():
        v = v.contiguous()
        bufs = [torch.empty_like(v) for _ in range(dp.world_size)]
        dist.all_gather(bufs, v, group=dp.group)
        for r in range(dp.world_size):
            got[r][k] = bufs[r]
    return got if dp.rank == 0 else None


_SLAB_STATE = ("m", "v")   # optimiser state laid out like the parameter slab


def _param_ranges(trainer, opt):
    """(parameter name, start, end) of every parameter of ``opt``'s slab segment, relative to the segment."""
    flat = trainer.flat
    name_of = {id(p): n for n, p in trainer.model.named_parameters()}
    out = []
    for p, off in zip(flat.params, flat.offsets):
        if opt.start <= off < opt.end:
            out.append((name_of[id(p)], off - opt.start, off - opt.start + p.numel()))
    return out


def _load_opt_state(trainer, opt, g, t, path):
    """Optimiser state of group ``g``: m / v scattered by parameter name; a bundle written before the per-name form
    (whole slab vectors) is accepted only when its size matches this slab."""
    sd = {}
    for k, v in t.items():
        if not k.startswith(f"_acamd/opt/{g}/"):
            continue
        rest = k[len(f"_acamd/opt/{g}/"):]
        if "/" not in rest:
            sd[rest] = torch.as_tensor(np.array(v))
    for k in _SLAB_STATE:
        per_name = {kk[len(f"_acamd/opt/{g}/{k}/"):]: v for kk, v in t.items() if kk.startswith(f"_acamd/opt/{g}/{k}/")}
        if not per_name:
            if k in sd and sd[k].numel() != getattr(opt, k).numel():
                raise ValueError(f"checkpoint {path}: optimiser state {g}/{k} has {sd[k].numel()} elements, this "
                                 f"slab {getattr(opt, k).numel()} (written with another parameter layout)")
            continue
        vec = torch.zeros_like(getattr(opt, k), device="cpu")
        for name, a, b in _param_ranges(trainer, opt):
            if name not in per_name:
                raise KeyError(f"checkpoint {path} lacks optimiser state {g}/{k}/{name}")
            vec[a:b] = torch.as_tensor(np.array(per_name[name])).reshape(-1)
        sd[k] = vec
    if sd:
        sd = {k: (v.reshape(()) if v.numel() == 1 and k in ("t", "lr") else v) for k, v in sd.items()}
        opt.load_state_dict(sd)


def save_trainer(trainer, path=None):
    """Checkpoint of an :class:`..algos.trainer.ActorCriticTrainer` (model + optimiser + counters + env banks).

    Without DP it is called on rank 0. With DP every rank must call it (the env states are gathered); rank 0
    writes and returns the path, the others return None. Resume is exact for the strict / single-graph schedules; a
    lag-1 DP run resumes without the in-flight delayed gradient."""
    cfg = trainer.cfg
    envs = _gather_env_states(trainer)
    if envs is None:
        return None
    base = f"model-{env_prefix(cfg.env)}"
    if path is None:
        os.makedirs(cfg.checkpoint_dir, exist_ok=True)
        path = os.path.join(cfg.checkpoint_dir, f"{base}-{trainer.iteration}")
    tensors = dict(model_tensors(trainer.model, cfg.model_variant, trainer.opts))
    for g, opt in trainer.opts.items():
        for k, v in opt.state_dict().items():
            if k in _SLAB_STATE:   # per parameter name: independent of the slab layout (parameter order, padding)
                for name, a, b in _param_ranges(trainer, opt):
                    tensors[f"_acamd/opt/{g}/{k}/{name}"] = v[a:b]
            else:
                tensors[f"_acamd/opt/{g}/{k}"] = v.reshape(-1) if v.dim() else v
    tensors["_acamd/iteration"] = np.asarray(trainer.iteration, dtype=np.int64)
    tensors["_acamd/env_steps"] = np.asarray(trainer.env_steps, dtype=np.int64)
    for k, v in envs[0].items():
        tensors[f"_acamd/env/{k}"] = v
    if len(envs) > 1:
        for r, st in envs.items():
            for k, v in st.items():
                tensors[f"_acamd/env/rank{r}/{k}"] = v
    tensors["_acamd/world_size"] = np.asarray(len(envs), dtype=np.int64)
    tensors["_acamd/update_counter"] = trainer.update_counter
    tensors["_acamd/ent_coef"] = trainer.ent_coef
    tensors["_acamd/kl_coef"] = trainer.kl_coef
    save_tensors(path, tensors)
    directory = os.path.dirname(path) or "."
    kept = _prune(directory, os.path.basename(path).rsplit("-", 1)[0], cfg.keep_checkpoints)
    _write_state_file(directory, path, kept or [path])
    return path


def _assign(dst, arr):
    with torch.no_grad():
        dst.copy_(torch.as_tensor(np.array(arr)).reshape(dst.shape).to(dst.device, dst.dtype))


def load_model(model, tensors, variant="basic", strict=True):
    """Copies bundle tensors into ``model`` (reference names for the MLP family, ``acamd/`` names otherwise)."""
    names = model_tensors(model, variant)
    missing = []
    for k, p in names.items():
        if not isinstance(p, torch.nn.Parameter):
            continue  # scalar hyper-parameter variables
        if k in tensors:
            _assign(p, tensors[k])
        else:
            missing.append(k)
    if strict and missing:
        raise KeyError(f"checkpoint lacks {missing}")
    return missing


def load_trainer(trainer, path):
    t = load_tensors(path)
    load_model(trainer.model, t, trainer.cfg.model_variant)
    # the model parameters are views into the flat slab; refresh the bf16 shadow of the native engine
    if trainer.shadow is not None:
        trainer.shadow.copy_(trainer.flat.data)
        if getattr(trainer, "engine", None) is not None:   # the engine's fragment-ordered conv weight copies
            trainer.engine.sync_frag()
    if getattr(trainer, "mlp", None) is not None:   # the MLP engine's weight fragment copies
        trainer.mlp.sync_shadow()
    for g, opt in trainer.opts.items():
        _load_opt_state(trainer, opt, g, t, path)
    if "_acamd/iteration" in t:
        trainer.iteration = int(t["_acamd/iteration"])
        trainer.env_steps = int(t["_acamd/env_steps"])
        world, rank = getattr(trainer, "world", 1), getattr(trainer, "rank", 0)
        saved = int(t["_acamd/world_size"]) if "_acamd/world_size" in t else 1
        if saved != world:
            raise ValueError(f"checkpoint {path} holds the env banks of {saved} rank(s); this job has {world}")
        pre = f"_acamd/env/rank{rank}/" if saved > 1 else "_acamd/env/"
        for k in ("state", "t", "tg", "ep_ret"):
            _assign(getattr(trainer.env, k), t[pre + k])
        _assign(trainer.storage.obs[0], t[pre + "obs"])
        if "_acamd/update_counter" in t:
            _assign(trainer.update_counter, t["_acamd/update_counter"])
        _assign(trainer.ent_coef, t["_acamd/ent_coef"])
        _assign(trainer.kl_coef, t["_acamd/kl_coef"])
    return trainer


def detect_variant(names):
    names = list(names)
    if any(n.startswith("global_actor/") for n in names):
        return "a3c"
    if any(n.startswith("Actor/") for n in names):
        return "basic"
    return "generic"


__all__ = ["codec", "save_trainer", "load_trainer", "save_tensors", "load_tensors", "load_model",
           "reference_tensors", "model_tensors", "latest_checkpoint", "detect_variant"]
