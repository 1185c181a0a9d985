"""Scalar statistics used in logs.

``var_accounted_for`` is the reference "explained variance" (``Basic_AC/util.py:4-12``): the Pearson
correlation of standardised target and prediction, population std (numpy ``ddof=0``), in [-1, 1].
``explained_variance`` is the conventional ``1 - Var[y - y_hat] / Var[y]`` offered alongside.
"""
from __future__ import annotations

import numpy as np
import torch


def var_accounted_for(target, pred):
    if isinstance(target, torch.Tensor) or isinstance(pred, torch.Tensor):
        t = torch.as_tensor(target, dtype=torch.float64).reshape(-1)
        p = torch.as_tensor(pred, dtype=torch.float64).reshape(-1).to(t.device)
        p = (p - p.mean()) / p.std(unbiased=False)
        t = (t - t.mean()) / t.std(unbiased=False)
        return float((t * p).mean())
    pred, target = np.asarray(pred).reshape(-1), np.asarray(target).reshape(-1)
    pred = (pred - np.mean(pred)) / np.std(pred)
    target = (target - np.mean(target)) / np.std(target)
    return float(np.mean(target * pred))


def var_accounted_for_tensor(target: torch.Tensor, pred: torch.Tensor) -> torch.Tensor:
    """Device-side EV correlation (no host sync); returns a 0-d fp32 tensor."""
    t = target.reshape(-1).float()
    p = pred.reshape(-1).float()
    p = (p - p.mean()) / p.std(unbiased=False)
    t = (t - t.mean()) / t.std(unbiased=False)
    return (t * p).mean()


def explained_variance(target, pred):
    t = np.asarray(target, dtype=np.float64).reshape(-1)
    p = np.asarray(pred, dtype=np.float64).reshape(-1)
    vy = np.var(t)
    return float("nan") if vy == 0 else float(1.0 - np.var(t - p) / vy)


def make_np(*t):
    """Lists -> numpy arrays (``Basic_AC/util.py:44-48``)."""
    return (np.array(x) for x in t)


def ob_feature_augment(obs_path):
    """obs, obs^2, t, t^2 features (``Basic_AC/util.py:108-118``; dead code in the reference, kept for API parity)."""
    obs_path = np.array(obs_path)
    obs2 = obs_path ** 2
    n = len(obs_path)
    tt = np.arange(n, dtype=np.float32).reshape(-1, 1) / max(n - 1, 1)
    tt2 = tt ** 2
    tt = tt * 2 - 1
    return list(np.concatenate([obs_path, obs2, tt, tt2], axis=1))


def summarize_tensor(x: torch.Tensor):
    """mean / stddev / max / min of a variable (the ``variable_summaries`` quartet, ``Basic_AC/policies.py:9-18``)."""
    x = x.detach().float()
    m = x.mean()
    return {"mean": float(m), "stddev": float(((x - m) ** 2).mean().sqrt()), "max": float(x.max()),
            "min": float(x.min())}
