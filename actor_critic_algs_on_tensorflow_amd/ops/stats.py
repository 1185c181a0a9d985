"""Device statistics reductions: the reference's ``variable_summaries`` (per-variable mean /
stddev / max / min, ``Basic_AC/policies.py:9-18``) over the flat parameter slab in ONE launch
(``seg_stats_kernel``, ``csrc/kernels/returns.hip``), with the PyTorch oracle for CPU tensors."""
from __future__ import annotations

import torch

from .. import _native


def param_segments(flat, params):
    """int64 [n, 2] (offset, numel) of ``params`` inside ``flat`` (a :class:`.optim.FlatParams`)."""
    idx = {id(p): i for i, p in enumerate(flat.params)}
    rows = [[flat.offsets[idx[id(p)]], p.numel()] for p in params]
    return torch.tensor(rows, dtype=torch.int64, device=flat.data.device)


def seg_stats_ref(x, segs):
    out = []
    for off, n in segs.tolist():
        v = x[off:off + n].double()
        out.append([v.mean(), v.var(unbiased=False).sqrt(), v.max(), v.min()])
    return torch.tensor(out, dtype=torch.float32, device=x.device)


def seg_stats(x, segs, out=None):
    """-> float32 [n, 4] (mean, population std, max, min) of each (offset, numel) segment of the flat tensor ``x``."""
    n = segs.shape[0]
    if _native.use_native(x):
        out = torch.empty(n, 4, dtype=torch.float32, device=x.device) if out is None else out
        _native.require().seg_stats(x.contiguous(), segs.contiguous(), out)
        return out
    r = seg_stats_ref(x, segs)
    if out is not None:
        out.copy_(r)
        return out
    return r
