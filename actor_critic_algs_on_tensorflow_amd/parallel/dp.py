"""Synchronous data parallelism over RCCL (``torch.distributed`` backend "nccl" == RCCL on ROCm) or gloo on CPU.

The reference has no collective communication at all -- only the asynchronous parameter server of
``A3C/process.py:156-214`` (reproduced in :mod:`.a3c`). This module is the BASELINE.json "sync-A2C data-parallel"
mode: one process per GPU, each owning its own env bank (``env_offset = rank * N`` so every
rank simulates different envs), identical parameters, and per update

  * ONE all-reduce of the flat fp32 gradient slab (every parameter's gradient is a view into it, so there is no
    bucketing bookkeeping: the whole model is one contiguous message -- 6.75 MB for the Atari CNN, one ring pass
    over xGMI), averaged;
  * ONE packed all-reduce of the scalar statistics that must be global (advantage sum / sum of squares / count
    for normalisation; the KL proxy for the adaptive lr), so every rank takes bit-identical optimiser steps.

Parameters are broadcast from rank 0 at start (the reference's race where every worker re-initialises the PS
variables, SURVEY §2.9 #11, cannot happen). RCCL timeouts surface as exceptions (fail fast).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def init_from_env(backend="auto", timeout_s=300):
    """Initialises the default process group from torchrun-style env vars; returns (rank, world, local_rank)."""
    if not dist.is_available():
        return 0, 1, 0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world <= 1:
        return 0, 1, 0
    if not dist.is_initialized():
        if backend == "auto":
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return dist.get_rank(), dist.get_world_size(), local


class DataParallel:
    """``compress="bf16"`` all-reduces the gradient slab as bf16 (half the xGMI bytes: 3.4 MB instead of 6.75 MB
    for the Atari CNN): a captured cast packs the fp32 slab (or a bucket range of it) into a persistent bf16 comm
    buffer, RCCL sums that, a captured cast unpacks it. Summation then happens in bf16 (rounding error grows with
    the world size); the default keeps fp32 buckets."""

    def __init__(self, group=None, average=True, compress=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.average = average
        if compress in ("none", "fp32"):
            compress = None
        if compress not in (None, "bf16"):
            raise ValueError(f"compress must be None/'none'/'bf16', got {compress!r}")
        self.compress = compress
        self._cbufs = {}   # gradient slab address -> its persistent bf16 comm buffer
        # bf16 buckets read in place by the optimisers (trainer binds them): unpack is then a no-op
        self.direct_read = False
        # RCCL ("nccl") collectives are stream-ordered and capturable: the trainer records them INSIDE its
        # hipGraph (one graph per update, the collective as a graph node on RCCL's stream with event joins).
        # gloo collectives run on the host, so a captured gloo update is a chain of graphs cut at each one.
        self.backend = dist.get_backend(group)
        self.issued = 0   # collectives issued from the host (a replayed one-graph update issues none)
        # RCCL: the stream-ordered all-reduces go straight to the process group's communicator ON THE CURRENT STREAM
        # (native rccl_allreduce) instead of through torch's collective, which runs on the group's internal stream
        # joined to the compute stream by two events -- graph edges that cost more than the all-reduce itself at the
        # per-minibatch gradient sizes (profiles/r6_dp_world1.txt). The async form (allreduce_async, overlapped with
        # compute) keeps torch's stream.
        # (while an async collective is outstanding on the group's stream, the stream-ordered ones go there too: two
        # collectives of one communicator must never run concurrently on two streams)
        self._comm = self._direct_comm() if self.backend == "nccl" else 0
        self._pending = 0

    def _direct_comm(self):
        from .. import _native
        if not (torch.cuda.is_available() and _native.available()):
            return 0
        dev = torch.device("cuda", torch.cuda.current_device())
        pg = self.group if self.group is not None else dist.distributed_c10d._get_default_group()
        try:
            # the communicator exists from init when the group was created with a device_id (init_from_env does
            # that); otherwise it is created lazily by torch and this returns 0 (torch's collectives are used)
            return int(pg._get_backend(dev)._comm_ptr())
        except (AttributeError, RuntimeError):
            return 0

    def _allreduce_now(self, t):
        """Stream-ordered in-place SUM all-reduce of ``t`` (on the current stream when the communicator is ours)."""
        self.issued += 1
        if self._comm and not self._pending:
            from .. import _native
            _native.require().rccl_allreduce(t, self._comm)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    # -- gradient buckets (optionally bf16) ----------------------------------------------------------------------
    def prepare(self, grad):
        """Allocates the persistent comm buffer of gradient slab ``grad`` (call outside any graph capture)."""
        if self.compress:
            b = self._cbufs.get(grad.data_ptr())
            if b is None or b.numel() != grad.numel():
                self._cbufs[grad.data_ptr()] = torch.zeros(grad.numel(), dtype=torch.bfloat16, device=grad.device)

    def comm_view(self, grad, s=0, e=None):
        """The tensor the collective runs on for range [s, e) of gradient slab ``grad``."""
        if self.compress:
            self.prepare(grad)
            return self._cbufs[grad.data_ptr()][s:e]
        return grad[s:e]

    @torch.no_grad()
    def pack(self, grad, s=0, e=None):
        if self.compress:
            self.comm_view(grad, s, e).copy_(grad[s:e])

    @torch.no_grad()
    def unpack(self, grad, s=0, e=None):
        if self.compress and not self.direct_read:
            grad[s:e].copy_(self.comm_view(grad, s, e))

    @torch.no_grad()
    def allreduce_packed(self, grad, s=0, e=None):
        """Synchronous (stream-ordered) SUM all-reduce of the packed range."""
        self._allreduce_now(self.comm_view(grad, s, e))

    # -- parameters ---------------------------------------------------------------------------------------------
    @torch.no_grad()
    def broadcast_params(self, flat, src=0):
        dist.broadcast(flat.data, src=src, group=self.group)

    # -- gradients ----------------------------------------------------------------------------------------------
    @property
    def graph_capturable(self):
        """Collectives can be recorded inside a hipGraph (RCCL); gloo needs host-side cuts."""
        return self.backend == "nccl"

    @property
    def grad_mul(self):
        """Factor the optimisers fold into their gradient read (1/world when averaging): the all-reduce leaves the
        SUM in the slab and no separate scaling pass runs."""
        return 1.0 / self.world_size if self.average else 1.0

    @torch.no_grad()
    def allreduce_grads(self, flat, scale=True):
        """Synchronous all-reduce of the whole gradient slab; ``scale=False`` leaves the sum (optimisers carrying
        ``grad_mul`` average on read)."""
        dist.all_reduce(flat.grad, op=dist.ReduceOp.SUM, group=self.group)
        if scale and self.average and self.world_size > 1:
            flat.grad.mul_(1.0 / self.world_size)

    @torch.no_grad()
    def allreduce_async(self, buf):
        """Issues the SUM all-reduce of ``buf`` (a contiguous slab segment) on the RCCL stream, ordered after the
        work already queued on the current stream, and returns the work handle. ``handle.wait()`` makes the
        *current stream* wait for it (no host block), so the caller keeps queueing compute that overlaps it."""
        self.issued += 1
        self._pending += 1
        return _Work(self, dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    # -- statistics ---------------------------------------------------------------------------------------------
    @torch.no_grad()
    def normalize_advantages(self, adv, eps=1e-8, extra=None):
        """Global population-std normalisation across ranks (one packed all-reduce of [sum, sumsq, n]). ``extra``:
        a small fp64 tensor summed in the same collective (written back in place; e.g. the deferred KL slot)."""
        a = adv.float()
        s = torch.stack([a.sum(), (a * a).sum(), torch.tensor(float(a.numel()), device=a.device)]).double()
        if extra is not None:
            s = torch.cat([s, extra.reshape(-1)])
        self.issued += 1
        dist.all_reduce(s, group=self.group)
        if extra is not None:
            extra.copy_(s[3:].reshape(extra.shape))
        mean = s[0] / s[2]
        var = torch.clamp(s[1] / s[2] - mean * mean, min=0.0)
        return ((a - mean.float()) / (eps + var.sqrt().float()))

    @torch.no_grad()
    def allreduce_sum_(self, t):
        """In-place SUM all-reduce of a small device tensor (e.g. the packed fp64 return-scan moments): no host
        round trip, capturable."""
        if t.dtype in (torch.float32, torch.bfloat16, torch.float64) and t.is_contiguous():
            self._allreduce_now(t)
        else:
            self.issued += 1
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    @torch.no_grad()
    def mean_scalar(self, x):
        y = x.detach().float().reshape(1).clone()
        dist.all_reduce(y, group=self.group)
        return (y / self.world_size).reshape(())

    @torch.no_grad()
    def sum_tensor(self, x):
        y = x.clone()
        dist.all_reduce(y, group=self.group)
        return y

    def barrier(self):
        dist.barrier(group=self.group)


class _Work:
    """Handle of an async all-reduce; ``wait()`` joins it to the current stream and lets the stream-ordered
    collectives take the direct path again."""

    def __init__(self, dp, work):
        self._dp, self._work, self._open = dp, work, True

    def wait(self):
        self._work.wait()
        if self._open:
            self._open = False
            self._dp._pending -= 1
