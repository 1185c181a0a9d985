"""Flat parameter slabs and fused optimisers (kernel K10 of SURVEY §2.4).

The reference runs ``clip_by_value`` + ``ApplyAdam`` per variable (17 variables for Pendulum,
``Basic_AC/policies.py:79-82``). Here every parameter of a model is a *view into one contiguous fp32 slab*
and so is its gradient; an optimiser step is ONE kernel over a slab segment:

    g = clip(g, -c, c)                      (element-wise, optional; reference: +-1 Basic, +-0.1 A3C)
    g *= min(1, max_norm / ||g||)           (optional global-norm clip; norm from a device reduction)
    m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2
    p -= lr * sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps)      (TF1 AdamOptimizer "epsilon hat" form)

``lr`` and the step ``t`` are device scalars, so the KL-adaptive lr controller and the schedules update them
without a host sync and the step can be captured in a hipGraph. The flat gradient slab is also exactly the
buffer the data-parallel engine all-reduces (one RCCL call per update, :mod:`..parallel.dp`). Optionally the
same kernel writes a bf16 shadow copy of the parameters for the MFMA forward/backward kernels.
"""
from __future__ import annotations

import torch

from .. import _native


class FlatParams:
    """Re-homes ``params`` into one fp32 slab (``data``) with a matching gradient slab (``grad``).

    ``groups`` maps a group name to ``(start, end)`` element offsets; params are laid out group by group.
    """

    ALIGN = 64  # group starts are 256-byte aligned (vectorised optimiser / all-reduce segments)
    PARAM_ALIGN = 8  # every param starts 16-byte aligned in the bf16 shadow too (16-byte vector loads in kernels)

    def __init__(self, named_groups, device=None):
        self.groups = {}
        self.params = []
        self.offsets = []
        total = 0
        for name, plist in named_groups.items():
            total = (total + self.ALIGN - 1) // self.ALIGN * self.ALIGN
            start = total
            for p in plist:
                total = (total + self.PARAM_ALIGN - 1) // self.PARAM_ALIGN * self.PARAM_ALIGN
                self.params.append(p)
                self.offsets.append(total)
                total += p.numel()
            self.groups[name] = (start, total)
        dev = device if device is not None else (self.params[0].device if self.params else "cpu")
        self.numel = total
        self.data = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        for p, off in zip(self.params, self.offsets):
            n = p.numel()
            self.data[off:off + n].copy_(p.data.reshape(-1).to(dev, torch.float32))
            p.data = self.data[off:off + n].view(p.shape)
            p.grad = self.grad[off:off + n].view(p.shape)

    def zero_grad(self):
        self.grad.zero_()

    def segment(self, name):
        s, e = self.groups[name]
        return self.data[s:e], self.grad[s:e]


class FusedAdam:
    """Adam (TF1 semantics) + optional element-wise / global-norm gradient clipping over a slab segment."""

    def __init__(self, flat: FlatParams, group="shared", lr=1e-3, betas=(0.9, 0.999), eps=1e-8, clip_value=None,
                 max_grad_norm=None, bf16_shadow=None):
        self.flat = flat
        self.group = group
        s, e = flat.groups[group]
        self.start, self.end = s, e
        dev = flat.data.device
        self.p, self.g = flat.data[s:e], flat.grad[s:e]
        self.m = torch.zeros_like(self.p)
        self.v = torch.zeros_like(self.p)
        self.lr = torch.tensor(float(lr), dtype=torch.float32, device=dev)
        self.t = torch.zeros((), dtype=torch.float32, device=dev)
        self.b1, self.b2 = betas
        self.eps = eps
        self.clip_value = clip_value
        self.max_grad_norm = max_grad_norm
        self.gnorm = torch.zeros((), dtype=torch.float32, device=dev)
        self.shadow = bf16_shadow  # optional bf16 tensor of the same numel (written by the native kernel)
        # sumsq partials (reduced by every optimiser workgroup) + the Adam step ticket (self-cleaning)
        self._partial = torch.zeros(256, dtype=torch.float32, device=dev)
        # (optim.hip: 8 shard counters + a top counter, one per 128-byte line)
        self._ticket = torch.zeros(9 * 32, dtype=torch.int32, device=dev)
        # native engine: the update kernel zeroes each gradient after reading it (saves a memset per step)
        self.zero_grad_after = False
        # data parallelism: the slab holds the SUM over ranks; the kernel folds the 1/world average into its read
        self.grad_mul = 1.0
        # sumsq partials already produced by the gradient kernel (MLP engine): the norm needs no extra launch
        self.ext_parts = None
        # fragment-ordered bf16 copies of some weights, written by the update (set_frag)
        self.frag = []
        self._frag_table = None
        # optional device int32 gate: the update is skipped while it is 0 (set_gate)
        self.gate = None
        # optional bf16 gradient read instead of g (bind_grad16: the all-reduced bf16 DP bucket, no cast back)
        self.g16 = None

    def bind_grad(self, grad_slab):
        """Read gradients from this group's segment of another slab (lag-1 DP reads the all-reduced copy)."""
        self.g = grad_slab[self.start:self.end]

    def bind_grad16(self, slab16):
        """Native step: read the gradient from this group's segment of a bf16 slab (bf16 DP buckets: the all-reduced
        comm buffer itself -- no cast back into the fp32 slab; the sum of squares reads it too). ``None`` unbinds."""
        self.g16 = None if slab16 is None else slab16[self.start:self.end]

    def set_frag(self, entries):
        """Fragment-ordered bf16 weight copies the update writes as it goes: ``entries`` = [(W fp32 view into this
        group, K rows, N cols, dst bf16 [K * N][, layout])]. layout -1 (default, ``optim.hip`` OptTrans): the conv
        kernels' order (``frag_order``), read as one contiguous 1 KB load per wave fragment (``cnn_fused.hip``
        frag_w1..3); layout -2 (at most one): the 32x32x16 B-fragment order of the rollout fc product
        (``frag_order_kc``, ``fc_rollout.hip``), whose region the kernel updates by wave items with a transposed
        512-byte store per wave."""
        self.frag = [tuple(e) if len(e) == 5 else tuple(e) + (-1,) for e in entries]
        for W, K, N, dst, lay in self.frag:
            off = (W.data_ptr() - self.p.data_ptr()) // 4
            assert 0 <= off and off + K * N <= self.p.numel() and W.numel() == K * N and lay in (-1, -2)
            assert K % 16 == 0 and N % 32 == 0 and dst.dtype == torch.bfloat16 and dst.numel() == K * N
            assert lay == -1 or (off % 4 == 0 and dst.data_ptr() % 16 == 0)
        assert sum(e[4] == -2 for e in self.frag) <= 1
        self._frag_table = self._table()

    def set_gate(self, gate):
        """Device int32 flag (``optim.hip`` OptSeg::gate): while it is 0 the native update is skipped -- parameters,
        moments and the Adam step count stay as they are (lag-1 data parallelism before its first all-reduced
        gradient, ``trainer.py`` _update_body_lag1). ``None`` removes it."""
        self.gate = gate
        self._frag_table = self._table()

    def table_rows(self):
        """Rows (offset, K, N, code, ptr) of this optimiser's copy / gate table (``optim.hip`` opt_load_trans)."""
        rows = [[(W.data_ptr() - self.p.data_ptr()) // 4, K, N, lay, dst.data_ptr()] for W, K, N, dst, lay in self.frag]
        if self.gate is not None:
            assert self.gate.dtype == torch.int32 and self.gate.numel() == 1
            rows.append([0, 1, 1, -9, self.gate.data_ptr()])
        return rows

    def _table(self):
        rows = self.table_rows()
        if not rows:
            return None
        assert len(rows) <= 8
        t = torch.zeros(8, 5, dtype=torch.int64)
        t[:len(rows)] = torch.tensor(rows, dtype=torch.int64)
        return t

    def _torch_frag(self):
        for W, K, N, dst, lay in getattr(self, "frag", ()):
            dst.copy_(frag_order(W, K, N) if lay == -1 else frag_order_kc(W, K, N))

    def set_lr(self, lr):
        self.lr.fill_(float(lr))

    def get_lr(self):
        return float(self.lr)

    @torch.no_grad()
    def step(self):
        if _native.use_native(self.p):
            self._native_step()
        elif self.gate is None or int(self.gate) != 0:
            self._torch_step()

    def _native_norm(self, ops):
        """Partial sums of squares of the (clipped) gradient; the update kernel reduces them to the global norm
        (and writes it to ``self.gnorm``). Returns the partials or None without a norm clip."""
        self._norm_mul = 1.0
        if self.max_grad_norm is None:
            return None
        if self.ext_parts is not None:
            return self.ext_parts
        if self.clip_value is not None:
            # the norm is taken after the element-wise clip (torch oracle order)
            assert self.g16 is None, "element-wise clip with bf16 gradient reads"
            g = self.g * self.grad_mul if self.grad_mul != 1.0 else self.g
            ops.sumsq(torch.clamp(g, -self.clip_value, self.clip_value), self._partial)
        else:
            ops.sumsq(self.g if self.g16 is None else self.g16, self._partial)
            self._norm_mul = self.grad_mul * self.grad_mul
        return self._partial

    def _native_step(self):
        ops = _native.require()
        parts = self._native_norm(ops)
        ops.adam_step(self.p, self.g, self.m, self.v, self.lr, self.t, parts, self.gnorm, self.shadow,
                      float(self.b1), float(self.b2), float(self.eps),
                      float(self.clip_value) if self.clip_value is not None else -1.0,
                      float(self.max_grad_norm) if self.max_grad_norm is not None else -1.0, self._ticket,
                      bool(self.zero_grad_after), float(self.grad_mul), float(self._norm_mul),
                      getattr(self, "_frag_table", None), self.g16)

    def _torch_step(self):
        g = self.g if self.g16 is None else self.g16.float()
        g = g * self.grad_mul if self.grad_mul != 1.0 else g
        if self.clip_value is not None:
            g = torch.clamp(g, -self.clip_value, self.clip_value)
        if self.max_grad_norm is not None:
            n = torch.sqrt((g * g).sum())
            self.gnorm.copy_(n * n)
            g = g * torch.clamp(self.max_grad_norm / (n + 1e-6), max=1.0)
        self.t += 1
        self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
        self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
        lr_t = self.lr * torch.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        self.p.sub_(lr_t * self.m / (torch.sqrt(self.v) + self.eps))
        if self.shadow is not None:
            self.shadow.copy_(self.p)
        self._torch_frag()

    def state_dict(self):
        return {"m": self.m, "v": self.v, "t": self.t, "lr": self.lr}

    def load_state_dict(self, sd):
        for k in ("m", "v", "t", "lr"):
            if k in sd:
                getattr(self, k).copy_(torch.as_tensor(sd[k]).to(getattr(self, k).device))


class FusedRMSprop(FusedAdam):
    """RMSprop (TF semantics: ``ms = rho ms + (1-rho) g^2; p -= lr g / sqrt(ms + eps)``), same slab mechanics.

    The usual Atari A2C optimiser (alpha=0.99, eps=1e-5, lr=7e-4, global-norm clip 0.5).
    """

    def __init__(self, flat, group="shared", lr=7e-4, alpha=0.99, eps=1e-5, clip_value=None, max_grad_norm=None,
                 bf16_shadow=None):
        super().__init__(flat, group, lr, (0.0, alpha), eps, clip_value, max_grad_norm, bf16_shadow)
        self.alpha = alpha

    def _native_step(self):
        ops = _native.require()
        parts = self._native_norm(ops)
        ops.rmsprop_step(self.p, self.g, self.v, self.lr, parts, self.gnorm, self.shadow,
                         float(self.alpha), float(self.eps),
                         float(self.clip_value) if self.clip_value is not None else -1.0,
                         float(self.max_grad_norm) if self.max_grad_norm is not None else -1.0,
                         bool(self.zero_grad_after), float(self.grad_mul), float(self._norm_mul),
                         getattr(self, "_frag_table", None), self.g16)

    def _torch_step(self):
        g = self.g if self.g16 is None else self.g16.float()
        g = g * self.grad_mul if self.grad_mul != 1.0 else g
        if self.clip_value is not None:
            g = torch.clamp(g, -self.clip_value, self.clip_value)
        if self.max_grad_norm is not None:
            n = torch.sqrt((g * g).sum())
            self.gnorm.copy_(n * n)
            g = g * torch.clamp(self.max_grad_norm / (n + 1e-6), max=1.0)
        self.v.mul_(self.alpha).addcmul_(g, g, value=1 - self.alpha)
        self.p.sub_(self.lr * g / torch.sqrt(self.v + self.eps))
        if self.shadow is not None:
            self.shadow.copy_(self.p)
        self._torch_frag()


class FusedGroupStep:
    """Steps several optimisers of the same kind and hyper-parameters (e.g. the reference's separate actor and critic
    Adam, ``Basic_AC/policies.py:79-82,142-143``) with ONE native launch (``opt_multi_kernel``): each group keeps its
    own lr / step / clip / norm; any sum-of-squares launches they need run first."""

    MAXT = 8

    def __init__(self, opts, copies=None):
        """``copies``: optional per-optimiser lists of (W view, K, N, F, G or None) -- the MLP engine's fp32 weight
        fragment copies (``ops/mlp.py``), written by the update itself: such a segment runs on the ITEM path of
        ``optim.hip`` (one workgroup per item of :meth:`item_table`)."""
        self.opts = list(opts)
        o0 = self.opts[0]
        self.adam = not isinstance(o0, FusedRMSprop)
        self._key = None
        self._words = self._fvals = None
        self._trans = None
        self._items = [None] * len(self.opts)
        if copies is not None:
            for k, o in enumerate(self.opts):
                if copies[k]:
                    self._items[k] = self.item_table(o, copies[k])
        own = [o.table_rows() for o in self.opts]
        if any(own):
            t = torch.zeros(len(self.opts), self.MAXT, 5, dtype=torch.int64)
            for k, rows in enumerate(own):
                assert len(rows) <= self.MAXT
                if rows:
                    t[k, :len(rows)] = torch.tensor(rows, dtype=torch.int64)
            self._trans = t

    @staticmethod
    def item_table(o, copies):
        """Item records (``optim.hip`` opt_items, 8 int64 each) covering optimiser ``o``'s whole segment: every weight
        with N % 64 == 0 as 16-row x 64-column blocks (type 1: the update plus whole 1 KB F / G fragment stores),
        other copied weights whole (type 2, K * N <= 1024), the rest as element ranges of <= 1024 (type 0)."""
        from .mlp import ngp2
        n = o.p.numel()
        recs, covered = [], []
        for W, K, N, F, G in copies:
            off = (W.data_ptr() - o.p.data_ptr()) // 4
            assert 0 <= off and off + K * N <= n and W.numel() == K * N
            assert F.numel() == ngp2(K) * ngp2(N) * 256 and (G is None or G.numel() == F.numel())
            if N % 64 == 0:
                assert off % 4 == 0 and F.data_ptr() % 16 == 0 and (G is None or G.data_ptr() % 16 == 0)
                gk, gn = ngp2(K), ngp2(N)
                for kt in range((K + 15) // 16):
                    for cg in range(N // 64):
                        fp = F.data_ptr() + 4 * ((4 * cg) * gk + kt) * 256
                        gp = G.data_ptr() + 4 * (kt * gn + 4 * cg) * 256 if G is not None else 0
                        recs.append([1, off + kt * 16 * N + cg * 64, min(16, K - kt * 16), N, fp, gp, gk * 256, 0])
            else:
                assert K * N <= 1024, "small copied weights are one workgroup item"
                recs.append([2, off, K, N, F.data_ptr(), G.data_ptr() if G is not None else 0, 0, 0])
            covered.append((off, off + K * N))
        pos = 0
        for a, b in sorted(covered) + [(n, n)]:
            assert a >= pos or b <= pos, "overlapping copied weights"
            while pos < a:
                c = min(1024, a - pos)
                recs.append([0, pos, c, 0, 0, 0, 0, 0])
                pos += c
            pos = max(pos, b)
        return torch.tensor(recs, dtype=torch.int64, device=o.p.device)

    @staticmethod
    def compatible(opts):
        if len(opts) < 2 or len(opts) > 4:
            return False
        kinds = {type(o) for o in opts}
        if len(kinds) != 1:
            return False
        o0 = opts[0]
        return all((o.b1, o.b2, o.eps) == (o0.b1, o0.b2, o0.eps) for o in opts)

    @torch.no_grad()
    def step(self, t_off=None):
        """``t_off`` (Adam): this step is step ``t + t_off + 1`` of a sequence whose counters the caller advances
        afterwards (:meth:`advance`) -- the launch skips the step ticket (one agent-scope atomic chain per launch)."""
        ops = _native.require()
        plain = [o for o in self.opts if o.max_grad_norm is not None and o.ext_parts is None and o.clip_value is None]
        if len(plain) > 1:
            # the groups' plain sums of squares (data parallelism: no engine-written partials) in ONE launch
            ops.sumsq_multi([o.g for o in plain], [o._partial for o in plain])
            for o in plain:
                o._norm_mul = o.grad_mul * o.grad_mul
            parts = [o._partial if o in plain else o._native_norm(ops) for o in self.opts]
        else:
            parts = [o._native_norm(ops) for o in self.opts]
        key = tuple((p.data_ptr() if p is not None else 0, o._norm_mul, o.grad_mul, o.g.data_ptr())
                    for p, o in zip(parts, self.opts))
        if key != self._key:
            words, fvals = [], []
            for p, o in zip(parts, self.opts):
                shadow = o.shadow.data_ptr() if o.shadow is not None else 0
                adam = self.adam
                items = self._items[len(words)]
                words.append([o.p.data_ptr(), o.g.data_ptr(), o.m.data_ptr() if adam else 0, o.v.data_ptr(),
                              o.p.numel(), o.lr.data_ptr(), o.t.data_ptr() if adam else 0,
                              p.data_ptr() if p is not None else 0, o.gnorm.data_ptr(), shadow,
                              o._ticket.data_ptr() if adam else 0,
                              items.data_ptr() if items is not None else 0,
                              items.shape[0] if items is not None else 0])
                fvals.append([float(o.clip_value) if o.clip_value is not None else -1.0,
                              float(o.max_grad_norm) if o.max_grad_norm is not None else -1.0,
                              float(o.grad_mul), float(o._norm_mul)])
            self._words = torch.tensor(words, dtype=torch.int64)
            self._fvals = torch.tensor(fvals, dtype=torch.float32)
            self._key = key
        o0 = self.opts[0]
        zero = all(o.zero_grad_after for o in self.opts)
        assert zero or not any(o.zero_grad_after for o in self.opts)
        ops.opt_multi(self._words, self._fvals, self._trans, self.adam, float(o0.b1), float(o0.b2), float(o0.eps),
                      zero, o0.p, -1 if (t_off is None or not self.adam) else int(t_off))

    def advance(self, n):
        """After ``n`` steps taken with ``t_off`` = 0 .. n-1: the Adam step counters move by ``n`` (one device add
        per group)."""
        if self.adam:
            for o in self.opts:
                o.t.add_(float(n))


def frag_order(W, K, N):
    """bf16 fragment-ordered copy of the row-major [K][N] weight ``W`` (``optim.hip`` OptTrans, ldt < 0): MFMA
    fragment (16-row tile, 32-wide k-step) of lane ``lg * 16 + row16`` at ((tile * N / 32 + kstep) * 64 + lane) * 8."""
    return W.reshape(K // 16, 16, N // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(-1).to(torch.bfloat16)


def frag_order_kc(W, K, N):
    """bf16 copy of the row-major [K][N] weight ``W`` in 32x32x16-MFMA B-fragment order (``fc_rollout.hip``): the
    fragment of (16-deep k block kb, 32-wide column block nb) is 1 KB contiguous, lane ``(k / 8 % 2) * 32 + n % 32``
    holding the 8 consecutive k at ((kb * N / 32 + nb) * 64 + lane) * 8."""
    return W.reshape(K // 16, 2, 8, N // 32, 32).permute(0, 3, 1, 4, 2).reshape(-1).to(torch.bfloat16)


SUMSQ_PARTS = 256   # optim.hip: partial slots of the global-norm reduction = max finaliser workgroups


def finalize_jobs(segments, device, return_max=False, split_planes=True):
    """Job table of the gradient finaliser (``grad_finalize``): ``segments`` = [(dst_ptr, src_ptr, n, stride, S)]
    (``src_ptr`` 0: final already, read for the norm). Plane reductions are cut into jobs of about equal load count
    (``n * S`` spread over the workgroups: 256- / 512-element jobs for the many-plane conv gradients when the budget
    allows -- more workgroups streaming the planes; the kernel splits such a job's planes over its thread groups --,
    long jobs for a two-plane fc gradient of 1.6 M elements, which at 1024 elements per job would not fit the job
    budget; ``split_planes`` False: 1024-element jobs throughout), per-sample
    bias rows (n <= 64) take one job each, and the read-only segments share the remaining workgroups in equal
    multiples of 1024 elements; at most ``SUMSQ_PARTS`` jobs. ``S = -1`` with ``src_ptr`` 0: ``n`` presummed sums of
    squares at ``dst_ptr`` (fc_bwd's per-tile partials), one job that adds them."""
    pre = [sg for sg in segments if not sg[1] and sg[4] < 0]   # presummed sums of squares: one job each
    segments = [sg for sg in segments if sg[1] or sg[4] >= 0]
    small = [sg for sg in segments if sg[1] and sg[2] <= 64]
    big = [sg for sg in segments if sg[1] and sg[2] > 64]
    ro = [sg for sg in segments if not sg[1]]
    budget = max(1, SUMSQ_PARTS - len(pre) - len(small) - max(1, len(ro)))
    target = max(1024.0, sum(n * S for _, _, n, _, S in big) / budget)   # plane loads per job
    while True:
        jobs = [list(sg) for sg in pre] + [[dst, src, n, stride, S] for dst, src, n, stride, S in small]
        for dst, src, n, stride, S in big:
            # many-plane segments in 256-element steps (the kernel splits their planes over thread groups), the
            # rest in multiples of 1024
            q = 256 if S >= 16 and split_planes else 1024
            ch = max(q, -(-int(target // max(1, S)) // q) * q)
            if q == 256 and ch > 512:
                ch = -(-ch // 1024) * 1024
            for a in range(0, n, ch):
                jobs.append([dst + 4 * a, src + 4 * a, min(ch, n - a), stride, S])
        left = SUMSQ_PARTS - len(jobs)
        total_ro = sum(sg[2] for sg in ro)
        if left >= max(1, len(ro)) or target > 1 << 40:
            break
        target *= 1.25
    if ro:
        ch = max(1024, -(-total_ro // max(1, left - len(ro))))
        ch = -(-ch // 1024) * 1024
        for dst, _, n, _, _ in ro:
            for a in range(0, n, ch):
                jobs.append([dst + 4 * a, 0, min(ch, n - a), 0, 0])
    if len(jobs) > SUMSQ_PARTS:
        raise ValueError("finalize_jobs: %d jobs exceed %d norm partials" % (len(jobs), SUMSQ_PARTS))
    rows = []
    for dst, src, n, stride, S in jobs:
        vec = int(dst % 16 == 0 and (not src or (src % 16 == 0 and stride % 4 == 0)))
        rows.append([dst, src, n, stride, S, vec, 0, 0])
    words = torch.tensor(rows, dtype=torch.int64).to(device)
    if return_max:   # the largest job (the fused finaliser + optimiser holds one job's elements in LDS)
        return words, max(r[2] for r in rows)
    return words


def make_optimizer(name, flat, group, lr, clip_value=None, max_grad_norm=None, bf16_shadow=None):
    if name == "adam":
        return FusedAdam(flat, group, lr, clip_value=clip_value, max_grad_norm=max_grad_norm,
                         bf16_shadow=bf16_shadow)
    if name == "rmsprop":
        return FusedRMSprop(flat, group, lr, clip_value=clip_value, max_grad_norm=max_grad_norm,
                            bf16_shadow=bf16_shadow)
    raise ValueError(name)
