"""Native GPU engine for the Nature-CNN actor-critic: explicit forward / backward on hand-written gfx950 kernels.

Autograd is replaced by a fixed schedule of launches over preallocated buffers (static addresses => the whole
rollout step and the whole learner step are hipGraph-capturable). Per batch of B observations:

forward   gemm(col1, W1^T) +b relu  -> y1   [B*400, 32]    col1 = im2col(obs uint8 NCHW)/255, k (c,i,j)
          gemm(col2, W2^T) +b relu  -> y2   [B*81, 64]     col2 = im2col(y1 NHWC), k (i,j,c)
          gemm(col3, W3^T) +b relu  -> y3   [B*49, 64] == [B, 3136]
          gemm(y3, Wfc)    +b relu  -> h    [B, 512]       (slab split-K for small B)
          gemm(h, Wh)      +b       -> z    [B, A+1] fp32  (logits | value)
loss      ac_loss(z, ...)           -> dz   [B, A+1] bf16, stats
backward  dWh += h^T dz ; dbh += colsum(dz)
          dh  = (dz Wh^T) * (h > 0)             (+ colsum -> dbfc)
          dWfc += y3^T dh
          dy3 = (dh Wfc^T) * (y3 > 0)           (+ per-channel colsum -> db3)
          dW3 += dy3^T col3 ; dy2 = conv_transpose(dy3, W3) * (y2 > 0)       (+ colsum -> db2)
          dW2 += dy2^T col2 ; dy1 = conv_transpose(dy2, W2) * (y1 > 0)       (+ colsum -> db1)
          (the transposed convs are GEMMs whose A rows are gathered from dy on the stride grid and whose B is the
          OHWI weight read as [(i, j, o)][c]; ``tconv_dgrad=False`` materialises dcol = dy W and runs col2im)
          dW1 += dy1^T col1
For rollout-sized batches (``fused_trunk_max_b``) conv1..conv3 run as ONE fused kernel (``cnn_fused.hip``: one env
per workgroup, activations handed off through LDS, MFMA 16x16x32); y1/y2/y3 still land in the buffers above so the
learner can reuse them. The column matrices ``col*`` are never materialised in the default (``implicit=True``) mode: the GEMM gathers its
k-contiguous A rows (forward) or n-contiguous B rows (weight gradient) straight from the activation image
(implicit im2col, ``gemm_impl.h``). ``implicit=False`` runs explicit im2col kernels + plain GEMMs (A/B reference).
Weight gradients accumulate (split-K atomics) straight into the fp32 gradient slab of :class:`FlatParams` (zeroed
by the optimiser after use), which is also the buffer the data-parallel engine all-reduces. Weights are read from
the bf16 shadow of the slab that the fused optimiser rewrites every step.
"""
from __future__ import annotations

import torch

from .. import _native
from ..ops import gemm as G

H0 = 84
FC_PLANES = 32   # split-K partial planes of the rollout fc product (cnn_head.h FC_MAX_PLANES)


class _Bufs:
    """Activation / gradient buffers for one batch size."""

    def __init__(self, B, A1, dev, with_grad, implicit=True):
        bf = torch.bfloat16
        self.B = B
        self.obs = None
        if not implicit:
            self.col1 = torch.empty(B * 400, 256, dtype=bf, device=dev)
            self.col2 = torch.empty(B * 81, 512, dtype=bf, device=dev)
            self.col3 = torch.empty(B * 49, 576, dtype=bf, device=dev)
        self.y1 = torch.empty(B * 400, 32, dtype=bf, device=dev)
        self.y2 = torch.empty(B * 81, 64, dtype=bf, device=dev)
        self.y3 = torch.empty(B * 49, 64, dtype=bf, device=dev)
        self.h = torch.empty(B, 512, dtype=bf, device=dev)
        self.z = torch.empty(B, A1, dtype=torch.float32, device=dev)
        if with_grad:
            self.dz = torch.empty(B, A1, dtype=bf, device=dev)
            self.dh = torch.empty(B, 512, dtype=bf, device=dev)
            self.dy3 = torch.empty(B * 49, 64, dtype=bf, device=dev)
            self.dy2 = torch.empty(B * 81, 64, dtype=bf, device=dev)
            self.dy1 = torch.empty(B * 400, 32, dtype=bf, device=dev)
            self.biasp = torch.zeros(B, 160, dtype=torch.float32, device=dev)   # per-sample db3 | db2 | db1
            self.stats = torch.zeros(8, dtype=torch.float32, device=dev)

    def rows(self, r0, n):
        """Forward-only view of rows [r0, r0+n) (one rollout step writing into a learner-sized buffer)."""
        v = _Bufs.__new__(_Bufs)
        v.B = n
        v.obs = None
        v.y1 = self.y1[r0 * 400:(r0 + n) * 400]
        v.y2 = self.y2[r0 * 81:(r0 + n) * 81]
        v.y3 = self.y3[r0 * 49:(r0 + n) * 49]
        v.h = self.h[r0:r0 + n]
        v.z = self.z[r0:r0 + n]
        for name in ("col1", "col2", "col3"):
            if hasattr(self, name):
                k = {"col1": 400, "col2": 81, "col3": 49}[name]
                setattr(v, name, getattr(self, name)[r0 * k:(r0 + n) * k])
        return v


class CNNEngine:
    """Explicit forward/backward of :class:`..models.policy.CNNActorCritic` over a :class:`FlatParams` slab."""

    def __init__(self, model, flat, shadow, implicit=True, fused_trunk_max_b=None, tconv_dgrad=None, opts=None):
        from ..config import EngineOpts
        net = model.net
        o = self.opts = opts if opts is not None else EngineOpts()
        self.implicit = implicit
        # data gradients of conv3/conv2 as transposed-conv GEMMs gathered from dy (no dcol matrix, no col2im pass)
        self.tconv_dgrad = implicit if tconv_dgrad is None else tconv_dgrad
        # one workgroup per env: the fused trunk wins whenever the per-layer GEMMs are launch/latency bound
        self.fused_trunk_max_b = 4096 if fused_trunk_max_b is None else fused_trunk_max_b
        # rollout batches up to trunk_rows_max_b envs: seven row workgroups per env (224 CUs at 32 envs; mode 2 issues
        # the conv2/conv3 weight loads after conv1, leaving conv1 the registers to pipeline its LDS reads). Larger
        # batches already fill the chip with one workgroup per env (mode 3), where the split's recomputed receptive
        # fields only cost
        self.trunk_mode = 2
        self.trunk_rows_max_b = o.trunk_rows_max_b
        # learner data-gradient chain dy3 -> dy2 -> dy1 as ONE per-sample kernel (cnn_trunk_bwd; bias gradients as
        # per-sample partial rows reduced by the gradient finaliser) instead of two transposed-conv GEMMs
        self.fused_bwd = implicit and o.fused_bwd
        self.fin_parts = torch.zeros(256, dtype=torch.float32, device=flat.data.device)
        # A2C head in one launch (head_bwd: loss + dz + dh + dWh + dbh + dbfc, no GEMMs) for categorical heads of up
        # to 7 actions and learner batches up to 1024 rows
        self.fused_head = o.fused_head
        # A2C head v2 (loss.hip a2c_head_kernel): bootstrap value + returns + loss + head backward in one launch of 32
        # narrow workgroups (off: fc_value + the 8-workgroup head_bwd kernel of round 2)
        self.a2c_head = o.a2c_head
        self._a2c_bar = None
        self._fcb_sq = None    # fc_bwd's per-tile dWfc sums of squares (the finaliser's presummed norm job)
        self._cur_presum = False
        # A2C head v3 (loss.hip a2c_head_env_kernel): one workgroup per env, no grid-wide hand-off; the head's weight /
        # bias gradients as per-env planes and the statistics as per-env rows, both reduced by the finaliser
        self.a2c_head_env = o.a2c_head_env
        self._ae = {}
        self._stats_duty = None
        # A2C learner on ONE stream with grouped GEMM launches instead of a side stream joined by events
        self.grouped = o.grouped
        # conv weight gradients as split-K partial planes reduced in plane order by the finaliser (deterministic);
        # off: split-K fp32 atomics into the slab (nondeterministic summation order)
        self.det_wgrad = implicit and o.det_wgrad
        self.wgrad_planes = o.wgrad_planes
        # learner batches from large_batch_min_b rows up: the conv1 weight gradient by the per-sample kernel
        # (conv_wgrad.hip: frames + dy1 staged once per sample) or folded into the persistent trunk backward instead
        # of the implicit-im2col GEMM; conv2 / conv3 weight gradients by the batched-position MFMA kernel (one
        # workgroup per plane: 256 planes cover the CUs); the backward on ONE stream (Breakout PPO 18.3 -> 17.0 ms per
        # update, profiles/r3_breakout_ab.txt); the fused trunk backward as a persistent kernel (weights in registers,
        # one workgroup per CU walking the samples)
        self.large_b = o.large_batch_min_b
        self.nhwc_planes = o.nhwc_planes
        self.trunk_bwd_persist = o.trunk_bwd_persist
        self._planes = {}
        self._wsplits = {}
        self._cur_planes = {}
        self._fin_words = {}
        self._retired = []     # outgrown plane buffers (+ the tables naming them) kept for captured graphs
        # rollout fc product left as split-K partial planes, reduced by its consumer kernel (no in-launch fence)
        self.fc_parts = True
        # split-K planes the fc GEMM may use (more planes: more workgroups stream Wfc, more for the consumer to sum)
        self.fc_max_planes = min(FC_PLANES, o.fc_max_planes)
        self._hpart = {}
        self.last_fc = None
        self._head_planes = {}   # plane sets written by ppo_head, merged into the next backward's finaliser jobs
        self._ph = {}
        self.model = model
        self.flat = flat
        self.shadow = shadow
        self.A = net.num_actions
        self.A1 = self.A + 1
        self.dev = flat.data.device
        self.ws = G.GemmWorkspace(self.dev)
        self.big_ws = G.GemmBigWorkspace(self.dev) if self.dev.type == "cuda" else None
        tr = net.trunk
        assert tr.conv1.cin == 4 and tr.conv1.layout == "oihw" and tr.conv2.layout == "ohwi"
        idx = {id(p): i for i, p in enumerate(flat.params)}

        def views(p):
            i = idx[id(p)]
            off, n = flat.offsets[i], p.numel()
            return (flat.data[off:off + n], flat.grad[off:off + n], shadow[off:off + n])

        self.W1, self.gW1, self.sW1 = views(tr.conv1.weight)
        self.b1, self.gb1, _ = views(tr.conv1.bias)
        self.W2, self.gW2, self.sW2 = views(tr.conv2.weight)
        self.b2, self.gb2, _ = views(tr.conv2.bias)
        self.W3, self.gW3, self.sW3 = views(tr.conv3.weight)
        self.b3, self.gb3, _ = views(tr.conv3.bias)
        self.Wfc, self.gWfc, self.sWfc = views(tr.fc.kernel)
        self.bfc, self.gbfc, _ = views(tr.fc.bias)
        self.Wh, self.gWh, self.sWh = views(net.heads.kernel)
        self.bh, self.gbh, _ = views(net.heads.bias)
        self._gslab = flat.grad
        self._bufs = {}
        # fragment-ordered bf16 copies of the conv weights (ops/optim.py frag_order), rewritten by the optimiser step
        # itself (FusedAdam.set_frag): the fused trunk kernels' weight loads read 1 KB per wave contiguously instead
        # of 16 rows x 64 bytes (profiles/r4_l2_stream_probe.txt: 16 vs ~60 B/clk/CU from L2)
        self.frag = None
        if o.frag_weights and self.dev.type == "cuda" and implicit:
            self.frag = [torch.empty(n, dtype=torch.bfloat16, device=self.dev) for n in (32 * 256, 64 * 512, 64 * 576)]
            self.sync_frag()
        # fragment-ordered bf16 copy of Wfc for the rollout fc product (fc_rollout.hip, EngineOpts.fc_frag)
        self.fc_frag = o.fc_frag if (self.dev.type == "cuda" and o.fc_frag >= 0) else -1
        self.wfc_frag = None
        if self.fc_frag >= 0:
            self.wfc_frag = torch.empty(3136 * 512, dtype=torch.bfloat16, device=self.dev)
            self.sync_fc_frag()
        self.side = torch.cuda.Stream(device=self.dev) if self.dev.type == "cuda" else None
        self._ev = [torch.cuda.Event() for _ in range(6)] if self.side is not None else None

    _FRAG_SHAPES = ((32, 256), (64, 512), (64, 576))

    def use_grad_slab(self, slab):
        """Every gradient this engine writes goes to ``slab`` (a tensor laid out like ``flat.grad``) from now on: the
        captured launches record its addresses (lag-1 data parallelism captures the two ring-phase graph sets on
        two slabs -- one written by the backward while the other is all-reduced and applied; no C <- G copy)."""
        assert slab.shape == self.flat.grad.shape and slab.dtype == self.flat.grad.dtype
        net = self.model.net
        tr = net.trunk
        idx = {id(p): i for i, p in enumerate(self.flat.params)}

        def gv(p):
            off = self.flat.offsets[idx[id(p)]]
            return slab[off:off + p.numel()]

        self.gW1, self.gb1 = gv(tr.conv1.weight), gv(tr.conv1.bias)
        self.gW2, self.gb2 = gv(tr.conv2.weight), gv(tr.conv2.bias)
        self.gW3, self.gb3 = gv(tr.conv3.weight), gv(tr.conv3.bias)
        self.gWfc, self.gbfc = gv(tr.fc.kernel), gv(tr.fc.bias)
        self.gWh, self.gbh = gv(net.heads.kernel), gv(net.heads.bias)
        # the finaliser job tables built for the old slab, re-pointed at the new one (tables are uploaded outside
        # graph capture: a capture of the other ring phase must find its tables ready)
        old = self._gslab
        if old.data_ptr() != slab.data_ptr():
            lo, hi, delta = old.data_ptr(), old.data_ptr() + old.numel() * 4, slab.data_ptr() - old.data_ptr()
            for key, (words, mx) in list(self._fin_words.items()):
                nk = key[:-1] + (slab.data_ptr(),)
                if key[-1] == lo and nk not in self._fin_words:
                    w = words.cpu().clone()
                    hit = (w[:, 0] >= lo) & (w[:, 0] < hi)
                    w[hit, 0] += delta
                    self._fin_words[nk] = (w.to(words.device), mx)
        self._gslab = slab

    def frag_entries(self):
        """(fp32 W view, rows, cols, fragment-ordered bf16 copy, layout) of conv1..3 (layout -1) and, with
        ``fc_frag``, of Wfc (layout -2: the rollout fc product's B-fragment order) for the optimiser
        (``set_frag``): the update writes them as it goes."""
        ent = []
        if self.frag is not None:
            ent += [(W, K, N, F, -1) for W, (K, N), F in zip((self.W1, self.W2, self.W3), self._FRAG_SHAPES, self.frag)]
        if self.wfc_frag is not None:
            ent.append((self.Wfc, 3136, 512, self.wfc_frag, -2))
        return ent

    @torch.no_grad()
    def sync_frag(self):
        """Rebuild the fragment-ordered copies from the bf16 shadow (parameters changed outside the optimiser:
        construction, checkpoint load, parameter-server pull)."""
        self.sync_fc_frag()
        if self.frag is None:
            return
        from ..ops.optim import frag_order
        for S, (K, N), F in zip((self.sW1, self.sW2, self.sW3), self._FRAG_SHAPES, self.frag):
            F.copy_(frag_order(S, K, N))

    @torch.no_grad()
    def sync_fc_frag(self):
        """Rebuild the fragment-ordered Wfc copy from the bf16 shadow."""
        if getattr(self, "wfc_frag", None) is not None:
            from ..ops.optim import frag_order_kc
            self.wfc_frag.copy_(frag_order_kc(self.sWfc, 3136, 512))

    def _fc_rollout(self, b, hp):
        """Split-K planes of the rollout fc product into ``hp``; returns the plane count."""
        # (up to 32 envs: variant fc_frag, one 32-row block per wave; 33..128 envs: fc_frag_big -- the per-wave
        # row-block loop measured slower than the general GEMM at 128 envs, the row blocks split over workgroups
        # slightly faster, profiles/r5_fc_frag_breakout.txt)
        if self.fc_frag >= 0 and b.B <= 32:
            return int(_native.require().fc_rollout(b.y3.view(b.B, 3136), self.wfc_frag, hp, self.fc_frag))
        if self.fc_frag >= 0 and self.opts.fc_frag_big >= 0 and b.B <= 128:
            return int(_native.require().fc_rollout(b.y3.view(b.B, 3136), self.wfc_frag, hp, self.opts.fc_frag_big))
        return G.gemm(b.y3, 3136, True, self.sWfc, 512, False, hp, 512, 3, b.B, 512, 3136, workspace=self.ws,
                      max_planes=self.fc_max_planes)

    def trunk_w(self):
        """(W1, W2, W3) operands of the fused trunk kernels and whether they are fragment-ordered."""
        if self.frag is not None:
            return (*self.frag, True)
        return (self.sW1, self.sW2, self.sW3, False)

    def bufs(self, B, with_grad=False):
        key = (B, with_grad)
        if key not in self._bufs:
            self._bufs[key] = _Bufs(B, self.A1, self.dev, with_grad, self.implicit)
        return self._bufs[key]

    # ------------------------------------------------------------------------------------------------ forward
    def hpart(self, B, slot=0):
        """fp32 [FC_PLANES, B, 512] split-K partial planes of the rollout fc product (GEMM out_mode 3)."""
        key = (B, slot)
        if key not in self._hpart:
            self._hpart[key] = torch.zeros(FC_PLANES * B * 512, dtype=torch.float32, device=self.dev)
        return self._hpart[key]

    def value(self, obs, b: _Bufs, out):
        """Bootstrap value of ``obs`` written straight into ``out`` [B] (trunk + the value column of the head)."""
        if self.fc_parts:
            self.forward(obs, b, head=False, fc_parts=True)
            hp, S = self.last_fc
            _native.require().fc_value(hp, S, self.bfc, self.sWh, self.bh, out, None)
            return out
        self.forward(obs, b, head=False)
        A, A1 = self.A, self.A1
        G.gemm(b.h, 512, True, self.sWh[A:], A1, False, out, 1, 0, b.B, 1, 512, bias=self.bh[A:],
               workspace=self.ws)
        return out

    def a2c_head_timed_out(self):
        """True if an ``a2c_head`` launch's bounded in-launch hand-off ever gave up waiting (word 2 of its barrier
        block, sticky): V(s_T) may then have been read before it was written, so the returns, advantages and
        gradients of that update are wrong. One host read (syncs); the trainer checks it at log / checkpoint time
        and after the capture warm-up."""
        return self._a2c_bar is not None and int(self._a2c_bar[2]) != 0

    def health_errors(self):
        """Names of the in-launch hand-offs that timed out since the engine was built (empty = healthy)."""
        return ["a2c_head bootstrap-value hand-off"] if self.a2c_head_timed_out() else []

    def fused_step_ok(self, B):
        """The rollout step can run as ONE launch of policy/env + the next observation's row-split trunk."""
        return (self.opts.fused_step and self.implicit and B <= min(self.trunk_rows_max_b, self.fused_trunk_max_b)
                and 2 <= self.A <= 6)

    def fused_env_step_ok(self, B):
        """Banks too large for the row-split trunk: ONE per-env launch of policy/env + the next observation's trunk
        (``pong_fused_env_step``) per rollout step."""
        return (self.opts.fused_step and self.implicit and self.trunk_rows_max_b < B <= self.fused_trunk_max_b
                and 2 <= self.A <= 6)

    def fc_planes(self, b: _Bufs):
        """fc product of ``b.y3`` as split-K partial planes (consumed by the fused step / value kernels)."""
        hp = self.hpart(b.B)
        S = self._fc_rollout(b, hp)
        self.last_fc = (hp, S)
        return hp, S

    def obs_index_ok(self, B):
        """A learner batch of ``B`` rows can read its observations through an index (PPO minibatch gathered by
        index, ``mb_gather`` index mode): the per-env lean-LDS trunk kernel and the per-sample conv1 weight-gradient
        kernel are the only readers of the frames then (``EngineOpts.mb_index`` off: copy the minibatch's
        observations)."""
        return (self.opts.mb_index and self.implicit and self.det_wgrad and B <= self.fused_trunk_max_b
                and B > self.trunk_rows_max_b and B >= self.large_b)

    def forward(self, obs, b: _Bufs, head=True, shift_out=None, fc_parts=False, obs_idx=None):
        """obs uint8 [B, 4, 84, 84] -> b.z fp32 [B, A+1] (logits | value); ``head=False`` stops at ``b.h`` (the
        rollout fuses the head into the sampling + env-step kernel). ``shift_out``: the next observation buffer,
        whose frames 0..2 the fused trunk fills with frames 1..3 of ``obs``; returns True iff it did."""
        B = b.B
        ws = self.ws
        b.obs = obs  # the conv1 weight gradient re-gathers its columns from the frames
        b.obs_idx = obs_idx   # None, or: sample r is row obs_idx[r] of obs
        assert obs_idx is None or (self.obs_index_ok(B) and obs_idx.numel() == B and shift_out is None)
        shifted = False
        want_shift = shift_out is not None
        if self.implicit and B <= self.fused_trunk_max_b:
            if B > self.trunk_rows_max_b and self.frag is not None:
                F1, F2, F3 = self.frag   # mode 5: the bf16-staged kernel on the fragment-ordered weights
                G.cnn_trunk_fwd(obs, F1, self.b1, F2, self.b2, F3, self.b3, b.y1, b.y2, b.y3, shift_out=shift_out,
                                mode=5, obs_idx=obs_idx)
            elif B <= self.trunk_rows_max_b and self.frag is not None:
                _, F2, F3 = self.frag   # modes 6 / 7: the row-split kernel on fragment-ordered conv2 / conv3 weights
                G.cnn_trunk_fwd(obs, self.sW1, self.b1, F2, self.b2, F3, self.b3, b.y1, b.y2, b.y3,
                                shift_out=shift_out, mode=self.trunk_mode + 5, obs_idx=obs_idx)
            else:
                G.cnn_trunk_fwd(obs, self.sW1, self.b1, self.sW2, self.b2, self.sW3, self.b3, b.y1, b.y2, b.y3,
                                shift_out=shift_out, mode=self.trunk_mode if B <= self.trunk_rows_max_b else 3,
                                obs_idx=obs_idx)
            shifted = shift_out is not None
        elif self.implicit:
            G.gemm(obs, 0, True, self.sW1, 256, True, b.y1, 32, 1, B * 400, 32, 256, bias=self.b1, relu=True,
                   workspace=ws, ga=[1, B, 4, 84, 84, 8, 8, 4], ga_scale=1.0 / 255.0)
            G.gemm(b.y1, 0, True, self.sW2, 512, True, b.y2, 64, 1, B * 81, 64, 512, bias=self.b2, relu=True,
                   workspace=ws, ga=[2, B, 32, 20, 20, 4, 4, 2])
            G.gemm(b.y2, 0, True, self.sW3, 576, True, b.y3, 64, 1, B * 49, 64, 576, bias=self.b3, relu=True,
                   workspace=ws, ga=[2, B, 64, 9, 9, 3, 3, 1])
        else:
            G.im2col_u8(obs, b.col1, 8, 8, 4)
            G.gemm(b.col1, 256, True, self.sW1, 256, True, b.y1, 32, 1, B * 400, 32, 256, bias=self.b1, relu=True,
                   workspace=ws)
            G.im2col_nhwc(b.y1, b.col2, B, 20, 20, 32, 4, 4, 2)
            G.gemm(b.col2, 512, True, self.sW2, 512, True, b.y2, 64, 1, B * 81, 64, 512, bias=self.b2, relu=True,
                   workspace=ws)
            G.im2col_nhwc(b.y2, b.col3, B, 9, 9, 64, 3, 3, 1)
            G.gemm(b.col3, 576, True, self.sW3, 576, True, b.y3, 64, 1, B * 49, 64, 576, bias=self.b3, relu=True,
                   workspace=ws)
        if fc_parts and not head and self.big_gemm_ok(B):
            # learner batch: the two split-K planes of the large-tile product, reduced (+ bias, ReLU) by ppo_head
            hp = self._big_planes("hfc", 2 * B * 512)
            G.gemm_big(b.y3, 3136, True, self.sWfc, 512, False, hp, 512, 3, B, 512, 3136, splits=2)
            self.last_fc = (hp, 2)
            return shifted if want_shift else b.z
        if fc_parts and not head:
            # partial planes only: the consumer (fused policy/env kernel or fc_value) reduces, adds the bias,
            # applies ReLU and writes b.h
            hp = self.hpart(B)
            S = self._fc_rollout(b, hp)
            self.last_fc = (hp, S)
            return shifted if want_shift else b.z
        if self.big_gemm_ok(B):   # 128 x 128 tiles, 2 splits: 256 workgroups at B = 4096
            G.gemm_big(b.y3, 3136, True, self.sWfc, 512, False, b.h, 512, 1, B, 512, 3136, bias=self.bfc, relu=True,
                       splits=2, workspace=self.big_ws)
        else:
            G.gemm(b.y3, 3136, True, self.sWfc, 512, False, b.h, 512, 1, B, 512, 3136, bias=self.bfc, relu=True,
                   workspace=ws)
        if head:
            G.gemm(b.h, 512, True, self.sWh, self.A1, False, b.z, self.A1, 0, B, self.A1, 512, bias=self.bh,
                   workspace=ws)
        return shifted if want_shift else b.z

    # ------------------------------------------------------------------------------------------------ backward
    def tail_bucket(self):
        """(start, end) slab offsets of the parameters whose gradients are final after the ``"tail"`` backward stage:
        the fc weight (95% of the bytes), stored by the fc-layer backward. It sits at the end of the slab
        (``CNNActorCritic.param_groups``), so data parallelism can all-reduce it while the conv backward (``"trunk"``
        stage) runs and then the rest -- conv, head and fc-bias gradients, the latter two summed from the head
        launch's partial planes by the trunk stage's finaliser -- as the contiguous range before it."""
        base = self._gslab.data_ptr()
        start = (self.gWfc.data_ptr() - base) // 4
        end = start + self.gWfc.numel()
        assert self._gslab.numel() - end < 64, "the fc weight must close the slab (up to alignment padding)"
        for g in (self.gW1, self.gb1, self.gW2, self.gb2, self.gW3, self.gb3, self.gbfc, self.gWh, self.gbh):
            assert (g.data_ptr() - base) // 4 + g.numel() <= start, "every other gradient must precede the fc weight"
        return start, end

    def _wgrad(self, name, gview, A, lda, B_, ldb, M, N, K, ws, gb, gb_scale=1.0):
        """Conv weight gradient dW = A^T-ish product over the batch rows (K): deterministic split-K planes reduced
        by the finaliser (``det_wgrad``), else atomics straight into the slab."""
        if not self.det_wgrad:
            G.gemm(A, lda, False, B_, ldb, False, gview, N, 2, M, N, K, workspace=ws, gb=gb, gb_scale=gb_scale)
            return
        buf = self._planes.get(name)
        if buf is None:
            buf = torch.zeros(self.wgrad_planes * M * N, dtype=torch.float32, device=self.dev)
            self._planes[name] = buf
        S = G.gemm(A, lda, False, B_, ldb, False, buf, N, 3, M, N, K, workspace=ws, gb=gb, gb_scale=gb_scale,
                   max_planes=self.wgrad_planes)
        self._wsplits[name] = S
        self._cur_planes[name] = S

    def _trunk_bwd(self, b, fold=False):
        """dy3 -> dy2 -> dy1 (+ the bias-gradient rows); ``fold``: the persistent form of a large batch also computes
        the conv1 weight gradient (one plane per workgroup, dy1 never stored; returns True when it did)."""
        persist = self.trunk_bwd_persist if b.B >= self.large_b else 0
        acc = self.bias_rows(b.B) < b.B
        if fold and persist and self.conv1_fold_ok(b.B):
            R = min(persist, b.B)
            buf = self._plane_buf("W1f", R * 32 * 256)
            _native.require().cnn_trunk_bwd(b.dy3, self.sW3, b.y2, self.sW2, b.y1, b.dy2, b.dy1, b.biasp, None,
                                            persist, b.obs, getattr(b, "obs_idx", None), buf, 1.0 / 255.0, acc, True)
            self._cur_planes["W1f"] = R
            return True
        _native.require().cnn_trunk_bwd(b.dy3, self.sW3, b.y2, self.sW2, b.y1, b.dy2, b.dy1, b.biasp, None, persist,
                                        None, None, None, 1.0, acc)
        return False

    def conv1_fold_ok(self, B):
        """The persistent trunk backward of a ``B``-row batch also computes the conv1 weight gradient."""
        return (self.dev.type == "cuda" and self.det_wgrad and self.implicit and B >= self.large_b
                and self.trunk_bwd_persist > 0)

    def bias_rows(self, B):
        """Bias-gradient partial rows the trunk backward of a ``B``-row batch leaves for the finaliser: one per
        sample, or one per workgroup of the persistent kernel."""
        if B >= self.large_b and self.trunk_bwd_persist < B:
            return self.trunk_bwd_persist
        return B

    def _wgrad_conv23(self, name, b, ws2):
        B = b.B
        if not (self.det_wgrad and self.implicit and B >= self.large_b):
            if name == "W2":
                self._wgrad("W2", self.gW2, b.dy2, 64, b.y1, 0, 64, 512, B * 81, ws2, [2, B, 32, 20, 20, 4, 4, 2])
            else:
                self._wgrad("W3", self.gW3, b.dy3, 64, b.y2, 0, 64, 576, B * 49, ws2, [2, B, 64, 9, 9, 3, 3, 1])
            return
        n = 512 if name == "W2" else 576
        P = max(1, min(self.nhwc_planes, B))
        buf = self._planes.get(name)
        if buf is None or buf.numel() < P * 64 * n:
            buf = self._plane_buf(name, max(P, self.wgrad_planes) * 64 * n)
        # batched-position MFMA 32x32x16 kernel
        fn = _native.require().conv_wgrad_gemm
        if name == "W2":
            fn(2, b.y1, b.dy2, buf, P)
        else:
            fn(3, b.y2, b.dy3, buf, P)
        self._wsplits[name] = P
        self._cur_planes[name] = P

    def _wgrad_conv1(self, b, ws):
        B = b.B
        if not (self.det_wgrad and self.implicit and B >= self.large_b):
            self._wgrad("W1", self.gW1, b.dy1, 32, b.obs, 0, 32, 256, B * 400, ws, [1, B, 4, 84, 84, 8, 8, 4],
                        1.0 / 255.0)
            return
        P = max(1, min(self.opts.conv1_v2_planes, B))
        buf = self._planes.get("W1")
        if buf is None or buf.numel() < P * 32 * 256:
            buf = self._plane_buf("W1", max(P, self.wgrad_planes) * 32 * 256)
        _native.require().conv1_wgrad(b.obs, b.dy1, buf, P, 1.0 / 255.0, getattr(b, "obs_idx", None))
        self._wsplits["W1"] = P
        self._cur_planes["W1"] = P

    def ppo_head_ok(self, B):
        """The large-batch head launch (``ppo_head.hip``) can take a learner batch of ``B`` rows: categorical head of
        2..7 actions, the grouped deterministic backward that starts at the fc layer."""
        return (self.opts.ppo_head and self.dev.type == "cuda" and 3 <= self.A1 <= 8 and self.grouped
                and self.fused_bwd and self.det_wgrad and B >= 1)

    def _big_planes(self, name, n):
        return self._plane_buf(name, n)

    def _plane_buf(self, name, n):
        """Plane set ``name`` with room for ``n`` floats. A buffer outgrown here is retired, not freed: captured graphs
        and the cached finaliser tables may still name it (the tables are dropped, to be rebuilt on the new one)."""
        buf = self._planes.get(name)
        if buf is None or buf.numel() < n:
            if buf is not None:
                self._retired.append(buf)
                self._retired.extend(self._fin_words.values())
                self._fin_words = {}
            buf = torch.zeros(n, dtype=torch.float32, device=self.dev)
            self._planes[name] = buf
        return buf

    def ppo_head(self, b: _Bufs, actions, logp_old, adv, ret, v_old, ent_coef, kl_coef, vf_coef, ppo_clip, v_clip,
                 stats, z_out=None, fc=None):
        """z = h Wh + bh, the clipped-surrogate (or A2C) + value loss, dz, dh and the head's weight / bias gradient
        planes in ONE launch (replaces the head GEMM, the loss launch, the dWh / dh GEMMs and the bias column sums).
        ``b.h`` must hold the fc activations (``forward(head=False)``); :meth:`backward` then starts at the fc layer
        (``head_done=True``) and its finaliser reduces the head planes. ``fc`` = (partial planes, count) of the fc
        product (``forward(head=False, fc_parts=True)`` at learner batch sizes): the head reduces them into h itself
        (``b.h`` is then not written)."""
        B, A1 = b.B, self.A1
        ops = _native.require()
        ph = self._ph.get(B)
        if ph is None:
            P = int(ops.ppo_head_planes(B))
            dev = self.dev
            ph = dict(P=P, Wh=torch.zeros(P * 512 * A1, device=dev), bh=torch.zeros(P * A1, device=dev),
                      bfc=torch.zeros(P * 512, device=dev), st=torch.zeros(P * 6, dtype=torch.float64, device=dev),
                      ticket=torch.zeros(1, dtype=torch.int32, device=dev))
            self._ph[B] = ph
        # the statistics records go to the finaliser that reduces this launch's planes (no last-arriver ticket in the
        # head: it cost every head workgroup an agent-scope release); det_wgrad: the planes always reach a finaliser
        defer = self.det_wgrad
        ops.ppo_head(b.h, self.sWh, self.bh, actions, logp_old, adv, ret, v_old if v_clip else None, ent_coef,
                     kl_coef, float(vf_coef), float(ppo_clip or 0.0), float(v_clip or 0.0), b.dh, z_out, ph["Wh"],
                     ph["bh"], ph["bfc"], ph["st"], None if defer else ph["ticket"], stats,
                     fc[0] if fc else None, fc[1] if fc else 0, self.bfc if fc else None)
        for name in ("Wh", "bh", "bfc"):
            self._planes["ph_" + name] = ph[name]
        self._head_planes = {"ph_Wh": ph["P"], "ph_bh": ph["P"], "ph_bfc": ph["P"]}
        if defer:
            self._stats_duty = (ph["st"].view(ph["P"], 6), B, ent_coef, kl_coef, stats)
        return stats

    # limits of loss.hip head_bwd_kernel: B rows staged in LDS (HB_MAXB), the bootstrap row of N values after them
    HB_MAXB, HB_MAXN = 512, 256

    def head_ok(self, B, N):
        """Gate of the fused A2C head (``head_bwd``): the same limits the kernel's launcher checks, so a config
        outside them takes the loss + GEMM path instead of failing at launch."""
        return (self.fused_head and 2 <= self.A <= 7 and 1 <= B <= self.HB_MAXB and 1 <= N <= self.HB_MAXN
                and B % N == 0)

    def head_env_ok(self, T, N, norm_adv):
        """The per-env A2C head (``a2c_head_env``) applies: no advantage normalisation (no batch-wide moments), at
        most 64 rollout steps."""
        return (self.a2c_head_env and self.a2c_head and not norm_adv and 1 <= T <= 64 and 2 <= self.A <= 7
                and self.grouped and self.fused_bwd and self.det_wgrad)   # the grouped backward's finaliser sums them

    def head_backward(self, b: _Bufs, actions, logp_old, ent_coef, kl_coef, vf_coef, stats, returns, boot=None,
                      planes_ok=False):
        """A2C fast path: ``a2c_head`` (or round 2's ``head_bwd``) -- returns/EV/adv-norm + loss + dz and the head's
        backward (dh, dWh, dbh, dbfc) in one launch; :meth:`backward` then starts at the fc layer (``head_done=True``).
        ``boot`` = (fc partial planes, count) of the bootstrap observation: V(s_T) is computed in the same launch and
        written into ``returns["val"][T]`` (the rollout then skips its ``fc_value`` launch)."""
        r = returns
        T, N = r["rew"].shape
        if planes_ok and self.head_env_ok(T, N, r["norm_adv"]):
            # the head's gradients stay per-env planes until THIS backward's finaliser (planes_ok: the caller runs the
            # whole backward with its finaliser before anything reads the fc/head gradients)
            ae = self._ae.get(N)
            if ae is None:
                dev, A1 = self.dev, self.A1
                ae = dict(Wh=torch.zeros(N * 512 * A1, device=dev), bfc=torch.zeros(N * 512, device=dev),
                          bh=torch.zeros(N * A1, device=dev), st=torch.zeros(N, 10, dtype=torch.float64, device=dev))
                self._ae[N] = ae
            hp, S = boot if boot is not None else (None, 0)
            _native.require().a2c_head_env(b.z, actions, logp_old, ent_coef, kl_coef, float(vf_coef), r["rew"],
                                           r["val"], r["dones"], int(r["L"]), int(r["mode"]), float(r["gamma"]),
                                           float(r["lam"]), r["ret_w"], r["adv_w"], b.h, self.sWh, b.dh, hp, int(S),
                                           self.bfc if hp is not None else None, self.bh if hp is not None else None,
                                           ae["Wh"], ae["bfc"], ae["bh"], ae["st"])
            for name in ("Wh", "bh", "bfc"):
                self._planes["ae_" + name] = ae[name]
            self._head_planes = {"ae_Wh": N, "ae_bh": N, "ae_bfc": N}
            self._stats_duty = (ae["st"], T * N, ent_coef, kl_coef, stats)
            return stats
        if self.a2c_head:
            if self._a2c_bar is None:
                self._a2c_bar = torch.zeros(4, dtype=torch.int32, device=self.dev)
            hp, S = boot if boot is not None else (None, 0)
            _native.require().a2c_head(b.z, actions, logp_old, ent_coef, kl_coef, float(vf_coef), r["rew"], r["val"],
                                       r["dones"], int(r["L"]), int(r["mode"]), bool(r["norm_adv"]), float(r["gamma"]),
                                       float(r["lam"]), r["ret_w"], r["adv_w"], b.h, self.sWh, b.dh, self.gWh,
                                       self.gbh, self.gbfc, stats, hp, int(S), self.bfc if hp is not None else None,
                                       self.bh if hp is not None else None, self._a2c_bar)
            return stats
        assert boot is None, "the bootstrap value is fused only into a2c_head"
        _native.require().head_bwd(b.z, actions, logp_old, ent_coef, kl_coef, float(vf_coef), r["rew"], r["val"],
                                   r["dones"], int(r["L"]), int(r["mode"]), bool(r["norm_adv"]), float(r["gamma"]),
                                   float(r["lam"]), r["ret_w"], r["adv_w"], b.h, self.sWh, b.dh, self.gWh, self.gbh,
                                   self.gbfc, stats)
        return stats

    def backward(self, b: _Bufs, head_bias_done=False, stage="all", head_done=False):
        """Accumulates d(loss)/d(params) into the gradient slab from ``b.dz`` (written by the loss kernel).

        Two streams: the activation-gradient chain (dh -> dy3 -> dy2 -> dy1) runs on the current stream while
        every weight-gradient product runs on a side stream as soon as its input gradient exists, so the
        critical path is the dX chain plus the last dW (captured as parallel branches of the hipGraph).

        ``stage``: ``"all"``; or ``"tail"`` (head + fc gradients, ending with both streams joined so the fc/head
        gradient bucket is final) followed later by ``"trunk"`` (conv gradients) -- data parallelism issues the
        all-reduce of :meth:`tail_bucket` between the two (overlapping the conv backward).
        """
        B, A1, ws = b.B, self.A1, self.ws
        ops = _native.require()
        main = torch.cuda.current_stream(self.dev)
        # serial_bwd: the weight-gradient products run on the compute stream too (large batches: the persistent
        # trunk backward holds every CU, and a side-stream product beside it only waits for LDS room)
        side = main if b.B >= self.large_b else self.side
        ev = self._ev
        ws2 = self._side_ws()
        grouped = self.grouped and (head_done or stage == "trunk") and self.fused_bwd and self.det_wgrad
        # every gradient element of this backward is STORED (fused head, dWfc out_mode 0, conv planes and bias rows
        # through the finaliser): the optimiser may skip zeroing the slab (trainer._run_optimizers). A "tail" stage
        # decides it for the "trunk" stage that completes the same backward.
        if stage != "trunk":
            self.last_bwd_stores_all = grouped and head_done and stage in ("all", "tail")
        if stage == "trunk":
            if grouped:
                return self._backward_grouped(b, stage, ws, ws2)
            return self._backward_trunk(b, main, side, ev, ws, ws2)
        # weight-gradient plane sets written by THIS backward (reduced by its finaliser), plus the head's planes when
        # ppo_head ran just before it; whether dWfc's norm comes as fc_bwd's presummed partials
        self._cur_planes, self._head_planes = dict(self._head_planes) if head_done else {}, {}
        self._cur_presum = False
        if grouped:
            return self._backward_grouped(b, stage, ws, ws2)
        head_bias_done = head_bias_done or getattr(b, "bias_done", False)
        if not head_done:
            ev[0].record(main)
            side.wait_event(ev[0])
            with torch.cuda.stream(side):   # heads: dWh = h^T dz, dbh = colsum(dz)
                if self.det_wgrad and stage == "all":   # split-K planes, reduced in order by the finaliser
                    self._wgrad("Wh", self.gWh, b.h, 512, b.dz, A1, 512, A1, B, ws2, None)
                else:
                    G.gemm(b.h, 512, False, b.dz, A1, False, self.gWh, A1, 2, 512, A1, B, workspace=ws2)
                if not head_bias_done:
                    ops.colsum_bf16(b.dz, B, A1, A1, self.gbh)
            G.gemm(b.dz, A1, True, self.sWh, A1, True, b.dh, 512, 1, B, 512, A1, mask=b.h, ldm=512,
                   colsum=self.gbfc, workspace=ws)
        ev[1].record(main)
        side.wait_event(ev[1])
        with torch.cuda.stream(side):   # fc weight gradient (det_wgrad: store; split-K slabs reduced in order)
            G.gemm(b.y3, 3136, False, b.dh, 512, False, self.gWfc, 512, 0 if self.det_wgrad else 2, 3136, 512, B,
                   workspace=ws2)
        G.gemm(b.dh, 512, True, self.sWfc, 512, True, b.dy3, 3136, 1, B, 3136, 512, mask=b.y3, ldm=3136,
               colsum=None if self.fused_bwd else self.gb3, colsum_mod=0 if self.fused_bwd else 64, workspace=ws)
        if stage == "tail":
            ev[5].record(side)
            main.wait_event(ev[5])
            return
        return self._backward_trunk(b, main, side, ev, ws, ws2)

    def fc_bwd_ok(self, B):
        """The learner's fc backward of a ``B``-row batch runs as the dedicated two-product launch (``fc_bwd.hip``,
        ``EngineOpts.fc_bwd``: at most 256 rows)."""
        return self.opts.fc_bwd and self.dev.type == "cuda" and 1 <= B <= 256

    def big_gemm_ok(self, B):
        """The fc products of a ``B``-row learner batch run on gemm_big.hip (large tiles, LDS-DMA ring)."""
        return self.big_ws is not None and 0 < self.large_b <= B and B % 64 == 0

    def _backward_grouped(self, b, stage, ws, ws2):
        """One stream, no cross-stream edges: the independent products of each stage run as ONE grouped launch
        (ops.gemm.group) -- {dWfc, dy3}, then the fused dy3 -> dy2 -> dy1 kernel, then {dW3, dW2, dW1} as split-K
        planes, then the finaliser. Inside a captured graph every event edge between streams costs several
        microseconds of inter-queue synchronisation; here the critical path is the chain of launches itself."""
        B = b.B
        if stage in ("all", "tail") and self.big_gemm_ok(B):
            # dy3 = (dh Wfc^T) * (y3 > 0) [B, 3136] (K 512: no split), dWfc = y3^T dh [3136, 512] (K = B: 2 splits;
            # whole backward: as two partial planes the finaliser reduces, else stored through the split-K slabs so
            # the fc/head bucket is final at the end of the "tail" stage)
            G.gemm_big(b.dh, 512, True, self.sWfc, 512, True, b.dy3, 3136, 1, B, 3136, 512, mask=b.y3, ldm=3136,
                       workspace=self.big_ws)
            if stage == "all" and self.det_wgrad:
                buf = self._big_planes("Wfc", 2 * 3136 * 512)
                G.gemm_big(b.y3, 3136, False, b.dh, 512, False, buf, 512, 3, 3136, 512, B, splits=2)
                self._cur_planes["Wfc"] = 2
            elif stage == "tail" and self.det_wgrad:
                # data parallelism: the same two planes, summed into the slab by a finaliser launch of the fc weight
                # alone (the bucket must be final before its all-reduce): cheaper than the in-launch split reduction
                buf = self._big_planes("Wfc", 2 * 3136 * 512)
                G.gemm_big(b.y3, 3136, False, b.dh, 512, False, buf, 512, 3, 3136, 512, B, splits=2)
                self.finalize(b, planes={"Wfc": 2}, parts=False, bias_rows=False)
            else:
                G.gemm_big(b.y3, 3136, False, b.dh, 512, False, self.gWfc, 512, 0, 3136, 512, B, splits=2,
                           workspace=self.big_ws)
            if stage == "tail":
                return
        elif stage in ("all", "tail") and self.fc_bwd_ok(B):
            # both fc products in one launch of two job kinds (fc_bwd.hip): dWfc tiles staged in LDS, dy3 tiles
            # from whole-line row loads; with the finaliser's norm partials wanted, the dWfc tiles also leave their
            # sums of squares (the finaliser adds those instead of re-reading the 6.4 MB gradient)
            sq = None
            if self.want_parts and stage == "all":
                if self._fcb_sq is None:
                    self._fcb_sq = torch.zeros(392 * 4, dtype=torch.float32, device=self.dev)
                sq = self._fcb_sq
                self._cur_presum = True
            _native.require().fc_bwd(b.dh, self.sWfc, b.y3, b.dy3, self.gWfc, None, sq)
            if stage == "tail":
                return
        elif stage in ("all", "tail"):
            with G.group():   # workgroups start in product order: the critical-path product first
                G.gemm(b.dh, 512, True, self.sWfc, 512, True, b.dy3, 3136, 1, B, 3136, 512, mask=b.y3, ldm=3136,
                       workspace=ws)
                G.gemm(b.y3, 3136, False, b.dh, 512, False, self.gWfc, 512, 0, 3136, 512, B, workspace=ws2)
            if stage == "tail":
                return
        folded = self._trunk_bwd(b, fold=True)
        with G.group():   # the longest product (conv1, K = 400 B) first
            if not folded:
                self._wgrad_conv1(b, ws)
            self._wgrad_conv23("W2", b, ws2)
            self._wgrad_conv23("W3", b, ws2)
        self.finalize(b)

    def _backward_trunk(self, b, main, side, ev, ws, ws2):
        B = b.B
        imp = self.implicit
        ev[2].record(main)
        side.wait_event(ev[2])
        with torch.cuda.stream(side):   # conv3 weight gradient
            if imp:
                self._wgrad_conv23("W3", b, ws2)
            else:
                G.gemm(b.dy3, 64, False, b.col3, 576, False, self.gW3, 576, 2, 64, 576, B * 49, workspace=ws2)
        if self.fused_bwd:
            # dy2 = tconv(dy3, W3) * (y2 > 0) and dy1 = tconv(dy2, W2) * (y1 > 0) in one per-sample launch; the
            # bias-gradient partial rows (db3 | db2 | db1) are reduced by the finaliser
            self._trunk_bwd(b)
        elif self.tconv_dgrad:   # dy2 = conv_transpose(dy3, W3) * (y2 > 0) as one gathered GEMM (+ colsum -> db2)
            G.gemm(b.dy3, 0, True, self.sW3, 0, False, b.dy2, 64, 1, B * 81, 64, 576, mask=b.y2, ldm=64,
                   colsum=self.gb2, workspace=ws, ga=[3, B, 64, 9, 9, 3, 3, 1], gb=[4, 1, 64, 1, 64, 3, 3, 1])
        else:
            G.gemm(b.dy3, 64, True, self.sW3, 576, False, self.dcol3(b), 576, 1, B * 49, 576, 64, workspace=ws)
            G.col2im_nhwc(self.dcol3(b), b.y2, b.dy2, self.gb2, B, 9, 9, 64, 3, 3, 1)
        ev[3].record(main)
        side.wait_event(ev[3])
        with torch.cuda.stream(side):   # conv2 weight gradient
            if imp:
                self._wgrad_conv23("W2", b, ws2)
            else:
                G.gemm(b.dy2, 64, False, b.col2, 512, False, self.gW2, 512, 2, 64, 512, B * 81, workspace=ws2)
        if self.fused_bwd:
            pass
        elif self.tconv_dgrad:   # dy1 = conv_transpose(dy2, W2) * (y1 > 0) (+ colsum -> db1)
            # stride 2: sub-pixel form -- rows grouped by stride phase, only the 2x2 taps on each phase's grid
            G.gemm(b.dy2, 0, True, self.sW2, 0, False, b.dy1, 32, 1, B * 400, 32, 256, mask=b.y1, ldm=32,
                   colsum=self.gb1, workspace=ws, ga=[5, B, 64, 20, 20, 4, 4, 2], gb=[6, 1, 64, 1, 32, 4, 4, 2])
        else:
            G.gemm(b.dy2, 64, True, self.sW2, 512, False, self.dcol2(b), 512, 1, B * 81, 512, 64, workspace=ws)
            G.col2im_nhwc(self.dcol2(b), b.y1, b.dy1, self.gb1, B, 20, 20, 32, 4, 4, 2)
        # conv1 weight gradient (last product of the chain: on the main stream)
        if imp:
            self._wgrad_conv1(b, ws)
        else:
            G.gemm(b.dy1, 32, False, b.col1, 256, False, self.gW1, 256, 2, 32, 256, B * 400, workspace=ws)
        ev[4].record(side)
        main.wait_event(ev[4])
        if self.fused_bwd or self.want_parts or self.det_wgrad:
            self.finalize(b)

    # ------------------------------------------------------------------------------------------------ finaliser
    want_parts = False   # set by the trainer when the optimiser may take the finaliser's sum-of-squares partials

    def finalize(self, b: _Bufs, planes=None, parts=None, bias_rows=True):
        """One launch after the backward (``grad_finalize``): reduces the per-sample conv bias-gradient rows
        (fused backward) into the slab and, with ``want_parts``, writes the global-norm partials of the whole
        gradient (``fin_parts``) so the optimiser needs no sum-of-squares pass. ``planes``: only these plane sets
        (default: every set of this backward); ``parts`` / ``bias_rows`` False: no norm partials / no bias rows."""
        words = self._fin_table(b, planes, parts, bias_rows)
        # the per-env head's statistics go with the finaliser that sums its gradient planes (not whichever finaliser
        # runs first: under DP a tail-stage launch sums the fc weight alone)
        cur = self._cur_planes if planes is None else planes
        sums_head = "ae_Wh" in cur or "ph_Wh" in cur
        sd = self._stats_duty if sums_head else None
        if sd is not None:
            self._stats_duty = None
        if sd is not None:   # the per-env head's statistics rows -> stats[0..7] (one extra finaliser workgroup)
            spart, B, ent, kl, stats = sd
            _native.require().grad_finalize(words[0], self.fin_parts, spart, B, ent, kl, stats)
        else:
            _native.require().grad_finalize(words[0], self.fin_parts)

    def _fin_table(self, b: _Bufs, planes=None, parts=None, bias_rows=True):
        """The finaliser's device job table for these plane sets (built once per key, outside graph capture: the
        head launches pre-build their tail-stage tables on first use)."""
        want_parts = self.want_parts if parts is None else parts
        fused_rows = self.fused_bwd and bias_rows
        planes = tuple(sorted((self._cur_planes if planes is None else planes).items())) if self.det_wgrad else ()
        presum = want_parts and self._cur_presum and self._fcb_sq is not None
        key = (b.B, want_parts, fused_rows, planes, presum, self._gslab.data_ptr())
        words = self._fin_words.get(key)
        if words is None:
            segs = []
            flat = self.flat
            src_of = {}   # gradient slot -> (source, stride, planes)
            if fused_rows:
                bp, R = b.biasp.data_ptr(), self.bias_rows(b.B)
                src_of = {self.gb3.data_ptr(): (bp, 160, R), self.gb2.data_ptr(): (bp + 64 * 4, 160, R),
                          self.gb1.data_ptr(): (bp + 128 * 4, 160, R)}
            for name, S in planes:
                g = {"W1": self.gW1, "W1f": self.gW1, "W2": self.gW2, "W3": self.gW3, "Wh": self.gWh,
                     "ph_Wh": self.gWh, "ph_bh": self.gbh, "ph_bfc": self.gbfc, "Wfc": self.gWfc, "ae_Wh": self.gWh,
                     "ae_bh": self.gbh, "ae_bfc": self.gbfc}[name]
                src_of[g.data_ptr()] = (self._planes[name].data_ptr(), g.numel(), S)
            for p, off in zip(flat.params, flat.offsets):
                g = self._gslab[off:off + p.numel()]
                src = src_of.get(g.data_ptr())
                if src is not None:
                    segs.append((g.data_ptr(), src[0], g.numel(), src[1], src[2]))
                elif presum and g.data_ptr() == self.gWfc.data_ptr():
                    segs.append((self._fcb_sq.data_ptr(), 0, self._fcb_sq.numel(), 0, -1))
                elif want_parts:
                    segs.append((g.data_ptr(), 0, g.numel(), 0, 0))
            from ..ops.optim import finalize_jobs
            words = finalize_jobs(segs, self.dev, return_max=True, split_planes=True)
            self._fin_words[key] = words
        return words

    @staticmethod
    def dcol3(b):   # only the col2im data-gradient path materialises the column gradients
        if not hasattr(b, "dcol3"):
            b.dcol3 = torch.empty(b.B * 49, 576, dtype=torch.bfloat16, device=b.dy3.device)
        return b.dcol3

    @staticmethod
    def dcol2(b):
        if not hasattr(b, "dcol2"):
            b.dcol2 = torch.empty(b.B * 81, 512, dtype=torch.bfloat16, device=b.dy2.device)
        return b.dcol2

    def _side_ws(self):
        if not hasattr(self, "_ws2"):
            self._ws2 = G.GemmWorkspace(self.dev)
        return self._ws2

    # ------------------------------------------------------------------------------------------------ loss
    def loss(self, b: _Bufs, actions, logp_old, adv, ret, v_old, ent_coef, kl_coef, vf_coef, ppo_clip, v_clip,
             stats=None, returns=None):
        """Fused loss + head gradient -> ``b.dz``; statistics [pg, kl, ent, vloss, clipfrac, actor loss, ratio, ev].

        ``returns`` (A2C fast path): dict(mode=1|2, rew, val, dones, L, gamma, lam, norm_adv, ret_w, adv_w) --
        targets/advantages, EV-before and advantage normalisation are computed inside the same launch, and the
        head-bias gradient is written by it too (the backward then skips its column-sum)."""
        B, A, A1 = b.B, self.A, self.A1
        zl = b.z
        out = b.stats if stats is None else stats
        ops = _native.require()
        if returns is None:
            # det_wgrad: the loss kernel also writes the head-bias gradient (fixed-order sums), so the backward needs
            # no atomic column sum
            ops.ac_loss(zl, A1, zl[:, A:], A1, actions, None, None, logp_old, adv, ret, v_old, ent_coef, kl_coef,
                        float(vf_coef), float(ppo_clip or 0.0), float(v_clip or 0.0), b.dz, A1, b.dz[:, A:], A1,
                        None, out, B, A, False, dbias=self.gbh if self.det_wgrad else None)
            b.bias_done = self.det_wgrad
        else:
            r = returns
            ops.ac_loss(zl, A1, zl[:, A:], A1, actions, None, None, logp_old, None, None, None, ent_coef, kl_coef,
                        float(vf_coef), 0.0, 0.0, b.dz, A1, b.dz[:, A:], A1, None, out, B, A, False, r["mode"],
                        r["rew"], r["val"], r["dones"], int(r["L"]), float(r["gamma"]), float(r["lam"]),
                        bool(r["norm_adv"]), r["ret_w"], r["adv_w"], self.gbh)
        return out
