"""bf16 MFMA GEMM + convolution lowering ops (``csrc/kernels/gemm.hip``, ``conv.hip``).

``gemm`` computes ``C = epilogue(alpha * A @ B)`` for strided bf16 operands stored either way round (see the
kernel header) and is the only matrix product the native engine uses -- forward, dX and dW of every conv / dense
layer. :func:`plan` picks the tile and the split-K factor from the problem shape so that small-batch products
(rollout inference at 32 rows) still put >= one workgroup on most of the 256 CUs.

Each function has a PyTorch reference (``*_ref``) that the GPU tests compare against in fp32.
"""
from __future__ import annotations

import os

import torch

from .. import _native

# tile id -> (BM, BN) ; must match aca_gemm_tile_dims
TILES = {0: (64, 64), 1: (32, 64), 2: (64, 32), 3: (128, 64), 4: (32, 32), 5: (64, 256), 6: (32, 256),
         7: (128, 128)}
# supported k-step depths per tile (aca_gemm_supported): deeper k-steps for the small tiles of latency-bound products;
# the wide tiles (5, 6: skinny-M weight gradients over huge K, the operand that every N tile re-reads is read 4-8x
# less; 7: large-batch products) only with 64-deep k-steps (LDS)
BKS = {0: (64, 128), 1: (64, 128), 2: (64, 128), 3: (64,), 4: (64, 128, 256), 5: (64,), 6: (64,), 7: (64,)}
NUM_CUS = 256


def _cdiv(a, b):
    return (a + b - 1) // b


def effective_splits(K, bk, splits):
    kt = _cdiv(K, bk)
    splits = max(1, min(splits, kt if kt > 0 else 1))
    per = _cdiv(kt, splits) if kt > 0 else 0
    return _cdiv(kt, per) if kt > 0 else 1


def plan(M, N, K, atomic=False, max_splits=64, target_wgs=256):
    """Static ``(tile, bk, splits)`` heuristic (used when autotuning is off or during graph capture).

    Prefer the largest tile that still yields ``target_wgs`` workgroups; when even the smallest tile leaves the
    chip mostly idle, split K (each split keeps >= 2 k-steps). ``atomic`` products (weight gradients) may split
    deeper because their reduction costs nothing extra.
    """
    best = None
    for tile in (3, 0, 2, 1, 4):
        bm, bn = TILES[tile]
        if bm > 64 and M < 4 * bm:
            continue
        wgs = _cdiv(M, bm) * _cdiv(N, bn)
        if wgs >= target_wgs:
            return tile, 64, 1
        if best is None or wgs > best[1]:
            best = (tile, wgs)
    tile, wgs = best
    kt = _cdiv(K, 64)
    splits = 1
    cap = max_splits if atomic else 16
    while wgs * splits * 2 <= 2 * target_wgs and kt // (splits * 2) >= 2 and splits * 2 <= cap:
        splits *= 2
    return tile, 64, splits


def workspace_elems(M, N, tile, splits):
    bm, bn = TILES[tile]
    return _cdiv(M, bm) * _cdiv(N, bn) * splits * bm * bn, _cdiv(M, bm) * _cdiv(N, bn)


class GemmWorkspace:
    """Slab + ticket workspace shared by the split-K products of one engine (sized on first use, then static)."""

    def __init__(self, device, elems=1 << 20, tickets=1 << 14):
        self.ws = torch.zeros(elems, dtype=torch.float32, device=device)
        self.tickets = torch.zeros(tickets, dtype=torch.int32, device=device)
        self.part = torch.zeros(1 << 16, dtype=torch.float32, device=device)

    def part_buf(self, elems):
        """Per-row-tile column-sum partials (fully rewritten by every GEMM that uses them)."""
        if elems > self.part.numel():
            self.part = torch.zeros(elems, dtype=torch.float32, device=self.part.device)
        return self.part

    def ensure(self, elems, tiles):
        if elems > self.ws.numel():
            self.ws = torch.zeros(elems, dtype=torch.float32, device=self.ws.device)
        if tiles > self.tickets.numel():
            self.tickets = torch.zeros(tiles, dtype=torch.int32, device=self.ws.device)


# ------------------------------------------------------------------------------------------------ autotuning
# The engine issues ~20 distinct GEMM shapes, all small and latency-bound (32..64k rows); the fastest
# (tile, k-step depth, split-K) triple depends on how many workgroups a shape yields against 256 CUs and how many
# k-steps each serial chain has to walk. Each new shape is timed once on its first (eager, never captured) call
# against scratch outputs and the winner is cached for the process. ACAMD_GEMM_TUNE=0 uses :func:`plan`.
_TUNED: dict = {}
PARTIAL_MAX_SPLITS = 8   # out_mode 3: the consumer kernels reduce at most this many partial planes
# with >= 2 row tiles the bias column sums go through per-tile partials + one ordered reduce (deterministic; one
# tile row adds each column once, also deterministic)
COLSUM_PART_MIN_TILES = 2
TUNE = os.environ.get("ACAMD_GEMM_TUNE", "1") == "1"


def tuned_plans():
    return dict(_TUNED)


# Tuned plans measured on an MI355X for the engine's shapes (scripts/dump_gemm_plans.py): loaded at import so runs
# start with the measured winners (no tuning pass, and no run-to-run plan noise); shapes not in the file are still
# tuned on first use. ACAMD_GEMM_PLANS=0 ignores the file; ACAMD_GEMM_PLANS=<path> loads another plans file.
PLANS_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_plans.json")
if os.environ.get("ACAMD_GEMM_PLANS", "1") not in ("0", "1", ""):
    PLANS_FILE = os.environ["ACAMD_GEMM_PLANS"]


def _key_from_json(k):
    return tuple(tuple(x) if isinstance(x, list) else x for x in k)


def load_plans(path=PLANS_FILE):
    import json
    if not os.path.exists(path) or os.environ.get("ACAMD_GEMM_PLANS", "1") == "0":
        return 0
    with open(path) as f:
        rows = json.load(f)
    for r in rows:
        _TUNED.setdefault(_key_from_json(r["key"]), tuple(r["plan"]))
    return len(rows)


def save_plans(path=PLANS_FILE):
    import json
    rows = [{"key": [list(x) if isinstance(x, tuple) else x for x in k], "plan": list(v)}
            for k, v in sorted(_TUNED.items(), key=lambda kv: str(kv[0]))]
    with open(path, "w") as f:
        json.dump(rows, f, indent=0)
    return len(rows)


load_plans()


def _candidates(M, N, K, atomic, max_splits=None, row_block=None):
    for tile, (bm, bn) in TILES.items():
        if row_block is not None and row_block % bm:
            continue  # sub-pixel gathers: a tile must not straddle two stride phases
        if bm >= 2 * max(32, M) or bn >= 2 * max(32, N):
            continue  # a tile at least twice the problem in one dimension only wastes MFMA issue
        for bk in BKS[tile]:
            kt = _cdiv(K, bk)
            if bk > 64 and kt < 1:
                continue
            for s in (1, 2, 4, 8, 16, 32, 64):
                if s > 1 and kt < 2 * s:
                    break
                if not atomic and s > 16:
                    break
                if max_splits is not None and s > max_splits:
                    break
                yield tile, bk, s


def _run(ops, A, lda, a_k, B, ldb, b_k, C, ldc, out_mode, M, N, K, alpha, bias, relu, mask, ldm, colsum,
         colsum_mod, tile, bk, splits, workspace, ga, ga_scale, gb, gb_scale, stamps=None):
    eff = effective_splits(K, bk, splits)
    ws = tk = None
    if eff > 1 and out_mode < 2:
        if workspace is None:
            raise ValueError("slab split-K needs a GemmWorkspace")
        e, t = workspace_elems(M, N, tile, eff)
        workspace.ensure(e, t)
        ws, tk = workspace.ws, workspace.tickets
    # bias column sums of products with many row tiles: per-tile partials + one reduce launch instead of every
    # workgroup adding into the same few addresses (thousands of same-address atomics serialise in L2)
    part, R = None, 0
    if colsum is not None and eff == 1 and out_mode != 3 and workspace is not None:
        R = (M + TILES[tile][0] - 1) // TILES[tile][0]
        if R >= COLSUM_PART_MIN_TILES:
            if _GROUP_DEPTH:
                raise ValueError("gemm group: products with column-sum partials cannot be grouped")
            part = workspace.part_buf(R * N)
    ops.gemm(A, lda, a_k, B, ldb, b_k, C, ldc, out_mode, M, N, K, float(alpha), bias, bool(relu), mask, ldm,
             colsum, int(colsum_mod), tile, bk, splits, ws, tk, list(ga or []), float(ga_scale), list(gb or []),
             float(gb_scale), stamps, part)
    if part is not None:
        ops.colsum_reduce(part, R, N, colsum, int(colsum_mod))
    return eff


_GROUP_DEPTH = 0
GROUP_STATS = {"grouped": 0, "fallback": 0}


class group:
    """Context manager: the :func:`gemm` calls inside (independent products, one stream) run as ONE grouped
    launch when an instantiation covers their tile configurations (csrc/kernels/gemm_group.hip), else one launch
    each in issue order. Products in a group must not use the column-sum partial path (its reduce launch would
    run before the group) -- the learner's grouped products have no column sums."""

    def __enter__(self):
        global _GROUP_DEPTH
        assert _GROUP_DEPTH == 0, "gemm groups do not nest"
        _native.require().gemm_group_begin()
        _GROUP_DEPTH = 1
        return self

    def __exit__(self, exc_type, exc, tb):
        global _GROUP_DEPTH
        _GROUP_DEPTH = 0
        ran = _native.require().gemm_group_end() if exc_type is None else _abort_group()
        GROUP_STATS["grouped" if ran else "fallback"] += 1
        return False


def _abort_group():
    try:
        _native.require().gemm_group_end()
    except Exception:   # pragma: no cover - already failing
        pass
    return 0


def _row_block(ga):
    """Rows per stride phase of a sub-pixel (mode 5) gather, else None."""
    if ga and ga[0] == 5:
        return ga[1] * (ga[3] // ga[7]) * (ga[4] // ga[7])
    return None


def _tune(key, ops, A, lda, a_k, B, ldb, b_k, C, ldc, out_mode, M, N, K, alpha, bias, relu, mask, ldm, colsum,
          colsum_mod, workspace, ga, ga_scale, gb, gb_scale, max_planes=PARTIAL_MAX_SPLITS):
    dev = C.device
    planes = max_planes if out_mode == 3 else 1
    Cs = torch.zeros(planes * M * ldc, dtype=C.dtype, device=dev)
    cs = torch.zeros(max(N, colsum_mod or 0), dtype=torch.float32, device=dev) if colsum is not None else None
    ws = workspace if workspace is not None else GemmWorkspace(dev)
    best = None
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for tile, bk, s in _candidates(M, N, K, out_mode in (2, 3), max_planes if out_mode == 3 else None,
                                   _row_block(ga)):
        args = (ops, A, lda, a_k, B, ldb, b_k, Cs, ldc, out_mode, M, N, K, alpha, bias, relu, mask, ldm, cs,
                colsum_mod, tile, bk, s, ws, ga, ga_scale, gb, gb_scale)
        _run(*args)
        ms = float("inf")
        for _trial in range(3):   # min over trials: robust to clock ramps and co-running noise
            ev0.record()
            for _ in range(8):
                _run(*args)
            ev1.record()
            ev1.synchronize()
            ms = min(ms, ev0.elapsed_time(ev1) / 8)
        if best is None or ms < best[0]:
            best = (ms, tile, bk, s)
    _TUNED[key] = (best[1], best[2], best[3], best[0])
    return best[1], best[2], best[3]


def gemm(A, lda, a_k, B, ldb, b_k, C, ldc, out_mode, M, N, K, alpha=1.0, bias=None, relu=False, mask=None, ldm=0,
         colsum=None, tile=None, splits=None, workspace: GemmWorkspace | None = None, colsum_mod=0, bk=None,
         ga=None, ga_scale=1.0, gb=None, gb_scale=1.0, stamps=None, max_planes=PARTIAL_MAX_SPLITS):
    """Native GEMM; ``out_mode``: 0 fp32 store, 1 bf16 store, 2 fp32 atomic add (C pre-zeroed), 3 fp32 split-K
    partial planes ``C[z, M, ldc]`` (no bias/activation: the consumer reduces, in plane order -- deterministic;
    ``max_planes`` bounds the split count, C must hold that many planes). Returns the effective split count.

    ``ga`` / ``gb``: implicit-im2col gathers ``[mode, B, C, H, W, KH, KW, S]`` (mode 1 uint8 NCHW, 2 bf16 NHWC)
    reading operand A (k-contiguous) / B (n-contiguous) straight from the activation image ``A`` / ``B``.
    """
    ops = _native.require()
    if tile is None or splits is None or bk is None:
        key = (M, N, K, bool(a_k), bool(b_k), out_mode, lda % 8 == 0, ldb % 8 == 0, tuple(ga or ()), tuple(gb or ()),
               max_planes if out_mode == 3 else 0)
        hit = _TUNED.get(key)
        if hit is not None:
            t, k, s = hit[0], hit[1], hit[2]
        elif TUNE and C.is_cuda and not torch.cuda.is_current_stream_capturing():
            if _GROUP_DEPTH:
                ops.gemm_group_pause(True)   # trials launch directly, not into the open group
            try:
                t, k, s = _tune(key, ops, A, lda, a_k, B, ldb, b_k, C, ldc, out_mode, M, N, K, alpha, bias, relu,
                                mask, ldm, colsum, colsum_mod, workspace, ga, ga_scale, gb, gb_scale, max_planes)
            finally:
                if _GROUP_DEPTH:
                    ops.gemm_group_pause(False)
        else:
            t, k, s = plan(M, N, K, atomic=(out_mode in (2, 3)))
            if out_mode == 3:
                s = min(s, max_planes)
            rb = _row_block(ga)
            if rb is not None and rb % TILES[t][0]:
                t = next(tt for tt in (2, 0, 4, 1) if rb % TILES[tt][0] == 0)
        tile = t if tile is None else tile
        bk = k if bk is None else bk
        splits = s if splits is None else splits
    if colsum_mod and colsum is None:
        raise ValueError("colsum_mod without colsum")
    if out_mode == 3 and effective_splits(K, bk, splits) > max_planes:
        raise ValueError("out_mode 3: more split-K planes than C holds (%d)" % max_planes)
    return _run(ops, A, lda, a_k, B, ldb, b_k, C, ldc, out_mode, M, N, K, alpha, bias, relu, mask, ldm, colsum,
                colsum_mod, tile, bk, splits, workspace, ga, ga_scale, gb, gb_scale, stamps)


# gemm_big launch variant: bit 0 XCD-grouped workgroup order, bits 1-2 LDS ring depth - 2 (2: 64 KB LDS, two
# workgroups per CU -- measured fastest on all three fc products), bit 3 scalar bf16 epilogue
GEMM_BIG_VARIANT = 1


class GemmBigWorkspace:
    """Split-K slabs + self-cleaning tickets of :func:`gemm_big` (grown outside graph capture, shared by the
    stream-ordered launches of one engine)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.ws = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.tickets = torch.zeros(1, dtype=torch.int32, device=self.device)

    def fit(self, M, N, splits):
        need = int(_native.require().gemm_big_ws(M, N, splits))
        if self.ws.numel() < need:
            self.ws = torch.zeros(need, dtype=torch.float32, device=self.device)
        tiles = -(-M // 128) * -(-N // 128)
        if self.tickets.numel() < tiles:
            self.tickets = torch.zeros(tiles, dtype=torch.int32, device=self.device)
        return self


def gemm_big(A, lda, a_k, B, ldb, b_k, C, ldc, out_mode, M, N, K, alpha=1.0, bias=None, relu=False, mask=None,
             ldm=0, splits=1, workspace=None, variant=GEMM_BIG_VARIANT, stamps=None):
    """Large plain bf16 product on the 128 x 128 / 32x32x16-MFMA kernel with LDS-DMA staging (``gemm_big.hip``):
    out_mode 0 fp32 / 1 bf16 store, bias / relu / mask epilogue, slab split-K (deterministic); out_mode 3: the
    ``splits`` fp32 partial planes ``C[z, M, ldc]`` for a consumer that reduces them (no epilogue). K % 64 == 0."""
    ws = workspace.fit(M, N, splits) if splits > 1 and out_mode != 3 else None
    _native.require().gemm_big(A, lda, a_k, B, ldb, b_k, C, ldc, out_mode, M, N, K, float(alpha), bias, bool(relu),
                               mask, ldm, splits, ws.ws if ws else None, ws.tickets if ws else None, stamps,
                               int(variant))


def _view(t, rows, cols, ld, k_contig_rows):
    """Strided [rows, cols] view of a flat tensor with row stride ld (contiguous columns)."""
    return torch.as_strided(t, (rows, cols), (ld, 1), t.storage_offset())


def gemm_ref(A, lda, a_k, B, ldb, b_k, M, N, K, alpha=1.0, bias=None, relu=False, mask=None, ldm=0):
    """fp32 PyTorch oracle of :func:`gemm` (returns the fp32 result; no store/colsum semantics)."""
    Am = _view(A, M, K, lda, True) if a_k else _view(A, K, M, lda, False).t()
    Bm = _view(B, N, K, ldb, True).t() if b_k else _view(B, K, N, ldb, False)
    y = alpha * (Am.float() @ Bm.float())
    if bias is not None:
        y = y + bias[:N].float()
    if relu:
        y = torch.relu(y)
    if mask is not None:
        y = y * (_view(mask, M, N, ldm, True).float() > 0)
    return y


# ------------------------------------------------------------------------------------------------ conv lowering
def conv_out(h, k, s):
    return (h - k) // s + 1


def im2col_u8(x, col, kh, kw, s, scale=1.0 / 255.0):
    _native.require().im2col_u8(x, col, kh, kw, s, float(scale))


def im2col_u8_ref(x, kh, kw, s, scale=1.0 / 255.0):
    """uint8 NCHW -> [B*OH*OW, C*KH*KW] with k order (c, i, j)."""
    B, C, H, W = x.shape
    u = torch.nn.functional.unfold(x.float() * scale, (kh, kw), stride=s)  # [B, C*kh*kw, L]
    return u.transpose(1, 2).reshape(-1, C * kh * kw)


def im2col_nhwc(x, col, B, H, W, C, kh, kw, s):
    _native.require().im2col_nhwc(x, col, B, H, W, C, kh, kw, s)


def im2col_nhwc_ref(x, B, H, W, C, kh, kw, s):
    """NHWC [B, H, W, C] -> [B*OH*OW, KH*KW*C] with k order (i, j, c)."""
    xn = x.reshape(B, H, W, C).permute(0, 3, 1, 2).float()
    u = torch.nn.functional.unfold(xn, (kh, kw), stride=s)  # [B, C*kh*kw, L], k order (c, i, j)
    L = u.shape[-1]
    u = u.view(B, C, kh * kw, L).permute(0, 3, 2, 1)      # [B, L, kh*kw, C]
    return u.reshape(B * L, kh * kw * C)


def cnn_trunk_fwd(obs, W1, b1, W2, b2, W3, b3, y1, y2, y3, scale=1.0 / 255.0, shift_out=None, mode=1,
                  copy_out=None, obs_idx=None):
    """Fused Nature-CNN conv1..conv3, activations through LDS (``cnn_fused.hip``). ``mode`` 1: seven workgroups per
    env, one per conv3 output row (its receptive field recomputed), 2: the same with the conv2 / conv3 weight loads
    after conv1; 3: one workgroup per env with the frame converted to bf16 once; 5: mode 3 reading fragment-ordered
    W1..W3 (``ops.optim.frag_order``), 6 / 7: modes 1 / 2 reading fragment-ordered W2 / W3.
    ``shift_out``: also write frames 1..3 of every observation as frames 0..2 of this buffer (frame-stack shift);
    ``copy_out`` (mode 1): also copy the whole observation there. ``obs_idx`` (int64 [B], modes 3 / 5): sample b is row
    ``obs_idx[b]`` of ``obs`` (a PPO minibatch gathered by index)."""
    _native.require().cnn_trunk_fwd(obs, W1, b1, W2, b2, W3, b3, y1, y2, y3, float(scale), shift_out, None,
                                    int(mode), copy_out, obs_idx)


def col2im_nhwc(dcol, ymask, dx, colsum, B, H, W, C, kh, kw, s):
    _native.require().col2im_nhwc(dcol, ymask, dx, colsum, B, H, W, C, kh, kw, s)


def col2im_nhwc_ref(dcol, ymask, B, H, W, C, kh, kw, s):
    OH, OW = conv_out(H, kh, s), conv_out(W, kw, s)
    d = dcol.float().view(B, OH * OW, kh * kw, C).permute(0, 3, 2, 1).reshape(B, C * kh * kw, OH * OW)
    x = torch.nn.functional.fold(d, (H, W), (kh, kw), stride=s)  # [B, C, H, W]
    x = x.permute(0, 2, 3, 1).reshape(B * H * W, C)
    return x * (ymask.float().view(B * H * W, C) > 0)
