// bf16 MFMA GEMM with fused epilogues and implicit-im2col operand gathers -- the workhorse behind every dense and
// conv forward / backward product of the engine.
//
//   C[M, N] = epilogue( alpha * A[M, K] . B[K, N] )
//
// Operands are bf16 (or gathered from uint8 / bf16 images, see gemm_desc.h), accumulation fp32 on
// v_mfma_f32_16x16x32_bf16. Each operand may be stored either way round:
//   A_K = true : A stored [M][K] (k contiguous)      A_K = false: A stored [K][M] (m contiguous)
//   B_K = true : B stored [N][K] (k contiguous)      B_K = false: B stored [K][N] (n contiguous)
// Global->LDS staging always copies 16-byte runs in the operand's natural orientation; k-contiguous tiles feed the
// MFMA through ds_read_b128, m/n-contiguous tiles through the gfx950 transposing read ds_read_b64_tr_b16, so no
// operand is ever transposed element by element. A convolution is a GEMM whose k-contiguous A (forward) or
// n-contiguous B (weight gradient) rows are gathered on the fly from the activation image (AG / BG modes): the
// column matrix never exists in memory.
//
// Workgroup = 256 threads = 4 waves (2 x 2), tile BM x BN x BK (BK 64..256: small-K products take 1-3 k-steps so
// their latency is one or two memory round trips, not eight), LDS double-buffered with register prefetch, one
// barrier per k-step. Split-K over gridDim.z in two flavours:
//   * atomic: every split adds alpha*acc into fp32 C (pre-zeroed gradient slab) -- weight gradients, whose
//     reduction dimension is the batch (up to 64k rows);
//   * slab:   each split writes its fp32 partial tile to a workspace slab, the last-arriving split (agent-scope
//     release/acquire ticket, Guideline 16) sums the slabs in split order and runs the full epilogue --
//     deterministic, used for skinny forward products (M = 32 rollout rows against K = 3136).
// Epilogue (in order): *alpha, +bias[n], relu, *(mask[m,n] > 0) (ReLU backward), store fp32 | bf16 | atomic-add
// fp32, and optional column sums of the final values atomically added to colsum[n % colsum_mod] (bias gradients).
// out_mode 3 ("partials"): split z stores alpha*acc into plane z of C [splits, M, ldc] with no reduction, no
// ticket and no fence; the consumer kernel sums the planes in fixed order (deterministic) and applies bias and
// activation itself -- the rollout's fc product, whose only consumer is the fused policy/env kernel.
#pragma once
#include <type_traits>

#include "common.h"
#include "gemm_desc.h"

namespace aca {

typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));

// LDS layouts. k-contiguous tiles (read by ds_read_b128, whose lane groups are {0-3,12-15,20-27} /
// {4-11,16-19,28-31} per 32 lanes, bank = dword % 64) pad each row by 32 bytes: a 16-byte pad gave a 2-way
// conflict on every fragment read at any BK. m/n-contiguous tiles (rows of W = BM or BN elements, read by
// ds_read_b64_tr_b16: a 32-lane group reads k rows {r..r+3, r+8..r+11} x 32 bytes) are unpadded with the 16-byte
// chunk index XOR-swizzled by the row (gemm_tr_swz): no pad can separate rows r and r + 8 (2-way on every read);
// the swizzle makes both the transposed reads and the 16-byte staging stores conflict-free for W = 32..256.
constexpr int GEMM_PAD_K = 16;
constexpr int GEMM_PAD = 0;

template <int W>
__device__ __forceinline__ int gemm_tr_swz(int row) {
  static_assert(W == 32 || W == 64 || W == 128 || W == 256, "swizzle defined for 32..256-wide tiles");
  if constexpr (W == 32) return ((row >> 3) & 1) << 1;
  else if constexpr (W == 64) return (((row >> 1) & 1) << 1) ^ (((row >> 3) & 1) << 2);
  else return ((row & 1) << 1) ^ (((row >> 1) & 1) << 2) ^ (((row >> 3) & 1) << 3);
}

__device__ __forceinline__ uint4 pack8(const u16* t) {
  uint4 r;
  r.x = t[0] | ((uint32_t)t[1] << 16);
  r.y = t[2] | ((uint32_t)t[3] << 16);
  r.z = t[4] | ((uint32_t)t[5] << 16);
  r.w = t[6] | ((uint32_t)t[7] << 16);
  return r;
}

// 64 zero bytes in global memory: out-of-range operand chunks are loaded from here, so the loaded registers need
// no post-processing and their first use is the LDS store after the MFMAs of the current k-step (a select on the
// loaded data made the compiler drain every load right after issuing it, i.e. no prefetch overlap)
static __device__ __attribute__((aligned(64))) const unsigned char aca_zero_line[64] = {0};

template <typename T>
__device__ __forceinline__ const T* zero_or(bool ok, const T* p) {
  return ok ? p : reinterpret_cast<const T*>(aca_zero_line);
}

// loads through an explicit global (address space 1) pointer: a select between two generic pointers would
// otherwise compile to flat_load, which also counts against lgkmcnt and stalls every LDS wait of the k-loop
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4v gl_u32x4;
typedef const __attribute__((address_space(1))) unsigned int gl_u32;
__device__ __forceinline__ uint4 gload16(const void* p) {
  const u32x4v v = *(gl_u32x4*)(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t gload4(const void* p) { return *(gl_u32*)(p); }

// Branch-free 16-byte operand chunk (VEC operands: 16-byte aligned rows, ld % 8 == 0 and the contiguous extent
// % 8 == 0, so a chunk is wholly inside or wholly outside). No per-chunk branch means every chunk load of a k-step
// is in flight at once; the guarded form below made the compiler wait for each chunk before issuing the next (one
// memory round trip per chunk).
__device__ __forceinline__ uint4 load8v(const u16* base, int64_t row_off, int idx, int lim, bool row_ok) {
  const bool ok = row_ok && idx < lim;
  return gload16(zero_or(ok, base + row_off + idx));
}

// 8 contiguous bf16 at base[row_off + idx] (valid while idx+j < lim): any alignment / extent (scalar fallback)
__device__ __forceinline__ uint4 load8(const u16* base, int64_t row_off, int idx, int lim, bool row_ok) {
  if (!row_ok) return make_uint4(0, 0, 0, 0);
  const u16* p = base + row_off + idx;
  if (idx + 8 <= lim && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) return *reinterpret_cast<const uint4*>(p);
  u16 tmp[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) tmp[j] = (idx + j < lim) ? p[j] : (u16)0;
  return pack8(tmp);
}

__device__ __forceinline__ int fdiv(int n, AcaFastDiv f) {
  return (int)((__umulhi((unsigned int)n, f.m) + (unsigned int)n) >> f.s);
}

// Implicit-im2col gathers. Each thread stages fixed (row, column-chunk) slots of every k-step, so the part of the
// address that depends only on its fixed index is decoded ONCE before the k-loop (GCtx) and each k-step decodes
// only the varying index, with multiply-shift division (an integer-division sequence per index was ~30x the
// MFMA work of a tile).
struct GCtx {
  int64_t base;   // element offset of the fixed part
  int p, q;       // mode 3: input-image row / column of the output pixel
  int ok;
};

// A operand (modes 1/2/3): fixed conv row m of this chunk
template <int MODE>
__device__ __forceinline__ GCtx gctx_a(const AcaConvGather& g, int m, bool ok) {
  GCtx c{0, 0, 0, ok ? 1 : 0};
  if (!ok) return c;
  if (MODE == 3) {
    const int b = fdiv(m, g.fd_hw), p = m - b * g.H * g.W;
    const int ih = fdiv(p, g.fd_w);
    c.base = (int64_t)b * g.OH * g.OW;
    c.p = ih;
    c.q = p - ih * g.W;
  } else if (MODE == 5) {
    const int ph_pw = fdiv(m, g.fd_phase), r = m - ph_pw * g.B * g.HS * g.WS;
    const int b = fdiv(r, g.fd_hsws), p = r - b * g.HS * g.WS;
    const int a = fdiv(p, g.fd_ws);
    c.base = (int64_t)b * g.OH * g.OW;
    c.p = a;
    c.q = p - a * g.WS;
  } else {
    const int b = fdiv(m, g.fd_ohw), p = m - b * g.OH * g.OW;
    const int oh = fdiv(p, g.fd_ow), ow = p - oh * g.OW;
    c.base = MODE == 1 ? (((int64_t)b * g.C) * g.H + oh * g.S) * g.W + ow * g.S
                       : (((int64_t)b * g.H + oh * g.S) * g.W + ow * g.S) * g.C;
  }
  return c;
}

// mode-1 (uint8) chunks travel as two raw 32-bit words (x, y) and are converted when stored to LDS
__device__ __forceinline__ uint4 u8x8_raw(const uint8_t* src) {
  return make_uint4(gload4(src), gload4(src + 4), 0u, 0u);
}

__device__ __forceinline__ uint4 u8x8_convert(uint4 raw, float scale) {
  const uint32_t w0 = raw.x, w1 = raw.y;
  u16 t[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    t[e] = f2bf((float)((w0 >> (8 * e)) & 0xFF) * scale);
    t[4 + e] = f2bf((float)((w1 >> (8 * e)) & 0xFF) * scale);
  }
  return pack8(t);
}

// 8 consecutive k of the A row described by c (k % 8 == 0); branch-free (see load8v)
template <int MODE>
__device__ __forceinline__ uint4 gather_a(const AcaConvGather& g, const GCtx& c, int k, bool kok) {
  bool ok = c.ok && kok;
  if (MODE == 1) {
    const int ci = fdiv(k, g.fd_khw), r = k - ci * g.KH * g.KW;
    const int i = fdiv(r, g.fd_kw), j = r - i * g.KW;
    const int64_t off = c.base + ((int64_t)ci * g.H + i) * g.W + j;
    return u8x8_raw(zero_or(ok, reinterpret_cast<const uint8_t*>(g.src) + off));
  }
  if (MODE == 5) {
    // k = (di, dj, o): source pixel (a - di, c - dj) of the output gradient
    const int di = fdiv(k, g.fd_kwsc), r = k - di * g.KWS * g.C;
    const int dj = fdiv(r, g.fd_c), cc = r - dj * g.C;
    const int sh = c.p - di, sw = c.q - dj;
    ok = ok && sh >= 0 && sw >= 0 && sh < g.OH && sw < g.OW;
    const int64_t off5 = (c.base + (int64_t)sh * g.OW + sw) * g.C + cc;
    return gload16(zero_or(ok, reinterpret_cast<const u16*>(g.src) + off5));
  }
  const int i = fdiv(k, g.fd_kwc), r = k - i * g.KW * g.C;
  const int j = fdiv(r, g.fd_c), cc = r - j * g.C;
  int64_t off;
  if (MODE == 2) {
    off = c.base + (i * g.W + j) * g.C + cc;
  } else {
    // MODE 3: transposed conv (data gradient): source pixel ((ih - i) / S, (iw - j) / S) when on the stride grid
    const int th = c.p - i, tw = c.q - j;
    const int sh = fdiv(max(th, 0), g.fd_s), sw = fdiv(max(tw, 0), g.fd_s);
    ok = ok && th >= 0 && tw >= 0 && sh * g.S == th && sw * g.S == tw && sh < g.OH && sw < g.OW;
    off = (c.base + (int64_t)sh * g.OW + sw) * g.C + cc;
  }
  return gload16(zero_or(ok, reinterpret_cast<const u16*>(g.src) + off));
}

// B operand (modes 1/2: weight gradient, B[k = conv row][n = conv column]; mode 4: OHWI weight read as
// B[k = (i, j, o)][n]): fixed column n of this chunk
template <int MODE>
__device__ __forceinline__ GCtx gctx_b(const AcaConvGather& g, int n, bool ok, int phase = 0) {
  GCtx c{0, 0, 0, ok ? 1 : 0};
  if (!ok) return c;
  if (MODE == 6) {   // phase (ph, pw) of the workgroup's rows
    const int ph = fdiv(phase, g.fd_s);
    c.p = ph;
    c.q = phase - ph * g.S;
    c.base = n;
    return c;
  }
  if (MODE == 1) {
    const int ci = fdiv(n, g.fd_khw), r = n - ci * g.KH * g.KW;
    const int i = fdiv(r, g.fd_kw), j = r - i * g.KW;
    c.base = ((int64_t)ci * g.H + i) * g.W + j;
  } else if (MODE == 2) {
    const int i = fdiv(n, g.fd_kwc), r = n - i * g.KW * g.C;
    const int j = fdiv(r, g.fd_c), cc = r - j * g.C;
    c.base = ((int64_t)i * g.W + j) * g.C + cc;
  } else {
    c.base = n;
  }
  return c;
}

template <int MODE>
__device__ __forceinline__ uint4 gather_b(const AcaConvGather& g, const GCtx& c, int k, bool kok) {
  const bool ok = c.ok && kok;
  if (MODE == 6) {
    const int di = fdiv(k, g.fd_kwsc), r = k - di * g.KWS * g.C;
    const int dj = fdiv(r, g.fd_c), o = r - dj * g.C;
    const int i = c.p + g.S * di, j = c.q + g.S * dj;
    const int64_t off = (((int64_t)o * g.KH + i) * g.KW + j) * g.W + c.base;
    return gload16(zero_or(ok, reinterpret_cast<const u16*>(g.src) + off));
  }
  if (MODE == 4) {
    const int ij = fdiv(k, g.fd_c), o = k - ij * g.C;
    const int64_t off = ((int64_t)o * g.KH * g.KW + ij) * g.W + c.base;
    return gload16(zero_or(ok, reinterpret_cast<const u16*>(g.src) + off));
  }
  const int b = fdiv(k, g.fd_ohw), p = k - b * g.OH * g.OW;
  const int oh = fdiv(p, g.fd_ow), ow = p - oh * g.OW;
  if (MODE == 1) {
    const int64_t rb = (((int64_t)b * g.C) * g.H + oh * g.S) * g.W + ow * g.S;
    return u8x8_raw(zero_or(ok, reinterpret_cast<const uint8_t*>(g.src) + rb + c.base));
  }
  const int64_t rb = (((int64_t)b * g.H + oh * g.S) * g.W + ow * g.S) * g.C;
  return gload16(zero_or(ok, reinterpret_cast<const u16*>(g.src) + rb + c.base));
}

struct GemmParams {
  AcaGemmDesc d;
  int k_tiles_per_split;
  int splits;
};

// LDS footprint (bf16 elements) of one tile configuration: double-buffered A and B k-step tiles
template <int BM, int BN, int BK, bool A_K, bool B_K>
struct GemmSmem {
  static constexpr int A_ELEMS = A_K ? BM * (BK + GEMM_PAD_K) : BK * (BM + GEMM_PAD);
  static constexpr int B_ELEMS = B_K ? BN * (BK + GEMM_PAD_K) : BK * (BN + GEMM_PAD);
  static constexpr int ELEMS = 2 * (A_ELEMS + B_ELEMS);
};

// One output tile x one K split of a product: the body shared by the one-product kernel (gemm_kernel, tile =
// blockIdx.x, z = blockIdx.z) and the grouped kernel (gemm_group_kernel: several independent products of up to two
// tile configurations in ONE launch, so a backward pass issues its independent products without cross-stream
// dependencies). `smem` is the caller's LDS array (>= GemmSmem::ELEMS), `ntiles` the product's tile count.
template <int BM, int BN, int BK, bool A_K, bool B_K, int AG, int BG, bool VEC>
__device__ __forceinline__ void gemm_block(const GemmParams& P, const int tile, const int z, const int ntiles,
                                           u16* const smem, int& sh_flag) {
  const AcaGemmDesc& g = P.d;
  constexpr int A_ELEMS = GemmSmem<BM, BN, BK, A_K, B_K>::A_ELEMS;
  constexpr int B_ELEMS = GemmSmem<BM, BN, BK, A_K, B_K>::B_ELEMS;
  constexpr int TM = BM / 32, TN = BN / 32;   // 16x16 MFMA tiles per wave (2 x 2 waves)
  constexpr int A_CHUNKS = BM * BK / 8 / 256;  // 16-byte chunks per thread per k-step
  constexpr int B_CHUNKS = BN * BK / 8 / 256;
  static_assert(A_CHUNKS >= 1 && B_CHUNKS >= 1, "tile too small");
  static_assert(!AG || A_K, "A gather needs a k-contiguous A");
  static_assert(!BG || !B_K, "B gather needs an n-contiguous B");
  u16* const As0 = smem;
  u16* const Bs0 = smem + 2 * A_ELEMS;
  const u16* Ag = reinterpret_cast<const u16*>(g.A);
  const u16* Bg = reinterpret_cast<const u16*>(g.B);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int k_tiles_total = (g.K + BK - 1) / BK;
  const int kt0 = z * P.k_tiles_per_split;
  const int kt1 = min(kt0 + P.k_tiles_per_split, k_tiles_total);

  unsigned long long* const st =
      g.stamps ? g.stamps + ((size_t)z * ntiles + tile) * 4 : nullptr;
  if (st && tid == 0) st[0] = __builtin_amdgcn_s_memrealtime();
  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // two register sets: the k-loop keeps two k-steps of operand loads in flight (prefetch distance 2)
  uint4 ra0[A_CHUNKS], rb0[B_CHUNKS], ra1[A_CHUNKS], rb1[B_CHUNKS];
  // gather contexts of this thread's fixed staging slots (decoded once)
  GCtx actx[AG ? A_CHUNKS : 1], bctx[BG ? B_CHUNKS : 1];
  if (AG) {
#pragma unroll
    for (int c = 0; c < A_CHUNKS; ++c) {
      const int r = (tid + c * 256) / (BK / 8);
      actx[c] = gctx_a<AG>(g.ga, m0 + r, m0 + r < g.M);
    }
  }
  if (BG) {
#pragma unroll
    for (int c = 0; c < B_CHUNKS; ++c) {
      const int nc = ((tid + c * 256) % (BN / 8)) * 8;
      bctx[c] = gctx_b<BG>(g.gb, n0 + nc, n0 + nc < g.N, BG == 6 ? fdiv(m0, g.ga.fd_phase) : 0);
    }
  }

  auto gload = [&](int kt, uint4 (&ra)[A_CHUNKS], uint4 (&rb)[B_CHUNKS]) {
    const int k0 = kt * BK;
#pragma unroll
    for (int c = 0; c < A_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      if (A_K) {
        const int r = ch / (BK / 8), kc = (ch % (BK / 8)) * 8;
        const int m = m0 + r;
        if (AG) ra[c] = gather_a<AG>(g.ga, actx[AG ? c : 0], k0 + kc, k0 + kc < g.K);
        else if (VEC) ra[c] = load8v(Ag, (int64_t)m * g.lda, k0 + kc, g.K, m < g.M);
        else ra[c] = load8(Ag, (int64_t)m * g.lda, k0 + kc, g.K, m < g.M);
      } else {
        const int kr = ch / (BM / 8), mc = (ch % (BM / 8)) * 8;
        const int k = k0 + kr;
        ra[c] = VEC ? load8v(Ag, (int64_t)k * g.lda, m0 + mc, g.M, k < g.K)
                    : load8(Ag, (int64_t)k * g.lda, m0 + mc, g.M, k < g.K);
      }
    }
#pragma unroll
    for (int c = 0; c < B_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      if (B_K) {
        const int r = ch / (BK / 8), kc = (ch % (BK / 8)) * 8;
        const int n = n0 + r;
        rb[c] = VEC ? load8v(Bg, (int64_t)n * g.ldb, k0 + kc, g.K, n < g.N)
                    : load8(Bg, (int64_t)n * g.ldb, k0 + kc, g.K, n < g.N);
      } else {
        const int kr = ch / (BN / 8), nc = (ch % (BN / 8)) * 8;
        const int k = k0 + kr;
        if (BG) rb[c] = gather_b<BG>(g.gb, bctx[BG ? c : 0], k, k < g.K);
        else if (VEC) rb[c] = load8v(Bg, (int64_t)k * g.ldb, n0 + nc, g.N, k < g.K);
        else rb[c] = load8(Bg, (int64_t)k * g.ldb, n0 + nc, g.N, k < g.K);
      }
    }
  };
  auto sstore = [&](int buf, const uint4 (&ra)[A_CHUNKS], const uint4 (&rb)[B_CHUNKS]) {
#pragma unroll
    for (int c = 0; c < A_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      int off;
      if (A_K) off = (ch / (BK / 8)) * (BK + GEMM_PAD_K) + (ch % (BK / 8)) * 8;
      else {
        const int kr = ch / (BM / 8);
        off = kr * (BM + GEMM_PAD) + ((ch % (BM / 8)) ^ gemm_tr_swz<BM>(kr)) * 8;
      }
      *reinterpret_cast<uint4*>(As0 + buf * A_ELEMS + off) = AG == 1 ? u8x8_convert(ra[c], g.ga.scale) : ra[c];
    }
#pragma unroll
    for (int c = 0; c < B_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      int off;
      if (B_K) off = (ch / (BK / 8)) * (BK + GEMM_PAD_K) + (ch % (BK / 8)) * 8;
      else {
        const int kr = ch / (BN / 8);
        off = kr * (BN + GEMM_PAD) + ((ch % (BN / 8)) ^ gemm_tr_swz<BN>(kr)) * 8;
      }
      *reinterpret_cast<uint4*>(Bs0 + buf * B_ELEMS + off) = BG == 1 ? u8x8_convert(rb[c], g.gb.scale) : rb[c];
    }
  };

  const int lr16 = lane & 15, lg = lane >> 4;   // row-in-tile, k-group
  const int q = lr16 >> 2, p = lr16 & 3;        // transposed-read address roles (lane 4q+p of each 16-lane group)
  typedef __attribute__((address_space(3))) short4v lds_s4;

  // m/n-contiguous operand: element (k, col) of a W-wide tile at row k, 16-byte chunk (col / 8) ^ swz(k)
  auto tr_addr = [&](const u16* base, auto wtag, int k, int col) -> const u16* {
    constexpr int W = decltype(wtag)::value;
    return base + k * (W + GEMM_PAD) + (((col >> 3) ^ gemm_tr_swz<W>(k)) << 3) + (col & 7);
  };
  auto frag = [&](const u16* base, bool kc, auto wtag, int rowbase, int ks) -> bf16x8 {
    if (kc) {
      return *reinterpret_cast<const bf16x8*>(base + (rowbase + lr16) * (BK + GEMM_PAD_K) + ks * 32 + lg * 8);
    } else {
      const int kb = ks * 32 + lg * 8;
      const u16* p0 = tr_addr(base, wtag, kb + q, rowbase + 4 * p);
      const u16* p1 = tr_addr(base, wtag, kb + 4 + q, rowbase + 4 * p);
      const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p0));
      const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p1));
      const short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  };

  auto compute = [&](int buf) {
    const u16* as = As0 + buf * A_ELEMS;
    const u16* bs = Bs0 + buf * B_ELEMS;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = frag(as, A_K, std::integral_constant<int, BM>{}, wm * (BM / 2) + i * 16, ks);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = frag(bs, B_K, std::integral_constant<int, BN>{}, wn * (BN / 2) + j * 16, ks);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // Pipeline (small products are latency-bound: a k-step's MFMA work is far shorter than an L2 round trip, so
  // with one step of prefetch every step costs a full round trip). Register set s holds k-step kt+2 while LDS
  // buffer b holds kt and the other register set waits to be stored as kt+1: loads are issued two k-steps ahead,
  // unconditionally (steps past the end read the zero line or a neighbouring split's data that is never stored),
  // so the loop body has no data-dependent branch around its loads.
  if (kt0 < kt1) {
    gload(kt0, ra0, rb0);
    gload(kt0 + 1, ra1, rb1);
    sstore(0, ra0, rb0);
    __syncthreads();
    if (st && tid == 0) st[1] = __builtin_amdgcn_s_memrealtime();
    // (the LDS stores are unconditional too: a store past the last k-step is never read, and a conditional one
    // leaves loads pending on one path, which makes the compiler drain them at the loop head)
    for (int kt = kt0; kt < kt1; kt += 2) {
      gload(kt + 2, ra0, rb0);
      compute(0);
      sstore(1, ra1, rb1);
      __syncthreads();
      if (kt + 1 >= kt1) break;
      gload(kt + 3, ra1, rb1);
      compute(1);
      sstore(0, ra0, rb0);
      __syncthreads();
    }
  }

  if (st && tid == 0) st[2] = __builtin_amdgcn_s_memrealtime();
  // ---------------------------------------------------------------- split-K reduction (slab flavour)
  if (P.splits > 1 && g.out_mode < 2) {
    float* slab = g.ws + ((size_t)tile * P.splits + z) * (BM * BN);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[((i * TN + j) * 4 + r) * 256 + tid] = acc[i][j][r];
    if (!last_block_arrival(&g.tickets[tile], P.splits, &sh_flag)) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // slabs summed in split order, four splits' loads in flight per round (missing ones read the zero line)
    typedef const __attribute__((address_space(1))) float gl_f32;
    for (int s0 = 0; s0 < P.splits; s0 += 4) {
      float v[4][TM][TN][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool on = s0 + u < P.splits;
        const float* sl = g.ws + ((size_t)tile * P.splits + (on ? s0 + u : 0)) * (BM * BN);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float* q = sl + ((i * TN + j) * 4 + r) * 256 + tid;
              v[u][i][j][r] = *(gl_f32*)(on ? q : reinterpret_cast<const float*>(aca_zero_line));
            }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] += v[u][i][j][r];
    }
  }

  // ---------------------------------------------------------------- epilogue
  // output row of GEMM row m (mode 5 rows are phase-major: write each back to its NHWC pixel)
  auto out_row = [&](int m) -> int64_t {
    if (AG != 5) return m;
    const AcaConvGather& a = g.ga;
    const int ph_pw = fdiv(m, a.fd_phase), r = m - ph_pw * a.B * a.HS * a.WS;
    const int b = fdiv(r, a.fd_hsws), p = r - b * a.HS * a.WS;
    const int aa = fdiv(p, a.fd_ws), cc = p - aa * a.WS;
    const int ph = fdiv(ph_pw, a.fd_s), pw = ph_pw - ph * a.S;
    return ((int64_t)b * a.H + aa * a.S + ph) * a.W + cc * a.S + pw;
  };
  // bias and ReLU-backward mask operands are fetched for every output of this thread up front, branch-free (a
  // guarded load per output element serialised TM*TN*4 memory round trips at the end of every product)
  typedef const __attribute__((address_space(1))) u16 gl_u16;
  typedef const __attribute__((address_space(1))) float gl_f32e;
  const u16* mask = reinterpret_cast<const u16*>(g.mask);
  float bias_v[TN];
  u16 mk[TM][TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 16 + lr16;
    const bool n_ok = n < g.N;
    bias_v[j] = g.bias ? *(gl_f32e*)(n_ok ? g.bias + n : reinterpret_cast<const float*>(aca_zero_line)) : 0.f;
    if (mask) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * (BM / 2) + i * 16 + lg * 4 + r;
          const bool ok = n_ok && m < g.M;
          const int64_t mr = out_row(m);
          mk[i][j][r] = *(gl_u16*)(ok ? mask + mr * g.ldm + n : reinterpret_cast<const u16*>(aca_zero_line));
        }
    }
  }
  float csums[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 16 + lr16;
    const bool n_ok = n < g.N;
    const float b = bias_v[j];
    float csum = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + lg * 4 + r;
        if (!(n_ok && m < g.M)) continue;
        if (g.out_mode == 3) {   // split-K partial plane z, reduced (with bias / activation) by the consumer
          reinterpret_cast<float*>(g.C)[((int64_t)z * g.M + m) * g.ldc + n] = acc[i][j][r] * g.alpha;
          continue;
        }
        float v = acc[i][j][r] * g.alpha + b;
        if (g.relu) v = fmaxf(v, 0.f);
        if (mask) v = (bf2f(mk[i][j][r]) > 0.f) ? v : 0.f;
        const int64_t ci = out_row(m) * g.ldc + n;
        if (g.out_mode == 0) reinterpret_cast<float*>(g.C)[ci] = v;
        else if (g.out_mode == 1) reinterpret_cast<u16*>(g.C)[ci] = f2bf(v);
        else atomicAdd(reinterpret_cast<float*>(g.C) + ci, v);
        csum += v;
      }
    }
    csum += lane_xor(csum, 16);
    csum += lane_xor(csum, 32);
    csums[j] = csum;
    if (g.colsum && !g.colsum_part && lg == 0 && n_ok)
      atomicAdd(&g.colsum[g.colsum_mod ? n % g.colsum_mod : n], csum);
  }
  if (g.colsum_part) {
    // the two waves sharing these columns (wm = 0, 1) combine through LDS, then one plain store per column
    float* csh = reinterpret_cast<float*>(smem);
    __syncthreads();   // every wave is past its last LDS operand read
    if (wm == 1 && lg == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) csh[wn * (BN / 2) + j * 16 + lr16] = csums[j];
    __syncthreads();
    if (wm == 0 && lg == 0)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wn * (BN / 2) + j * 16 + lr16;
        if (n0 + nl < g.N) g.colsum_part[(int64_t)(m0 / BM) * g.N + n0 + nl] = csums[j] + csh[nl];
      }
  }
  if (st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) st[3] = __builtin_amdgcn_s_memrealtime();
  }
}

template <int BM, int BN, int BK, bool A_K, bool B_K, int AG, int BG, bool VEC>
__global__ void __launch_bounds__(256) gemm_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(16))) u16 smem[GemmSmem<BM, BN, BK, A_K, B_K>::ELEMS];
  __shared__ int sh_flag;
  // XCD-grouped order: the tiles of one K split (which share their operand rows) run on one XCD
  const int L = xcd_chunk_remap(blockIdx.z * gridDim.x + blockIdx.x, gridDim.x * gridDim.z, gridDim.x);
  gemm_block<BM, BN, BK, A_K, B_K, AG, BG, VEC>(P, L % gridDim.x, L / gridDim.x, gridDim.x, smem, sh_flag);
}

// ---------------------------------------------------------------------------------------------- grouped launch
// Up to GEMM_GROUP_MAX independent products in one launch; product k uses tile configuration CA (cfg[k] == 0) or
// CB (cfg[k] == 1). Its workgroups are blocks [start[k], start[k + 1]) of the flat grid: tile = local % tiles[k],
// split = local / tiles[k].
constexpr int GEMM_GROUP_MAX = 3;
struct GemmGroupArgs {
  GemmParams p[GEMM_GROUP_MAX];
  int tiles[GEMM_GROUP_MAX];
  int start[GEMM_GROUP_MAX + 1];
  int cfg[GEMM_GROUP_MAX];
  int n;
};

template <int BM, int BN, int BK, bool A_K, bool B_K, int AG, int BG, bool VEC>
struct GemmCfg {
  static constexpr int bm = BM, bn = BN, smem = GemmSmem<BM, BN, BK, A_K, B_K>::ELEMS;
  static __device__ __forceinline__ void run(const GemmParams& P, int tile, int z, int ntiles, u16* sm, int& f) {
    gemm_block<BM, BN, BK, A_K, B_K, AG, BG, VEC>(P, tile, z, ntiles, sm, f);
  }
};

template <class CA, class CB>
__global__ void __launch_bounds__(256) gemm_group_kernel(GemmGroupArgs G) {
  constexpr int SM = CA::smem > CB::smem ? CA::smem : CB::smem;
  __shared__ __attribute__((aligned(16))) u16 smem[SM];
  __shared__ int sh_flag;
  const int b = blockIdx.x;
  int k = 0;
  if (G.n > 1 && b >= G.start[1]) k = 1;
  if (G.n > 2 && b >= G.start[2]) k = 2;
  // XCD-grouped order per product: the tiles of one K split (sharing their operand rows: the conv weight gradients'
  // input pixels) run on one XCD, the splits rotate over the XCDs (profiles/r5_pong_pmc.txt: 53 MB fetched for
  // ~17 MB of operands in plain order)
  const int tiles = G.tiles[k];
  const int local = xcd_chunk_remap(b - G.start[k], G.start[k + 1] - G.start[k], tiles);
  if (G.cfg[k] == 0) CA::run(G.p[k], local % tiles, local / tiles, tiles, smem, sh_flag);
  else CB::run(G.p[k], local % tiles, local / tiles, tiles, smem, sh_flag);
}

template <class CA, class CB>
hipError_t gemm_group_launch(GemmGroupArgs& G, hipStream_t s) {
  int total = 0;
  for (int k = 0; k < G.n; ++k) {
    const int bm = G.cfg[k] == 0 ? CA::bm : CB::bm, bn = G.cfg[k] == 0 ? CA::bn : CB::bn;
    G.tiles[k] = ((G.p[k].d.M + bm - 1) / bm) * ((G.p[k].d.N + bn - 1) / bn);
    G.start[k] = total;
    total += G.tiles[k] * G.p[k].splits;
  }
  G.start[G.n] = total;
  gemm_group_kernel<CA, CB><<<total, 256, 0, s>>>(G);
  return hipGetLastError();
}

template <int BM, int BN, int BK, bool A_K, bool B_K, int AG, int BG, bool VEC>
hipError_t gemm_launch(const GemmParams& P, hipStream_t s) {
  const int tiles = ((P.d.M + BM - 1) / BM) * ((P.d.N + BN - 1) / BN);
  dim3 grid(tiles, 1, P.splits);
  gemm_kernel<BM, BN, BK, A_K, B_K, AG, BG, VEC><<<grid, 256, 0, s>>>(P);
  return hipGetLastError();
}

// dispatch over the supported (tile, bk) pairs for one operand family
template <bool A_K, bool B_K, int AG, int BG, bool VEC>
hipError_t gemm_dispatch_tiles(const GemmParams& P, hipStream_t s) {
  const int t = P.d.tile, bk = P.d.bk;
  if (bk == 64) {
    switch (t) {
      case 0: return gemm_launch<64, 64, 64, A_K, B_K, AG, BG, VEC>(P, s);
      case 1: return gemm_launch<32, 64, 64, A_K, B_K, AG, BG, VEC>(P, s);
      case 2: return gemm_launch<64, 32, 64, A_K, B_K, AG, BG, VEC>(P, s);
      case 3: return gemm_launch<128, 64, 64, A_K, B_K, AG, BG, VEC>(P, s);
      case 4: return gemm_launch<32, 32, 64, A_K, B_K, AG, BG, VEC>(P, s);
      case 5: return gemm_launch<64, 256, 64, A_K, B_K, AG, BG, VEC>(P, s);
      case 6: return gemm_launch<32, 256, 64, A_K, B_K, AG, BG, VEC>(P, s);
      case 7: return gemm_launch<128, 128, 64, A_K, B_K, AG, BG, VEC>(P, s);
    }
  } else if (bk == 128) {
    switch (t) {
      case 0: return gemm_launch<64, 64, 128, A_K, B_K, AG, BG, VEC>(P, s);
      case 1: return gemm_launch<32, 64, 128, A_K, B_K, AG, BG, VEC>(P, s);
      case 2: return gemm_launch<64, 32, 128, A_K, B_K, AG, BG, VEC>(P, s);
      case 4: return gemm_launch<32, 32, 128, A_K, B_K, AG, BG, VEC>(P, s);
    }
  } else if (bk == 256) {
    if (t == 4) return gemm_launch<32, 32, 256, A_K, B_K, AG, BG, VEC>(P, s);
  }
  return hipErrorInvalidValue;
}

// vector-loadable plain operand: 16-byte aligned base, row stride % 8 == 0, contiguous extent % 8 == 0
inline bool gemm_operand_vec(const void* p, int64_t ld, int contig_extent) {
  return (reinterpret_cast<uintptr_t>(p) % 16 == 0) && (ld % 8 == 0) && (contig_extent % 8 == 0);
}

}  // namespace aca
