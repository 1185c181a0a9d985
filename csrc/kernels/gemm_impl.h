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
#pragma once
#include "common.h"
#include "gemm_desc.h"

namespace aca {

typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));

constexpr int GEMM_PAD = 8;  // 16 bytes per LDS row

__device__ __forceinline__ uint4 pack8(const u16* t) {
  uint4 r;
  r.x = t[0] | ((uint32_t)t[1] << 16);
  r.y = t[2] | ((uint32_t)t[3] << 16);
  r.z = t[4] | ((uint32_t)t[5] << 16);
  r.w = t[6] | ((uint32_t)t[7] << 16);
  return r;
}

// 8 contiguous bf16 at base[row_off + idx] (valid while idx+j < lim)
__device__ __forceinline__ uint4 load8(const u16* base, int64_t row_off, int idx, int lim, bool row_ok) {
  if (!row_ok) return make_uint4(0, 0, 0, 0);
  const u16* p = base + row_off + idx;
  if (idx + 8 <= lim && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) return *reinterpret_cast<const uint4*>(p);
  u16 tmp[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) tmp[j] = (idx + j < lim) ? p[j] : (u16)0;
  return pack8(tmp);
}

// implicit im2col: 8 consecutive k of conv-output row m (k % 8 == 0)
template <int MODE>
__device__ __forceinline__ uint4 gather8(const AcaConvGather& g, int m, int k, bool ok) {
  if (!ok) return make_uint4(0, 0, 0, 0);
  if (MODE == 3) {
    // transposed conv (data gradient): row m = (b, ih, iw) of the conv INPUT, k = (i, j, c) over the output-gradient
    // channels; the source pixel is ((ih - i) / S, (iw - j) / S) when that lands on the stride grid, else zero
    const int hw = g.H * g.W;
    const int b = m / hw, p = m - b * hw;
    const int ih = p / g.W, iw = p - ih * g.W;
    const int kwc = g.KW * g.C;
    const int i = k / kwc, r = k - i * kwc;
    const int j = r / g.C, c = r - j * g.C;
    const int th = ih - i, tw = iw - j;
    if (th < 0 || tw < 0) return make_uint4(0, 0, 0, 0);
    const int sh = th / g.S, sw = tw / g.S;
    if (sh * g.S != th || sw * g.S != tw || sh >= g.OH || sw >= g.OW) return make_uint4(0, 0, 0, 0);
    return *reinterpret_cast<const uint4*>(reinterpret_cast<const u16*>(g.src) +
                                           (((int64_t)b * g.OH + sh) * g.OW + sw) * g.C + c);
  }
  if (MODE == 4) {
    // OHWI conv weight read as B[k = (i, j, o)][n = input channel] (the transposed-conv operand): row m = k here
    const int khw = g.KH * g.KW;
    const int ij = m / g.C, o = m - ij * g.C;
    return *reinterpret_cast<const uint4*>(reinterpret_cast<const u16*>(g.src) + ((int64_t)o * khw + ij) * g.W + k);
  }
  const int ohw = g.OH * g.OW;
  const int b = m / ohw, p = m - b * ohw;
  const int oh = p / g.OW, ow = p - oh * g.OW;
  if (MODE == 1) {
    const int khw = g.KH * g.KW;
    const int c = k / khw, r = k - c * khw;
    const int i = r / g.KW, j = r - i * g.KW;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(g.src) +
                         (((int64_t)b * g.C + c) * g.H + oh * g.S + i) * g.W + ow * g.S + j;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(src);
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(src + 4);
    u16 t[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      t[e] = f2bf((float)((w0 >> (8 * e)) & 0xFF) * g.scale);
      t[4 + e] = f2bf((float)((w1 >> (8 * e)) & 0xFF) * g.scale);
    }
    return pack8(t);
  } else {
    const int kwc = g.KW * g.C;
    const int i = k / kwc, r = k - i * kwc;
    const int j = r / g.C, c = r - j * g.C;
    const u16* src = reinterpret_cast<const u16*>(g.src) +
                     (((int64_t)b * g.H + oh * g.S + i) * g.W + ow * g.S + j) * g.C + c;
    return *reinterpret_cast<const uint4*>(src);
  }
}

struct GemmParams {
  AcaGemmDesc d;
  int k_tiles_per_split;
  int splits;
};

template <int BM, int BN, int BK, bool A_K, bool B_K, int AG, int BG>
__global__ void __launch_bounds__(256) gemm_kernel(GemmParams P) {
  const AcaGemmDesc& g = P.d;
  constexpr int A_ELEMS = A_K ? BM * (BK + GEMM_PAD) : BK * (BM + GEMM_PAD);
  constexpr int B_ELEMS = B_K ? BN * (BK + GEMM_PAD) : BK * (BN + GEMM_PAD);
  constexpr int TM = BM / 32, TN = BN / 32;   // 16x16 MFMA tiles per wave (2 x 2 waves)
  constexpr int A_CHUNKS = BM * BK / 8 / 256;  // 16-byte chunks per thread per k-step
  constexpr int B_CHUNKS = BN * BK / 8 / 256;
  static_assert(A_CHUNKS >= 1 && B_CHUNKS >= 1, "tile too small");
  static_assert(!AG || A_K, "A gather needs a k-contiguous A");
  static_assert(!BG || !B_K, "B gather needs an n-contiguous B");
  __shared__ __attribute__((aligned(16))) u16 smem[2 * (A_ELEMS + B_ELEMS)];
  __shared__ int sh_flag;
  u16* const As0 = smem;
  u16* const Bs0 = smem + 2 * A_ELEMS;
  const u16* Ag = reinterpret_cast<const u16*>(g.A);
  const u16* Bg = reinterpret_cast<const u16*>(g.B);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int tile = blockIdx.x;
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int z = blockIdx.z;
  const int k_tiles_total = (g.K + BK - 1) / BK;
  const int kt0 = z * P.k_tiles_per_split;
  const int kt1 = min(kt0 + P.k_tiles_per_split, k_tiles_total);

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[A_CHUNKS], rb[B_CHUNKS];

  auto gload = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int c = 0; c < A_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      if (A_K) {
        const int r = ch / (BK / 8), kc = (ch % (BK / 8)) * 8;
        const int m = m0 + r;
        if (AG) ra[c] = gather8<AG>(g.ga, m, k0 + kc, m < g.M && k0 + kc < g.K);
        else ra[c] = load8(Ag, (int64_t)m * g.lda, k0 + kc, g.K, m < g.M);
      } else {
        const int kr = ch / (BM / 8), mc = (ch % (BM / 8)) * 8;
        const int k = k0 + kr;
        ra[c] = load8(Ag, (int64_t)k * g.lda, m0 + mc, g.M, k < g.K);
      }
    }
#pragma unroll
    for (int c = 0; c < B_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      if (B_K) {
        const int r = ch / (BK / 8), kc = (ch % (BK / 8)) * 8;
        const int n = n0 + r;
        rb[c] = load8(Bg, (int64_t)n * g.ldb, k0 + kc, g.K, n < g.N);
      } else {
        const int kr = ch / (BN / 8), nc = (ch % (BN / 8)) * 8;
        const int k = k0 + kr;
        if (BG) rb[c] = gather8<BG>(g.gb, k, n0 + nc, k < g.K && n0 + nc < g.N);
        else rb[c] = load8(Bg, (int64_t)k * g.ldb, n0 + nc, g.N, k < g.K);
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int c = 0; c < A_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      int off;
      if (A_K) off = (ch / (BK / 8)) * (BK + GEMM_PAD) + (ch % (BK / 8)) * 8;
      else off = (ch / (BM / 8)) * (BM + GEMM_PAD) + (ch % (BM / 8)) * 8;
      *reinterpret_cast<uint4*>(As0 + buf * A_ELEMS + off) = ra[c];
    }
#pragma unroll
    for (int c = 0; c < B_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      int off;
      if (B_K) off = (ch / (BK / 8)) * (BK + GEMM_PAD) + (ch % (BK / 8)) * 8;
      else off = (ch / (BN / 8)) * (BN + GEMM_PAD) + (ch % (BN / 8)) * 8;
      *reinterpret_cast<uint4*>(Bs0 + buf * B_ELEMS + off) = rb[c];
    }
  };

  const int lr16 = lane & 15, lg = lane >> 4;   // row-in-tile, k-group
  const int q = lr16 >> 2, p = lr16 & 3;        // transposed-read address roles (lane 4q+p of each 16-lane group)
  typedef __attribute__((address_space(3))) short4v lds_s4;

  auto frag = [&](const u16* base, bool kc, int ld_dim, int rowbase, int ks) -> bf16x8 {
    if (kc) {
      return *reinterpret_cast<const bf16x8*>(base + (rowbase + lr16) * (BK + GEMM_PAD) + ks * 32 + lg * 8);
    } else {
      const int kb = ks * 32 + lg * 8;
      const u16* p0 = base + (kb + q) * (ld_dim + GEMM_PAD) + rowbase + 4 * p;
      const u16* p1 = base + (kb + 4 + q) * (ld_dim + GEMM_PAD) + rowbase + 4 * p;
      const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p0));
      const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p1));
      const short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  };

  if (kt0 < kt1) {
    gload(kt0);
    sstore(0);
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int buf = (kt - kt0) & 1;
      const bool more = kt + 1 < kt1;
      if (more) gload(kt + 1);
      const u16* as = As0 + buf * A_ELEMS;
      const u16* bs = Bs0 + buf * B_ELEMS;
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag(as, A_K, BM, wm * (BM / 2) + i * 16, ks);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag(bs, B_K, BN, wn * (BN / 2) + j * 16, ks);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
      if (more) sstore(buf ^ 1);
      __syncthreads();
    }
  }

  // ---------------------------------------------------------------- split-K reduction (slab flavour)
  if (P.splits > 1 && g.out_mode != 2) {
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
    for (int s = 0; s < P.splits; ++s) {
      const float* sl = g.ws + ((size_t)tile * P.splits + s) * (BM * BN);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += sl[((i * TN + j) * 4 + r) * 256 + tid];
    }
  }

  // ---------------------------------------------------------------- epilogue
  const u16* mask = reinterpret_cast<const u16*>(g.mask);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 16 + lr16;
    const bool n_ok = n < g.N;
    const float b = (g.bias && n_ok) ? g.bias[n] : 0.f;
    float csum = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + lg * 4 + r;
        if (!(n_ok && m < g.M)) continue;
        float v = acc[i][j][r] * g.alpha + b;
        if (g.relu) v = fmaxf(v, 0.f);
        if (mask) v = (bf2f(mask[(int64_t)m * g.ldm + n]) > 0.f) ? v : 0.f;
        const int64_t ci = (int64_t)m * g.ldc + n;
        if (g.out_mode == 0) reinterpret_cast<float*>(g.C)[ci] = v;
        else if (g.out_mode == 1) reinterpret_cast<u16*>(g.C)[ci] = f2bf(v);
        else atomicAdd(reinterpret_cast<float*>(g.C) + ci, v);
        csum += v;
      }
    }
    if (g.colsum) {
      csum += __shfl_xor(csum, 16, 64);
      csum += __shfl_xor(csum, 32, 64);
      if (lg == 0 && n_ok) atomicAdd(&g.colsum[g.colsum_mod ? n % g.colsum_mod : n], csum);
    }
  }
}

template <int BM, int BN, int BK, bool A_K, bool B_K, int AG, int BG>
hipError_t gemm_launch(const GemmParams& P, hipStream_t s) {
  const int tiles = ((P.d.M + BM - 1) / BM) * ((P.d.N + BN - 1) / BN);
  dim3 grid(tiles, 1, P.splits);
  gemm_kernel<BM, BN, BK, A_K, B_K, AG, BG><<<grid, 256, 0, s>>>(P);
  return hipGetLastError();
}

// dispatch over the supported (tile, bk) pairs for one operand family
template <bool A_K, bool B_K, int AG, int BG>
hipError_t gemm_dispatch_tiles(const GemmParams& P, hipStream_t s) {
  const int t = P.d.tile, bk = P.d.bk;
  if (bk == 64) {
    switch (t) {
      case 0: return gemm_launch<64, 64, 64, A_K, B_K, AG, BG>(P, s);
      case 1: return gemm_launch<32, 64, 64, A_K, B_K, AG, BG>(P, s);
      case 2: return gemm_launch<64, 32, 64, A_K, B_K, AG, BG>(P, s);
      case 3: return gemm_launch<128, 64, 64, A_K, B_K, AG, BG>(P, s);
      case 4: return gemm_launch<32, 32, 64, A_K, B_K, AG, BG>(P, s);
    }
  } else if (bk == 128) {
    switch (t) {
      case 0: return gemm_launch<64, 64, 128, A_K, B_K, AG, BG>(P, s);
      case 1: return gemm_launch<32, 64, 128, A_K, B_K, AG, BG>(P, s);
      case 2: return gemm_launch<64, 32, 128, A_K, B_K, AG, BG>(P, s);
      case 4: return gemm_launch<32, 32, 128, A_K, B_K, AG, BG>(P, s);
    }
  } else if (bk == 256) {
    if (t == 4) return gemm_launch<32, 32, 256, A_K, B_K, AG, BG>(P, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace aca
