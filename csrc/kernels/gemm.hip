// bf16 MFMA GEMM with fused epilogues -- the workhorse behind every dense / conv forward and backward product of
// the engine.
//
//   C[M, N] = epilogue( alpha * A[M, K] . B[K, N] )
//
// Operands are bf16, accumulation fp32 on v_mfma_f32_16x16x32_bf16. Each operand may be stored either way round:
//   A_K = true : A stored [M][K] (k contiguous)      A_K = false: A stored [K][M] (m contiguous)
//   B_K = true : B stored [N][K] (k contiguous)      B_K = false: B stored [K][N] (n contiguous)
// Global->LDS staging always copies 16-byte rows in the operand's natural orientation; k-contiguous tiles feed the
// MFMA through ds_read_b128, m/n-contiguous tiles through the gfx950 transposing read ds_read_b64_tr_b16, so no
// operand is ever transposed in memory or element-by-element.
//
// Workgroup = 256 threads = 4 waves in a 2x2 arrangement; tile BM x BN x 64, LDS double-buffered with register
// prefetch (one barrier per k-tile). Split-K over gridDim.z in two flavours:
//   * atomic: every split adds alpha*acc into fp32 C (C pre-zeroed: the engine zeroes the gradient slab once per
//     learner step) -- used for weight gradients, whose reduction dimension is the batch (up to 64k rows);
//   * slab:   every split writes its fp32 partial tile to a workspace slab, the last-arriving split (agent-scope
//     release/acquire ticket, Guideline 16) sums the slabs in split order and runs the full epilogue --
//     deterministic, used for skinny forward GEMMs (M = 32 rollout rows against K = 3136).
// Epilogue (in order): *alpha, +bias[n], relu, *(mask[m,n] > 0) (ReLU backward), store fp32 | bf16 | atomic-add
// fp32, and optional column sums of the final values atomically added to colsum[n] (bias gradients).
#include "common.h"

namespace aca {

typedef short short4v __attribute__((ext_vector_type(4)));

struct GemmArgs {
  const u16* A;
  const u16* B;
  void* C;
  const float* bias;
  const u16* mask;
  float* colsum;
  float* ws;               // slab split-K workspace
  unsigned int* tickets;   // one per output tile, zero-initialised, self-cleaning
  int64_t lda, ldb, ldc, ldm;
  int M, N, K;
  int k_tiles_per_split;
  int splits;
  float alpha;
  int relu;
  int out_mode;            // 0 fp32 store, 1 bf16 store, 2 fp32 atomic add
  int colsum_mod;          // >0: colsum index = n % colsum_mod (per-channel sums of an NHWC-flattened matrix)
};

constexpr int BK = 64;
constexpr int PAD = 8;  // 16 bytes

template <int BM, int BN, bool A_K, bool B_K>
struct GemmSmem {
  // A image: A_K ? [BM][BK+PAD] : [BK][BM+PAD]; same for B
  static constexpr int A_ELEMS = A_K ? BM * (BK + PAD) : BK * (BM + PAD);
  static constexpr int B_ELEMS = B_K ? BN * (BK + PAD) : BK * (BN + PAD);
};

// load 8 contiguous bf16 starting at p (element index `idx` along the contiguous dim, valid if idx+8 <= lim)
__device__ __forceinline__ uint4 load8(const u16* base, int64_t row_off, int idx, int lim, bool row_ok) {
  uint4 r = make_uint4(0, 0, 0, 0);
  if (!row_ok) return r;
  const u16* p = base + row_off + idx;
  if (idx + 8 <= lim && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
    r = *reinterpret_cast<const uint4*>(p);
  } else {
    u16 tmp[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) tmp[j] = (idx + j < lim) ? p[j] : (u16)0;
    r.x = tmp[0] | ((uint32_t)tmp[1] << 16);
    r.y = tmp[2] | ((uint32_t)tmp[3] << 16);
    r.z = tmp[4] | ((uint32_t)tmp[5] << 16);
    r.w = tmp[6] | ((uint32_t)tmp[7] << 16);
  }
  return r;
}

template <int BM, int BN, bool A_K, bool B_K>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs g) {
  using S = GemmSmem<BM, BN, A_K, B_K>;
  constexpr int TM = BM / 32, TN = BN / 32;          // 16x16 MFMA tiles per wave
  constexpr int A_CHUNKS = BM * BK / 8 / 256;         // 16-byte chunks per thread per tile
  constexpr int B_CHUNKS = BN * BK / 8 / 256;
  static_assert(A_CHUNKS >= 1 && B_CHUNKS >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) u16 smem[2 * (S::A_ELEMS + S::B_ELEMS)];
  __shared__ int sh_flag;
  u16* const As0 = smem;
  u16* const Bs0 = smem + 2 * S::A_ELEMS;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int tile = blockIdx.x;
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int z = blockIdx.z;
  const int k_tiles_total = (g.K + BK - 1) / BK;
  const int kt0 = z * g.k_tiles_per_split;
  const int kt1 = min(kt0 + g.k_tiles_per_split, k_tiles_total);

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
        ra[c] = load8(g.A, (int64_t)m * g.lda, k0 + kc, g.K, m < g.M);
      } else {
        const int kr = ch / (BM / 8), mc = (ch % (BM / 8)) * 8;
        const int k = k0 + kr;
        ra[c] = load8(g.A, (int64_t)k * g.lda, m0 + mc, g.M, k < g.K);
      }
    }
#pragma unroll
    for (int c = 0; c < B_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      if (B_K) {
        const int r = ch / (BK / 8), kc = (ch % (BK / 8)) * 8;
        const int n = n0 + r;
        rb[c] = load8(g.B, (int64_t)n * g.ldb, k0 + kc, g.K, n < g.N);
      } else {
        const int kr = ch / (BN / 8), nc = (ch % (BN / 8)) * 8;
        const int k = k0 + kr;
        rb[c] = load8(g.B, (int64_t)k * g.ldb, n0 + nc, g.N, k < g.K);
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int c = 0; c < A_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      int off;
      if (A_K) off = (ch / (BK / 8)) * (BK + PAD) + (ch % (BK / 8)) * 8;
      else off = (ch / (BM / 8)) * (BM + PAD) + (ch % (BM / 8)) * 8;
      *reinterpret_cast<uint4*>(As0 + buf * S::A_ELEMS + off) = ra[c];
    }
#pragma unroll
    for (int c = 0; c < B_CHUNKS; ++c) {
      const int ch = tid + c * 256;
      int off;
      if (B_K) off = (ch / (BK / 8)) * (BK + PAD) + (ch % (BK / 8)) * 8;
      else off = (ch / (BN / 8)) * (BN + PAD) + (ch % (BN / 8)) * 8;
      *reinterpret_cast<uint4*>(Bs0 + buf * S::B_ELEMS + off) = rb[c];
    }
  };

  const int lr16 = lane & 15, lg = lane >> 4;   // row-in-tile, k-group
  const int q = lr16 >> 2, p = lr16 & 3;        // transposed-read address roles

  auto frag_a = [&](const u16* as, int i, int ks) -> bf16x8 {
    const int mrow = wm * (BM / 2) + i * 16;
    if (A_K) {
      return *reinterpret_cast<const bf16x8*>(as + (mrow + lr16) * (BK + PAD) + ks * 32 + lg * 8);
    } else {
      const int kb = ks * 32 + lg * 8;
      typedef __attribute__((address_space(3))) short4v lds_s4;
      const u16* p0 = as + (kb + q) * (BM + PAD) + mrow + 4 * p;
      const u16* p1 = as + (kb + 4 + q) * (BM + PAD) + mrow + 4 * p;
      short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p0));
      short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p1));
      short __attribute__((ext_vector_type(8))) v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  };
  auto frag_b = [&](const u16* bs, int j, int ks) -> bf16x8 {
    const int ncol = wn * (BN / 2) + j * 16;
    if (B_K) {
      return *reinterpret_cast<const bf16x8*>(bs + (ncol + lr16) * (BK + PAD) + ks * 32 + lg * 8);
    } else {
      const int kb = ks * 32 + lg * 8;
      typedef __attribute__((address_space(3))) short4v lds_s4;
      const u16* p0 = bs + (kb + q) * (BN + PAD) + ncol + 4 * p;
      const u16* p1 = bs + (kb + 4 + q) * (BN + PAD) + ncol + 4 * p;
      short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p0));
      short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p1));
      short __attribute__((ext_vector_type(8))) v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
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
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag_a(As0 + buf * S::A_ELEMS, i, ks);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag_b(Bs0 + buf * S::B_ELEMS, j, ks);
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

  // ---------------------------------------------------------------- split-K reduction
  if (g.splits > 1 && g.out_mode != 2) {
    float* slab = g.ws + ((size_t)tile * g.splits + z) * (BM * BN);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[((i * TN + j) * 4 + r) * 256 + tid] = acc[i][j][r];
    if (!last_block_arrival(&g.tickets[tile], g.splits, &sh_flag)) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < g.splits; ++s) {
      const float* sl = g.ws + ((size_t)tile * g.splits + s) * (BM * BN);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += sl[((i * TN + j) * 4 + r) * 256 + tid];
    }
  }

  // ---------------------------------------------------------------- epilogue
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
        if (g.mask) v = (bf2f(g.mask[(int64_t)m * g.ldm + n]) > 0.f) ? v : 0.f;
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

template <int BM, int BN, bool A_K, bool B_K>
static hipError_t launch_t(const GemmArgs& g, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  dim3 grid(tiles, 1, g.splits);
  gemm_kernel<BM, BN, A_K, B_K><<<grid, 256, 0, s>>>(g);
  return hipGetLastError();
}

template <int BM, int BN>
static hipError_t launch_layout(const GemmArgs& g, bool a_k, bool b_k, hipStream_t s) {
  if (a_k && b_k) return launch_t<BM, BN, true, true>(g, s);
  if (a_k && !b_k) return launch_t<BM, BN, true, false>(g, s);
  if (!a_k && b_k) return launch_t<BM, BN, false, true>(g, s);
  return launch_t<BM, BN, false, false>(g, s);
}

}  // namespace aca

using namespace aca;

// tile: 0 -> 64x64, 1 -> 32x64, 2 -> 64x32, 3 -> 128x64, 4 -> 32x32
extern "C" hipError_t aca_gemm(const void* A, int64_t lda, bool a_kcontig, const void* B, int64_t ldb,
                               bool b_kcontig, void* C, int64_t ldc, int out_mode, int M, int N, int K, float alpha,
                               const float* bias, int relu, const void* mask, int64_t ldm, float* colsum, int tile,
                               int splits, float* ws, unsigned int* tickets, int colsum_mod, hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  GemmArgs g;
  g.A = (const u16*)A; g.B = (const u16*)B; g.C = C; g.bias = bias; g.mask = (const u16*)mask; g.colsum = colsum;
  g.ws = ws; g.tickets = tickets; g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldm = ldm; g.M = M; g.N = N; g.K = K;
  const int kt = (K + BK - 1) / BK;
  if (splits < 1) splits = 1;
  if (splits > kt) splits = kt > 0 ? kt : 1;
  g.k_tiles_per_split = (kt + splits - 1) / splits;
  // recompute the effective split count so that no split is empty
  g.splits = kt > 0 ? (kt + g.k_tiles_per_split - 1) / g.k_tiles_per_split : 1;
  g.alpha = alpha; g.relu = relu; g.out_mode = out_mode; g.colsum_mod = colsum_mod;
  if (g.splits > 1 && out_mode != 2 && (ws == nullptr || tickets == nullptr)) return hipErrorInvalidValue;
  switch (tile) {
    case 1: return launch_layout<32, 64>(g, a_kcontig, b_kcontig, stream);
    case 2: return launch_layout<64, 32>(g, a_kcontig, b_kcontig, stream);
    case 3: return launch_layout<128, 64>(g, a_kcontig, b_kcontig, stream);
    case 4: return launch_layout<32, 32>(g, a_kcontig, b_kcontig, stream);
    default: return launch_layout<64, 64>(g, a_kcontig, b_kcontig, stream);
  }
}

// effective split count actually launched (the host needs it to size the slab workspace)
extern "C" int aca_gemm_effective_splits(int K, int splits) {
  const int kt = (K + BK - 1) / BK;
  if (splits < 1) splits = 1;
  if (splits > kt) splits = kt > 0 ? kt : 1;
  const int per = (kt + splits - 1) / splits;
  return kt > 0 ? (kt + per - 1) / per : 1;
}

extern "C" int aca_gemm_tile_dims(int tile, int* bm, int* bn) {
  switch (tile) {
    case 1: *bm = 32; *bn = 64; break;
    case 2: *bm = 64; *bn = 32; break;
    case 3: *bm = 128; *bn = 64; break;
    case 4: *bm = 32; *bn = 32; break;
    default: *bm = 64; *bn = 64; break;
  }
  return 0;
}
