// Large-shape bf16 GEMM on the 32x32x16 MFMA (PPO minibatch products of the Nature-CNN fc layer: M = 4096 rows
// against K or N = 3136 / 512; SURVEY §2.4 K01/K02 at BASELINE config 3).
//
//   C[M, N] = epilogue( alpha * A[M, K] . B[K, N] )     (operand storage as gemm_impl.h: A_K / B_K)
//
// The general GEMM (gemm_impl.h, 4 waves, 16x16x32 MFMA) keeps small rollout products short; at these sizes the
// 32x32x16 MFMA moves twice the MACs per operand byte read from LDS, so this kernel uses it with 8 waves per
// 128 x 128 tile (wave tile 32 x 64: one A fragment and two B fragments per 16-deep k-step, 2 MFMAs), a 64-deep
// k-step staged through double-buffered LDS with the next step's global loads in flight in registers (one barrier
// per k-step). k-contiguous operands are stored [row][k] in LDS and read with ds_read_b128; m/n-contiguous ones are
// stored [k][row] and read with the transposing ds_read_b64_tr_b16 -- no element-wise transpose anywhere.
// Epilogue: *alpha, +bias[n], relu, *(mask[m][n] > 0), store fp32 / bf16, or (out_mode 3) fp32 split-K partial
// plane z of C[z][M][ldc] (reduced in plane order by the consumer: deterministic, no atomics).
// Requirements (host-checked): 16-byte aligned operands, lda / ldb % 8 == 0, K % 64 == 0 per split.
#include "common.h"
#include "gemm_desc.h"

namespace aca {

typedef float g32_floatx16 __attribute__((ext_vector_type(16)));
typedef short g32_short4 __attribute__((ext_vector_type(4)));
typedef short g32_short8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) g32_short4 g32_lds4;

constexpr int G32_BN = 128, G32_BK = 64;
constexpr int G32_KLD = G32_BK + 8;     // [row][k] LDS row (k-contiguous operand), 144 B: the 16 rows a b128 read
                                        // group touches start 36 dwords apart -> 64 distinct banks
constexpr int G32_MLD = 128 + 32;       // [k][row] LDS row (m/n-contiguous operand), 320 B = 80 dwords: the four
                                        // rows of a transposing read start 16 banks apart -> no overlap
constexpr int G32_TILE_E = 128 * G32_KLD > G32_BK * G32_MLD ? 128 * G32_KLD : G32_BK * G32_MLD;

struct G32Params {
  const u16* A;
  const u16* B;
  void* C;
  const float* bias;
  const u16* mask;
  int64_t lda, ldb, ldc, ldm;
  int M, N, K;
  int k_per_split;   // multiple of G32_BK
  int out_mode;      // 0 fp32, 1 bf16, 3 fp32 planes (one per split)
  int relu;
  float alpha;
};

// one 16-byte chunk of an operand tile (zero outside the matrix)
__device__ __forceinline__ uint4 g32_load(const u16* base, int64_t ld, int r, int c, int rlim, int clim) {
  if (r < rlim && c < clim) return *reinterpret_cast<const uint4*>(base + (int64_t)r * ld + c);
  return make_uint4(0u, 0u, 0u, 0u);
}

// fragment (8 bf16) of a 32-row operand tile for lanes (row l & 31, k 8 (l >> 5) + 0..7):
// KC: tile stored [row][k] -> one ds_read_b128; else stored [k][row] -> two transposing reads
template <bool KC>
__device__ __forceinline__ bf16x8 g32_frag(const u16* tile, int row0, int k0, int lane) {
  if constexpr (KC) {
    const u16* p = tile + (row0 + (lane & 31)) * G32_KLD + k0 + 8 * (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    // 16-lane group gl covers rows row0 + 16 (gl & 1) .. + 15 and k half 8 (gl >> 1); lane 4q + p supplies row q
    // of the 4-deep block, columns 4p .. 4p + 3
    const int gl = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int col = row0 + (gl & 1) * 16 + 4 * p, kb = k0 + 8 * (gl >> 1);
    const g32_short4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((g32_lds4*)(tile + (kb + q) * G32_MLD + col));
    const g32_short4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((g32_lds4*)(tile + (kb + 4 + q) * G32_MLD + col));
    const g32_short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// BM = 128 (8 waves) or 64 (4 waves): wave w owns rows 32 (w % (BM / 32)) .. + 31 and columns 64 (w / (BM / 32))
// .. + 63 of the BM x 128 tile. The 64-row form doubles the workgroups of products with few 128 x 128 tiles.
template <bool A_K, bool B_K, int BM>
__global__ void __launch_bounds__(BM * 4) gemm_mfma32_kernel(G32Params p) {
  constexpr int G32_T = BM * 4;                    // threads
  constexpr int CA = BM * G32_BK / 8 / G32_T;      // A staging chunks per thread (2)
  constexpr int CB = G32_BN * G32_BK / 8 / G32_T;  // B staging chunks per thread (2 | 4)
  constexpr int WM = BM / 32;                      // waves along m
  __shared__ __attribute__((aligned(16))) u16 s_a[2][G32_TILE_E];
  __shared__ __attribute__((aligned(16))) u16 s_b[2][G32_TILE_E];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * G32_BN, z = blockIdx.z;
  const int kbeg = z * p.k_per_split, kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg) / G32_BK;
  // staging: 16-byte chunks; k-contiguous [row][k] tile: chunk c -> row c >> 3, k 8 (c & 7); m/n-contiguous
  // [k][row] tile: k c / (rows / 8), row 8 (c % (rows / 8)). The next k-step's chunks wait in registers.
  uint4 ra[CA], rb[CB];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < CA; ++u) {
      const int c = tid + u * G32_T;
      if (A_K) ra[u] = g32_load(p.A, p.lda, m0 + (c >> 3), k0 + 8 * (c & 7), p.M, p.K);
      else ra[u] = g32_load(p.A, p.lda, k0 + c / (BM / 8), m0 + 8 * (c % (BM / 8)), p.K, p.M);
    }
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const int c = tid + u * G32_T;
      if (B_K) rb[u] = g32_load(p.B, p.ldb, n0 + (c >> 3), k0 + 8 * (c & 7), p.N, p.K);
      else rb[u] = g32_load(p.B, p.ldb, k0 + (c >> 4), n0 + 8 * (c & 15), p.K, p.N);
    }
  };
  auto store = [&](int buf) {
    u16* ta = s_a[buf];
    u16* tb = s_b[buf];
#pragma unroll
    for (int u = 0; u < CA; ++u) {
      const int c = tid + u * G32_T;
      if (A_K) *reinterpret_cast<uint4*>(ta + (c >> 3) * G32_KLD + 8 * (c & 7)) = ra[u];
      else *reinterpret_cast<uint4*>(ta + (c / (BM / 8)) * G32_MLD + 8 * (c % (BM / 8))) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const int c = tid + u * G32_T;
      if (B_K) *reinterpret_cast<uint4*>(tb + (c >> 3) * G32_KLD + 8 * (c & 7)) = rb[u];
      else *reinterpret_cast<uint4*>(tb + (c >> 4) * G32_MLD + 8 * (c & 15)) = rb[u];
    }
  };
  // wave tile: rows wm .. wm + 31 (one 32-row A fragment), columns wn .. wn + 63 (two 32-column B fragments)
  const int wm = (wid % WM) * 32, wn = (wid / WM) * 64;
  g32_floatx16 acc0, acc1;
#pragma unroll
  for (int i = 0; i < 16; ++i) { acc0[i] = 0.f; acc1[i] = 0.f; }
  if (nk > 0) {
    load(kbeg);
    store(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load(kbeg + (kt + 1) * G32_BK);   // in flight while this k-step multiplies
    const u16* ta = s_a[cur];
    const u16* tb = s_b[cur];
#pragma unroll
    for (int kk = 0; kk < G32_BK; kk += 16) {
      const bf16x8 a = g32_frag<A_K>(ta, wm, kk, lane);
      const bf16x8 b0 = g32_frag<B_K>(tb, wn, kk, lane);
      const bf16x8 b1 = g32_frag<B_K>(tb, wn + 32, kk, lane);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b1, acc1, 0, 0, 0);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }
  // epilogue: acc register i of lane l is C[wm + (i & 3) + 8 (i >> 2) + 4 (l >> 5)][wn + (l & 31)] (+32 for acc1)
  const int col = lane & 31, rh = 4 * (lane >> 5);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn + 32 * j + col;
    if (n >= p.N) continue;
    const float bv = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = m0 + wm + (i & 3) + 8 * (i >> 2) + rh;
      if (m >= p.M) continue;
      float v = (j == 0 ? acc0[i] : acc1[i]) * p.alpha;
      if (p.out_mode == 3) {
        reinterpret_cast<float*>(p.C)[((int64_t)z * p.M + m) * p.ldc + n] = v;
        continue;
      }
      v += bv;
      if (p.relu) v = fmaxf(v, 0.f);
      if (p.mask && !(bf2f(p.mask[(int64_t)m * p.ldm + n]) > 0.f)) v = 0.f;
      if (p.out_mode == 1) reinterpret_cast<u16*>(p.C)[(int64_t)m * p.ldc + n] = f2bf(v);
      else reinterpret_cast<float*>(p.C)[(int64_t)m * p.ldc + n] = v;
    }
  }
}

}  // namespace aca

using namespace aca;

// splits: split-K count (out_mode 3: one partial plane per split; out_modes 0 / 1 need splits == 1). Returns
// hipErrorInvalidValue for shapes / layouts this kernel does not take (the caller uses the general GEMM).
extern "C" hipError_t aca_gemm_mfma32(const AcaGemmDesc* d, hipStream_t stream) {
  if (d->M <= 0 || d->N <= 0) return hipSuccess;
  if (d->ga.mode || d->gb.mode || d->colsum || d->colsum_part) return hipErrorInvalidValue;
  if (d->out_mode != 0 && d->out_mode != 1 && d->out_mode != 3) return hipErrorInvalidValue;
  const int splits = d->splits < 1 ? 1 : d->splits;
  if (splits > 1 && d->out_mode != 3) return hipErrorInvalidValue;
  if (d->out_mode == 3 && (d->bias || d->relu || d->mask)) return hipErrorInvalidValue;
  if (d->K % (G32_BK * splits)) return hipErrorInvalidValue;
  if ((d->lda % 8) || (d->ldb % 8) || (reinterpret_cast<uintptr_t>(d->A) % 16) ||
      (reinterpret_cast<uintptr_t>(d->B) % 16))
    return hipErrorInvalidValue;
  // the staging chunks of a tile must be wholly inside or outside the matrix along the contiguous dimension
  if ((d->a_k ? d->K : d->M) % 8 || (d->b_k ? d->K : d->N) % 8) return hipErrorInvalidValue;
  G32Params p;
  p.A = reinterpret_cast<const u16*>(d->A);
  p.B = reinterpret_cast<const u16*>(d->B);
  p.C = d->C;
  p.bias = d->bias;
  p.mask = reinterpret_cast<const u16*>(d->mask);
  p.lda = d->lda; p.ldb = d->ldb; p.ldc = d->ldc; p.ldm = d->ldm;
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.k_per_split = d->K / splits;
  p.out_mode = d->out_mode;
  p.relu = d->relu;
  p.alpha = d->alpha;
  // 64-row tiles when 128 x 128 tiles would leave CUs idle (fewer than 256 workgroups)
  const int tn = (d->N + G32_BN - 1) / G32_BN;
  const bool small = (int64_t)((d->M + 127) / 128) * tn * splits < 256;
  const int bm = small ? 64 : 128;
  dim3 grid((d->M + bm - 1) / bm, tn, splits);
#define G32_LAUNCH(AK, BK_)                                                                              \
  if (small) gemm_mfma32_kernel<AK, BK_, 64><<<grid, 256, 0, stream>>>(p);                               \
  else gemm_mfma32_kernel<AK, BK_, 128><<<grid, 512, 0, stream>>>(p);
  if (d->a_k && d->b_k) { G32_LAUNCH(true, true) }
  else if (d->a_k) { G32_LAUNCH(true, false) }
  else if (d->b_k) { G32_LAUNCH(false, true) }
  else { G32_LAUNCH(false, false) }
#undef G32_LAUNCH
  return hipGetLastError();
}
