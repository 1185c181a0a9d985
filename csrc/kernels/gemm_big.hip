// Large bf16 products on 128 x 128 tiles of the 32x32x16 MFMA with LDS-DMA staging (SURVEY §2.4 K01 / K02 at the
// PPO learner's batch: the Nature-CNN fc layer at B = 4096 rows against K or N = 3136 / 512).
//
//   C[M, N] = epilogue( alpha * A[M, K] . B[K, N] )       (operand storage as gemm_impl.h: A_K / B_K)
//
// Why a second GEMM: the general kernel (gemm_impl.h) keeps the small rollout products short with 4-wave 64 x 64 (or
// smaller) tiles and register-staged loads; at B = 4096 those tiles move 4x the operand bytes per MAC of a 128 x 128
// tile and ran the three fc products at 274-321 TF/s (the library reaches 550 on the forward). Here:
//   * 4 waves, each a 64 x 64 quarter of the 128 x 128 tile as 2 x 2 accumulators of v_mfma_f32_32x32x16_bf16
//     (16 MFMAs = 512 cycles per 64-deep k-step per wave);
//   * operand tiles copied global -> LDS by LDS-DMA (global_load_lds_dwordx4: no staging registers, no LDS store
//     instructions), 8 wave-instructions per wave per k-step, into a 3-stage ring: the loads of k-step kt + 2 are in
//     flight while kt is multiplied; ONE raw barrier per k-step behind a counted `s_waitcnt vmcnt(8)` (the newest
//     k-step's 8 copies stay in flight across it), no __syncthreads in the loop (its implicit vmcnt(0) would drain
//     the ring);
//   * conflict-free LDS images without padding (the DMA writes lane-linear 1 KB pieces, so the swizzle is applied to
//     the per-lane GLOBAL source address): k-contiguous tiles [128 rows][64 k] (128-byte rows) XOR the 16-byte chunk
//     index with (row >> 1) & 7 -- every ds_read_b128 lane group of a fragment read then covers 16 distinct 16-byte
//     bank slots --; m/n-contiguous tiles [64 k][128] (256-byte rows) XOR it with 4 (k & 3), which puts the four
//     k-rows of a ds_read_b64_tr_b16 group in four different 64-byte bank quarters;
//   * split-K over the grid: each split writes its fp32 partial tile to a slab, the last-arriving split (agent-scope
//     release / acquire ticket) sums the slabs in split order and runs the epilogue (deterministic).
// Epilogue: *alpha, +bias[n], relu, *(mask[m][n] > 0), store fp32 | bf16; or out_mode 3: each split stores its fp32
// partial tile into its own plane and the consumer reduces (no in-launch reduction).
// Requirements (host-checked): plain bf16 operands, 16-byte aligned, lda / ldb % 8 == 0, K % 64 == 0 (splits take
// ceil(K / 64 / splits) k-steps each, the last one the rest), the m/n-contiguous extents % 8 == 0.
#include "common.h"
#include "gemm_desc.h"

namespace aca {

constexpr int GB_BM = 128, GB_BN = 128, GB_BK = 64, GB_T = 256;
constexpr int GB_TILE = 128 * 64;                      // bf16 elements of one operand stage (16 KB)
// ring of ST stages + the last-arriver flag (one __shared__ array: a second object makes hipcc wait vmcnt(0) before
// ds_reads)
template <int ST>
constexpr int gb_lds() { return ST * 2 * GB_TILE + 64; }

typedef float gb_f32x16 __attribute__((ext_vector_type(16)));
typedef short gb_s4 __attribute__((ext_vector_type(4)));
typedef short gb_s8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) gb_s4 gb_lds_s4;

// LDS-DMA of one operand stage. KC: tile [128 rows][64 k], a 1 KB piece = 8 rows; lane -> (row, physical chunk),
// source = the logical chunk (physical ^ swizzle). MN: tile [64 k][128], a piece = 4 k-rows of 256 B. Rows past the
// matrix (`lim`) read the last valid row / column block (their outputs are never stored).
template <bool KC>
__device__ __forceinline__ void gb_stage(const u16* __restrict__ g, int64_t ld, int r0, int lim, int k0,
                                         u16* __restrict__ tile) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int piece = wid + 4 * u;
    const u16* src;
    if constexpr (KC) {
      const int r = piece * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ ((r >> 1) & 7);
      const int gr = min(r0 + r, lim - 1);
      src = g + (int64_t)gr * ld + k0 + lc * 8;
    } else {
      const int kr = piece * 4 + (lane >> 4);
      const int lc = (lane & 15) ^ (4 * (kr & 3));
      const int col = min(r0 + lc * 8, lim - 8);
      src = g + (int64_t)(k0 + kr) * ld + col;
    }
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(src),
                                     (__attribute__((address_space(3))) void*)(tile + piece * 512), 16, 0, 0);
  }
}

// 32 x 16 fragment (lane l: row / column base + (l & 31), k = 16 kk + 8 (l >> 5) + 0..7) of a k-contiguous tile
__device__ __forceinline__ bf16x8 gb_frag_kc(const u16* __restrict__ t, int base, int kk, int lane) {
  const int r = base + (lane & 31);
  const int pc = (2 * kk + (lane >> 5)) ^ ((r >> 1) & 7);
  return *reinterpret_cast<const bf16x8*>(t + r * 64 + pc * 8);
}

// the same fragment of an m/n-contiguous tile by two transposing reads (16-lane group gl: columns 16 (gl & 1) .. + 15,
// k half gl >> 1; lane 4q + p supplies k-row q of the 4-deep block, columns 4p .. 4p + 3)
__device__ __forceinline__ bf16x8 gb_frag_mn(const u16* __restrict__ t, int base, int kk, int lane) {
  const int gl = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = base + (gl & 1) * 16 + 4 * p, kb = kk * 16 + 8 * (gl >> 1);
  const int k_lo = kb + q, k_hi = kb + 4 + q;
  const u16* a_lo = t + k_lo * 128 + ((((col >> 3) ^ (4 * (k_lo & 3)))) << 3) + (col & 7);
  const u16* a_hi = t + k_hi * 128 + ((((col >> 3) ^ (4 * (k_hi & 3)))) << 3) + (col & 7);
  const gb_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((gb_lds_s4*)(a_lo));
  const gb_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((gb_lds_s4*)(a_hi));
  const gb_s8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

struct GbParams {
  AcaGemmDesc d;
  int tiles_n, splits, ksteps_per_split;
  int xcd;       // XCD-grouped workgroup order (grid % 8 == 0)
  int vec_epi;   // bf16 output staged through LDS, 16-byte mask loads / C stores (N, ldc, ldm % 8 == 0, aligned)
};

template <bool A_K, bool B_K, int ST>
__global__ void __launch_bounds__(GB_T) gemm_big_kernel(GbParams P) {
  __shared__ __attribute__((aligned(16))) u16 smem[gb_lds<ST>()];
  const AcaGemmDesc& d = P.d;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // diagnostics: [start, k-loop done, split reduce done, end, HW_ID, XCC_ID] per workgroup (vector stores)
  unsigned long long* st = d.stamps ? d.stamps + (size_t)blockIdx.x * 8 : nullptr;
  if (st && tid == 0) {
    st[0] = __builtin_amdgcn_s_memrealtime();
    st[4] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    st[5] = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20);
  }
  // workgroups are dealt round-robin over the 8 XCDs (each its own L2): give every XCD a contiguous run of tiles, so
  // the n-tiles sharing an A row block (and the splits of a tile) meet in one L2
  int bid = blockIdx.x;
  if (P.xcd) bid = (bid & 7) * (int)(gridDim.x >> 3) + (bid >> 3);
  const int tile = bid / P.splits, z = bid - tile * P.splits;
  const int m0 = (tile / P.tiles_n) * GB_BM, n0 = (tile % P.tiles_n) * GB_BN;
  const int ks0 = z * P.ksteps_per_split;
  const int nk = min(P.ksteps_per_split, d.K / GB_BK - ks0);
  const u16* Ag = reinterpret_cast<const u16*>(d.A);
  const u16* Bg = reinterpret_cast<const u16*>(d.B);
  auto stA = [&](int s) { return smem + s * 2 * GB_TILE; };
  auto stB = [&](int s) { return smem + s * 2 * GB_TILE + GB_TILE; };
  auto issue = [&](int kt) {
    const int s = kt % ST, k0 = (ks0 + kt) * GB_BK;
    gb_stage<A_K>(Ag, d.lda, m0, d.M, k0, stA(s));
    gb_stage<B_K>(Bg, d.ldb, n0, d.N, k0, stB(s));
  };
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
  gb_f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll
  for (int q = 0; q < ST - 1; ++q)
    if (q < nk) issue(q);
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's copies of k-step kt have landed (the newer k-steps' 8 each may still fly), every wave's LDS reads
    // of the stage the next issue overwrites are done; the barrier publishes both
    const int newer = min(ST - 2, nk - 1 - kt);
    if constexpr (ST >= 4) {
      if (newer >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (newer == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (ST == 3) {
      if (newer >= 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + ST - 1 < nk) issue(kt + ST - 1);
    const u16* ta = stA(kt % ST);
    const u16* tb = stB(kt % ST);
    // every fragment of the k-step requested before the first MFMA (the LDS reads of later 16-deep slices overlap
    // the MFMAs of earlier ones; the compiler counts lgkmcnt down slice by slice)
    bf16x8 af[GB_BK / 16][2], bfr[GB_BK / 16][2];
#pragma unroll
    for (int kk = 0; kk < GB_BK / 16; ++kk) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[kk][i] = A_K ? gb_frag_kc(ta, wm + 32 * i, kk, lane) : gb_frag_mn(ta, wm + 32 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[kk][j] = B_K ? gb_frag_kc(tb, wn + 32 * j, kk, lane) : gb_frag_mn(tb, wn + 32 * j, kk, lane);
    }
#pragma unroll
    for (int kk = 0; kk < GB_BK / 16; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
  }
  if (st && tid == 0) st[1] = __builtin_amdgcn_s_memrealtime();
  // ---------------------------------------------------------------- partial planes (out_mode 3): no reduction here
  if (d.out_mode == 3) {
    // split z stores its fp32 tile into plane z of C ([splits][M][ldc]); the consumer sums the planes in order
    // (the gradient finaliser, or the PPO head for the fc activations): no slab round trip, no agent-scope
    // release / acquire (an L2 write-back + invalidate per arrival on a multi-XCD part)
    float* Cz = reinterpret_cast<float*>(d.C) + (size_t)z * d.M * d.ldc;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + 32 * j + (lane & 31);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (m < d.M && n < d.N) Cz[(int64_t)m * d.ldc + n] = acc[i][j][r];
        }
    }
    if (st) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tid == 0) st[3] = __builtin_amdgcn_s_memrealtime();
    }
    return;
  }
  // ---------------------------------------------------------------- split-K: slabs + last arriver, in split order
  if (P.splits > 1) {
    float* slab = d.ws + ((size_t)tile * P.splits + z) * (GB_BM * GB_BN);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) slab[((i * 2 + j) * 16 + r) * GB_T + tid] = acc[i][j][r];
    int* flag = reinterpret_cast<int*>(smem + ST * 2 * GB_TILE);
    if (!last_block_arrival(&d.tickets[tile], P.splits, flag)) return;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int s = 0; s < P.splits; ++s) {
      const float* sl = d.ws + ((size_t)tile * P.splits + s) * (GB_BM * GB_BN);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] += sl[((i * 2 + j) * 16 + r) * GB_T + tid];
    }
  }
  if (st && tid == 0) st[2] = __builtin_amdgcn_s_memrealtime();
  // ---------------------------------------------------------------- epilogue
  const u16* mask = reinterpret_cast<const u16*>(d.mask);
  if (d.out_mode == 1 && P.vec_epi) {
    // bf16 tile staged through LDS ([128][136]: the two 32-lane halves of a ds_write_b16 land in disjoint banks,
    // every 16-lane ds_read_b128 phase reads one conflict-free 256-byte row), then whole 16-byte mask loads and C
    // stores (8 per thread instead of 64 two-byte ones: full cache lines)
    constexpr int LDC = GB_BN + 8;
    const int er = tid >> 4, ec = (tid & 15) * 8;
    uint4 mv[8];
    if (mask) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {   // issued first: their latency hides behind the LDS staging
        const int m = min(m0 + q * 16 + er, d.M - 1), n = min(n0 + ec, d.N - 8);
        mv[q] = *reinterpret_cast<const uint4*>(mask + (int64_t)m * d.ldm + n);
      }
    }
    float bv[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) bv[j] = d.bias ? d.bias[min(n0 + wn + 32 * j + (lane & 31), d.N - 1)] : 0.f;
    __syncthreads();   // every wave is past its last ring read
    u16* sc = smem;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[i][j][r] * d.alpha + bv[j];
          if (d.relu) v = fmaxf(v, 0.f);
          const int row = wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          sc[row * LDC + wn + 32 * j + (lane & 31)] = f2bf(v);
        }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int row = q * 16 + er, m = m0 + row, n = n0 + ec;
      uint4 v = *reinterpret_cast<const uint4*>(sc + row * LDC + ec);
      if (mask) {
        uint32_t* w = reinterpret_cast<uint32_t*>(&v);
        const uint32_t* mw = reinterpret_cast<const uint32_t*>(&mv[q]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t lo = (mw[e] << 16), hi = (mw[e] & 0xFFFF0000u);
          const uint32_t keep = (__uint_as_float(lo) > 0.f ? 0x0000FFFFu : 0u) | (__uint_as_float(hi) > 0.f ? 0xFFFF0000u : 0u);
          w[e] &= keep;
        }
      }
      if (m < d.M && n < d.N) *reinterpret_cast<uint4*>(reinterpret_cast<u16*>(d.C) + (int64_t)m * d.ldc + n) = v;
    }
    if (st) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tid == 0) st[3] = __builtin_amdgcn_s_memrealtime();
    }
    return;
  }
  // bias and mask operands fetched for every output of this thread up front, from clamped (always valid) addresses:
  // a guarded load per output would be one dependent memory round trip each
  float bv[2];
  u16 mk[2][2][16];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = min(n0 + wn + 32 * j + (lane & 31), d.N - 1);
    bv[j] = d.bias ? d.bias[n] : 0.f;
    if (mask) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = min(m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), d.M - 1);
          mk[i][j][r] = mask[(int64_t)m * d.ldm + n];
        }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn + 32 * j + (lane & 31);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        float v = acc[i][j][r] * d.alpha + bv[j];
        if (d.relu) v = fmaxf(v, 0.f);
        if (mask && !(bf2f(mk[i][j][r]) > 0.f)) v = 0.f;
        if (m < d.M && n < d.N) {
          if (d.out_mode == 1) reinterpret_cast<u16*>(d.C)[(int64_t)m * d.ldc + n] = f2bf(v);
          else reinterpret_cast<float*>(d.C)[(int64_t)m * d.ldc + n] = v;
        }
      }
    }
  }
  if (st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) st[3] = __builtin_amdgcn_s_memrealtime();
  }
}

}  // namespace aca

using namespace aca;

// workspace floats / tickets a split-K launch of this shape needs (0 when splits == 1)
extern "C" int64_t aca_gemm_big_ws(int M, int N, int splits) {
  if (splits <= 1) return 0;
  const int64_t tiles = (int64_t)((M + GB_BM - 1) / GB_BM) * ((N + GB_BN - 1) / GB_BN);
  return tiles * splits * GB_BM * GB_BN;
}

extern "C" hipError_t aca_gemm_big(const AcaGemmDesc* d, hipStream_t stream) {
  if (d->M <= 0 || d->N <= 0) return hipSuccess;
  if (d->ga.mode || d->gb.mode || d->colsum || d->colsum_part) return hipErrorInvalidValue;
  if (d->out_mode != 0 && d->out_mode != 1 && d->out_mode != 3) return hipErrorInvalidValue;
  if (d->out_mode == 3 && (d->bias || d->relu || d->mask || d->alpha != 1.0f)) return hipErrorInvalidValue;
  const int splits = d->splits < 1 ? 1 : d->splits;
  const int ksteps = d->K / GB_BK;
  const int per = (ksteps + splits - 1) / splits;   // the last split may be shorter; every split gets >= 1 k-step
  if (d->K % GB_BK || ksteps < 1 || per * (splits - 1) >= ksteps) return hipErrorInvalidValue;
  if ((d->lda % 8) || (d->ldb % 8) || (reinterpret_cast<uintptr_t>(d->A) % 16) ||
      (reinterpret_cast<uintptr_t>(d->B) % 16))
    return hipErrorInvalidValue;
  if ((!d->a_k && d->M % 8) || (!d->b_k && d->N % 8)) return hipErrorInvalidValue;
  if (splits > 1 && d->out_mode != 3 && (!d->ws || !d->tickets)) return hipErrorInvalidValue;
  GbParams P;
  P.d = *d;
  P.tiles_n = (d->N + GB_BN - 1) / GB_BN;
  P.splits = splits;
  P.ksteps_per_split = per;
  const int tiles = ((d->M + GB_BM - 1) / GB_BM) * P.tiles_n;
  const dim3 grid(tiles * splits);
  // d->tile: variant bits (bit 0 XCD-grouped order, bits 1-2 ring depth - 2, bit 3 scalar bf16 epilogue)
  P.xcd = (d->tile & 1) && (grid.x % 8 == 0);
  P.vec_epi = d->out_mode == 1 && d->N % 8 == 0 && d->ldc % 8 == 0 && reinterpret_cast<uintptr_t>(d->C) % 16 == 0 &&
              (!d->mask || (d->ldm % 8 == 0 && reinterpret_cast<uintptr_t>(d->mask) % 16 == 0)) && !(d->tile & 8);
  const int st = 2 + ((d->tile >> 1) & 3);
#define GB_LAUNCH(S)                                                                        \
  if (d->a_k && d->b_k) gemm_big_kernel<true, true, S><<<grid, GB_T, 0, stream>>>(P);       \
  else if (d->a_k) gemm_big_kernel<true, false, S><<<grid, GB_T, 0, stream>>>(P);           \
  else if (d->b_k) gemm_big_kernel<false, true, S><<<grid, GB_T, 0, stream>>>(P);           \
  else gemm_big_kernel<false, false, S><<<grid, GB_T, 0, stream>>>(P);
  if (st == 2) { GB_LAUNCH(2) }
  else if (st == 3) { GB_LAUNCH(3) }
  else { GB_LAUNCH(4) }
#undef GB_LAUNCH
  return hipGetLastError();
}
