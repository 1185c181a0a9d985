// Rollout fc product of the Nature-CNN (SURVEY §2.4 K01 at the headline's rollout batch): the fc layer's split-K
// partial planes  P[s][m][n] = sum_{k in chunk s} X[m][k] * W[k][n]  for the M <= 128 envs of one rollout step
// (X = y3 [M, 3136] bf16, W = Wfc [3136, 512]), consumed by the fused rollout step / the A2C head, which sum the
// planes in plane order, add the bias and apply ReLU (cnn_head.h).
//
// Why not the general GEMM (gemm_impl.h, 5.0 us per launch at this shape): its 32 x 32 tiles stream W through LDS
// as 64-byte row pieces (16 rows per wave instruction: ~16 B/clk/CU from L2 against 50-60 for whole-line wave loads,
// profiles/r4_l2_stream_probe.txt) and walk 4 dependent k-steps of load -> LDS -> barrier -> transposing read ->
// MFMA. Here W is read from a FRAGMENT-ORDERED bf16 copy kept by the optimiser step (ops/optim.py frag_order_kc):
// the 32x32x16 MFMA's B fragment of (16-deep k block kb, 32-wide column block nb) is 1 KB contiguous --
//     u16 index  ((kb * N/32 + nb) * 64 + (k / 8 % 2) * 32 + n % 32) * 8 + k % 8
// -- so every operand goes global -> VGPRs in ONE round of loads (no LDS staging, no barrier before the MFMAs):
// each wave issues its KR A fragments (16 bytes of an X row per lane) and KR B fragments (1 KB wave loads) at once,
// runs KR MFMAs, and the W waves of a workgroup (consecutive k ranges of one 32-column block) sum their
// accumulators through LDS in wave order into ONE plane: S = (K/16) / (KR * W) planes, fixed summation order
// (deterministic), no atomics, no in-launch cross-workgroup hand-off.
// Workgroup order is XCD-grouped: the 16 column blocks of a k chunk run on one XCD, so their shared X lines meet in
// one L2; the same workgroup reads the same W fragments every launch (they stay in that XCD's L2 across steps).
#include "common.h"

namespace aca {

typedef float fr_f32x16 __attribute__((ext_vector_type(16)));

struct FcRolloutArgs {
  const u16* X; int64_t ldx; int M;
  const u16* Wf; int K, N;
  float* P; int64_t pstride;
  unsigned long long* stamps;   // diagnostics: per wave [entry, operands landed, MFMAs done, stores drained]
};

template <int KR, int W, int MT>
__global__ void __launch_bounds__(64 * W) fc_rollout_kernel(FcRolloutArgs a) {
  __shared__ float red[W > 1 ? W * 16 * 64 : 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  unsigned long long* st = a.stamps ? a.stamps + ((size_t)blockIdx.x * W + w) * 4 : nullptr;
  if (st && lane == 0) st[0] = __builtin_amdgcn_s_memrealtime();
  const int NB = a.N >> 5;
  // XCD-grouped order: workgroups are dealt round-robin over the 8 XCDs; logical index L runs contiguously per XCD
  const int G = gridDim.x, bid = blockIdx.x;
  const int L = (G & 7) ? bid : (bid & 7) * (G >> 3) + (bid >> 3);
  const int s = L / NB, nb = L - s * NB;
  const int kb0 = (s * W + w) * KR;
  // MT 32-row blocks of X (rows past M read row M - 1, never stored); the B fragments are shared by all of them
  const u16* wb = a.Wf + ((int64_t)kb0 * NB + nb) * 512 + lane * 8;
  // gridDim.y > 1: the 32-row blocks are split over workgroups instead (MT == 1; B fragments re-read per block)
  const int m0 = blockIdx.y * 32;
  bf16x8 af[MT][KR], bf[KR];
#pragma unroll
  for (int q = 0; q < KR; ++q) bf[q] = *reinterpret_cast<const bf16x8*>(wb + (int64_t)q * NB * 512);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = min(m0 + mt * 32 + (lane & 31), a.M - 1);
    const u16* xa = a.X + (int64_t)m * a.ldx + kb0 * 16 + 8 * (lane >> 5);
#pragma unroll
    for (int q = 0; q < KR; ++q) af[mt][q] = *reinterpret_cast<const bf16x8*>(xa + q * 16);
  }
  fr_f32x16 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[mt][r] = 0.f;
  if (st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) st[1] = __builtin_amdgcn_s_memrealtime();
  }
#pragma unroll
  for (int q = 0; q < KR; ++q)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mt][q], bf[q], acc[mt], 0, 0, 0);
  if (st && lane == 0) st[2] = __builtin_amdgcn_s_memrealtime() + (unsigned long long)(acc[0][0] != acc[0][0]);
  float* plane = a.P + (int64_t)s * a.pstride + (int64_t)m0 * a.N + nb * 32 + (lane & 31);
  const int mr = 4 * (lane >> 5);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    if (m0 + mt * 32 >= a.M) break;
    if constexpr (W == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = mt * 32 + (r & 3) + 8 * (r >> 2) + mr;
        if (m0 + row < a.M) plane[(int64_t)row * a.N] = acc[mt][r];
      }
    } else {
      if (mt > 0) __syncthreads();   // the previous block's reduction has read the buffer
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(w * 16 + r) * 64 + lane] = acc[mt][r];
      __syncthreads();
      // wave w sums accumulator rows r = w, w + W, ... over the waves in wave order (the same order for every r)
      for (int r = w; r < 16; r += W) {
        float v = red[r * 64 + lane];
#pragma unroll
        for (int ww = 1; ww < W; ++ww) v += red[(ww * 16 + r) * 64 + lane];
        const int row = mt * 32 + (r & 3) + 8 * (r >> 2) + mr;
        if (m0 + row < a.M) plane[(int64_t)row * a.N] = v;
      }
    }
  }
  if (st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) st[3] = __builtin_amdgcn_s_memrealtime();
  }
}

}  // namespace aca

// variant: (KR, W) = 0: (2, 7) -> 14 planes, 1: (4, 7) -> 7 planes, 2: (1, 14) -> 14 planes, 3: (7, 4) -> 7 planes,
// 4: (7, 2) -> 14 planes, 5: (2, 14) -> 7 planes, 6: (1, 7) -> 28 planes, 7: (7, 7) -> 4 planes, 8: (14, 1) -> 14
// planes, 9: (7, 14) -> 2 planes. Returns the plane count through *S_out.
extern "C" hipError_t aca_fc_rollout(const uint16_t* X, int64_t ldx, int M, const uint16_t* Wf, int K, int N,
                                     float* P, int64_t pstride, int variant, int max_planes, int* S_out,
                                     unsigned long long* stamps, int msplit, hipStream_t stream) {
  static const int cfg[10][2] = {{2, 7}, {4, 7}, {1, 14}, {7, 4}, {7, 2}, {2, 14}, {1, 7}, {7, 7}, {14, 1}, {7, 14}};
  if (variant < 0 || variant > 9 || M < 1 || M > 128 || K % 16 || N % 32 || ldx % 8 ||
      reinterpret_cast<uintptr_t>(X) % 16 || reinterpret_cast<uintptr_t>(Wf) % 16 || (N >> 5) % 8)
    return hipErrorInvalidValue;
  const int kr = cfg[variant][0], w = cfg[variant][1];
  const int KB = K / 16;
  if (KB % (kr * w)) return hipErrorInvalidValue;
  const int S = KB / (kr * w);
  if (S > max_planes || pstride < (int64_t)M * N) return hipErrorInvalidValue;
  if (S_out) *S_out = S;
  aca::FcRolloutArgs a{reinterpret_cast<const aca::u16*>(X), ldx, M, reinterpret_cast<const aca::u16*>(Wf), K, N, P,
                       pstride, stamps};
  const int grid = S * (N >> 5);
  // 32-row blocks of X per wave (the fc's B fragments loaded once for all of them), or with msplit one block per
  // workgroup row (gridDim.y)
  const int MB = (M + 31) / 32;
  const int MT = msplit ? 1 : MB;
  if (variant == 9 && MT > 2) return hipErrorInvalidValue;   // 14 waves x 7 k-blocks x 3-4 row blocks would spill
  const dim3 gdim(grid, msplit ? MB : 1);
  switch (variant * 4 + (MT - 1)) {
#define ACA_FR_CASE(v, KR, W)                                                                      \
  case 4 * v + 0: aca::fc_rollout_kernel<KR, W, 1><<<gdim, 64 * W, 0, stream>>>(a); break;         \
  case 4 * v + 1: aca::fc_rollout_kernel<KR, W, 2><<<gdim, 64 * W, 0, stream>>>(a); break;         \
  case 4 * v + 2: aca::fc_rollout_kernel<KR, W, 3><<<gdim, 64 * W, 0, stream>>>(a); break;         \
  case 4 * v + 3: aca::fc_rollout_kernel<KR, W, 4><<<gdim, 64 * W, 0, stream>>>(a); break;
    ACA_FR_CASE(0, 2, 7) ACA_FR_CASE(1, 4, 7) ACA_FR_CASE(2, 1, 14) ACA_FR_CASE(3, 7, 4) ACA_FR_CASE(4, 7, 2)
    ACA_FR_CASE(5, 2, 14) ACA_FR_CASE(6, 1, 7) ACA_FR_CASE(7, 7, 7) ACA_FR_CASE(8, 14, 1) ACA_FR_CASE(9, 7, 14)
#undef ACA_FR_CASE
  }
  return hipGetLastError();
}
