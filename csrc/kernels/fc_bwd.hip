// Learner fc-layer backward at rollout-sized batches (A2C: B = T x N <= 256 rows; SURVEY §2.4 K01, backward):
//   dy3  = (dh Wfc^T) * (y3 > 0)   [B, 3136] bf16   -- the conv trunk backward's input
//   dWfc = y3^T dh                 [3136, 512] fp32 -- stored final into the gradient slab
// as ONE launch of two job kinds (replaces the grouped general-GEMM launch, 21.7 us in the headline update trace,
// profiles/r5_headline.txt, for ~1 GFLOP and ~12 MB).
//
// dWfc jobs (64 x 64 output tiles, 49 x 8): both operands have the reduction index b as their ROW index, so the tile's
// y3 columns [B][64] and dh columns [B][64] are staged whole in LDS (one round of 16-byte loads, 128-byte row pieces)
// and both MFMA operands are read with the transposing ds_read_b64_tr_b16. The images are kept as 32-column halves
// with unpadded 64-byte rows: the four rows of a transposed read fall into four disjoint 16-bank windows
// (conflict-free), 40 KB at B = 160 (4 workgroups per CU). Wave w owns the 32 x 32 quadrant
// (kf rows 32 (w >> 1).., n columns 32 (w & 1)..), K = B in 16-deep steps (rows past B are zero). Every output
// element is written once: no planes, no atomics.
// dy3 jobs (32 b x 32 kf tiles): both operands are k-contiguous rows (32 dh rows, 32 Wfc rows of 1 KB), loaded by
// whole-line loads (fragment-shaped global loads -- 32 rows x 32 bytes per wave instruction -- issued at a fraction
// of the line rate: 1.4 us of issue for 64 KB), staged in LDS one K half at a time (34 KB) and read back as MFMA
// fragments by ds_read_b128; wave w takes the K quarter w of each half, the quarters added through LDS in wave
// order, then the ReLU mask of y3 (requested with the operands) and the bf16 rounding.
// Workgroup order is XCD-grouped per job kind (contiguous tile ranges per XCD), so the tiles sharing y3 / Wfc
// column blocks meet in one L2.
#include "common.h"

namespace aca {

typedef float fb_f32x16 __attribute__((ext_vector_type(16)));
typedef short fb_s4 __attribute__((ext_vector_type(4)));
typedef short fb_s8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) fb_s4 fb_lds4;
typedef unsigned int fb_u4 __attribute__((ext_vector_type(4)));   // staging registers (a uint4 struct copy is a
                                                                  // memcpy that SROA leaves in scratch)

constexpr int FB_THREADS = 256;
constexpr int FB_MAXB = 256;
constexpr int FB_KF = 3136, FB_N = 512;
constexpr int FB_DW_TILES = (FB_KF / 64) * (FB_N / 64);   // 392
constexpr int FB_LDH = FB_N / 2 + 8;  // LDS row of the dy3 operand blocks (bf16): one K half, 512 + 16 bytes
                                      // (rows 4 banks apart: conflict-free b128 fragment reads)

struct FcBwdArgs {
  const u16* dh;      // [B][512] bf16
  const u16* W;       // Wfc [3136][512] bf16 (row-major shadow)
  const u16* y3;      // [B][3136] bf16 (saved activations, ReLU outputs)
  u16* dy3;           // [B][3136] bf16
  float* dW;          // [3136][512] fp32
  int B;
  int n_dy;           // dy3 tiles: ceil(B / 32) x 98
  uint64_t* stamps;   // diagnostics: per workgroup [entry, operands in, MFMAs done, stores issued]
  float* sq;          // optional: per (dWfc tile, wave) sum of squares [392 x 4] (the finaliser's norm partials
                      // then need no 6.4 MB re-read of dWfc)
};

__device__ __forceinline__ void fb_stamp(uint64_t* st, int slot) {
  if (st && threadIdx.x == 0) st[(size_t)blockIdx.x * 4 + slot] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ bf16x8 fb_tr8(const u16* lo, const u16* hi) {
  const fb_s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((fb_lds4*)(lo));
  const fb_s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((fb_lds4*)(hi));
  const fb_s8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void fb_dw_job(const FcBwdArgs& a, int t, u16* smem) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int B = a.B, Bp = (B + 15) & ~15, KS = Bp >> 4;
  const int i = t >> 3, j = t & 7;   // kf block of 64, n block of 64
  // images of 32-column halves with 64-byte rows: element (b, c) at (c / 32) * Bp * 32 + b * 32 + c % 32
  u16* sY = smem;                    // y3[b][64 i + c]
  u16* sD = smem + 2 * Bp * 32;      // dh[b][64 j + c]
  // ---- staging: Bp rows x 8 chunks of 16 bytes per image, every load of the thread in flight at once
  const int nch = Bp * 8;            // chunks per image (<= 2048)
  uint4 vy[8], vd[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {   // branch-free (clamped rows): a guarded load kept the arrays in scratch
    const int c = tid + u * FB_THREADS;
    const int b = min(c >> 3, B - 1), q = c & 7;
    vy[u] = *reinterpret_cast<const uint4*>(a.y3 + (size_t)b * FB_KF + 64 * i + 8 * q);
    vd[u] = *reinterpret_cast<const uint4*>(a.dh + (size_t)b * FB_N + 64 * j + 8 * q);
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = tid + u * FB_THREADS;
    if (c < nch) {   // rows past B: zero (masked word by word; a select of whole uint4s went through scratch)
      const int b = c >> 3, q = c & 7;
      const unsigned m = b < B ? 0xFFFFFFFFu : 0u;
      const int o = (q >> 2) * Bp * 32 + b * 32 + (q & 3) * 8;
      *reinterpret_cast<uint4*>(sY + o) = make_uint4(vy[u].x & m, vy[u].y & m, vy[u].z & m, vy[u].w & m);
      *reinterpret_cast<uint4*>(sD + o) = make_uint4(vd[u].x & m, vd[u].y & m, vd[u].z & m, vd[u].w & m);
    }
  }
  fb_stamp(a.stamps, 1);
  __syncthreads();
  // ---- MFMAs: wave w -> quadrant (kf rows 32 mq.., n columns 32 nq..); transposing reads of both images (a 32-lane
  // half reads 4 rows x 64 bytes: all 64 banks once, conflict-free)
  const int mq = w >> 1, nq = w & 1;
  const int gl = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  const int cin = 16 * (gl & 1) + 4 * p4;
  const u16* pA = sY + mq * Bp * 32 + cin;
  const u16* pB = sD + nq * Bp * 32 + cin;
  const int khalf = 8 * (gl >> 1);
  fb_f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int ks = 0; ks < KS; ++ks) {
    const int kb = 16 * ks + khalf;
    const bf16x8 af = fb_tr8(pA + (kb + q) * 32, pA + (kb + 4 + q) * 32);
    const bf16x8 bf = fb_tr8(pB + (kb + q) * 32, pB + (kb + 4 + q) * 32);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc, 0, 0, 0);
  }
  fb_stamp(a.stamps, 2);
  // ---- the quadrant, written once: 32 lanes per row x 4 bytes
  const int col = lane & 31, rh = 4 * (lane >> 5);
  float* dst = a.dW + (size_t)(64 * i + 32 * mq) * FB_N + 64 * j + 32 * nq + col;
#pragma unroll
  for (int r = 0; r < 16; ++r) dst[(size_t)((r & 3) + 8 * (r >> 2) + rh) * FB_N] = acc[r];
  if (a.sq) {   // the quadrant's sum of squares: lane terms in register order, then a fixed xor tree
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) v = fmaf(acc[r], acc[r], v);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += lane_xor(v, o);
    if (lane == 0) a.sq[t * 4 + w] = v;
  }
}

__device__ __forceinline__ void fb_dy_job(const FcBwdArgs& a, int t, u16* smem) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int B = a.B, nbb = (B + 31) >> 5;
  const int jb = t / nbb, ib = t - jb * nbb;   // kf block of 32, b block of 32
  u16* sA = smem;                              // [32][FB_LDH]: dh rows 32 ib .., one K half
  u16* sB = smem + 32 * FB_LDH;                // [32][FB_LDH]: Wfc rows 32 jb .., one K half
  // ---- every load at once: thread -> 16-byte chunks q and q + 32 (one per K half) of rows tid / 32 + 8 u
  const int q = tid & 31, r0 = tid >> 5;
  fb_u4 va[2][4], vb[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = r0 + 8 * u;
      va[h][u] = *reinterpret_cast<const fb_u4*>(a.dh + (size_t)min(32 * ib + r, B - 1) * FB_N + 8 * (q + 32 * h));
      vb[h][u] = *reinterpret_cast<const fb_u4*>(a.W + (size_t)(32 * jb + r) * FB_N + 8 * (q + 32 * h));
    }
  // the ReLU mask of this lane's 16 outputs, requested with the operands (used by wave 0)
  const int col = 32 * jb + (lane & 31), rh = 4 * (lane >> 5);
  const u16* ym = a.y3 + col;
  u16 mk[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) mk[r] = ym[(size_t)min(32 * ib + (r & 3) + 8 * (r >> 2) + rh, B - 1) * FB_KF];
  fb_f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  // wave w: K quarter w of each half (4 steps of 32x32x16, fragments by ds_read_b128)
  const int ro = (lane & 31) * FB_LDH + 64 * w + 8 * (lane >> 5);
  const int so = r0 * FB_LDH + 8 * q;
#define FB_ST1(H, U)                                                                  \
  *reinterpret_cast<fb_u4*>(sA + so + 8 * (U) * FB_LDH) = va[H][U];                   \
  *reinterpret_cast<fb_u4*>(sB + so + 8 * (U) * FB_LDH) = vb[H][U];
#define FB_STAGE(H) FB_ST1(H, 0) FB_ST1(H, 1) FB_ST1(H, 2) FB_ST1(H, 3)
#define FB_MM1(S)                                                                     \
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(sA + ro + 16 * (S)), \
                                                *reinterpret_cast<const bf16x8*>(sB + ro + 16 * (S)), acc, 0, 0, 0);
#define FB_HALF() FB_MM1(0) FB_MM1(1) FB_MM1(2) FB_MM1(3)
  FB_STAGE(0)
  fb_stamp(a.stamps, 1);
  __syncthreads();
  FB_HALF()
  __syncthreads();   // every wave is past its reads of the first half
  FB_STAGE(1)
  __syncthreads();
  FB_HALF()
#undef FB_ST1
#undef FB_STAGE
#undef FB_MM1
#undef FB_HALF
  fb_stamp(a.stamps, 2);
  // ---- K quarters summed through LDS in wave order (deterministic), then the mask and the bf16 rounding
  __syncthreads();   // every wave is past its operand reads
  float* red = reinterpret_cast<float*>(smem);
  if (w > 0)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[((w - 1) * 16 + r) * 64 + lane] = acc[r];
  __syncthreads();
  if (w > 0) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int b = 32 * ib + (r & 3) + 8 * (r >> 2) + rh;
    const float v = ((acc[r] + red[r * 64 + lane]) + red[(16 + r) * 64 + lane]) + red[(32 + r) * 64 + lane];
    if (b < B) a.dy3[(size_t)b * FB_KF + col] = bf2f(mk[r]) > 0.f ? f2bf(v) : (u16)0;
  }
}

__global__ void __launch_bounds__(FB_THREADS, 4) fc_bwd_kernel(FcBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) u16 fb_smem[];
  fb_stamp(a.stamps, 0);
  const int id = blockIdx.x;
  if (id < FB_DW_TILES) {
    fb_dw_job(a, xcd_remap(id, FB_DW_TILES), fb_smem);
  } else {
    fb_dy_job(a, xcd_remap(id - FB_DW_TILES, a.n_dy), fb_smem);
  }
  fb_stamp(a.stamps, 3);
}

}  // namespace aca

// dh [B][512], W = Wfc [3136][512], y3 [B][3136] bf16 -> dy3 [B][3136] bf16, dW [3136][512] fp32; 1 <= B <= 256,
// every pointer 16-byte aligned, the row strides dense.
extern "C" hipError_t aca_fc_bwd(const uint16_t* dh, const uint16_t* W, const uint16_t* y3, uint16_t* dy3, float* dW,
                                 int B, float* sq, uint64_t* stamps, hipStream_t stream) {
  if (B < 1 || B > aca::FB_MAXB) return hipErrorInvalidValue;
  for (const void* p : {(const void*)dh, (const void*)W, (const void*)y3, (const void*)dy3, (const void*)dW})
    if (!p || reinterpret_cast<uintptr_t>(p) % 16) return hipErrorInvalidValue;
  aca::FcBwdArgs a{dh, W, y3, dy3, dW, B, ((B + 31) / 32) * (aca::FB_KF / 32), stamps, sq};
  const int Bp = (B + 15) & ~15;
  const size_t lds = std::max((size_t)4 * Bp * 32 * 2, (size_t)2 * 32 * aca::FB_LDH * 2);
  aca::fc_bwd_kernel<<<aca::FB_DW_TILES + a.n_dy, aca::FB_THREADS, lds, stream>>>(a);
  return hipGetLastError();
}
