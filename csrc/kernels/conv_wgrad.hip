// Weight gradients of the Nature-CNN trunk for large learner batches (PPO minibatches), as deterministic partial
// planes (each written once, no atomics) that the gradient finaliser reduces in plane order:
//
//   conv1:  dW1[o][c] = scale * sum_b sum_p dy1[b][p][o] * obs[b][ch][4 oy + ky][4 ox + kx],  c = (ch, ky, kx)
//   conv2 / conv3:  dW[o][(ky, kx, c)] = sum_b sum_p dy[b][p][o] * img[b][S oy + ky][S ox + kx][c]
//
// As implicit-im2col GEMMs (conv1: M 32, N 256, K = 400 B) every K chunk re-gathers its patches from global memory
// and every N tile re-reads dy: at B = 4096 the conv1 product fetched 2.4x its operand bytes and ran at ~6 % of the
// MFMA rate. Both kernels here stage the operands in LDS once per sample and read the patch matrix through the
// transposing ds_read_b64_tr_b16 WITHOUT materialising it (each lane points its read at the contiguous pixels of its
// own position / kernel tap).
#include "common.h"

namespace aca {

typedef short cw_short8 __attribute__((ext_vector_type(8)));

// 4 uint8 -> 4 bf16 (exact integers)
__device__ __forceinline__ uint2 cw_u8x4(uint32_t w) {
  uint2 r;
  r.x = (__float_as_uint((float)(w & 0xFF)) >> 16) | (__float_as_uint((float)((w >> 8) & 0xFF)) & 0xFFFF0000u);
  r.y = (__float_as_uint((float)((w >> 16) & 0xFF)) >> 16) | (__float_as_uint((float)(w >> 24)) & 0xFFFF0000u);
  return r;
}

// ------------------------------------------------------------------------------------------------------------
// conv1 weight gradient, all four input channels per workgroup on the 32x32x16 MFMA (conv1_wgrad2_kernel; a
//   first version staged a sample's dy1 rows once PER CHANNEL in four workgroups on 16x16 tiles and was bound by
//   staging and LDS reads: 48 % bank conflicts, ~380 TF/s at B = 4096). Workgroup g walks the samples of plane g and stages, per sample, the dy1 rows [416][32] (64-byte rows: the 4
//   rows of a transposing read land in disjoint bank windows) and all four frames as exact bf16 (56 KB) ONCE; the next
//   sample is in flight in registers. Wave w = (k quarter w >> 1, column half w & 1) owns a 32 x 128 output slice
//   (four 32x32 fp32 accumulators) over the k-steps ks = kq, kq + 4, ... of 16 positions: per k-step one A fragment
//   (dy1 rows, two transposing reads) feeds four MFMAs whose B fragments point each lane's transposing read at the 4
//   contiguous frame pixels of its (position, ch, ky, kx0..kx0+3) -- no im2col. The k quarters meet in LDS in order
//   at the end; plane g ([32][256] fp32) is written once, scaled. Deterministic (fixed order, no atomics).
// ------------------------------------------------------------------------------------------------------------
typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int C2_T = 512;
constexpr int C2_FR = 4 * 84 * 84;                 // 28224 frame pixels per sample (bf16 in LDS) + a zero chunk
constexpr int C2_FR4 = C2_FR / 16;                 // 1764 16-byte chunks of uint8 pixels
constexpr int C2_DY4 = 400 * 4;                    // 1600 16-byte chunks of dy1
constexpr int C2_DYOFF = (C2_FR + 8) * 2;          // byte offset of the dy1 rows in LDS
constexpr int C2_RED = 3 * 2 * 32 * 128 * 4;       // k-quarter partials at the end (96 KB, aliases the staging)
constexpr int C2_LDS = C2_RED > C2_DYOFF + 416 * 64 ? C2_RED : C2_DYOFF + 416 * 64;
static_assert(C2_DYOFF % 16 == 0 && C2_FR4 <= 4 * C2_T && C2_DY4 <= 4 * C2_T, "conv1_wgrad2 staging geometry");

__global__ void __launch_bounds__(C2_T) conv1_wgrad2_kernel(const uint8_t* __restrict__ obs,
                                                            const u16* __restrict__ dy1, float* __restrict__ planes,
                                                            int B, int P, float scale,
                                                            const int64_t* __restrict__ obs_idx) {
  __shared__ __attribute__((aligned(16))) unsigned char s_raw[C2_LDS];
  u16* const s_fr = reinterpret_cast<u16*>(s_raw);
  u16* const s_dy = reinterpret_cast<u16*>(s_raw + C2_DYOFF);
  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b0 = (int)((int64_t)g * B / P), b1 = (int)((int64_t)(g + 1) * B / P);
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  // padding positions 400..415: zero dy1 rows and the zero frame chunk, written once (never restaged)
  if (tid < 64) *reinterpret_cast<uint4*>(s_dy + 400 * 32 + tid * 8) = z4;
  if (tid == 0) *reinterpret_cast<uint4*>(s_fr + C2_FR) = z4;

  uint4 f0, f1, f2, f3, d0, d1, d2, d3;   // the next sample (named registers: arrays of uint4 went to scratch)
  auto load = [&](int b) {
    const uint4* f = reinterpret_cast<const uint4*>(obs + (size_t)(obs_idx ? obs_idx[b] : b) * C2_FR);
    const uint4* d = reinterpret_cast<const uint4*>(dy1 + (size_t)b * 400 * 32);
    f0 = f[tid];
    f1 = f[tid + C2_T];
    f2 = f[tid + 2 * C2_T];
    f3 = f[min(tid + 3 * C2_T, C2_FR4 - 1)];
    d0 = d[tid];
    d1 = d[tid + C2_T];
    d2 = d[tid + 2 * C2_T];
    d3 = d[min(tid + 3 * C2_T, C2_DY4 - 1)];
  };
  auto put_fr = [&](const uint4& w, int i) {
    const uint2 a = cw_u8x4(w.x), b_ = cw_u8x4(w.y), c = cw_u8x4(w.z), d = cw_u8x4(w.w);
    *reinterpret_cast<uint4*>(s_fr + i * 16) = make_uint4(a.x, a.y, b_.x, b_.y);
    *reinterpret_cast<uint4*>(s_fr + i * 16 + 8) = make_uint4(c.x, c.y, d.x, d.y);
  };
  auto store = [&]() {
    put_fr(f0, tid);
    put_fr(f1, tid + C2_T);
    put_fr(f2, tid + 2 * C2_T);
    if (tid + 3 * C2_T < C2_FR4) put_fr(f3, tid + 3 * C2_T);
    *reinterpret_cast<uint4*>(s_dy + tid * 8) = d0;
    *reinterpret_cast<uint4*>(s_dy + (tid + C2_T) * 8) = d1;
    *reinterpret_cast<uint4*>(s_dy + (tid + 2 * C2_T) * 8) = d2;
    if (tid + 3 * C2_T < C2_DY4) *reinterpret_cast<uint4*>(s_dy + (tid + 3 * C2_T) * 8) = d3;
  };

  const int nh = wid & 1, kq = wid >> 1;
  // lane roles of the transposing reads: 16-lane group gl, lane 4 q + p4 of the group
  const int gl = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  const int acol = (gl & 1) * 16 + 4 * p4, khalf = 8 * (gl >> 1);
  int noff[4];   // (ch, ky, kx0) pixel offset of this lane's 4 B columns, per 32-column tile
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int c = nh * 128 + t * 32 + (gl & 1) * 16 + 4 * p4;
    noff[t] = (c >> 6) * 7056 + ((c >> 3) & 7) * 84 + (c & 7);
  }
  floatx16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  typedef short short4x __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) short4x lds4;
  auto pos = [&](int p) -> int {   // frame offset of position p's (4 oy, 4 ox) pixel; padding -> -1
    const int oy = (p * 3277) >> 16;   // p / 20 for p < 5000
    return p < 400 ? (4 * oy) * 84 + 4 * (p - 20 * oy) : -1;
  };
  if (b0 < b1) load(b0);
  for (int b = b0; b < b1; ++b) {
    store();
    __syncthreads();
    if (b + 1 < b1) load(b + 1);
    for (int ks = kq; ks < 26; ks += 4) {
      const int kb = ks * 16 + khalf;
      const short4x a_lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(s_dy + (kb + q) * 32 + acol));
      const short4x a_hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(s_dy + (kb + 4 + q) * 32 + acol));
      const cw_short8 av = {a_lo[0], a_lo[1], a_lo[2], a_lo[3], a_hi[0], a_hi[1], a_hi[2], a_hi[3]};
      const bf16x8 af = __builtin_bit_cast(bf16x8, av);
      const int pa = pos(kb + q), pb = pos(kb + 4 + q);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const short4x lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(s_fr + (pa < 0 ? C2_FR : pa + noff[t])));
        const short4x hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(s_fr + (pb < 0 ? C2_FR : pb + noff[t])));
        const cw_short8 bv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, __builtin_bit_cast(bf16x8, bv), acc[t], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // k quarters 1..3 -> LDS, quarter 0 adds them in order and writes the plane
  float* const red = reinterpret_cast<float*>(s_raw);
  if (kq > 0)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) red[(((kq - 1) * 2 + nh) * 64 + t * 16 + i) * 64 + lane] = acc[t][i];
  __syncthreads();
  if (kq == 0) {
    float* const dst = planes + (size_t)g * 32 * 256;
    const int col = lane & 31, rh = 4 * (lane >> 5);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float v = acc[t][i];
#pragma unroll
        for (int k = 0; k < 3; ++k) v += red[((k * 2 + nh) * 64 + t * 16 + i) * 64 + lane];
        const int o = (i & 3) + 8 * (i >> 2) + rh;
        dst[o * 256 + nh * 128 + t * 32 + col] = v * scale;
      }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Batched-position weight gradient of a bf16 NHWC conv layer on the 32x32x16 MFMA (large learner batches):
//   dW[o][n] = sum_P dy[P][o] * col[P][n],   P = (sample, oy, ox) over the workgroup's samples,
//                                              n = (ky, kx, c),  col[P][n] = img[sample][S oy + ky][S ox + kx][c]
// i.e. ONE GEMM with M = 64 output channels, N = KS KS C, K = the positions of SB samples at a time (positions of
// consecutive samples are consecutive K rows -- no per-sample padding of the 49 / 81 positions to a k-step). The
// per-sample form (one kernel row per workgroup, retired) multiplied 12-16 MFMAs per wave per staged sample and spends its time staging and at
// barriers; here every workgroup owns ALL 64 x N outputs of its plane (8 waves: wave w holds m-tile w & 1 and the
// n-tiles (w >> 1) + 4 i, 32x32 fp32 accumulators in registers), stages SB samples per LDS fill (the next fill is in
// flight in registers meanwhile) and runs KP / 16 k-steps of 4-5 MFMAs per wave between two barriers. Both MFMA
// operands come from K-major LDS rows through the transposing ds_read_b64_tr_b16: A = dy rows (position-major,
// 64 channels), B = the implicit im2col -- each lane points its read at the 4 contiguous channels of its
// (position, ky, kx, c0) pixel, no column matrix. Plane g (samples [g B / P, (g + 1) B / P)) is written once, in
// full; the gradient finaliser reduces the P planes in plane order (deterministic, no atomics).
// ---------------------------------------------------------------------------------------------------------------
template <int H, int W, int C, int KS, int S, int OH, int OW, int SB>
__global__ void __launch_bounds__(512) conv_wgrad_gemm_kernel(const u16* __restrict__ img,
                                                              const u16* __restrict__ dy,
                                                              float* __restrict__ planes, int B, int P) {
  constexpr int T = 512;
  constexpr int NPOS = OH * OW, NCOL = KS * KS * C;
  constexpr int GP = SB * NPOS, KST = (GP + 15) / 16, KP = KST * 16;
  // LDS rows: the 4 rows of a transposing read (positions kb + q) land in 4 disjoint 16-bank windows -- dy rows of
  // 192 bytes, image pixels of 96 bytes at stride 2 / 192 bytes at stride 1 (S x pixel bytes = 64 mod 256 or 192);
  // the +8 / 144-byte layouts read 2x / 1.9x the ideal cycles (tests/test_lds_layouts_cpu.py models both reads)
  constexpr int LDI = S == 2 ? C + 16 : C + 32, LDD = 96, IMG_E = H * W * LDI;
  static_assert((S * LDI * 2) % 256 == 64 || (S * LDI * 2) % 256 == 192, "conflict-free image rows");
  constexpr int NT = NCOL / 32;                         // n tiles of 32
  constexpr int TPW = (NT + 3) / 4;                     // n tiles per wave (wave pairs share an n tile set)
  constexpr int CPP = C / 8;                            // 16-byte chunks per pixel
  constexpr int IMG4 = SB * H * W * CPP, DY4 = SB * NPOS * 8;
  constexpr int IPER = (IMG4 + T - 1) / T, DPER = (DY4 + T - 1) / T;
  static_assert(NCOL % 32 == 0 && C % 16 == 0, "tile shapes");
  __shared__ __attribute__((aligned(16))) u16 s_img[SB * IMG_E + 8];   // + a zero chunk for padding positions
  __shared__ __attribute__((aligned(16))) u16 s_dy[KP * LDD];
  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b0 = (int)((int64_t)g * B / P), b1 = (int)((int64_t)(g + 1) * B / P);
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  // padding rows GP..KP of the dy image and the zero chunk: written once, never restaged
  for (int c = tid; c < (KP - GP) * (LDD / 8); c += T) *reinterpret_cast<uint4*>(s_dy + GP * LDD + c * 8) = z4;
  if (tid == 0) *reinterpret_cast<uint4*>(s_img + SB * IMG_E) = z4;

  // the next fill in flight in NAMED registers (arrays of uint4 here were placed in scratch / LDS by the compiler)
  static_assert(IPER <= 8 && DPER <= 3, "register set holds 8 image + 3 dy chunks per thread");
  uint4 ri0 = z4, ri1 = z4, ri2 = z4, ri3 = z4, ri4 = z4, ri5 = z4, ri6 = z4, ri7 = z4, rd0 = z4, rd1 = z4, rd2 = z4;
#define CWG_LDI(R, u)                                                                                     \
  if ((u) < IPER) {                                                                                       \
    const int c = min(tid + (u) * T, IMG4 - 1);                                                           \
    const int sm = c / (H * W * CPP), r = c - sm * (H * W * CPP);                                         \
    R = reinterpret_cast<const uint4*>(img + (size_t)min(bs + sm, b1 - 1) * H * W * C)[r];                \
  }
#define CWG_LDD(R, u)                                                                                     \
  if ((u) < DPER) {                                                                                       \
    const int c = min(tid + (u) * T, DY4 - 1);                                                            \
    const int sm = c / (NPOS * 8), r = c - sm * (NPOS * 8);                                               \
    const uint4 v = reinterpret_cast<const uint4*>(dy + (size_t)min(bs + sm, b1 - 1) * NPOS * 64)[r];     \
    R = bs + sm < b1 ? v : z4;                                                                            \
  }
  // samples bs .. bs + SB - 1 -> registers (past b1: the image of sample b1 - 1, zero dy rows)
#define CWG_LOAD(bs_)                                                                                     \
  {                                                                                                       \
    const int bs = (bs_);                                                                                 \
    CWG_LDI(ri0, 0) CWG_LDI(ri1, 1) CWG_LDI(ri2, 2) CWG_LDI(ri3, 3)                                       \
    CWG_LDI(ri4, 4) CWG_LDI(ri5, 5) CWG_LDI(ri6, 6) CWG_LDI(ri7, 7)                                       \
    CWG_LDD(rd0, 0) CWG_LDD(rd1, 1) CWG_LDD(rd2, 2)                                                       \
  }
#define CWG_STI(R, u)                                                                                     \
  if ((u) < IPER && tid + (u) * T < IMG4) {                                                               \
    const int c = tid + (u) * T;                                                                          \
    const int sm = c / (H * W * CPP), r = c - sm * (H * W * CPP);                                         \
    const int px = r / CPP, part = r - px * CPP;                                                          \
    *reinterpret_cast<uint4*>(s_img + sm * IMG_E + px * LDI + part * 8) = R;                              \
  }
#define CWG_STD(R, u)                                                                                     \
  if ((u) < DPER && tid + (u) * T < DY4) {                                                                \
    const int c = tid + (u) * T;                                                                          \
    *reinterpret_cast<uint4*>(s_dy + (c >> 3) * LDD + (c & 7) * 8) = R;                                   \
  }
#define CWG_STORE()                                                                                       \
  {                                                                                                       \
    CWG_STI(ri0, 0) CWG_STI(ri1, 1) CWG_STI(ri2, 2) CWG_STI(ri3, 3)                                       \
    CWG_STI(ri4, 4) CWG_STI(ri5, 5) CWG_STI(ri6, 6) CWG_STI(ri7, 7)                                       \
    CWG_STD(rd0, 0) CWG_STD(rd1, 1) CWG_STD(rd2, 2)                                                       \
  }

  floatx16 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  // lane roles in the transposing reads: 16-lane group gl, lane 4q + p of the group; a group covers 16 columns
  const int gl = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  const int mt = wid & 1, nb = wid >> 1;
  const int acol = mt * 32 + (gl & 1) * 16 + 4 * p4;   // dy column block of this lane's A read
  const int khalf = 8 * (gl >> 1);
  int noff[TPW];                                        // (ky, kx, c0) pixel offset of this lane's B columns
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int nt = min(nb + 4 * t, NT - 1);
    const int n0 = nt * 32 + (gl & 1) * 16 + 4 * p4;
    const int kyx = n0 / C, c0 = n0 - kyx * C, ky = kyx / KS, kx = kyx - ky * KS;
    noff[t] = (ky * W + kx) * LDI + c0;
  }
  typedef short short4x __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) short4x lds4;
  auto pos_off = [&](int Pk) -> int {   // LDS element offset of pixel (S oy, S ox) of position Pk; padding -> zero
    if (Pk >= GP) return SB * IMG_E;
    const int sm = Pk / NPOS, pp = Pk - sm * NPOS, oy = pp / OW, ox = pp - oy * OW;
    return sm * IMG_E + (S * oy * W + S * ox) * LDI;
  };
  const int ngroups = (b1 - b0 + SB - 1) / SB;
  if (ngroups > 0) CWG_LOAD(b0)
  for (int gi = 0; gi < ngroups; ++gi) {
    CWG_STORE()
    __syncthreads();
    if (gi + 1 < ngroups) CWG_LOAD(b0 + (gi + 1) * SB)
#pragma unroll 2
    for (int ks = 0; ks < KST; ++ks) {
      const int kb = ks * 16 + khalf;
      const short4x a_lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(s_dy + (kb + q) * LDD + acol));
      const short4x a_hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(s_dy + (kb + 4 + q) * LDD + acol));
      const cw_short8 av = {a_lo[0], a_lo[1], a_lo[2], a_lo[3], a_hi[0], a_hi[1], a_hi[2], a_hi[3]};
      const bf16x8 af = __builtin_bit_cast(bf16x8, av);
      const int pa = pos_off(kb + q), pb = pos_off(kb + 4 + q);
      const bool padded = kb + 4 + q >= GP;
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        if (nb + 4 * t < NT) {   // wave-uniform
          const int oa = pa == SB * IMG_E ? pa : pa + noff[t];
          const int ob = padded ? SB * IMG_E : pb + noff[t];
          const short4x lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(s_img + oa));
          const short4x hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(s_img + ob));
          const cw_short8 bv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, __builtin_bit_cast(bf16x8, bv), acc[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
#undef CWG_LDI
#undef CWG_LDD
#undef CWG_LOAD
#undef CWG_STI
#undef CWG_STD
#undef CWG_STORE
  // plane g: [64][NCOL] fp32, each element written exactly once (zero for an empty sample range)
  float* dst = planes + (size_t)g * 64 * NCOL;
  const int col = lane & 31, rh = 4 * (lane >> 5);
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int nt = nb + 4 * t;
    if (nt < NT)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = mt * 32 + (i & 3) + 8 * (i >> 2) + rh;
        dst[(size_t)row * NCOL + nt * 32 + col] = acc[t][i];
      }
  }
}

}  // namespace aca

// All four channels per workgroup (conv1_wgrad2_kernel): grid P, plane g of [32][256] per workgroup.
extern "C" hipError_t aca_conv1_wgrad2(const uint8_t* obs, const uint16_t* dy1, float* planes, int B, int P,
                                       float scale, const int64_t* obs_idx, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if (P < 1 || P > 1024 || reinterpret_cast<uintptr_t>(obs) % 16 || reinterpret_cast<uintptr_t>(dy1) % 16)
    return hipErrorInvalidValue;
  aca::conv1_wgrad2_kernel<<<P, aca::C2_T, 0, stream>>>(obs, dy1, planes, B, P, scale, obs_idx);
  return hipGetLastError();
}

// Batched-position form (conv_wgrad_gemm_kernel): grid P, plane g of [64][N] per workgroup. layer 2 / 3 as below.
extern "C" hipError_t aca_conv_wgrad_gemm(int layer, const uint16_t* img, const uint16_t* dy, float* planes, int B,
                                          int P, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if (P < 1 || P > 1024) return hipErrorInvalidValue;
  if (layer == 2)
    aca::conv_wgrad_gemm_kernel<20, 20, 32, 4, 2, 9, 9, 2><<<P, 512, 0, stream>>>(img, dy, planes, B, P);
  else if (layer == 3)
    aca::conv_wgrad_gemm_kernel<9, 9, 64, 3, 1, 7, 7, 2><<<P, 512, 0, stream>>>(img, dy, planes, B, P);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
