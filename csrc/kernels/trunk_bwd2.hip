// Fused data-gradient chain of the conv trunk, v2 (learner backward; same contract as cnn_fused.hip
// cnn_trunk_bwd_kernel / _persist_kernel, selected by EngineOpts.trunk_bwd_v2):
//   dy2 = conv_transpose(dy3, W3) * (y2 > 0)        M 81 positions, N 64, K 576 = (tap i j, o)
//   dy1 = conv_transpose(dy2, W2) * (y1 > 0)        sub-pixel form: per output parity class (py, px) only its
//                                                    2 x 2 taps, K 256 = (di, dj, o), M 100, N 32
//   biasp[b] = [ sum_p dy3 | sum_p dy2 | sum_p dy1 ]  (64 | 64 | 32, fixed summation order)
// v1 runs both products as 16x16x32 MFMAs whose waves re-read the A operand once per 16-column N tile (1 MB of LDS
// reads per sample) and moves dy2 / dy1 through extra LDS passes. Here both products run TRANSPOSED as 32x32x16
// MFMAs (A = weights, B = image pixels), so each lane ends with one output position and 4 runs of 4 consecutive
// channels:
//   dy2^T: 6 waves = 3 position tiles x 2 channel tiles, K = 576; masked, rounded, written as 8-byte runs into the
//          dy2 image (dy1's input) and straight to dy2 in memory; db2 by xor shuffles over the positions;
//   dy1^T: wave w = parity class w / 2, output tiles 2 (w & 1) + {0, 1}; the class's W2 fragments held in
//          registers; y1 mask (requested at the sample's start), bf16, 8-byte stores straight to memory; db1 by
//          shuffles. No staging pass, no per-sample border re-zeroing.
// LDS images (dy3: 11 x 25 pixels, dy2: 11 x 26, 64 channels, unpadded 128-byte pixels) keep each pixel's 16-byte
// channel chunks XOR-swizzled by (pixel >> 1) & 7; with image widths = 9 / 10 (mod 16) the 16 lanes of every
// ds_read_b128 group (16 output positions, one chunk) then hit 16 distinct bank quads (tests/test_lds_layouts_cpu.py
// models every fragment read). W3 B rows: 128 bytes, chunk ^ ((row >> 1) & 1) << 2 (4-row x 64-byte transposing
// reads conflict-free); W2 B rows: 64 bytes, plain.
#include "common.h"

namespace aca {

constexpr int B2_T = 512;
constexpr int B2_P3W = 25, B2_P2W = 26, B2_IH = 11;
constexpr int B2_P3E = B2_IH * B2_P3W * 64;   // 17600 u16 (35.2 KB)
constexpr int B2_P2E = B2_IH * B2_P2W * 64;   // 18304 u16 (36.6 KB)
constexpr int B2_W3E = 576 * 64;              // 36864 u16 (72 KB)
constexpr int B2_M2E = 81 * 64;               // 5184 u16 (y2 mask)
static_assert(1024 * 32 <= B2_P3E + B2_P2E, "W2 rows stage in the image region before the walk");

typedef float b2_f32x16 __attribute__((ext_vector_type(16)));
typedef short b2_s4 __attribute__((ext_vector_type(4)));
typedef short b2_s8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) b2_s4 b2_lds4;
typedef unsigned int b2_u4 __attribute__((ext_vector_type(4)));   // register-held chunks (a uint4 struct copy is a
                                                                  // memcpy that SROA leaves in scratch)

// u16 offset of 16-byte channel chunk `ch` (0..7) of image pixel `pix`
__device__ __forceinline__ int b2_px(int pix, int ch) { return pix * 64 + ((ch ^ ((pix >> 1) & 7)) << 3); }
__device__ __forceinline__ int b2_sw3(int r) { return ((r >> 1) & 1) << 2; }
// exact small-range divisions as multiply-shifts (n / 9 for n < 200, n / 10 for n < 1029, n / 7 for n < 64)
__device__ __forceinline__ int b2_div9(int n) { return (int)(((unsigned)n * 57u) >> 9); }
__device__ __forceinline__ int b2_div10(int n) { return (int)(((unsigned)n * 205u) >> 11); }
__device__ __forceinline__ int b2_div7(int n) { return (int)(((unsigned)n * 37u) >> 8); }
__device__ __forceinline__ float b2_lane(uint32_t w, int hi) {
  return __uint_as_float(hi ? (w & 0xFFFF0000u) : (w << 16));
}
__device__ __forceinline__ uint32_t b2_mask(uint32_t w, uint32_t m) {   // zero each bf16 of w whose mask is <= 0
  const uint32_t lo = (__uint_as_float(m << 16) > 0.f) ? 0x0000FFFFu : 0u;
  const uint32_t hi = (__uint_as_float(m & 0xFFFF0000u) > 0.f) ? 0xFFFF0000u : 0u;
  return w & (lo | hi);
}
// 32x32x16 B fragment (k = 8 (lane >> 5) + 0..7, n = col0 + lane & 31) from k-major rows by two transposing reads;
// rows[r * ld + swizzled col]; SW: W3 rows (128 B, chunk ^ b2_sw3(r)) or plain rows
template <bool SW>
__device__ __forceinline__ bf16x8 b2_trb(const u16* rows, int ld, int row0, int col0, int lane) {
  const int gl = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r0 = row0 + 8 * (gl >> 1) + q, r1 = r0 + 4, col = col0 + 16 * (gl & 1) + 4 * p;
  const int c0 = SW ? ((((col >> 3) ^ b2_sw3(r0)) << 3) | (col & 7)) : col;
  const int c1 = SW ? ((((col >> 3) ^ b2_sw3(r1)) << 3) | (col & 7)) : col;
  const b2_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((b2_lds4*)(rows + r0 * ld + c0));
  const b2_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((b2_lds4*)(rows + r1 * ld + c1));
  const b2_s8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// WALK: the workgroup walks several samples (W3 rows resident, W2 fragments extracted once up front); else one
// sample per workgroup, whose W2 rows are loaded into registers at entry and staged over the W3 rows after dy2.
template <bool WALK>
__global__ void __launch_bounds__(B2_T) cnn_trunk_bwd2_kernel(
    const u16* __restrict__ dy3g, const u16* __restrict__ W3, const u16* __restrict__ y2g,
    const u16* __restrict__ W2, const u16* __restrict__ y1g, u16* __restrict__ dy2g, u16* __restrict__ dy1g,
    float* __restrict__ biasp, int B, uint64_t* __restrict__ stamps) {
  auto pst = [&](int it, int k) {   // diagnostics: stamps of the first two samples ([blockIdx][16]: 8 per sample)
    if (stamps && it < 2 && threadIdx.x == 0)
      stamps[(size_t)blockIdx.x * 16 + it * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };
  __shared__ __attribute__((aligned(16))) u16 s_w3[B2_W3E];   // W3 B rows; one-sample mode: then the W2 rows
  // dy3 image | dy2 image; walking mode, before the walk: the W2 rows
  __shared__ __attribute__((aligned(16))) u16 s_img[B2_P3E + B2_P2E];
  u16* const s_p3 = s_img;
  u16* const s_p2 = s_img + B2_P3E;
  __shared__ __attribute__((aligned(16))) u16 s_m2[B2_M2E];   // y2 mask rows
  __shared__ float s_red[8 * 128 + 192 + 8 * 32];   // db3 rows per wave | db2 per position tile | db1 per wave
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cls = wid >> 1, py = cls >> 1, px = cls & 1;   // dy1: this wave's parity class

  constexpr int M2_CH = 81 * 8;   // 648
  uint4 vp0, vm0, vm1_;   // the next sample's dy3 chunk and y2 mask chunks
  auto fetch = [&](int b) {
    vp0 = *reinterpret_cast<const uint4*>(dy3g + (size_t)b * 49 * 64 + min(tid, 391) * 8);
    vm0 = *reinterpret_cast<const uint4*>(y2g + (size_t)b * 81 * 64 + min(tid, M2_CH - 1) * 8);
    vm1_ = *reinterpret_cast<const uint4*>(y2g + (size_t)b * 81 * 64 + min(tid + B2_T, M2_CH - 1) * 8);
  };
  if ((int)blockIdx.x < B) fetch(blockIdx.x);
  // ---- W3 B rows k = (t, o) <- W3[o][t][:] (k-major rows of 64 output channels): all 9 chunks per thread in
  // flight at once (a load -> store loop serialised one round trip per chunk: ~4 us of prologue)
  {
    b2_u4 vw3[9];
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      const int c = tid + u * B2_T, k = c >> 3, part = c & 7, t = k >> 6, o = k & 63;
      vw3[u] = *reinterpret_cast<const b2_u4*>(W3 + o * 576 + t * 64 + part * 8);
    }
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      const int c = tid + u * B2_T, k = c >> 3, part = c & 7;
      *reinterpret_cast<b2_u4*>(s_w3 + k * 64 + ((part ^ b2_sw3(k)) << 3)) = vw3[u];
    }
  }
  // W2 B rows (tap, o) <- W2[o][tap][:]: 1024 rows x 32; chunk c of this thread: rows c >> 2 for c = tid + 512 u
  // the class's 16 W2 fragments (k-step s: tap d = s / 4 of the class, channels (s % 4) * 16 ..): the A operand of
  // the transposed dy1 product
  bf16x8 w2f[16];
  auto extract_w2 = [&](const u16* rows) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int d = s >> 2, di = d >> 1, dj = d & 1;
      const int tap = (py + 2 * di) * 4 + (px + 2 * dj);
      w2f[s] = b2_trb<false>(rows, 32, tap * 64 + (s & 3) * 16, 0, lane);
    }
  };
  b2_u4 vw2[8];   // one-sample mode: the W2 rows in registers until dy2 is done
  if constexpr (WALK) {
    {
      b2_u4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = tid + u * B2_T, row = c >> 2, part = c & 3, tap = row >> 6, o = row & 63;
        v[u] = *reinterpret_cast<const b2_u4*>(W2 + o * 512 + tap * 32 + part * 8);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) *reinterpret_cast<b2_u4*>(s_img + (tid + u * B2_T) * 8) = v[u];
    }
    __syncthreads();
    extract_w2(s_img);
    __syncthreads();   // the staging area becomes the images
  } else {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = tid + u * B2_T, row = c >> 2, part = c & 3, tap = row >> 6, o = row & 63;
      vw2[u] = *reinterpret_cast<const b2_u4*>(W2 + o * 512 + tap * 32 + part * 8);
    }
  }
  // dy2 image border (rows / cols outside [1, 10)): zero once, the interior is rewritten for every sample
  for (int c = tid; c < B2_IH * B2_P2W * 8; c += B2_T) {
    const int pix = c >> 3, ch = c & 7, pa = pix / B2_P2W, pb = pix - pa * B2_P2W;
    if (pa < 1 || pa >= 10 || pb < 1 || pb >= 10)
      *reinterpret_cast<uint4*>(s_p2 + b2_px(pix, ch)) = make_uint4(0u, 0u, 0u, 0u);
  }

  // dy3 image border (rows / cols outside [2, 9)): zero once, nothing but the interior is written afterwards
  for (int c = tid; c < B2_IH * B2_P3W * 8; c += B2_T) {
    const int pix = c >> 3, ch = c & 7, pa = pix / B2_P3W, pb = pix - pa * B2_P3W;
    if (pa < 2 || pa >= 9 || pb < 2 || pb >= 9)
      *reinterpret_cast<uint4*>(s_p3 + b2_px(pix, ch)) = make_uint4(0u, 0u, 0u, 0u);
  }
  for (int b = blockIdx.x, it = 0; b < B; b += gridDim.x, ++it) {
    pst(it, 0);
    // opaque zero (per iteration): keeps the unrolled loops' LDS address arithmetic inside the sample loop
    int z0;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z0));
    u16* const p3 = s_p3 + z0;
    u16* const p2 = s_p2 + z0;
    const u16* const w3 = s_w3 + z0;
    const int ln = lane + z0, td = tid + z0;   // laundered per iteration: no hoisted per-lane address sets
    const int hl = ln >> 5;                    // half-wave: channel runs c + 4 of the transposed products
    // ---- this sample's dy3 image interior + y2 mask; db3 channel sums from the loaded chunks (lanes of one
    // channel group by xor shuffles, the waves' rows in order below)
    {
      float part3[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (td < 392) {
        const int pxl = td >> 3, pa = b2_div7(pxl), pb = pxl - pa * 7;
        *reinterpret_cast<uint4*>(p3 + b2_px((pa + 2) * B2_P3W + pb + 2, td & 7)) = vp0;
        const uint32_t wv[4] = {vp0.x, vp0.y, vp0.z, vp0.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) part3[e] = b2_lane(wv[e >> 1], e & 1);
      }
      *reinterpret_cast<uint4*>(s_m2 + td * 8) = vm0;
      if (td + B2_T < M2_CH) *reinterpret_cast<uint4*>(s_m2 + (td + B2_T) * 8) = vm1_;
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) part3[e] += lane_xor(part3[e], o);
      if (ln < 8)
#pragma unroll
        for (int e = 0; e < 8; ++e) s_red[wid * 128 + ln * 8 + e] = part3[e];
    }
    // this lane's dy1 outputs (class cls, tiles 2 (wid & 1) + h, output u = 32 tile + lane % 32): their y1 mask runs
    // (4 x 4 channels from 4 (lane / 32)), requested now, consumed after dy1
    const int mtb = 2 * (wid & 1);
    int d1off[2];
    uint2 mk1[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = min(32 * (mtb + h) + (ln & 31), 99), yy = b2_div10(u), xx = u - 10 * yy;
      d1off[h] = ((2 * yy + py) * 20 + 2 * xx + px) * 32 + 4 * hl;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        mk1[h][g] = *reinterpret_cast<const uint2*>(y1g + (size_t)b * 400 * 32 + d1off[h] + 8 * g);
    }
    __syncthreads();
    pst(it, 1);
    if (b + (int)gridDim.x < B) fetch(b + gridDim.x);

    // ---- dy2^T = W3^T (64 channels) x im2col(dy3)^T (81 positions): waves 0..5 -> (position tile wid % 3, channel
    // tile wid / 3), K = 576 in 36 steps; A = W3 rows (transposing reads), B = dy3-image pixels (16-byte reads).
    // Each lane ends with ONE position and 4 runs of 4 consecutive channels: masked, rounded, then 8-byte writes
    // into the dy2 image AND straight to dy2 in memory; db2 partials by xor shuffles over the 32 positions.
    if (wid < 6) {
      const int pt = wid % 3, ct = wid / 3;
      const int p = 32 * pt + (ln & 31);
      const int pm = p < 81 ? p : 64 + (p & 15);   // padding positions: a real one of the same residue (no conflict)
      const int a = b2_div9(pm), cc = pm - 9 * a;
      b2_f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll 4
      for (int s = 0; s < 36; ++s) {
        const int t = s >> 2, ti = t / 3, tj = t - 3 * ti;
        const bf16x8 wf = b2_trb<true>(w3, 64, 16 * s, 32 * ct, ln);
        const bf16x8 xf = *reinterpret_cast<const bf16x8*>(
            p3 + b2_px((a + 2 - ti) * B2_P3W + (cc + 2 - tj), 2 * (s & 3) + hl));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xf, acc, 0, 0, 0);
      }
      pst(it, 6);
      const bool live = p < 81;
      const int pix = (a + 1) * B2_P2W + cc + 1;
      float sums[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 32 * ct + 8 * g + 4 * hl;
        const uint2 mk = *reinterpret_cast<const uint2*>(s_m2 + pm * 64 + c);
        const uint32_t lo = b2_mask((uint32_t)f2bf(acc[4 * g]) | ((uint32_t)f2bf(acc[4 * g + 1]) << 16), mk.x);
        const uint32_t hi = b2_mask((uint32_t)f2bf(acc[4 * g + 2]) | ((uint32_t)f2bf(acc[4 * g + 3]) << 16), mk.y);
        if (live) {
          *reinterpret_cast<uint2*>(p2 + b2_px(pix, c >> 3) + (c & 7)) = make_uint2(lo, hi);
          *reinterpret_cast<uint2*>(dy2g + ((size_t)b * 81 + p) * 64 + c) = make_uint2(lo, hi);
        }
        const uint32_t ml = live ? 0xFFFFFFFFu : 0u;
        sums[4 * g] = b2_lane(lo & ml, 0);
        sums[4 * g + 1] = b2_lane(lo & ml, 1);
        sums[4 * g + 2] = b2_lane(hi & ml, 0);
        sums[4 * g + 3] = b2_lane(hi & ml, 1);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) sums[r] += lane_xor(sums[r], o);
      if ((ln & 31) == 0)   // channel 32 ct + 8 g + 4 half + j of position tile pt
#pragma unroll
        for (int r = 0; r < 16; ++r) s_red[1024 + pt * 64 + 32 * ct + 8 * (r >> 2) + 4 * hl + (r & 3)] = sums[r];
    }
    __syncthreads();   // dy2 image complete; every dy3-image and W3 read done; db2 / db3 rows complete
    pst(it, 2);
    if (td < 128) {   // db3 (0..63): the 8 waves' rows in order | db2 (64..127): the 3 position tiles in order
      float v = 0.f;
      if (td < 64) {
#pragma unroll
        for (int w = 0; w < 8; ++w) v += s_red[w * 128 + td];
      } else {
        v = (s_red[1024 + td - 64] + s_red[1024 + 64 + td - 64]) + s_red[1024 + 128 + td - 64];
      }
      biasp[(size_t)b * 160 + td] = v;
    }
    if constexpr (!WALK) {   // one-sample mode: the W2 rows over the dead W3 rows, then this wave's fragments
      u16* const w2r = s_w3 + z0;
#pragma unroll
      for (int u = 0; u < 8; ++u) *reinterpret_cast<b2_u4*>(w2r + (td + u * B2_T) * 8) = vw2[u];
      __syncthreads();
      extract_w2(s_w3 + z0);
    }

    // ---- dy1^T = W2sub^T (32 channels) x im2col(dy2)^T (the class's 100 outputs): wave -> class wid / 2, output
    // tiles 2 (wid & 1) + {0, 1}; A = the class's W2 fragments (registers), B = dy2-image pixels. Each lane ends
    // with one output pixel per tile and 4 runs of 4 channels: y1 mask, bf16, 8-byte stores straight to dy1 in
    // memory; db1 partials by xor shuffles over the positions
    {
      b2_f32x16 d0, d1;
#pragma unroll
      for (int r = 0; r < 16; ++r) { d0[r] = 0.f; d1[r] = 0.f; }
      const int u0 = min(32 * mtb + (ln & 31), 99), u1 = min(32 * (mtb + 1) + (ln & 31), 99);
      const int y0 = b2_div10(u0), x0 = u0 - 10 * y0, y1 = b2_div10(u1), x1 = u1 - 10 * y1;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int d = s >> 2, di = d >> 1, dj = d & 1, ch = 2 * (s & 3) + hl;
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(p2 + b2_px((y0 + 1 - di) * B2_P2W + x0 + 1 - dj, ch));
        const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(p2 + b2_px((y1 + 1 - di) * B2_P2W + x1 + 1 - dj, ch));
        d0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2f[s], a0, d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2f[s], a1, d1, 0, 0, 0);
      }
      pst(it, 3);
      float sums[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) sums[r] = 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool live = 32 * (mtb + h) + (ln & 31) < 100;
        const uint32_t ml = live ? 0xFFFFFFFFu : 0u;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float e0 = h ? d1[4 * g] : d0[4 * g], e1 = h ? d1[4 * g + 1] : d0[4 * g + 1];
          const float e2 = h ? d1[4 * g + 2] : d0[4 * g + 2], e3 = h ? d1[4 * g + 3] : d0[4 * g + 3];
          const uint32_t lo = b2_mask((uint32_t)f2bf(e0) | ((uint32_t)f2bf(e1) << 16), mk1[h][g].x) & ml;
          const uint32_t hi = b2_mask((uint32_t)f2bf(e2) | ((uint32_t)f2bf(e3) << 16), mk1[h][g].y) & ml;
          if (live) *reinterpret_cast<uint2*>(dy1g + (size_t)b * 400 * 32 + d1off[h] + 8 * g) = make_uint2(lo, hi);
          sums[4 * g] += b2_lane(lo, 0);
          sums[4 * g + 1] += b2_lane(lo, 1);
          sums[4 * g + 2] += b2_lane(hi, 0);
          sums[4 * g + 3] += b2_lane(hi, 1);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) sums[r] += lane_xor(sums[r], o);
      if ((ln & 31) == 0)   // channel 8 g + 4 half + j, this wave's two tiles of its class
#pragma unroll
        for (int r = 0; r < 16; ++r) s_red[1024 + 192 + wid * 32 + 8 * (r >> 2) + 4 * hl + (r & 3)] = sums[r];
    }
    __syncthreads();   // db1 rows complete (and every wave past its dy2-image reads before the next sample)
    if (td < 32) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += s_red[1024 + 192 + w * 32 + td];
      biasp[(size_t)b * 160 + 128 + td] = v;
    }
    pst(it, 5);
  }
}

}  // namespace aca

// grid: min(B, max_wg) workgroups walking the samples (max_wg <= 0: one per sample)
extern "C" hipError_t aca_cnn_trunk_bwd2(const uint16_t* dy3, const uint16_t* W3, const uint16_t* y2,
                                         const uint16_t* W2, const uint16_t* y1, uint16_t* dy2, uint16_t* dy1,
                                         float* biasp, int B, uint64_t* stamps, int max_wg, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  for (const void* p : {(const void*)dy3, (const void*)W3, (const void*)y2, (const void*)W2, (const void*)y1,
                        (const void*)dy2, (const void*)dy1})
    if (reinterpret_cast<uintptr_t>(p) % 16) return hipErrorInvalidValue;
  const int grid = max_wg > 0 && max_wg < B ? max_wg : B;
  if (grid < B)
    aca::cnn_trunk_bwd2_kernel<true><<<grid, aca::B2_T, 0, stream>>>(dy3, W3, y2, W2, y1, dy2, dy1, biasp, B, stamps);
  else
    aca::cnn_trunk_bwd2_kernel<false><<<grid, aca::B2_T, 0, stream>>>(dy3, W3, y2, W2, y1, dy2, dy1, biasp, B, stamps);
  return hipGetLastError();
}
