// Fused Nature-CNN trunk for rollout inference: conv1 -> conv2 -> conv3 of ONE env per workgroup, activations in
// LDS, one launch for the whole trunk (SURVEY §2.4 K03, §7.5 hard part 1: at 32 envs per GPU the rollout is
// latency-bound, so the three per-layer GEMM launches -- each a couple of memory round trips plus a kernel
// boundary -- collapse into one launch whose layers hand off through LDS).
//
//   obs uint8 [4, 84, 84] --LDS (bf16 integers 0..255, exact)--> conv1 (K 256 = (c, i, j), MFMA 16x16x32) --> y1 [400, 32] bf16 (LDS + global)
//                                  conv2 (K 512 = (i, j, c))                  --> y2 [81, 64]  bf16 (LDS + global)
//                                  conv3 (K 576 = (i, j, c))                  --> y3 [49, 64]  bf16 (global)
//
// With `shift_out` (rollout) the kernel also writes frames 1..3 of each observation as frames 0..2 of the next
// one -- the frame-stack shift of the env step, from registers it already holds.
// y1 / y2 / y3 are also written to global memory: they are the learner's saved activations (the A2C learner reuses
// the rollout's forward pass) and y3 feeds the fc GEMM. Weights are the bf16 shadow of the parameter slab in the
// engine's layouts (W1 [32][256] OIHW, W2 [64][512] / W3 [64][576] OHWI); conv1 weights are staged in LDS, conv2/3
// B fragments are streamed from L2 straight into registers (each is used once per wave), all issued before the
// first MFMA of the layer (W2's at kernel entry, W3's at conv2 entry, so their latency hides behind the previous
// layer). The frames are staged as exact bf16 integers and the 1/255 scale is applied to the fp32 accumulator in
// the conv1 epilogue (one conversion per pixel instead of one per im2col element). Work split: conv1 -- waves take M tiles round-robin and both N tiles; conv2/3 -- wave w
// owns output-channel tile w for every M tile, so every B fragment is loaded exactly once per workgroup.
#include <cstdlib>

#include "common.h"
#include "cnn_head.h"
#include "pong_env.h"

namespace aca {

constexpr int T_THREADS = 256;
constexpr int OBS_BYTES = 4 * 84 * 84;       // 28224
constexpr int W1_LD = 256 + 8;               // padded LDS row (bf16)
constexpr int Y1_ROWS = 400, Y1_C = 32;
constexpr int Y2_ROWS = 81, Y2_C = 64;
// LDS pixel strides (bf16 elements) padded against ds_read_b128 bank conflicts of the stride-2 / stride-1 im2col
// fragment reads (64 -> 80 B and 128 -> 160 B: 4.2x / 3.3x -> 1.8x of the conflict-free cycle count, simulated
// over every fragment read of the two layers with the gfx950 b128 lane groups)
constexpr int Y1_LD = 40, Y2_LD = 80;
constexpr int Y3_ROWS = 49, Y3_C = 64;

typedef short short8v __attribute__((ext_vector_type(8)));

// 4 uint8 -> 4 bf16 (exact: integers below 256 have at most 8 significant bits)
__device__ __forceinline__ uint2 u8x4_to_bf16(uint32_t w) {
  uint2 r;
  r.x = (__float_as_uint((float)(w & 0xFF)) >> 16) | (__float_as_uint((float)((w >> 8) & 0xFF)) & 0xFFFF0000u);
  r.y = (__float_as_uint((float)((w >> 16) & 0xFF)) >> 16) | (__float_as_uint((float)(w >> 24)) & 0xFFFF0000u);
  return r;
}

// optional phase timestamps (s_memrealtime, 100 MHz) for in-kernel latency analysis; null in production
__device__ __forceinline__ void stamp(uint64_t* st, int slot) {
  if (st && threadIdx.x == 0) st[(size_t)blockIdx.x * 16 + slot] = __builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------------------------------------------------------------
// One observation copied global -> LDS by the LDS-DMA path (global_load_lds_dwordx4: no registers, tracked by the vm
// counter), padded to whole 1 KB wave copies.
constexpr int TP_OBS_PAD = 28 * 1024;   // one observation (28224 B) padded to whole 1 KB wave copies

// Per-env activation images in LDS (trunk_env_convs), conflict-free for the conv2 / conv3 A-fragment reads: a
// ds_read_b128 lane group holds 8 output positions at one channel chunk and 8 at the next; with the pixel strides
// Y1_LD = 40 (5 bank quads) / Y2_LD = 80 (10) they land in 16 distinct quads when the image's row pitch satisfies
// pitch * stride == output width * stride (mod 16 quads) for the stride-2 (conv2) / stride-1 (conv3) walk: y1 rows of
// 25 pixels for the 9-wide conv2 output (2 x 25 = 2 x 9 + 32), y2 rows of 15 for the 7-wide conv3 output
// (15 = 7 + 8) (tests/test_lds_layouts_cpu.py). Tight 20 / 9 pitches: 1.8 / 1.75 LDS cycles per read. y2 lives in
// the staged observation's bytes (dead after conv1), which keeps two workgroups per CU.
constexpr int E1_W = 25, E2_W = 15;
constexpr int E1_ELEMS = 20 * E1_W * Y1_LD;   // 20000 u16 = 40 KB
constexpr int E2_ELEMS = 9 * E2_W * Y2_LD;    // 10800 u16 = 21.6 KB
static_assert(E2_ELEMS * 2 <= TP_OBS_PAD, "y2 image aliases the staged observation");

__device__ __forceinline__ void trunk_obs_dma(const uint8_t* __restrict__ src, uint8_t* dst_lds) {
  // 28 wave-copies of 64 x 16 B: wave w copies blocks w, w + (waves), ...; lanes past the observation read its
  // last chunk again (their bytes land in the padding)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int blk = wid; blk < TP_OBS_PAD / 1024; blk += nw) {
    const int c = min(blk * 64 + lane, OBS_BYTES / 16 - 1);
    uint8_t* base = dst_lds + blk * 1024;   // wave-uniform LDS base (lane i lands at base + 16 i)
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(src) + c,
                                     (__attribute__((address_space(3))) void*)(base), 16, 0, 0);
  }
}

// Frames 0..2, input rows [IA, IB) of one observation to the same offsets of the LDS image (the rollout step renders
// frame 3 itself): per frame ceil((IB - IA) * 84 / 1024) wave copies, the lanes past a frame's range masked off
// (their slots would be the next frame's first rows).
template <int IA, int IB>
__device__ __forceinline__ void obs_rows_dma(const uint8_t* __restrict__ src, uint8_t* dst_lds) {
  constexpr int NCH = (IB - IA) * 84 / 16, NCOPY = (NCH + 63) / 64, C0 = IA * 84 / 16;
  static_assert(IA * 84 % 16 == 0 && (IB - IA) * 84 % 16 == 0, "16-byte rows ranges");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int k = wid; k < 3 * NCOPY; k += nw) {
    const int f = k / NCOPY, blk = k - f * NCOPY;
    const int c = f * (FRAME / 16) + C0 + blk * 64 + lane;
    uint8_t* base = dst_lds + f * FRAME + IA * 84 + blk * 1024;
    if (blk * 64 + lane < NCH)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(src) + c,
                                       (__attribute__((address_space(3))) void*)(base), 16, 0, 0);
  }
}

// ------------------------------------------------------------------------------------------------------------
// Per-env trunk, lean-LDS form: the observation is staged as its uint8 bytes by LDS-DMA (28 KB instead of 56 KB of
// bf16, no staging registers) and the conv1 weight fragments come straight from L2 into registers (no 17 KB W1
// stage), so a workgroup needs 74 KB of LDS and TWO fit a CU: while one sample waits on a barrier or a memory round
// trip the other one's MFMAs run (the 118 KB form above runs one workgroup -- one wave per SIMD -- per CU). conv1
// converts the pixels to exact bf16 integers on the fly; same MFMA order and epilogues: bit-identical outputs.
// The conv chain is a device function shared with the per-env fused rollout step (pong_fused_env_step_kernel).
// conv1 / conv2 weight fragments of this wave (output-channel tile wid for conv2)
__device__ __forceinline__ void trunk_env_w1(const u16* __restrict__ W1, bf16x8 (&bw)[2][8]) {
  const int lane = threadIdx.x & 63, l16 = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      bw[nt][ks] = *reinterpret_cast<const bf16x8*>(W1 + (nt * 16 + l16) * 256 + ks * 32 + lg * 8);
}
__device__ __forceinline__ void trunk_env_w2(const u16* __restrict__ W2, bf16x8 (&bw2)[16]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, l16 = lane & 15, lg = lane >> 4;
  const int n2 = wid * 16 + l16;
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) bw2[ks] = *reinterpret_cast<const bf16x8*>(W2 + n2 * 512 + ks * 32 + lg * 8);
}
__device__ __forceinline__ void trunk_env_w12(const u16* __restrict__ W1, const u16* __restrict__ W2,
                                              bf16x8 (&bw)[2][8], bf16x8 (&bw2)[16]) {
  trunk_env_w1(W1, bw);
  trunk_env_w2(W2, bw2);
}

// Fragment-ordered weight copies (written by the optimiser step, optim.hip OptTrans): fragment (tile, k-step) of lane l at ((tile * KS + ks) * 64 +
// l) * 8 -- a wave's fragment load is ONE contiguous 1 KB read. The row-major fragment loads above touch 16 rows x
// 64 bytes per wave instruction, which the L2 -> CU path serves at 16 B/clk/CU against ~60 for whole-line wave loads
// (profiles/r4_l2_stream_probe.txt).
__device__ __forceinline__ void frag_w1(const u16* __restrict__ F1, bf16x8 (&bw)[2][8]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) bw[nt][ks] = *reinterpret_cast<const bf16x8*>(F1 + ((nt * 8 + ks) * 64 + lane) * 8);
}
__device__ __forceinline__ void frag_w2(const u16* __restrict__ F2, bf16x8 (&bw2)[16]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) bw2[ks] = *reinterpret_cast<const bf16x8*>(F2 + ((wid * 16 + ks) * 64 + lane) * 8);
}
__device__ __forceinline__ void frag_w3(const u16* __restrict__ F3, bf16x8 (&bw3)[18]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int ks = 0; ks < 18; ++ks) bw3[ks] = *reinterpret_cast<const bf16x8*>(F3 + ((wid * 18 + ks) * 64 + lane) * 8);
}

// conv2 / conv3 fragments of this wave from the row-major weights or (FRAG) their fragment-ordered copies
template <bool FRAG>
__device__ __forceinline__ void load_w2(const u16* __restrict__ W2, bf16x8 (&bw2)[16]) {
  if constexpr (FRAG) frag_w2(W2, bw2);
  else trunk_env_w2(W2, bw2);
}
template <bool FRAG>
__device__ __forceinline__ void load_w3(const u16* __restrict__ W3, bf16x8 (&bw3)[18]) {
  if constexpr (FRAG) {
    frag_w3(W3, bw3);
  } else {
    const int lane = threadIdx.x & 63, n2 = (threadIdx.x >> 6) * 16 + (lane & 15), lg = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) bw3[ks] = *reinterpret_cast<const bf16x8*>(W3 + n2 * 576 + ks * 32 + lg * 8);
  }
}

// ------------------------------------------------------------------------------------------------------------
// Output rows computed / stored by part PART of an env's trunk: -1 the whole env (one workgroup per env), 0 / 1 the
// two halves of the split rollout step (pong_fused_env_step_kernel<A1, 2>): conv3 rows [c3a, c3b), the conv2 / conv1 /
// input rows of their receptive field (recomputed by both halves where they overlap), and the rows each half OWNS
// (stores) -- every y1 / y2 row and every input row of the next observation has exactly one owner.
template <int PART>
struct EnvRows {
  static constexpr int c3a = PART == 1 ? 3 : 0, c3b = PART == 0 ? 3 : 7;   // half 0 (it also commits) the smaller
  static constexpr int c2a = c3a, c2b = c3b + 2;          // conv2 rows [c2a, c2b)
  static constexpr int c1a = 2 * c2a, c1b = 2 * c2b + 2;  // conv1 rows [c1a, c1b)
  static constexpr int ia = 4 * c1a, ib = 4 * c1b + 4;    // input rows [ia, ib)
  static constexpr int o1a = PART == 1 ? 10 : 0, o1b = PART == 0 ? 10 : 20;   // owned y1 rows
  static constexpr int o2a = PART == 1 ? 4 : 0, o2b = PART == 0 ? 4 : 9;      // owned y2 rows
  static constexpr int oia = PART == 1 ? 40 : 0, oib = PART == 0 ? 40 : 84;   // owned input rows (16-byte aligned)
  static constexpr int P1 = (c1b - c1a) * 20, T1 = (P1 + 15) / 16;   // conv1 positions / M tiles
  static constexpr int P2 = (c2b - c2a) * 9, T2 = (P2 + 15) / 16;
  static constexpr int P3 = (c3b - c3a) * 7, T3 = (P3 + 15) / 16;
  static_assert(c1b <= 20 && ib <= 84 && oia * 84 % 16 == 0, "row ranges");
};
static_assert(EnvRows<-1>::P1 == 400 && EnvRows<-1>::P2 == 81 && EnvRows<-1>::P3 == 49, "whole env");
static_assert(EnvRows<0>::T1 == 15 && EnvRows<1>::T1 == 18 && EnvRows<0>::ib == 52 && EnvRows<1>::ia == 24 &&
              EnvRows<0>::c1b >= EnvRows<0>::o1b && EnvRows<1>::c1a <= EnvRows<1>::o1a &&
              EnvRows<0>::c2b >= EnvRows<0>::o2b && EnvRows<1>::c2a <= EnvRows<1>::o2a &&
              EnvRows<0>::ib >= EnvRows<0>::oib && EnvRows<1>::ia <= EnvRows<1>::oia, "halves own what they compute");
constexpr int E1P_ELEMS = 14 * E1_W * Y1_LD;   // the y1 image of a half (at most 14 conv1 rows): 28 KB

// conv1 -> conv2 -> conv3 of env e (part PART) from its staged uint8 observation (s_obs8, complete behind a barrier;
// image rows are global, the y1 / y2 images hold the part's rows from c1a / c2a); bw / bw2: this wave's conv1 / conv2
// weight fragments (already in registers), W3's are loaded after conv1. Every output's MFMA order is the same in
// every part: the halves are bit-identical to the whole-env form.
template <int PART, bool FRAG = false>
__device__ __forceinline__ void trunk_env_convs(const uint8_t* __restrict__ s_obs8, u16* __restrict__ s_y1,
                                                u16* __restrict__ s_y2, int e, const bf16x8 (&bw)[2][8],
                                                const bf16x8 (&bw2)[16], const u16* __restrict__ W3, float bias0,
                                                float bias1, float bias2, float bias3, u16* __restrict__ y1g,
                                                u16* __restrict__ y2g, u16* __restrict__ y3g, float scale,
                                                uint64_t* __restrict__ stamps = nullptr) {
  using R = EnvRows<PART>;
  constexpr int NW = 4;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const int n2 = wid * 16 + l16;
  // ---------------------------------------------------------------- conv1: M P1 (T1 tiles), N 32 (2), K 256 (8)
  for (int mt = wid; mt < R::T1; mt += NW) {
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const int m = min(mt * 16 + l16, R::P1 - 1);
    const int oh = R::c1a + m / 20, ow = m % 20;   // global conv1 row
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int k = ks * 32 + lg * 8;
      const int c = k >> 6, i = (k >> 3) & 7;
      const uint8_t* p = s_obs8 + (c * 84 + oh * 4 + i) * 84 + ow * 4;   // 4-byte aligned
      const uint2 lo = u8x4_to_bf16(*reinterpret_cast<const uint32_t*>(p));
      const uint2 hi = u8x4_to_bf16(*reinterpret_cast<const uint32_t*>(p + 4));
      const bf16x8 a = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[0][ks], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[1][ks], acc1, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = mt * 16 + lg * 4 + r;   // local position
      if (R::P1 % 16 == 0 || row < R::P1) {
        const u16 v0 = f2bf(fmaxf(acc0[r] * scale + bias0, 0.f));
        const u16 v1 = f2bf(fmaxf(acc1[r] * scale + bias1, 0.f));
        const int lr = row / 20, col = row % 20;
        const int px1 = lr * E1_W + col;
        s_y1[px1 * Y1_LD + l16] = v0;
        s_y1[px1 * Y1_LD + 16 + l16] = v1;
        if (PART < 0 || (R::c1a + lr >= R::o1a && R::c1a + lr < R::o1b)) {
          const size_t g = (size_t)e * Y1_ROWS + R::c1a * 20 + row;
          y1g[g * Y1_C + l16] = v0;
          y1g[g * Y1_C + 16 + l16] = v1;
        }
      }
    }
  }
  bf16x8 bw3[18];
  load_w3<FRAG>(W3, bw3);
  __syncthreads();
  stamp(stamps, 5);
  // ---------------------------------------------------------------- conv2: M P2 (T2 tiles), N 64 (wave = N tile), K 512
  {
    floatx4 acc[R::T2];
#pragma unroll
    for (int mt = 0; mt < R::T2; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int k = ks * 32 + lg * 8;
      const int i = k >> 7, j = (k >> 5) & 3, c0 = k & 31;
#pragma unroll
      for (int mt = 0; mt < R::T2; ++mt) {
        const int m = min(mt * 16 + l16, R::P2 - 1);
        const int oh = m / 9, ow = m - oh * 9;   // local conv2 row (its y1 rows start at local 2 * oh)
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(s_y1 + ((oh * 2 + i) * E1_W + ow * 2 + j) * Y1_LD + c0);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw2[ks], acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < R::T2; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r;
        if (row < R::P2) {
          const u16 v = f2bf(fmaxf(acc[mt][r] + bias2, 0.f));
          const int lr = row / 9;
          s_y2[(lr * E2_W + row % 9) * Y2_LD + n2] = v;
          if (PART < 0 || (R::c2a + lr >= R::o2a && R::c2a + lr < R::o2b))
            y2g[((size_t)e * Y2_ROWS + R::c2a * 9 + row) * Y2_C + n2] = v;
        }
      }
    }
  }
  __syncthreads();
  stamp(stamps, 6);
  // ---------------------------------------------------------------- conv3: M P3 (T3 tiles), N 64 (wave = N tile), K 576
  {
    floatx4 acc[R::T3];
#pragma unroll
    for (int mt = 0; mt < R::T3; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int k = ks * 32 + lg * 8;
      const int i = k / 192, j = (k >> 6) % 3, c0 = k & 63;
#pragma unroll
      for (int mt = 0; mt < R::T3; ++mt) {
        const int m = min(mt * 16 + l16, R::P3 - 1);
        const int oh = m / 7, ow = m - oh * 7;   // local conv3 row = local y2 row
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(s_y2 + ((oh + i) * E2_W + ow + j) * Y2_LD + c0);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw3[ks], acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < R::T3; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r;
        if (row < R::P3)
          y3g[((size_t)e * Y3_ROWS + R::c3a * 7 + row) * Y3_C + n2] = f2bf(fmaxf(acc[mt][r] + bias3, 0.f));
      }
    }
  }
  stamp(stamps, 7);
}

// W1 [32][256] bf16 (16 KB) copied global -> LDS by the LDS-DMA path, each 512-byte row's 16-byte chunks
// XOR-swizzled by (row & 15) so the fragment reads (16 rows at one column per lane group) are conflict-free; lane i
// of a wave copy lands at base + 16 i, so the swizzle is applied to the SOURCE chunk it fetches.
__device__ __forceinline__ void w1_lds_dma(const u16* __restrict__ W1, u16* dst_lds) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int blk = wid; blk < 16; blk += nw) {
    const int q = blk * 64 + lane, row = q >> 5, lc = (q & 31) ^ (row & 15);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(W1) + row * 32 + lc,
                                     (__attribute__((address_space(3))) void*)(dst_lds + blk * 512), 16, 0, 0);
  }
}
__device__ __forceinline__ void w1_frags_from_lds(const u16* __restrict__ s_w, bf16x8 (&bw)[2][8]) {
  const int lane = threadIdx.x & 63, l16 = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int row = nt * 16 + l16, pc = (ks * 4 + lg) ^ (row & 15);
      bw[nt][ks] = *reinterpret_cast<const bf16x8*>(s_w + row * 256 + pc * 8);
    }
}

// ------------------------------------------------------------------------------------------------------------
// Per-env trunk, bf16-staged form (the learner's minibatch forward): a lean form (retired) converted every observation
// byte to bf16 in conv1's inner loop, ~3.6 times per byte (the 8x8 / stride-4 windows overlap) -- conv1 is then
// vector-issue bound (2.4k VALU vs 0.27k MFMA instructions per wave, profiles/r4_trunk_mix.txt). Here the bytes are
// converted ONCE into a bf16 image (56 KB: still two workgroups per CU), conv1's outputs wait in registers until
// every wave is done with the image, and y1 (unpadded 20 x 20 x 64 B, columns even-then-odd, chunk XOR-swizzled:
// e1t_addr) + y2 (padded, conflict-free) then reuse its bytes. y1 / y2 / y3 leave through LDS as 16-byte rows.
// Same MFMA order per output as every other trunk form: bit-identical activations.
// ------------------------------------------------------------------------------------------------------------
constexpr int E1T_ELEMS = 20 * 20 * Y1_C;   // 12800 u16
__device__ __forceinline__ int e1t_addr(int h, int w, int ch) {
  return (h * 20 + (w & 1) * 10 + (w >> 1)) * Y1_C + (((ch >> 3) ^ (((h >> 1) & 1) << 1)) << 3) + (ch & 7);
}
constexpr int OB16_ELEMS = 4 * 84 * 84;     // 28224 u16
static_assert(E1T_ELEMS + E2_ELEMS <= OB16_ELEMS && Y3_ROWS * Y3_C <= E1T_ELEMS, "y1 + y2 (+ y3) reuse the image");

template <bool FRAG>
__global__ void __launch_bounds__(256) cnn_trunk_fwd_s16_kernel(
    const uint8_t* __restrict__ obs, const u16* __restrict__ W1, const float* __restrict__ b1,
    const u16* __restrict__ W2, const float* __restrict__ b2, const u16* __restrict__ W3,
    const float* __restrict__ b3, u16* __restrict__ y1g, u16* __restrict__ y2g, u16* __restrict__ y3g,
    float scale, uint8_t* __restrict__ shift_out, const int64_t* __restrict__ obs_idx) {
  __shared__ __attribute__((aligned(16))) u16 s_img[OB16_ELEMS];
  u16* const s_y1 = s_img;               // after conv1
  u16* const s_y2 = s_img + E1T_ELEMS;   // after conv1
  u16* const s_y3 = s_img;               // after conv2 (y1 dead)
  const int e = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const int n2 = wid * 16 + l16;
  // ---------------------------------------------------------------- loads: observation bytes, conv1 fragments
  constexpr int NCH = OBS_BYTES / 16, PER = (NCH + 255) / 256;   // 1764 chunks, 7 per thread
  const uint4* src = reinterpret_cast<const uint4*>(obs + (size_t)(obs_idx ? obs_idx[e] : e) * OBS_BYTES);
  uint4 v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) v[u] = src[min(tid + u * 256, NCH - 1)];
  bf16x8 bw[2][8];
  if constexpr (FRAG) frag_w1(W1, bw);
  else trunk_env_w1(W1, bw);
  const float bias0 = b1[l16], bias1 = b1[16 + l16], bias2 = b2[n2], bias3 = b3[n2];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = tid + u * 256;
    if (i < NCH) {
      const uint2 a = u8x4_to_bf16(v[u].x), b = u8x4_to_bf16(v[u].y);
      const uint2 c = u8x4_to_bf16(v[u].z), d = u8x4_to_bf16(v[u].w);
      uint4* dst = reinterpret_cast<uint4*>(s_img) + 2 * i;
      dst[0] = make_uint4(a.x, a.y, b.x, b.y);
      dst[1] = make_uint4(c.x, c.y, d.x, d.y);
      if (shift_out && i >= NCH / 4)   // rollout: frames 1..3 become frames 0..2 of the next observation
        reinterpret_cast<uint4*>(shift_out + (size_t)e * OBS_BYTES)[i - NCH / 4] = v[u];
    }
  }
  __syncthreads();
  // ---------------------------------------------------------------- conv1: M 400 (25 tiles), N 32 (2), K 256 (8);
  // the outputs stay in registers (bf16 pairs) until every wave is done reading the image
  constexpr int MT1 = 7;   // tiles per wave (wave w: w, w + 4, ...; 7, 6, 6, 6)
  uint32_t yr[MT1][4];
#pragma unroll
  for (int q = 0; q < MT1; ++q) {
    const int mt = wid + 4 * q;
    if (mt < 25) {
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const int m = mt * 16 + l16;
      const int oh = m / 20, ow = m - oh * 20;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int k = ks * 32 + lg * 8;
        const int c = k >> 6, i = (k >> 3) & 7;
        const u16* p = s_img + (c * 84 + oh * 4 + i) * 84 + ow * 4;   // 8-byte aligned
        const uint2 lo = *reinterpret_cast<const uint2*>(p), hi = *reinterpret_cast<const uint2*>(p + 4);
        const bf16x8 a = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[0][ks], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[1][ks], acc1, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        yr[q][r] = (uint32_t)f2bf(fmaxf(acc0[r] * scale + bias0, 0.f)) |
                   ((uint32_t)f2bf(fmaxf(acc1[r] * scale + bias1, 0.f)) << 16);
    }
  }
  bf16x8 bw2[16];
  load_w2<FRAG>(W2, bw2);
  __syncthreads();   // the image is dead
#pragma unroll
  for (int q = 0; q < MT1; ++q) {
    const int mt = wid + 4 * q;
    if (mt < 25)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r, h = row / 20, w = row - h * 20;
        s_y1[e1t_addr(h, w, l16)] = (u16)(yr[q][r] & 0xFFFFu);
        s_y1[e1t_addr(h, w, 16 + l16)] = (u16)(yr[q][r] >> 16);
      }
  }
  __syncthreads();
  // y1 -> global as 16-byte chunks (pixel p, channel chunk cq) while conv2 runs
  for (int i = tid; i < Y1_ROWS * 4; i += 256) {
    const int p = i >> 2, cq = i & 3, h = p / 20, w = p - h * 20;
    *reinterpret_cast<uint4*>(y1g + ((size_t)e * Y1_ROWS + p) * Y1_C + cq * 8) =
        *reinterpret_cast<const uint4*>(s_y1 + e1t_addr(h, w, cq * 8));
  }
  // ---------------------------------------------------------------- conv2: M 81 (6 tiles), N 64 (wave = N tile), K 512
  {
    floatx4 acc[6];
#pragma unroll
    for (int mt = 0; mt < 6; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int k = ks * 32 + lg * 8;
      const int i = k >> 7, j = (k >> 5) & 3, c0 = k & 31;
#pragma unroll
      for (int mt = 0; mt < 6; ++mt) {
        const int m = min(mt * 16 + l16, Y2_ROWS - 1);
        const int oh = m / 9, ow = m - oh * 9;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(s_y1 + e1t_addr(oh * 2 + i, ow * 2 + j, c0));
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw2[ks], acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 6; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r;
        if (row < Y2_ROWS)
          s_y2[((row / 9) * E2_W + row % 9) * Y2_LD + n2] = f2bf(fmaxf(acc[mt][r] + bias2, 0.f));
      }
  }
  bf16x8 bw3[18];
  load_w3<FRAG>(W3, bw3);
  __syncthreads();   // y2 complete; y1 dead (its global copy read it before the barrier)
  for (int i = tid; i < Y2_ROWS * 8; i += 256) {
    const int p = i >> 3, cq = i & 7;
    *reinterpret_cast<uint4*>(y2g + ((size_t)e * Y2_ROWS + p) * Y2_C + cq * 8) =
        *reinterpret_cast<const uint4*>(s_y2 + ((p / 9) * E2_W + p % 9) * Y2_LD + cq * 8);
  }
  // ---------------------------------------------------------------- conv3: M 49 (4 tiles), N 64 (wave = N tile), K 576
  {
    floatx4 acc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int k = ks * 32 + lg * 8;
      const int i = k / 192, j = (k >> 6) % 3, c0 = k & 63;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int m = min(mt * 16 + l16, Y3_ROWS - 1);
        const int oh = m / 7, ow = m - oh * 7;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(s_y2 + ((oh + i) * E2_W + ow + j) * Y2_LD + c0);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw3[ks], acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r;
        if (row < Y3_ROWS) s_y3[row * Y3_C + n2] = f2bf(fmaxf(acc[mt][r] + bias3, 0.f));
      }
  }
  __syncthreads();
  for (int i = tid; i < Y3_ROWS * 8; i += 256)
    reinterpret_cast<uint4*>(y3g + (size_t)e * Y3_ROWS * Y3_C)[i] = reinterpret_cast<const uint4*>(s_y3)[i];
}

// ------------------------------------------------------------------------------------------------------------
// Row-split trunk: 7 workgroups per env, workgroup r computes the receptive field of conv3 output row r only
// (conv2 rows r..r+2, conv1 rows 2r..2r+7, input rows 8r..8r+35). The per-env kernel above keeps one CU busy per
// env (32 of 256 CUs at the bench's 32 envs) and its layers run at one wave per SIMD; here 7x the CUs each do
// ~1/3 of the work (the overlapping conv1/conv2 rows are recomputed: 56 conv1 rows for 20), so the step latency
// falls to about a third. Each output row of y1 / y2 / y3 has exactly ONE owner workgroup that stores it (the
// recomputed copies are bit-identical anyway: same operands, same MFMA order):
//   y1 rows [ceil(20r/7), ceil(20(r+1)/7)), y2 row r (+ rows 7, 8 for r = 6), y3 row r,
//   input rows [12r, 12r + 12) for the frame-stack outputs (shift_out: frames 1..3 -> 0..2 of the next
//   observation; copy_out: all 4 frames, the rollover of the last observation into slot 0 of the next rollout).
// ------------------------------------------------------------------------------------------------------------
constexpr int TR_ROWS = 7;                 // workgroups per env (conv3 output rows)
constexpr int TR_IN_ROWS = 36;             // staged input rows per frame
constexpr int TR_C1_ROWS = 8;              // conv1 rows per workgroup
constexpr int TR_C1_POS = TR_C1_ROWS * 20; // 160 = 10 M tiles
constexpr int TR_C2_POS = 27;              // 3 conv2 rows x 9
constexpr int TR_IN_ELEMS = 768 * 16;   // 4 x 36 x 84 = 12096 bf16, padded to 3 x 256 16-byte chunks x 2

__device__ __forceinline__ int tr_y1_own_begin(int r) { return (20 * r + 6) / 7; }

// conv1 -> conv3 of row workgroup (e, r) from its staged input rows (s_in: 4 frames x 36 rows of bf16 pixel values,
// complete) and the conv1 weights (s_w1, complete); stores the owned y1 / y2 rows and its y3 row. Shared by the
// trunk kernel and the fused policy/env + trunk kernel.
// WMODE (when the conv2 / conv3 weight fragments are requested): 0 at entry (the staging barrier waited for obs +
// W1 only), 1 after conv1's MFMAs (trunk mode 2), 2 W2 at entry and W3 after conv1's MFMAs, 3 W2 already requested
// by the caller and W3 after conv1's MFMAs (the fused step: W2's 64 KB per workgroup lands during the render)
template <int WMODE, bool FRAG = false>
__device__ __forceinline__ void trunk_rows_compute(const u16* __restrict__ s_in, const u16* __restrict__ s_w1,
                                                   u16* __restrict__ s_y1, u16* __restrict__ s_y2, int e, int r,
                                                   const float bias1a, const float bias1b, const float bias2,
                                                   const float bias3, const u16* __restrict__ W2,
                                                   const u16* __restrict__ W3, u16* __restrict__ y1g,
                                                   u16* __restrict__ y2g, u16* __restrict__ y3g, float scale,
                                                   uint64_t* __restrict__ stamps, bf16x8 (&bw2)[16],
                                                   bf16x8 (&bw3)[18]) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const int n2 = wid * 16 + l16;
  if constexpr (WMODE == 0 || WMODE == 2) {
    load_w2<FRAG>(W2, bw2);
  }
  if constexpr (WMODE == 0) {
    load_w3<FRAG>(W3, bw3);
  }

  // ---------------------------------------------------------------- conv1: 160 positions (10 M tiles) x 32 x K 256
  {
    bf16x8 bw1[2][8];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
        bw1[nt][ks] = *reinterpret_cast<const bf16x8*>(s_w1 + (nt * 16 + l16) * W1_LD + ks * 32 + lg * 8);
    const float bias0 = bias1a, bias1 = bias1b;
    // im2col A fragments of M tile mt: 8 k-steps, lane (l16, lg) reads one 8-pixel patch row (16 bytes, 8-byte
    // aligned: two 8-byte halves)
    auto c1_load = [&](int mt, bf16x8 (&a)[8]) {
      const int m = mt * 16 + l16;
      const int oh = m / 20, ow = m - oh * 20;      // local conv1 row, column
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int k = ks * 32 + lg * 8;
        const int c = k >> 6, i = (k >> 3) & 7;
        const u16* p = s_in + (c * TR_IN_ROWS + oh * 4 + i) * 84 + ow * 4;
        const uint2 lo = *reinterpret_cast<const uint2*>(p), hi = *reinterpret_cast<const uint2*>(p + 4);
        a[ks] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
    };
    // 10 M tiles over 4 waves (3, 3, 2, 2): a fixed trip count with a guard, no global stores in the loop (they
    // would sit in the vm counter in front of the W3 fragment loads that conv2 waits for). The next tile's A
    // fragments are read while this tile's MFMAs run (two register buffers): read one k-step ahead, as the
    // compiler schedules it on its own, every MFMA pair waited out an LDS round trip.
    bf16x8 abuf[2][8];
    c1_load(wid, abuf[0]);
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      const int mt = wid + 4 * it;
      if (mt >= TR_C1_POS / 16) break;
      if (it < 2 && mt + 4 < TR_C1_POS / 16) c1_load(mt + 4, abuf[(it + 1) & 1]);
      const bf16x8 (&a)[8] = abuf[it & 1];
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], bw1[0][ks], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], bw1[1][ks], acc1, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = mt * 16 + lg * 4 + q;        // local position
        const u16 v0 = f2bf(fmaxf(acc0[q] * scale + bias0, 0.f));
        const u16 v1 = f2bf(fmaxf(acc1[q] * scale + bias1, 0.f));
        s_y1[row * Y1_LD + l16] = v0;
        s_y1[row * Y1_LD + 16 + l16] = v1;
      }
    }
  }
  stamp(stamps, 10);
  if constexpr (WMODE == 1) {
    load_w2<FRAG>(W2, bw2);
  }
  if constexpr (WMODE >= 1) {
    load_w3<FRAG>(W3, bw3);
  }
  __syncthreads();
  stamp(stamps, 2);
  // ---------------------------------------------------------------- conv2: 27 positions (2 M tiles), N 64, K 512
  {
    const int n = n2;
    const float bias = bias2;
    floatx4 acc[2];
    acc[0] = floatx4{0.f, 0.f, 0.f, 0.f};
    acc[1] = floatx4{0.f, 0.f, 0.f, 0.f};
    // A fragments in chunks of 4 k-steps x 2 M tiles, the next chunk read while this one's MFMAs run (the W2 / W3
    // fragments hold 136 registers, so not all 32 A fragments at once)
    auto c2_load = [&](int ks0, bf16x8 (&a)[4][2]) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = (ks0 + u) * 32 + lg * 8;   // (i, j, c0)
        const int i = k >> 7, j = (k >> 5) & 3, c0 = k & 31;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int m = min(mt * 16 + l16, TR_C2_POS - 1);
          const int oh = m / 9, ow = m - oh * 9;     // local conv2 row (0..2), column
          a[u][mt] = *reinterpret_cast<const bf16x8*>(s_y1 + ((oh * 2 + i) * 20 + ow * 2 + j) * Y1_LD + c0);
        }
      }
    };
    bf16x8 a2[2][4][2];
    c2_load(0, a2[0]);
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) {
      if (ch < 3) c2_load(4 * (ch + 1), a2[(ch + 1) & 1]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[ch & 1][u][mt], bw2[4 * ch + u], acc[mt], 0, 0, 0);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = mt * 16 + lg * 4 + q;
        if (row < TR_C2_POS) s_y2[row * Y2_LD + n] = f2bf(fmaxf(acc[mt][q] + bias, 0.f));
      }
    }
  }
  __syncthreads();
  stamp(stamps, 3);
  // ---------------------------------------------------------------- conv3: 7 positions (1 M tile), N 64, K 576
  {
    const int n = n2;
    const float bias = bias3;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const int m = min(l16, 6);
    bf16x8 a3[18];   // all A fragments read up front (W2's registers are free by now)
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int k = ks * 32 + lg * 8;
      const int i = k / 192, j = (k >> 6) % 3, c0 = k & 63;
      a3[ks] = *reinterpret_cast<const bf16x8*>(s_y2 + (i * 9 + m + j) * Y2_LD + c0);
    }
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3[ks], bw3[ks], acc, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = lg * 4 + q;
      const u16 v = f2bf(fmaxf(acc[q] + bias, 0.f));
      if (row < 7) y3g[((size_t)e * Y3_ROWS + r * 7 + row) * Y3_C + n] = v;
    }
  }
  // ---------------------------------------------------------------- owned y1 / y2 rows: LDS -> global, 16-byte rows
  {
    const int p1 = tr_y1_own_begin(r) * 20, p1e = tr_y1_own_begin(r + 1) * 20;   // owned conv1 pixels (global)
    const int n1 = (p1e - p1) * 4;                                                // 16-byte chunks (4 per pixel)
    for (int c = tid; c < n1; c += T_THREADS) {
      const int px = p1 + (c >> 2), lp = px - 2 * r * 20, q = (c & 3) * 8;
      *reinterpret_cast<uint4*>(y1g + ((size_t)e * Y1_ROWS + px) * Y1_C + q) =
          *reinterpret_cast<const uint4*>(s_y1 + lp * Y1_LD + q);
    }
    const int n2c = ((r == TR_ROWS - 1) ? 27 : 9) * 8;   // y2 row r (and rows 7, 8 for the last workgroup)
    if (tid < n2c) {
      const int lp = tid >> 3, q = (tid & 7) * 8;
      *reinterpret_cast<uint4*>(y2g + ((size_t)e * Y2_ROWS + r * 9 + lp) * Y2_C + q) =
          *reinterpret_cast<const uint4*>(s_y2 + lp * Y2_LD + q);
    }
  }
  if (stamps) {
    stamp(stamps, 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(stamps, 5);
  }
}


template <bool LATE_W, bool FRAG>
__global__ void __launch_bounds__(T_THREADS) cnn_trunk_rows_kernel(
    const uint8_t* __restrict__ obs, const u16* __restrict__ W1, const float* __restrict__ b1,
    const u16* __restrict__ W2, const float* __restrict__ b2, const u16* __restrict__ W3,
    const float* __restrict__ b3, u16* __restrict__ y1g, u16* __restrict__ y2g, u16* __restrict__ y3g,
    float scale, uint8_t* __restrict__ shift_out, uint8_t* __restrict__ copy_out, uint64_t* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) u16 s_in[TR_IN_ELEMS];
  __shared__ __attribute__((aligned(16))) u16 s_w1[32 * W1_LD];
  __shared__ __attribute__((aligned(16))) u16 s_y1[TR_C1_POS * Y1_LD];
  __shared__ __attribute__((aligned(16))) u16 s_y2[TR_C2_POS * Y2_LD];

  const int r = blockIdx.x % TR_ROWS, e = blockIdx.x / TR_ROWS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const int in0 = 8 * r;                   // first staged input row
  stamp(stamps, 0);

  // ---------------------------------------------------------------- loads, oldest first in the order they are
  // consumed (the vm counter retires in issue order): biases, the staged input rows, conv1 weight fragments, conv2
  // weight fragments; conv3's are issued after the staging barrier. Weights go straight to registers (each B
  // fragment is used by one wave only), the input rows through LDS (the im2col reads overlap).
  const int n2 = wid * 16 + l16;
  const float bias1a = b1[l16], bias1b = b1[16 + l16], bias2 = b2[n2], bias3 = b3[n2];
  constexpr int FR_CH = TR_IN_ROWS * 84 / 16;            // 189 chunks per frame (rows of 84 B never cross frames)
  constexpr int IN_CH = 4 * FR_CH;                        // 756
  constexpr int IN_PER = (IN_CH + T_THREADS - 1) / T_THREADS;   // 3
  uint4 vo[IN_PER];
  {
    const uint8_t* src = obs + (size_t)e * OBS_BYTES + (size_t)in0 * 84;
#pragma unroll
    for (int u = 0; u < IN_PER; ++u) {
      const int i = min(tid + u * T_THREADS, IN_CH - 1);    // clamped: unconditional loads
      const int f = i / FR_CH, c = i - f * FR_CH;
      vo[u] = *reinterpret_cast<const uint4*>(src + (size_t)f * 84 * 84 + c * 16);
    }
  }
  constexpr int W1_PER = 32 * 256 / 8 / T_THREADS;   // 4: W1 staged once through LDS (all 4 waves read it)
  uint4 vw[W1_PER];
#pragma unroll
  for (int u = 0; u < W1_PER; ++u) vw[u] = reinterpret_cast<const uint4*>(W1)[tid + u * T_THREADS];
  {
    uint4* dst = reinterpret_cast<uint4*>(s_in);
#pragma unroll
    for (int u = 0; u < IN_PER; ++u) {   // branch-free (slots past IN_CH land in the pad): no block splits
      const int i = tid + u * T_THREADS;
      const uint2 a = u8x4_to_bf16(vo[u].x), b = u8x4_to_bf16(vo[u].y);
      const uint2 c = u8x4_to_bf16(vo[u].z), d = u8x4_to_bf16(vo[u].w);
      dst[2 * i] = make_uint4(a.x, a.y, b.x, b.y);
      dst[2 * i + 1] = make_uint4(c.x, c.y, d.x, d.y);
    }
#pragma unroll
    for (int u = 0; u < W1_PER; ++u) {
      const int i = tid + u * T_THREADS, rr = i / 32, c8 = (i % 32) * 8;
      *reinterpret_cast<uint4*>(s_w1 + rr * W1_LD + c8) = vw[u];
    }
    // frame-stack outputs of the owned input rows [12r, 12r + 12), straight from the registers above: the window
    // starts 4r rows into the staged rows and spans 12 x 84 B = 63 whole 16-byte chunks (336r B = 21r chunks in),
    // so every chunk is wholly owned or not
    if (shift_out || copy_out) {
#pragma unroll
      for (int u = 0; u < IN_PER; ++u) {
        const int i = tid + u * T_THREADS;
        const int f = i / FR_CH, c = i - f * FR_CH;
        const bool own = i < IN_CH && c >= 21 * r && c < 21 * r + 63;
        const size_t goff = (size_t)e * OBS_BYTES + (size_t)in0 * 84 + c * 16;
        if (own && copy_out) *reinterpret_cast<uint4*>(copy_out + (size_t)f * 84 * 84 + goff) = vo[u];
        if (own && shift_out && f >= 1)
          *reinterpret_cast<uint4*>(shift_out + (size_t)(f - 1) * 84 * 84 + goff) = vo[u];
      }
    }
    __syncthreads();
  }
  stamp(stamps, 1);
  bf16x8 bw2[16], bw3[18];
  trunk_rows_compute<LATE_W ? 1 : 0, FRAG>(s_in, s_w1, s_y1, s_y2, e, r, bias1a, bias1b, bias2, bias3, W2, W3, y1g,
                                           y2g, y3g, scale, stamps, bw2, bw3);
}

// ------------------------------------------------------------------------------------------------------------
// Rollout step t fused with the trunk of step t + 1 (Pong-shaped bank, row-split trunk layout: workgroup (e, r)):
//   policy/value head of env e from the fc partial planes, Gumbel-max sample, env physics (all three paddle
//   directions evaluated while the head runs), then the NEW frame rendered straight into the staged input rows of
//   conv row r (bf16 in LDS), the owned rows stored to the next observation (and shifted into the one after), and
//   conv1 -> conv3 of that observation. The 7 row workgroups of an env evaluate the (tiny) head, sampling and physics
//   redundantly -- bit-identical inputs and maths, so the same action everywhere -- and workgroup r = 0 alone
//   writes the step's outputs. The env state is read from the current parity buffers and the committed state goes
//   to the other parity (`nx`): no workgroup can overwrite state another one still has to read. One launch and one
//   kernel boundary less per rollout step than policy/env kernel + trunk kernel, and the new frame never makes a
//   global round trip before conv1.
// ------------------------------------------------------------------------------------------------------------
struct PongNext {   // the next parity's env state buffers (written by the committing workgroup)
  float* state;
  int32_t* tsteps;
  int64_t* tglob;
  float* ep_ret;
};

__device__ __forceinline__ void pong_commit_next(const PongIO& io, const PongNext& nx, int e, const PongOut& r,
                                                 int64_t tg_old) {
  nx.tglob[e] = tg_old + 1;
  io.reward[e] = r.rew;
  io.done_out[e] = r.done;
  io.trunc_out[e] = r.trunc;
  if (r.done) {
    atomicAdd(&io.ep_stats[0], r.er);
    atomicAdd(&io.ep_stats[1], 1.0f);
    atomicAdd(&io.ep_stats[2], (float)r.t);
  }
  nx.tsteps[e] = r.done ? 0 : r.t;
  nx.ep_ret[e] = r.done ? 0.0f : r.er;
  float* sp = nx.state + (size_t)e * 8;
  const PongState& q = r.s;
  sp[0] = q.bx; sp[1] = q.by; sp[2] = q.vx; sp[3] = q.vy; sp[4] = q.pa; sp[5] = q.po; sp[6] = q.sa; sp[7] = q.so;
}

template <int A1, bool FRAG>
__global__ void __launch_bounds__(T_THREADS) pong_fused_step_kernel(
    PongIO io, PongNext nx, FcParts fc, u16* __restrict__ h, const u16* __restrict__ Wh,
    const float* __restrict__ bh, float* __restrict__ z_out, int32_t* __restrict__ act, float* __restrict__ logp,
    float* __restrict__ ent, float* __restrict__ vout, int key_shift, uint32_t pseed, const u16* __restrict__ W1,
    const float* __restrict__ b1, const u16* __restrict__ W2, const float* __restrict__ b2,
    const u16* __restrict__ W3, const float* __restrict__ b3, u16* __restrict__ y1g, u16* __restrict__ y2g,
    u16* __restrict__ y3g, float scale, uint8_t* __restrict__ shift_out, uint64_t* __restrict__ stamps) {
  constexpr int A = A1 - 1;
  __shared__ __attribute__((aligned(16))) u16 s_in[TR_IN_ELEMS];
  __shared__ __attribute__((aligned(16))) u16 s_w1[32 * W1_LD];
  __shared__ __attribute__((aligned(16))) u16 s_y1[TR_C1_POS * Y1_LD];
  __shared__ __attribute__((aligned(16))) u16 s_y2[TR_C2_POS * Y2_LD];
  __shared__ float s_acc[4][A1];
  __shared__ PongOut cand[3];
  __shared__ int sh_act;
  const int r = blockIdx.x % TR_ROWS, e = blockIdx.x / TR_ROWS;
  const bool lead = r == 0;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l16 = lane & 15;
  const int in0 = 8 * r;
  stamp(stamps, 0);
  // ---------------------------------------------------------------- every independent operand requested first, the
  // head's first (env state, Wh rows, fc planes of obs t: the vm counter retires in issue order, so the sampling
  // waits on them only), then the staged input rows and W1
  const bool phys = tid >= 64 && tid < 67;   // the three paddle directions' physics candidates
  PongIn pin;
  if (phys) pin = pong_load(io, e);
  const int64_t tg0 = io.tglob[e], id0 = io.env_ids[e];
  const float bhj = bh[lane < A1 ? lane : 0];
  uint32_t wv[A1];   // this thread's two Wh rows
#pragma unroll
  for (int u = 0; u < A1; ++u) wv[u] = reinterpret_cast<const uint32_t*>(Wh)[A1 * tid + u];
  FcH2<16> fch;
  fch.issue(fc.hpart, fc.S, fc.plane_stride, fc.bfc, e, tid);
  const int n2 = wid * 16 + l16;
  const float bias1a = b1[l16], bias1b = b1[16 + l16], bias2 = b2[n2], bias3 = b3[n2];
  // frames 0..2 of the next observation (shifted in by the previous trunk launch): the staged rows
  constexpr int FR_CH = TR_IN_ROWS * 84 / 16;                      // 189 chunks per frame
  constexpr int IN3_CH = 3 * FR_CH;                                // 567
  constexpr int IN3_PER = (IN3_CH + T_THREADS - 1) / T_THREADS;    // 3
  uint4 vo[IN3_PER];
  {
    const uint8_t* src = io.out + (size_t)e * OBS_BYTES + (size_t)in0 * 84;
#pragma unroll
    for (int u = 0; u < IN3_PER; ++u) {
      const int i = min(tid + u * T_THREADS, IN3_CH - 1);
      const int f = i / FR_CH, c = i - f * FR_CH;
      vo[u] = *reinterpret_cast<const uint4*>(src + (size_t)f * FRAME + c * 16);
    }
  }
  constexpr int W1_PER = 32 * 256 / 8 / T_THREADS;   // 4
  uint4 vw[W1_PER];
#pragma unroll
  for (int u = 0; u < W1_PER; ++u) vw[u] = reinterpret_cast<const uint4*>(W1)[tid + u * T_THREADS];
  // The conv2 / conv3 weight fragments (136 KB per workgroup) are requested after conv1's MFMAs (trunk_rows_compute
  // WMODE 1). Requesting them at kernel entry or after the policy head measured slower: the vm counter retires in
  // issue order, so the head's fc-plane loads or the render's stores queue behind them
  // (profiles/r3_fused_step_wpos_ab.txt).
  bf16x8 bw2[16], bw3[18];
  // ---------------------------------------------------------------- policy head (every row workgroup of env e)
  float hf[2];
  if (phys) cand[tid - 64] = pong_advance_in(io, pin, (float)(tid - 65));
  fch.finish(fc.hpart, fc.S, fc.plane_stride, e, tid, lead ? h : nullptr, hf);
  float acc[A1];
#pragma unroll
  for (int j = 0; j < A1; ++j) {
    const uint32_t w0 = wv[j >> 1], w1 = wv[(A1 + j) >> 1];
    const float a0 = __uint_as_float((j & 1) ? (w0 & 0xFFFF0000u) : (w0 << 16));
    const float a1 = __uint_as_float(((A1 + j) & 1) ? (w1 & 0xFFFF0000u) : (w1 << 16));
    acc[j] = wave_sum(hf[0] * a0 + hf[1] * a1);
  }
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < A1; ++j) s_acc[wid][j] = acc[j];
  // staging of everything that does not depend on the action: conv1 weights, frames 0..2 (bf16)
  {
    uint4* dst = reinterpret_cast<uint4*>(s_in);
#pragma unroll
    for (int u = 0; u < IN3_PER; ++u) {   // branch-free: slots past IN3_CH land in frame 3's rows (rendered later)
      const int i = tid + u * T_THREADS;
      const uint2 a = u8x4_to_bf16(vo[u].x), b = u8x4_to_bf16(vo[u].y);
      const uint2 c = u8x4_to_bf16(vo[u].z), d = u8x4_to_bf16(vo[u].w);
      dst[2 * i] = make_uint4(a.x, a.y, b.x, b.y);
      dst[2 * i + 1] = make_uint4(c.x, c.y, d.x, d.y);
    }
#pragma unroll
    for (int u = 0; u < W1_PER; ++u) {
      const int i = tid + u * T_THREADS, rr = i / 32, c8 = (i % 32) * 8;
      *reinterpret_cast<uint4*>(s_w1 + rr * W1_LD + c8) = vw[u];
    }
  }
  __syncthreads();
  stamp(stamps, 8);
  if (wid == 0) {
    const int64_t key = tg0 * ((int64_t)1 << key_shift) + id0;   // pre-step counter
    const int jj = lane < A1 ? lane : 0;
    const float zj = ((s_acc[0][jj] + s_acc[1][jj]) + (s_acc[2][jj] + s_acc[3][jj])) + bhj;
    if (lead && lane < A1) z_out[(size_t)e * A1 + lane] = zj;
    const float value = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(zj), A));
    const CatSample cs = cat_sample<8>(zj, A, lane, pseed, key);   // A1 <= 7
    const int bi = cs.act;
    const float lpa = cs.lpa, H = cs.H;
    if (lane == 0) {
      if (lead) {
        act[e] = bi;
        logp[e] = lpa;
        ent[e] = H;
        vout[e] = value;
      }
      sh_act = bi;
    }
  }
  __syncthreads();
  stamp(stamps, 9);
  load_w2<FRAG>(W2, bw2);   // conv2's fragments, landing during the render (trunk_rows_compute WMODE 3)
  const PongOut& res = cand[pong_dir_index(sh_act)];
  const bool done = res.done != 0;
  if (lead && tid == 0) pong_commit_next(io, nx, e, res, tg0);
  // ---------------------------------------------------------------- the new frame: staged rows (all 4 frames
  // after an episode restart), owned rows [12r, 12r + 12) to the next observation and the shifted one after it
  {
    constexpr int WPR = PW / 4;   // 21 words of 4 pixels per row
    const PongGeom gm = pong_geom(res.s);
    uint32_t* ob = reinterpret_cast<uint32_t*>(io.out + (size_t)e * OBS_BYTES);
    uint32_t* sb = shift_out ? reinterpret_cast<uint32_t*>(shift_out + (size_t)e * OBS_BYTES) : nullptr;
    for (int w = tid; w < TR_IN_ROWS * WPR; w += T_THREADS) {
      const int row = w / WPR, x0 = (w - row * WPR) * 4, y = in0 + row;
      const uint32_t word = pong_word(gm, y, x0);
      const uint2 bw = u8x4_to_bf16(word);
      *reinterpret_cast<uint2*>(s_in + (3 * TR_IN_ROWS + row) * 84 + x0) = bw;
      if (done)
#pragma unroll
        for (int f = 0; f < 3; ++f) *reinterpret_cast<uint2*>(s_in + (f * TR_IN_ROWS + row) * 84 + x0) = bw;
      if (y >= 12 * r && y < 12 * r + 12) {
        const int px = (y * 84 + x0) >> 2;
        ob[(3 * FRAME >> 2) + px] = word;
        if (done)
#pragma unroll
          for (int f = 0; f < 3; ++f) ob[(f * FRAME >> 2) + px] = word;
        if (sb) {
          sb[(2 * FRAME >> 2) + px] = word;
          if (done) {
            sb[px] = word;
            sb[(FRAME >> 2) + px] = word;
          }
        }
      }
    }
    if (sb && !done) {   // next-next observation frames 0, 1 <- frames 1, 2 (owned 16-byte chunks, from registers)
#pragma unroll
      for (int u = 0; u < IN3_PER; ++u) {
        const int i = tid + u * T_THREADS;
        const int f = i / FR_CH, c = i - f * FR_CH;
        if (i < IN3_CH && f >= 1 && c >= 21 * r && c < 21 * r + 63)
          *reinterpret_cast<uint4*>(shift_out + (size_t)e * OBS_BYTES + (size_t)(f - 1) * FRAME +
                                    (size_t)in0 * 84 + c * 16) = vo[u];
      }
    }
  }
  __syncthreads();
  stamp(stamps, 1);
  trunk_rows_compute<3, FRAG>(s_in, s_w1, s_y1, s_y2, e, r, bias1a, bias1b, bias2, bias3, W2, W3, y1g, y2g, y3g,
                              scale, stamps, bw2, bw3);
}

// ------------------------------------------------------------------------------------------------------------
// Rollout step t fused with the trunk of step t + 1, per-env layout (one workgroup per env: the large banks,
// Breakout-shape PPO at 128 envs, where 7 row workgroups per env would not fit the chip in one wave):
//   every load first -- the next observation's frames (LDS-DMA: frames 0..2 were shifted in by the previous launch),
//   the conv1 / conv2 weight fragments, the head's Wh rows, the fc partial planes of obs t --; then h (planes summed
//   in order + bias + ReLU), the policy/value head, Gumbel-max sampling, the env physics (all three paddle directions
//   evaluated while the head runs) and the commit; the new frame is rendered straight into the staged uint8 image
//   (all 4 frames after an episode restart) and to obs t+1 in memory; frames 1..3 of obs t+1 go to obs t+2 (shift);
//   then conv1 -> conv3 of obs t+1 (trunk_env_convs, bit-identical to the per-env trunk kernel).
// One launch instead of the trunk kernel + the policy/env kernel of the unfused step, and the new frame never makes a
// global round trip before conv1.
// ------------------------------------------------------------------------------------------------------------
// The body of one (env, part) workgroup; PART -1: the whole env (one workgroup per env, commits into io), 0 / 1:
// the halves of the split step (two workgroups per env: at 128 envs the whole-env form leaves half the CUs idle
// for the ~22 us of the step). Both halves evaluate the head, sampling and physics redundantly (bit-identical inputs
// and maths, so the same action), half 0 alone writes the step's outputs and commits the env state into the other
// parity (nx: the halves read the current one), each half renders the input rows it needs and stores the rows it
// owns, and runs the conv chain of its rows (trunk_env_convs<PART>).
template <int A1, int PART, bool FRAG>
__device__ __forceinline__ void env_step_body(
    uint8_t* __restrict__ s_obs8, u16* __restrict__ s_y1, float (*s_acc)[A1], PongOut* cand, int* sh_act,
    const PongIO& io, const PongNext& nx, const FcParts& fc, int e, u16* __restrict__ h,
    const u16* __restrict__ Wh, const float* __restrict__ bh, float* __restrict__ z_out, int32_t* __restrict__ act,
    float* __restrict__ logp, float* __restrict__ ent, float* __restrict__ vout, int key_shift, uint32_t pseed,
    const u16* __restrict__ W1, const float* __restrict__ b1, const u16* __restrict__ W2,
    const float* __restrict__ b2, const u16* __restrict__ W3, const float* __restrict__ b3, u16* __restrict__ y1g,
    u16* __restrict__ y2g, u16* __restrict__ y3g, float scale, uint8_t* __restrict__ shift_out,
    uint64_t* __restrict__ stamps) {
  using R = EnvRows<PART>;
  constexpr int A = A1 - 1;
  constexpr bool lead = PART <= 0;
  u16* const s_y2 = reinterpret_cast<u16*>(s_obs8);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, l16 = lane & 15;
  const int n2 = wid * 16 + l16;
  stamp(stamps, 0);
  // ---------------------------------------------------------------- loads, in the order they are needed (the vm
  // counter retires in issue order): the head's operands (Wh rows, fc planes of obs t, env state), then the next
  // observation's frames (LDS-DMA: frames 0..2 were shifted in by the previous launch) and the conv1 fragments;
  // the conv2 fragments after the render (they land while conv1 runs), conv3's after conv1
  const bool phys = tid >= 64 && tid < 67;   // the three paddle directions' physics candidates
  PongIn pin;
  if (phys) pin = pong_load(io, e);
  const int64_t tg0 = io.tglob[e], id0 = io.env_ids[e];
  const float bhj = bh[lane < A1 ? lane : 0];
  uint32_t wv[A1];   // this thread's two Wh rows
#pragma unroll
  for (int u = 0; u < A1; ++u) wv[u] = reinterpret_cast<const uint32_t*>(Wh)[A1 * tid + u];
  FcH2<16> fch;
  fch.issue(fc.hpart, fc.S, fc.plane_stride, fc.bfc, e, tid);
  obs_rows_dma<R::ia, R::ib>(io.out + (size_t)e * OBS_BYTES, s_obs8);   // obs t+1 frames 0..2 (3 is rendered)
  w1_lds_dma(W1, s_y1);   // W1 once per workgroup (16 KB; the y1 image is written only from conv1's epilogue on)
  bf16x8 bw[2][8], bw2[16];
  const float bias0 = b1[l16], bias1 = b1[16 + l16], bias2 = b2[n2], bias3 = b3[n2];
  if (phys) cand[tid - 64] = pong_advance_in(io, pin, (float)(tid - 65));
  if (stamps && tid == 64) stamps[(size_t)blockIdx.x * 16 + 10] = __builtin_amdgcn_s_memrealtime();
  // ---------------------------------------------------------------- policy head of obs t
  float hf[2];
  fch.finish(fc.hpart, fc.S, fc.plane_stride, e, tid, lead ? h : nullptr, hf);
  stamp(stamps, 8);
  float accj[A1];
#pragma unroll
  for (int j = 0; j < A1; ++j) {
    const uint32_t w0 = wv[j >> 1], w1 = wv[(A1 + j) >> 1];
    const float a0 = __uint_as_float((j & 1) ? (w0 & 0xFFFF0000u) : (w0 << 16));
    const float a1 = __uint_as_float(((A1 + j) & 1) ? (w1 & 0xFFFF0000u) : (w1 << 16));
    accj[j] = wave_sum(hf[0] * a0 + hf[1] * a1);
  }
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < A1; ++j) s_acc[wid][j] = accj[j];
  stamp(stamps, 9);
  __syncthreads();
  stamp(stamps, 1);
  // the staged frames and W1 have landed (waited for before the sampling wave's output stores join the vm counter)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (wid == 0) {
    const int64_t key = tg0 * ((int64_t)1 << key_shift) + id0;   // pre-step counter
    const int jj = lane < A1 ? lane : 0;
    const float zj = ((s_acc[0][jj] + s_acc[1][jj]) + (s_acc[2][jj] + s_acc[3][jj])) + bhj;
    if (lead && lane < A1) z_out[(size_t)e * A1 + lane] = zj;
    const float value = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(zj), A));
    const CatSample cs = cat_sample<8>(zj, A, lane, pseed, key);   // A1 <= 7
    const int bi = cs.act;
    const float lpa = cs.lpa, H = cs.H;
    if (lane == 0) {
      if (lead) {
        act[e] = bi;
        logp[e] = lpa;
        ent[e] = H;
        vout[e] = value;
      }
      *sh_act = bi;
    }
  }
  __syncthreads();
  stamp(stamps, 2);
  w1_frags_from_lds(s_y1, bw);   // read before the next barrier: conv1's epilogue overwrites them
  load_w2<FRAG>(W2, bw2);        // lands during the render and conv1
  const PongOut& res = cand[pong_dir_index(*sh_act)];
  const bool done = res.done != 0;
  if (tid == 0) {
    if constexpr (PART < 0) pong_commit(io, e, res, tg0);
    else if constexpr (PART == 0) pong_commit_next(io, nx, e, res, tg0);
  }
  // ---------------------------------------------------------------- the new frame: the part's rows of the staged
  // image (all 4 frames after an episode restart), its owned rows of obs t+1 in memory
  {
    constexpr int WPR = PW / 4, NWORDS = PH * WPR;   // 21, 1764
    const PongGeom gm = pong_geom(res.s);
    uint32_t* ob = reinterpret_cast<uint32_t*>(io.out + (size_t)e * OBS_BYTES);
    uint32_t* sw = reinterpret_cast<uint32_t*>(s_obs8);
    for (int w = R::ia * WPR + tid; w < R::ib * WPR; w += 256) {
      const int y = w / WPR, x0 = (w - y * WPR) * 4;
      const uint32_t word = pong_word(gm, y, x0);
      const bool own = PART < 0 || (y >= R::oia && y < R::oib);
      sw[3 * NWORDS + w] = word;
      if (own) ob[3 * NWORDS + w] = word;
      if (done)
#pragma unroll
        for (int f = 0; f < 3; ++f) {
          sw[f * NWORDS + w] = word;
          if (own) ob[f * NWORDS + w] = word;
        }
    }
  }
  __syncthreads();
  stamp(stamps, 3);
  if (shift_out) {   // frames 1..3 of obs t+1 become frames 0..2 of obs t+2 (the owned rows of each frame)
    uint4* so = reinterpret_cast<uint4*>(shift_out + (size_t)e * OBS_BYTES);
    const uint4* si = reinterpret_cast<const uint4*>(s_obs8);
    constexpr int FC = FRAME / 16, C0 = R::oia * 84 / 16, NC = (R::oib - R::oia) * 84 / 16;   // chunks
    for (int i = tid; i < 3 * NC; i += 256) {
      const int f = i / NC, c = C0 + i - f * NC;
      so[f * FC + c] = si[(f + 1) * FC + c];
    }
  }
  stamp(stamps, 4);
  trunk_env_convs<PART, FRAG>(s_obs8, s_y1, s_y2, e, bw, bw2, W3, bias0, bias1, bias2, bias3, y1g, y2g, y3g, scale,
                              stamps);
}

// ------------------------------------------------------------------------------------------------------------
// Rollout step t fused with the trunk of step t + 1, per-env layout (the large banks, Breakout-shape PPO at 128
// envs, where 7 row workgroups per env would not fit the chip in one wave): SPLIT 1 -- one workgroup per env,
// SPLIT 2 -- two per env (env_step_body PART 0 / 1; the env state alternates parity slots as in the row-split step):
//   every load first -- the next observation's frames (LDS-DMA: frames 0..2 were shifted in by the previous launch),
//   the conv1 / conv2 weight fragments, the head's Wh rows, the fc partial planes of obs t --; then h (planes summed
//   in order + bias + ReLU), the policy/value head, Gumbel-max sampling, the env physics (all three paddle directions
//   evaluated while the head runs) and the commit; the new frame is rendered straight into the staged uint8 image
//   (all 4 frames after an episode restart) and to obs t+1 in memory; frames 1..3 of obs t+1 go to obs t+2 (shift);
//   then conv1 -> conv3 of obs t+1 (trunk_env_convs, bit-identical to the per-env trunk kernel).
// One launch instead of the trunk kernel + the policy/env kernel of the unfused step, and the new frame never makes a
// global round trip before conv1.
// ------------------------------------------------------------------------------------------------------------
template <int A1, int SPLIT, bool FRAG>
__global__ void __launch_bounds__(256) pong_fused_env_step_kernel(
    PongIO io, PongNext nx, FcParts fc, u16* __restrict__ h, const u16* __restrict__ Wh, const float* __restrict__ bh,
    float* __restrict__ z_out, int32_t* __restrict__ act, float* __restrict__ logp, float* __restrict__ ent,
    float* __restrict__ vout, int key_shift, uint32_t pseed, const u16* __restrict__ W1,
    const float* __restrict__ b1, const u16* __restrict__ W2, const float* __restrict__ b2,
    const u16* __restrict__ W3, const float* __restrict__ b3, u16* __restrict__ y1g, u16* __restrict__ y2g,
    u16* __restrict__ y3g, float scale, uint8_t* __restrict__ shift_out, uint64_t* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) uint8_t s_obs8[TP_OBS_PAD];   // later the y2 image
  __shared__ __attribute__((aligned(16))) u16 s_y1[SPLIT == 1 ? E1_ELEMS : E1P_ELEMS];
  __shared__ float s_acc[4][A1];
  __shared__ PongOut cand[3];
  __shared__ int sh_act;
#define ACA_ENV_BODY(PART, E)                                                                                    \
  env_step_body<A1, PART, FRAG>(s_obs8, s_y1, s_acc, cand, &sh_act, io, nx, fc, E, h, Wh, bh, z_out, act, logp,     \
                                ent, vout, key_shift, pseed, W1, b1, W2, b2, W3, b3, y1g, y2g, y3g, scale, shift_out, stamps)
  if constexpr (SPLIT == 1) {
    ACA_ENV_BODY(-1, blockIdx.x);
  } else {
    if (blockIdx.x & 1) ACA_ENV_BODY(1, blockIdx.x >> 1);
    else ACA_ENV_BODY(0, blockIdx.x >> 1);
  }
#undef ACA_ENV_BODY
}

// ------------------------------------------------------------------------------------------------------------
// Fused data-gradient chain of the conv trunk, one workgroup per sample (learner backward):
//   dy2 = conv_transpose(dy3, W3) * (y2 > 0)        M 81 positions, N 64, K 576 = (tap i j, o)
//   dy1 = conv_transpose(dy2, W2) * (y1 > 0)        sub-pixel form: per output parity class (py, px) only the
//                                                    2 x 2 taps on its grid, K 256 = (di, dj, o)
// plus the per-sample bias-gradient partials  biasp[b] = [ sum_p dy3 | sum_p dy2 | sum_p dy1 ]  (64 | 64 | 32).
// Both products are per sample (no reduction over the batch), so they run back to back out of LDS: dy3 lands in
// a zero-bordered image (taps off the grid read zeros, no bounds tests), dy2 is written into a second zero-bordered
// image that feeds dy1, and the weights are staged as B rows [k][n] read with the transposing ds_read_b64_tr_b16.
// W2 is prefetched into registers while dy2 runs, so its staging costs no round trip. dy2 / dy1 leave through LDS
// in 16-byte rows (the weight-gradient GEMMs read them); masks are applied in those passes. The bias partials
// are summed in a fixed order (deterministic); the gradient finaliser reduces them over the batch.
// Replaces two implicit transposed-conv GEMM launches (dy2: mode 3/4, dy1: sub-pixel mode 5/6) + their colsums.
// ------------------------------------------------------------------------------------------------------------
// LDS layouts, conflict-free for every fragment read (tests/test_lds_layouts_cpu.py models them):
//  * the A operands of the 16x16x32 MFMA are pixel rows of zero-bordered images: lane l reads 16 bytes of output
//    position m0 + (l & 15) at channel chunk (l >> 4). A ds_read_b128 lane group holds 8 positions at one chunk
//    and 8 at the next; with a 160-byte pixel stride (10 bank quads) those land in 16 distinct quads whenever the
//    8 positions of each chunk are distinct mod 8, which holds when the image width == the output width mod 8:
//    dy3 image 17 wide for the 9-wide dy2 output (17 = 9 + 8), dy2 image 18 wide for the 10-wide sub-pixel
//    classes of dy1 (18 = 10 + 8). (The previous 144-byte stride over 11-wide images: 2.6-2.7 cycles per read.)
//  * the B operands are weight rows read by ds_read_b64_tr_b16 (8 rows x 16 columns per 32-lane group): W3 rows of
//    64 and W2 rows of 32 elements unpadded, each row's 16-byte chunks XOR-swizzled (bw_sw3 / bw_sw2), so the 8
//    rows of a group cover all 64 banks (unswizzled padded rows: 2 cycles per read instead of 1).
// exact small-range divisions as full-rate multiply-shifts (the compiler's signed division is a quarter-rate
// mul_hi sequence): n / 9 for 0 <= n < 200, n / 10 for n < 1029, n / 7 for n < 64 (tests/test_lds_layouts_cpu.py)
__device__ __forceinline__ int div9(int n) { return (int)(((unsigned)n * 57u) >> 9); }
__device__ __forceinline__ int div10(int n) { return (int)(((unsigned)n * 205u) >> 11); }
__device__ __forceinline__ int div7(int n) { return (int)(((unsigned)n * 37u) >> 8); }
constexpr int BW_LDW3 = 64;                 // W3 B rows [576][64], chunks ^ bw_sw3(row)
constexpr int BW_LDW2 = 32;                 // W2 B rows [1024][32], chunks ^ bw_sw2(row)
constexpr int BW_PS = 80;                   // image pixel stride (64 channels + 16 unused)
constexpr int BW_P3H = 11, BW_P3W = 17;     // dy3 image: 7x7 at (2, 2), zero border
constexpr int BW_P2H = 11, BW_P2W = 18;     // dy2 image: 9x9 at (1, 1), zero border
constexpr int BW_RW = 576 * BW_LDW3;        // >= 1024 * BW_LDW2
constexpr int BW_P3E = BW_P3H * BW_P3W * BW_PS;
constexpr int BW_M2E = 81 * 64;
constexpr int BW_P2E = BW_P2H * BW_P2W * BW_PS;
static_assert(400 * 32 + 32 <= BW_P3E + BW_M2E, "dy1 staging (+ its discard slots) aliases the dy3 image + y2 mask");
static_assert(1024 * BW_LDW2 <= BW_RW, "W2 rows fit the W3 region");
static_assert(BW_P3W % 8 == 9 % 8 && BW_P2W % 8 == 10 % 8 && BW_PS == 80, "conflict-free image geometry");
__device__ __forceinline__ int bw_sw3(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int bw_sw2(int r) { return ((r >> 3) & 1) << 1; }
// zero the border pixels of an H x W image (interior rows / cols [LO, LO + N)), the 8 data chunks of each pixel
template <int H, int W, int LO, int N, int NT>
__device__ __forceinline__ void bw_zero_border(u16* img) {
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  for (int c = threadIdx.x; c < H * W * 8; c += NT) {
    const int px = c >> 3, part = c & 7, pa = px / W, pb = px - pa * W;
    if (pa < LO || pa >= LO + N || pb < LO || pb >= LO + N)
      *reinterpret_cast<uint4*>(img + px * BW_PS + part * 8) = z4;
  }
}

// element e (0..7) of 8 packed bf16 as float, without taking the vector's address (that would go to scratch)
__device__ __forceinline__ float bf_lane(const uint4& v, int e) {
  const uint32_t w = e < 2 ? v.x : (e < 4 ? v.y : (e < 6 ? v.z : v.w));
  return __uint_as_float((e & 1) ? (w & 0xFFFF0000u) : (w << 16));
}
__device__ __forceinline__ uint32_t mask_pair(uint32_t w, uint32_t m) {   // zero each bf16 of w whose mask is <= 0
  const uint32_t lo = (__uint_as_float(m << 16) > 0.f) ? 0x0000FFFFu : 0u;
  const uint32_t hi = (__uint_as_float(m & 0xFFFF0000u) > 0.f) ? 0xFFFF0000u : 0u;
  return w & (lo | hi);
}

// tr_frag over XOR-swizzled rows (SW 3: bw_sw3, 2: bw_sw2); `rows` at a row index that is a multiple of 16
template <int SW>
__device__ __forceinline__ bf16x8 tr_frag_sw(const u16* rows, int ld, int col0, int lane) {
  const int lr16 = lane & 15, lg = lane >> 4, q = lr16 >> 2, p = lr16 & 3;
  const int r0 = lg * 8 + q, r1 = r0 + 4, col = col0 + 4 * p;
  const int s0 = SW == 3 ? bw_sw3(r0) : bw_sw2(r0), s1 = SW == 3 ? bw_sw3(r1) : bw_sw2(r1);
  const u16* p0 = rows + r0 * ld + ((((col >> 3) ^ s0) << 3) | (col & 7));
  const u16* p1 = rows + r1 * ld + ((((col >> 3) ^ s1) << 3) | (col & 7));
  typedef short short4x __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) short4x lds4;
  const short4x lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(p0));
  const short4x hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(p1));
  const short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 tr_frag(const u16* rows, int ld, int col0, int lane) {
  // B fragment (k = 8 (lane >> 4) + 0..7, n = col0 + lane & 15) from n-contiguous rows via two transposing reads
  const int lr16 = lane & 15, lg = lane >> 4, q = lr16 >> 2, p = lr16 & 3;
  const u16* p0 = rows + (lg * 8 + q) * ld + col0 + 4 * p;
  const u16* p1 = rows + (lg * 8 + 4 + q) * ld + col0 + 4 * p;
  typedef short short4x __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) short4x lds4;
  const short4x lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(p0));
  const short4x hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(p1));
  const short8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// 8 waves (2 per SIMD: one wave per SIMD left every LDS read latency exposed); one workgroup per CU by LDS.
constexpr int BW_T = 512;
// The conv1 weight gradient folded into the persistent data-gradient chain (cnn_trunk_bwd_persist_kernel W1G):
// dW1[o][c] = scale * sum_p dy1[p][o] * obs[ch][4 oy + ky][4 ox + kx], c = (ch, ky, kx), p = (oy, ox).
struct W1Fold {
  const uint8_t* obs;        // [*, 4, 84, 84] uint8 frames
  const int64_t* obs_idx;    // sample b reads obs row obs_idx[b] (null: row b)
  float* planes;             // [B][32 * 256]
  float scale;               // 1 / 255
};
constexpr int BW_FR = 4 * 84 * 84;   // frame pixels of a sample (bf16 in LDS: 56.4 KB over the dead W2 rows)
static_assert(BW_FR + 8 <= BW_RW, "the bf16 frames + a zero chunk fit the weight region");
static_assert(416 * 32 <= BW_P3E + BW_M2E, "dy1 rows + 16 zero padding rows (13 k-steps of 32) fit the staging");

__global__ void __launch_bounds__(BW_T) cnn_trunk_bwd_kernel(
    const u16* __restrict__ dy3g, const u16* __restrict__ W3, const u16* __restrict__ y2g,
    const u16* __restrict__ W2, const u16* __restrict__ y1g, u16* __restrict__ dy2g, u16* __restrict__ dy1g,
    float* __restrict__ biasp, uint64_t* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) u16 s_w[BW_RW];
  __shared__ __attribute__((aligned(16))) u16 s_p3m2[BW_P3E + BW_M2E];   // dy3 image + y2 mask; later dy1 staging
  __shared__ __attribute__((aligned(16))) u16 s_p2[BW_P2E];
  __shared__ float s_red[8 * 128 + 8 * 32];
  u16* const s_p3 = s_p3m2;
  u16* const s_m2 = s_p3m2 + BW_P3E;
  u16* const s_d1 = s_p3m2;
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  stamp(stamps, 0);

  // ---------------------------------------------------------------- loads: dy3 image, W3 rows, y2 mask; W2 + y1
  // mask prefetched into registers (consumed in the dy1 phase)
  {
    constexpr int W3_CH = 576 * 8, W3_PER = W3_CH / BW_T;      // 9
    constexpr int M2_CH = 81 * 8;                              // 648
    constexpr int M2_PER = (M2_CH + BW_T - 1) / BW_T;          // 2
    uint4 vw[W3_PER], vm[M2_PER];
    // dy3: 49 pixels x 8 chunks = 392 <= BW_T, one 16-byte load per thread (the border is zeroed below)
    const uint4 vp = *reinterpret_cast<const uint4*>(dy3g + (size_t)b * 49 * 64 + min(tid, 391) * 8);
#pragma unroll
    for (int u = 0; u < W3_PER; ++u) {
      // B row k = (i, j, o) <- W3[o][i][j][:] (64 contiguous channels = 8 chunks)
      const int c = tid + u * BW_T, k = c >> 3, part = c & 7;
      const int t = k >> 6, o = k & 63;
      vw[u] = *reinterpret_cast<const uint4*>(W3 + o * 576 + t * 64 + part * 8);
    }
#pragma unroll
    for (int u = 0; u < M2_PER; ++u) {
      const int c = min(tid + u * BW_T, M2_CH - 1);
      vm[u] = *reinterpret_cast<const uint4*>(y2g + (size_t)b * 81 * 64 + c * 8);
    }
    if (tid < 392) {
      const int px = tid >> 3, pa = px / 7, pb = px - pa * 7;
      *reinterpret_cast<uint4*>(s_p3 + ((pa + 2) * BW_P3W + pb + 2) * BW_PS + (tid & 7) * 8) = vp;
    }
    bw_zero_border<BW_P3H, BW_P3W, 2, 7, BW_T>(s_p3);
#pragma unroll
    for (int u = 0; u < W3_PER; ++u) {
      const int c = tid + u * BW_T, k = c >> 3;
      *reinterpret_cast<uint4*>(s_w + k * BW_LDW3 + (((c & 7) ^ bw_sw3(k)) << 3)) = vw[u];
    }
#pragma unroll
    for (int u = 0; u < M2_PER; ++u) {
      const int c = tid + u * BW_T;
      if (c < M2_CH) *reinterpret_cast<uint4*>(s_m2 + c * 8) = vm[u];
    }
    // dy2 image: zero border; the interior is written by the dy2 epilogue
    bw_zero_border<BW_P2H, BW_P2W, 1, 9, BW_T>(s_p2);
  }
  // held across the dy2 phase in named registers (hipcc left a uint4 array for this in scratch)
  static_assert(64 * 512 / 8 / BW_T == 8, "W2 prefetch is written out for 8 chunks per thread");
#define ACA_W2_LD(u) const uint4 vw2_##u = *reinterpret_cast<const uint4*>(W2 + (tid + (u) * BW_T) * 8);
  ACA_W2_LD(0) ACA_W2_LD(1) ACA_W2_LD(2) ACA_W2_LD(3) ACA_W2_LD(4) ACA_W2_LD(5) ACA_W2_LD(6) ACA_W2_LD(7)
#undef ACA_W2_LD
  constexpr int M1_CH = 400 * 4, M1_PER = (M1_CH + BW_T - 1) / BW_T;   // 1600 -> 4
  uint4 vm1[M1_PER];
#pragma unroll
  for (int u = 0; u < M1_PER; ++u) {
    const int c = min(tid + u * BW_T, M1_CH - 1);
    vm1[u] = *reinterpret_cast<const uint4*>(y1g + (size_t)b * 400 * 32 + c * 8);
  }
  __syncthreads();
  stamp(stamps, 1);

  // ---------------------------------------------------------------- dy2: wave -> (N tile wid % 4, M tiles 3 x half)
  {
    const int n0 = (wid & 3) * 16, mh = (wid >> 2) * 3;
    floatx4 acc[3];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
    // per-lane A row offsets once, every k-step's read at a compile-time immediate from them (persist kernel notes)
    constexpr int P3_LO = 2 * BW_P3W + 2;
    int pb[3];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
      const int m = min((mh + mt) * 16 + l16, 80);
      const int a = div9(m), c = m - a * 9;
      pb[mt] = ((a + 2) * BW_P3W + (c + 2) - P3_LO) * BW_PS + lg * 8;
    }
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int t = ks >> 1, ti = t / 3, tj = t - ti * 3;
      const int off = (P3_LO - ti * BW_P3W - tj) * BW_PS + (ks & 1) * 32;
      const bf16x8 bf = tr_frag_sw<3>(s_w + ks * 32 * BW_LDW3, BW_LDW3, n0, lane);
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(s_p3 + pb[mt] + off);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[mt], 0, 0, 0);
      }
    }
    const int n = n0 + l16;
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (mh + mt) * 16 + lg * 4 + r;
        const int a = div9(m), c = m - a * 9;
        const float v = bf2f(s_m2[min(m, 80) * 64 + n]) > 0.f ? acc[mt][r] : 0.f;
        const int dst = m < 81 ? ((a + 1) * BW_P2W + (c + 1)) * BW_PS + n : 64 + l16;   // past 81: unread slot
        s_p2[dst] = f2bf(v);
      }
  }
  // db3 partial from the dy3 image (before it is overwritten): thread -> channel group tid % 8, fixed order
  float part3[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int c = tid; c < 49 * 8; c += BW_T) {
    const int px = c >> 3, g = c & 7, pa = div7(px), pb = px - pa * 7;
    const uint4 v = *reinterpret_cast<const uint4*>(s_p3 + ((pa + 2) * BW_P3W + (pb + 2)) * BW_PS + g * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) part3[e] += bf_lane(v, e);
  }
  __syncthreads();   // dy2 image complete; the W3 rows and the dy3 image are dead
  stamp(stamps, 2);

  // ---------------------------------------------------------------- W2 rows in; dy2 out (16-byte rows) + db2
  // W2 chunk c -> B row (tap, o): o = c / 64, tap = (c / 4) % 16, part = c % 4
#define ACA_W2_ST(u)                                                                                  \
  {                                                                                                   \
    const int c = tid + (u) * BW_T, o = c >> 6, t = (c >> 2) & 15, part = c & 3;                     \
    *reinterpret_cast<uint4*>(s_w + (t * 64 + o) * BW_LDW2 + ((part ^ bw_sw2(t * 64 + o)) << 3)) = vw2_##u; \
  }
  ACA_W2_ST(0) ACA_W2_ST(1) ACA_W2_ST(2) ACA_W2_ST(3) ACA_W2_ST(4) ACA_W2_ST(5) ACA_W2_ST(6) ACA_W2_ST(7)
#undef ACA_W2_ST
  float part2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int c = tid; c < 81 * 8; c += BW_T) {
    const int m = c >> 3, g = c & 7, a = div9(m), cc = m - a * 9;
    const uint4 v = *reinterpret_cast<const uint4*>(s_p2 + ((a + 1) * BW_P2W + (cc + 1)) * BW_PS + g * 8);
    *reinterpret_cast<uint4*>(dy2g + ((size_t)b * 81 + m) * 64 + g * 8) = v;
#pragma unroll
    for (int e = 0; e < 8; ++e) part2[e] += bf_lane(v, e);
  }
  // channel sums (fixed order, deterministic): lanes of one channel group (tid % 8 == g) are combined by xor
  // shuffles inside each wave, then the 8 waves' rows are summed in wave order
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      part3[e] += lane_xor(part3[e], o);
      part2[e] += lane_xor(part2[e], o);
    }
  if (lane < 8)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s_red[wid * 128 + lane * 8 + e] = part3[e];          // channel lane * 8 + e
      s_red[wid * 128 + 64 + lane * 8 + e] = part2[e];
    }
  __syncthreads();   // W2 rows + the reduction rows complete
  if (tid < 128) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += s_red[w * 128 + tid];
    biasp[(size_t)b * 160 + tid] = v;                      // db3 (0..63) | db2 (64..127)
  }
  stamp(stamps, 3);

  // ---------------------------------------------------------------- dy1 (sub-pixel): wave -> (N tile wid % 2,
  // parity class wid / 2 = (py, px): its 7 M tiles of 16 of the class's 10 x 10 outputs)
  {
    const int nt = wid & 1, cls = wid >> 1, py = cls >> 1, px = cls & 1;
    floatx4 acc[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    constexpr int P2_LO = BW_P2W + 1;
    int pb1[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const int u = min(i * 16 + l16, 99), yy = div10(u), xx = u - yy * 10;
      pb1[i] = ((yy + 1) * BW_P2W + (xx + 1) - P2_LO) * BW_PS + lg * 8;
    }
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int d = ks >> 1, di = d >> 1, dj = d & 1, ob = (ks & 1) * 32;
      const int tap = (py + 2 * di) * 4 + (px + 2 * dj);
      const int off = (P2_LO - di * BW_P2W - dj) * BW_PS + ob;
      const bf16x8 bf = tr_frag_sw<2>(s_w + (tap * 64 + ob) * BW_LDW2, BW_LDW2, nt * 16, lane);
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(s_p2 + pb1[i] + off);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[i], 0, 0, 0);
      }
    }
    // unmasked dy1 -> LDS [400][32] (the mask is applied in the 16-byte output pass)
    const int n = nt * 16 + l16;
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int u = i * 16 + lg * 4 + r;
        const int yy = div10(u), xx = u - yy * 10;
        const int dst = u < 100 ? ((2 * yy + py) * 20 + 2 * xx + px) * 32 + n : 400 * 32 + n;   // past 100: unread
        s_d1[dst] = f2bf(acc[i][r]);
      }
  }
  __syncthreads();
  stamp(stamps, 4);
  // dy1 out: mask (prefetched y1 rows) applied, 16-byte stores, db1 partials (thread -> channel group tid % 4)
  float part1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < M1_PER; ++u) {
    const int c = tid + u * BW_T;
    if (c < M1_CH) {
      uint4 v = *reinterpret_cast<const uint4*>(s_d1 + c * 8);
      v.x = mask_pair(v.x, vm1[u].x);
      v.y = mask_pair(v.y, vm1[u].y);
      v.z = mask_pair(v.z, vm1[u].z);
      v.w = mask_pair(v.w, vm1[u].w);
#pragma unroll
      for (int e = 0; e < 8; ++e) part1[e] += bf_lane(v, e);
      *reinterpret_cast<uint4*>(dy1g + (size_t)b * 400 * 32 + c * 8) = v;
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) part1[e] += lane_xor(part1[e], o);
  if (lane < 4)
#pragma unroll
    for (int e = 0; e < 8; ++e) s_red[1024 + wid * 32 + lane * 8 + e] = part1[e];   // channel lane * 8 + e
  __syncthreads();
  if (tid < 32) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += s_red[1024 + w * 32 + tid];
    biasp[(size_t)b * 160 + 128 + tid] = v;
  }
  if (stamps) {
    stamp(stamps, 5);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(stamps, 6);
  }
}

// Persistent form of the data-gradient chain above for large learner batches (PPO minibatches): one workgroup per
// CU walks samples b = blockIdx.x, blockIdx.x + gridDim.x, ... The per-sample kernel restages W3 (74 KB) and W2
// (64 KB) from L2 into LDS for every sample and leaves the CU idle while each sample's operands arrive; here W3's B
// rows are staged into LDS ONCE and stay resident, and every wave extracts the 8 W2 fragments it uses (its N tile x
// its parity class's k-steps, 32 registers) once, through a staging pass that aliases the image buffers, and keeps
// them in registers for all of its samples; the next sample's dy3 image, y2 mask and y1 mask are loaded into
// registers while the current one is processed. Same MFMA order per sample as the per-sample kernel: bit-identical
// outputs.
// W1G: the conv1 weight gradient folded in (W1Fold): after a sample's dy1 rows are
// masked they stay in LDS and its four frames (prefetched with the sample's other operands) are staged as exact bf16
// over the dead image region (which is extended for it; the dy2 image border is then re-zeroed per sample); 13 k-steps
// of 16x16x32 MFMAs accumulate the workgroup's [32][256] slice in registers across its samples, written once at the
// end as plane blockIdx.x (scaled). dy1 itself is then not stored (dy1g null): conv1 is the first layer, so its
// weight gradient was dy1's only consumer -- the 105 MB dy1 write and re-read of a 4096-row minibatch disappear.
template <bool W1G>
__global__ void __launch_bounds__(BW_T) cnn_trunk_bwd_persist_kernel(
    const u16* __restrict__ dy3g, const u16* __restrict__ W3, const u16* __restrict__ y2g,
    const u16* __restrict__ W2, const u16* __restrict__ y1g, u16* __restrict__ dy2g, u16* __restrict__ dy1g,
    float* __restrict__ biasp, int B, uint64_t* __restrict__ stamps, int bias_acc, W1Fold wf) {
  // bias_acc: the bias-gradient partials summed over the workgroup's samples (in walk order) into ONE row per
  // workgroup, biasp[blockIdx.x] -- gridDim.x rows for the finaliser instead of B (its latency-bound walk over the
  // per-sample rows was the longest job of the Breakout finaliser)
  float bacc = 0.f, bacc1 = 0.f;
  // diagnostics: phase stamps of the first two samples of every workgroup ([blockIdx][16]: 8 per sample)
  auto pst = [&](int it, int k) {
    if (stamps && it < 2 && threadIdx.x == 0)
      stamps[(size_t)blockIdx.x * 16 + it * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };
  // staging area for the weight fragments (aliases the images: used before the sample loop only)
  constexpr int STAGE = BW_P3E + BW_M2E + BW_P2E;   // 14960 + 5184 + 15840 u16 = 70 KB
  constexpr int FR_OFF = 416 * 32;                   // W1G: bf16 frames behind the 416 dy1 rows
  constexpr int IMG_E = W1G && FR_OFF + BW_FR + 8 > STAGE ? FR_OFF + BW_FR + 8 : STAGE;
  __shared__ __attribute__((aligned(16))) u16 s_w3[576 * BW_LDW3];   // 72 KB
  __shared__ __attribute__((aligned(16))) u16 s_img[IMG_E];
  __shared__ float s_red[8 * 128 + 8 * 32];
  u16* const s_p2i = s_img + BW_P3E + BW_M2E;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  static_assert(512 * BW_LDW2 <= STAGE, "half of the W2 rows fit the staging area");

  // ---- W3 B rows k = (t, o) <- W3[o][t][:], resident in LDS for the whole walk
  for (int c = tid; c < 576 * 8; c += BW_T) {
    const int k = c >> 3, part = c & 7, t = k >> 6, o = k & 63;
    *reinterpret_cast<uint4*>(s_w3 + k * BW_LDW3 + ((part ^ bw_sw3(k)) << 3)) =
        *reinterpret_cast<const uint4*>(W3 + o * 576 + t * 64 + part * 8);
  }
  // ---- W2 fragments of this wave's (N tile, parity class): rows (t, o) <- W2[o][t][:], staged 512 rows at a time
  bf16x8 w2f[8];
  {
    const int nt = wid & 1, cls = wid >> 1, py = cls >> 1, px = cls & 1;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      for (int c = tid; c < 512 * 4; c += BW_T) {
        const int row = half * 512 + (c >> 2), part = c & 3, t = row >> 6, o = row & 63;
        *reinterpret_cast<uint4*>(s_img + (c >> 2) * BW_LDW2 + ((part ^ bw_sw2(c >> 2)) << 3)) =
            *reinterpret_cast<const uint4*>(W2 + o * 512 + t * 32 + part * 8);
      }
      __syncthreads();
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int d = ks >> 1, di = d >> 1, dj = d & 1, ob = (ks & 1) * 32;
        const int tap = (py + 2 * di) * 4 + (px + 2 * dj);
        if ((tap >> 3) == half)
          w2f[ks] = tr_frag_sw<2>(s_img + ((tap & 7) * 64 + ob) * BW_LDW2, BW_LDW2, nt * 16, lane);
      }
      __syncthreads();
    }
  }
  // dy2 image border: zero once (the interior is rewritten for every sample, the border never)
  bw_zero_border<BW_P2H, BW_P2W, 1, 9, BW_T>(s_p2i);

  constexpr int M2_CH = 81 * 8, M2_PER = (M2_CH + BW_T - 1) / BW_T;              // 648 -> 2
  constexpr int M1_CH = 400 * 4, M1_PER = (M1_CH + BW_T - 1) / BW_T;             // 1600 -> 4
  static_assert(M2_PER == 2 && M1_PER == 4, "prefetch registers are written out");
  uint4 vp0, vm0, vm1_, m10, m11, m12, m13;   // next sample
  uint4 fr0, fr1, fr2, fr3;                   // W1G: its frames, 16-pixel chunks (1764: <= 4 per thread)
  constexpr int FR_CH = BW_FR / 16;
  floatx4 w1acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) w1acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  // (the frames are fetched right after the previous sample's frames were staged: a phase later than the rest)
  auto fetch_fr = [&](int b) {
    if constexpr (W1G) {
      const uint4* f = reinterpret_cast<const uint4*>(wf.obs + (size_t)(wf.obs_idx ? wf.obs_idx[b] : b) * BW_FR);
      fr0 = f[tid];
      fr1 = f[tid + BW_T];
      fr2 = f[tid + 2 * BW_T];
      fr3 = f[min(tid + 3 * BW_T, FR_CH - 1)];
    }
  };
  auto fetch = [&](int b) {
    // dy3: 49 pixels x 8 chunks = 392 <= BW_T: one 16-byte load per thread
    vp0 = *reinterpret_cast<const uint4*>(dy3g + (size_t)b * 49 * 64 + min(tid, 391) * 8);
    vm0 = *reinterpret_cast<const uint4*>(y2g + (size_t)b * 81 * 64 + min(tid, M2_CH - 1) * 8);
    vm1_ = *reinterpret_cast<const uint4*>(y2g + (size_t)b * 81 * 64 + min(tid + BW_T, M2_CH - 1) * 8);
    m10 = *reinterpret_cast<const uint4*>(y1g + (size_t)b * 400 * 32 + tid * 8);
    m11 = *reinterpret_cast<const uint4*>(y1g + (size_t)b * 400 * 32 + (tid + BW_T) * 8);
    m12 = *reinterpret_cast<const uint4*>(y1g + (size_t)b * 400 * 32 + (tid + 2 * BW_T) * 8);
    m13 = *reinterpret_cast<const uint4*>(y1g + (size_t)b * 400 * 32 + min(tid + 3 * BW_T, M1_CH - 1) * 8);
  };
  if ((int)blockIdx.x < B) {
    fetch(blockIdx.x);
    fetch_fr(blockIdx.x);
  }
  for (int b = blockIdx.x, it = 0; b < B; b += gridDim.x, ++it) {
    pst(it, 0);
    // opaque zero (per iteration): keeps the LDS address arithmetic of the unrolled MFMA loops inside the sample
    // loop -- hoisted out of it, the loop-invariant addresses alone took more registers than the kernel has
    int z0;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z0));
    u16* const s_p3 = s_img + z0;
    u16* const s_m2 = s_img + BW_P3E + z0;
    u16* const s_d1 = s_img + z0;
    u16* const s_p2 = s_img + BW_P3E + BW_M2E + z0;
    const u16* const s_w3z = s_w3 + z0;
    const int lane = (threadIdx.x & 63) + z0, l16 = lane & 15, lg = lane >> 4;   // shadow: per-iteration values
    // ---- this sample's dy3 image + y2 mask to LDS (the border re-zeroed: the previous sample's dy1 staging
    // aliased it); y1 mask kept in registers; the next sample's loads issued
    {
      if (tid < 392) {
        const int px = tid >> 3, pa = px / 7, pb = px - pa * 7;
        *reinterpret_cast<uint4*>(s_p3 + ((pa + 2) * BW_P3W + pb + 2) * BW_PS + (tid & 7) * 8) = vp0;
      }
      bw_zero_border<BW_P3H, BW_P3W, 2, 7, BW_T>(s_p3);
      if constexpr (W1G) bw_zero_border<BW_P2H, BW_P2W, 1, 9, BW_T>(s_p2);   // the frames overwrote it
      *reinterpret_cast<uint4*>(s_m2 + tid * 8) = vm0;
      if (tid + BW_T < M2_CH) *reinterpret_cast<uint4*>(s_m2 + (tid + BW_T) * 8) = vm1_;
    }
    const uint4 vm1[4] = {m10, m11, m12, m13};
    __syncthreads();
    pst(it, 1);
    if (b + (int)gridDim.x < B) fetch(b + gridDim.x);

    // ---- dy2: wave -> (N tile wid % 4, M tiles 3 x half)
    {
      const int n0 = (wid & 3) * 16, mh = (wid >> 2) * 3;
      floatx4 acc[3];
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
      // operands of k-step ks + 1 read while ks's MFMAs run (two register buffers): left to the compiler, every
      // MFMA waited out the LDS read issued just before it
      // A rows: per-lane LDS offsets (pixel, channel chunk lg) computed once per sample, relative to the largest tap
      // displacement, so every k-step's read is that base + a compile-time immediate (k-step ks = tap ks / 2,
      // channels (ks & 1) * 32 + lg * 8: lg * 8 < 32 never carries into the tap). Divisions by 9 / 10 below are
      // exact multiply-shifts over their ranges (tests/test_lds_layouts_cpu.py); no per-read multiply or divide.
      constexpr int P3_LO = 2 * BW_P3W + 2;
      int pb[3];
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) {
        const int m = min((mh + mt) * 16 + l16, 80);
        const int a = div9(m), c = m - a * 9;
        pb[mt] = ((a + 2) * BW_P3W + (c + 2) - P3_LO) * BW_PS + lg * 8;
      }
      bf16x8 af[2][3], bwf[2];
      auto ld2 = [&](int ks, int buf) {
        const int t = ks >> 1, ti = t / 3, tj = t - ti * 3;
        const int off = (P3_LO - ti * BW_P3W - tj) * BW_PS + (ks & 1) * 32;   // >= 0
        bwf[buf] = tr_frag_sw<3>(s_w3z + ks * 32 * BW_LDW3, BW_LDW3, n0, lane);
#pragma unroll
        for (int mt = 0; mt < 3; ++mt) af[buf][mt] = *reinterpret_cast<const bf16x8*>(s_p3 + pb[mt] + off);
      };
      ld2(0, 0);
#pragma unroll
      for (int ks = 0; ks < 18; ++ks) {
        if (ks + 1 < 18) ld2(ks + 1, (ks + 1) & 1);
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks & 1][mt], bwf[ks & 1], acc[mt], 0, 0, 0);
      }
      pst(it, 6);
      const int n = n0 + l16;
      // rows past the 81 outputs go to an unread slot (channel 64 + l16 of the dy2 image's first border pixel):
      // select instead of branch
#pragma unroll
      for (int mt = 0; mt < 3; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = (mh + mt) * 16 + lg * 4 + r;
          const int a = div9(m), c = m - a * 9;
          const float v = bf2f(s_m2[min(m, 80) * 64 + n]) > 0.f ? acc[mt][r] : 0.f;
          const int dst = m < 81 ? ((a + 1) * BW_P2W + (c + 1)) * BW_PS + n : 64 + l16;
          s_p2[dst] = f2bf(v);
        }
    }
    float part3[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = tid; c < 49 * 8; c += BW_T) {
      const int px = c >> 3, g = c & 7, pa = div7(px), pb = px - pa * 7;
      const uint4 v = *reinterpret_cast<const uint4*>(s_p3 + ((pa + 2) * BW_P3W + (pb + 2)) * BW_PS + g * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) part3[e] += bf_lane(v, e);
    }
    pst(it, 7);
    __syncthreads();   // dy2 image complete; the dy3 image and the y2 mask are dead
    pst(it, 2);

    // ---- dy2 out (16-byte rows) + db2 / db3 channel sums
    float part2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = tid; c < 81 * 8; c += BW_T) {
      const int m = c >> 3, g = c & 7, a = div9(m), cc = m - a * 9;
      const uint4 v = *reinterpret_cast<const uint4*>(s_p2 + ((a + 1) * BW_P2W + (cc + 1)) * BW_PS + g * 8);
      *reinterpret_cast<uint4*>(dy2g + ((size_t)b * 81 + m) * 64 + g * 8) = v;
#pragma unroll
      for (int e = 0; e < 8; ++e) part2[e] += bf_lane(v, e);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        part3[e] += lane_xor(part3[e], o);
        part2[e] += lane_xor(part2[e], o);
      }
    if (lane < 8)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s_red[wid * 128 + lane * 8 + e] = part3[e];
        s_red[wid * 128 + 64 + lane * 8 + e] = part2[e];
      }

    // ---- dy1 (sub-pixel): wave -> (N tile wid % 2, parity class wid / 2)
    {
      const int nt = wid & 1, cls = wid >> 1, py = cls >> 1, px = cls & 1;
      floatx4 acc[7];
#pragma unroll
      for (int i = 0; i < 7; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      constexpr int P2_LO = BW_P2W + 1;   // largest tap displacement (di = dj = 1)
      int pb1[7];
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const int u = min(i * 16 + l16, 99), yy = div10(u), xx = u - yy * 10;
        pb1[i] = ((yy + 1) * BW_P2W + (xx + 1) - P2_LO) * BW_PS + lg * 8;
      }
      bf16x8 a1[2][7];   // k-step ks + 1's A fragments read while ks's MFMAs run
      auto ld1 = [&](int ks, int buf) {
        const int d = ks >> 1, di = d >> 1, dj = d & 1, ob = (ks & 1) * 32;
        const int off = (P2_LO - di * BW_P2W - dj) * BW_PS + ob;   // >= 0
#pragma unroll
        for (int i = 0; i < 7; ++i) a1[buf][i] = *reinterpret_cast<const bf16x8*>(s_p2 + pb1[i] + off);
      };
      ld1(0, 0);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        if (ks + 1 < 8) ld1(ks + 1, (ks + 1) & 1);
#pragma unroll
        for (int i = 0; i < 7; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[ks & 1][i], w2f[ks], acc[i], 0, 0, 0);
      }
      pst(it, 3);
      __syncthreads();   // every wave is past its dy2-image reads of the db sums; s_red rows complete
      if (tid < 128) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) v += s_red[w * 128 + tid];
        if (bias_acc) bacc += v;
        else biasp[(size_t)b * 160 + tid] = v;                 // db3 (0..63) | db2 (64..127)
      }
      const int n = nt * 16 + l16;
      // outputs past the class's 100 go to an unread slot (the dead y2-mask region behind the [400][32] dy1 rows)
#pragma unroll
      for (int i = 0; i < 7; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int u = i * 16 + lg * 4 + r;
          const int yy = div10(u), xx = u - yy * 10;
          const int dst = u < 100 ? ((2 * yy + py) * 20 + 2 * xx + px) * 32 + n : 400 * 32 + n;
          s_d1[dst] = f2bf(acc[i][r]);
        }
    }
    __syncthreads();
    pst(it, 4);
    // ---- dy1 out: y1 mask applied, 16-byte stores, db1 partials
    float part1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + u * BW_T;
      if (c < M1_CH) {
        uint4 v = *reinterpret_cast<const uint4*>(s_d1 + c * 8);
        v.x = mask_pair(v.x, vm1[u].x);
        v.y = mask_pair(v.y, vm1[u].y);
        v.z = mask_pair(v.z, vm1[u].z);
        v.w = mask_pair(v.w, vm1[u].w);
#pragma unroll
        for (int e = 0; e < 8; ++e) part1[e] += bf_lane(v, e);
        if (dy1g) *reinterpret_cast<uint4*>(dy1g + (size_t)b * 400 * 32 + c * 8) = v;
        if constexpr (W1G) *reinterpret_cast<uint4*>(s_d1 + c * 8) = v;   // masked rows: dW1's A operand
      }
    }
    if constexpr (W1G) {
      // frames as exact bf16 behind the dy1 rows (the dy2 image is dead), a zero chunk behind them; zero dy1 rows
      // 400..415 (the dy1 epilogue's discard slots live there)
      u16* const s_fr = s_img + FR_OFF + z0;
      auto put = [&](const uint4& w, int i) {
        const uint2 a = u8x4_to_bf16(w.x), b2 = u8x4_to_bf16(w.y), c = u8x4_to_bf16(w.z), d = u8x4_to_bf16(w.w);
        *reinterpret_cast<uint4*>(s_fr + i * 16) = make_uint4(a.x, a.y, b2.x, b2.y);
        *reinterpret_cast<uint4*>(s_fr + i * 16 + 8) = make_uint4(c.x, c.y, d.x, d.y);
      };
      put(fr0, tid);
      put(fr1, tid + BW_T);
      put(fr2, tid + 2 * BW_T);
      if (tid + 3 * BW_T < FR_CH) put(fr3, tid + 3 * BW_T);
      if (tid == 0) *reinterpret_cast<uint4*>(s_fr + BW_FR) = make_uint4(0u, 0u, 0u, 0u);
      s_d1[400 * 32 + tid] = 0;
      if (b + (int)gridDim.x < B) fetch_fr(b + gridDim.x);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) part1[e] += lane_xor(part1[e], o);
    if (lane < 4)
#pragma unroll
      for (int e = 0; e < 8; ++e) s_red[1024 + wid * 32 + lane * 8 + e] = part1[e];
    __syncthreads();   // also: every s_d1 read is done before the next sample's dy3 image lands on it
    if (tid < 32) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += s_red[1024 + w * 32 + tid];
      if (bias_acc) bacc1 += v;
      else biasp[(size_t)b * 160 + 128 + tid] = v;
    }
    if constexpr (W1G) {
      // dW1 += dy1^T patches: wave -> (o tiles 0, 1) x (c tiles 2 wid, 2 wid + 1), 13 k-steps of 32 positions
      const u16* const s_fr = s_img + FR_OFF + z0;
      const int q = l16 >> 2, pq = l16 & 3;
      for (int ks = 0; ks < 13; ++ks) {
        const bf16x8 a0 = tr_frag(s_d1 + ks * 32 * 32, 32, 0, lane);
        const bf16x8 a1 = tr_frag(s_d1 + ks * 32 * 32, 32, 16, lane);
        const int pa = ks * 32 + lg * 8 + q, pb = pa + 4;
        const int oya = (pa * 3277) >> 16, oyb = (pb * 3277) >> 16;   // / 20
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int c = (2 * wid + n) * 16 + 4 * pq;
          const int co = (c >> 6) * 7056 + ((c >> 3) & 7) * 84 + (c & 7);
          const int offa = pa < 400 ? co + 4 * oya * 84 + 4 * (pa - oya * 20) : BW_FR;
          const int offb = pb < 400 ? co + 4 * oyb * 84 + 4 * (pb - oyb * 20) : BW_FR;
          typedef short short4x __attribute__((ext_vector_type(4)));
          typedef __attribute__((address_space(3))) short4x lds4;
          const short4x lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(s_fr + offa));
          const short4x hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(s_fr + offb));
          const short8v bv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          const bf16x8 bf = __builtin_bit_cast(bf16x8, bv);
          w1acc[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf, w1acc[0][n], 0, 0, 0);
          w1acc[1][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf, w1acc[1][n], 0, 0, 0);
        }
      }
      __syncthreads();   // the dy1 rows / frames are read before the next sample's images land on them
    }
    pst(it, 5);
  }
  if constexpr (W1G) {
    float* const pl = wf.planes + (size_t)blockIdx.x * 32 * 256;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          pl[(size_t)(16 * m + 4 * lg + r) * 256 + (2 * wid + n) * 16 + l16] = w1acc[m][n][r] * wf.scale;
  }
  if (bias_acc) {
    if (tid < 128) biasp[(size_t)blockIdx.x * 160 + tid] = bacc;
    if (tid < 32) biasp[(size_t)blockIdx.x * 160 + 128 + tid] = bacc1;
  }
}

// Bootstrap value V(s_T) straight from the fc partial planes: one workgroup per env, thread t -> hidden units 2t,
// 2t + 1 (fc_h2_from_parts: every plane's load of a round in flight, planes summed in order, bias + ReLU + bf16
// rounding as the GEMM epilogue), value = h . Wh[:, A] + bh[A] reduced per wave (xor tree) then over the 4 waves in
// order -- the same arithmetic as loss.hip a2c_head_kernel's bootstrap phase, so both give bit-identical values.
// Replaces GEMM-reduce + value GEMM.
__global__ void __launch_bounds__(256) fc_value_kernel(const float* __restrict__ hpart, int S, int64_t plane_stride,
                                                       const float* __restrict__ bfc, const u16* __restrict__ Wh,
                                                       int A1, const float* __restrict__ bh, float* __restrict__ out,
                                                       u16* __restrict__ h_out, int N) {
  __shared__ float s_vw[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int e = blockIdx.x;
  const int A = A1 - 1;
  const float w0 = bf2f(Wh[(2 * tid) * A1 + A]), w1 = bf2f(Wh[(2 * tid + 1) * A1 + A]);
  float hv[2];
  fc_h2_from_parts<32>(hpart, S, plane_stride, bfc, e, tid, h_out, hv);
  const float part = wave_sum(hv[0] * w0 + hv[1] * w1);
  if (lane == 0) s_vw[wv] = part;
  __syncthreads();
  if (tid == 0) out[e] = ((s_vw[0] + s_vw[1]) + (s_vw[2] + s_vw[3])) + bh[A];
}

}  // namespace aca

extern "C" hipError_t aca_fc_value(const float* hpart, int S, int64_t plane_stride, const float* bfc,
                                   const uint16_t* Wh, int A1, const float* bh, float* out, uint16_t* h_out, int N,
                                   hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  if (S < 1 || S > aca::FC_MAX_PLANES || reinterpret_cast<uintptr_t>(hpart) % 16 ||
      reinterpret_cast<uintptr_t>(bfc) % 16 || plane_stride % 4)
    return hipErrorInvalidValue;
  aca::fc_value_kernel<<<N, 256, 0, stream>>>(hpart, S, plane_stride, bfc, Wh, A1, bh, out, h_out, N);
  return hipGetLastError();
}

extern "C" hipError_t aca_cnn_trunk_fwd_s16(const uint8_t* obs, const uint16_t* W1, const float* b1,
                                            const uint16_t* W2, const float* b2, const uint16_t* W3, const float* b3,
                                            uint16_t* y1, uint16_t* y2, uint16_t* y3, int B, float scale,
                                            uint8_t* shift_out, const int64_t* obs_idx, int frag,
                                            hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if (frag)
    aca::cnn_trunk_fwd_s16_kernel<true><<<B, 256, 0, stream>>>(obs, W1, b1, W2, b2, W3, b3, y1, y2, y3, scale,
                                                                shift_out, obs_idx);
  else
    aca::cnn_trunk_fwd_s16_kernel<false><<<B, 256, 0, stream>>>(obs, W1, b1, W2, b2, W3, b3, y1, y2, y3, scale,
                                                                 shift_out, obs_idx);
  return hipGetLastError();
}

extern "C" hipError_t aca_cnn_trunk_rows(const uint8_t* obs, const uint16_t* W1, const float* b1, const uint16_t* W2,
                                         const float* b2, const uint16_t* W3, const float* b3, uint16_t* y1,
                                         uint16_t* y2, uint16_t* y3, int B, float scale, uint8_t* shift_out,
                                         uint8_t* copy_out, uint64_t* stamps, int late_w, int frag,
                                         hipStream_t stream) {
  // frag: W2 / W3 are the fragment-ordered copies (W1 row-major: the kernel stages it through LDS)
  if (B <= 0) return hipSuccess;
#define ACA_ROWS(LW, FR)                                                                                         \
  aca::cnn_trunk_rows_kernel<LW, FR><<<B * aca::TR_ROWS, aca::T_THREADS, 0, stream>>>(                          \
      obs, W1, b1, W2, b2, W3, b3, y1, y2, y3, scale, shift_out, copy_out, stamps);
  if (late_w && frag) ACA_ROWS(true, true)
  else if (late_w) ACA_ROWS(true, false)
  else if (frag) ACA_ROWS(false, true)
  else ACA_ROWS(false, false)
#undef ACA_ROWS
  return hipGetLastError();
}

extern "C" hipError_t aca_cnn_trunk_bwd(const uint16_t* dy3, const uint16_t* W3, const uint16_t* y2, const uint16_t* W2,
                                        const uint16_t* y1, uint16_t* dy2, uint16_t* dy1, float* biasp, int B,
                                        uint64_t* stamps, int persist, const uint8_t* w1_obs,
                                        const int64_t* w1_obs_idx, float* w1_planes, float w1_scale, int bias_acc,
                                        hipStream_t stream) {
  // bias_acc (persistent form): one bias-gradient row per workgroup (min(persist, B) rows) instead of one per sample
  // w1_obs: the conv1 weight gradient folded into the persistent kernel (one [32][256] plane per workgroup)
  if (B <= 0) return hipSuccess;
  for (const void* p : {(const void*)dy3, (const void*)W3, (const void*)y2, (const void*)W2, (const void*)y1,
                        (const void*)dy2, (const void*)dy1})
    if (reinterpret_cast<uintptr_t>(p) % 16) return hipErrorInvalidValue;
  if (persist > 0 && w1_obs) {
    if (!w1_planes || reinterpret_cast<uintptr_t>(w1_obs) % 16) return hipErrorInvalidValue;
    const aca::W1Fold wf{w1_obs, w1_obs_idx, w1_planes, w1_scale};
    aca::cnn_trunk_bwd_persist_kernel<true><<<persist < B ? persist : B, aca::BW_T, 0, stream>>>(
        dy3, W3, y2, W2, y1, dy2, dy1, biasp, B, stamps, bias_acc, wf);
  } else if (persist > 0) {
    aca::cnn_trunk_bwd_persist_kernel<false><<<persist < B ? persist : B, aca::BW_T, 0, stream>>>(
        dy3, W3, y2, W2, y1, dy2, dy1, biasp, B, stamps, bias_acc, aca::W1Fold{nullptr, nullptr, nullptr, 0.f});
  } else if (w1_obs) {
    return hipErrorInvalidValue;   // the conv1 fold is a persistent-kernel feature
  } else {
    aca::cnn_trunk_bwd_kernel<<<B, aca::BW_T, 0, stream>>>(dy3, W3, y2, W2, y1, dy2, dy1, biasp, stamps);
  }
  return hipGetLastError();
}

extern "C" hipError_t aca_pong_fused_step(
    uint16_t* h, const float* hpart, int S, int64_t plane_stride, const float* bfc, const uint16_t* Wh,
    const float* bh, int A, float* z, int32_t* act, float* logp, float* ent, float* value, int key_shift,
    uint32_t pseed, float* state, int32_t* t, int64_t* tg, float* ep_ret, float* state_n, int32_t* t_n,
    int64_t* tg_n, float* ep_ret_n, float* ep_stats, const int64_t* ids, const uint8_t* prev, uint8_t* out,
    float* reward, uint8_t* done, uint8_t* trunc, uint32_t seed, int max_steps, const uint16_t* W1, const float* b1,
    const uint16_t* W2, const float* b2, const uint16_t* W3, const float* b3, uint16_t* y1, uint16_t* y2,
    uint16_t* y3, float scale, uint8_t* shift_out, uint64_t* stamps, int frag, int N, hipStream_t stream) {
  // frag: W2 / W3 are the fragment-ordered copies (W1 stays row-major: the kernel stages it through LDS)
  if (N <= 0) return hipSuccess;
  aca::PongIO io;
  io.state = state; io.tsteps = t; io.tglob = tg; io.ep_ret = ep_ret; io.ep_stats = ep_stats; io.env_ids = ids;
  io.prev = prev; io.out = out; io.reward = reward; io.done_out = done; io.trunc_out = trunc; io.seed = seed;
  io.max_steps = max_steps; io.k = 4;
  aca::PongNext nx{state_n, t_n, tg_n, ep_ret_n};
  aca::FcParts fc{hpart, S, plane_stride, bfc};
  const int grid = N * aca::TR_ROWS;
  switch (A + 1) {
#define ACA_FUSED_CASE(A1)                                                                                       \
  case A1:                                                                                                       \
    if (frag)                                                                                                    \
      aca::pong_fused_step_kernel<A1, true><<<grid, aca::T_THREADS, 0, stream>>>(                                \
          io, nx, fc, h, Wh, bh, z, act, logp, ent, value, key_shift, pseed, W1, b1, W2, b2, W3, b3, y1, y2, y3,  \
          scale, shift_out, stamps);                                                                             \
    else                                                                                                         \
      aca::pong_fused_step_kernel<A1, false><<<grid, aca::T_THREADS, 0, stream>>>(                               \
          io, nx, fc, h, Wh, bh, z, act, logp, ent, value, key_shift, pseed, W1, b1, W2, b2, W3, b3, y1, y2, y3,  \
          scale, shift_out, stamps);                                                                             \
    break;
    ACA_FUSED_CASE(3) ACA_FUSED_CASE(4) ACA_FUSED_CASE(5) ACA_FUSED_CASE(6) ACA_FUSED_CASE(7)
#undef ACA_FUSED_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t aca_pong_fused_env_step(
    uint16_t* h, const float* hpart, int S, int64_t plane_stride, const float* bfc, const uint16_t* Wh,
    const float* bh, int A, float* z, int32_t* act, float* logp, float* ent, float* value, int key_shift,
    uint32_t pseed, float* state, int32_t* t, int64_t* tg, float* ep_ret, float* ep_stats, const int64_t* ids,
    uint8_t* out, float* reward, uint8_t* done, uint8_t* trunc, uint32_t seed, int max_steps, const uint16_t* W1,
    const float* b1, const uint16_t* W2, const float* b2, const uint16_t* W3, const float* b3, uint16_t* y1,
    uint16_t* y2, uint16_t* y3, float scale, uint8_t* shift_out, float* state_n, int32_t* t_n, int64_t* tg_n,
    float* ep_ret_n, uint64_t* stamps, int frag, int N, hipStream_t stream) {
  // state_n .. ep_ret_n: the other parity's env state -> two workgroups per env (commit there); null -> one.
  // frag: W2 / W3 are the fragment-ordered copies (W1 stays row-major: LDS-DMA staged)
  if (N <= 0) return hipSuccess;
  if (S < 1 || S > aca::FC_MAX_PLANES) return hipErrorInvalidValue;
  const bool split = state_n != nullptr;
  if (split && (!t_n || !tg_n || !ep_ret_n)) return hipErrorInvalidValue;
  aca::PongNext nx{state_n, t_n, tg_n, ep_ret_n};
  aca::PongIO io;
  io.state = state; io.tsteps = t; io.tglob = tg; io.ep_ret = ep_ret; io.ep_stats = ep_stats; io.env_ids = ids;
  io.prev = out; io.out = out; io.reward = reward; io.done_out = done; io.trunc_out = trunc; io.seed = seed;
  io.max_steps = max_steps; io.k = 4;
  aca::FcParts fc{hpart, S, plane_stride, bfc};
#define ACA_FES_LAUNCH(A1, SPLIT, FRAG, GRID)                                                                   \
  aca::pong_fused_env_step_kernel<A1, SPLIT, FRAG><<<GRID, 256, 0, stream>>>(                                    \
      io, nx, fc, h, Wh, bh, z, act, logp, ent, value, key_shift, pseed, W1, b1, W2, b2, W3, b3, y1, y2, y3, scale, \
      shift_out, stamps);
  switch (A + 1) {
#define ACA_FES_CASE(A1)                                                                                         \
  case A1:                                                                                                       \
    if (split && frag) ACA_FES_LAUNCH(A1, 2, true, 2 * N)                                                      \
    else if (split) ACA_FES_LAUNCH(A1, 2, false, 2 * N)                                                          \
    else if (frag) ACA_FES_LAUNCH(A1, 1, true, N)                                                                \
    else ACA_FES_LAUNCH(A1, 1, false, N)                                                                         \
    break;
    ACA_FES_CASE(3) ACA_FES_CASE(4) ACA_FES_CASE(5) ACA_FES_CASE(6) ACA_FES_CASE(7)
#undef ACA_FES_CASE
#undef ACA_FES_LAUNCH
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
