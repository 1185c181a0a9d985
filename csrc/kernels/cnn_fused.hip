// Fused Nature-CNN trunk for rollout inference: conv1 -> conv2 -> conv3 of ONE env per workgroup, activations in
// LDS, one launch for the whole trunk (SURVEY §2.4 K03, §7.5 hard part 1: at 32 envs per GPU the rollout is
// latency-bound, so the three per-layer GEMM launches -- each a couple of memory round trips plus a kernel
// boundary -- collapse into one launch whose layers hand off through LDS).
//
//   obs uint8 [4, 84, 84] --LDS--> conv1 (K 256 = (c, i, j), MFMA 16x16x32) --> y1 [400, 32] bf16 (LDS + global)
//                                  conv2 (K 512 = (i, j, c))                  --> y2 [81, 64]  bf16 (LDS + global)
//                                  conv3 (K 576 = (i, j, c))                  --> y3 [49, 64]  bf16 (global)
//
// y1 / y2 / y3 are also written to global memory: they are the learner's saved activations (the A2C learner reuses
// the rollout's forward pass) and y3 feeds the fc GEMM. Weights are the bf16 shadow of the parameter slab in the
// engine's layouts (W1 [32][256] OIHW, W2 [64][512] / W3 [64][576] OHWI); conv1 weights are staged in LDS, conv2/3
// B fragments are streamed from L2 straight into registers (each is used once per wave), all issued before the
// first MFMA of the layer. Work split: conv1 -- waves take M tiles round-robin and both N tiles; conv2/3 -- wave w
// owns output-channel tile w for every M tile, so every B fragment is loaded exactly once per workgroup.
#include "common.h"

namespace aca {

constexpr int T_THREADS = 256;
constexpr int OBS_BYTES = 4 * 84 * 84;       // 28224
constexpr int W1_LD = 256 + 8;               // padded LDS row (bf16)
constexpr int Y1_ROWS = 400, Y1_C = 32;
constexpr int Y2_ROWS = 81, Y2_C = 64;
constexpr int Y3_ROWS = 49, Y3_C = 64;

typedef short short8v __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8 u8x8_to_bf16(uint32_t w0, uint32_t w1, float scale) {
  short8v r;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    r[e] = (short)f2bf((float)((w0 >> (8 * e)) & 0xFF) * scale);
    r[4 + e] = (short)f2bf((float)((w1 >> (8 * e)) & 0xFF) * scale);
  }
  return __builtin_bit_cast(bf16x8, r);
}

__global__ void __launch_bounds__(T_THREADS) cnn_trunk_fwd_kernel(
    const uint8_t* __restrict__ obs, const u16* __restrict__ W1, const float* __restrict__ b1,
    const u16* __restrict__ W2, const float* __restrict__ b2, const u16* __restrict__ W3,
    const float* __restrict__ b3, u16* __restrict__ y1g, u16* __restrict__ y2g, u16* __restrict__ y3g,
    float scale) {
  __shared__ __attribute__((aligned(16))) uint8_t s_obs[OBS_BYTES];
  __shared__ __attribute__((aligned(16))) u16 s_w1[32 * W1_LD];
  __shared__ __attribute__((aligned(16))) u16 s_y1[Y1_ROWS * Y1_C];
  __shared__ __attribute__((aligned(16))) u16 s_y2[Y2_ROWS * Y2_C];

  const int e = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;

  // ---------------------------------------------------------------- stage obs + W1 in LDS (16-byte copies)
  {
    const uint4* src = reinterpret_cast<const uint4*>(obs + (size_t)e * OBS_BYTES);
    uint4* dst = reinterpret_cast<uint4*>(s_obs);
    for (int i = tid; i < OBS_BYTES / 16; i += T_THREADS) dst[i] = src[i];
    for (int i = tid; i < 32 * 256 / 8; i += T_THREADS) {
      const int r = i / 32, c8 = (i % 32) * 8;
      *reinterpret_cast<uint4*>(s_w1 + r * W1_LD + c8) = *reinterpret_cast<const uint4*>(W1 + r * 256 + c8);
    }
  }
  __syncthreads();

  // ---------------------------------------------------------------- conv1: M 400 (25 tiles), N 32 (2), K 256 (8)
  {
    bf16x8 bw[2][8];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
        bw[nt][ks] = *reinterpret_cast<const bf16x8*>(s_w1 + (nt * 16 + l16) * W1_LD + ks * 32 + lg * 8);
    const float bias0 = b1[l16], bias1 = b1[16 + l16];
    for (int mt = wid; mt < 25; mt += 4) {
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const int m = mt * 16 + l16;
      const int oh = m / 20, ow = m - oh * 20;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int k = ks * 32 + lg * 8;             // (c, i, j0 = 0): c = k / 64, i = (k / 8) % 8
        const int c = k >> 6, i = (k >> 3) & 7;
        const uint8_t* p = s_obs + (c * 84 + oh * 4 + i) * 84 + ow * 4;
        const uint32_t w0 = *reinterpret_cast<const uint32_t*>(p);
        const uint32_t w1 = *reinterpret_cast<const uint32_t*>(p + 4);
        const bf16x8 a = u8x8_to_bf16(w0, w1, scale);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[0][ks], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[1][ks], acc1, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r;
        const u16 v0 = f2bf(fmaxf(acc0[r] + bias0, 0.f));
        const u16 v1 = f2bf(fmaxf(acc1[r] + bias1, 0.f));
        s_y1[row * Y1_C + l16] = v0;
        s_y1[row * Y1_C + 16 + l16] = v1;
        y1g[((size_t)e * Y1_ROWS + row) * Y1_C + l16] = v0;
        y1g[((size_t)e * Y1_ROWS + row) * Y1_C + 16 + l16] = v1;
      }
    }
  }
  __syncthreads();

  // ---------------------------------------------------------------- conv2: M 81 (6 tiles), N 64 (wave = N tile), K 512
  {
    const int n = wid * 16 + l16;
    bf16x8 bw[16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) bw[ks] = *reinterpret_cast<const bf16x8*>(W2 + n * 512 + ks * 32 + lg * 8);
    const float bias = b2[n];
    floatx4 acc[6];
#pragma unroll
    for (int mt = 0; mt < 6; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int k = ks * 32 + lg * 8;   // (i, j, c0): i = k / 128, j = (k / 32) % 4, c0 = k % 32
      const int i = k >> 7, j = (k >> 5) & 3, c0 = k & 31;
#pragma unroll
      for (int mt = 0; mt < 6; ++mt) {
        const int m = mt * 16 + l16;
        bf16x8 a;
        if (m < Y2_ROWS) {
          const int oh = m / 9, ow = m - oh * 9;
          a = *reinterpret_cast<const bf16x8*>(s_y1 + ((oh * 2 + i) * 20 + ow * 2 + j) * Y1_C + c0);
        } else {
          a = __builtin_bit_cast(bf16x8, short8v{0, 0, 0, 0, 0, 0, 0, 0});
        }
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[ks], acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 6; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r;
        if (row < Y2_ROWS) {
          const u16 v = f2bf(fmaxf(acc[mt][r] + bias, 0.f));
          s_y2[row * Y2_C + n] = v;
          y2g[((size_t)e * Y2_ROWS + row) * Y2_C + n] = v;
        }
      }
    }
  }
  __syncthreads();

  // ---------------------------------------------------------------- conv3: M 49 (4 tiles), N 64 (wave = N tile), K 576
  {
    const int n = wid * 16 + l16;
    bf16x8 bw[18];
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) bw[ks] = *reinterpret_cast<const bf16x8*>(W3 + n * 576 + ks * 32 + lg * 8);
    const float bias = b3[n];
    floatx4 acc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int k = ks * 32 + lg * 8;   // (i, j, c0): i = k / 192, j = (k / 64) % 3, c0 = k % 64
      const int i = k / 192, j = (k >> 6) % 3, c0 = k & 63;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int m = mt * 16 + l16;
        bf16x8 a;
        if (m < Y3_ROWS) {
          const int oh = m / 7, ow = m - oh * 7;
          a = *reinterpret_cast<const bf16x8*>(s_y2 + ((oh + i) * 9 + ow + j) * Y2_C + c0);
        } else {
          a = __builtin_bit_cast(bf16x8, short8v{0, 0, 0, 0, 0, 0, 0, 0});
        }
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[ks], acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r;
        if (row < Y3_ROWS) y3g[((size_t)e * Y3_ROWS + row) * Y3_C + n] = f2bf(fmaxf(acc[mt][r] + bias, 0.f));
      }
    }
  }
}

}  // namespace aca

extern "C" hipError_t aca_cnn_trunk_fwd(const uint8_t* obs, const uint16_t* W1, const float* b1, const uint16_t* W2,
                                        const float* b2, const uint16_t* W3, const float* b3, uint16_t* y1,
                                        uint16_t* y2, uint16_t* y3, int B, float scale, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  aca::cnn_trunk_fwd_kernel<<<B, aca::T_THREADS, 0, stream>>>(obs, W1, b1, W2, b2, W3, b3, y1, y2, y3, scale);
  return hipGetLastError();
}
