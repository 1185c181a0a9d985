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
#include "common.h"
#include "cnn_head.h"

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

__global__ void __launch_bounds__(T_THREADS) cnn_trunk_fwd_kernel(
    const uint8_t* __restrict__ obs, const u16* __restrict__ W1, const float* __restrict__ b1,
    const u16* __restrict__ W2, const float* __restrict__ b2, const u16* __restrict__ W3,
    const float* __restrict__ b3, u16* __restrict__ y1g, u16* __restrict__ y2g, u16* __restrict__ y3g,
    float scale, uint8_t* __restrict__ shift_out, uint64_t* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) u16 s_obs[OBS_BYTES];
  __shared__ __attribute__((aligned(16))) u16 s_w1[32 * W1_LD];
  __shared__ __attribute__((aligned(16))) u16 s_y1[Y1_ROWS * Y1_LD];
  __shared__ __attribute__((aligned(16))) u16 s_y2[Y2_ROWS * Y2_LD];

  const int e = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;

  // ---------------------------------------------------------------- stage obs + W1 in LDS (16-byte copies)
  stamp(stamps, 0);
  const int n2 = wid * 16 + l16;
  bf16x8 bw2[16];
  // every staging load of a thread is issued before its first LDS store (11 x 16 B in flight): one round trip
  {
    constexpr int OBS_CH = OBS_BYTES / 16, OBS_PER = (OBS_CH + T_THREADS - 1) / T_THREADS;   // 1764 -> 7
    constexpr int W1_PER = 32 * 256 / 8 / T_THREADS;                                         // 4
    const uint4* src = reinterpret_cast<const uint4*>(obs + (size_t)e * OBS_BYTES);
    uint4 vo[OBS_PER], vw[W1_PER];
#pragma unroll
    for (int u = 0; u < OBS_PER; ++u)
      if (tid + u * T_THREADS < OBS_CH) vo[u] = src[tid + u * T_THREADS];
#pragma unroll
    for (int u = 0; u < W1_PER; ++u) vw[u] = reinterpret_cast<const uint4*>(W1)[tid + u * T_THREADS];
    // W2 B fragments for conv2 (wave w owns output-channel tile w): issued behind the staging loads (returns are
    // in order, so the staging wait does not cover them), consumed two phases later
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) bw2[ks] = *reinterpret_cast<const bf16x8*>(W2 + n2 * 512 + ks * 32 + lg * 8);
    uint4* dst = reinterpret_cast<uint4*>(s_obs);
#pragma unroll
    for (int u = 0; u < OBS_PER; ++u) {
      const int i = tid + u * T_THREADS;
      if (i < OBS_CH) {
        const uint2 a = u8x4_to_bf16(vo[u].x), b = u8x4_to_bf16(vo[u].y);
        const uint2 c = u8x4_to_bf16(vo[u].z), d = u8x4_to_bf16(vo[u].w);
        dst[2 * i] = make_uint4(a.x, a.y, b.x, b.y);
        dst[2 * i + 1] = make_uint4(c.x, c.y, d.x, d.y);
      }
    }
#pragma unroll
    for (int u = 0; u < W1_PER; ++u) {
      const int i = tid + u * T_THREADS, r = i / 32, c8 = (i % 32) * 8;
      *reinterpret_cast<uint4*>(s_w1 + r * W1_LD + c8) = vw[u];
    }
    __syncthreads();
    stamp(stamps, 1);
    if (shift_out) {
      // rollout: the next observation's frame stack starts with frames 1..3 of this one (the env step then only
      // renders the newest frame): the bytes are still in registers; the stores drain behind conv1
      uint4* so = reinterpret_cast<uint4*>(shift_out + (size_t)e * OBS_BYTES);
#pragma unroll
      for (int u = 0; u < OBS_PER; ++u) {
        const int i = tid + u * T_THREADS;
        if (i >= OBS_CH / 4 && i < OBS_CH) so[i - OBS_CH / 4] = vo[u];
      }
    }
  }

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
        const u16* p = s_obs + (c * 84 + oh * 4 + i) * 84 + ow * 4;   // 8-byte aligned
        const uint2 lo = *reinterpret_cast<const uint2*>(p), hi = *reinterpret_cast<const uint2*>(p + 4);
        const bf16x8 a = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[0][ks], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[1][ks], acc1, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r;
        const u16 v0 = f2bf(fmaxf(acc0[r] * scale + bias0, 0.f));
        const u16 v1 = f2bf(fmaxf(acc1[r] * scale + bias1, 0.f));
        s_y1[row * Y1_LD + l16] = v0;
        s_y1[row * Y1_LD + 16 + l16] = v1;
        y1g[((size_t)e * Y1_ROWS + row) * Y1_C + l16] = v0;
        y1g[((size_t)e * Y1_ROWS + row) * Y1_C + 16 + l16] = v1;
      }
    }
  }
  __syncthreads();

  stamp(stamps, 2);
  // W3 B fragments, issued before conv2's MFMAs
  bf16x8 bw3[18];
#pragma unroll
  for (int ks = 0; ks < 18; ++ks) bw3[ks] = *reinterpret_cast<const bf16x8*>(W3 + n2 * 576 + ks * 32 + lg * 8);
  // ---------------------------------------------------------------- conv2: M 81 (6 tiles), N 64 (wave = N tile), K 512
  {
    const int n = n2;
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
        // rows past the 81 outputs are computed on a clamped (valid) pixel and never stored: no branch, so all
        // 96 fragment reads of the layer stay in flight together
        const int m = min(mt * 16 + l16, Y2_ROWS - 1);
        const int oh = m / 9, ow = m - oh * 9;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(s_y1 + ((oh * 2 + i) * 20 + ow * 2 + j) * Y1_LD + c0);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw2[ks], acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 6; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r;
        if (row < Y2_ROWS) {
          const u16 v = f2bf(fmaxf(acc[mt][r] + bias, 0.f));
          s_y2[row * Y2_LD + n] = v;
          y2g[((size_t)e * Y2_ROWS + row) * Y2_C + n] = v;
        }
      }
    }
  }
  __syncthreads();

  stamp(stamps, 3);
  // ---------------------------------------------------------------- conv3: M 49 (4 tiles), N 64 (wave = N tile), K 576
  {
    const int n = n2;
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
        const int m = min(mt * 16 + l16, Y3_ROWS - 1);
        const int oh = m / 7, ow = m - oh * 7;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(s_y2 + ((oh + i) * 9 + ow + j) * Y2_LD + c0);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw3[ks], acc[mt], 0, 0, 0);
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
  if (stamps) {
    stamp(stamps, 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(stamps, 5);
  }
}

// Bootstrap value V(s_T) straight from the fc partial planes: one wave per env, h = relu(sum planes + bfc)
// (bf16-rounded like the GEMM epilogue), value = h . Wh[:, A] + bh[A]. Replaces GEMM-reduce + value GEMM.
__global__ void __launch_bounds__(256) fc_value_kernel(const float* __restrict__ hpart, int S, int64_t plane_stride,
                                                       const float* __restrict__ bfc, const u16* __restrict__ Wh,
                                                       int A1, const float* __restrict__ bh, float* __restrict__ out,
                                                       u16* __restrict__ h_out, int N) {
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= N) return;
  const int A = A1 - 1;
  float wv[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) wv[r] = bf2f(Wh[(lane * 8 + r) * A1 + A]);
  float hv[8];
  fc_h_from_parts(hpart, S, plane_stride, bfc, e, lane, h_out, hv);
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < 8; ++r) acc += hv[r] * wv[r];
  acc = wave_sum(acc);
  if (lane == 0) out[e] = acc + bh[A];
}

}  // namespace aca

extern "C" hipError_t aca_fc_value(const float* hpart, int S, int64_t plane_stride, const float* bfc,
                                   const uint16_t* Wh, int A1, const float* bh, float* out, uint16_t* h_out, int N,
                                   hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  if (S < 1 || S > aca::FC_MAX_PLANES || reinterpret_cast<uintptr_t>(hpart) % 16 ||
      reinterpret_cast<uintptr_t>(bfc) % 16 || plane_stride % 4)
    return hipErrorInvalidValue;
  aca::fc_value_kernel<<<(N + 3) / 4, 256, 0, stream>>>(hpart, S, plane_stride, bfc, Wh, A1, bh, out, h_out, N);
  return hipGetLastError();
}

extern "C" hipError_t aca_cnn_trunk_fwd(const uint8_t* obs, const uint16_t* W1, const float* b1, const uint16_t* W2,
                                        const float* b2, const uint16_t* W3, const float* b3, uint16_t* y1,
                                        uint16_t* y2, uint16_t* y3, int B, float scale, uint8_t* shift_out,
                                        uint64_t* stamps, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  aca::cnn_trunk_fwd_kernel<<<B, aca::T_THREADS, 0, stream>>>(obs, W1, b1, W2, b2, W3, b3, y1, y2, y3, scale,
                                                               shift_out, stamps);
  return hipGetLastError();
}
