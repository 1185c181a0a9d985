// Convolution lowering for the Nature-CNN: im2col / col2im around the MFMA GEMM of gemm.hip.
//
// Layouts (chosen so that every GEMM operand is a plain strided matrix and every copy here is 16 bytes wide):
//   conv1 input   obs uint8 [B, C, H, W] (frame stack = channels), im2col k order (c, i, j), weight [O][C][KH][KW]
//                 (the /255 scaling is folded into the uint8 -> bf16 conversion)
//   conv2/3 input activations bf16 NHWC [B, H, W, C] (= the previous GEMM's [B*H*W, C] output), im2col k order
//                 (i, j, c), weight [O][KH][KW][C]
// col2im gathers (no atomics): each thread owns 8 channels of one input pixel and sums every (kernel position,
// output pixel) that touched it, applies the ReLU-backward mask of the previous layer's activation and reduces
// per-channel sums for that layer's bias gradient (LDS atomics, one global atomic per channel per workgroup).
#include "common.h"

namespace aca {

__global__ void im2col_u8_nchw_kernel(const uint8_t* __restrict__ x, u16* __restrict__ col, int B, int C, int H,
                                      int W, int KH, int KW, int S, int OH, int OW, float scale) {
  const int K = C * KH * KW, KC = K / 8;
  const int64_t total = (int64_t)B * OH * OW * KC;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int kc = (int)(idx % KC);
    const int64_t m = idx / KC;
    const int ow = (int)(m % OW), oh = (int)((m / OW) % OH), b = (int)(m / ((int64_t)OW * OH));
    union { uint4 v; u16 h[8]; } o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = kc * 8 + e;
      const int j = k % KW, i = (k / KW) % KH, c = k / (KW * KH);
      const uint8_t px = x[(((int64_t)b * C + c) * H + oh * S + i) * W + ow * S + j];
      o.h[e] = f2bf((float)px * scale);
    }
    reinterpret_cast<uint4*>(col)[idx] = o.v;
  }
}

// fast path: KW % 4 == 0, S % 4 == 0, W % 4 == 0 -> every 8-element k chunk is two aligned 4-byte loads
__global__ void im2col_u8_nchw_vec_kernel(const uint8_t* __restrict__ x, u16* __restrict__ col, int B, int C, int H,
                                          int W, int KH, int KW, int S, int OH, int OW, float scale) {
  const int K = C * KH * KW, KC = K / 8;
  const int64_t total = (int64_t)B * OH * OW * KC;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int kc = (int)(idx % KC);
    const int64_t m = idx / KC;
    const int ow = (int)(m % OW), oh = (int)((m / OW) % OH), b = (int)(m / ((int64_t)OW * OH));
    const int k0 = kc * 8;
    const int j0 = k0 % KW, i = (k0 / KW) % KH, c = k0 / (KW * KH);
    const uint8_t* src = x + (((int64_t)b * C + c) * H + oh * S + i) * W + ow * S + j0;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(src);
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(src + 4);
    union { uint4 v; u16 h[8]; } o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o.h[e] = f2bf((float)((w0 >> (8 * e)) & 0xFF) * scale);
      o.h[4 + e] = f2bf((float)((w1 >> (8 * e)) & 0xFF) * scale);
    }
    reinterpret_cast<uint4*>(col)[idx] = o.v;
  }
}

__global__ void im2col_nhwc_kernel(const u16* __restrict__ x, u16* __restrict__ col, int B, int C, int H, int W,
                                   int KH, int KW, int S, int OH, int OW) {
  const int CC = C / 8, KC = KH * KW * CC;
  const int64_t total = (int64_t)B * OH * OW * KC;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int kc = (int)(idx % KC);
    const int64_t m = idx / KC;
    const int ow = (int)(m % OW), oh = (int)((m / OW) % OH), b = (int)(m / ((int64_t)OW * OH));
    const int cc = kc % CC, j = (kc / CC) % KW, i = kc / (CC * KW);
    const uint4 v = reinterpret_cast<const uint4*>(x)[((((int64_t)b * H + oh * S + i) * W + ow * S + j) * C) / 8 + cc];
    reinterpret_cast<uint4*>(col)[idx] = v;
  }
}

// dcol [B*OH*OW, KH*KW*C] (k order (i, j, c)) -> dx [B, H, W, C], masked by (ymask > 0), bias-grad colsum
__global__ void __launch_bounds__(256) col2im_nhwc_kernel(const u16* __restrict__ dcol, const u16* __restrict__ ymask,
                                                          u16* __restrict__ dx, float* __restrict__ colsum, int B,
                                                          int C, int H, int W, int KH, int KW, int S, int OH,
                                                          int OW) {
  extern __shared__ __attribute__((aligned(16))) float csum[];  // [C]
  for (int c = threadIdx.x; c < C; c += blockDim.x) csum[c] = 0.f;
  __syncthreads();
  const int CC = C / 8;
  const int K = KH * KW * C;
  const int64_t total = (int64_t)B * H * W * CC;
  float part[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(idx % CC);
    const int64_t pix = idx / CC;
    const int xw = (int)(pix % W), yh = (int)((pix / W) % H), b = (int)(pix / ((int64_t)W * H));
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < KH; ++i) {
      const int ty = yh - i;
      if (ty < 0 || ty % S) continue;
      const int oh = ty / S;
      if (oh >= OH) continue;
      for (int j = 0; j < KW; ++j) {
        const int tx = xw - j;
        if (tx < 0 || tx % S) continue;
        const int ow = tx / S;
        if (ow >= OW) continue;
        const int64_t m = ((int64_t)b * OH + oh) * OW + ow;
        union { uint4 v; u16 h[8]; } d;
        d.v = *reinterpret_cast<const uint4*>(dcol + m * K + (i * KW + j) * C + cc * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += bf2f(d.h[e]);
      }
    }
    union { uint4 v; u16 h[8]; } mk, o;
    mk.v = reinterpret_cast<const uint4*>(ymask)[idx];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = bf2f(mk.h[e]) > 0.f ? acc[e] : 0.f;
      o.h[e] = f2bf(v);
      part[e] += bf2f(o.h[e]);
    }
    reinterpret_cast<uint4*>(dx)[idx] = o.v;
  }
  if (colsum) {
    // lanes l, l+CC, l+2CC, ... of a wave hold the same channel chunk (CC divides 64 and the grid stride is a
    // multiple of 64): reduce across them in registers, then one LDS atomic per channel per wave
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = part[e];
#pragma unroll
      for (int o = 32; o >= CC; o >>= 1) v += lane_xor(v, o);
      part[e] = v;
    }
    const int lane = threadIdx.x & 63;
    if (lane < CC) {
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(&csum[lane * 8 + e], part[e]);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) atomicAdd(&colsum[c], csum[c]);
  }
}

// column sums of a bf16 [M, N] matrix (bias gradient when no producer kernel fused it)
__global__ void colsum_bf16_kernel(const u16* __restrict__ x, int64_t M, int N, int64_t ld, float* __restrict__ out) {
  const int n = blockIdx.y * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int64_t m = blockIdx.x; m < M; m += gridDim.x) s += bf2f(x[m * ld + n]);
  atomicAdd(&out[n], s);
}

// out[n % mod] += sum_r part[r][n] (the GEMM's per-row-tile column-sum partials): 8 row lanes x 32 columns per
// workgroup over 512 rows, one atomic per column per workgroup (a few dozen adds per address instead of thousands)
__global__ void __launch_bounds__(256) colsum_reduce_kernel(const float* __restrict__ part, int R, int N,
                                                            float* __restrict__ out, int mod) {
  __shared__ float sh[8][33];
  const int c = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int n = blockIdx.y * 32 + c;
  const int r1 = min(R, (int)(blockIdx.x + 1) * 512);
  float s = 0.f;
  if (n < N) {
#pragma unroll 8
    for (int r = blockIdx.x * 512 + rl; r < r1; r += 8) s += part[(int64_t)r * N + n];
  }
  sh[rl][c] = s;
  __syncthreads();
  if (rl == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += sh[i][c];
    atomicAdd(&out[mod ? n % mod : n], t);
  }
}

static int grid_for(int64_t total, int bs) {
  int64_t g = (total + bs - 1) / bs;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace aca

using namespace aca;

extern "C" hipError_t aca_im2col_u8_nchw(const uint8_t* x, uint16_t* col, int B, int C, int H, int W, int KH, int KW,
                                         int S, float scale, hipStream_t stream) {
  const int OH = (H - KH) / S + 1, OW = (W - KW) / S + 1;
  if ((C * KH * KW) % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)B * OH * OW * (C * KH * KW / 8);
  if (KW % 8 == 0 && S % 4 == 0 && W % 4 == 0)
    im2col_u8_nchw_vec_kernel<<<grid_for(total, 256), 256, 0, stream>>>(x, col, B, C, H, W, KH, KW, S, OH, OW, scale);
  else
    im2col_u8_nchw_kernel<<<grid_for(total, 256), 256, 0, stream>>>(x, col, B, C, H, W, KH, KW, S, OH, OW, scale);
  return hipGetLastError();
}

extern "C" hipError_t aca_im2col_nhwc(const uint16_t* x, uint16_t* col, int B, int C, int H, int W, int KH, int KW,
                                      int S, hipStream_t stream) {
  const int OH = (H - KH) / S + 1, OW = (W - KW) / S + 1;
  if (C % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)B * OH * OW * KH * KW * (C / 8);
  im2col_nhwc_kernel<<<grid_for(total, 256), 256, 0, stream>>>(x, col, B, C, H, W, KH, KW, S, OH, OW);
  return hipGetLastError();
}

extern "C" hipError_t aca_col2im_nhwc(const uint16_t* dcol, const uint16_t* ymask, uint16_t* dx, float* colsum, int B,
                                      int C, int H, int W, int KH, int KW, int S, hipStream_t stream) {
  const int OH = (H - KH) / S + 1, OW = (W - KW) / S + 1;
  if (C % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)B * H * W * (C / 8);
  if (64 % (C / 8)) return hipErrorInvalidValue;  // the wave-level channel reduction needs C/8 | 64
  col2im_nhwc_kernel<<<grid_for(total, 256), 256, C * sizeof(float), stream>>>(dcol, ymask, dx, colsum, B, C, H, W,
                                                                               KH, KW, S, OH, OW);
  return hipGetLastError();
}

extern "C" hipError_t aca_colsum_bf16(const uint16_t* x, int64_t M, int N, int64_t ld, float* out,
                                      hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  dim3 grid((unsigned)(M < 256 ? M : 256), (N + 63) / 64);
  colsum_bf16_kernel<<<grid, 64, 0, stream>>>(x, M, N, ld, out);
  return hipGetLastError();
}

extern "C" hipError_t aca_colsum_reduce(const float* part, int R, int N, float* out, int mod, hipStream_t stream) {
  if (R <= 0 || N <= 0) return hipSuccess;
  dim3 grid((R + 511) / 512, (N + 31) / 32);
  colsum_reduce_kernel<<<grid, 256, 0, stream>>>(part, R, N, out, mod);
  return hipGetLastError();
}
