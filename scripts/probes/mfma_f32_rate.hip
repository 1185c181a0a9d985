// Probe: shader cycles per v_mfma_f32_16x16x4_f32 on this part, one workgroup of 8 waves (2 per SIMD) as in the
// MLP engine kernels: (a) one dependent accumulator chain per wave, operands in registers; (b) four independent
// chains; (c) one chain with A/B fragments read from LDS each k-group (the engine's pattern); (d) bf16 16x16x32.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/probes/mfma_f32_rate.hip -o /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int NM = 256;

template <int MODE, bool RANDOM = false>
__global__ void __launch_bounds__(512) probe(float* out, long long* cyc, float seed) {
  extern __shared__ float dyn[];   // MODE 7 / 8: operands at float offset 24576 (96 KB) / 2048 (8 KB) of 150 KB
  __shared__ float lds_s[MODE >= 7 ? 1 : 3 * 16 * 132 + 128 * 132 + 128];
  float* lds = MODE == 7 ? dyn + 24576 : MODE == 8 ? dyn + 2048 : lds_s;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 3 * 16 * 132 + 128 * 132 + 128; i += 512) {
    if (RANDOM) {   // full-entropy operands (hashed), as trained weights / activations are
      unsigned h = (unsigned)i * 2654435761u + 12345u;
      h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
      lds[i] = ((float)(h & 0xffffff) / 16777216.0f - 0.5f) * 0.2f;
    } else {
      lds[i] = seed * (float)(i & 7) * 0.01f;
    }
  }
  __syncthreads();
  float a = seed + lane, b = seed * 2.f - lane;
  floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (MODE == 0) {
#pragma unroll 16
    for (int i = 0; i < NM; ++i) c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
  } else if (MODE == 1) {
#pragma unroll 16
    for (int i = 0; i < NM; i += 4) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
  } else if (MODE == 2) {
    const float* xr = lds + (lane & 15) * 132 + 4 * (lane >> 4);
    const float* wr = lds + 4096 + (lane & 15) * 132 + 4 * (lane >> 4) + wave * 16;
    for (int rep = 0; rep < NM / 32; ++rep) {
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const float4 a4 = *reinterpret_cast<const float4*>(xr + 16 * g);
        const float4 b4 = *reinterpret_cast<const float4*>(wr + 16 * g);
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b4.x, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b4.y, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b4.z, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b4.w, c0, 0, 0, 0);
      }
    }
  } else if (MODE >= 4 && MODE <= 8) {
    // the engine's rollout layer (mlp.hip layer_fwd_lds_t<8>): X [16][132] and W [128][132] in LDS, bias, lrelu,
    // Y [16][132] written back; one 16-column tile per wave; NM / 32 layers with a barrier after each
    float* X = lds;
    float* Wm = lds + 16 * 132;
    float* Y = lds + 16 * 132 + 128 * 132;
    const float* bias = lds + 16 * 132 + 128 * 132 + 16 * 132;
    const int r = lane & 15, q = lane >> 4;
    long long mf = 0;
    for (int rep = 0; rep < NM / 32; ++rep) {
      const long long tm0 = __builtin_amdgcn_s_memtime();
      const int c = wave * 16 + r;
      const float* wrow = Wm + c * 132 + 4 * q;
      floatx4 bv[8];
#pragma unroll
      for (int g = 0; g < 8; ++g) bv[g] = *reinterpret_cast<const floatx4*>(wrow + 16 * g);
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* Xr = X + r * 132 + 4 * q;
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const float4 a4 = *reinterpret_cast<const float4*>(&Xr[16 * g]);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, bv[g][0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, bv[g][1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, bv[g][2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, bv[g][3], acc, 0, 0, 0);
      }
      const float bb = bias[c];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = acc[i] + bb;
        Y[(4 * q + i) * 132 + c] = v > 0.f ? v : 0.2f * v;
      }
      __builtin_amdgcn_s_waitcnt(0);
      mf += __builtin_amdgcn_s_memtime() - tm0;
      __syncthreads();
      if (MODE == 5) {   // an idle gap between layers (as the rollout's head / env phases): ~6k cycles asleep
        for (int z = 0; z < 48; ++z) __builtin_amdgcn_s_sleep(2);
      }
      if (MODE == 6) {   // a VALU-only gap of similar length
        float u = acc[0];
#pragma unroll 1
        for (int z = 0; z < 600; ++z) u = __builtin_fmaf(u, 0.999f, 0.001f);
        Y[lane] += u * 1e-30f;
      }
      const long long tl = __builtin_amdgcn_s_memtime();
      if (MODE != 4 && MODE < 7 && lane == 0 && rep == NM / 32 - 1) cyc[2048 + wave] = tl;
      float* t = X;   // ping-pong: this layer's output is the next one's input
      X = Y;
      Y = t;
    }
    c0 = floatx4{X[lane], 0.f, 0.f, 0.f};
    if (lane == 0) cyc[1024 + blockIdx.x * 8 + wave] = mf;   // cycles inside the layers (MFMA loop + epilogue)
  } else {
    bf16x8 av, bv;
    for (int j = 0; j < 8; ++j) { av[j] = (__bf16)(a + j); bv[j] = (__bf16)(b - j); }
#pragma unroll 16
    for (int i = 0; i < NM; ++i) c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c0, 0, 0, 0);
  }
  // consume the results before the closing stamp
  const float s = (c0[0] + c1[1]) + (c2[2] + c3[3]);
  out[blockIdx.x * 512 + threadIdx.x] = s;
  __builtin_amdgcn_s_waitcnt(0);
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}


__device__ __forceinline__ int ngp2(int w) {
  const int g = (w + 15) >> 4;
  return g <= 1 ? 1 : g <= 2 ? 2 : g <= 4 ? 4 : g <= 8 ? 8 : 16;
}
template <int NG>
__device__ void layer_rt(const float* __restrict__ X, int ldx, const float* __restrict__ W, int ldw,
                         const float* __restrict__ bias, int N, int act, float* __restrict__ Y, int ldy) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int ntile = ngp2(N);
  for (int tile = wave; tile < ntile; tile += 8) {
    const int c = tile * 16 + r;
    const bool cok = c < N;
    const int cc = cok ? c : N - 1;
    const float* wrow = W + cc * ldw + 4 * q;
    floatx4 bv[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) bv[g] = *reinterpret_cast<const floatx4*>(wrow + 16 * g);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* Xr = X + r * ldx + 4 * q;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const float4 a4 = *reinterpret_cast<const float4*>(&Xr[16 * g]);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, bv[g][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, bv[g][1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, bv[g][2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, bv[g][3], acc, 0, 0, 0);
    }
    const float bb = bias[cc];
    const float slope = act == 1 ? 0.f : act == 2 ? 0.2f : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = acc[i] + bb;
      Y[(4 * q + i) * ldy + c] = cok ? (v > 0.f ? v : slope * v) : 0.f;
    }
  }
}
__device__ void layer_sw(const float* X, int ldx, int K, const float* W, const float* bias, int N, int act, float* Y,
                         int ldy) {
  const int ldw = 16 * ngp2(K) + 4;
  switch (ngp2(K)) {
    case 1: layer_rt<1>(X, ldx, W, ldw, bias, N, act, Y, ldy); break;
    case 2: layer_rt<2>(X, ldx, W, ldw, bias, N, act, Y, ldy); break;
    case 4: layer_rt<4>(X, ldx, W, ldw, bias, N, act, Y, ldy); break;
    case 8: layer_rt<8>(X, ldx, W, ldw, bias, N, act, Y, ldy); break;
    default: layer_rt<16>(X, ldx, W, ldw, bias, N, act, Y, ldy); break;
  }
}
// MODE 10 kernel: layers of runtime shape (K, N) = (kk, nn) through the switch, as mlp_rollout_kernel calls them
__global__ void __launch_bounds__(512) probe_rt(float* out, long long* cyc, int kk, int nn, int nl) {
  extern __shared__ float sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ldx = 16 * ngp2(kk) + 4;
  float* X = sm;
  float* Y = sm + 16 * 260;
  float* W = sm + 2 * 16 * 260;
  float* bias = W + 256 * 260;
  for (int i = threadIdx.x; i < 2 * 16 * 260 + 256 * 260 + 256; i += 512) {
    unsigned h = (unsigned)i * 2654435761u + 12345u;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    sm[i] = ((float)(h & 0xffffff) / 16777216.0f - 0.5f) * 0.2f;
  }
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int l = 0; l < nl; ++l) {
    layer_sw(X, ldx, kk, W, bias, nn, 2, Y, ldx);
    __syncthreads();
    float* t = X; X = Y; Y = t;
  }
  out[threadIdx.x] = X[threadIdx.x];
  __builtin_amdgcn_s_waitcnt(0);
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[wave] = t1 - t0;
}

extern "C" int run_probe() {
  hipFuncSetAttribute(reinterpret_cast<const void*>(&probe<7>), hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  hipFuncSetAttribute(reinterpret_cast<const void*>(&probe<8>), hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&cyc, 4096 * 8);
  const char* names[10] = {"f32 16x16x4, 1 chain (regs)", "f32 16x16x4, 4 chains (regs)",
                          "f32 16x16x4, 1 chain, A/B from LDS", "bf16 16x16x32, 1 chain (regs)",
                          "engine LDS layer 128x128 (+barrier)", "engine layer, ~6k-cycle sleep between layers",
                          "engine layer, ~VALU gap between layers", "engine layer, operands at 96 KB of 150 KB dyn LDS",
                          "engine layer, operands at 8 KB of 150 KB dyn LDS",
                          "engine layer, RANDOM full-entropy operands"};
  for (int grid : {1, 64}) {
    for (int mode = 0; mode < 10; ++mode) {
      for (int rep = 0; rep < 3; ++rep) {
        if (mode == 0) probe<0><<<grid, 512>>>(out, cyc, 1.0f);
        if (mode == 1) probe<1><<<grid, 512>>>(out, cyc, 1.0f);
        if (mode == 2) probe<2><<<grid, 512>>>(out, cyc, 1.0f);
        if (mode == 3) probe<3><<<grid, 512>>>(out, cyc, 1.0f);
        if (mode == 4) probe<4><<<grid, 512>>>(out, cyc, 1.0f);
        if (mode == 5) probe<5><<<grid, 512>>>(out, cyc, 1.0f);
        if (mode == 6) probe<6><<<grid, 512>>>(out, cyc, 1.0f);
        if (mode == 7) probe<7><<<grid, 512, 150 * 1024>>>(out, cyc, 1.0f);
        if (mode == 8) probe<8><<<grid, 512, 150 * 1024>>>(out, cyc, 1.0f);
        if (mode == 9) probe<4, true><<<grid, 512>>>(out, cyc, 1.0f);
      }
      hipDeviceSynchronize();
      long long h[8];
      hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      long long mx = 0;
      for (int w = 0; w < 8; ++w) mx = h[w] > mx ? h[w] : mx;
      printf("grid %3d  %-45s  max wave cycles %7lld  -> %.1f cycles per MFMA per wave, %.1f per SIMD (2 waves)\n",
             grid, names[mode], mx, (double)mx / NM, (double)mx / (2 * NM));
      if (mode >= 4) {  // (mode 9 is MODE 4 on random data)
        hipMemcpy(h, cyc + 1024, sizeof(h), hipMemcpyDeviceToHost);
        long long m2 = 0;
        for (int w = 0; w < 8; ++w) m2 = h[w] > m2 ? h[w] : m2;
        printf("          cycles inside the 8 layers (MFMA loop + epilogue, max wave): %lld = %.0f per layer\n", m2,
               m2 / 8.0);
      }
    }
  }
  hipFuncSetAttribute(reinterpret_cast<const void*>(&probe_rt), hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  for (int rep = 0; rep < 3; ++rep) probe_rt<<<1, 512, 150 * 1024>>>(out, cyc, 128, 128, 8);
  hipDeviceSynchronize();
  long long h2[8];
  hipMemcpy(h2, cyc, sizeof(h2), hipMemcpyDeviceToHost);
  long long m3 = 0;
  for (int w = 0; w < 8; ++w) m3 = h2[w] > m3 ? h2[w] : m3;
  printf("runtime-shape layer via switch (the engine's code), 8 layers 128x128: %lld cycles = %.0f per layer\n", m3,
         m3 / 8.0);
  return 0;
}

#ifndef PROBE_LIB
int main() { return run_probe(); }
#endif
