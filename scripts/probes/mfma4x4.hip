// Probe of v_mfma_f32_4x4x1f32 (16 blocks): (1) lane layout -- lane l supplies a = 1000 + l, b = l; the 4 result
// registers of each lane give the A / B / D mappings (D[i][j] = a(lane of A[i]) * b(lane of B[j])); (2) issue rate of
// 4x4x1 vs 16x16x4 f32 MFMAs: one wave per SIMD, 4 independent accumulators, shader clocks per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out) {
  const int l = threadIdx.x;
  floatx4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(1000.f + l, (float)l, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) out[l * 4 + i] = c[i];
}
template <int KIND>
__global__ void rate(float* out, long long* cyc) {
  floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  const float a = threadIdx.x * 1e-3f, b = 1e-3f;
  const long long t0 = clock64();
  for (int i = 0; i < 1024; ++i) {
    if (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  float* d;
  long long* cy;
  (void)hipMalloc(&d, 1024 * sizeof(float));
  (void)hipMalloc(&cy, sizeof(long long));
  k<<<1, 64>>>(d);
  float h[256];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 8; ++l) printf("lane %d: %.0f %.0f %.0f %.0f\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  printf("lane 63: %.0f %.0f %.0f %.0f\n", h[252], h[253], h[254], h[255]);
  long long c;
  rate<0><<<1, 256>>>(d, cy);
  rate<0><<<1, 256>>>(d, cy);
  (void)hipMemcpy(&c, cy, sizeof(c), hipMemcpyDeviceToHost);
  printf("4x4x1 f32: %.2f clocks per MFMA per wave (4096 per wave)\n", c / 4096.0);
  rate<1><<<1, 256>>>(d, cy);
  rate<1><<<1, 256>>>(d, cy);
  (void)hipMemcpy(&c, cy, sizeof(c), hipMemcpyDeviceToHost);
  printf("16x16x4 f32: %.2f clocks per MFMA per wave\n", c / 4096.0);
  return 0;
}
