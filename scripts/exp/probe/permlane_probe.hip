// Probe of the gfx950 cross-lane moves used by the wave reductions: prints, per lane, the value each form returns
// when every lane holds its own index (v_permlane32_swap / v_permlane16_swap pairs, DPP row_ror:8, ds_swizzle xor 4).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  const int v = threadIdx.x;
  auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const int r8 = __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);
  const int s4 = __builtin_amdgcn_ds_swizzle(v, 0x101F);
  int* o = out + threadIdx.x * 6;
  o[0] = a[0]; o[1] = a[1]; o[2] = b[0]; o[3] = b[1]; o[4] = r8; o[5] = s4;
}
int main() {
  int* d; hipMalloc(&d, 64 * 6 * 4);
  k<<<1, 64>>>(d);
  int h[64 * 6];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("lane p32[0] p32[1] p16[0] p16[1] ror8 swz4\n");
  for (int i = 0; i < 64; ++i) printf("%d %d %d %d %d %d %d\n", i, h[i*6], h[i*6+1], h[i*6+2], h[i*6+3], h[i*6+4], h[i*6+5]);
  hipFree(d);
  return 0;
}
