// Consumer side of the rollout's fc product (Nature-CNN hidden layer, 512 units): the fc GEMM leaves its split-K
// partial sums as fp32 planes (GEMM out_mode 3, no in-launch reduction / fence); the kernel that needs h sums the
// planes in plane order (deterministic), adds the bias, applies ReLU and rounds to bf16 -- exactly the GEMM
// epilogue it replaces -- and stores the row for the learner, which reuses the rollout's activations.
#pragma once
#include "common.h"

namespace aca {

constexpr int FC_UNITS = 512;
constexpr int FC_MAX_PLANES = 32;  // = engine.py FC_PLANES (split-K planes of the rollout fc product)

// One wave: lane l produces hidden units 8l..8l+7 of env e into hv (bf16-rounded, as floats) and, if h_out,
// stores them. Planes are summed in plane order (deterministic), 8 planes' loads in flight per round (planes past S
// are loaded from plane 0 and discarded by a select: no data-dependent branch around the loads).
__device__ __forceinline__ void fc_h_from_parts(const float* __restrict__ hpart, int S, int64_t plane_stride,
                                                const float* __restrict__ bfc, int e, int lane,
                                                u16* __restrict__ h_out, float (&hv)[8]) {
  const float4* b4 = reinterpret_cast<const float4*>(bfc + lane * 8);
  const float4 b0 = b4[0], b1 = b4[1];
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int z0 = 0; z0 < S; z0 += 8) {
    float4 p[8][2];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int zz = z0 + u < S ? z0 + u : 0;
      const float4* src = reinterpret_cast<const float4*>(hpart + zz * plane_stride + (int64_t)e * FC_UNITS + lane * 8);
      p[u][0] = src[0];
      p[u][1] = src[1];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool on = z0 + u < S;   // select, not multiply: unused planes may hold anything
      a[0] += on ? p[u][0].x : 0.f; a[1] += on ? p[u][0].y : 0.f; a[2] += on ? p[u][0].z : 0.f;
      a[3] += on ? p[u][0].w : 0.f; a[4] += on ? p[u][1].x : 0.f; a[5] += on ? p[u][1].y : 0.f;
      a[6] += on ? p[u][1].z : 0.f; a[7] += on ? p[u][1].w : 0.f;
    }
  }
  const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  u16 hb[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    hb[r] = f2bf(fmaxf(a[r] + bb[r], 0.f));
    hv[r] = bf2f(hb[r]);
  }
  if (h_out) {
    uint4 o;
    o.x = hb[0] | ((uint32_t)hb[1] << 16);
    o.y = hb[2] | ((uint32_t)hb[3] << 16);
    o.z = hb[4] | ((uint32_t)hb[5] << 16);
    o.w = hb[6] | ((uint32_t)hb[7] << 16);
    reinterpret_cast<uint4*>(h_out + (int64_t)e * FC_UNITS)[lane] = o;
  }
}

// One workgroup of 256 threads: thread t produces hidden units 2t, 2t+1 of env e (8 planes' loads in flight per
// round; slots past S read plane 0 and are discarded by a select), bf16-rounded like the GEMM epilogue; stores
// them if h_out.
struct FcParts {        // optional: h comes from the fc GEMM's split-K partial planes
  const float* hpart;    // null: h is read as a finished bf16 row
  int S;
  int64_t plane_stride;
  const float* bfc;
};

__device__ __forceinline__ void fc_h2_from_parts(const float* __restrict__ hpart, int S, int64_t plane_stride,
                                                 const float* __restrict__ bfc, int e, int t,
                                                 u16* __restrict__ h_out, float (&hv)[2]) {
  const float2 b = *reinterpret_cast<const float2*>(bfc + 2 * t);
  float a0 = 0.f, a1 = 0.f;
  for (int z0 = 0; z0 < S; z0 += 8) {
    float2 p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int zz = z0 + u < S ? z0 + u : 0;
      p[u] = *reinterpret_cast<const float2*>(hpart + zz * plane_stride + (int64_t)e * FC_UNITS + 2 * t);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a0 += z0 + u < S ? p[u].x : 0.f;
      a1 += z0 + u < S ? p[u].y : 0.f;
    }
  }
  const u16 h0 = f2bf(fmaxf(a0 + b.x, 0.f)), h1 = f2bf(fmaxf(a1 + b.y, 0.f));
  hv[0] = bf2f(h0);
  hv[1] = bf2f(h1);
  if (h_out) reinterpret_cast<uint32_t*>(h_out + (int64_t)e * FC_UNITS)[t] = h0 | ((uint32_t)h1 << 16);
}

}  // namespace aca
