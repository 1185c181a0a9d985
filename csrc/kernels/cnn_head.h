// Consumer side of the rollout's fc product (Nature-CNN hidden layer, 512 units): the fc GEMM leaves its split-K
// partial sums as fp32 planes (GEMM out_mode 3, no in-launch reduction / fence); the kernel that needs h sums the
// planes in plane order (deterministic), adds the bias, applies ReLU and rounds to bf16 -- exactly the GEMM
// epilogue it replaces -- and stores the row for the learner, which reuses the rollout's activations.
#pragma once
#include "common.h"

namespace aca {

constexpr int FC_UNITS = 512;
constexpr int FC_MAX_PLANES = 32;  // = engine.py FC_PLANES (split-K planes of the rollout fc product)

// One workgroup of 256 threads: thread t produces hidden units 2t, 2t+1 of env e (16 planes' loads in flight per
// round; slots past S read plane 0 and are discarded by a select), bf16-rounded like the GEMM epilogue; stores them
// if h_out.
struct FcParts {        // optional: h comes from the fc GEMM's split-K partial planes
  const float* hpart;    // null: h is read as a finished bf16 row
  int S;
  int64_t plane_stride;
  const float* bfc;
};

// Two-phase form: issue() requests the first round of plane loads (and the bias pair) and returns at once, so a
// kernel can queue other loads behind them; finish() sums in plane order (further rounds loaded there), exactly as
// fc_h2_from_parts.
template <int RND = 16>
struct FcH2 {
  float2 p[RND];
  float2 b;
  __device__ __forceinline__ void issue(const float* __restrict__ hpart, int S, int64_t plane_stride,
                                        const float* __restrict__ bfc, int e, int t) {
    b = *reinterpret_cast<const float2*>(bfc + 2 * t);
#pragma unroll
    for (int u = 0; u < RND; ++u)   // S is uniform: slots past it issue no load (finish() discards them)
      p[u] = u < S ? *reinterpret_cast<const float2*>(hpart + u * plane_stride + (int64_t)e * FC_UNITS + 2 * t)
                   : make_float2(0.f, 0.f);
  }
  __device__ __forceinline__ void finish(const float* __restrict__ hpart, int S, int64_t plane_stride, int e, int t,
                                         u16* __restrict__ h_out, float (&hv)[2]) {
    float a0 = 0.f, a1 = 0.f;
    for (int z0 = 0; z0 < S; z0 += RND) {
      if (z0 > 0) {
#pragma unroll
        for (int u = 0; u < RND; ++u) {
          const int zz = z0 + u < S ? z0 + u : 0;
          p[u] = *reinterpret_cast<const float2*>(hpart + zz * plane_stride + (int64_t)e * FC_UNITS + 2 * t);
        }
      }
#pragma unroll
      for (int u = 0; u < RND; ++u) {
        a0 += z0 + u < S ? p[u].x : 0.f;
        a1 += z0 + u < S ? p[u].y : 0.f;
      }
    }
    const u16 h0 = f2bf(fmaxf(a0 + b.x, 0.f)), h1 = f2bf(fmaxf(a1 + b.y, 0.f));
    hv[0] = bf2f(h0);
    hv[1] = bf2f(h1);
    if (h_out) reinterpret_cast<uint32_t*>(h_out + (int64_t)e * FC_UNITS)[t] = h0 | ((uint32_t)h1 << 16);
  }
};

template <int RND = 16>
__device__ __forceinline__ void fc_h2_from_parts(const float* __restrict__ hpart, int S, int64_t plane_stride,
                                                 const float* __restrict__ bfc, int e, int t,
                                                 u16* __restrict__ h_out, float (&hv)[2]) {
  // RND planes' loads in flight per round (the rounds are dependent memory round trips: 16 -> two rounds at the
  // rollout's 32 planes, 32 -> one; the fused rollout step keeps 16 for its register budget); the adds run in plane
  // order, so the sums are the same bit for bit whatever the round size. Planes past S are loaded from plane 0 and
  // discarded by a select.
  FcH2<RND> f;
  f.issue(hpart, S, plane_stride, bfc, e, t);
  f.finish(hpart, S, plane_stride, e, t, h_out, hv);
}

}  // namespace aca
