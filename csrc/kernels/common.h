// Shared device helpers for the gfx950 kernels of this package.
//
// Everything here is CDNA4-specific: 64-lane waves, bf16 MFMA fragments, wave-level shuffles over 64 lanes.
// The kernels are plain HIP compiled by hipcc --offload-arch=gfx950; the host wrappers in each .hip file take raw
// pointers + a hipStream_t so that only csrc/bindings.cpp has to see the (slow to compile) torch headers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ACA_WAVE 64

namespace aca {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

// per-env A2C statistics row (loss.hip a2c_head_env_kernel -> optim.hip a2c_stats_duty):
// [pg, kl, entropy, value loss, R, R^2, V, V^2, R V, unused] as fp64 sums over the env's rows
constexpr int A2C_STATS = 10;

// ------------------------------------------------------------------------------------------------------------
// Counter-based RNG. Bit-identical to actor_critic_algs_on_tensorflow_amd/envs/rng.py (lowbias32 finaliser).
// ------------------------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__host__ __device__ __forceinline__ uint32_t hash_u32(uint32_t seed, uint32_t env, uint32_t step, uint32_t stream) {
  uint32_t h = mix32(seed ^ 0x9E3779B9u);
  h = mix32(h ^ env);
  h = mix32(h ^ (step * 0x27D4EB2Fu));
  h = mix32(h ^ (stream * 0x165667B1u));
  return h;
}

// [0, 1) with 24 random bits (envs)
__device__ __forceinline__ float uniform01(uint32_t seed, uint32_t env, uint32_t step, uint32_t stream) {
  return (float)(hash_u32(seed, env, step, stream) >> 8) * (1.0f / 16777216.0f);
}

// (0, 1) open interval (policy sampling); key = 64-bit per-row key split into (lo, hi) words
__device__ __forceinline__ float uniform_open(uint32_t seed, int64_t key, uint32_t stream) {
  uint32_t lo = (uint32_t)((uint64_t)key & 0xFFFFFFFFull);
  uint32_t hi = (uint32_t)(((uint64_t)key >> 32) & 0xFFFFFFFFull);
  uint32_t h = hash_u32(seed, lo, hi, stream);
  return ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

// Keyed pseudo-random permutation of [0, n) (PPO minibatch shuffles; identical to envs/rng.py prp): three rounds
// of xor-key / odd multiply / xorshift -- each a bijection of the k-bit domain, k = ceil(log2 n) -- with cycle
// walking back into [0, n) (expected < 2 rounds since 2^k < 2n; exactly one when n is a power of two).
__host__ __device__ __forceinline__ uint32_t prp_index(uint32_t i, uint32_t n, uint32_t key) {
  uint32_t k = 1;
  while (k < 32 && (1u << k) < n) ++k;
  const uint32_t mask = k >= 32 ? 0xFFFFFFFFu : ((1u << k) - 1u);
  const uint32_t sh = (k + 1) >> 1;
  const uint32_t c0 = hash_u32(key, 0, 0x5BD1u, 3) & mask, c1 = hash_u32(key, 1, 0x5BD1u, 3) & mask,
                 c2 = hash_u32(key, 2, 0x5BD1u, 3) & mask;
  uint32_t x = i;
  do {
    x = ((x ^ c0) * 0x9E3779B1u) & mask;
    x ^= x >> sh;
    x = ((x ^ c1) * 0x85EBCA77u) & mask;
    x ^= x >> sh;
    x = ((x ^ c2) * 0xC2B2AE3Du) & mask;
    x ^= x >> sh;
  } while (x >= n);
  return x;
}

// key of the minibatch permutation of PPO epoch `ep` in update `uc` (envs/rng.py minibatch_key)
__host__ __device__ __forceinline__ uint32_t minibatch_key(uint32_t seed, int64_t uc, int ep) {
  return hash_u32(seed, (uint32_t)((uint64_t)(uc * 64 + ep) & 0xFFFFFFFFull), 7, 11);
}

// ------------------------------------------------------------------------------------------------------------
// MLP engine weight FRAGMENT copies (mlp.hip, written by the optimiser step, optim.hip OptTrans ldt -3 / -4).
// The f32 MFMA 16x16x4 B operand of a wave is 64 lanes x 4 floats; with the k index of a 16-deep k-group remapped
// to k = 16 g + 4 (lane >> 4) + s, lane l's four values of group g are 16 consecutive bytes and the wave's whole
// fragment is ONE contiguous 1 KB block at ((tile * NG + g) * 64 + l) * 4 -- a whole-line wave load (the row-major
// or transposed forms read 16 rows x 64 B per wave instruction, which the L2 -> CU path serves at a third of the
// rate, profiles/r4_l2_stream_probe.txt).
//   F (forward, Y = X W): column tiles c / 16 (ngp2(N) of them, pad zero), k-groups over K (NG = ngp2(K)):
//     element (k, c) of W [K][N] at ((c/16 * NG + k/16) * 64 + (k/4 % 4) * 16 + c % 16) * 4 + k % 4
//   G (data gradient, dX = dP W^T): tiles over K (ngp2(K)), k-groups over N (NG = ngp2(N)):
//     element (k, c) at ((k/16 * NG + c/16) * 64 + (c/4 % 4) * 16 + k % 16) * 4 + c % 4
// ------------------------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ int mlp_ngp2(int w) {   // 16-wide groups of a width, rounded up to a power of 2
  const int g = (w + 15) >> 4;
  return g <= 1 ? 1 : g <= 2 ? 2 : g <= 4 ? 4 : g <= 8 ? 8 : 16;
}
__host__ __device__ __forceinline__ uint32_t mlp_frag_f(uint32_t k, uint32_t c, int K) {
  return (((c >> 4) * (uint32_t)mlp_ngp2(K) + (k >> 4)) * 64u + ((k >> 2) & 3u) * 16u + (c & 15u)) * 4u + (k & 3u);
}
__host__ __device__ __forceinline__ uint32_t mlp_frag_g(uint32_t k, uint32_t c, int N) {
  return (((k >> 4) * (uint32_t)mlp_ngp2(N) + (c >> 4)) * 64u + ((c >> 2) & 3u) * 16u + (k & 15u)) * 4u + (c & 3u);
}

// ------------------------------------------------------------------------------------------------------------
// bf16 helpers (round-to-nearest-even through the compiler's cvt; NaN stays NaN)
// ------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ float bf2f(u16 x) { return __uint_as_float(((uint32_t)x) << 16); }
__device__ __forceinline__ u16 f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(u16, b);
}

// ------------------------------------------------------------------------------------------------------------
// wave / block reductions (64-lane waves)
// ------------------------------------------------------------------------------------------------------------
// The xor butterfly (round o pairs lane i with lane i ^ o, o = 32 .. 1), every round a register move instead of an
// LDS-crossbar permute: xor 32 / 16 by v_permlane32_swap / v_permlane16_swap (+ a select of the half that holds the
// partner), xor 8 by DPP row_ror:8, xor 4 by DPP row_shl:4 / row_shr:4 (+ select), xor 2 / 1 by quad-permute DPP.
// Same pairing and operand order as the ds_bpermute form (wave_sum_ref): bit-identical results in every lane
// (tests/test_gpu_r4.py checks both on random data).
__device__ __forceinline__ float xor32f(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float((threadIdx.x & 32) ? p[0] : p[1]);
}
__device__ __forceinline__ float xor16f(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float((threadIdx.x & 16) ? p[0] : p[1]);
}
__device__ __forceinline__ float xor8f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));   // row_ror:8
}
__device__ __forceinline__ float xor4f(float v) {
  const int up = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x104, 0xF, 0xF, false);   // row_shl:4 (i + 4)
  const int dn = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xF, 0xF, false);   // row_shr:4 (i - 4)
  return __int_as_float((threadIdx.x & 4) ? dn : up);
}
__device__ __forceinline__ float xor2f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ float xor1f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}
// partner value of lane i ^ o (o a compile-time power of two after unrolling): the register move for it
__device__ __forceinline__ float lane_xor(float v, int o) {
  switch (o) {
    case 32: return xor32f(v);
    case 16: return xor16f(v);
    case 8: return xor8f(v);
    case 4: return xor4f(v);
    case 2: return xor2f(v);
    case 1: return xor1f(v);
    default: return __shfl_xor(v, o, 64);
  }
}
__device__ __forceinline__ float wave_sum(float v) {
  v += xor32f(v);
  v += xor16f(v);
  v += xor8f(v);
  v += xor4f(v);
  v += xor2f(v);
  v += xor1f(v);
  return v;
}
__device__ __forceinline__ float wave_sum_ref(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// wave-aggregated episode statistics [sum_ret, count, sum_len] (one atomic per wave and field)
__device__ __forceinline__ void add_ep_stats(float* ep_stats, bool active, bool done, float ret, float len) {
  if (__builtin_amdgcn_ballot_w64(active && done) == 0) return;   // no episode ended in this wave (the usual step)
  float a = (active && done) ? ret : 0.f;
  float b = (active && done) ? 1.f : 0.f;
  float c = (active && done) ? len : 0.f;
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0 && b > 0.f) {
    atomicAdd(&ep_stats[0], a);
    atomicAdd(&ep_stats[1], b);
    atomicAdd(&ep_stats[2], c);
  }
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, xor32f(v));
  v = fmaxf(v, xor16f(v));
  v = fmaxf(v, xor8f(v));
  v = fmaxf(v, xor4f(v));
  v = fmaxf(v, xor2f(v));
  return fmaxf(v, xor1f(v));
}
// ------------------------------------------------------------------------------------------------------------
// Categorical head of one wave: lanes 0..A-1 hold the logits (z), the log-softmax, entropy and a Gumbel-max sample
// (first-index tie break) come back in every lane. W = 64: xor butterflies over the whole wave; W = 8 (A <= 8): the
// same trees' last three rounds only -- lanes >= A hold the neutral element (0 for sums, -inf / index 2^30 for the
// max and the argmax), so the 64-lane tree's first three rounds leave lanes 0..7 at (v + 0) and the results are
// bit-identical -- every round a register move (the ds_bpermute form was a chain of 32 LDS-crossbar round trips,
// ~1 us of the fused rollout step's sampling wave).
// ------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ int xor4i(int v) {
  const int up = __builtin_amdgcn_update_dpp(0, v, 0x104, 0xF, 0xF, false);
  const int dn = __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
  return (threadIdx.x & 4) ? dn : up;
}
__device__ __forceinline__ int xor2i(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false); }
__device__ __forceinline__ int xor1i(int v) { return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false); }

template <int W>
__device__ __forceinline__ float red_sum(float v) {
  if constexpr (W == 64) {
    return wave_sum(v);
  } else {
    static_assert(W == 8, "8 or 64 lanes");
    v = v + 0.0f;   // the first three rounds of the 64-lane tree (+0 partners): canonicalises -0
    v += xor4f(v);
    v += xor2f(v);
    v += xor1f(v);
    return v;
  }
}
template <int W>
__device__ __forceinline__ float red_max(float v) {
  if constexpr (W == 64) {
    return wave_max(v);
  } else {
    v = fmaxf(v, xor4f(v));
    v = fmaxf(v, xor2f(v));
    return fmaxf(v, xor1f(v));
  }
}
__device__ __forceinline__ void argmax_step(float& best, int& bi, float ob, int oi) {
  if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
}

struct CatSample {
  int act;     // sampled action (Gumbel-max)
  float lpa;   // its log-probability
  float H;     // entropy
};
template <int W>
__device__ __forceinline__ CatSample cat_sample(float zin, int A, int lane, uint32_t seed, int64_t key) {
  const bool on = lane < A;
  const float z = on ? zin : -INFINITY;
  const float m = red_max<W>(z);
  const float ex = on ? expf(z - m) : 0.f;
  const float lse = m + logf(red_sum<W>(ex));
  const float lp = z - lse;
  const float H = red_sum<W>(on ? -expf(lp) * lp : 0.f);
  float best = -INFINITY;
  if (on) best = z + (-logf(-logf(uniform_open(seed, key, (uint32_t)lane))));
  int bi = on ? lane : 1 << 30;
  if constexpr (W == 64) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) argmax_step(best, bi, __shfl_xor(best, o, 64), __shfl_xor(bi, o, 64));
  } else {
    argmax_step(best, bi, xor4f(best), xor4i(bi));
    argmax_step(best, bi, xor2f(best), xor2i(bi));
    argmax_step(best, bi, xor1f(best), xor1i(bi));
  }
  return CatSample{bi, __shfl(lp, bi, 64), H};
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `sh` must hold >= 16 floats. Result valid in every thread.
// global-norm clip factor min(1, max_norm / (||g|| + 1e-6)) (TF clip_by_global_norm form; <= 0: no clip). Shared by
// the optimisers (optim.hip) and the MLP weight-gradient launch with Adam folded in (mlp.hip).
__device__ __forceinline__ float grad_scale(float gnorm_sq, float max_norm) {
  if (max_norm <= 0.f) return 1.f;
  const float n = sqrtf(gnorm_sq);
  return fminf(max_norm / (n + 1e-6f), 1.0f);
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += sh[i];
  return r;
}

__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum_d(v);
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  double r = 0.0;
  for (int i = 0; i < nw; ++i) r += sh[i];
  return r;
}

// Block-wide sums of N doubles with ONE barrier pair (wave shuffles, then one cross-wave pass); `sh` must hold
// 16 * N doubles. Results valid in every thread.
template <int N>
__device__ __forceinline__ void block_sum_multi(double (&v)[N], double* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = wave_sum_d(v[i]);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < N; ++i) sh[wid * N + i] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double r = 0.0;
    for (int w = 0; w < nw; ++w) r += sh[w * N + i];
    v[i] = r;
  }
  __syncthreads();
}

// Fixed-order sum of per-workgroup records (N doubles each, `stride` apart) read by the last-arriving workgroup:
// every thread takes a strided subset (independent loads in flight), then block_sum_multi. A one-thread walk is one
// dependent cross-XCD load per record (~0.2 us each). `sh` as for block_sum_multi; results valid in every thread.
template <int N>
__device__ __forceinline__ void grid_records_sum(const double* part, int stride, unsigned nrec, double (&v)[N],
                                                 double* sh) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = 0.0;
  for (unsigned r = threadIdx.x; r < nrec; r += blockDim.x)
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += part[(size_t)r * stride + i];
  block_sum_multi<N>(v, sh);
}

// XCD-grouped work order: workgroups are dealt round-robin over the 8 XCDs (block b on XCD b % 8, observed, not
// guaranteed: a wrong guess costs locality, never correctness), so logical index xcd_remap(b, T) gives every XCD ONE
// contiguous range of the T work items -- neighbouring items (tiles of one K split, sharing their operand lines) meet
// in one L2 instead of being fetched by every XCD. A bijection on [0, T).
__device__ __forceinline__ int xcd_remap(int b, int T) {
  const int x = b & 7, s = b >> 3, q = T >> 3, rem = T & 7;
  return x * q + min(x, rem) + s;
}

// The same in chunks of g items: chunk c of g consecutive items runs on XCD c % 8, so a chunk (the tiles of one K
// split) shares one L2 while the chunks of every product are spread over all XCDs (balance). The tail past the last
// full round of 8 chunks keeps the plain order. A bijection on [0, T).
__device__ __forceinline__ int xcd_chunk_remap(int b, int T, int g) {
  const int full = (T / (8 * g)) * 8 * g;
  if (b >= full) return b;
  const int x = b & 7, s = b >> 3;
  return (x + 8 * (s / g)) * g + s % g;
}

// Last-arriver ticket (Guideline 16 counter form): every wave drains its stores, the block releases at agent
// scope and takes a ticket; returns true in every thread of the block that arrived last. The caller then reads
// the other blocks' results with plain loads (this function already performed the acquire).
__device__ __forceinline__ bool last_block_arrival(unsigned int* ticket, unsigned int nblocks, int* sh_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned int t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = (t == nblocks - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // self-cleaning: the next launch starts from 0 again
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *sh_flag = last;
  }
  __syncthreads();
  return *sh_flag != 0;
}

}  // namespace aca

#define ACA_LAUNCH_CHECK() \
  do {                     \
    (void)hipGetLastError(); \
  } while (0)
