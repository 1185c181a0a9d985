// Policy heads: fused sample + log-prob + entropy, one launch per rollout step.
//
// categorical: logits [B, A] (fp32, row stride ldl) -> log_softmax, Gumbel-max sample with the counter-based
//   hash (stream = action index), logp(a), entropy. One 64-lane wave per row; A <= 64 handled by one pass.
// gaussian:    mu [B, A], log_std [A] clipped to [-2.5, 2.5] (Basic_AC/policies.py:49-58), Box-Muller sample,
//   sum_i log N(a_i), sum_i (1/2 + 1/2 log 2pi + log sigma_i).
// Oracles: ops/distributions.py (*_ref).
#include "common.h"

namespace aca {

// keys: explicit per-row keys, or (keys == nullptr) key = tg[row] << key_shift | env_ids[row] computed here (the
// env bank's global step counter and env id -- saves the host-side key arithmetic launches per rollout step).
// vout (optional): vout[row] = logits[row * ldl + A], i.e. copies the value column of a fused [logits | value] head.
__global__ void __launch_bounds__(256) categorical_sample_kernel(const float* __restrict__ logits, int ldl, int B,
                                                                 int A, const int64_t* __restrict__ keys,
                                                                 const int64_t* __restrict__ tg,
                                                                 const int64_t* __restrict__ env_ids, int key_shift,
                                                                 uint32_t seed, int32_t* __restrict__ act,
                                                                 float* __restrict__ logp, float* __restrict__ ent,
                                                                 float* __restrict__ vout) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= B) return;
  const bool on = lane < A;
  const float z = on ? logits[(size_t)row * ldl + lane] : -INFINITY;
  const float m = wave_max(z);
  const float ex = on ? expf(z - m) : 0.f;
  const float se = wave_sum(ex);
  const float lse = m + logf(se);
  const float lp = z - lse;  // log_softmax
  const float h = on ? -expf(lp) * lp : 0.f;
  const float H = wave_sum(h);
  // Gumbel-max
  float g = -INFINITY;
  if (on) {
    const int64_t key = keys ? keys[row] : (tg[row] * ((int64_t)1 << key_shift) + env_ids[row]);
    const float u = uniform_open(seed, key, (uint32_t)lane);
    g = z + (-logf(-logf(u)));
  }
  // argmax with first-index tie breaking
  float best = g;
  int bi = on ? lane : 1 << 30;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ob = __shfl_xor(best, o, 64);
    int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  const float lpa = __shfl(lp, bi, 64);
  if (lane == 0) {
    act[row] = bi;
    logp[row] = lpa;
    ent[row] = H;
    if (vout) vout[row] = logits[(size_t)row * ldl + A];
  }
}

__global__ void gaussian_sample_kernel(const float* __restrict__ mu, int ldm, int B, int A,
                                       const float* __restrict__ log_std, const int64_t* __restrict__ keys,
                                       uint32_t seed, float* __restrict__ act, float* __restrict__ logp,
                                       float* __restrict__ ent) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B) return;
  const float HALF_LOG_2PI = 0.91893853320467274178f, TWO_PI = 6.28318530717958647692f;
  const int64_t key = keys[row];
  float lp = 0.f, H = 0.f;
  for (int j = 0; j < A; ++j) {
    const float ls = fminf(fmaxf(log_std[j], -2.5f), 2.5f);
    const float u1 = uniform_open(seed, key, 2 * j), u2 = uniform_open(seed, key, 2 * j + 1);
    const float eps = sqrtf(-2.0f * logf(u1)) * cosf(TWO_PI * u2);
    const float m = mu[(size_t)row * ldm + j];
    const float a = m + expf(ls) * eps;
    act[(size_t)row * A + j] = a;
    const float zz = (a - m) * expf(-ls);
    lp += -0.5f * zz * zz - ls - HALF_LOG_2PI;
    H += 0.5f + HALF_LOG_2PI + ls;
  }
  logp[row] = lp;
  ent[row] = H;
}

// Policy/value head of a large learner batch (PPO minibatches, B in the thousands):
//   z[b][j] = bh[j] + sum_k h[b][k] Wh[k][j]        h bf16 [B][512], Wh bf16 [512][A1] (ld A1), z fp32 [B][A1]
// The generic GEMM runs this N = A1 <= 8 product in few workgroups that walk every k-step of an unaligned
// [512][A1] operand (~15 us at B = 4096); here 8 lanes share a row, each reading 8 interleaved 16-byte chunks of it
// (8 consecutive lanes cover 128 contiguous bytes), with Wh staged once per workgroup in LDS as fp32. Lane sums are
// combined in a fixed xor tree: deterministic, not bit-equal to the MFMA order of the GEMM path.
constexpr int HF_ROWS = 32;   // rows per 256-thread workgroup

template <int A1>
__global__ void __launch_bounds__(256) head_fwd_kernel(const u16* __restrict__ h, const u16* __restrict__ Wh,
                                                       const float* __restrict__ bh, float* __restrict__ z, int B) {
  __shared__ float s_w[512 * A1];
  for (int i = threadIdx.x; i < 512 * A1; i += 256) s_w[i] = bf2f(Wh[i]);
  const int g = threadIdx.x >> 3, t = threadIdx.x & 7;
  const int row = blockIdx.x * HF_ROWS + g;
  uint4 v[8];
  const uint4* hp = reinterpret_cast<const uint4*>(h + (size_t)min(row, B - 1) * 512);
#pragma unroll
  for (int c = 0; c < 8; ++c) v[c] = hp[c * 8 + t];   // chunk c * 8 + t: k = 64 c + 8 t + e
  __syncthreads();
  float acc[A1];
#pragma unroll
  for (int j = 0; j < A1; ++j) acc[j] = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint32_t w[4] = {v[c].x, v[c].y, v[c].z, v[c].w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = __uint_as_float((e & 1) ? (w[e >> 1] & 0xFFFF0000u) : (w[e >> 1] << 16));
      const float* wr = s_w + (64 * c + 8 * t + e) * A1;
#pragma unroll
      for (int j = 0; j < A1; ++j) acc[j] += x * wr[j];
    }
  }
#pragma unroll
  for (int j = 0; j < A1; ++j) {
    acc[j] += __shfl_xor(acc[j], 1, 64);
    acc[j] += __shfl_xor(acc[j], 2, 64);
    acc[j] += __shfl_xor(acc[j], 4, 64);
  }
  if (t == 0 && row < B)
#pragma unroll
    for (int j = 0; j < A1; ++j) z[(size_t)row * A1 + j] = acc[j] + bh[j];
}

}  // namespace aca

extern "C" hipError_t aca_head_fwd(const uint16_t* h, const uint16_t* Wh, const float* bh, float* z, int B, int A1,
                                   hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if ((reinterpret_cast<uintptr_t>(h) & 15) != 0) return hipErrorInvalidValue;
  const int grid = (B + aca::HF_ROWS - 1) / aca::HF_ROWS;
  switch (A1) {
#define ACA_HF(N) \
  case N: aca::head_fwd_kernel<N><<<grid, 256, 0, stream>>>(h, Wh, bh, z, B); break;
    ACA_HF(2) ACA_HF(3) ACA_HF(4) ACA_HF(5) ACA_HF(6) ACA_HF(7) ACA_HF(8)
#undef ACA_HF
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t aca_categorical_sample(const float* logits, int ldl, int B, int A, const int64_t* keys,
                                             const int64_t* tg, const int64_t* ids, int key_shift, uint32_t seed,
                                             int32_t* act, float* logp, float* ent, float* vout,
                                             hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if (A > 64) return hipErrorInvalidValue;
  if (!keys && (!tg || !ids)) return hipErrorInvalidValue;
  const int rows_per_block = 4;
  aca::categorical_sample_kernel<<<(B + rows_per_block - 1) / rows_per_block, 256, 0, stream>>>(
      logits, ldl, B, A, keys, tg, ids, key_shift, seed, act, logp, ent, vout);
  return hipGetLastError();
}

extern "C" hipError_t aca_gaussian_sample(const float* mu, int ldm, int B, int A, const float* log_std,
                                          const int64_t* keys, uint32_t seed, float* act, float* logp, float* ent,
                                          hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  aca::gaussian_sample_kernel<<<(B + 127) / 128, 128, 0, stream>>>(mu, ldm, B, A, log_std, keys, seed, act, logp,
                                                                   ent);
  return hipGetLastError();
}
