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
  const float z = on ? logits[(size_t)row * ldl + lane] : 0.f;
  const int64_t key = keys ? keys[row] : (tg[row] * ((int64_t)1 << key_shift) + env_ids[row]);
  // log_softmax, entropy, Gumbel-max with first-index tie breaking (common.h cat_sample: 8-lane trees for A <= 8,
  // bit-identical to the 64-lane ones)
  const CatSample cs = A <= 8 ? cat_sample<8>(z, A, lane, seed, key) : cat_sample<64>(z, A, lane, seed, key);
  const int bi = cs.act;
  const float lpa = cs.lpa, H = cs.H;
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

}  // namespace aca

// Diagnostics (tests/test_gpu_r4.py): every lane's result of the register-move wave reductions next to the
// ds_bpermute reference forms -- out [rows, 4, 64]: wave_sum, wave_sum_ref, wave_max, max via __shfl_xor.
__global__ void wave_reduce_check_kernel(const float* __restrict__ x, float* __restrict__ out, int rows) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float v = x[(size_t)row * 64 + lane];
  float m = v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float* o = out + (size_t)row * 256;
  o[lane] = aca::wave_sum(v);
  o[64 + lane] = aca::wave_sum_ref(v);
  o[128 + lane] = aca::wave_max(v);
  o[192 + lane] = m;
}

extern "C" hipError_t aca_wave_reduce_check(const float* x, float* out, int rows, hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  wave_reduce_check_kernel<<<(rows + 3) / 4, 256, 0, stream>>>(x, out, rows);
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
