// Fused optimisers over flat fp32 parameter slabs.
//
// The reference runs clip_by_value + ApplyAdam per variable (17 TF ops for Pendulum, Basic_AC/policies.py:79-82).
// Here one launch updates a whole slab segment:  g = clip(g, +-c) ; g *= min(1, max_norm / ||g||) ;
// Adam (TF1 "epsilon hat" form) or RMSprop (TF form, eps inside the sqrt) ; optional bf16 shadow write for the
// MFMA GEMMs. lr and the step count live in device memory, so the KL-adaptive lr controller and the schedules
// never sync with the host and the whole learner step can be captured in a hipGraph.
//
// The step counter t is read by every workgroup and advanced by the workgroup that finishes last (ticket), so no
// extra launch is needed. sumsq is deterministic: per-block partials summed in block order by the last block.
#include "common.h"

namespace aca {

constexpr int OPT_THREADS = 256;

__global__ void __launch_bounds__(OPT_THREADS) sumsq_kernel(const float* __restrict__ x, size_t n,
                                                             float* __restrict__ partial,
                                                             unsigned int* __restrict__ ticket,
                                                             float* __restrict__ out) {
  __shared__ float sh[16];
  __shared__ int flag;
  float s = 0.f;
  const size_t n4 = n / 4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = x4[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0)
    for (size_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) s += x[i] * x[i];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
  if (last_block_arrival(ticket, gridDim.x, &flag)) {
    // parallel, fixed-order (deterministic for a given grid) reduction of the per-block partials
    float t = 0.f;
    for (unsigned int b = threadIdx.x; b < gridDim.x; b += blockDim.x) t += partial[b];
    t = block_sum(t, sh);
    if (threadIdx.x == 0) *out = t;
  }
}

__device__ __forceinline__ float grad_scale(const float* gnorm_sq, float max_norm) {
  if (max_norm <= 0.f) return 1.f;
  const float n = sqrtf(*gnorm_sq);
  return fminf(max_norm / (n + 1e-6f), 1.0f);
}

template <bool ADAM>
__global__ void __launch_bounds__(OPT_THREADS) opt_kernel(float* __restrict__ p, float* __restrict__ g,
                                                          float* __restrict__ m, float* __restrict__ v, size_t n,
                                                          const float* __restrict__ lr_ptr, float* __restrict__ t_ptr,
                                                          const float* __restrict__ gnorm_sq, u16* __restrict__ shadow,
                                                          float b1, float b2, float eps, float clip, float max_norm,
                                                          unsigned int* __restrict__ ticket, int zero_grad) {
  __shared__ int flag;
  const float lr = *lr_ptr;
  const float t = ADAM ? (*t_ptr + 1.0f) : 0.f;
  const float scale = grad_scale(gnorm_sq, max_norm);
  float lr_t = lr;
  if (ADAM) lr_t = lr * sqrtf(1.0f - powf(b2, t)) / (1.0f - powf(b1, t));
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float gi = g[i];
    if (zero_grad) g[i] = 0.f;  // the next learner step accumulates into a clean slab without a memset
    if (clip > 0.f) gi = fminf(fmaxf(gi, -clip), clip);
    gi *= scale;
    float vi = v[i];
    vi = b2 * vi + (1.0f - b2) * gi * gi;
    v[i] = vi;
    float pi = p[i];
    if (ADAM) {
      float mi = b1 * m[i] + (1.0f - b1) * gi;
      m[i] = mi;
      pi -= lr_t * mi / (sqrtf(vi) + eps);
    } else {
      pi -= lr * gi / sqrtf(vi + eps);
    }
    p[i] = pi;
    if (shadow) shadow[i] = f2bf(pi);
  }
  if (ADAM) {
    if (last_block_arrival(ticket, gridDim.x, &flag)) {
      if (threadIdx.x == 0) *t_ptr = t;
    }
  }
}

__global__ void cast_bf16_kernel(const float* __restrict__ x, u16* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

static int opt_grid(size_t n) {
  size_t b = (n + OPT_THREADS * 4 - 1) / (OPT_THREADS * 4);
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (int)b;
}

}  // namespace aca

using namespace aca;

extern "C" hipError_t aca_sumsq(const float* x, size_t n, float* partial, int max_blocks, unsigned int* ticket,
                                float* out, hipStream_t stream) {
  // one workgroup per CU at most: every workgroup pays an agent-scope release (L2 write-back) for its ticket
  int grid = (int)((n / 4 + OPT_THREADS * 4 - 1) / (OPT_THREADS * 4));
  if (grid < 1) grid = 1;
  if (grid > 256) grid = 256;
  if (grid > max_blocks) grid = max_blocks;
  sumsq_kernel<<<grid, OPT_THREADS, 0, stream>>>(x, n, partial, ticket, out);
  return hipGetLastError();
}

extern "C" hipError_t aca_adam_step(float* p, float* g, float* m, float* v, size_t n, const float* lr,
                                    float* t, const float* gnorm_sq, uint16_t* shadow, float b1, float b2, float eps,
                                    float clip, float max_norm, unsigned int* ticket, int zero_grad,
                                    hipStream_t stream) {
  if (n == 0) return hipSuccess;
  opt_kernel<true><<<opt_grid(n), OPT_THREADS, 0, stream>>>(p, g, m, v, n, lr, t, gnorm_sq, shadow, b1, b2, eps,
                                                            clip, max_norm, ticket, zero_grad);
  return hipGetLastError();
}

extern "C" hipError_t aca_rmsprop_step(float* p, float* g, float* v, size_t n, const float* lr,
                                       const float* gnorm_sq, uint16_t* shadow, float alpha, float eps, float clip,
                                       float max_norm, int zero_grad, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  opt_kernel<false><<<opt_grid(n), OPT_THREADS, 0, stream>>>(p, g, nullptr, v, n, lr, nullptr, gnorm_sq, shadow,
                                                             0.f, alpha, eps, clip, max_norm, nullptr, zero_grad);
  return hipGetLastError();
}

extern "C" hipError_t aca_cast_bf16(const float* x, uint16_t* y, size_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  cast_bf16_kernel<<<opt_grid(n), OPT_THREADS, 0, stream>>>(x, y, n);
  return hipGetLastError();
}
