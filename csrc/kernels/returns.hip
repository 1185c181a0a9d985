// Return / advantage estimators over [T, N] rollouts and small statistics (K12).
//
// * gae:    reverse scan per env column, A_t = delta_t + gamma*lambda*(1-d_t)*A_{t+1}; R_t = A_t + V_t.
// * nstep:  PathAdv generalised to [T, N] (Basic_AC/run_AC.py:55-80): window [t, min(t+L, T)),
//           discounted reward sum that stops at the first terminal transition, bootstrap gamma^(h-t) V[h] only if
//           the window did not end in a terminal. One thread per (t, n).
// * normalize_adv: (A - mean) / (1e-8 + std_pop) (Basic_AC/run_AC.py:241), one workgroup, fp64 sums.
// * moments: sum, sum of squares of x and y and cross term (EV correlation Basic_AC/util.py:4-12).
// Oracles: ops/returns.py, utils/stats.py.
#include "common.h"

namespace aca {

__global__ void gae_kernel(const float* __restrict__ r, const float* __restrict__ v, const uint8_t* __restrict__ d,
                           float* __restrict__ ret, float* __restrict__ adv, int T, int N, float gamma, float lam) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float last = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    const size_t i = (size_t)t * N + n;
    const float nd = d[i] ? 0.f : 1.f;
    const float delta = r[i] + gamma * v[i + N] * nd - v[i];
    last = delta + gamma * lam * nd * last;
    adv[i] = last;
    ret[i] = last + v[i];
  }
}

__global__ void nstep_kernel(const float* __restrict__ r, const float* __restrict__ v, const uint8_t* __restrict__ d,
                             float* __restrict__ tgt, float* __restrict__ adv, int T, int N, float gamma, int L) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= T * N) return;
  const int t = idx / N, n = idx % N;
  const int h = min(t + L, T);
  float acc = 0.f, disc = 1.f;
  bool alive = true;
  for (int k = t; k < h; ++k) {
    const size_t i = (size_t)k * N + n;
    acc += disc * r[i];
    disc *= gamma;
    if (d[i]) { alive = false; break; }
  }
  if (alive) acc += disc * v[(size_t)h * N + n];
  tgt[idx] = acc;
  adv[idx] = acc - v[idx];
}

__global__ void __launch_bounds__(1024) normalize_kernel(const float* __restrict__ a, float* __restrict__ out, int n,
                                                         float eps) {
  __shared__ double sh[16];
  double s = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double x = a[i];
    s += x;
    s2 += x * x;
  }
  s = block_sum_d(s, sh);
  s2 = block_sum_d(s2, sh);
  const double mean = s / n;
  const double var = fmax(s2 / n - mean * mean, 0.0);
  const float fm = (float)mean, inv = 1.0f / (eps + (float)sqrt(var));
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = (a[i] - fm) * inv;
}

// out[0..4] = sum x, sum x^2, sum y, sum y^2, sum x*y  (fp64 accumulation, fp32 results)
__global__ void __launch_bounds__(1024) moments_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                       float* __restrict__ out, int n) {
  __shared__ double sh[16];
  double a = 0, b = 0, c = 0, dd = 0, e = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double xi = x[i], yi = y[i];
    a += xi; b += xi * xi; c += yi; dd += yi * yi; e += xi * yi;
  }
  a = block_sum_d(a, sh); b = block_sum_d(b, sh); c = block_sum_d(c, sh);
  dd = block_sum_d(dd, sh); e = block_sum_d(e, sh);
  if (threadIdx.x == 0) { out[0] = a; out[1] = b; out[2] = c; out[3] = dd; out[4] = e; }
}

// EV correlation of the reference (Basic_AC/util.py:4-12): mean(z(x) * z(y)), population std, written to *out.
__global__ void __launch_bounds__(1024) ev_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                  float* __restrict__ out, int n) {
  __shared__ double sh[16];
  double a = 0, b = 0, c = 0, dd = 0, e = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double xi = x[i], yi = y[i];
    a += xi; b += xi * xi; c += yi; dd += yi * yi; e += xi * yi;
  }
  a = block_sum_d(a, sh); b = block_sum_d(b, sh); c = block_sum_d(c, sh);
  dd = block_sum_d(dd, sh); e = block_sum_d(e, sh);
  if (threadIdx.x == 0) {
    const double mx = a / n, my = c / n;
    const double vx = b / n - mx * mx, vy = dd / n - my * my;
    const double cov = e / n - mx * my;
    *out = (float)(cov / sqrt(fmax(vx, 0.0) * fmax(vy, 0.0)));
  }
}

// PPO minibatch permutation of one epoch (csrc/kernels/common.h prp_index; oracle envs/rng.py prp)
__global__ void prp_perm_kernel(int64_t* __restrict__ out, int n, uint32_t seed, const int64_t* __restrict__ uc,
                                int ep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = prp_index((uint32_t)i, (uint32_t)n, minibatch_key(seed, *uc, ep));
}

// Per-variable statistics of a flat fp32 parameter slab (the reference's variable_summaries, Basic_AC/policies.py:
// 9-18): out[v] = (mean, population stddev, max, min) of x[off_v, off_v + n_v). One workgroup per
// variable, double accumulation (single pass: E[x^2] - mean^2 in fp64 matches the two-pass fp32 form closely).
__global__ void __launch_bounds__(256) seg_stats_kernel(const float* __restrict__ x, const int64_t* __restrict__ segs,
                                                        float* __restrict__ out) {
  __shared__ double shd[16 * 2];
  __shared__ float shf[16];
  const int v = blockIdx.x;
  const int64_t off = segs[2 * v], n = segs[2 * v + 1];
  double s = 0.0, ss = 0.0;
  float mx = -INFINITY, mn = INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const float a = x[off + i];
    s += a;
    ss += (double)a * a;
    mx = fmaxf(mx, a);
    mn = fminf(mn, a);
  }
  double r[2] = {s, ss};
  block_sum_multi<2>(r, shd);
  mx = wave_max(mx);
  mn = -wave_max(-mn);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) shf[wid] = mx;
  __syncthreads();
  float M = -INFINITY;
  for (int w = 0; w < nw; ++w) M = fmaxf(M, shf[w]);
  __syncthreads();
  if (lane == 0) shf[wid] = mn;
  __syncthreads();
  float m = INFINITY;
  for (int w = 0; w < nw; ++w) m = fminf(m, shf[w]);
  if (threadIdx.x == 0) {
    const double mean = n ? r[0] / n : 0.0;
    const double var = n ? fmax(r[1] / n - mean * mean, 0.0) : 0.0;
    out[4 * v] = (float)mean;
    out[4 * v + 1] = (float)sqrt(var);
    out[4 * v + 2] = M;
    out[4 * v + 3] = m;
  }
}

}  // namespace aca

extern "C" hipError_t aca_ev(const float* x, const float* y, float* out, int n, hipStream_t stream) {
  aca::ev_kernel<<<1, 1024, 0, stream>>>(x, y, out, n);
  return hipGetLastError();
}

extern "C" hipError_t aca_gae(const float* r, const float* v, const uint8_t* d, float* ret, float* adv, int T, int N,
                              float gamma, float lam, hipStream_t stream) {
  if (T <= 0 || N <= 0) return hipSuccess;
  aca::gae_kernel<<<(N + 255) / 256, 256, 0, stream>>>(r, v, d, ret, adv, T, N, gamma, lam);
  return hipGetLastError();
}

extern "C" hipError_t aca_nstep(const float* r, const float* v, const uint8_t* d, float* tgt, float* adv, int T,
                                int N, float gamma, int L, hipStream_t stream) {
  if (T <= 0 || N <= 0) return hipSuccess;
  const int tot = T * N;
  aca::nstep_kernel<<<(tot + 255) / 256, 256, 0, stream>>>(r, v, d, tgt, adv, T, N, gamma, L);
  return hipGetLastError();
}

extern "C" hipError_t aca_normalize(const float* a, float* out, int n, float eps, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  aca::normalize_kernel<<<1, 1024, 0, stream>>>(a, out, n, eps);
  return hipGetLastError();
}

extern "C" hipError_t aca_moments(const float* x, const float* y, float* out, int n, hipStream_t stream) {
  aca::moments_kernel<<<1, 1024, 0, stream>>>(x, y, out, n);
  return hipGetLastError();
}

extern "C" hipError_t aca_prp_perm(int64_t* out, int n, uint32_t seed, const int64_t* uc, int ep,
                                   hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  aca::prp_perm_kernel<<<(n + 255) / 256, 256, 0, stream>>>(out, n, seed, uc, ep);
  return hipGetLastError();
}

extern "C" hipError_t aca_seg_stats(const float* x, const int64_t* segs, int nv, float* out, hipStream_t stream) {
  if (nv <= 0) return hipSuccess;
  aca::seg_stats_kernel<<<nv, 256, 0, stream>>>(x, segs, out);
  return hipGetLastError();
}
