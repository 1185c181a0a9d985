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

// PPO minibatch gather of the CNN engine (replaces six index_select copies + the permutation launch
// per minibatch): workgroup i copies batch row src = prp_index(off + i, n, key(seed, update, epoch)) -- the keyed
// epoch permutation of envs/rng.py, computed in place -- i.e. the frame stack (R bytes, 16 B vector copies) and the
// per-row action / logp / advantage / return / old value.
__global__ void __launch_bounds__(256) mb_gather_kernel(const uint8_t* __restrict__ obs, int64_t R,
                                                        const int* __restrict__ act, const float* __restrict__ logp,
                                                        const float* __restrict__ adv, const float* __restrict__ ret,
                                                        const float* __restrict__ v, uint8_t* __restrict__ o_obs,
                                                        int* __restrict__ o_act, float* __restrict__ o_logp,
                                                        float* __restrict__ o_adv, float* __restrict__ o_ret,
                                                        float* __restrict__ o_v, int n, uint32_t seed,
                                                        int64_t* uc, int ep, int off,
                                                        const double* __restrict__ mom, float eps,
                                                        unsigned int* __restrict__ bump_ticket,
                                                        int64_t* __restrict__ o_idx, int mb) {
  const int64_t ucv = *uc;
  if (o_idx) {
    // index mode (o_obs null): one thread per row writes the source row index instead of copying the observation;
    // the minibatch's trunk forward and conv1 weight gradient read obs[o_idx[i]] directly (one 28 KB copy per row
    // less)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < mb) {
      const uint32_t src = prp_index((uint32_t)(off + i), (uint32_t)n, minibatch_key(seed, ucv, ep));
      float a_ = adv[src];
      if (mom) {
        const double cnt = mom[0], mean = mom[1] / cnt, var = fmax(mom[2] / cnt - mean * mean, 0.0);
        a_ = (a_ - (float)mean) * (1.0f / (eps + (float)sqrt(var)));
      }
      o_idx[i] = src;
      o_act[i] = act[src];
      o_logp[i] = logp[src];
      o_adv[i] = a_;
      o_ret[i] = ret[src];
      o_v[i] = v[src];
    }
  } else {
  const int i = blockIdx.x;
  const uint32_t src = prp_index((uint32_t)(off + i), (uint32_t)n, minibatch_key(seed, ucv, ep));
  const uint8_t* s = obs + (size_t)src * R;
  uint8_t* d = o_obs + (size_t)i * R;
  if ((R & 15) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
    uint4* d4 = reinterpret_cast<uint4*>(d);
    const int n4 = (int)(R >> 4);
    int j = threadIdx.x;
    for (; j + 3 * 256 < n4; j += 4 * 256) {   // four 16 B loads in flight per thread
      const uint4 a = s4[j], b = s4[j + 256], c = s4[j + 512], e = s4[j + 768];
      d4[j] = a; d4[j + 256] = b; d4[j + 512] = c; d4[j + 768] = e;
    }
    for (; j < n4; j += 256) d4[j] = s4[j];
  } else {
    for (int64_t j = threadIdx.x; j < R; j += 256) d[j] = s[j];
  }
  if (threadIdx.x == 0) {
    float a_ = adv[src];
    if (mom) {   // advantage normalisation deferred from the returns scan (population std, fp64 totals)
      const double cnt = mom[0], mean = mom[1] / cnt, var = fmax(mom[2] / cnt - mean * mean, 0.0);
      a_ = (a_ - (float)mean) * (1.0f / (eps + (float)sqrt(var)));
    }
    o_act[i] = act[src];
    o_logp[i] = logp[src];
    o_adv[i] = a_;
    o_ret[i] = ret[src];
    o_v[i] = v[src];
  }
  }
  if (bump_ticket) {
    // last minibatch of the update: the workgroup that finishes last advances the update counter. Only a count is
    // handed over (every workgroup read *uc before its ticket), so the ticket is relaxed, with no release fence.
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned int prev = __hip_atomic_fetch_add(bump_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == gridDim.x - 1u) {
        *uc = ucv + 1;
        __hip_atomic_store(bump_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
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

// ------------------------------------------------------------------------------------------------------------------
// Chunked associative return scan fused with the batch statistics (reference
// Basic_AC/run_AC.py:63-75, 241 and Basic_AC/util.py:4-12).
//
// Both estimators are reverse affine recurrences x_t = a_t + c_t x_{t+1}:
//   GAE      a_t = r_t + gamma V_{t+1} (1-d_t) - V_t,  c_t = gamma lambda (1-d_t),  x_T = 0      -> adv, ret = adv + V
//   n-step   a_t = r_t,                              c_t = gamma (1-d_t),           x_T = V_T  -> target (L >= T)
// A workgroup owns E env columns x CH time chunks of K steps (thread = (chunk, env), env-fastest so every time
// step is one coalesced row segment). Pass 1 composes each chunk's affine map (fp64), a Hillis-Steele suffix scan
// over the CH chunk maps in LDS gives every chunk its incoming carry, pass 2 replays the chunk with that carry and
// writes the outputs. A truncated window (n-step, L < T) scans the un-bootstrapped return Gz (x_T = 0) together
// with the next-terminal index (suffix min) and fixes each window in a third pass:
//   target_t = Gz_t + [no terminal in [t, h)] gamma^(h-t) (V_h - Gz_h),  h = min(t + L, T), Gz_T = 0,
// the prefix-sum form of the O(L) window of Basic_AC/run_AC.py:63-75.
// Every workgroup reduces its moments (adv, adv^2, ret, ret^2, V, V^2, ret*V) in fixed order into its partial
// slot; the last workgroup to arrive sums the slots in block order (bitwise reproducible), writes the totals
// (mom[0] = count, for the DP all-reduce), the EV-before correlation, and -- if `norm` -- normalises the whole
// advantage array in place, so returns + EV + advantage normalisation are ONE launch.
constexpr int RS_THREADS = 256;
constexpr int RS_MOM = 7;
constexpr int RS_KREG = 8;   // chunks up to this many steps stay in registers between the passes

struct RetScanArgs {
  const float* r;
  const float* v;
  const uint8_t* d;
  float* ret;
  float* adv;
  double* gz;            // [T, N] (truncated n-step windows only)
  double* part;          // [gridDim.x, 8]
  unsigned int* ticket;  // zero before the first launch; self-cleaning
  double* mom;           // [8]: count, then the RS_MOM sums
  float* ev_out;         // EV(ret, V[:T]) or null
  int T, N, E, CH, K, mode, L, norm;
  float gamma, lam, eps;
};

__global__ void __launch_bounds__(RS_THREADS) returns_scan_kernel(RetScanArgs a) {
  __shared__ double s_a[RS_THREADS], s_c[RS_THREADS];
  __shared__ int s_ft[RS_THREADS];
  __shared__ double s_red[16 * RS_MOM];
  __shared__ double s_tot[8];
  __shared__ int s_flag;
  const int tid = threadIdx.x;
  const int e = tid % a.E, ch = tid / a.E;   // env-fastest: every time step of a chunk is one coalesced row
  const int T = a.T, N = a.N;
  const int n = blockIdx.x * a.E + e;
  const bool live = n < N && ch < a.CH;
  const int t0 = min(ch * a.K, T), t1 = min(t0 + a.K, T);
  const bool gae = a.mode == 2;
  const bool window = !gae && a.L < T;
  const double g = a.gamma, gl = (double)a.gamma * (double)a.lam;

  // every operand of the thread's chunk is requested up front (chunks of <= RS_KREG steps are kept in registers
  // for pass 2: one global round trip for the whole kernel instead of one per pass)
  const double init = (live && !gae && !window) ? (double)a.v[(size_t)T * N + n] : 0.0;
  const bool regs = a.K <= RS_KREG;
  float cr[RS_KREG], cv[RS_KREG], cvn[RS_KREG];
  uint8_t cd[RS_KREG];
  if (regs) {
#pragma unroll
    for (int u = 0; u < RS_KREG; ++u) {   // u-th step from the chunk's end; clamped (unconditional) loads
      const int t = max(t1 - 1 - u, 0);
      const size_t i = (size_t)t * N + (live ? n : 0);
      cr[u] = a.r[i];
      cv[u] = a.v[i];
      cvn[u] = a.v[i + N];
      cd[u] = a.d[i];
    }
  }
  // pass 1: chunk map x_{t0} = ca + cc x_{t1}, first terminal index in the chunk
  double ca = 0.0, cc = 1.0;
  int ft = T;
  if (live && regs) {
#pragma unroll
    for (int u = 0; u < RS_KREG; ++u) {
      const int t = t1 - 1 - u;
      if (t >= t0) {
        const bool dn = cd[u] != 0;
        const double nd = dn ? 0.0 : 1.0;
        ft = dn ? t : ft;
        const double x = gae ? (double)cr[u] + g * (double)cvn[u] * nd - (double)cv[u] : (double)cr[u];
        const double c = (gae ? gl : g) * nd;
        ca = x + c * ca;
        cc = c * cc;
      }
    }
  } else if (live) {
    for (int t = t1 - 1; t >= t0; --t) {
      const size_t i = (size_t)t * N + n;
      const bool dn = a.d[i] != 0;
      const double nd = dn ? 0.0 : 1.0;
      ft = dn ? t : ft;
      const double x = gae ? (double)a.r[i] + g * (double)a.v[i + N] * nd - (double)a.v[i] : (double)a.r[i];
      const double c = (gae ? gl : g) * nd;
      ca = x + c * ca;
      cc = c * cc;
    }
  }
  // suffix scan over the chunks of each env: F_ch = f_ch o F_{ch+1}
  double x = init;
  int ntc = T;
  {
    s_a[tid] = ca;
    s_c[tid] = cc;
    s_ft[tid] = ft;
    __syncthreads();
    for (int off = 1; off < a.CH; off <<= 1) {
      double na = ca, nc = cc;
      int nf = ft;
      if (ch + off < a.CH) {
        const int j = tid + off * a.E;
        na = ca + cc * s_a[j];
        nc = cc * s_c[j];
        nf = min(ft, s_ft[j]);
      }
      __syncthreads();
      s_a[tid] = ca = na;
      s_c[tid] = cc = nc;
      s_ft[tid] = ft = nf;
      __syncthreads();
    }
    if (ch + 1 < a.CH) {
      const int j = tid + a.E;
      x = s_a[j] + s_c[j] * init;
      ntc = s_ft[j];
    }
  }

  // pass 2: replay the chunk from its carry
  double m[RS_MOM];
#pragma unroll
  for (int k = 0; k < RS_MOM; ++k) m[k] = 0.0;
  if (live && regs) {
#pragma unroll
    for (int u = 0; u < RS_KREG; ++u) {
      const int t = t1 - 1 - u;
      if (t < t0) continue;
      const size_t i = (size_t)t * N + n;
      const double nd = cd[u] ? 0.0 : 1.0;
      const double vt = cv[u];
      if (gae) x = (double)cr[u] + g * (double)cvn[u] * nd - vt + gl * nd * x;
      else x = (double)cr[u] + g * nd * x;
      if (window) {
        a.gz[i] = x;
        continue;
      }
      const double rt = gae ? x + vt : x, ad = gae ? x : x - vt;
      const float rf = (float)rt, af = (float)ad;
      a.ret[i] = rf;
      a.adv[i] = af;
      m[0] += af; m[1] += (double)af * af; m[2] += rf; m[3] += (double)rf * rf;
      m[4] += vt; m[5] += vt * vt; m[6] += (double)rf * vt;
    }
  } else if (live) {
    for (int t = t1 - 1; t >= t0; --t) {
      const size_t i = (size_t)t * N + n;
      const double nd = a.d[i] ? 0.0 : 1.0;
      const double vt = a.v[i];
      if (gae) x = (double)a.r[i] + g * (double)a.v[i + N] * nd - vt + gl * nd * x;
      else x = (double)a.r[i] + g * nd * x;
      if (window) {
        a.gz[i] = x;
        continue;
      }
      const double rt = gae ? x + vt : x, ad = gae ? x : x - vt;
      const float rf = (float)rt, af = (float)ad;
      a.ret[i] = rf;
      a.adv[i] = af;
      m[0] += af; m[1] += (double)af * af; m[2] += rf; m[3] += (double)rf * rf;
      m[4] += vt; m[5] += vt * vt; m[6] += (double)rf * vt;
    }
  }
  if (window) {   // uniform across the grid: every thread reaches the barrier
    __syncthreads();   // the later chunks' Gz (same workgroup) are visible
    if (live) {
      int nt = ntc;
      const double gL = pow(g, (double)a.L);
      for (int t = t1 - 1; t >= t0; --t) {
        const size_t i = (size_t)t * N + n;
        nt = a.d[i] ? t : nt;
        const int h = min(t + a.L, T);
        double tg = a.gz[i];
        if (nt >= h) {
          const double gh = (h - t == a.L) ? gL : pow(g, (double)(h - t));
          tg += gh * ((double)a.v[(size_t)h * N + n] - (h < T ? a.gz[(size_t)h * N + n] : 0.0));
        }
        const double vt = a.v[i];
        const float rf = (float)tg, af = (float)(tg - vt);
        a.ret[i] = rf;
        a.adv[i] = af;
        m[0] += af; m[1] += (double)af * af; m[2] += rf; m[3] += (double)rf * rf;
        m[4] += vt; m[5] += vt * vt; m[6] += (double)rf * vt;
      }
    }
  }
  block_sum_multi<RS_MOM>(m, s_red);
  if (tid < RS_MOM) a.part[(size_t)blockIdx.x * 8 + tid] = m[tid];
  if (!last_block_arrival(a.ticket, gridDim.x, &s_flag)) return;
  {
    double s[RS_MOM];
    grid_records_sum<RS_MOM>(a.part, 8, gridDim.x, s, s_red);
    if (tid == 0)
#pragma unroll
      for (int k = 0; k < RS_MOM; ++k) s_tot[1 + k] = s[k];
  }
  __syncthreads();
  const double cnt = (double)T * N;
  const double mean = s_tot[1] / cnt;
  const double var = fmax(s_tot[2] / cnt - mean * mean, 0.0);
  if (tid == 0) {
    a.mom[0] = cnt;
    for (int k = 0; k < RS_MOM; ++k) a.mom[1 + k] = s_tot[1 + k];
    if (a.ev_out) {
      const double mx = s_tot[3] / cnt, my = s_tot[5] / cnt;
      const double vx = s_tot[4] / cnt - mx * mx, vy = s_tot[6] / cnt - my * my;
      *a.ev_out = (float)((s_tot[7] / cnt - mx * my) / sqrt(fmax(vx, 0.0) * fmax(vy, 0.0)));
    }
  }
  if (a.norm) {
    const float fm = (float)mean, inv = 1.0f / (a.eps + (float)sqrt(var));
    const int tot = T * N;
    if ((tot & 3) == 0 && (((uintptr_t)a.adv) & 15) == 0) {
      float4* p = reinterpret_cast<float4*>(a.adv);
      const int n4 = tot / 4;
      int i = tid;
      for (; i + 7 * RS_THREADS < n4; i += 8 * RS_THREADS) {   // 8 loads in flight per thread, then 8 stores
        float4 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = p[i + u * RS_THREADS];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          q[u].x = (q[u].x - fm) * inv; q[u].y = (q[u].y - fm) * inv;
          q[u].z = (q[u].z - fm) * inv; q[u].w = (q[u].w - fm) * inv;
          p[i + u * RS_THREADS] = q[u];
        }
      }
      for (; i < n4; i += RS_THREADS) {
        float4 q = p[i];
        q.x = (q.x - fm) * inv; q.y = (q.y - fm) * inv; q.z = (q.z - fm) * inv; q.w = (q.w - fm) * inv;
        p[i] = q;
      }
    } else {
      for (int i = tid; i < tot; i += RS_THREADS) a.adv[i] = (a.adv[i] - fm) * inv;
    }
  }
}

// Advantage normalisation from all-reduced totals (data-parallel runs: mom = sum over ranks of returns_scan's
// moments, mom[0] = global count): out = (a - mean) / (eps + std_pop). Elementwise, many workgroups.
__global__ void normalize_mom_kernel(const float* __restrict__ a, float* __restrict__ out,
                                     const double* __restrict__ mom, int n, float eps) {
  const double cnt = mom[0], mean = mom[1] / cnt;
  const double var = fmax(mom[2] / cnt - mean * mean, 0.0);
  const float fm = (float)mean, inv = 1.0f / (eps + (float)sqrt(var));
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = (a[i] - fm) * inv;
}

// EV correlation over many workgroups: fixed-order partial moments + last-arriver combine (the one-workgroup
// ev_kernel above caps at one CU; this is the PPO-sized form).
__global__ void __launch_bounds__(RS_THREADS) ev_multi_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                              float* __restrict__ out, int n, double* part,
                                                              unsigned int* ticket) {
  __shared__ double sh[16 * 5];
  __shared__ double s_tot[5];
  __shared__ int s_flag;
  double m[5] = {0, 0, 0, 0, 0};
  for (int i = blockIdx.x * RS_THREADS + threadIdx.x; i < n; i += gridDim.x * RS_THREADS) {
    const double xi = x[i], yi = y[i];
    m[0] += xi; m[1] += xi * xi; m[2] += yi; m[3] += yi * yi; m[4] += xi * yi;
  }
  block_sum_multi<5>(m, sh);
  if (threadIdx.x < 5) part[(size_t)blockIdx.x * 8 + threadIdx.x] = m[threadIdx.x];
  if (!last_block_arrival(ticket, gridDim.x, &s_flag)) return;
  {
    double s[5];
    grid_records_sum<5>(part, 8, gridDim.x, s, sh);
    if (threadIdx.x == 0)
#pragma unroll
      for (int k = 0; k < 5; ++k) s_tot[k] = s[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double mx = s_tot[0] / n, my = s_tot[2] / n;
    const double vx = s_tot[1] / n - mx * mx, vy = s_tot[3] / n - my * my;
    *out = (float)((s_tot[4] / n - mx * my) / sqrt(fmax(vx, 0.0) * fmax(vy, 0.0)));
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

// Launch geometry of returns_scan: chunk length ~RS_KREG steps (kept in registers), CH chunks (power of two,
// <= 256) per env, E = 256 / CH envs per workgroup.
extern "C" void aca_returns_scan_geometry(int T, int N, int* E, int* CH, int* K, int* blocks) {
  int ch = 1;
  while (ch < 256 && ch * aca::RS_KREG < T) ch <<= 1;
  *CH = ch;
  *E = aca::RS_THREADS / ch;
  *K = (T + ch - 1) / ch;
  *blocks = (N + *E - 1) / *E;
}

extern "C" hipError_t aca_returns_scan(const float* r, const float* v, const uint8_t* d, float* ret, float* adv,
                                       double* gz, double* part, unsigned int* ticket, double* mom, float* ev_out,
                                       int T, int N, int mode, int L, int norm, float gamma, float lam, float eps,
                                       hipStream_t stream) {
  if (T <= 0 || N <= 0) return hipSuccess;
  aca::RetScanArgs a{r, v, d, ret, adv, gz, part, ticket, mom, ev_out, T, N, 0, 0, 0, mode, L, norm, gamma, lam, eps};
  int blocks;
  aca_returns_scan_geometry(T, N, &a.E, &a.CH, &a.K, &blocks);
  aca::returns_scan_kernel<<<blocks, aca::RS_THREADS, 0, stream>>>(a);
  return hipGetLastError();
}

extern "C" hipError_t aca_normalize_mom(const float* a, float* out, const double* mom, int n, float eps,
                                        hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int blocks = std::min((n + 255) / 256, 1024);
  aca::normalize_mom_kernel<<<blocks, 256, 0, stream>>>(a, out, mom, n, eps);
  return hipGetLastError();
}

extern "C" int aca_ev_multi_blocks(int n) { return std::max(1, std::min(64, (n + 2047) / 2048)); }

extern "C" hipError_t aca_ev_multi(const float* x, const float* y, float* out, int n, double* part,
                                   unsigned int* ticket, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  aca::ev_multi_kernel<<<aca_ev_multi_blocks(n), aca::RS_THREADS, 0, stream>>>(x, y, out, n, part, ticket);
  return hipGetLastError();
}

extern "C" hipError_t aca_mb_gather(const uint8_t* obs, int64_t R, const int* act, const float* logp, const float* adv,
                                    const float* ret, const float* v, uint8_t* o_obs, int* o_act, float* o_logp,
                                    float* o_adv, float* o_ret, float* o_v, int mb, int n, uint32_t seed,
                                    int64_t* uc, int ep, int off, const double* mom, float eps,
                                    unsigned int* bump_ticket, int64_t* o_idx, hipStream_t stream) {
  if (mb <= 0) return hipSuccess;
  if (!o_idx && !o_obs) return hipErrorInvalidValue;
  if (o_idx)
    aca::mb_gather_kernel<<<(mb + 255) / 256, 256, 0, stream>>>(obs, R, act, logp, adv, ret, v, nullptr, o_act,
                                                                 o_logp, o_adv, o_ret, o_v, n, seed, uc, ep, off, mom,
                                                                 eps, bump_ticket, o_idx, mb);
  else
    aca::mb_gather_kernel<<<mb, 256, 0, stream>>>(obs, R, act, logp, adv, ret, v, o_obs, o_act, o_logp, o_adv, o_ret,
                                                  o_v, n, seed, uc, ep, off, mom, eps, bump_ticket, nullptr, mb);
  return hipGetLastError();
}
