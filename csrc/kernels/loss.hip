// Fused actor-critic loss + head gradient, one launch per learner (mini)batch.
//
// Per row (categorical head; logits z [B, A], value v [B]):
//   logp = log_softmax(z),  H = -sum p logp,  lpa = logp[a]
//   A2C (reference, Basic_AC/policies.py:72-78):  L_pi = -mean(adv*lpa) + beta*mean((lpo-lpa)^2) - c_ent*mean(H)
//   PPO-clip:  L_pi = -mean(min(r adv, clip(r, 1-e, 1+e) adv)) + beta*mean((lpo-lpa)^2) - c_ent*mean(H), r=e^(lpa-lpo)
//   L_v = vf_coef * mean((v - R)^2)   (optionally PPO-clipped: max((v-R)^2, (v_old + clip(v - v_old) - R)^2))
// and writes dL/dz, dL/dv as bf16 (the inputs of the backward GEMMs). Gaussian head (mu [B, A], log_std [A]):
//   logp = sum -0.5 ((a-mu)/sigma)^2 - log sigma - log sqrt(2 pi), sigma = exp(clip(log_std, -2.5, 2.5)), H const in mu;
//   d/dmu and d/dlog_std (zero outside the clip, Basic_AC/policies.py:50-51) -- log_std's gradient is summed over rows
//   and added atomically into its slot of the fp32 gradient slab.
// Coefficients (c_ent, beta) are read from device scalars (annealed by the schedules without a host sync).
// stats[0..6] = pg, kl, entropy, value_loss (unscaled mean), clipfrac, total actor loss, mean ratio.
// One 1024-thread workgroup: the stats reduction is deterministic.
//
// A2C fast path (returns_mode 1 = n-step / 2 = GAE): the kernel first computes the targets and advantages of the
// whole [T, N] rollout itself (same maths as returns.hip), the EV-before statistic (stats[7], Basic_AC/util.py:4-12)
// and, with norm_adv, the population-std advantage normalisation (Basic_AC/run_AC.py:241) -- the returns, EV and
// normalisation kernels of the generic path fold into this one launch. dbias (optional) receives the column sums of
// dz = the gradient of the head bias, written directly (the gradient slab is clean).
#include "common.h"

namespace aca {

struct LossArgs {
  const float* logits; int64_t ldl;     // or mu for the gaussian head
  const float* value; int64_t ldv;      // may be null (no critic term)
  const int32_t* act_i;                 // categorical actions
  const float* act_f;                   // gaussian actions [B, A]
  const float* log_std;                 // gaussian
  const float* logp_old;
  const float* adv;
  const float* ret;
  const float* v_old;                   // may be null
  const float* ent_coef;                // device scalar
  const float* kl_coef;                 // device scalar
  float vf_coef, ppo_clip, v_clip;
  u16* dlogits; int64_t lddl;
  u16* dvalue; int64_t lddv;
  float* dlog_std;                      // gaussian: fp32 [A] (atomic add)
  float* stats;
  int B, A;
  int gaussian;
  // fused returns (A2C): rew/done [T, N], val [T+1, N]; ret/adv (global scratch [B]) are written then read back
  int returns_mode;                     // 0: use ret/adv as given; 1: n-step (look-ahead L); 2: GAE(lambda)
  const float* rew; const float* val; const uint8_t* dn;
  int T, N, L;
  float gamma, lam;
  int norm_adv;
  float* ret_w; float* adv_w;
  float* dbias; int dbias_n;            // head bias gradient (A+1 columns: logits | value)
};

__global__ void __launch_bounds__(1024) ac_loss_kernel(LossArgs a) {
  __shared__ double sh[16 * 8];
  __shared__ float dls[64];
  __shared__ float dbs[64];
  float dbp[21];  // this thread's partial column sums of dz (head-bias gradient), A + 1 <= 21
#pragma unroll
  for (int j = 0; j < 21; ++j) dbp[j] = 0.f;
  if (threadIdx.x < 64) { dls[threadIdx.x] = 0.f; dbs[threadIdx.x] = 0.f; }
  __syncthreads();
  float adv_mean = 0.f, adv_inv = 1.f;
  if (a.returns_mode) {
    // ---- phase 0: targets / advantages of every (t, n), EV-before, normalisation constants
    double s_r = 0, s_rr = 0, s_v = 0, s_vv = 0, s_rv = 0, s_a = 0, s_aa = 0;
    for (int idx = threadIdx.x; idx < a.B; idx += blockDim.x) {
      const int t = idx / a.N, n = idx - t * a.N;
      float R;
      if (a.returns_mode == 1) {
        const int h = min(t + a.L, a.T);
        float acc = 0.f, disc = 1.f;
        bool alive = true;
        for (int k = t; k < h; ++k) {
          const int i = k * a.N + n;
          acc += disc * a.rew[i];
          disc *= a.gamma;
          if (a.dn[i]) { alive = false; break; }
        }
        if (alive) acc += disc * a.val[h * a.N + n];
        R = acc;
      } else {
        float last = 0.f, Rt = 0.f;
        for (int k = a.T - 1; k >= t; --k) {
          const int i = k * a.N + n;
          const float nd = a.dn[i] ? 0.f : 1.f;
          const float delta = a.rew[i] + a.gamma * a.val[i + a.N] * nd - a.val[i];
          last = delta + a.gamma * a.lam * nd * last;
        }
        Rt = last + a.val[idx];
        R = Rt;
      }
      const float v = a.val[idx];
      const float A_ = R - v;
      a.ret_w[idx] = R;
      a.adv_w[idx] = A_;
      s_r += R; s_rr += (double)R * R; s_v += v; s_vv += (double)v * v; s_rv += (double)R * v;
      s_a += A_; s_aa += (double)A_ * A_;
    }
    double red[7] = {s_r, s_rr, s_v, s_vv, s_rv, s_a, s_aa};
    block_sum_multi<7>(red, sh);
    s_r = red[0]; s_rr = red[1]; s_v = red[2]; s_vv = red[3]; s_rv = red[4]; s_a = red[5]; s_aa = red[6];
    const double n = a.B;
    if (threadIdx.x == 0) {
      const double mr = s_r / n, mv = s_v / n;
      const double vr = fmax(s_rr / n - mr * mr, 0.0), vv = fmax(s_vv / n - mv * mv, 0.0);
      a.stats[7] = (float)((s_rv / n - mr * mv) / sqrt(vr * vv));
    }
    if (a.norm_adv) {
      const double m = s_a / n;
      const double var = fmax(s_aa / n - m * m, 0.0);
      adv_mean = (float)m;
      adv_inv = 1.0f / (1e-8f + (float)sqrt(var));
    }
    __syncthreads();  // ret_w / adv_w written above are read by other threads below
  }
  const float* advp = a.returns_mode ? a.adv_w : a.adv;
  const float* retp = a.returns_mode ? a.ret_w : a.ret;
  const float invB = 1.0f / (float)a.B;
  const float c_ent = a.ent_coef ? *a.ent_coef : 0.f;
  const float beta = a.kl_coef ? *a.kl_coef : 0.f;
  const float HALF_LOG_2PI = 0.91893853320467274178f;
  double s_pg = 0, s_kl = 0, s_H = 0, s_vl = 0, s_cf = 0, s_ratio = 0;
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    const float* z = a.logits + (int64_t)b * a.ldl;
    float lpa = 0.f, H = 0.f, lse = 0.f;
    if (!a.gaussian) {
      float mx = -INFINITY;
      for (int j = 0; j < a.A; ++j) mx = fmaxf(mx, z[j]);
      float se = 0.f;
      for (int j = 0; j < a.A; ++j) se += expf(z[j] - mx);
      lse = mx + logf(se);
      for (int j = 0; j < a.A; ++j) {
        const float lz = z[j] - lse;
        H -= expf(lz) * lz;
      }
      lpa = z[a.act_i[b]] - lse;
    } else {
      for (int j = 0; j < a.A; ++j) {
        const float ls = fminf(fmaxf(a.log_std[j], -2.5f), 2.5f);
        const float zz = (a.act_f[(int64_t)b * a.A + j] - z[j]) * expf(-ls);
        lpa += -0.5f * zz * zz - ls - HALF_LOG_2PI;
        H += 0.5f + HALF_LOG_2PI + ls;
      }
    }
    const float lpo = a.logp_old[b], adv = (advp[b] - adv_mean) * adv_inv;
    float g_lpa;  // dL/dlpa (already divided by B)
    if (a.ppo_clip > 0.f) {
      const float ratio = expf(lpa - lpo);
      const float s1 = ratio * adv;
      const float rc = fminf(fmaxf(ratio, 1.0f - a.ppo_clip), 1.0f + a.ppo_clip);
      const float s2 = rc * adv;
      s_pg += -(double)fminf(s1, s2);
      const bool inside = ratio >= 1.0f - a.ppo_clip && ratio <= 1.0f + a.ppo_clip;
      g_lpa = (s1 <= s2 || inside) ? -adv * ratio * invB : 0.f;
      s_cf += fabsf(ratio - 1.0f) > a.ppo_clip ? 1.0 : 0.0;
      s_ratio += ratio;
    } else {
      s_pg += -(double)(adv * lpa);
      g_lpa = -adv * invB;
      s_ratio += 1.0;
    }
    const float dkl = lpo - lpa;
    s_kl += (double)(dkl * dkl);
    g_lpa += -2.0f * beta * dkl * invB;
    s_H += H;
    // head gradient
    u16* dz = a.dlogits + (int64_t)b * a.lddl;
    if (!a.gaussian) {
      const int ab = a.act_i[b];
      for (int j = 0; j < a.A; ++j) {
        const float oh = (j == ab) ? 1.0f : 0.0f;
        const float lz = z[j] - lse, pj = expf(lz);
        const float g = g_lpa * (oh - pj) + c_ent * invB * pj * (lz + H);
        const u16 gb = f2bf(g);
        dz[j] = gb;
#pragma unroll
        for (int q = 0; q < 21; ++q)
          if (q == j) dbp[q] += bf2f(gb);
      }
    } else {
      for (int j = 0; j < a.A; ++j) {
        const float ls_raw = a.log_std[j];
        const float ls = fminf(fmaxf(ls_raw, -2.5f), 2.5f);
        const float zz = (a.act_f[(int64_t)b * a.A + j] - z[j]) * expf(-ls);
        // dlogp/dmu = zz / sigma ; dlogp/dls = zz^2 - 1 ; dH/dls = 1
        dz[j] = f2bf(g_lpa * zz * expf(-ls));
        const bool in_clip = ls_raw >= -2.5f && ls_raw <= 2.5f;
        if (in_clip) atomicAdd(&dls[j], g_lpa * (zz * zz - 1.0f) - c_ent * invB);
      }
    }
    // critic
    if (a.value) {
      const float v = a.value[(int64_t)b * a.ldv], R = retp[b];
      float d = v - R;
      float vl = d * d;
      float gv = 2.0f * d;
      if (a.v_clip > 0.f && a.v_old) {
        const float vo = a.v_old[b];
        const float vc = vo + fminf(fmaxf(v - vo, -a.v_clip), a.v_clip);
        const float dc = vc - R;
        if (dc * dc > vl) {
          vl = dc * dc;
          const bool inside = (v - vo) >= -a.v_clip && (v - vo) <= a.v_clip;
          gv = inside ? 2.0f * dc : 0.f;
        }
      }
      s_vl += vl;
      const u16 gvb = f2bf(a.vf_coef * gv * invB);
      a.dvalue[(int64_t)b * a.lddv] = gvb;
#pragma unroll
      for (int q = 0; q < 21; ++q)
        if (q == a.A) dbp[q] += bf2f(gvb);
    }
  }
  {
    double red[6] = {s_pg, s_kl, s_H, s_vl, s_cf, s_ratio};
    block_sum_multi<6>(red, sh);
    s_pg = red[0]; s_kl = red[1]; s_H = red[2]; s_vl = red[3]; s_cf = red[4]; s_ratio = red[5];
  }
  if (a.dbias) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < 21; ++q) {
      if (q < a.dbias_n) {
        const float v = wave_sum(dbp[q]);
        if (lane == 0) atomicAdd(&dbs[q], v);
      }
    }
  }
  __syncthreads();
  if (a.gaussian && a.dlog_std && threadIdx.x < a.A) atomicAdd(&a.dlog_std[threadIdx.x], dls[threadIdx.x]);
  if (a.dbias && threadIdx.x < a.dbias_n) a.dbias[threadIdx.x] += dbs[threadIdx.x];
  if (threadIdx.x == 0) {
    const double inv = 1.0 / a.B;
    a.stats[0] = (float)(s_pg * inv);
    a.stats[1] = (float)(s_kl * inv);
    a.stats[2] = (float)(s_H * inv);
    a.stats[3] = (float)(s_vl * inv);
    a.stats[4] = (float)(s_cf * inv);
    a.stats[5] = (float)(s_pg * inv + beta * s_kl * inv - c_ent * s_H * inv);
    a.stats[6] = (float)(s_ratio * inv);
  }
}

}  // namespace aca

extern "C" hipError_t aca_ac_loss(const float* logits, int64_t ldl, const float* value, int64_t ldv,
                                  const int32_t* act_i, const float* act_f, const float* log_std,
                                  const float* logp_old, const float* adv, const float* ret, const float* v_old,
                                  const float* ent_coef, const float* kl_coef, float vf_coef, float ppo_clip,
                                  float v_clip, uint16_t* dlogits, int64_t lddl, uint16_t* dvalue, int64_t lddv,
                                  float* dlog_std, float* stats, int B, int A, int gaussian, int returns_mode,
                                  const float* rew, const float* val, const uint8_t* dn, int T, int N, int L,
                                  float gamma, float lam, int norm_adv, float* ret_w, float* adv_w, float* dbias,
                                  int dbias_n, hipStream_t stream) {
  if (A > 64 || dbias_n > 21) return hipErrorInvalidValue;
  if (returns_mode && (T * N != B || !rew || !val || !dn || !ret_w || !adv_w)) return hipErrorInvalidValue;
  aca::LossArgs a;
  a.logits = logits; a.ldl = ldl; a.value = value; a.ldv = ldv; a.act_i = act_i; a.act_f = act_f;
  a.log_std = log_std; a.logp_old = logp_old; a.adv = adv; a.ret = ret; a.v_old = v_old; a.ent_coef = ent_coef;
  a.kl_coef = kl_coef; a.vf_coef = vf_coef; a.ppo_clip = ppo_clip; a.v_clip = v_clip; a.dlogits = dlogits;
  a.lddl = lddl; a.dvalue = dvalue; a.lddv = lddv; a.dlog_std = dlog_std; a.stats = stats; a.B = B; a.A = A;
  a.gaussian = gaussian;
  a.returns_mode = returns_mode; a.rew = rew; a.val = val; a.dn = dn; a.T = T; a.N = N; a.L = L; a.gamma = gamma;
  a.lam = lam; a.norm_adv = norm_adv; a.ret_w = ret_w; a.adv_w = adv_w; a.dbias = dbias; a.dbias_n = dbias_n;
  aca::ac_loss_kernel<<<1, 1024, 0, stream>>>(a);
  return hipGetLastError();
}
