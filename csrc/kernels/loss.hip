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
// One workgroup: the stats reduction is deterministic.
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

constexpr int LOSS_THREADS = 256;
constexpr int LOSS_STAGE = 2048;   // fused-returns rollouts up to this many rows are staged in LDS
constexpr int CAT_MAX = 20;        // categorical heads: logits + value columns held in registers (A + 1 <= 21)

// Latency structure (one workgroup, B ~ 160 rows for the bench): every global operand is loaded in ONE round
// (rollout rewards / dones / values into LDS, each thread's logits row + action + old log-prob into registers),
// the returns recursion and the row maths then run out of LDS/registers; global writes (dz, targets for logging)
// are fire-and-forget.
// AC > 0: categorical head with AC actions fixed at compile time (the per-column loops lose their guards, so the
// row's loads and exp/log chains are scheduled together); AC == 0: any head (runtime A, gaussian).
template <int AC>
__global__ void __launch_bounds__(LOSS_THREADS) ac_loss_kernel(LossArgs a) {
  constexpr int NJ = AC ? AC : CAT_MAX;
  __shared__ double sh[16 * 8];
  __shared__ float dls[64];
  __shared__ float dbs[64];
  __shared__ float s_rew[LOSS_STAGE], s_val[LOSS_STAGE + 256], s_ret[LOSS_STAGE], s_adv[LOSS_STAGE];
  __shared__ uint8_t s_dn[LOSS_STAGE];
  float dbp[CAT_MAX + 1];  // this thread's partial column sums of dz (head-bias gradient)
#pragma unroll
  for (int j = 0; j <= CAT_MAX; ++j) dbp[j] = 0.f;
  if (threadIdx.x < 64) { dls[threadIdx.x] = 0.f; dbs[threadIdx.x] = 0.f; }
  const bool staged = a.returns_mode && a.B <= LOSS_STAGE && a.N <= 256;
  if (staged) {
    for (int i = threadIdx.x; i < a.B; i += blockDim.x) {
      s_rew[i] = a.rew[i];
      s_dn[i] = a.dn[i];
    }
    for (int i = threadIdx.x; i < a.B + a.N; i += blockDim.x) s_val[i] = a.val[i];
  }
  __syncthreads();
  const float* rew = staged ? s_rew : a.rew;
  const uint8_t* dn = staged ? s_dn : a.dn;
  const float* val = staged ? s_val : a.val;
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
          acc += disc * rew[i];
          disc *= a.gamma;
          if (dn[i]) { alive = false; break; }
        }
        if (alive) acc += disc * val[h * a.N + n];
        R = acc;
      } else {
        float last = 0.f;
        for (int k = a.T - 1; k >= t; --k) {
          const int i = k * a.N + n;
          const float nd = dn[i] ? 0.f : 1.f;
          const float delta = rew[i] + a.gamma * val[i + a.N] * nd - val[i];
          last = delta + a.gamma * a.lam * nd * last;
        }
        R = last + val[idx];
      }
      const float v = val[idx];
      const float A_ = R - v;
      a.ret_w[idx] = R;
      a.adv_w[idx] = A_;
      if (staged) { s_ret[idx] = R; s_adv[idx] = A_; }
      s_r += R; s_rr += (double)R * R; s_v += v; s_vv += (double)v * v; s_rv += (double)R * v;
      s_a += A_; s_aa += (double)A_ * A_;
    }
    if (!staged) __threadfence_block();   // global ret_w / adv_w are re-read by other threads after the barrier
    double red[7] = {s_r, s_rr, s_v, s_vv, s_rv, s_a, s_aa};
    block_sum_multi<7>(red, sh);   // ends with a barrier: s_ret / s_adv (or the global scratch) are complete
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
  }
  const float* advp = a.returns_mode ? (staged ? s_adv : a.adv_w) : a.adv;
  const float* retp = a.returns_mode ? (staged ? s_ret : a.ret_w) : a.ret;
  const float invB = 1.0f / (float)a.B;
  const float c_ent = a.ent_coef ? *a.ent_coef : 0.f;
  const float beta = a.kl_coef ? *a.kl_coef : 0.f;
  const float HALF_LOG_2PI = 0.91893853320467274178f;
  double s_pg = 0, s_kl = 0, s_H = 0, s_vl = 0, s_cf = 0, s_ratio = 0;
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    const float* z = a.logits + (int64_t)b * a.ldl;
    // every per-row operand is requested before any is used
    float zr[CAT_MAX];
    if (!a.gaussian) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) zr[j] = (AC || j < a.A) ? z[j] : -INFINITY;
    }
    const int ab = a.gaussian ? 0 : a.act_i[b];
    const float lpo = a.logp_old[b];
    const float v = a.value ? a.value[(int64_t)b * a.ldv] : 0.f;
    const float vo = (a.value && a.v_clip > 0.f && a.v_old) ? a.v_old[b] : 0.f;
    const float adv = (advp[b] - adv_mean) * adv_inv;
    const float R = a.value ? retp[b] : 0.f;
    float lpa = 0.f, H = 0.f, lse = 0.f;
    if (!a.gaussian) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < NJ; ++j) mx = fmaxf(mx, zr[j]);
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) se += (AC || j < a.A) ? expf(zr[j] - mx) : 0.f;
      lse = mx + logf(se);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (AC || j < a.A) {
          const float lz = zr[j] - lse;
          H -= expf(lz) * lz;
          lpa = (j == ab) ? lz : lpa;
        }
      }
    } else {
      for (int j = 0; j < a.A; ++j) {
        const float ls = fminf(fmaxf(a.log_std[j], -2.5f), 2.5f);
        const float zz = (a.act_f[(int64_t)b * a.A + j] - z[j]) * expf(-ls);
        lpa += -0.5f * zz * zz - ls - HALF_LOG_2PI;
        H += 0.5f + HALF_LOG_2PI + ls;
      }
    }
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
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (AC || j < a.A) {
          const float oh = (j == ab) ? 1.0f : 0.0f;
          const float lz = zr[j] - lse, pj = expf(lz);
          const float g = g_lpa * (oh - pj) + c_ent * invB * pj * (lz + H);
          const u16 gb = f2bf(g);
          dz[j] = gb;
          dbp[j] += bf2f(gb);
        }
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
      float d = v - R;
      float vl = d * d;
      float gv = 2.0f * d;
      if (a.v_clip > 0.f && a.v_old) {
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
      // the value column is column A of the fused head (dbias_n == A + 1)
      if (AC) {
        dbp[AC] += bf2f(gvb);
      } else {
#pragma unroll
        for (int q = 0; q <= CAT_MAX; ++q)
          if (q == a.A) dbp[q] += bf2f(gvb);
      }
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
    for (int q = 0; q <= CAT_MAX; ++q) {
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
  if (A > 64 || dbias_n > aca::CAT_MAX + 1 || (!gaussian && A > aca::CAT_MAX)) return hipErrorInvalidValue;
  if (returns_mode && (T * N != B || !rew || !val || !dn || !ret_w || !adv_w)) return hipErrorInvalidValue;
  aca::LossArgs a;
  a.logits = logits; a.ldl = ldl; a.value = value; a.ldv = ldv; a.act_i = act_i; a.act_f = act_f;
  a.log_std = log_std; a.logp_old = logp_old; a.adv = adv; a.ret = ret; a.v_old = v_old; a.ent_coef = ent_coef;
  a.kl_coef = kl_coef; a.vf_coef = vf_coef; a.ppo_clip = ppo_clip; a.v_clip = v_clip; a.dlogits = dlogits;
  a.lddl = lddl; a.dvalue = dvalue; a.lddv = lddv; a.dlog_std = dlog_std; a.stats = stats; a.B = B; a.A = A;
  a.gaussian = gaussian;
  a.returns_mode = returns_mode; a.rew = rew; a.val = val; a.dn = dn; a.T = T; a.N = N; a.L = L; a.gamma = gamma;
  a.lam = lam; a.norm_adv = norm_adv; a.ret_w = ret_w; a.adv_w = adv_w; a.dbias = dbias; a.dbias_n = dbias_n;
  if (!gaussian && A >= 2 && A <= 19) {
    switch (A) {
#define ACA_LOSS_CASE(n) \
  case n: aca::ac_loss_kernel<n><<<1, aca::LOSS_THREADS, 0, stream>>>(a); break;
      ACA_LOSS_CASE(2) ACA_LOSS_CASE(3) ACA_LOSS_CASE(4) ACA_LOSS_CASE(5) ACA_LOSS_CASE(6) ACA_LOSS_CASE(7)
      ACA_LOSS_CASE(8) ACA_LOSS_CASE(9) ACA_LOSS_CASE(10) ACA_LOSS_CASE(11) ACA_LOSS_CASE(12) ACA_LOSS_CASE(13)
      ACA_LOSS_CASE(14) ACA_LOSS_CASE(15) ACA_LOSS_CASE(16) ACA_LOSS_CASE(17) ACA_LOSS_CASE(18) ACA_LOSS_CASE(19)
#undef ACA_LOSS_CASE
    }
  } else {
    aca::ac_loss_kernel<0><<<1, aca::LOSS_THREADS, 0, stream>>>(a);
  }
  return hipGetLastError();
}
