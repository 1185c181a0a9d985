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
#include "cnn_head.h"

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

// threads of ac_loss_kernel: the categorical specialisations run 16 waves (a B = 4096 PPO minibatch is 4 row
// iterations per thread, not 16 -- each iteration is a dependent memory round trip); the generic form (runtime A,
// Gaussian head) keeps 4 waves and the widest categorical heads 8, where their per-thread column arrays fit the
// register file without spilling
template <int AC>
constexpr int loss_threads() { return AC == 0 ? 256 : (AC <= 16 ? 1024 : 512); }
constexpr int LOSS_STAGE = 2048;   // fused-returns rollouts up to this many rows are staged in LDS
constexpr int CAT_MAX = 20;        // categorical heads: logits + value columns held in registers (A + 1 <= 21)

// Latency structure (one workgroup, B ~ 160 rows for the bench): every global operand is loaded in ONE round
// (rollout rewards / dones / values into LDS, each thread's logits row + action + old log-prob into registers),
// the returns recursion and the row maths then run out of LDS/registers; global writes (dz, targets for logging)
// are fire-and-forget.
// AC > 0: categorical head with AC actions fixed at compile time (the per-column loops lose their guards, so the
// row's loads and exp/log chains are scheduled together); AC == 0: any head (runtime A, gaussian).
template <int AC>
__global__ void __launch_bounds__(loss_threads<AC>()) ac_loss_kernel(LossArgs a) {
  constexpr int LOSS_THREADS = loss_threads<AC>();
  constexpr int NJ = AC ? AC : CAT_MAX;
  __shared__ double sh[16 * 8];
  __shared__ float dls[LOSS_THREADS / 64][CAT_MAX + 1];   // per-wave partials, summed in wave order
  __shared__ float dbs[LOSS_THREADS / 64][CAT_MAX + 1];
  float dlp[CAT_MAX];   // gaussian: this thread's partial d/dlog_std
  __shared__ float s_rew[LOSS_STAGE], s_val[LOSS_STAGE + 256], s_ret[LOSS_STAGE], s_adv[LOSS_STAGE];
  __shared__ uint8_t s_dn[LOSS_STAGE];
  float dbp[CAT_MAX + 1];  // this thread's partial column sums of dz (head-bias gradient)
#pragma unroll
  for (int j = 0; j <= CAT_MAX; ++j) dbp[j] = 0.f;
#pragma unroll
  for (int j = 0; j < CAT_MAX; ++j) dlp[j] = 0.f;
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
#pragma unroll
        for (int q = 0; q < CAT_MAX; ++q)   // register partial (named slot, no dynamic indexing)
          if (q == j && in_clip) dlp[q] += g_lpa * (zz * zz - 1.0f) - c_ent * invB;
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
  // head-bias and log-std gradients: wave shuffle sums, then the waves' partials added in wave order by one thread
  // per column (fixed order: bitwise reproducible)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (a.dbias) {
#pragma unroll
    for (int q = 0; q <= CAT_MAX; ++q) {
      if (q < a.dbias_n) {
        const float v = wave_sum(dbp[q]);
        if (lane == 0) dbs[wid][q] = v;
      }
    }
  }
  if (a.gaussian && a.dlog_std) {
#pragma unroll
    for (int q = 0; q < CAT_MAX; ++q) {
      if (q < a.A) {
        const float v = wave_sum(dlp[q]);
        if (lane == 0) dls[wid][q] = v;
      }
    }
  }
  __syncthreads();
  if (a.gaussian && a.dlog_std && threadIdx.x < a.A) {
    float t = 0.f;
    for (int w = 0; w < LOSS_THREADS / 64; ++w) t += dls[w][threadIdx.x];
    a.dlog_std[threadIdx.x] += t;
  }
  if (a.dbias && threadIdx.x < a.dbias_n) {
    float t = 0.f;
    for (int w = 0; w < LOSS_THREADS / 64; ++w) t += dbs[w][threadIdx.x];
    a.dbias[threadIdx.x] += t;
  }
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

// ------------------------------------------------------------------------------------------------------------
// A2C learner head, one launch (the rollout's activations are the forward): n-step / GAE returns, EV-before and
// advantage normalisation, the actor-critic loss and dz = dL/d(logits | value) exactly as ac_loss_kernel's fused
// path, then the head's backward without GEMM launches:
//   dh[b, j]  = (h[b, j] > 0) * sum_a dz[b, a] Wh[j, a]      (bf16, the fc layer's data gradient)
//   dbfc[j]   = sum_b dh[b, j]          dWh[j, a] = sum_b h[b, j] dz[b, a]          dbh[a] = sum_b dz[b, a]
// written straight into their gradient-slab slots. HB_WG workgroups, each owning 64 of the 512 hidden columns;
// every workgroup recomputes the (tiny, B-row) loss so that no cross-workgroup hand-off is needed, and workgroup 0
// alone writes the statistics / returns / dbh. Every sum runs in a fixed order (deterministic, and the loss of
// every workgroup is bit-identical). Head phase: wave w, lane l -> 8-column chunk l % 8 of the workgroup's 64, rows
// w * 8 + l / 8 + 64 i (16-byte h loads and dh stores, all of a thread's rows in flight at once); per-wave column
// sums by xor shuffles, then the 8 waves in wave order through LDS. Replaces ac_loss + the dh / dWh GEMMs.
// ------------------------------------------------------------------------------------------------------------
constexpr int HB_THREADS = 512;             // 2 waves per SIMD: 256 registers for the head phase's columns
constexpr int HB_MAXB = 512;
constexpr int HB_H = 512;
constexpr int HB_WG = 8;                    // workgroups (64 hidden columns each)
constexpr int HB_RPT = HB_MAXB / 64;        // row slots per thread in the head phase (8)

struct HeadBwdArgs {
  const float* z;            // [B, A1] logits | value
  const int32_t* act;
  const float* logp_old;
  const float* ent_coef; const float* kl_coef;
  float vf_coef;
  const float* rew; const float* val; const uint8_t* dn;
  int T, N, L, returns_mode, norm_adv;
  float gamma, lam;
  float* ret_w; float* adv_w;
  const u16* h;              // [B, 512] bf16 (rollout activations)
  const u16* Wh;             // [512, A1] bf16 shadow
  u16* dh;                   // [B, 512] out
  float* gWh; float* gbh; float* gbfc;
  float* stats;
  int B;
  uint64_t* stamps;          // optional [HB_WG, 16] s_memrealtime phase stamps (diagnostics; null in production)
};

__device__ __forceinline__ void hb_stamp(const HeadBwdArgs& a, int slot) {
  if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)blockIdx.x * 16 + slot] = __builtin_amdgcn_s_memrealtime();
}

template <int AC>
__global__ void __launch_bounds__(HB_THREADS) head_bwd_kernel(HeadBwdArgs a) {
  constexpr int A1 = AC + 1;
  __shared__ double sh[16 * 8];
  __shared__ float s_dz[HB_MAXB * A1];
  __shared__ float s_rew[HB_MAXB], s_val[HB_MAXB + 256], s_ret[HB_MAXB], s_adv[HB_MAXB];
  __shared__ uint8_t s_dn[HB_MAXB];
  __shared__ float s_red[8 * 64 * (A1 + 1)];    // per wave: 64 columns x (dWh | dbfc)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int B = a.B;
  const bool lead = blockIdx.x == 0;
  const int col0 = blockIdx.x * 64;
  hb_stamp(a, 0);
  // ---- every global operand in one round: rollout slabs into LDS, this thread's loss row and its head-phase
  // operands (h rows, Wh columns) in registers
  for (int i = tid; i < B; i += HB_THREADS) {
    s_rew[i] = a.rew[i];
    s_dn[i] = a.dn[i];
  }
  for (int i = tid; i < B + a.N; i += HB_THREADS) s_val[i] = a.val[i];
  const bool row = tid < B;
  const int rb = row ? tid : 0;
  float zr[A1];
#pragma unroll
  for (int j = 0; j < A1; ++j) zr[j] = a.z[(int64_t)rb * A1 + j];
  const int ab = a.act[rb];
  const float lpo = a.logp_old[rb];
  const int ck = lane & 7, rsub = wv * 8 + (lane >> 3);   // head phase: column chunk, first row
  const int jc0 = col0 + ck * 8;                          // first of this thread's 8 columns
  float wj[8][A1];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int q = 0; q < A1; ++q) wj[c][q] = bf2f(a.Wh[(jc0 + c) * A1 + q]);
  uint4 hv[HB_RPT];
#pragma unroll
  for (int r = 0; r < HB_RPT; ++r) {
    const int b = min(rsub + 64 * r, B - 1);
    hv[r] = *reinterpret_cast<const uint4*>(a.h + (int64_t)b * HB_H + jc0);
  }
  const float c_ent = *a.ent_coef, beta = *a.kl_coef;
  __syncthreads();
  hb_stamp(a, 1);
  // ---- returns, EV-before, advantage statistics (same maths as ac_loss_kernel phase 0)
  double s_r = 0, s_rr = 0, s_v = 0, s_vv = 0, s_rv = 0, s_a = 0, s_aa = 0;
  if (row) {
    const int idx = tid, t = idx / a.N, n = idx - t * a.N;
    float R;
    if (a.returns_mode == 1) {
      const int hh = min(t + a.L, a.T);
      float acc = 0.f, disc = 1.f;
      bool alive = true;
      for (int k = t; k < hh; ++k) {
        const int i = k * a.N + n;
        acc += disc * s_rew[i];
        disc *= a.gamma;
        if (s_dn[i]) { alive = false; break; }
      }
      if (alive) acc += disc * s_val[hh * a.N + n];
      R = acc;
    } else {
      float last = 0.f;
      for (int k = a.T - 1; k >= t; --k) {
        const int i = k * a.N + n;
        const float nd = s_dn[i] ? 0.f : 1.f;
        const float delta = s_rew[i] + a.gamma * s_val[i + a.N] * nd - s_val[i];
        last = delta + a.gamma * a.lam * nd * last;
      }
      R = last + s_val[idx];
    }
    const float v = s_val[idx], A_ = R - v;
    if (lead) {
      a.ret_w[idx] = R;
      a.adv_w[idx] = A_;
    }
    s_ret[idx] = R;
    s_adv[idx] = A_;
    s_r = R; s_rr = (double)R * R; s_v = v; s_vv = (double)v * v; s_rv = (double)R * v; s_a = A_;
    s_aa = (double)A_ * A_;
  }
  double red[7] = {s_r, s_rr, s_v, s_vv, s_rv, s_a, s_aa};
  block_sum_multi<7>(red, sh);
  hb_stamp(a, 2);
  const double nB = B;
  if (lead && tid == 0) {
    const double mr = red[0] / nB, mv = red[2] / nB;
    const double vr = fmax(red[1] / nB - mr * mr, 0.0), vv = fmax(red[3] / nB - mv * mv, 0.0);
    a.stats[7] = (float)((red[4] / nB - mr * mv) / sqrt(vr * vv));
  }
  float adv_mean = 0.f, adv_inv = 1.f;
  if (a.norm_adv) {
    const double m = red[5] / nB, var = fmax(red[6] / nB - m * m, 0.0);
    adv_mean = (float)m;
    adv_inv = 1.0f / (1e-8f + (float)sqrt(var));
  }
  // ---- loss + dz (A2C: PG + KL proxy + entropy; value MSE)
  const float invB = 1.0f / (float)B;
  double s_pg = 0, s_kl = 0, s_H = 0, s_vl = 0;
  if (row) {
    const float adv = (s_adv[tid] - adv_mean) * adv_inv;
    const float R = s_ret[tid];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < AC; ++j) mx = fmaxf(mx, zr[j]);
    float se = 0.f;
#pragma unroll
    for (int j = 0; j < AC; ++j) se += expf(zr[j] - mx);
    const float lse = mx + logf(se);
    float H = 0.f, lpa = 0.f;
#pragma unroll
    for (int j = 0; j < AC; ++j) {
      const float lz = zr[j] - lse;
      H -= expf(lz) * lz;
      lpa = (j == ab) ? lz : lpa;
    }
    s_pg = -(double)(adv * lpa);
    const float dkl = lpo - lpa;
    s_kl = (double)(dkl * dkl);
    s_H = H;
    const float g_lpa = -adv * invB - 2.0f * beta * dkl * invB;
#pragma unroll
    for (int j = 0; j < AC; ++j) {
      const float lz = zr[j] - lse, pj = expf(lz);
      const float g = g_lpa * (((j == ab) ? 1.0f : 0.0f) - pj) + c_ent * invB * pj * (lz + H);
      s_dz[tid * A1 + j] = bf2f(f2bf(g));   // the bf16 rounding the GEMM path's dz buffer applied
    }
    const float d = zr[AC] - R;
    s_vl = (double)(d * d);
    s_dz[tid * A1 + AC] = bf2f(f2bf(a.vf_coef * 2.0f * d * invB));
  }
  {
    double r4[4] = {s_pg, s_kl, s_H, s_vl};
    block_sum_multi<4>(r4, sh);   // ends with a barrier: s_dz complete
    hb_stamp(a, 3);
    if (lead && tid == 0) {
      const double inv = 1.0 / B;
      a.stats[0] = (float)(r4[0] * inv);
      a.stats[1] = (float)(r4[1] * inv);
      a.stats[2] = (float)(r4[2] * inv);
      a.stats[3] = (float)(r4[3] * inv);
      a.stats[4] = 0.f;
      a.stats[5] = (float)(r4[0] * inv + beta * r4[1] * inv - c_ent * r4[2] * inv);
      a.stats[6] = 1.f;
    }
  }
  // ---- head backward over this thread's rows x 8 columns
  float dwp[8][A1], dbf[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    dbf[c] = 0.f;
#pragma unroll
    for (int q = 0; q < A1; ++q) dwp[c][q] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < HB_RPT; ++r) {
    const int b = rsub + 64 * r;
    if (b < B) {
      float dzb[A1];
#pragma unroll
      for (int q = 0; q < A1; ++q) dzb[q] = s_dz[b * A1 + q];
      const uint32_t hw[4] = {hv[r].x, hv[r].y, hv[r].z, hv[r].w};
      uint32_t out[4];
#pragma unroll
      for (int c2 = 0; c2 < 4; ++c2) {
        uint32_t packed = 0;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int c = 2 * c2 + e;
          const float hf = __uint_as_float(e ? (hw[c2] & 0xFFFF0000u) : (hw[c2] << 16));
          float sacc = 0.f;
#pragma unroll
          for (int q = 0; q < A1; ++q) {
            sacc += dzb[q] * wj[c][q];
            dwp[c][q] += hf * dzb[q];
          }
          const float d = hf > 0.f ? sacc : 0.f;
          dbf[c] += d;
          packed |= (uint32_t)f2bf(d) << (16 * e);
        }
        out[c2] = packed;
      }
      *reinterpret_cast<uint4*>(a.dh + (int64_t)b * HB_H + jc0) = make_uint4(out[0], out[1], out[2], out[3]);
    }
  }
  // per-wave column sums: lanes l, l ^ 8, l ^ 16, l ^ 32 share a column chunk (xor tree, fixed order)
#pragma unroll
  for (int c = 0; c < 8; ++c) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      dbf[c] += lane_xor(dbf[c], o);
#pragma unroll
      for (int q = 0; q < A1; ++q) dwp[c][q] += lane_xor(dwp[c][q], o);
    }
  }
  hb_stamp(a, 4);
  if (lane < 8) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float* dstw = s_red + (wv * 64 + lane * 8 + c) * (A1 + 1);
#pragma unroll
      for (int q = 0; q < A1; ++q) dstw[q] = dwp[c][q];
      dstw[A1] = dbf[c];
    }
  }
  __syncthreads();
  if (tid < 64 * (A1 + 1)) {   // (column, value) pairs: the 8 waves in wave order
    const int cl = tid / (A1 + 1), q = tid - cl * (A1 + 1);
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += s_red[(w * 64 + cl) * (A1 + 1) + q];
    if (q < A1) a.gWh[(col0 + cl) * A1 + q] = v;
    else a.gbfc[col0 + cl] = v;
  }
  if (lead && wv < A1) {   // head-bias gradient: column wv of dz, rows strided over a wave, xor tree (fixed order)
    float sb = 0.f;
    for (int bb = lane; bb < B; bb += 64) sb += s_dz[bb * A1 + wv];
    sb = wave_sum(sb);
    if (lane == 0) a.gbh[wv] = sb;
  }
  if (a.stamps) {
    hb_stamp(a, 5);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    hb_stamp(a, 6);
  }
}

// ------------------------------------------------------------------------------------------------------------
// A2C learner head v2: the bootstrap value V(s_T) + everything head_bwd_kernel does, in ONE launch of AH_WG narrow
// workgroups (replaces fc_value_kernel + head_bwd_kernel: 2 launches, 8 wide workgroups on the critical path).
//   phase 0: workgroup w computes V(s_T) of envs e = w + AH_WG k straight from the rollout's last fc partial planes
//            (fc_h2_from_parts: the rollout step's plane order and bf16 rounding of h; the value's dot product is
//            reduced per wave then across waves), stores them with agent-coherent (sc1) stores, and arrives at a
//            grid barrier. Every
//            operand that does not depend on V(s_T) (rewards, dones, values, logits, h columns, Wh) is requested
//            before the wait.
//   phase 1: returns / advantages of all B rows (each workgroup: identical code and order -> identical bits), the
//            advantage moments (2 fp64 sums), loss + dz. Side duties, one per workgroup so that no workgroup carries
//            them all: 0 writes ret / adv, 1 the EV-before sums (stats[7]), 2 the loss statistics, 3 dbh.
//   phase 2: the head backward for the workgroup's 16 hidden columns: thread t -> 4 columns (t & 3), rows
//            (t >> 2) + 64 i; dh stored as bf16, dWh / dbfc partials reduced over lanes (xor tree) then waves (LDS),
//            fixed order (deterministic, no atomics).
// The grid barrier needs the AH_WG workgroups co-resident (32 of 256 CUs; nothing else runs in the captured
// update); its spin is bounded and a timeout raises bar[2] instead of hanging. Cross-workgroup data (V(s_T)) moves
// only through sc1 (agent-coherent) stores / loads ordered by s_waitcnt, so no L2 write-back / invalidate is needed.
// ------------------------------------------------------------------------------------------------------------
constexpr int AH_THREADS = 256;
constexpr int AH_WG = 32;
constexpr int AH_COLS = HB_H / AH_WG;        // 16 hidden columns per workgroup
constexpr int AH_MAXB = 512;
constexpr int AH_MAXN = 256;
constexpr int AH_RPT = AH_MAXB / 64;         // row slots per thread in the head phase
constexpr unsigned int AH_SPIN_LIMIT = 1u << 21;

struct A2cHeadArgs {
  HeadBwdArgs h;
  const float* hpart; int S; int64_t plane_stride;   // last fc product (split-K planes) of s_T, or null: val holds V(s_T)
  const float* bfc; const float* bh;
  float* vboot;              // [N] = val + B (written in phase 0)
  unsigned int* bar;         // [0] arrivals, [1] departures, [2] timeout flag
};

template <int AC>
__global__ void __launch_bounds__(AH_THREADS) a2c_head_kernel(A2cHeadArgs args) {
  constexpr int A1 = AC + 1;
  const HeadBwdArgs& a = args.h;
  __shared__ double sh[4 * 8];
  __shared__ float s_dz[AH_MAXB * A1];
  __shared__ float s_rew[AH_MAXB], s_val[AH_MAXB + AH_MAXN], s_ret[AH_MAXB], s_adv[AH_MAXB];
  __shared__ uint8_t s_dn[AH_MAXB];
  __shared__ float s_wh[AH_COLS * A1];
  __shared__ float s_red[4 * AH_COLS * (A1 + 1)];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int B = a.B, N = a.N;
  // side duties spread over workgroups 0..3 (one extra reduction each instead of all on one straggler):
  // 0 targets / advantages out, 1 EV-before, 2 loss statistics, 3 head-bias gradient
  const bool lead = blockIdx.x == 0, ev_wg = blockIdx.x == 1, st_wg = blockIdx.x == 2, bh_wg = blockIdx.x == 3;
  const int col0 = blockIdx.x * AH_COLS;
  hb_stamp(a, 0);
  // ---- phase 0: bootstrap values of this workgroup's envs: the whole workgroup per env (thread t: hidden units
  // 2t, 2t + 1, every plane's load in flight at once -- fc_h2_from_parts, the fused rollout step's reduction), then
  // h . Wh[:, A] reduced in a fixed order (xor tree per wave, waves in order)
  if (args.hpart) {
    __shared__ float s_vw[4];
    const float w0 = bf2f(a.Wh[(2 * tid) * A1 + AC]), w1 = bf2f(a.Wh[(2 * tid + 1) * A1 + AC]);
    for (int e = blockIdx.x; e < N; e += AH_WG) {
      float hv[2];
      fc_h2_from_parts<32>(args.hpart, args.S, args.plane_stride, args.bfc, e, tid, nullptr, hv);
      const float part = wave_sum(hv[0] * w0 + hv[1] * w1);
      if (lane == 0) s_vw[wv] = part;
      __syncthreads();
      if (tid == 0)
        __hip_atomic_store(&args.vboot[e], ((s_vw[0] + s_vw[1]) + (s_vw[2] + s_vw[3])) + args.bh[AC],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
    }
  }
  // ---- operands independent of V(s_T), requested before the barrier wait
  for (int i = tid; i < B; i += AH_THREADS) {
    s_rew[i] = a.rew[i];
    s_dn[i] = a.dn[i];
    s_val[i] = a.val[i];
  }
  if (tid < AH_COLS * A1) s_wh[tid] = bf2f(a.Wh[col0 * A1 + tid]);   // columns col0.. are contiguous rows of Wh
  float zr[2][A1];
  int ab[2];
  float lpo[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int rb = min(tid + k * AH_THREADS, B - 1);
#pragma unroll
    for (int j = 0; j < A1; ++j) zr[k][j] = a.z[(int64_t)rb * A1 + j];
    ab[k] = a.act[rb];
    lpo[k] = a.logp_old[rb];
  }
  const int cg = tid & 3, rl = tid >> 2;   // head phase: 4-column group, first row
  const int jc0 = col0 + 4 * cg;
  uint2 hv2[AH_RPT];
#pragma unroll
  for (int r = 0; r < AH_RPT; ++r) {
    const int b = min(rl + 64 * r, B - 1);
    hv2[r] = *reinterpret_cast<const uint2*>(a.h + (int64_t)b * HB_H + jc0);
  }
  const float c_ent = *a.ent_coef, beta = *a.kl_coef;
  // ---- grid barrier (bootstrap values published)
  if (args.hpart) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's sc1 value stores are acknowledged
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(&args.bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned int spins = 0;
      int ok = 1;
      while (__hip_atomic_load(&args.bar[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned int)AH_WG) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > AH_SPIN_LIMIT) { ok = 0; break; }
      }
      if (!ok) __hip_atomic_store(&args.bar[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    for (int i = tid; i < N; i += AH_THREADS)
      s_val[B + i] = __hip_atomic_load(&args.vboot[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // departure: the last workgroup past the wait resets the barrier for the next launch (stream-ordered)
    if (tid == 0) {
      const unsigned int prev = __hip_atomic_fetch_add(&args.bar[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == (unsigned int)AH_WG - 1u) {
        __hip_atomic_store(&args.bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&args.bar[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else {
    for (int i = tid; i < N; i += AH_THREADS) s_val[B + i] = a.val[B + i];
  }
  __syncthreads();
  hb_stamp(a, 1);
  // ---- returns, advantage moments (+ EV-before sums on workgroup 0)
  double s_r = 0, s_rr = 0, s_v = 0, s_vv = 0, s_rv = 0, s_a = 0, s_aa = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + k * AH_THREADS;
    if (idx < B) {
      const int t = idx / N, n = idx - t * N;
      float R;
      if (a.returns_mode == 1) {
        const int hh = min(t + a.L, a.T);
        float acc = 0.f, disc = 1.f;
        bool alive = true;
        for (int q = t; q < hh; ++q) {
          const int i = q * N + n;
          acc += disc * s_rew[i];
          disc *= a.gamma;
          if (s_dn[i]) { alive = false; break; }
        }
        if (alive) acc += disc * s_val[hh * N + n];
        R = acc;
      } else {
        float last = 0.f;
        for (int q = a.T - 1; q >= t; --q) {
          const int i = q * N + n;
          const float nd = s_dn[i] ? 0.f : 1.f;
          const float delta = s_rew[i] + a.gamma * s_val[i + N] * nd - s_val[i];
          last = delta + a.gamma * a.lam * nd * last;
        }
        R = last + s_val[idx];
      }
      const float v = s_val[idx], A_ = R - v;
      if (lead) {
        a.ret_w[idx] = R;
        a.adv_w[idx] = A_;
      }
      s_ret[idx] = R;
      s_adv[idx] = A_;
      s_r += R; s_rr += (double)R * R; s_v += v; s_vv += (double)v * v; s_rv += (double)R * v; s_a += A_;
      s_aa += (double)A_ * A_;
    }
  }
  const double nB = B;
  float adv_mean = 0.f, adv_inv = 1.f;
  if (ev_wg) {
    double red[7] = {s_a, s_aa, s_r, s_rr, s_v, s_vv, s_rv};
    block_sum_multi<7>(red, sh);
    if (tid == 0) {
      const double mr = red[2] / nB, mv = red[4] / nB;
      const double vr = fmax(red[3] / nB - mr * mr, 0.0), vv = fmax(red[5] / nB - mv * mv, 0.0);
      a.stats[7] = (float)((red[6] / nB - mr * mv) / sqrt(vr * vv));
    }
    s_a = red[0];
    s_aa = red[1];
  } else {
    double red[2] = {s_a, s_aa};   // the same per-value tree as the lead's: bit-identical moments
    block_sum_multi<2>(red, sh);
    s_a = red[0];
    s_aa = red[1];
  }
  hb_stamp(a, 2);
  if (a.norm_adv) {
    const double m = s_a / nB, var = fmax(s_aa / nB - m * m, 0.0);
    adv_mean = (float)m;
    adv_inv = 1.0f / (1e-8f + (float)sqrt(var));
  }
  // ---- loss + dz
  const float invB = 1.0f / (float)B;
  double s_pg = 0, s_kl = 0, s_H = 0, s_vl = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + k * AH_THREADS;
    if (idx < B) {
      const float adv = (s_adv[idx] - adv_mean) * adv_inv;
      const float R = s_ret[idx];
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < AC; ++j) mx = fmaxf(mx, zr[k][j]);
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < AC; ++j) se += expf(zr[k][j] - mx);
      const float lse = mx + logf(se);
      float H = 0.f, lpa = 0.f;
#pragma unroll
      for (int j = 0; j < AC; ++j) {
        const float lz = zr[k][j] - lse;
        H -= expf(lz) * lz;
        lpa = (j == ab[k]) ? lz : lpa;
      }
      s_pg += -(double)(adv * lpa);
      const float dkl = lpo[k] - lpa;
      s_kl += (double)(dkl * dkl);
      s_H += H;
      const float g_lpa = -adv * invB - 2.0f * beta * dkl * invB;
#pragma unroll
      for (int j = 0; j < AC; ++j) {
        const float lz = zr[k][j] - lse, pj = expf(lz);
        const float g = g_lpa * (((j == ab[k]) ? 1.0f : 0.0f) - pj) + c_ent * invB * pj * (lz + H);
        s_dz[idx * A1 + j] = bf2f(f2bf(g));   // the bf16 rounding of the GEMM path's dz buffer
      }
      const float d = zr[k][AC] - R;
      s_vl += (double)(d * d);
      s_dz[idx * A1 + AC] = bf2f(f2bf(a.vf_coef * 2.0f * d * invB));
    }
  }
  if (st_wg) {
    double r4[4] = {s_pg, s_kl, s_H, s_vl};
    block_sum_multi<4>(r4, sh);   // ends with a barrier: s_dz complete
    if (tid == 0) {
      const double inv = 1.0 / B;
      a.stats[0] = (float)(r4[0] * inv);
      a.stats[1] = (float)(r4[1] * inv);
      a.stats[2] = (float)(r4[2] * inv);
      a.stats[3] = (float)(r4[3] * inv);
      a.stats[4] = 0.f;
      a.stats[5] = (float)(r4[0] * inv + beta * r4[1] * inv - c_ent * r4[2] * inv);
      a.stats[6] = 1.f;
    }
  } else {
    __syncthreads();   // s_dz complete
  }
  hb_stamp(a, 3);
  // ---- head backward: 4 columns x rows rl + 64 i
  float wj[4][A1];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int q = 0; q < A1; ++q) wj[c][q] = s_wh[(4 * cg + c) * A1 + q];
  float dwp[4][A1], dbf[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    dbf[c] = 0.f;
#pragma unroll
    for (int q = 0; q < A1; ++q) dwp[c][q] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < AH_RPT; ++r) {
    const int b = rl + 64 * r;
    if (b < B) {
      float dzb[A1];
#pragma unroll
      for (int q = 0; q < A1; ++q) dzb[q] = s_dz[b * A1 + q];
      const uint32_t hw[2] = {hv2[r].x, hv2[r].y};
      uint32_t out[2];
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        uint32_t packed = 0;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int c = 2 * c2 + e;
          const float hf = __uint_as_float(e ? (hw[c2] & 0xFFFF0000u) : (hw[c2] << 16));
          float sacc = 0.f;
#pragma unroll
          for (int q = 0; q < A1; ++q) {
            sacc += dzb[q] * wj[c][q];
            dwp[c][q] += hf * dzb[q];
          }
          const float d = hf > 0.f ? sacc : 0.f;
          dbf[c] += d;
          packed |= (uint32_t)f2bf(d) << (16 * e);
        }
        out[c2] = packed;
      }
      *reinterpret_cast<uint2*>(a.dh + (int64_t)b * HB_H + jc0) = make_uint2(out[0], out[1]);
    }
  }
  // lanes sharing a column group (lane & 3) -> xor over lane bits 2..5, fixed order
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) {
      dbf[c] += lane_xor(dbf[c], o);
#pragma unroll
      for (int q = 0; q < A1; ++q) dwp[c][q] += lane_xor(dwp[c][q], o);
    }
  }
  hb_stamp(a, 4);
  if (lane < 4) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float* dstw = s_red + (wv * AH_COLS + 4 * lane + c) * (A1 + 1);
#pragma unroll
      for (int q = 0; q < A1; ++q) dstw[q] = dwp[c][q];
      dstw[A1] = dbf[c];
    }
  }
  __syncthreads();
  if (tid < AH_COLS * (A1 + 1)) {   // (column, value) pairs: the 4 waves in wave order
    const int cl = tid / (A1 + 1), q = tid - cl * (A1 + 1);
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += s_red[(w * AH_COLS + cl) * (A1 + 1) + q];
    if (q < A1) a.gWh[(col0 + cl) * A1 + q] = v;
    else a.gbfc[col0 + cl] = v;
  }
  if (bh_wg) {   // head-bias gradient: column q of dz, rows strided over a wave, xor tree (fixed order)
    for (int q = wv; q < A1; q += 4) {
      float sb = 0.f;
      for (int bb = lane; bb < B; bb += 64) sb += s_dz[bb * A1 + q];
      sb = wave_sum(sb);
      if (lane == 0) a.gbh[q] = sb;
    }
  }
  if (a.stamps) {
    hb_stamp(a, 5);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    hb_stamp(a, 6);
  }
}

// ------------------------------------------------------------------------------------------------------------
// A2C learner head v3, one workgroup PER ENV, no grid-wide hand-off (A2C without advantage normalisation -- the
// headline pong_a2c config --: every quantity of env e's rows depends only on env e). Workgroup e:
//   * V(s_T, e) straight from the rollout's last fc partial planes (fc_h2_from_parts: the rollout step's plane order
//     and bf16 rounding of h), dot with the value column of Wh reduced in a fixed order, stored into val[T][e];
//   * the returns / advantages of its T rows (n-step or GAE), loss + dz (bf16-rounded like the GEMM path);
//   * the head backward of its rows: dh = (h > 0) * dz Wh^T (stored), and PER-ENV PARTIAL PLANES of dWh = h^T dz,
//     dbfc = colsum(dh) and dbh = colsum(dz): plane e of [N, 512 * A1] / [N, 512] / [N, A1], summed in plane order by
//     the gradient finaliser (engine._head_planes -> finalize jobs), as the large-batch ppo_head's planes are;
//   * its share of the statistics as one fp64 row [pg, kl, H, vl, R, R^2, V, V^2, R V] of `spart`, combined by the
//     finaliser's statistics duty (a2c_stats_duty) into stats[0..7].
// Replaces a2c_head's 32-workgroup grid barrier (the bootstrap values handed over with sc1 stores + a spinning
// counter: ~4.5 us of its ~15) and its per-column layout (which needed every V(s_T) in every workgroup).
// thread t: hidden units 2t, 2t + 1.
// ------------------------------------------------------------------------------------------------------------
constexpr int AE_THREADS = 256;
constexpr int AE_MAXT = 64;

struct A2cEnvArgs {
  HeadBwdArgs h;
  const float* hpart; int S; int64_t plane_stride;   // last fc product of s_T (split-K planes), or null: val[T] holds V
  const float* bfc; const float* bh;
  float* pWh; float* pbfc; float* pbh;               // planes [N][512 * A1], [N][512], [N][A1]
  double* spart;                                     // [N][A2C_STATS] statistics rows
};

template <int AC>
__global__ void __launch_bounds__(AE_THREADS) a2c_head_env_kernel(A2cEnvArgs args) {
  constexpr int A1 = AC + 1;
  const HeadBwdArgs& a = args.h;
  __shared__ float s_dz[AE_MAXT * A1];
  __shared__ float s_rew[AE_MAXT], s_val[AE_MAXT + 1];
  __shared__ uint8_t s_dn[AE_MAXT];
  __shared__ float s_vw[4];
  __shared__ double s_st[AE_MAXT * 9];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int e = blockIdx.x, N = a.N, T = a.T;
  hb_stamp(a, 0);
  // ---- loads: the bootstrap planes first (the longest chain), then everything else of this env
  FcH2<16> fh;
  if (args.hpart) fh.issue(args.hpart, args.S, args.plane_stride, args.bfc, e, tid);
  float w2[2][A1];
  {   // rows 2t, 2t + 1 of Wh = 2 A1 consecutive bf16 at a 4-byte aligned offset: A1 32-bit loads
    const uint32_t* wp = reinterpret_cast<const uint32_t*>(a.Wh) + tid * A1;
    uint32_t wu[A1];
#pragma unroll
    for (int q = 0; q < A1; ++q) wu[q] = wp[q];
#pragma unroll
    for (int i = 0; i < 2 * A1; ++i) {
      const float v = __uint_as_float((i & 1) ? (wu[i >> 1] & 0xFFFF0000u) : (wu[i >> 1] << 16));
      w2[i / A1][i % A1] = v;
    }
  }
  if (tid < T) {
    const int i = tid * N + e;
    s_rew[tid] = a.rew[i];
    s_dn[tid] = a.dn[i];
    s_val[tid] = a.val[i];
  }
  float zr[A1];
  int ab = 0;
  float lpo = 0.f;
  if (tid < T) {
    const int64_t row = (int64_t)tid * N + e;
#pragma unroll
    for (int j = 0; j < A1; ++j) zr[j] = a.z[row * A1 + j];
    ab = a.act[row];
    lpo = a.logp_old[row];
  }
  // this thread's two hidden units (bf16 pair) of rows 0..7, requested before the bootstrap wait (later rows: in
  // the backward loop, 8 at a time)
  constexpr int HR = 8;
  uint32_t hr[HR];
#pragma unroll
  for (int r = 0; r < HR; ++r)
    hr[r] = r < T ? reinterpret_cast<const uint32_t*>(a.h + ((int64_t)r * N + e) * HB_H)[tid] : 0u;
  const float c_ent = *a.ent_coef, beta = *a.kl_coef;
  // ---- bootstrap value V(s_T, e): fixed order (xor tree per wave, waves in order)
  if (args.hpart) {
    float hv[2];
    fh.finish(args.hpart, args.S, args.plane_stride, e, tid, nullptr, hv);
    const float part = wave_sum(hv[0] * w2[0][AC] + hv[1] * w2[1][AC]);
    if (lane == 0) s_vw[wv] = part;
    __syncthreads();
    const float vT = ((s_vw[0] + s_vw[1]) + (s_vw[2] + s_vw[3])) + args.bh[AC];
    if (tid == 0) {
      s_val[T] = vT;
      const_cast<float*>(a.val)[(int64_t)T * N + e] = vT;
    }
  } else if (tid == 0) {
    s_val[T] = a.val[(int64_t)T * N + e];
  }
  __syncthreads();
  hb_stamp(a, 1);
  // ---- returns, loss, dz of row t (thread t < T), statistics row
  double st[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (tid < T) {
    const int t = tid;
    float R;
    if (a.returns_mode == 1) {
      const int hh = min(t + a.L, T);
      float acc = 0.f, disc = 1.f;
      bool alive = true;
      for (int q = t; q < hh; ++q) {
        acc += disc * s_rew[q];
        disc *= a.gamma;
        if (s_dn[q]) { alive = false; break; }
      }
      if (alive) acc += disc * s_val[hh];
      R = acc;
    } else {
      float last = 0.f;
      for (int q = T - 1; q >= t; --q) {
        const float nd = s_dn[q] ? 0.f : 1.f;
        const float delta = s_rew[q] + a.gamma * s_val[q + 1] * nd - s_val[q];
        last = delta + a.gamma * a.lam * nd * last;
      }
      R = last + s_val[t];
    }
    const float v = s_val[t], adv = R - v;
    const int64_t row = (int64_t)t * N + e;
    a.ret_w[row] = R;
    a.adv_w[row] = adv;
    const float invB = 1.0f / (float)a.B;
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < AC; ++j) mx = fmaxf(mx, zr[j]);
    float se = 0.f;
#pragma unroll
    for (int j = 0; j < AC; ++j) se += expf(zr[j] - mx);
    const float lse = mx + logf(se);
    float H = 0.f, lpa = 0.f;
#pragma unroll
    for (int j = 0; j < AC; ++j) {
      const float lz = zr[j] - lse;
      H -= expf(lz) * lz;
      lpa = (j == ab) ? lz : lpa;
    }
    const float dkl = lpo - lpa;
    const float g_lpa = -adv * invB - 2.0f * beta * dkl * invB;
#pragma unroll
    for (int j = 0; j < AC; ++j) {
      const float lz = zr[j] - lse, pj = expf(lz);
      const float g = g_lpa * (((j == ab) ? 1.0f : 0.0f) - pj) + c_ent * invB * pj * (lz + H);
      s_dz[t * A1 + j] = bf2f(f2bf(g));   // the bf16 rounding of the GEMM path's dz buffer
    }
    const float d = zr[AC] - R;
    s_dz[t * A1 + AC] = bf2f(f2bf(a.vf_coef * 2.0f * d * invB));
    st[0] = -(double)(adv * lpa);
    st[1] = (double)(dkl * dkl);
    st[2] = H;
    st[3] = (double)(d * d);
    st[4] = R; st[5] = (double)R * R; st[6] = v; st[7] = (double)v * v; st[8] = (double)R * v;
  }
  // the statistics rows go through LDS and are summed by one thread after the backward (off the critical path:
  // a 64-lane fp64 xor tree per statistic was ~1.5 us of dependent shuffles before the barrier)
  if (tid < T) {
#pragma unroll
    for (int k = 0; k < 9; ++k) s_st[tid * 9 + k] = st[k];
  }
  __syncthreads();   // s_dz, s_st complete
  hb_stamp(a, 2);
  // ---- head backward of this env's rows: units 2t, 2t + 1
  float dwp[2][A1], dbf[2] = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int q = 0; q < A1; ++q) dwp[c][q] = 0.f;
  for (int r0 = 0; r0 < T; r0 += HR) {
    if (r0 > 0) {
#pragma unroll
      for (int u = 0; u < HR; ++u)
        hr[u] = r0 + u < T ? reinterpret_cast<const uint32_t*>(a.h + ((int64_t)(r0 + u) * N + e) * HB_H)[tid] : 0u;
    }
#pragma unroll
    for (int u = 0; u < HR; ++u) {
    const int r = r0 + u;
    if (r >= T) break;
    float dzb[A1];
#pragma unroll
    for (int q = 0; q < A1; ++q) dzb[q] = s_dz[r * A1 + q];
    uint32_t packed = 0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float hf = __uint_as_float(c ? (hr[u] & 0xFFFF0000u) : (hr[u] << 16));
      float sacc = 0.f;
#pragma unroll
      for (int q = 0; q < A1; ++q) {
        sacc += dzb[q] * w2[c][q];
        dwp[c][q] += hf * dzb[q];
      }
      const float d = hf > 0.f ? sacc : 0.f;
      dbf[c] += d;
      packed |= (uint32_t)f2bf(d) << (16 * c);
    }
    reinterpret_cast<uint32_t*>(a.dh + ((int64_t)r * N + e) * HB_H)[tid] = packed;
    }
  }
  hb_stamp(a, 3);
  float* pw = args.pWh + (int64_t)e * HB_H * A1 + 2 * tid * A1;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int q = 0; q < A1; ++q) pw[c * A1 + q] = dwp[c][q];
  reinterpret_cast<float2*>(args.pbfc + (int64_t)e * HB_H)[tid] = make_float2(dbf[0], dbf[1]);
  if (tid < A1) {   // head-bias gradient of this env: column tid of dz over the rows in order
    float sb = 0.f;
    for (int r = 0; r < T; ++r) sb += s_dz[r * A1 + tid];
    args.pbh[(int64_t)e * A1 + tid] = sb;
  }
  if (tid == 64) {   // this env's statistics row: the rows summed in order (a thread of the second wave)
    double tot[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < T; ++r)
#pragma unroll
      for (int k = 0; k < 9; ++k) tot[k] += s_st[r * 9 + k];
    double* sp = args.spart + (int64_t)e * A2C_STATS;
#pragma unroll
    for (int k = 0; k < 9; ++k) sp[k] = tot[k];
  }
  if (a.stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    hb_stamp(a, 4);
  }
}

}  // namespace aca

extern "C" hipError_t aca_head_bwd(const float* z, const int32_t* act, const float* logp_old, const float* ent_coef,
                                   const float* kl_coef, float vf_coef, const float* rew, const float* val,
                                   const uint8_t* dn, int T, int N, int L, int returns_mode, int norm_adv, float gamma,
                                   float lam, float* ret_w, float* adv_w, const uint16_t* h, const uint16_t* Wh,
                                   uint16_t* dh, float* gWh, float* gbh, float* gbfc, float* stats, int A,
                                   uint64_t* stamps, hipStream_t stream) {
  const int B = T * N;
  if (B < 1 || B > aca::HB_MAXB || N > 256 || A < 2 || A > 7 || (returns_mode != 1 && returns_mode != 2))
    return hipErrorInvalidValue;
  aca::HeadBwdArgs a{z, act, logp_old, ent_coef, kl_coef, vf_coef, rew, val, dn, T, N, L, returns_mode, norm_adv,
                     gamma, lam, ret_w, adv_w, h, Wh, dh, gWh, gbh, gbfc, stats, B, stamps};
  switch (A) {
#define ACA_HB_CASE(n) \
  case n: aca::head_bwd_kernel<n><<<aca::HB_WG, aca::HB_THREADS, 0, stream>>>(a); break;
    ACA_HB_CASE(2) ACA_HB_CASE(3) ACA_HB_CASE(4) ACA_HB_CASE(5) ACA_HB_CASE(6) ACA_HB_CASE(7)
#undef ACA_HB_CASE
  }
  return hipGetLastError();
}

extern "C" hipError_t aca_a2c_head(const float* z, const int32_t* act, const float* logp_old, const float* ent_coef,
                                   const float* kl_coef, float vf_coef, const float* rew, float* val,
                                   const uint8_t* dn, int T, int N, int L, int returns_mode, int norm_adv, float gamma,
                                   float lam, float* ret_w, float* adv_w, const uint16_t* h, const uint16_t* Wh,
                                   uint16_t* dh, float* gWh, float* gbh, float* gbfc, float* stats, int A,
                                   const float* hpart, int S, int64_t plane_stride, const float* bfc, const float* bh,
                                   unsigned int* bar, uint64_t* stamps, hipStream_t stream) {
  const int B = T * N;
  if (B < 1 || B > aca::AH_MAXB || N > aca::AH_MAXN || A < 2 || A > 7 || (returns_mode != 1 && returns_mode != 2))
    return hipErrorInvalidValue;
  if (hpart && (S < 1 || S > aca::FC_MAX_PLANES || !bfc || !bh || !bar || reinterpret_cast<uintptr_t>(hpart) % 16 ||
                reinterpret_cast<uintptr_t>(bfc) % 16 || plane_stride % 4))
    return hipErrorInvalidValue;
  aca::A2cHeadArgs a;
  a.h = aca::HeadBwdArgs{z, act, logp_old, ent_coef, kl_coef, vf_coef, rew, val, dn, T, N, L, returns_mode, norm_adv,
                         gamma, lam, ret_w, adv_w, h, Wh, dh, gWh, gbh, gbfc, stats, B, stamps};
  a.hpart = hpart; a.S = S; a.plane_stride = plane_stride; a.bfc = bfc; a.bh = bh; a.vboot = val + B; a.bar = bar;
  switch (A) {
#define ACA_AH_CASE(n) \
  case n: aca::a2c_head_kernel<n><<<aca::AH_WG, aca::AH_THREADS, 0, stream>>>(a); break;
    ACA_AH_CASE(2) ACA_AH_CASE(3) ACA_AH_CASE(4) ACA_AH_CASE(5) ACA_AH_CASE(6) ACA_AH_CASE(7)
#undef ACA_AH_CASE
  }
  return hipGetLastError();
}

extern "C" hipError_t aca_a2c_head_env(const float* z, const int32_t* act, const float* logp_old,
                                       const float* ent_coef, const float* kl_coef, float vf_coef, const float* rew,
                                       float* val, const uint8_t* dn, int T, int N, int L, int returns_mode,
                                       float gamma, float lam, float* ret_w, float* adv_w, const uint16_t* h,
                                       const uint16_t* Wh, uint16_t* dh, int A, const float* hpart, int S,
                                       int64_t plane_stride, const float* bfc, const float* bh, float* pWh,
                                       float* pbfc, float* pbh, double* spart, uint64_t* stamps,
                                       hipStream_t stream) {
  const int B = T * N;
  if (T < 1 || T > aca::AE_MAXT || N < 1 || A < 2 || A > 7 || (returns_mode != 1 && returns_mode != 2) || !pWh ||
      !pbfc || !pbh || !spart)
    return hipErrorInvalidValue;
  if (hpart && (S < 1 || S > aca::FC_MAX_PLANES || !bfc || !bh || reinterpret_cast<uintptr_t>(hpart) % 16 ||
                reinterpret_cast<uintptr_t>(bfc) % 16 || plane_stride % 4))
    return hipErrorInvalidValue;
  aca::A2cEnvArgs a;
  a.h = aca::HeadBwdArgs{z, act, logp_old, ent_coef, kl_coef, vf_coef, rew, val, dn, T, N, L, returns_mode, 0,
                         gamma, lam, ret_w, adv_w, h, Wh, dh, nullptr, nullptr, nullptr, nullptr, B, stamps};
  a.hpart = hpart; a.S = S; a.plane_stride = plane_stride; a.bfc = bfc; a.bh = bh;
  a.pWh = pWh; a.pbfc = pbfc; a.pbh = pbh; a.spart = spart;
  switch (A) {
#define ACA_AE_CASE(n) \
  case n: aca::a2c_head_env_kernel<n><<<N, aca::AE_THREADS, 0, stream>>>(a); break;
    ACA_AE_CASE(2) ACA_AE_CASE(3) ACA_AE_CASE(4) ACA_AE_CASE(5) ACA_AE_CASE(6) ACA_AE_CASE(7)
#undef ACA_AE_CASE
  }
  return hipGetLastError();
}

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
  case n: aca::ac_loss_kernel<n><<<1, aca::loss_threads<n>(), 0, stream>>>(a); break;
      ACA_LOSS_CASE(2) ACA_LOSS_CASE(3) ACA_LOSS_CASE(4) ACA_LOSS_CASE(5) ACA_LOSS_CASE(6) ACA_LOSS_CASE(7)
      ACA_LOSS_CASE(8) ACA_LOSS_CASE(9) ACA_LOSS_CASE(10) ACA_LOSS_CASE(11) ACA_LOSS_CASE(12) ACA_LOSS_CASE(13)
      ACA_LOSS_CASE(14) ACA_LOSS_CASE(15) ACA_LOSS_CASE(16) ACA_LOSS_CASE(17) ACA_LOSS_CASE(18) ACA_LOSS_CASE(19)
#undef ACA_LOSS_CASE
    }
  } else {
    aca::ac_loss_kernel<0><<<1, aca::loss_threads<0>(), 0, stream>>>(a);
  }
  return hipGetLastError();
}
