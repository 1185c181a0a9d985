// Fused MLP actor-critic engine (SURVEY §2.4 K01 / K02 / K05 / K07 / K08 for the reference's MLP family).
//
// The reference's networks (Basic_AC/policies.py:33-162, A3C/policies.py:34-182) are two separate towers:
//   actor  D -> 128 lrelu -> 128 lrelu -> 64 lrelu -> A  (tanh * ac_scale: diagonal Gaussian | logits: categorical)
//   critic D -> 256 relu -> 128 relu (-> 128 relu, A3C variant) -> 1
// At these widths every layer is a skinny GEMM (M = rows, K/N <= 256) and launch count, not FLOPs, sets the time:
// the TF reference runs ~10 ops per layer per Session.run. Here a whole tower runs inside ONE workgroup per 16-row
// tile, activations staying in LDS between layers:
//
// mlp_fwd_kernel   grid (row tiles, towers). mode 0 (rollout): forward + head (Gaussian Box-Muller / Gumbel-max
//                  sample with the env-counter RNG key, log-prob, entropy) + value; mode 1 (evaluate): log-prob /
//                  entropy of given actions + value; mode 2 (train): forward, per-row loss gradient (A2C or PPO-clip
//                  policy loss with the reference's KL-proxy and entropy terms, Gaussian or categorical head; MSE or
//                  clipped value loss) and the whole data-gradient chain dP_l -> dX_l = dP_l W_l^T -> * act'(y_{l-1})
//                  in LDS; layer inputs X_l and pre-activation gradients dP_l are written out for the weight
//                  gradients, the log-std gradient is reduced per tile and added atomically.
// mlp_wgrad_kernel one wave per 16x16 tile of every dW_l = X_l^T dP_l (+ the bias column sums): the whole batch is
//                  its K dimension, so every gradient element is written exactly once (no atomics, deterministic),
//                  and the wave also emits its sum of squares into a fixed slot -- the global-norm clip of the fused
//                  optimiser needs no separate reduction launch. It also publishes the loss statistics.
//
// Numerics: fp32 end to end (the reference is fp32). GEMM-shaped work runs on the f32-input MFMA
// v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulate; on gfx950 it runs at the f32 vector rate with 4x the
// operand reuse of a VALU FMA tile). Fragment maps (cdna_hip_programming.md §3): A[l&15][k=l>>4], B[k=l>>4][l&15],
// C/D col = l&15, row = 4(l>>4)+i. The k index of a 16-wide k-group is remapped k = 16g + 4(l>>4) + s for the four
// MFMAs s = 0..3, so each lane's A fragments for a k-group are one 16-byte LDS read and, in the data-gradient
// products, its B fragments one 16-byte load of a weight row ([in][out] = TF dense layout).
#include "common.h"
#include "mlp_desc.h"

namespace aca {

constexpr int MLP_BM = 16;          // rows per workgroup
constexpr int MLP_THREADS = 512;    // 8 waves
constexpr int MLP_MAXW = 256;       // widest layer
constexpr int MLP_MAXA = 16;        // widest head
constexpr int MLP_PARTS = 256;      // sumsq partial slots per tower (= optim.hip SUMSQ_PARTS)

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2, ACT_TANH = 3 };

template <typename T>
__device__ __forceinline__ T* P_(int64_t v) { return reinterpret_cast<T*>(v); }

__device__ __forceinline__ int rup16(int x) { return (x + 15) & ~15; }
__device__ __forceinline__ int ld_of(int w) { return rup16(w) + 4; }   // padded LDS row stride

__device__ __forceinline__ float act_fwd(float v, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_LRELU: return 0.8f * fmaxf(v, 0.f) + 0.2f * v;   // (1-a) relu(x) + a x, a = 0.2 (policies.py:20-21)
    case ACT_TANH: return tanhf(v);
    default: return v;
  }
}

// derivative from the activation OUTPUT y (relu/lrelu keep the sign of x; tanh' = 1 - y^2)
__device__ __forceinline__ float act_bwd(float y, int act) {
  switch (act) {
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_LRELU: return y > 0.f ? 1.f : 0.2f;
    case ACT_TANH: return 1.f - y * y;
    default: return 1.f;
  }
}

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Y[16][N] = act(X[16][K] W[K][N] + b) (* scale for the tanh head). X: LDS, zero-padded to rup16(K) columns.
// Y: LDS, columns [N, rup16(N)) written as 0 (so Y is a valid zero-padded input of the next layer).
// The tanh head stores tanh (unscaled) in Y so that act_bwd applies; the caller scales.
__device__ void layer_fwd(const float* __restrict__ X, int ldx, int K, const float* __restrict__ W,
                          const float* __restrict__ bias, int N, int act, float* __restrict__ Y, int ldy) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int ntile = (N + 15) >> 4, ng = rup16(K) >> 4;
  for (int tile = wave; tile < ntile; tile += MLP_THREADS / 64) {
    const int c = tile * 16 + r;
    const bool cok = c < N;
    const int cc = cok ? c : 0;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int g = 0; g < ng; ++g) {
      const int k0 = 16 * g + 4 * q;
      const float4 a4 = *reinterpret_cast<const float4*>(&X[r * ldx + k0]);
      float bv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bool ok = cok && (k0 + s) < K;
        const float w = W[(size_t)(ok ? k0 + s : 0) * N + cc];
        bv[s] = ok ? w : 0.f;
      }
      acc = mfma4(a4.x, bv[0], acc);
      acc = mfma4(a4.y, bv[1], acc);
      acc = mfma4(a4.z, bv[2], acc);
      acc = mfma4(a4.w, bv[3], acc);
    }
    const float bb = cok ? bias[cc] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) Y[(4 * q + i) * ldy + c] = cok ? act_fwd(acc[i] + bb, act) : 0.f;
  }
}

// dX[16][K] = dP[16][N] W[K][N]^T, then * act'(Yprev) (Yprev: LDS outputs of the previous layer, act_prev) ->
// dPprev (LDS, zero-padded) and, when gdst != null, the global rows of the previous layer's dP.
template <bool VEC>
__device__ void layer_dgrad(const float* __restrict__ dP, int ldp, int N, const float* __restrict__ W, int K,
                            const float* __restrict__ Yprev, int ldyp, int act_prev, float* __restrict__ dPprev,
                            int lddp, float* __restrict__ gdst, int rows) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int ntile = (K + 15) >> 4, ng = rup16(N) >> 4;
  for (int tile = wave; tile < ntile; tile += MLP_THREADS / 64) {
    const int kc = tile * 16 + r;   // output column = input feature of the layer
    const bool kok = kc < K;
    const float* wrow = W + (size_t)(kok ? kc : 0) * N;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int g = 0; g < ng; ++g) {
      const int n0 = 16 * g + 4 * q;
      const float4 a4 = *reinterpret_cast<const float4*>(&dP[r * ldp + n0]);
      float4 b4;
      if (VEC) {
        b4 = *reinterpret_cast<const float4*>(wrow + n0);
        if (!kok) b4 = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        float t[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bool ok = kok && (n0 + s) < N;
          const float w = wrow[ok ? n0 + s : 0];
          t[s] = ok ? w : 0.f;
        }
        b4 = make_float4(t[0], t[1], t[2], t[3]);
      }
      acc = mfma4(a4.x, b4.x, acc);
      acc = mfma4(a4.y, b4.y, acc);
      acc = mfma4(a4.z, b4.z, acc);
      acc = mfma4(a4.w, b4.w, acc);
    }
    // C layout: col = lane&15 = kc, rows 4q + i
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * q + i;
      float v = 0.f;
      if (kok) v = acc[i] * act_bwd(Yprev[row * ldyp + kc], act_prev);
      dPprev[row * lddp + kc] = v;
      if (gdst && kok && row < rows) gdst[(size_t)row * K + kc] = v;
    }
  }
}

__device__ __forceinline__ int64_t row_key(const MlpArgs& a, int grow) {
  return a.tg[grow] * ((int64_t)1 << a.key_shift) + a.env_ids[grow];
}

constexpr float HALF_LOG_2PI = 0.91893853320467274178f;
constexpr float TWO_PI = 6.28318530717958647692f;

__global__ void __launch_bounds__(MLP_THREADS) mlp_fwd_kernel(MlpArgs a) {
  extern __shared__ float sm[];
  __shared__ float s_red[MLP_BM][MLP_MAXA + 8];   // per-row partials: log-std grads + stats
  const int t = blockIdx.y + a.tw_base;
  const MlpTower& T = a.tw[t];
  const int nl = (int)T.nl;
  const int row0 = blockIdx.x * MLP_BM;
  const int rows = min(MLP_BM, a.B - row0);
  // ---- LDS layout: X0 | Y_0 .. Y_{nl-1} | dP ping-pong (train)
  const int ld0 = ld_of(a.D);
  float* X0 = sm;
  float* Y[MLP_MAXL];
  int ldy[MLP_MAXL];
  float* p = X0 + MLP_BM * ld0;
  for (int l = 0; l < nl; ++l) {
    ldy[l] = ld_of((int)T.out[l]);
    Y[l] = p;
    p += MLP_BM * ldy[l];
  }
  float* P0 = p;
  float* P1 = p + MLP_BM * (MLP_MAXW + 4);
  // ---- input tile (gathered rows; padded rows / columns are zero)
  for (int e = threadIdx.x; e < MLP_BM * ld0; e += MLP_THREADS) {
    const int r = e / ld0, c = e - r * ld0;
    float v = 0.f;
    if (r < rows && c < a.D) {
      const int64_t gr = a.idx ? a.idx[row0 + r] : (int64_t)(row0 + r);
      v = a.obs[gr * a.ld_obs + c];
    }
    X0[e] = v;
    if (a.mode == 2 && r < rows && c < a.D) P_<float>(T.xs[0])[(size_t)(row0 + r) * a.D + c] = v;
  }
  __syncthreads();
  // ---- forward
  const float* X = X0;
  int ldx = ld0;
  for (int l = 0; l < nl; ++l) {
    layer_fwd(X, ldx, (int)T.in[l], P_<const float>(T.W[l]), P_<const float>(T.b[l]), (int)T.out[l], (int)T.act[l],
              Y[l], ldy[l]);
    __syncthreads();
    if (a.mode == 2 && l + 1 < nl) {   // inputs of layer l+1 for its weight gradient
      const int w = (int)T.out[l];
      float* xs = P_<float>(T.xs[l + 1]);
      for (int e = threadIdx.x; e < rows * w; e += MLP_THREADS) {
        const int r = e / w, c = e - r * w;
        xs[(size_t)(row0 + r) * w + c] = Y[l][r * ldy[l] + c];
      }
    }
    X = Y[l];
    ldx = ldy[l];
  }
  const int L = nl - 1;
  const float* Yo = Y[L];
  const int ldo = ldy[L];
  // ---- heads: one thread per row
  const bool policy = (t == 0);
  float* dPtop = P0;
  const int ldP = MLP_MAXW + 4;
  if (a.mode == 2) {   // zero the top dP tile (the head writes only valid columns)
    for (int e = threadIdx.x; e < MLP_BM * ldP; e += MLP_THREADS) dPtop[e] = 0.f;
    __syncthreads();
  }
  const int tid = threadIdx.x;
  if (tid < MLP_BM) {
    const int r = tid;
    const bool live = r < rows;
    const int lrow = row0 + r;   // batch-local row (workspace / minibatch order)
    const int64_t grow = a.idx ? a.idx[lrow < a.B ? lrow : 0] : (int64_t)lrow;
    float st[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (!policy) {
      const float v = Yo[r * ldo];
      if (live && (a.mode == 0 || a.mode == 1) && a.v_out) a.v_out[grow] = v;
      if (live && a.mode == 2) {
        const float R = a.ret[grow];
        float dv = 2.f * (v - R), l2 = (v - R) * (v - R);
        if (a.v_old && a.v_clip > 0.f) {
          const float vo = a.v_old[grow];
          const float d = fminf(fmaxf(v - vo, -a.v_clip), a.v_clip);
          const float vc = vo + d;
          const float l2c = (vc - R) * (vc - R);
          const bool inr = (v - vo) >= -a.v_clip && (v - vo) <= a.v_clip;
          if (l2c > l2) { dv = inr ? 2.f * (vc - R) : 0.f; l2 = l2c; }
          else if (l2c == l2) dv = 0.5f * dv + 0.5f * (inr ? 2.f * (vc - R) : 0.f);
        }
        dPtop[r * ldP] = a.vf_coef * a.inv_B * dv;
        st[3] = l2;
      }
    } else if (a.head == 2) {   // diagonal Gaussian: mu = tanh(z) * scale
      const int A = a.A;
      float lp = 0.f, H = 0.f;
      float mu[MLP_MAXA], act[MLP_MAXA], ls[MLP_MAXA];
      const int64_t key = (a.mode == 0 && live) ? row_key(a, (int)grow) : 0;
      for (int j = 0; j < A; ++j) {
        ls[j] = fminf(fmaxf(a.log_std[j], -2.5f), 2.5f);
        mu[j] = Yo[r * ldo + j] * a.ac_scale[j];
        float aj;
        if (a.mode == 0) {
          const float u1 = uniform_open(a.seed, key, 2 * j), u2 = uniform_open(a.seed, key, 2 * j + 1);
          const float eps = sqrtf(-2.0f * logf(u1)) * cosf(TWO_PI * u2);
          aj = mu[j] + expf(ls[j]) * eps;
          if (live) a.act_f_out[grow * A + j] = aj;
        } else {
          aj = live ? a.act_f_in[grow * A + j] : mu[j];
        }
        act[j] = aj;
        const float zz = (aj - mu[j]) * expf(-ls[j]);
        lp += -0.5f * zz * zz - ls[j] - HALF_LOG_2PI;
        H += 0.5f + HALF_LOG_2PI + ls[j];
      }
      if (live && a.mode != 2) {
        if (a.logp_out) a.logp_out[grow] = lp;
        if (a.ent_out) a.ent_out[grow] = H;
      }
      if (a.mode == 2) {
        float g = 0.f;
        if (live) {
          const float lo = a.logp_old[grow], adv = a.adv[grow];
          const float beta = *a.kl_coef;
          float dsurr;
          if (a.ppo) {
            const float ratio = expf(lp - lo);
            const float s1 = ratio * adv;
            const float rc = fminf(fmaxf(ratio, 1.f - a.ppo_clip), 1.f + a.ppo_clip);
            const float s2 = rc * adv;
            dsurr = (s1 <= s2) ? ratio * adv : 0.f;
            st[0] = -fminf(s1, s2);
            st[4] = fabsf(ratio - 1.f) > a.ppo_clip ? 1.f : 0.f;
            st[6] = ratio;
          } else {
            dsurr = adv;
            st[0] = -adv * lp;
            st[6] = 1.f;
          }
          st[1] = (lo - lp) * (lo - lp);
          st[2] = H;
          g = a.inv_B * (-dsurr - 2.f * beta * (lo - lp));
        }
        const float ce = *a.ent_coef;
        for (int j = 0; j < A; ++j) {
          const float ivar = expf(-2.f * ls[j]);
          const float d = act[j] - mu[j];
          const float th = Yo[r * ldo + j];
          const float dmu = g * d * ivar;
          dPtop[r * ldP + j] = live ? dmu * a.ac_scale[j] * (1.f - th * th) : 0.f;
          const float raw = a.log_std[j];
          const bool inr = raw >= -2.5f && raw <= 2.5f;
          s_red[r][j] = (live && inr) ? g * (d * d * ivar - 1.f) - ce * a.inv_B : 0.f;
        }
      }
    } else {   // categorical logits
      const int A = a.A;
      float z[MLP_MAXA];
      float m = -INFINITY;
      for (int j = 0; j < A; ++j) { z[j] = Yo[r * ldo + j]; m = fmaxf(m, z[j]); }
      float se = 0.f;
      for (int j = 0; j < A; ++j) se += expf(z[j] - m);
      const float lse = m + logf(se);
      float H = 0.f;
      for (int j = 0; j < A; ++j) { const float lpj = z[j] - lse; H -= expf(lpj) * lpj; }
      int ai = 0;
      if (a.mode == 0) {
        const int64_t key = live ? row_key(a, (int)grow) : 0;
        float best = -INFINITY;
        for (int j = 0; j < A; ++j) {
          const float u = uniform_open(a.seed, key, (uint32_t)j);
          const float gj = z[j] + (-logf(-logf(u)));
          if (gj > best) { best = gj; ai = j; }
        }
        if (live) a.act_i_out[grow] = ai;
      } else {
        ai = live ? a.act_i_in[grow] : 0;
      }
      const float lpa = z[ai] - lse;
      if (live && a.mode != 2) {
        if (a.logp_out) a.logp_out[grow] = lpa;
        if (a.ent_out) a.ent_out[grow] = H;
      }
      if (a.mode == 2 && live) {
        const float lo = a.logp_old[grow], adv = a.adv[grow];
        const float beta = *a.kl_coef, ce = *a.ent_coef;
        float dsurr;
        if (a.ppo) {
          const float ratio = expf(lpa - lo);
          const float s1 = ratio * adv;
          const float rc = fminf(fmaxf(ratio, 1.f - a.ppo_clip), 1.f + a.ppo_clip);
          const float s2 = rc * adv;
          dsurr = (s1 <= s2) ? ratio * adv : 0.f;
          st[0] = -fminf(s1, s2);
          st[4] = fabsf(ratio - 1.f) > a.ppo_clip ? 1.f : 0.f;
          st[6] = ratio;
        } else {
          dsurr = adv;
          st[0] = -adv * lpa;
          st[6] = 1.f;
        }
        st[1] = (lo - lpa) * (lo - lpa);
        st[2] = H;
        const float g = a.inv_B * (-dsurr - 2.f * beta * (lo - lpa));
        for (int j = 0; j < A; ++j) {
          const float pj = expf(z[j] - lse);
          const float oh = j == ai ? 1.f : 0.f;
          dPtop[r * ldP + j] = g * (oh - pj) + ce * a.inv_B * pj * ((z[j] - lse) + H);
        }
      }
    }
    if (a.mode == 2) {
      // per-tile stats: reduce the 16 row threads (lanes 0..15 of wave 0)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = st[k];
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
        if (r == 0 && k != 5 && (policy ? (k != 3) : (k == 3)) && v != 0.f) atomicAdd(&a.mstats[k], v * a.inv_B);
      }
    }
  }
  if (a.mode != 2) return;
  __syncthreads();
  // log-std gradient: column sums over the tile's rows, one atomic per column
  if (policy && a.head == 2 && threadIdx.x < a.A) {
    float s = 0.f;
    for (int r = 0; r < MLP_BM; ++r) s += s_red[r][threadIdx.x];
    atomicAdd(&a.g_log_std[threadIdx.x], s);
  }
  // ---- top layer dP: apply the head activation derivative (tanh applied above) and publish
  {
    const int w = (int)T.out[L];
    float* dp = P_<float>(T.dp[L]);
    for (int e = threadIdx.x; e < rows * w; e += MLP_THREADS) {
      const int r = e / w, c = e - r * w;
      dp[(size_t)(row0 + r) * w + c] = dPtop[r * ldP + c];
    }
  }
  // ---- data-gradient chain: dP_l -> dP_{l-1}
  float* cur = P0;
  float* nxt = P1;
  for (int l = L; l >= 1; --l) {
    const int N = (int)T.out[l], K = (int)T.in[l];
    float* gdst = P_<float>(T.dp[l - 1]) + (size_t)row0 * K;
    const float* W = P_<const float>(T.W[l]);
    if ((N & 15) == 0)
      layer_dgrad<true>(cur, ldP, N, W, K, Y[l - 1], ldy[l - 1], (int)T.act[l - 1], nxt, ldP, gdst, rows);
    else
      layer_dgrad<false>(cur, ldP, N, W, K, Y[l - 1], ldy[l - 1], (int)T.act[l - 1], nxt, ldP, gdst, rows);
    __syncthreads();
    float* tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
}

// ------------------------------------------------------------------------------------------------ weight grads

__device__ __forceinline__ float clipsq(float v, float c) {
  if (c > 0.f) v = fminf(fmaxf(v, -c), c);
  return v * v;
}

__global__ void __launch_bounds__(256) mlp_wgrad_kernel(WgradArgs a) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int split = gw % a.nsplit;
  int item = gw / a.nsplit;
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.stats) {   // publish (and reset) the fused kernel's statistics
    float m[8];
    for (int k = 0; k < 8; ++k) m[k] = a.mstats[k];
    m[5] = m[0] + (*a.kl_coef) * m[1] - (*a.ent_coef) * m[2];
    for (int k = 0; k < 7; ++k) a.stats[k] = m[k];
    for (int k = 0; k < 8; ++k) a.mstats[k] = 0.f;
  }
  // locate (tower, layer, tile)
  int t = 0;
  if (item >= a.items[0]) {
    item -= a.items[0];
    t = 1;
    if (t >= a.ntw || item >= a.items[1]) return;
  }
  const int local_item = item;
  const MlpTower& T = a.tw[t];
  const int nl = (int)T.nl;
  int l = 0;
  for (; l < nl; ++l) {
    const int n = (((int)T.in[l] + 15) >> 4) * (((int)T.out[l] + 15) >> 4);
    if (item < n) break;
    item -= n;
  }
  if (l >= nl) return;
  const int K = (int)T.in[l], N = (int)T.out[l];
  const int tn = (N + 15) >> 4;
  const int ti = item / tn, tj = item - ti * tn;
  const int i0 = ti * 16, j0 = tj * 16;
  const int r = lane & 15, q = lane >> 4;
  const float* X = P_<const float>(T.xs[l]);
  const float* P = P_<const float>(T.dp[l]);
  const int ia = i0 + r, jb = j0 + r;
  const bool iok = ia < K, jok = jb < N;
  // rows of this split
  const int per = (((a.B + a.nsplit - 1) / a.nsplit) + 15) & ~15;
  const int rb = split * per, re = min(a.B, rb + per);
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  const bool do_bias = (ti == 0);
#pragma unroll 2
  for (int g0 = rb; g0 < re; g0 += 16) {
    float av[4], bv[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int row = g0 + 4 * q + s;
      const bool rok = row < re;
      const float xa = X[(size_t)(rok ? row : 0) * K + (iok ? ia : 0)];
      const float pb = P[(size_t)(rok ? row : 0) * N + (jok ? jb : 0)];
      av[s] = (rok && iok) ? xa : 0.f;
      bv[s] = (rok && jok) ? pb : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      acc = mfma4(av[s], bv[s], acc);
      bsum += bv[s];
    }
  }
  float ss = 0.f;
  const float c = a.clip[t];
  // C: col = lane&15 -> j, rows 4q+i -> i
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ii = i0 + 4 * q + i, jj = j0 + r;
    if (ii < K && jj < N) {
      float* dst = P_<float>(T.gW[l]) + (size_t)ii * N + jj;
      if (a.nsplit > 1) atomicAdd(dst, acc[i]);
      else {
        *dst = acc[i];
        ss += clipsq(acc[i], c);
      }
    }
  }
  if (do_bias) {
    // lanes with equal (lane & 15) hold partial column sums over rows = q (mod 4)
    bsum += __shfl_xor(bsum, 16, 64);
    bsum += __shfl_xor(bsum, 32, 64);
    if (q == 0 && jok) {
      if (a.nsplit > 1) atomicAdd(P_<float>(T.gb[l]) + jb, bsum);
      else {
        P_<float>(T.gb[l])[jb] = bsum;
        ss += clipsq(bsum, c);
      }
    }
  }
  if (a.nsplit == 1 && a.parts[t]) {
    if (t == 0 && local_item == 0 && a.g_log_std && lane < a.A) ss += clipsq(a.g_log_std[lane], c);
    ss = wave_sum(ss);
    if (lane == 0) a.parts[t][local_item] = ss;
    if (local_item == 0)   // unused slots are zero: the optimiser sums all MLP_PARTS in a fixed order
      for (int k = a.items[t] + lane; k < MLP_PARTS; k += 64) a.parts[t][k] = 0.f;
  }
}

}  // namespace aca

using namespace aca;

// Host launchers. The descriptor lives in device memory, so shape validation and the LDS size are the caller's
// (ops/mlp.py validates the tower shapes when it builds the descriptor and passes the LDS bytes it computed).
extern "C" hipError_t aca_mlp_fwd(const MlpArgs* a, int ntw, size_t lds, hipStream_t stream) {
  if (a->B <= 0) return hipSuccess;
  if (a->A > MLP_MAXA || a->D > MLP_MAXW || ntw < 1 || a->tw_base + ntw > 2 || !a->tw) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_fwd_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024) != hipSuccess)
      return hipErrorInvalidValue;
    attr = true;
  }
  if (lds > 140 * 1024) return hipErrorInvalidValue;
  dim3 grid((a->B + MLP_BM - 1) / MLP_BM, ntw);
  mlp_fwd_kernel<<<grid, MLP_THREADS, lds, stream>>>(*a);
  return hipGetLastError();
}

extern "C" hipError_t aca_mlp_wgrad(const WgradArgs* a, hipStream_t stream) {
  if (a->B <= 0) return hipSuccess;
  if (!a->tw || a->nsplit < 1 || a->ntw < 1 || a->ntw > 2) return hipErrorInvalidValue;
  for (int t = 0; t < a->ntw; ++t)
    if (a->parts[t] && a->nsplit == 1 && a->items[t] > MLP_PARTS) return hipErrorInvalidValue;
  const int total = a->items[0] + (a->ntw > 1 ? a->items[1] : 0);
  const int waves = total * a->nsplit;
  const int wpb = 4;
  mlp_wgrad_kernel<<<(waves + wpb - 1) / wpb, 64 * wpb, 0, stream>>>(*a);
  return hipGetLastError();
}
