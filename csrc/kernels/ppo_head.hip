// Large-batch learner head in ONE launch (PPO minibatches of the Nature-CNN engine, B = 4096 rows; SURVEY §2.4
// K04 / K07 / K08 and the head's share of K02):
//
//   z[b, :]   = h[b, :] . Wh + bh                       logits | value (A1 = A + 1 columns, fp32)
//   loss      = PPO-clip (or A2C) actor loss + KL proxy + entropy bonus + value loss    (ac_loss_kernel's maths)
//   dz[b, :]  = dL / dz[b, :]                            (fp32, never leaves the registers)
//   dh[b, k]  = (h[b, k] > 0) * sum_a dz[b, a] Wh[k, a]  (bf16: the fc layer's data gradient)
//   dWh[k, a] = sum_b h[b, k] dz[b, a],  dbh[a] = sum_b dz[b, a],  dbfc[k] = sum_b dh[b, k]
//
// It replaces the z GEMM, the 1024-thread loss launch, the dWh / dh GEMMs and the bias column sums of the generic
// path (5 launches, ~54 us per B = 4096 minibatch on MI355X, all latency-bound: N = A1 <= 8 columns). Every row is
// independent, so the grid is B / 16 workgroups of 4 waves (256 workgroups at B = 4096: every CU busy): wave w owns
// 4 rows, lane l owns hidden columns 8 l .. 8 l + 7 (one 16-byte h load and one 16-byte dh store per row) and holds
// the matching 8 x A1 slice of Wh in registers. z is a wave reduction; the row's loss maths then runs redundantly in
// every lane (no broadcast), so dz is lane-uniform and dh / dWh need no further communication.
//
// The cross-row sums are deterministic: each workgroup writes its partial dWh / dbh / dbfc as one plane (rows of
// the workgroup summed in a fixed order, waves combined in wave order through LDS) -- the engine's gradient
// finaliser reduces the planes in plane order -- and its loss statistics (fp64) as one record; the last-arriving
// workgroup (agent-scope release / acquire ticket, common.h last_block_arrival) sums the records in a fixed order
// (common.h grid_records_sum).
#include "common.h"
#include "ppo_head.h"

namespace aca {

template <int A1>
__global__ void __launch_bounds__(PH_THREADS) ppo_head_kernel(PpoHeadArgs p) {
  constexpr int A = A1 - 1;
  // per-wave dWh / dbfc partials (wave-ordered combine); lane l's 8 x A1 (8) values at l * (8 A1 + 1) (l * 9): an odd
  // lane stride keeps the 64 lanes' stores on distinct banks (stride 8 A1 / 8 was an 8-way conflict per store)
  constexpr int RS = 8 * A1 + 1, BS = 9;
  __shared__ float s_red[PH_THREADS / 64][64 * RS];
  __shared__ float s_rb[PH_THREADS / 64][64 * BS];
  __shared__ double s_st[PH_THREADS / 64][PH_NSTAT + A1];
  __shared__ double s_sum[16 * PH_NSTAT];                 // last workgroup: statistics reduction
  __shared__ int sh_flag;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wg = blockIdx.x;
  const int k0 = 8 * lane;
  // ---- every load issued before any use: Wh slice, bias, the wave's 4 rows (h chunk + row scalars)
  float W[8][A1];
  {
    const u16* wp = p.Wh + (size_t)k0 * A1;
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int a = 0; a < A1; ++a) W[e][a] = bf2f(wp[e * A1 + a]);
  }
  float bias[A1];
#pragma unroll
  for (int a = 0; a < A1; ++a) bias[a] = p.bh[a];
  const float c_ent = *p.ent_coef, beta = *p.kl_coef;
  const float invB = 1.0f / (float)p.B;
  uint4 hraw[PH_ROWS_PER_WAVE];
  int32_t ab[PH_ROWS_PER_WAVE];
  float lpo[PH_ROWS_PER_WAVE], adv[PH_ROWS_PER_WAVE], R[PH_ROWS_PER_WAVE], vo[PH_ROWS_PER_WAVE];
  if (p.hp) {
    // h from the fc product's split-K partial planes: sum in plane order, + bias, ReLU, bf16 -- the epilogue the
    // fc GEMM would have run (bitwise the same h), without its cross-workgroup reduction
    float hb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) hb[e] = p.hbias[k0 + e];
#pragma unroll
    for (int i = 0; i < PH_ROWS_PER_WAVE; ++i) {
      const int b = wg * PH_ROWS + wid * PH_ROWS_PER_WAVE + i;
      const int bc = b < p.B ? b : p.B - 1;
      float4 q[4][2];
#pragma unroll
      for (int z = 0; z < 4; ++z)
        if (z < p.hp_planes) {
          const float4* src = reinterpret_cast<const float4*>(p.hp + z * p.hp_stride + (size_t)bc * PH_H + k0);
          q[z][0] = src[0];
          q[z][1] = src[1];
        }
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
      for (int z = 0; z < 4; ++z)
        if (z < p.hp_planes) {
          v[0] += q[z][0].x; v[1] += q[z][0].y; v[2] += q[z][0].z; v[3] += q[z][0].w;
          v[4] += q[z][1].x; v[5] += q[z][1].y; v[6] += q[z][1].z; v[7] += q[z][1].w;
        }
      u16 hb16[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) hb16[e] = f2bf(fmaxf(v[e] * 1.0f + hb[e], 0.f));
      hraw[i].x = hb16[0] | ((uint32_t)hb16[1] << 16);
      hraw[i].y = hb16[2] | ((uint32_t)hb16[3] << 16);
      hraw[i].z = hb16[4] | ((uint32_t)hb16[5] << 16);
      hraw[i].w = hb16[6] | ((uint32_t)hb16[7] << 16);
    }
  }
#pragma unroll
  for (int i = 0; i < PH_ROWS_PER_WAVE; ++i) {
    const int b = wg * PH_ROWS + wid * PH_ROWS_PER_WAVE + i;
    const int bc = b < p.B ? b : p.B - 1;   // clamped: unconditional loads, contributions masked below
    if (!p.hp) hraw[i] = *reinterpret_cast<const uint4*>(p.h + (size_t)bc * PH_H + k0);
    ab[i] = p.act[bc];
    lpo[i] = p.logp_old[bc];
    adv[i] = p.adv[bc];
    R[i] = p.ret[bc];
    vo[i] = (p.v_clip > 0.f && p.v_old) ? p.v_old[bc] : 0.f;
  }
  float accW[8][A1], accB[8], accZ[A1];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    accB[e] = 0.f;
#pragma unroll
    for (int a = 0; a < A1; ++a) accW[e][a] = 0.f;
  }
#pragma unroll
  for (int a = 0; a < A1; ++a) accZ[a] = 0.f;
  double st[PH_NSTAT] = {0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < PH_ROWS_PER_WAVE; ++i) {
    const int b = wg * PH_ROWS + wid * PH_ROWS_PER_WAVE + i;
    const bool live = b < p.B;
    const uint32_t hw[4] = {hraw[i].x, hraw[i].y, hraw[i].z, hraw[i].w};
    float hv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) hv[e] = __uint_as_float((e & 1) ? (hw[e >> 1] & 0xFFFF0000u) : (hw[e >> 1] << 16));
    // z = h . Wh + bh (fp32, wave-reduced: every lane ends with the whole row)
    float z[A1];
#pragma unroll
    for (int a = 0; a < A1; ++a) {
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s += hv[e] * W[e][a];
      z[a] = wave_sum(s) + bias[a];
    }
    if (p.z_out && live && lane < A1) {
#pragma unroll
      for (int a = 0; a < A1; ++a)
        if (a == lane) p.z_out[(size_t)b * A1 + a] = z[a];
    }
    // categorical log-softmax, entropy, log-prob of the taken action
    float mx = -INFINITY;
#pragma unroll
    for (int a = 0; a < A; ++a) mx = fmaxf(mx, z[a]);
    float se = 0.f;
#pragma unroll
    for (int a = 0; a < A; ++a) se += expf(z[a] - mx);
    const float lse = mx + logf(se);
    float H = 0.f, lpa = 0.f;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float lz = z[a] - lse;
      H -= expf(lz) * lz;
      lpa = (a == ab[i]) ? lz : lpa;
    }
    float g_lpa;
    double pg, cf, rt;
    if (p.ppo_clip > 0.f) {
      const float ratio = expf(lpa - lpo[i]);
      const float s1 = ratio * adv[i];
      const float rc = fminf(fmaxf(ratio, 1.0f - p.ppo_clip), 1.0f + p.ppo_clip);
      const float s2 = rc * adv[i];
      pg = -(double)fminf(s1, s2);
      const bool inside = ratio >= 1.0f - p.ppo_clip && ratio <= 1.0f + p.ppo_clip;
      g_lpa = (s1 <= s2 || inside) ? -adv[i] * ratio * invB : 0.f;
      cf = fabsf(ratio - 1.0f) > p.ppo_clip ? 1.0 : 0.0;
      rt = ratio;
    } else {
      pg = -(double)(adv[i] * lpa);
      g_lpa = -adv[i] * invB;
      cf = 0.0;
      rt = 1.0;
    }
    const float dkl = lpo[i] - lpa;
    g_lpa += -2.0f * beta * dkl * invB;
    // critic (column A)
    const float v = z[A];
    float d = v - R[i], vl = d * d, gv = 2.0f * d;
    if (p.v_clip > 0.f && p.v_old) {
      const float vc = vo[i] + fminf(fmaxf(v - vo[i], -p.v_clip), p.v_clip);
      const float dc = vc - R[i];
      if (dc * dc > vl) {
        vl = dc * dc;
        const bool inside = (v - vo[i]) >= -p.v_clip && (v - vo[i]) <= p.v_clip;
        gv = inside ? 2.0f * dc : 0.f;
      }
    }
    float dz[A1];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float lz = z[a] - lse, pa = expf(lz);
      const float oh = (a == ab[i]) ? 1.0f : 0.0f;
      dz[a] = live ? g_lpa * (oh - pa) + c_ent * invB * pa * (lz + H) : 0.f;
    }
    dz[A] = live ? p.vf_coef * gv * invB : 0.f;
    if (live) {
      st[0] += pg;
      st[1] += (double)(dkl * dkl);
      st[2] += H;
      st[3] += vl;
      st[4] += cf;
      st[5] += rt;
    }
    // dh = (h > 0) * dz . Wh^T, and the partial sums of dWh / dbfc / dbh
    u16 dhb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s = 0.f;
#pragma unroll
      for (int a = 0; a < A1; ++a) s += dz[a] * W[e][a];
      s = hv[e] > 0.f ? s : 0.f;
      dhb[e] = f2bf(s);
      accB[e] += s;
#pragma unroll
      for (int a = 0; a < A1; ++a) accW[e][a] += hv[e] * dz[a];
    }
#pragma unroll
    for (int a = 0; a < A1; ++a) accZ[a] += dz[a];
    if (live) {
      uint4 o;
      o.x = dhb[0] | ((uint32_t)dhb[1] << 16);
      o.y = dhb[2] | ((uint32_t)dhb[3] << 16);
      o.z = dhb[4] | ((uint32_t)dhb[5] << 16);
      o.w = dhb[6] | ((uint32_t)dhb[7] << 16);
      *reinterpret_cast<uint4*>(p.dh + (size_t)b * PH_H + k0) = o;
    }
  }
  // ---- per-workgroup planes: waves combined in wave order through LDS
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s_rb[wid][lane * BS + e] = accB[e];
#pragma unroll
    for (int a = 0; a < A1; ++a) s_red[wid][lane * RS + e * A1 + a] = accW[e][a];
  }
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < PH_NSTAT; ++q) s_st[wid][q] = st[q];
#pragma unroll
    for (int a = 0; a < A1; ++a) s_st[wid][PH_NSTAT + a] = accZ[a];
  }
  __syncthreads();
  float* pw = p.pWh + (size_t)wg * PH_H * A1;
  // element j = k A1 + a (k = 8 l + e) sits at l RS + e A1 + a = j + l
  for (int j = tid; j < PH_H * A1; j += PH_THREADS) {
    const int o = j + j / (8 * A1);
    pw[j] = ((s_red[0][o] + s_red[1][o]) + s_red[2][o]) + s_red[3][o];
  }
  for (int j = tid; j < PH_H; j += PH_THREADS) {
    const int o = j + (j >> 3);
    p.pbfc[(size_t)wg * PH_H + j] = ((s_rb[0][o] + s_rb[1][o]) + s_rb[2][o]) + s_rb[3][o];
  }
  if (tid < A1)
    p.pbh[(size_t)wg * A1 + tid] = (float)(((s_st[0][PH_NSTAT + tid] + s_st[1][PH_NSTAT + tid]) +
                                            s_st[2][PH_NSTAT + tid]) + s_st[3][PH_NSTAT + tid]);
  if (tid < PH_NSTAT)
    p.pstats[(size_t)wg * PH_NSTAT + tid] = ((s_st[0][tid] + s_st[1][tid]) + s_st[2][tid]) + s_st[3][tid];
  // ---- statistics: the last workgroup sums the records (fixed order); no ticket: the gradient finaliser that
  // reduces this launch's planes sums them (optim.hip ppo_stats_duty)
  if (!p.ticket) return;
  if (!last_block_arrival(p.ticket, gridDim.x, &sh_flag)) return;
  {
    double t[PH_NSTAT];
    grid_records_sum<PH_NSTAT>(p.pstats, PH_NSTAT, gridDim.x, t, s_sum);
    if (tid == 0)
#pragma unroll
      for (int q = 0; q < PH_NSTAT; ++q) s_st[0][q] = t[q];
  }
  __syncthreads();
  if (tid == 0) {
    const double inv = 1.0 / p.B;
    const double pg = s_st[0][0] * inv, kl = s_st[0][1] * inv, H = s_st[0][2] * inv;
    p.stats[0] = (float)pg;
    p.stats[1] = (float)kl;
    p.stats[2] = (float)H;
    p.stats[3] = (float)(s_st[0][3] * inv);
    p.stats[4] = (float)(s_st[0][4] * inv);
    p.stats[5] = (float)(pg + beta * kl - c_ent * H);
    p.stats[6] = (float)(s_st[0][5] * inv);
  }
}

}  // namespace aca

// grid = ceil(B / 16) workgroups; the plane buffers hold one plane per workgroup (aca_ppo_head_planes).
extern "C" int aca_ppo_head_planes(int B) { return (B + aca::PH_ROWS - 1) / aca::PH_ROWS; }

extern "C" hipError_t aca_ppo_head(const aca::PpoHeadArgs* a, int A1, hipStream_t stream) {
  if (a->B <= 0) return hipSuccess;
  if ((!a->hp && reinterpret_cast<uintptr_t>(a->h) % 16) || reinterpret_cast<uintptr_t>(a->dh) % 16)
    return hipErrorInvalidValue;
  if (a->hp && (reinterpret_cast<uintptr_t>(a->hp) % 16 || a->hp_stride % 4 || a->hp_planes < 1 || a->hp_planes > 4 ||
                !a->hbias))
    return hipErrorInvalidValue;
  const int grid = aca_ppo_head_planes(a->B);
  switch (A1) {
#define ACA_PH(N) \
  case N: aca::ppo_head_kernel<N><<<grid, aca::PH_THREADS, 0, stream>>>(*a); break;
    ACA_PH(3) ACA_PH(4) ACA_PH(5) ACA_PH(6) ACA_PH(7) ACA_PH(8)
#undef ACA_PH
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
