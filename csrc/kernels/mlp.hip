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

// Descriptor words -> pointers. The cast goes through the global address space so the compiler emits global_load /
// global_store: a plain int -> generic pointer cast yields flat_* instructions, which count against lgkmcnt too, so
// every LDS fragment read would also wait for all outstanding weight loads.
typedef const __attribute__((address_space(1))) float gcf32;
typedef __attribute__((address_space(1))) float gf32;
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* P_(int64_t v) {
  return (__attribute__((address_space(1))) T*)v;
}

__device__ __forceinline__ int rup16(int x) { return (x + 15) & ~15; }
// k-groups of a width, rounded up to a power of two: the layer loops are instantiated for NG in {1, 2, 4, 8, 16} so
// they are straight-line code (a runtime group count means a branch per group, and the waitcnt pass then drains
// every group's loads before the next one issues)
__device__ __forceinline__ int ngp2(int w) {
  const int g = (w + 15) >> 4;
  return g <= 1 ? 1 : g <= 2 ? 2 : g <= 4 ? 4 : g <= 8 ? 8 : 16;
}
__device__ __forceinline__ int ld_of(int w) { return 16 * ngp2(w) + 4; }   // padded LDS row stride

// Hidden-layer activations as one branch-free form y = v > 0 ? v : slope * v (relu: slope 0, lrelu(0.2) of
// policies.py:20-21: 0.2, identity: 1); the tanh of the Gaussian head is applied by the head code itself (the
// layer stores the pre-activation z), so the MFMA epilogues carry no per-activation branches.
__device__ __forceinline__ float act_slope(int act) {
  return act == ACT_RELU ? 0.f : act == ACT_LRELU ? 0.2f : 1.f;
}
__device__ __forceinline__ float act_fwd(float v, float slope) { return v > 0.f ? v : slope * v; }
// derivative from the activation OUTPUT y (relu / lrelu / identity keep the sign of x)
__device__ __forceinline__ float act_bwd(float y, float slope) { return y > 0.f ? 1.f : slope; }

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int MLP_MAXG = MLP_MAXW / 16;   // k-groups of the widest layer

// Y[16][N] = act(X[16][K] W[K][N] + b). X: LDS, zero-padded to 16*NG columns (NG = ngp2(K)).
// Y: LDS; every column tile up to ngp2(N) is written, columns >= N as 0 (a valid zero-padded input of the next
// layer). For the tanh head Y holds z (the head code applies tanh and the scale).
// B operand from the transposed shadow Wt[N][16*NG] (zero-padded rows, refreshed after every optimiser step by
// mlp_tshadow_kernel): with the remapped k index a lane's four B values of a k-group are Wt[c][16g+4q .. +3], ONE
// 16-byte load at a constant offset -- all NG loads of a tile are issued before its first MFMA (one L2 round trip
// per tile, 4*NG live registers, no per-k address registers).
template <int NG>
__device__ void layer_fwd_t(const float* __restrict__ X, int ldx, gcf32* __restrict__ Wt, gcf32* __restrict__ bias,
                            int N, int act, float* __restrict__ Y, int ldy) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int ntile = ngp2(N);
  for (int tile = wave; tile < ntile; tile += MLP_THREADS / 64) {
    const int c = tile * 16 + r;
    const bool cok = c < N;
    const int cc = cok ? c : N - 1;   // discarded column: any in-range row
    const __attribute__((address_space(1))) floatx4* wrow =
        (const __attribute__((address_space(1))) floatx4*)(Wt + (size_t)cc * (16 * NG) + 4 * q);
    floatx4 bv[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) bv[g] = wrow[4 * g];
    // keep every load above this point (under register pressure the scheduler would sink each load to its MFMA)
    __builtin_amdgcn_sched_barrier(0);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    // opaque zero tied to the tile: keeps the A-fragment reads inside the tile loop (hoisted, all NG of them would
    // stay live across the loop -- 4*NG more registers for no reuse when a wave owns a single tile)
    const int z0 = __builtin_amdgcn_readfirstlane(tile) - tile;
    const float* Xr = X + r * ldx + 4 * q + z0;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const float4 a4 = *reinterpret_cast<const float4*>(&Xr[16 * g]);
      acc = mfma4(a4.x, bv[g][0], acc);
      acc = mfma4(a4.y, bv[g][1], acc);
      acc = mfma4(a4.z, bv[g][2], acc);
      acc = mfma4(a4.w, bv[g][3], acc);
      // one A-fragment LDS read per 4 MFMAs (not all reads hoisted: that would double the live registers)
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    const float bb = bias[cc];
    const float slope = act_slope(act);
#pragma unroll
    for (int i = 0; i < 4; ++i) Y[(4 * q + i) * ldy + c] = cok ? act_fwd(acc[i] + bb, slope) : 0.f;
  }
}

__device__ __forceinline__ void layer_fwd(const float* X, int ldx, int K, gcf32* Wt, gcf32* bias, int N, int act,
                                          float* Y, int ldy) {
  switch (ngp2(K)) {
    case 1: layer_fwd_t<1>(X, ldx, Wt, bias, N, act, Y, ldy); break;
    case 2: layer_fwd_t<2>(X, ldx, Wt, bias, N, act, Y, ldy); break;
    case 4: layer_fwd_t<4>(X, ldx, Wt, bias, N, act, Y, ldy); break;
    case 8: layer_fwd_t<8>(X, ldx, Wt, bias, N, act, Y, ldy); break;
    default: layer_fwd_t<16>(X, ldx, Wt, bias, N, act, Y, ldy); break;
  }
}

// dX[16][K] = dP[16][N] W[K][N]^T, then * act'(Yprev) (Yprev: LDS outputs of the previous layer, act_prev) ->
// dPprev (LDS; every column tile up to ngp2(K) written, columns >= K as 0) and, when gdst != null, the global rows
// of the previous layer's dP. dP is zero-padded to 16*NG columns (NG = ngp2(N)).
// VEC: N % 16 == 0, each k-group's B fragment is one 16-byte load of a weight row; all groups loaded up front.
template <int NG, bool VEC>
__device__ void layer_dgrad_t(const float* __restrict__ dP, int ldp, int N, gcf32* __restrict__ W, int K,
                              const float* __restrict__ Yprev, int ldyp, int act_prev, float* __restrict__ dPprev,
                              int lddp, gf32* __restrict__ gdst, int rows) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int ntile = ngp2(K);
  for (int tile = wave; tile < ntile; tile += MLP_THREADS / 64) {
    const int kc = tile * 16 + r;   // output column = input feature of the layer
    const bool kok = kc < K;
    gcf32* wrow = W + (size_t)(kok ? kc : 0) * N;
    float4 bv[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int n0 = 16 * g + 4 * q;
      // (kc >= K rows are discarded, n >= N meets a zero-padded dP column: clamped loads, no selects)
      if (VEC) {
        const int nn = N >= 16 * NG ? n0 : min(n0, N - 4);
        const floatx4 w4 = *(const __attribute__((address_space(1))) floatx4*)(wrow + nn);
        bv[g] = make_float4(w4[0], w4[1], w4[2], w4[3]);
      } else {
        bv[g] = make_float4(wrow[min(n0, N - 1)], wrow[min(n0 + 1, N - 1)], wrow[min(n0 + 2, N - 1)],
                            wrow[min(n0 + 3, N - 1)]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const int z0 = __builtin_amdgcn_readfirstlane(tile) - tile;
    const float* Pr = dP + r * ldp + 4 * q + z0;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const float4 a4 = *reinterpret_cast<const float4*>(&Pr[16 * g]);
      acc = mfma4(a4.x, bv[g].x, acc);
      acc = mfma4(a4.y, bv[g].y, acc);
      acc = mfma4(a4.z, bv[g].z, acc);
      acc = mfma4(a4.w, bv[g].w, acc);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    // C layout: col = lane&15 = kc, rows 4q + i
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * q + i;
      float v = 0.f;
      if (kok) v = acc[i] * act_bwd(Yprev[row * ldyp + kc], act_slope(act_prev));
      dPprev[row * lddp + kc] = v;
      if (gdst && kok && row < rows) gdst[(size_t)row * K + kc] = v;
    }
  }
}

__device__ __forceinline__ void layer_dgrad(const float* dP, int ldp, int N, gcf32* W, int K, const float* Yprev,
                                            int ldyp, int act_prev, float* dPprev, int lddp, gf32* gdst, int rows) {
  const bool vec = (N & 15) == 0;
#define ACA_DG(NG_)                                                                                      \
  if (vec) layer_dgrad_t<NG_, true>(dP, ldp, N, W, K, Yprev, ldyp, act_prev, dPprev, lddp, gdst, rows);  \
  else layer_dgrad_t<NG_, false>(dP, ldp, N, W, K, Yprev, ldyp, act_prev, dPprev, lddp, gdst, rows);
  // (non-multiple-of-16 widths above 32 are rejected by the host: ops/mlp.py)
  switch (ngp2(N)) {
    case 1: ACA_DG(1) break;
    case 2: ACA_DG(2) break;
    case 4: layer_dgrad_t<4, true>(dP, ldp, N, W, K, Yprev, ldyp, act_prev, dPprev, lddp, gdst, rows); break;
    case 8: layer_dgrad_t<8, true>(dP, ldp, N, W, K, Yprev, ldyp, act_prev, dPprev, lddp, gdst, rows); break;
    default: layer_dgrad_t<16, true>(dP, ldp, N, W, K, Yprev, ldyp, act_prev, dPprev, lddp, gdst, rows); break;
  }
#undef ACA_DG
}

// rows [0, rows) x [0, w) of an LDS tile (row stride ld, 16-byte aligned rows) -> global rows of w floats. Widths
// that are multiples of 4 go as 16-byte copies with the row index by shift when w / 4 is a power of two (these
// copies sit between two layers of the dependent chain: the scalar form spent ~40 instructions per element on the
// runtime division alone)
__device__ __forceinline__ void rows_out(const float* __restrict__ src, int ld, gf32* __restrict__ dst, int w,
                                         int rows) {
  if ((w & 3) == 0) {
    const int w4 = w >> 2, sh = __builtin_ctz(w4);
    const bool p2 = (w4 & (w4 - 1)) == 0;
    for (int e = threadIdx.x; e < rows * w4; e += MLP_THREADS) {
      const int r = p2 ? e >> sh : e / w4, c4 = e - r * w4;
      const floatx4 v = *reinterpret_cast<const floatx4*>(src + r * ld + 4 * c4);
      *(__attribute__((address_space(1))) floatx4*)(dst + (size_t)r * w + 4 * c4) = v;
    }
  } else {
    for (int e = threadIdx.x; e < rows * w; e += MLP_THREADS) {
      const int r = e / w, c = e - r * w;
      dst[(size_t)r * w + c] = src[r * ld + c];
    }
  }
}

__device__ __forceinline__ int64_t row_key(const MlpArgs& a, int grow) {
  return a.tg[grow] * ((int64_t)1 << a.key_shift) + a.env_ids[grow];
}

constexpr float HALF_LOG_2PI = 0.91893853320467274178f;
constexpr float TWO_PI = 6.28318530717958647692f;

__global__ void __launch_bounds__(MLP_THREADS) mlp_fwd_kernel(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];   // 16-byte base: the b128 LDS reads stay aligned
  __shared__ float s_red[MLP_BM][MLP_MAXA + 8];   // per-row partials: log-std grads + stats
  const int t = blockIdx.y + a.tw_base;
  const MlpTower& T = a.tw[t];
  const int nl = (int)T.nl;
  const int row0 = blockIdx.x * MLP_BM;
  const int rows = min(MLP_BM, a.B - row0);
  // diagnostics: s_memrealtime (100 MHz) at phase ends, thread 0 of workgroup (0, tower) after the barrier; slots 12
  // and 13 hold s_memtime (shader clock) at the ends of the input tile and of the data-gradient chain
  auto stamp = [&](int slot) {
    if (a.stamps && blockIdx.x == 0 && threadIdx.x == 0) a.stamps[blockIdx.y * 16 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  auto cstamp = [&](int slot) {
    if (a.stamps && blockIdx.x == 0 && threadIdx.x == 0) a.stamps[blockIdx.y * 16 + slot] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  // ---- LDS layout: X0 | Y_0 .. Y_{nl-1} | dP ping-pong (train)
  const int ld0 = ld_of(a.D);
  // (offsets recomputed from the descriptor rather than kept in per-layer pointer arrays: a runtime-indexed array
  // of LDS pointers lives in scratch and its loads come back as generic (flat) pointers)
  float* X0 = sm;
  auto ldyf = [&](int l) { return ld_of((int)T.out[l]); };
  auto Yp = [&](int l) {
    int off = MLP_BM * ld0;
    for (int j = 0; j < l; ++j) off += MLP_BM * ldyf(j);
    return sm + off;
  };
  float* P0 = Yp(nl);
  float* P1 = P0 + MLP_BM * (MLP_MAXW + 4);
  // per-layer LDS offsets and strides, computed once (one LDS read per use instead of a chain over the earlier
  // layers' widths read from the descriptor)
  __shared__ int s_yo[MLP_MAXL], s_ld[MLP_MAXL];
  if (threadIdx.x == 64) {
    for (int l = 0; l < nl; ++l) {
      s_yo[l] = (int)(Yp(l) - sm);
      s_ld[l] = ldyf(l);
    }
  }
  // the tower descriptor's per-layer words staged in LDS once: indexed by the runtime layer number they are vector
  // memory loads, and on gfx9 a load issued after the layer's workspace stores waits for those stores (vmcnt counts
  // both, in order) -- each layer paid that before it could even address its weights
  __shared__ int s_in[MLP_MAXL], s_out[MLP_MAXL], s_act[MLP_MAXL];
  __shared__ int64_t s_Wt[MLP_MAXL], s_bb[MLP_MAXL], s_W[MLP_MAXL], s_xs[MLP_MAXL], s_dp[MLP_MAXL];
  if (threadIdx.x >= 96 && threadIdx.x < 96 + nl) {
    const int l = threadIdx.x - 96;
    s_in[l] = (int)T.in[l];
    s_out[l] = (int)T.out[l];
    s_act[l] = (int)T.act[l];
    s_Wt[l] = T.Wt[l];
    s_bb[l] = T.b[l];
    s_W[l] = T.W[l];
    s_xs[l] = T.xs[l];
    s_dp[l] = T.dp[l];
  }
  // ---- row gather: explicit index list, the keyed minibatch permutation (PPO), or identity
  __shared__ int64_t s_grow[MLP_BM];
  if (threadIdx.x < MLP_BM) {
    const int lrow = min(row0 + (int)threadIdx.x, a.B - 1);
    int64_t g = lrow;
    if (a.idx) g = a.idx[lrow];
    else if (a.perm_uc)
      g = prp_index((uint32_t)(a.perm_off + lrow), (uint32_t)a.perm_n,
                    minibatch_key(a.perm_seed, *a.perm_uc, a.perm_ep));
    s_grow[threadIdx.x] = g;
  }
  __syncthreads();
  // ---- train: every layer's weights (forward shadow Wt and, for the data-gradient chain, W) requested at entry, one
  // dword per 128-byte line by LDS-DMA into a dead slot (no registers, nothing waits on it): the optimiser step just
  // rewrote them, so each layer's own loads would otherwise start a cold miss only once the previous layer is done.
  // The tower's workgroups on one XCD (linear id % 8 when the row tiles are a multiple of 8) split the lines.
  // ---- train: the loss head's per-row inputs loaded now, consumed after the forward (issued behind the forward's
  // first weight loads they were a dependent global round trip in the middle of the chain): gaussian-phase thread
  // (r, j) the action component, row thread r the old log-prob and advantage (policy) or return and old value
  // (critic) -- the same threads that read them below
  const bool policy = (t == 0);
  float e_act = 0.f, e_lo = 0.f, e_adv = 0.f, e_ret = 0.f, e_vo = 0.f;
  int e_ai = 0;
  if (a.mode == 2) {
    const int r = threadIdx.x / MLP_MAXA, j = threadIdx.x % MLP_MAXA;
    if (policy && a.head == 2 && threadIdx.x < MLP_BM * MLP_MAXA && j < a.A && r < rows)
      e_act = a.act_f_in[s_grow[r] * a.A + j];
    if (threadIdx.x < rows) {
      const int64_t grow = s_grow[threadIdx.x];
      if (policy) {
        e_lo = a.logp_old[grow];
        e_adv = a.adv[grow];
        if (a.head != 2) e_ai = a.act_i_in[grow];
      } else {
        e_ret = a.ret[grow];
        if (a.v_old && a.v_clip > 0.f) e_vo = a.v_old[grow];
      }
    }
  }
  __shared__ float s_pf[64];
  if (a.mode == 2 && a.prefetch) {
    const bool split = (gridDim.x & 7) == 0;
    const int per = split ? (int)gridDim.x >> 3 : 1, me = split ? (int)blockIdx.x >> 3 : 0;
    const int step = per * MLP_THREADS;
    for (int l = 0; l < nl; ++l) {
      const int K = s_in[l], N = s_out[l];
      for (int rg = (l == 0 ? 0 : -1); rg < 1; ++rg) {   // rg -1: W (row-major, data-gradient), 0: Wt (forward)
        const float* base = reinterpret_cast<const float*>(rg < 0 ? s_W[l] : s_Wt[l]);
        const int n = rg < 0 ? K * N : N * 16 * ngp2(K);
        const int lines = (n + 31) >> 5;
        for (int i = me + per * (int)threadIdx.x; i < lines; i += step)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(base + ((size_t)i << 5)),
                                           (__attribute__((address_space(3))) void*)s_pf, 4, 0, 0);
      }
    }
  }
  stamp(1);
  // ---- input tile (gathered rows; padded rows / columns are zero)
  for (int e = threadIdx.x; e < MLP_BM * ld0; e += MLP_THREADS) {
    const int r = e / ld0, c = e - r * ld0;
    float v = 0.f;
    if (r < rows && c < a.D) v = a.obs[s_grow[r] * a.ld_obs + c];
    X0[e] = v;
    if (a.mode == 2 && r < rows && c < a.D) P_<float>(s_xs[0])[(size_t)(row0 + r) * a.D + c] = v;
  }
  __syncthreads();
  stamp(2);
  cstamp(12);
  // ---- forward
  const float* X = X0;
  int ldx = ld0;
  for (int l = 0; l < nl; ++l) {
    float* Yl = sm + s_yo[l];
    const int ldl = s_ld[l];
    layer_fwd(X, ldx, s_in[l], P_<const float>(s_Wt[l]), P_<const float>(s_bb[l]), s_out[l], s_act[l],
              Yl, ldl);
    __syncthreads();
    stamp(3 + l);
    if (a.mode == 2 && l + 1 < nl)   // inputs of layer l+1 for its weight gradient
      rows_out(Yl, ldl, P_<float>(s_xs[l + 1]) + (size_t)row0 * s_out[l], s_out[l], rows);
    X = Yl;
    ldx = ldl;
  }
  const int L = nl - 1;
  const float* Yo = sm + s_yo[L];
  const int ldo = s_ld[L];
  // ---- heads: one thread per row
  float* dPtop = P0;
  const int ldP = MLP_MAXW + 4;
  if (a.mode == 2) {   // zero the top dP tile (the head writes only valid columns)
    for (int e = threadIdx.x; e < MLP_BM * ldP; e += MLP_THREADS) dPtop[e] = 0.f;
    __syncthreads();
  }
  const int tid = threadIdx.x;
  // Gaussian policy head, phase A: one thread per (row, action component) -- mean, sample (rollout) or given action,
  // the component's log-prob term (a per-row loop of tanh / hash / log / sqrt / cos / exp chains on 16 lanes would
  // idle 7 of 8 waves; the per-row sums below keep the sequential order, so the results do not change)
  __shared__ float s_hl[MLP_BM][MLP_MAXA], s_ht[MLP_BM][MLP_MAXA], s_hd[MLP_BM][MLP_MAXA];
  __shared__ float s_g[MLP_BM];
  const bool gauss = policy && a.head == 2;
  if (gauss) {
    if (tid < MLP_BM * MLP_MAXA) {
      const int r = tid / MLP_MAXA, j = tid % MLP_MAXA;
      if (j < a.A) {
        const bool live = r < rows;
        const int64_t grow = s_grow[r];
        const float ls = fminf(fmaxf(a.log_std[j], -2.5f), 2.5f);
        const float th = tanhf(Yo[r * ldo + j]);
        const float mu = th * a.ac_scale[j];
        float aj;
        if (a.mode == 0) {
          const int64_t key = live ? row_key(a, (int)grow) : 0;
          const float u1 = uniform_open(a.seed, key, 2 * j), u2 = uniform_open(a.seed, key, 2 * j + 1);
          const float eps = sqrtf(-2.0f * logf(u1)) * cosf(TWO_PI * u2);
          aj = mu + expf(ls) * eps;
          if (live) a.act_f_out[grow * a.A + j] = aj;
        } else {
          aj = live ? (a.mode == 2 ? e_act : a.act_f_in[grow * a.A + j]) : mu;
        }
        const float zz = (aj - mu) * expf(-ls);
        s_hl[r][j] = -0.5f * zz * zz - ls - HALF_LOG_2PI;
        s_ht[r][j] = th;
        s_hd[r][j] = aj - mu;
      }
    }
    __syncthreads();
  }
  if (tid < MLP_BM) {
    const int r = tid;
    const bool live = r < rows;
    const int lrow = row0 + r;   // batch-local row (workspace / minibatch order)
    const int64_t grow = s_grow[r];
    float st[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (!policy) {
      const float v = Yo[r * ldo];
      if (live && (a.mode == 0 || a.mode == 1) && a.v_out) a.v_out[grow] = v;
      if (live && a.mode == 2) {
        const float R = e_ret;
        float dv = 2.f * (v - R), l2 = (v - R) * (v - R);
        if (a.v_old && a.v_clip > 0.f) {
          const float vo = e_vo;
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
    } else if (a.head == 2) {   // diagonal Gaussian: per-component terms computed above, fixed-order sums here
      const int A = a.A;
      float lp = 0.f, H = 0.f;
      for (int j = 0; j < A; ++j) {
        lp += s_hl[r][j];
        H += 0.5f + HALF_LOG_2PI + fminf(fmaxf(a.log_std[j], -2.5f), 2.5f);
      }
      if (live && a.mode != 2) {
        if (a.logp_out) a.logp_out[grow] = lp;
        if (a.ent_out) a.ent_out[grow] = H;
      }
      float g = 0.f;
      if (a.mode == 2 && live) {
        const float lo = e_lo, adv = e_adv;
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
      s_g[r] = g;
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
        ai = live ? (a.mode == 2 ? e_ai : a.act_i_in[grow]) : 0;
      }
      const float lpa = z[ai] - lse;
      if (live && a.mode != 2) {
        if (a.logp_out) a.logp_out[grow] = lpa;
        if (a.ent_out) a.ent_out[grow] = H;
      }
      if (a.mode == 2 && live) {
        const float lo = e_lo, adv = e_adv;
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
        for (int o = 8; o > 0; o >>= 1) v += lane_xor(v, o);
        if (r == 0 && (policy ? (k != 3) : (k == 3))) {
          // partial rows: every workgroup owns a row, the weight-gradient kernel sums them in a fixed order
          // (atomics from every workgroup to one 32-byte line serialise in L2, ~12 ns each)
          if (a.mpart) a.mpart[(size_t)blockIdx.x * MPART_W + k] = v * a.inv_B;
          else if (k != 5 && v != 0.f) atomicAdd(&a.mstats[k], v * a.inv_B);
        }
      }
    }
  }
  if (a.mode != 2) return;
  __syncthreads();
  stamp(8);
  if (gauss) {   // phase C: d(loss)/d(pre-tanh mean) and the per-row log-std gradient terms, per component
    if (tid < MLP_BM * MLP_MAXA) {
      const int r = tid / MLP_MAXA, j = tid % MLP_MAXA;
      if (j < a.A) {
        const bool live = r < rows;
        const float raw = a.log_std[j];
        const float ls = fminf(fmaxf(raw, -2.5f), 2.5f);
        const float ivar = expf(-2.f * ls);
        const float d = s_hd[r][j], th = s_ht[r][j], g = s_g[r];
        const float dmu = g * d * ivar;
        dPtop[r * ldP + j] = live ? dmu * a.ac_scale[j] * (1.f - th * th) : 0.f;
        const bool inr = raw >= -2.5f && raw <= 2.5f;
        s_red[r][j] = (live && inr) ? g * (d * d * ivar - 1.f) - (*a.ent_coef) * a.inv_B : 0.f;
      }
    }
    __syncthreads();
  }
  // log-std gradient: column sums over the tile's rows, one atomic per column
  if (policy && a.head == 2 && threadIdx.x < a.A) {
    float s = 0.f;
    for (int r = 0; r < MLP_BM; ++r) s += s_red[r][threadIdx.x];
    if (a.mpart) a.mpart[(size_t)blockIdx.x * MPART_W + 8 + threadIdx.x] = s;
    else atomicAdd(&a.g_log_std[threadIdx.x], s);
  }
  stamp(14);   // head phase C + log-std sums (the data-gradient layers take slots 9 ..)
  // ---- top layer dP: apply the head activation derivative (tanh applied above) and publish
  rows_out(dPtop, ldP, P_<float>(s_dp[L]) + (size_t)row0 * s_out[L], s_out[L], rows);
  // ---- data-gradient chain: dP_l -> dP_{l-1}
  float* cur = P0;
  float* nxt = P1;
  for (int l = L; l >= 1; --l) {
    const int N = s_out[l], K = s_in[l];
    gf32* gdst = P_<float>(s_dp[l - 1]) + (size_t)row0 * K;
    gcf32* W = P_<const float>(s_W[l]);
    layer_dgrad(cur, ldP, N, W, K, sm + s_yo[l - 1], s_ld[l - 1], s_act[l - 1], nxt, ldP, gdst, rows);
    __syncthreads();
    stamp(9 + L - l);
    float* tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  cstamp(13);
  // the prefetch DMA must land before the workgroup's LDS is handed to another workgroup
  if (a.prefetch) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------------------------------------ weight grads

__device__ __forceinline__ float clipsq(float v, float c) {
  if (c > 0.f) v = fminf(fmaxf(v, -c), c);
  return v * v;
}

// One 4-wave workgroup per 16x16 gradient tile: the waves take interleaved 128-row chunks of the batch (all 64
// operand loads of a chunk in flight before its MFMAs), then the four partial tiles are summed through LDS.
constexpr int WG_CHUNK = 32;   // loads per operand per lane per chunk (128 rows)

__global__ void __launch_bounds__(256) mlp_wgrad_kernel(WgradArgs a) {
  __shared__ float red[4][64][5];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (blockIdx.x == gridDim.x - 1) {
    // The bookkeeping workgroup (one past the tiles): the train kernel's partial rows summed in a fixed order
    // (deterministic), the log-std gradient finished and its sum of squares written to its own slot, the loss
    // statistics published, the update counter advanced. Done by a tile workgroup, this chain of dependent global
    // round trips made that workgroup -- and so the launch -- finish last.
    if (wave != 0) return;
    float v[MPART_W];
#pragma unroll
    for (int c = 0; c < MPART_W; ++c) v[c] = 0.f;
    if (a.mpart) {
      for (int row = lane; row < a.mpart_rows; row += 64) {
#pragma unroll
        for (int c = 0; c < MPART_W; ++c) v[c] += a.mpart[(size_t)row * MPART_W + c];
      }
#pragma unroll
      for (int c = 0; c < MPART_W; ++c) v[c] = wave_sum(v[c]);
    }
    float g = 0.f;
    if (a.g_log_std && lane < a.A) {
      if (a.mpart) {
        // the train kernel left its log-std terms in the partial rows only: the gradient is STORED (like every
        // other element of this launch), so the slab needs no zeroing between minibatches
        float part = 0.f;   // v[8 + lane] with compile-time indices (a runtime index would put v in scratch)
#pragma unroll
        for (int j = 0; j < MLP_MAXA; ++j) part = lane == j ? v[8 + j] : part;
        g = part;
        a.g_log_std[lane] = g;
      } else {
        g = a.g_log_std[lane];   // added atomically by the train kernel
      }
    }
    if (a.g_log_std && a.nsplit == 1 && a.parts[0]) {
      const float ss = wave_sum(lane < a.A ? clipsq(g, a.clip[0]) : 0.f);
      if (lane == 0) a.parts[0][a.items[0]] = ss;   // the slot after tower 0's tiles (host-checked < MLP_PARTS)
    }
    if (lane == 0) {
      if (a.mpart)
        for (int k = 0; k < 8; ++k) a.mstats[k] += v[k];
      if (a.stats) {   // publish (and reset) the fused kernel's statistics
        float m[8];
        for (int k = 0; k < 8; ++k) m[k] = a.mstats[k];
        m[5] = m[0] + (*a.kl_coef) * m[1] - (*a.ent_coef) * m[2];
        for (int k = 0; k < 7; ++k) a.stats[k] = m[k];
        for (int k = 0; k < 8; ++k) a.mstats[k] = 0.f;
      }
      // the train kernel (the counter's only reader in this minibatch) has finished: stream order
      if (a.bump) *a.bump += 1;
    }
    return;
  }
  const int split = blockIdx.x % a.nsplit;
  int item = blockIdx.x / a.nsplit;
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
  gcf32* X = P_<const float>(T.xs[l]);
  gcf32* P = P_<const float>(T.dp[l]);
  const int ia = i0 + r, jb = j0 + r;
  const bool iok = ia < K, jok = jb < N;
  const int iac = iok ? ia : 0, jbc = jok ? jb : 0;
  // split ranges are whole 128-row chunks; the workspace is zero-padded to a multiple of 128 rows, so a chunk is
  // always in bounds and its pad rows contribute zero (no selects on loaded values: all 64 loads stay in flight)
  const int per = (((a.B + a.nsplit - 1) / a.nsplit) + 127) & ~127;
  const int rb = split * per, re = min(a.B, rb + per);
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  for (int c0 = rb + wave * 4 * WG_CHUNK; c0 < re; c0 += 16 * WG_CHUNK) {
    float av[WG_CHUNK], bv[WG_CHUNK];
#pragma unroll
    for (int u = 0; u < WG_CHUNK; ++u) {
      const int row = c0 + 16 * (u >> 2) + 4 * q + (u & 3);
      av[u] = X[(size_t)row * K + iac];
      bv[u] = P[(size_t)row * N + jbc];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < WG_CHUNK; ++u) {
      acc = mfma4(av[u], bv[u], acc);
      bsum += bv[u];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][lane][i] = acc[i];
  red[wave][lane][4] = bsum;
  __syncthreads();
  if (wave) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = red[0][lane][i] + red[1][lane][i] + red[2][lane][i] + red[3][lane][i];
  bsum = red[0][lane][4] + red[1][lane][4] + red[2][lane][4] + red[3][lane][4];
  float ss = 0.f;
  const float c = a.clip[t];
  // C: col = lane&15 -> j, rows 4q+i -> i
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ii = i0 + 4 * q + i, jj = j0 + r;
    if (ii < K && jj < N) {
      gf32* dst = P_<float>(T.gW[l]) + (size_t)ii * N + jj;
      if (a.nsplit > 1) atomicAdd((float*)dst, acc[i]);
      else {
        *dst = acc[i];
        ss += clipsq(acc[i], c);
      }
    }
  }
  if (ti == 0) {
    // lanes with equal (lane & 15) hold partial column sums over rows = q (mod 4)
    bsum += lane_xor(bsum, 16);
    bsum += lane_xor(bsum, 32);
    if (q == 0 && jok) {
      if (a.nsplit > 1) atomicAdd((float*)(P_<float>(T.gb[l]) + jb), bsum);
      else {
        P_<float>(T.gb[l])[jb] = bsum;
        ss += clipsq(bsum, c);
      }
    }
  }
  if (a.nsplit == 1 && a.parts[t]) {
    ss = wave_sum(ss);
    if (lane == 0) a.parts[t][local_item] = ss;
    if (local_item == 0) {   // unused slots are zero: the optimiser sums all MLP_PARTS in a fixed order
      const int first = a.items[t] + (t == 0 && a.g_log_std ? 1 : 0);   // (tower 0: the log-std slot is taken)
      for (int k = first + lane; k < MLP_PARTS; k += 64) a.parts[t][k] = 0.f;
    }
  }
}

// Wt[c][k] = W[k][c] (rows padded to 16 * ngp2(K), pad stays zero) for every layer of the launched towers: the
// forward's B operand. One thread per weight element; runs after each optimiser step (and at engine creation).
__global__ void __launch_bounds__(256) mlp_tshadow_kernel(const MlpTower* __restrict__ tw, int ntw, int total) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  for (int t = 0; t < ntw; ++t) {
    const MlpTower& T = tw[t];
    for (int l = 0; l < (int)T.nl; ++l) {
      const int K = (int)T.in[l], N = (int)T.out[l];
      if (e < K * N) {
        const int k = e / N, c = e - k * N;
        P_<float>(T.Wt[l])[(size_t)c * (16 * ngp2(K)) + k] = P_<const float>(T.W[l])[e];
        return;
      }
      e -= K * N;
    }
  }
}

// ------------------------------------------------------------------------------------------------ fused rollout
// mlp_rollout_kernel: the whole T-step rollout of the MuJoCo-shaped linear bank in ONE launch (SURVEY §7.5 item 1,
// "a persistent rollout kernel for the MLP configs"). One workgroup owns 16 envs for all T steps:
//   actor forward (layer_fwd; the transposed weight shadows stay hot in this CU's L2 across steps) -> Gaussian sample /
//   log-prob / entropy (the mode-0 head of mlp_fwd_kernel, same RNG keys) -> env step by 32-lane groups (the
//   arithmetic of env_classic.hip linear_step_kernel, fma contraction off) -> frame-stack push straight into the LDS
//   observation tile of the next step (double-buffered).
// Env state, step counters and episode returns live in LDS for the whole rollout (read once, written back once); the
// observation slab, actions, log-probs, entropies, rewards and done flags stream out. The critic's values of all
// (T+1)*N observations are one batched mlp_fwd launch afterwards (ops/mlp.py), off this serial chain.
constexpr int LIN_OBS = 17, LIN_ACT = 6, LIN_LANES = 32;

__device__ __forceinline__ float lin_row(const float* s, const float* av, const float* sA, const float* sB, int r,
                                         float nz) {
#pragma clang fp contract(off)
  float acc = 0.f, acc2 = 0.f;
  for (int c = 0; c < LIN_OBS; ++c) acc += s[c] * sA[r * LIN_OBS + c];
  for (int c = 0; c < LIN_ACT; ++c) acc2 += av[c] * sB[r * LIN_ACT + c];
  return acc + acc2 + (nz - 0.5f) * 0.02f;
}
__device__ __forceinline__ float lin_asq(const float* av) {
#pragma clang fp contract(off)
  float asq = 0.f;
  for (int j = 0; j < LIN_ACT; ++j) asq += av[j] * av[j];
  return asq;
}
__device__ __forceinline__ float lin_reward(float y8, float asq) {
#pragma clang fp contract(off)
  return y8 - 0.1f * asq;
}
__device__ __forceinline__ float lin_reset(float u) {
#pragma clang fp contract(off)
  return (u - 0.5f) * 0.2f;
}

// Y = act(X W + b) with the transposed weights W[N][ldw] and the bias in LDS (ldw = 16*NG + 4: consecutive output
// columns land 4 banks apart, so a 16-byte fragment read is conflict-free). No global memory at all.
template <int NG>
__device__ void layer_fwd_lds_t(const float* __restrict__ X, int ldx, const float* __restrict__ W, int ldw,
                                const float* __restrict__ bias, int N, int act, float* __restrict__ Y, int ldy,
                                int64_t* dbg) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int ntile = ngp2(N);
  if (dbg && lane == 0) dbg[wave * 8 + 0] = __builtin_amdgcn_s_memtime();
  for (int tile = wave; tile < ntile; tile += MLP_THREADS / 64) {
    const int c = tile * 16 + r;
    const bool cok = c < N;
    const int cc = cok ? c : N - 1;
    const float* wrow = W + cc * ldw + 4 * q;
    floatx4 bv[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) bv[g] = *reinterpret_cast<const floatx4*>(wrow + 16 * g);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* Xr = X + r * ldx + 4 * q;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const float4 a4 = *reinterpret_cast<const float4*>(&Xr[16 * g]);
      acc = mfma4(a4.x, bv[g][0], acc);
      acc = mfma4(a4.y, bv[g][1], acc);
      acc = mfma4(a4.z, bv[g][2], acc);
      acc = mfma4(a4.w, bv[g][3], acc);
    }
    const float bb = bias[cc];
    const float slope = act_slope(act);
    if (dbg && lane == 0) dbg[wave * 8 + 1] = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < 4; ++i) Y[(4 * q + i) * ldy + c] = cok ? act_fwd(acc[i] + bb, slope) : 0.f;
    if (dbg && lane == 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the epilogue's LDS stores (and so the MFMA results) done
      dbg[wave * 8 + 2] = __builtin_amdgcn_s_memtime();
    }
  }
}

__device__ __forceinline__ void layer_fwd_lds(const float* X, int ldx, int K, const float* W, const float* bias, int N,
                                              int act, float* Y, int ldy, int64_t* dbg = nullptr) {
  const int ldw = 16 * ngp2(K) + 4;
  switch (ngp2(K)) {
    case 1: layer_fwd_lds_t<1>(X, ldx, W, ldw, bias, N, act, Y, ldy, dbg); break;
    case 2: layer_fwd_lds_t<2>(X, ldx, W, ldw, bias, N, act, Y, ldy, dbg); break;
    case 4: layer_fwd_lds_t<4>(X, ldx, W, ldw, bias, N, act, Y, ldy, dbg); break;
    case 8: layer_fwd_lds_t<8>(X, ldx, W, ldw, bias, N, act, Y, ldy, dbg); break;
    default: layer_fwd_lds_t<16>(X, ldx, W, ldw, bias, N, act, Y, ldy, dbg); break;
  }
}

// WLDS: the actor's weights and biases are staged in LDS once (the reference actor at D = 17 is ~120 KB, SURVEY
// §2.4 K01), so the step loop issues no global loads at all. That matters beyond the load latency: on gfx9 global
// stores count on vmcnt too, so every wait for a load issued after the previous step's stores (observations,
// actions, rewards) would first drain those stores. The descriptor, head parameters and env ids are staged as well.
// !WLDS (wider frame stacks): weights stream from the L2-resident transposed shadows.
template <bool WLDS>
__global__ void __launch_bounds__(MLP_THREADS) mlp_rollout_kernel(RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];   // 16-byte base: the b128 LDS reads stay aligned
  __shared__ int64_t s_tg[MLP_BM];
  __shared__ int64_t s_ids[MLP_BM];
  __shared__ int s_t[MLP_BM];
  __shared__ float s_er[MLP_BM];
  __shared__ float s_ls[MLP_MAXA], s_sc[MLP_MAXA];
  __shared__ float s_hl[MLP_BM * MLP_MAXA];
  __shared__ int s_in[MLP_MAXL], s_out[MLP_MAXL], s_actc[MLP_MAXL];
  __shared__ int64_t s_wt[MLP_MAXL], s_b[MLP_MAXL];
  const MlpTower& T = a.tw[0];
  const int nl = (int)T.nl;
  const int row0 = blockIdx.x * MLP_BM;
  const int rows = min(MLP_BM, a.N - row0);
  const int tid = threadIdx.x;
  const int A = a.A, D = a.D;
  const int ld0 = ld_of(D);
  if (tid < nl) {
    s_in[tid] = (int)T.in[tid];
    s_out[tid] = (int)T.out[tid];
    s_actc[tid] = (int)T.act[tid];
    s_wt[tid] = T.Wt[tid];
    s_b[tid] = T.b[tid];
  }
  if (tid < MLP_MAXA) {
    s_ls[tid] = tid < A ? fminf(fmaxf(a.log_std[tid], -2.5f), 2.5f) : 0.f;
    s_sc[tid] = tid < A ? a.ac_scale[tid] : 0.f;
  }
  if (tid < MLP_BM) {
    const bool live = tid < rows;
    s_tg[tid] = live ? a.tg[row0 + tid] : 0;
    s_ids[tid] = live ? a.env_ids[row0 + tid] : 0;
    s_t[tid] = live ? a.t[row0 + tid] : 0;
    s_er[tid] = live ? a.ep_ret[row0 + tid] : 0.f;
  }
  __syncthreads();
  // diagnostics: 100 MHz stamps at phase boundaries (workgroup 0, wave 0 after the barrier), steps 0..15
  auto stamp = [&](int step, int slot) {
    if (a.stamps && blockIdx.x == 0 && tid == 0 && step < 16) a.stamps[step * 8 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  auto ldyf = [&](int l) { return ld_of(s_out[l]); };
  auto Yp = [&](int l) {
    int off = 2 * MLP_BM * ld0;
    for (int j = 0; j < l; ++j) off += MLP_BM * ldyf(j);
    return sm + off;
  };
  // LDS: obs tile x2 | Y_0 .. Y_{nl-1} | A | B | env state [16][17] | actions [16][16] | (WLDS) W_l, b_l per layer
  float* sA = Yp(nl);
  float* sB = sA + LIN_OBS * LIN_OBS;
  float* s_state = sB + LIN_OBS * LIN_ACT;
  float* s_act = s_state + MLP_BM * LIN_OBS;
  float* s_w0 = sm + (((s_act - sm) + MLP_BM * MLP_MAXA + 3) & ~3);   // 16-byte aligned (b128 reads)
  auto Wl = [&](int l) {
    float* p = s_w0;
    for (int j = 0; j < l; ++j) p += s_out[j] * (16 * ngp2(s_in[j]) + 4) + 16 * ngp2(s_out[j]);
    return p;
  };
  // per-layer LDS offsets, computed once: in the step loop each is one LDS read instead of a dependent chain of
  // reads over the earlier layers' widths
  __shared__ int s_yo[MLP_MAXL + 1], s_wo[MLP_MAXL];
  if (tid == 0) {
    for (int l = 0; l <= nl; ++l) s_yo[l] = (int)(Yp(l) - sm);
    for (int l = 0; l < nl; ++l) s_wo[l] = (int)(Wl(l) - sm);
  }
  if (WLDS) {   // W_l [out][16*ngp2(in) + 4] (from the zero-padded transposed shadow), then b_l [16*ngp2(out)]
    for (int l = 0; l < nl; ++l) {
      const int K4 = 4 * ngp2(s_in[l]), N = s_out[l], ldw = 16 * ngp2(s_in[l]) + 4;
      float* w = Wl(l);
      const __attribute__((address_space(1))) floatx4* src =
          (const __attribute__((address_space(1))) floatx4*)P_<const float>(s_wt[l]);
      for (int e = tid; e < N * K4; e += MLP_THREADS) {
        const int c = e / K4, k4 = e - c * K4;
        *reinterpret_cast<floatx4*>(w + c * ldw + 4 * k4) = src[e];
      }
      float* b = w + N * ldw;
      gcf32* bsrc = P_<const float>(s_b[l]);
      for (int e = tid; e < 16 * ngp2(N); e += MLP_THREADS) b[e] = e < N ? bsrc[e] : 0.f;
    }
  }
  for (int e = tid; e < 2 * MLP_BM * ld0; e += MLP_THREADS) {   // step-0 tile (+ a zeroed second buffer)
    const int r = e / ld0, c = e - r * ld0;
    float v = 0.f;
    if (r < rows && c < D) v = a.obs[(size_t)(row0 + r) * D + c];
    sm[e] = v;
  }
  for (int j = tid; j < LIN_OBS * LIN_OBS; j += MLP_THREADS) sA[j] = a.lin_A[j];
  for (int j = tid; j < LIN_OBS * LIN_ACT; j += MLP_THREADS) sB[j] = a.lin_B[j];
  for (int e = tid; e < MLP_BM * LIN_OBS; e += MLP_THREADS)
    s_state[e] = e / LIN_OBS < rows ? a.state[(size_t)row0 * LIN_OBS + e] : 0.f;
  for (int e = tid; e < MLP_BM * MLP_MAXA; e += MLP_THREADS) s_act[e] = 0.f;
  __syncthreads();
  // diagnostics only (stamps[255] == 1): the step loop runs the actor layers alone (no head, no env step)
  const bool layers_only = a.stamps && a.stamps[255] == 1;
  for (int step = 0; step < a.T; ++step) {
    float* Xc = sm + (step & 1) * MLP_BM * ld0;
    float* Xn = sm + ((step & 1) ^ 1) * MLP_BM * ld0;
    // ---- actor forward
    const float* X = Xc;
    int ldx = ld0;
    for (int l = 0; l < nl; ++l) {
      float* Yl = sm + s_yo[l];
      const int ldl = ldyf(l);
      if (WLDS) {
        const float* w = sm + s_wo[l];
        // diagnostics: per-wave shader-clock stamps inside layer 1 of step 5 (entry, MFMAs issued, epilogue landed,
        // after the barrier) at stamps[128 + wave * 8 + k]
        int64_t* dbg = (a.stamps && blockIdx.x == 0 && step == 5 && l == 1) ? a.stamps + 128 : nullptr;
        layer_fwd_lds(X, ldx, s_in[l], w, w + s_out[l] * (16 * ngp2(s_in[l]) + 4), s_out[l], s_actc[l], Yl, ldl, dbg);
        if (dbg) {
          __syncthreads();
          if ((threadIdx.x & 63) == 0) dbg[(threadIdx.x >> 6) * 8 + 3] = __builtin_amdgcn_s_memtime();
        }
      } else {
        layer_fwd(X, ldx, s_in[l], P_<const float>(s_wt[l]), P_<const float>(s_b[l]), s_out[l], s_actc[l], Yl, ldl);
      }
      __syncthreads();
      stamp(step, l);
      X = Yl;
      ldx = ldl;
    }
    if (layers_only) {
      stamp(step, 6);
      continue;
    }
    // ---- Gaussian head, one thread per (env, action component): mean, Box-Muller sample and the component's
    // log-prob term in parallel (a serial per-env loop of hash + log/sqrt/cos/tanh/exp chains on 16 lanes would
    // leave 7 of 8 waves idle for most of the step), then fixed-order per-env sums: bit-identical to the
    // one-thread-per-row head of mlp_fwd_kernel mode 0
    if (tid < MLP_BM * MLP_MAXA) {
      const int r = tid / MLP_MAXA, j = tid % MLP_MAXA;
      if (j < A) {
        const bool live = r < rows;
        const float* Yo = X + r * ldx;
        const int64_t key = live ? s_tg[r] * ((int64_t)1 << a.key_shift) + s_ids[r] : 0;
        const float ls = s_ls[j];
        const float mu = tanhf(Yo[j]) * s_sc[j];
        const float u1 = uniform_open(a.policy_seed, key, 2 * j), u2 = uniform_open(a.policy_seed, key, 2 * j + 1);
        const float eps = sqrtf(-2.0f * logf(u1)) * cosf(TWO_PI * u2);
        const float aj = mu + expf(ls) * eps;
        const float zz = (aj - mu) * expf(-ls);
        s_hl[r * MLP_MAXA + j] = -0.5f * zz * zz - ls - HALF_LOG_2PI;
        s_act[r * MLP_MAXA + j] = aj;
        if (live) a.act[((size_t)step * a.N + row0 + r) * A + j] = aj;
      }
    }
    __syncthreads();
    stamp(step, 5);
    if (tid < rows) {
      float lp = 0.f, H = 0.f;
      for (int j = 0; j < A; ++j) {
        lp += s_hl[tid * MLP_MAXA + j];
        H += 0.5f + HALF_LOG_2PI + s_ls[j];
      }
      a.logp[(size_t)step * a.N + row0 + tid] = lp;
      a.ent[(size_t)step * a.N + row0 + tid] = H;
    }
    // ---- env step: 32 lanes per env, lane r < 17 owns state row r (linear_step_kernel)
    {
      const int e = tid / LIN_LANES, r = tid % LIN_LANES;
      const bool active = e < rows;
      const bool owner = active && r == 0;
      bool done = false;
      float ret = 0.f, len = 0.f;
      if (active) {
        const int i = row0 + e;
        float* s = s_state + e * LIN_OBS;
        const int64_t tg = s_tg[e] + 1;
        const uint32_t id = (uint32_t)s_ids[e], st = (uint32_t)tg;
        float av[LIN_ACT];
        for (int j = 0; j < LIN_ACT; ++j) av[j] = fminf(fmaxf(s_act[e * MLP_MAXA + j], -1.0f), 1.0f);
        const float asq = lin_asq(av);
        float y = 0.f;
        if (r < LIN_OBS) y = lin_row(s, av, sA, sB, r, uniform01(a.env_seed, id, st, 300 + r));
        // reward reads row 8 (lane 8 of the group); every lane of the group has read s before lane r rewrites s[r]
        const float y8 = __shfl(y, (tid & 63 & ~(LIN_LANES - 1)) + 8, 64);
        const float rew = lin_reward(y8, asq);
        const int t = s_t[e] + 1;
        const bool trunc = t >= a.max_steps;
        done = trunc;
        const float er = s_er[e] + rew;
        ret = er;
        len = (float)t;
        if (done && r < LIN_OBS) y = lin_reset(uniform01(a.env_seed, id, st, 100 + r));
        if (r < LIN_OBS) {
          s[r] = y;
          const int k = a.k;
          const float* pv = Xc + e * ld0;
          float* xo = Xn + e * ld0;
          float* go = a.obs + ((size_t)(step + 1) * a.N + i) * D;
          for (int f = 0; f < k - 1; ++f) {
            const float v = done ? y : pv[(f + 1) * LIN_OBS + r];
            xo[f * LIN_OBS + r] = v;
            go[f * LIN_OBS + r] = v;
          }
          xo[(k - 1) * LIN_OBS + r] = y;
          go[(k - 1) * LIN_OBS + r] = y;
        }
        if (owner) {
          const size_t o = (size_t)step * a.N + i;
          s_tg[e] = tg;
          a.reward[o] = rew;
          a.done[o] = done;
          a.trunc[o] = trunc;
          s_t[e] = done ? 0 : t;
          s_er[e] = done ? 0.f : er;
        }
      }
      add_ep_stats(a.ep_stats, owner, done, ret, len);
    }
    __syncthreads();
    stamp(step, 6);
  }
  // ---- env bank write-back
  for (int e = tid; e < rows * LIN_OBS; e += MLP_THREADS) a.state[(size_t)row0 * LIN_OBS + e] = s_state[e];
  if (tid < rows) {
    a.tg[row0 + tid] = s_tg[tid];
    a.t[row0 + tid] = s_t[tid];
    a.ep_ret[row0 + tid] = s_er[tid];
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
  if (a->g_log_std && a->parts[0] && a->nsplit == 1 && a->items[0] >= MLP_PARTS) return hipErrorInvalidValue;
  const int total = a->items[0] + (a->ntw > 1 ? a->items[1] : 0);
  // + the bookkeeping workgroup (statistics, log-std gradient, update counter)
  mlp_wgrad_kernel<<<total * a->nsplit + 1, 256, 0, stream>>>(*a);
  return hipGetLastError();
}

extern "C" hipError_t aca_mlp_tshadow(const MlpTower* tw, int ntw, int total, hipStream_t stream) {
  if (total <= 0) return hipSuccess;
  mlp_tshadow_kernel<<<(total + 255) / 256, 256, 0, stream>>>(tw, ntw, total);
  return hipGetLastError();
}

constexpr size_t ROLLOUT_MAX_LDS = 152 * 1024;   // + ~0.5 KB static: within the 160 KB of a CU

extern "C" hipError_t aca_mlp_rollout(const RolloutArgs* a, size_t lds, hipStream_t stream) {
  if (a->N <= 0 || a->T <= 0) return hipSuccess;
  if (!a->tw || a->head != 2 || a->A != LIN_ACT || a->k < 1 || a->D != LIN_OBS * a->k || a->D > MLP_MAXW)
    return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_rollout_kernel<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, ROLLOUT_MAX_LDS) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_rollout_kernel<false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, ROLLOUT_MAX_LDS) != hipSuccess)
      return hipErrorInvalidValue;
    attr = true;
  }
  if (lds > ROLLOUT_MAX_LDS) return hipErrorInvalidValue;
  const dim3 grid((a->N + MLP_BM - 1) / MLP_BM);
  if (a->wlds) mlp_rollout_kernel<true><<<grid, MLP_THREADS, lds, stream>>>(*a);
  else mlp_rollout_kernel<false><<<grid, MLP_THREADS, lds, stream>>>(*a);
  return hipGetLastError();
}
