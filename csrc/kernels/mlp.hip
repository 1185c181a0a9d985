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
//                  gradients, the log-std gradient is reduced per tile.
//                  SPEC > 0 (train launches of the reference towers, actor D -> 128 -> 128 -> 64 -> A and the Basic
//                  critic D -> 256 -> 128 -> 1, D <= 64): the tower's layer sequence is compile-time, so every wave
//                  requests ALL of its weight fragments for the whole forward + data-gradient chain at entry (up to
//                  ~180 registers; 216 / 304 KB per actor / critic workgroup as whole 1 KB wave loads) and the layer
//                  chain then runs out of registers and LDS with no global round trip between layers; one-tile
//                  layers (the head and the value layer) split their k-groups over the waves.
// mlp_wgrad_kernel one wave per 16x16 tile of every dW_l = X_l^T dP_l (+ the bias column sums): the whole batch is
//                  its K dimension, so every gradient element is written exactly once (no atomics, deterministic),
//                  and the wave also emits its sum of squares into a fixed slot -- the global-norm clip of the fused
//                  optimiser needs no separate reduction launch. It also publishes the loss statistics.
//
// Numerics: fp32 end to end (the reference is fp32). GEMM-shaped work runs on the f32-input MFMA
// v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulate; on gfx950 it runs at the f32 vector rate with 4x the
// operand reuse of a VALU FMA tile). Fragment maps (cdna_hip_programming.md §3): A[l&15][k=l>>4], B[k=l>>4][l&15],
// C/D col = l&15, row = 4(l>>4)+i. The k index of a 16-wide k-group is remapped k = 16g + 4(l>>4) + s for the four
// MFMAs s = 0..3, so each lane's A fragments for a k-group are one 16-byte LDS read and its B fragments 16 bytes of
// a FRAGMENT copy of the weight (common.h mlp_frag_f / mlp_frag_g: a wave's k-group is one contiguous 1 KB block),
// rewritten by the optimiser step itself (optim.hip OptTrans ldt -3 / -4). Weights are [in][out] = TF dense layout
// in the parameter slab; the fragment copies are the only form the kernels read.
#include <type_traits>

#include "common.h"
#include "mlp_desc.h"

namespace aca {

constexpr int MLP_BM = 16;          // rows per workgroup
constexpr int MLP_THREADS = 512;    // 8 waves
constexpr int MLP_WAVES = MLP_THREADS / 64;
constexpr int MLP_MAXW = 256;       // widest layer
constexpr int MLP_MAXA = 16;        // widest head
constexpr int MLP_PARTS = 256;      // sumsq partial slots per tower (= optim.hip SUMSQ_PARTS)

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2, ACT_TANH = 3 };

// Descriptor words -> pointers. The cast goes through the global address space so the compiler emits global_load /
// global_store: a plain int -> generic pointer cast yields flat_* instructions, which count against lgkmcnt too, so
// every LDS fragment read would also wait for all outstanding weight loads.
typedef const __attribute__((address_space(1))) float gcf32;
typedef __attribute__((address_space(1))) float gf32;
typedef const __attribute__((address_space(1))) floatx4 gcfx4;
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* P_(int64_t v) {
  return (__attribute__((address_space(1))) T*)v;
}

__device__ __forceinline__ int rup16(int x) { return (x + 15) & ~15; }
// k-groups of a width, rounded up to a power of two: the layer loops are instantiated for NG in {1, 2, 4, 8, 16} so
// they are straight-line code (a runtime group count means a branch per group, and the waitcnt pass then drains
// every group's loads before the next one issues)
__device__ __forceinline__ int ngp2(int w) { return mlp_ngp2(w); }
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
// B operand from the forward fragment copy F: a lane's four B values of k-group g are 16 bytes, the wave's group one
// contiguous 1 KB block -- all NG loads of a tile are issued before its first MFMA (one L2 round trip per tile).
template <int NG>
__device__ void layer_fwd_t(const float* __restrict__ X, int ldx, gcf32* __restrict__ F, gcf32* __restrict__ bias,
                            int N, int act, float* __restrict__ Y, int ldy) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int ntile = ngp2(N);
  for (int tile = wave; tile < ntile; tile += MLP_WAVES) {
    const int c = tile * 16 + r;
    const bool cok = c < N;
    const int cc = cok ? c : N - 1;   // discarded column: any in-range bias
    gcfx4* wf = (gcfx4*)(F + ((size_t)tile * NG * 64 + lane) * 4);
    floatx4 bv[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) bv[g] = wf[64 * g];
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

__device__ __forceinline__ void layer_fwd(const float* X, int ldx, int K, gcf32* F, gcf32* bias, int N, int act,
                                          float* Y, int ldy) {
  switch (ngp2(K)) {
    case 1: layer_fwd_t<1>(X, ldx, F, bias, N, act, Y, ldy); break;
    case 2: layer_fwd_t<2>(X, ldx, F, bias, N, act, Y, ldy); break;
    case 4: layer_fwd_t<4>(X, ldx, F, bias, N, act, Y, ldy); break;
    case 8: layer_fwd_t<8>(X, ldx, F, bias, N, act, Y, ldy); break;
    default: layer_fwd_t<16>(X, ldx, F, bias, N, act, Y, ldy); break;
  }
}

// dX[16][K] = dP[16][N] W[K][N]^T, then * act'(Yprev) (Yprev: LDS outputs of the previous layer, act_prev) ->
// dPprev (LDS; every column tile up to ngp2(K) written, columns >= K as 0) and, when gdst != null, the row tile's
// blocks of the previous layer's dP in the training workspace (blk_out layout). dP is zero-padded to 16*NG columns (NG = ngp2(N)); B operand from the data-gradient
// fragment copy G (zero pad, so no clamped loads).
template <int NG>
__device__ void layer_dgrad_t(const float* __restrict__ dP, int ldp, gcf32* __restrict__ G, int K,
                              const float* __restrict__ Yprev, int ldyp, int act_prev, float* __restrict__ dPprev,
                              int lddp, gf32* __restrict__ gdst, int rows) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int ntile = ngp2(K);
  for (int tile = wave; tile < ntile; tile += MLP_WAVES) {
    const int kc = tile * 16 + r;   // output column = input feature of the layer
    const bool kok = kc < K;
    gcfx4* wg = (gcfx4*)(G + ((size_t)tile * NG * 64 + lane) * 4);
    floatx4 bv[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) bv[g] = wg[64 * g];
    __builtin_amdgcn_sched_barrier(0);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const int z0 = __builtin_amdgcn_readfirstlane(tile) - tile;
    const float* Pr = dP + r * ldp + 4 * q + z0;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const float4 a4 = *reinterpret_cast<const float4*>(&Pr[16 * g]);
      acc = mfma4(a4.x, bv[g][0], acc);
      acc = mfma4(a4.y, bv[g][1], acc);
      acc = mfma4(a4.z, bv[g][2], acc);
      acc = mfma4(a4.w, bv[g][3], acc);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    // C layout: col = lane&15 = kc, rows 4q + i -- in the workspace's block layout one 16-byte store per lane
    floatx4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * q + i;
      float v = 0.f;
      if (kok) v = acc[i] * act_bwd(Yprev[row * ldyp + kc], act_slope(act_prev));
      dPprev[row * lddp + kc] = v;
      o[i] = v;
    }
    if (gdst && kok) *(__attribute__((address_space(1))) floatx4*)(gdst + tile * 256 + r * 16 + 4 * q) = o;
  }
}

__device__ __forceinline__ void layer_dgrad(const float* dP, int ldp, int N, gcf32* G, int K, const float* Yprev,
                                            int ldyp, int act_prev, float* dPprev, int lddp, gf32* gdst, int rows) {
  switch (ngp2(N)) {
    case 1: layer_dgrad_t<1>(dP, ldp, G, K, Yprev, ldyp, act_prev, dPprev, lddp, gdst, rows); break;
    case 2: layer_dgrad_t<2>(dP, ldp, G, K, Yprev, ldyp, act_prev, dPprev, lddp, gdst, rows); break;
    case 4: layer_dgrad_t<4>(dP, ldp, G, K, Yprev, ldyp, act_prev, dPprev, lddp, gdst, rows); break;
    case 8: layer_dgrad_t<8>(dP, ldp, G, K, Yprev, ldyp, act_prev, dPprev, lddp, gdst, rows); break;
    default: layer_dgrad_t<16>(dP, ldp, G, K, Yprev, ldyp, act_prev, dPprev, lddp, gdst, rows); break;
  }
}

// ---- SPEC path: one wave's register share of a layer (tiles wave, wave + 8, ... < NT; NG k-groups each) and, for
// forward layers, the bias of the lane's output column per tile. Loaded at kernel entry, consumed by the layer.
template <int NG, int NT>
struct WSet {
  static constexpr int NS = (NT + MLP_WAVES - 1) / MLP_WAVES;
  floatx4 w[NS][NG];
  float b[NS];
};

// Every wave issues the same loads (a wave without a tile of a narrow layer re-reads the last tile): the waitcnt pass
// merges the two sides of a wave-dependent branch conservatively, so a skipped load on one side would make every
// later wait of the loaded side count too few outstanding loads.
template <int NG, int NT, bool BIAS>
__device__ __forceinline__ void wset_load(WSet<NG, NT>& R, int64_t frag, int64_t bias, int N, int wave, int lane) {
#pragma unroll
  for (int s = 0; s < WSet<NG, NT>::NS; ++s) {
    const int tile = min(wave + MLP_WAVES * s, NT - 1);
    if (BIAS) {
      const int c = tile * 16 + (lane & 15);
      R.b[s] = P_<const float>(bias)[c < N ? c : N - 1];
    }
    gcfx4* p = (gcfx4*)(P_<const float>(frag) + ((size_t)tile * NG * 64 + lane) * 4);
#pragma unroll
    for (int g = 0; g < NG; ++g) R.w[s][g] = p[64 * g];
  }
}

// one (tile slot s, k-group g) fragment of a WSet (wset_load's addressing, no bias)
template <int NG, int NT>
__device__ __forceinline__ void wset_load_one(WSet<NG, NT>& R, int64_t frag, int s, int g, int wave, int lane) {
  const int tile = min(wave + MLP_WAVES * s, NT - 1);
  R.w[s][g] = *((gcfx4*)(P_<const float>(frag) + ((size_t)tile * NG * 64 + lane) * 4) + 64 * g);
}

// forward layer from registers: the A fragment of a k-group (X rows) is shared by the wave's tiles
template <int NG, int NT>
__device__ __forceinline__ void wset_fwd(const WSet<NG, NT>& R, const float* __restrict__ X, int ldx, int N,
                                         float slope, float* __restrict__ Y, int ldy, int wave, int lane) {
  constexpr int NS = WSet<NG, NT>::NS;
  const int r = lane & 15, q = lane >> 4;
  if (!(NT % MLP_WAVES == 0 || wave < NT)) return;
  floatx4 acc[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) acc[s] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float* Xr = X + r * ldx + 4 * q;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const float4 a4 = *reinterpret_cast<const float4*>(&Xr[16 * g]);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (NT % MLP_WAVES == 0 || wave + MLP_WAVES * s < NT) {
        acc[s] = mfma4(a4.x, R.w[s][g][0], acc[s]);
        acc[s] = mfma4(a4.y, R.w[s][g][1], acc[s]);
        acc[s] = mfma4(a4.z, R.w[s][g][2], acc[s]);
        acc[s] = mfma4(a4.w, R.w[s][g][3], acc[s]);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (NT % MLP_WAVES == 0 || wave + MLP_WAVES * s < NT) {
      const int c = (wave + MLP_WAVES * s) * 16 + r;
      const bool cok = c < N;
#pragma unroll
      for (int i = 0; i < 4; ++i) Y[(4 * q + i) * ldy + c] = cok ? act_fwd(acc[s][i] + R.b[s], slope) : 0.f;
    }
  }
}

// wset_fwd (one tile per wave) that also issues one fragment load of a LATER layer after each k-group's MFMAs:
// side(g). The later layer's weight stream then goes out under this layer's MFMAs instead of ahead of the first
// layer (in-order issue: a wave cannot reach its first MFMA before every load ahead of it has been issued, and the
// CU's address path takes a 1 KB wave load per ~16 clocks).
template <int NG, int NT, class Side>
__device__ __forceinline__ void wset_fwd_side(const WSet<NG, NT>& R, const float* __restrict__ X, int ldx, int N,
                                              float slope, float* __restrict__ Y, int ldy, int wave, int lane,
                                              Side side) {
  static_assert(WSet<NG, NT>::NS == 1 && NT == MLP_WAVES, "one tile per wave");
  const int r = lane & 15, q = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* Xr = X + r * ldx + 4 * q;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const float4 a4 = *reinterpret_cast<const float4*>(&Xr[16 * g]);
    acc = mfma4(a4.x, R.w[0][g][0], acc);
    acc = mfma4(a4.y, R.w[0][g][1], acc);
    acc = mfma4(a4.z, R.w[0][g][2], acc);
    acc = mfma4(a4.w, R.w[0][g][3], acc);
    side(g);
  }
  const int c = wave * 16 + r;
  const bool cok = c < N;
#pragma unroll
  for (int i = 0; i < 4; ++i) Y[(4 * q + i) * ldy + c] = cok ? act_fwd(acc[i] + R.b[0], slope) : 0.f;
}

// wset_fwd with the A operands (rows of the layer input) already in registers: xa[g] = the lane's four k values of
// group g (lane (r, q): row r, columns 16 g + 4 q .. + 3)
template <int NG, int NT>
__device__ __forceinline__ void wset_fwd_rega(const WSet<NG, NT>& R, const float (&xa)[NG][4], int N, float slope,
                                              float* __restrict__ Y, int ldy, int wave, int lane) {
  constexpr int NS = WSet<NG, NT>::NS;
  const int r = lane & 15, q = lane >> 4;
  if (!(NT % MLP_WAVES == 0 || wave < NT)) return;
  floatx4 acc[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) acc[s] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < NG; ++g) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (NT % MLP_WAVES == 0 || wave + MLP_WAVES * s < NT) {
        acc[s] = mfma4(xa[g][0], R.w[s][g][0], acc[s]);
        acc[s] = mfma4(xa[g][1], R.w[s][g][1], acc[s]);
        acc[s] = mfma4(xa[g][2], R.w[s][g][2], acc[s]);
        acc[s] = mfma4(xa[g][3], R.w[s][g][3], acc[s]);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (NT % MLP_WAVES == 0 || wave + MLP_WAVES * s < NT) {
      const int c = (wave + MLP_WAVES * s) * 16 + r;
      const bool cok = c < N;
#pragma unroll
      for (int i = 0; i < 4; ++i) Y[(4 * q + i) * ldy + c] = cok ? act_fwd(acc[s][i] + R.b[s], slope) : 0.f;
    }
  }
}

// data-gradient layer from registers (G fragments: tiles over K, k-groups over N)
template <int NG, int NT>
__device__ __forceinline__ void wset_dgrad(const WSet<NG, NT>& R, const float* __restrict__ dP, int ldp, int K,
                                           const float* __restrict__ Yprev, int ldyp, float slope_prev,
                                           float* __restrict__ dPprev, int lddp, gf32* __restrict__ gdst, int rows,
                                           int wave, int lane) {
  constexpr int NS = WSet<NG, NT>::NS;
  const int r = lane & 15, q = lane >> 4;
  if (!(NT % MLP_WAVES == 0 || wave < NT)) return;
  floatx4 acc[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) acc[s] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float* Pr = dP + r * ldp + 4 * q;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const float4 a4 = *reinterpret_cast<const float4*>(&Pr[16 * g]);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (NT % MLP_WAVES == 0 || wave + MLP_WAVES * s < NT) {
        acc[s] = mfma4(a4.x, R.w[s][g][0], acc[s]);
        acc[s] = mfma4(a4.y, R.w[s][g][1], acc[s]);
        acc[s] = mfma4(a4.z, R.w[s][g][2], acc[s]);
        acc[s] = mfma4(a4.w, R.w[s][g][3], acc[s]);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (NT % MLP_WAVES == 0 || wave + MLP_WAVES * s < NT) {
      const int kc = (wave + MLP_WAVES * s) * 16 + r;
      const bool kok = kc < K;
      floatx4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 4 * q + i;
        const float v = kok ? acc[s][i] * act_bwd(Yprev[row * ldyp + kc], slope_prev) : 0.f;
        dPprev[row * lddp + kc] = v;
        o[i] = v;
      }
      if (kok) *(__attribute__((address_space(1))) floatx4*)(gdst + (wave + MLP_WAVES * s) * 256 + r * 16 + 4 * q) = o;
    }
  }
}

// One-tile forward layer (the policy head 64 -> A, the value layer 128 -> 1) with its NG k-groups split over the
// first NG waves (4 MFMAs each instead of one wave's 4 * NG dependent MFMAs), the partial tiles summed in a fixed
// order through `scratch` (NG * 256 floats of LDS). Contains one workgroup barrier.
template <int NG>
struct WHead {
  floatx4 w;
  float b;
};
template <int NG>
__device__ __forceinline__ void whead_load(WHead<NG>& R, int64_t frag, int64_t bias, int N, int wave, int lane,
                                           int tid) {
  R.w = *((gcfx4*)P_<const float>(frag) + min(wave, NG - 1) * 64 + lane);   // (same loads on every wave, above)
  const int c = tid & 15;
  R.b = P_<const float>(bias)[c < N ? c : N - 1];
}
template <int NG>
__device__ __forceinline__ void whead_fwd(const WHead<NG>& R, const float* __restrict__ X, int ldx, int N,
                                          float slope, float* __restrict__ Y, int ldy, float* __restrict__ scratch,
                                          int wave, int lane, int tid) {
  static_assert(NG <= MLP_WAVES, "one k-group per wave");
  if (wave < NG) {
    const int r = lane & 15, q = lane >> 4;
    const float4 a4 = *reinterpret_cast<const float4*>(&X[r * ldx + 16 * wave + 4 * q]);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = mfma4(a4.x, R.w[0], acc);
    acc = mfma4(a4.y, R.w[1], acc);
    acc = mfma4(a4.z, R.w[2], acc);
    acc = mfma4(a4.w, R.w[3], acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) scratch[wave * 256 + (4 * q + i) * 16 + r] = acc[i];
  }
  __syncthreads();
  if (tid < 256) {
    const int row = tid >> 4, c = tid & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NG; ++w) v += scratch[w * 256 + tid];
    Y[row * ldy + c] = c < N ? act_fwd(v + R.b, slope) : 0.f;
  }
}

// Training workspace layout (xs: layer inputs X_l, dp: pre-activation gradients dP_l, written by the train kernel):
// 16 x 16 BLOCKS, column-major inside -- element (row, col) of a [B][w] array at
//   ((row / 16) * ceil(w / 16) + col / 16) * 256 + (col % 16) * 16 + row % 16
// so the weight-gradient MFMA's operand for column c and rows 4q .. 4q + 3 of a row tile is one 16-byte load and a
// wave's 16 x 16 block one contiguous 1 KB read (row-major, each wave load was 4 rows x 64 B and one float per lane).

// LDS tile rows [0, 16) x [0, w) (row stride ld) -> the row tile's blocks at dst (rows past the batch are written
// too: their dP is zero, so their X -- finite -- adds nothing)
__device__ __forceinline__ void blk_out(const float* __restrict__ src, int ld, gf32* __restrict__ dst, int w) {
  const int nct = (w + 15) >> 4;
  for (int e = threadIdx.x; e < nct * 64; e += MLP_THREADS) {
    const int ct = e >> 6, c = (e >> 2) & 15, r4 = e & 3;
    const int col = ct * 16 + c;
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (col < w) {
#pragma unroll
      for (int s = 0; s < 4; ++s) v[s] = src[(4 * r4 + s) * ld + col];
    }
    *(__attribute__((address_space(1))) floatx4*)(dst + ct * 256 + c * 16 + 4 * r4) = v;
  }
}

// blk_out with at most NCT column tiles: straight-line (predicated) stores, so the waitcnt pass can count them
// (a store loop between the SPEC weight loads and their MFMAs makes it drain the whole weight stream)
template <int NCT>
__device__ __forceinline__ void blk_out_c(const float* __restrict__ src, int ld, gf32* __restrict__ dst, int w) {
  const int nct = (w + 15) >> 4;
#pragma unroll
  for (int j = 0; j < (NCT * 64 + MLP_THREADS - 1) / MLP_THREADS; ++j) {
    const int e = threadIdx.x + MLP_THREADS * j;
    if (e < nct * 64) {
      const int ct = e >> 6, c = (e >> 2) & 15, r4 = e & 3;
      const int col = ct * 16 + c;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (col < w) {
#pragma unroll
        for (int s = 0; s < 4; ++s) v[s] = src[(4 * r4 + s) * ld + col];
      }
      *(__attribute__((address_space(1))) floatx4*)(dst + ct * 256 + c * 16 + 4 * r4) = v;
    }
  }
}

__device__ __forceinline__ int64_t row_key(const MlpArgs& a, int grow) {
  return a.tg[grow] * ((int64_t)1 << a.key_shift) + a.env_ids[grow];
}

constexpr float HALF_LOG_2PI = 0.91893853320467274178f;
constexpr float TWO_PI = 6.28318530717958647692f;

// static LDS of the fused kernel
struct MlpShared {
  float red[MLP_BM][MLP_MAXA + 8];   // per-row partials: log-std grads
  int yo[MLP_MAXL], ld[MLP_MAXL];     // per-layer LDS offsets / strides
  int in[MLP_MAXL], out[MLP_MAXL], act[MLP_MAXL];
  int64_t F[MLP_MAXL], b[MLP_MAXL], G[MLP_MAXL], xs[MLP_MAXL], dp[MLP_MAXL];
  int64_t grow[MLP_BM];
  float hl[MLP_BM][MLP_MAXA], ht[MLP_BM][MLP_MAXA], hd[MLP_BM][MLP_MAXA];
  float g[MLP_BM];
  float hls[MLP_MAXA], hsc[MLP_MAXA], hco[2];   // head parameters: raw log-std, action scale, kl / entropy coefs
  int64_t ts[16];                               // SPEC diagnostics stamps
  float er[5][MLP_BM];                          // SPEC: the loss head's row inputs (log-prob, adv, ret, v, action)
};

// SPEC register sets of the reference towers (NG0 = k-groups of the observation width)
template <int NG0>
struct ActorRegs {   // D -> 128 -> 128 -> 64 -> A
  WSet<NG0, 8> f0;
  WSet<8, 8> f1;
  WSet<8, 4> f2;
  WHead<4> f3;
  WSet<1, 4> g3;     // W3 [64][A]: tiles over 64, one k-group over A
  WSet<4, 8> g2;     // W2 [128][64]
  WSet<8, 8> g1;     // W1 [128][128]
};
template <int NG0>
struct CriticRegs {  // D -> 256 -> 128 -> 1
  WSet<NG0, 16> f0;
  WSet<16, 8> f1;
  WHead<8> f2;
  WSet<1, 8> g2;     // W2 [128][1]
  WSet<8, 16> g1;    // W1 [256][128]
};

// (the scheduling barriers pin the issue order to the use order: the waitcnt pass merges the two load sites of
// mlp_tower conservatively, so they must issue every layer's loads in the same order)
template <int NG0>
__device__ __forceinline__ void spec_load(ActorRegs<NG0>& R, const MlpTower& T, int wave, int lane, int tid) {
  __builtin_amdgcn_sched_barrier(0);
  wset_load<NG0, 8, true>(R.f0, T.F[0], T.b[0], (int)T.out[0], wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  wset_load<8, 8, true>(R.f1, T.F[1], T.b[1], (int)T.out[1], wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  wset_load<8, 4, true>(R.f2, T.F[2], T.b[2], (int)T.out[2], wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  whead_load<4>(R.f3, T.F[3], T.b[3], (int)T.out[3], wave, lane, tid);
  __builtin_amdgcn_sched_barrier(0);
  wset_load<1, 4, false>(R.g3, T.G[3], 0, 0, wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  wset_load<4, 8, false>(R.g2, T.G[2], 0, 0, wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  // (g1, W1's data-gradient set: issued under layer 1's MFMAs, wset_fwd_side)
}
template <int NG0>
__device__ __forceinline__ void spec_load(CriticRegs<NG0>& R, const MlpTower& T, int wave, int lane, int tid) {
  __builtin_amdgcn_sched_barrier(0);
  wset_load<NG0, 16, true>(R.f0, T.F[0], T.b[0], (int)T.out[0], wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  wset_load<16, 8, true>(R.f1, T.F[1], T.b[1], (int)T.out[1], wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  whead_load<8>(R.f2, T.F[2], T.b[2], (int)T.out[2], wave, lane, tid);
  __builtin_amdgcn_sched_barrier(0);
  wset_load<1, 8, false>(R.g2, T.G[2], 0, 0, wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  // (g1, W1's data-gradient set: issued under layer 1's MFMAs, wset_fwd_side)
}

// one tower of mlp_fwd_kernel. SPEC 0: any tower (t at run time, layer loops over the device descriptor); SPEC > 0:
// tower TW of the reference shapes in train mode, weights from registers.
template <int SPEC, int TW>
__device__ __forceinline__ void mlp_tower(const MlpArgs& a, const int t, float* sm, MlpShared& S) {
  constexpr bool SP = SPEC > 0;
  using Regs = typename std::conditional<TW == 0, ActorRegs<SP ? SPEC : 1>, CriticRegs<SP ? SPEC : 1>>::type;
  const MlpTower& T = a.tw[t];
  const int nl = SP ? (TW == 0 ? 4 : 3) : (int)T.nl;
  const int row0 = blockIdx.x * MLP_BM;
  const int rows = min(MLP_BM, a.B - row0);
  // (the wave index through readfirstlane: the compiler then knows it is uniform, so `wave`-dependent branches are
  // scalar branches with exclusive sides, not two exec-masked blocks run one after the other -- the waitcnt pass would
  // otherwise see both sides' weight loads in sequence and drain the stream at the first MFMA)
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  // diagnostics: s_memrealtime (100 MHz) at phase ends, thread 0 of workgroup (0, tower) after the barrier; slots 12
  // and 13 hold s_memtime (shader clock) at the ends of the input tile and of the data-gradient chain
  // (SPEC: kept in LDS and stored at the end -- a global store between the weight loads and their MFMAs makes the
  // waitcnt pass drain the weight stream)
  auto stamp = [&](int slot) {
    if (a.stamps && blockIdx.x == 0 && tid == 0) {
      if (SP) S.ts[slot] = __builtin_amdgcn_s_memrealtime();
      else a.stamps[blockIdx.y * 16 + slot] = __builtin_amdgcn_s_memrealtime();
    }
  };
  auto cstamp = [&](int slot) {
    if (a.stamps && blockIdx.x == 0 && tid == 0) {
      if (SP) S.ts[slot] = __builtin_amdgcn_s_memtime();
      else a.stamps[blockIdx.y * 16 + slot] = __builtin_amdgcn_s_memtime();
    }
  };
  if (SP && a.stamps && blockIdx.x == 0 && tid < 16) S.ts[tid] = 0;
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
  // per-layer LDS offsets and strides, computed once (one LDS read per use instead of a chain over the earlier
  // layers' widths read from the descriptor); SPEC: compile-time (the reference widths; A <= 16, D <= 16 * SPEC)
  constexpr int SLD[2][4] = {{132, 132, 68, 20}, {260, 132, 20, 20}};
  auto LDY = [&](int l) { return SP ? SLD[TW == 0 ? 0 : 1][l] : S.ld[l]; };
  auto YO = [&](int l) {
    if (!SP) return S.yo[l];
    int o = MLP_BM * (16 * (SP ? SPEC : 1) + 4);
    for (int j = 0; j < l; ++j) o += MLP_BM * SLD[TW == 0 ? 0 : 1][j];
    return o;
  };
  // descriptor words: SPEC from the kernel-argument copy (compile-time layer indices: scalar loads), else LDS-staged
  auto INW = [&](int l) { return SP ? (int)a.htw[TW == 0 ? 0 : 1].in[l] : S.in[l]; };
  auto OUTW = [&](int l) { return SP ? (int)a.htw[TW == 0 ? 0 : 1].out[l] : S.out[l]; };
  auto ACT = [&](int l) { return SP ? (int)a.htw[TW == 0 ? 0 : 1].act[l] : S.act[l]; };
  auto XS = [&](int l) { return SP ? a.htw[TW == 0 ? 0 : 1].xs[l] : S.xs[l]; };
  auto DPW = [&](int l) { return SP ? a.htw[TW == 0 ? 0 : 1].dp[l] : S.dp[l]; };
  if (!SP && tid == 64) {
    for (int l = 0; l < nl; ++l) {
      S.yo[l] = (int)(Yp(l) - sm);
      S.ld[l] = ldyf(l);
    }
  }
  // the tower descriptor's per-layer words staged in LDS once: indexed by the runtime layer number they are vector
  // memory loads, and on gfx9 a load issued after the layer's workspace stores waits for those stores (vmcnt counts
  // both, in order) -- each layer paid that before it could even address its weights
  // head parameters (log-std, action scale, regulariser coefficients) staged in LDS: the head reads them inside
  // the dependent chain (SPEC: wave 0 loads them below, ahead of its weights)
  auto head_params = [&](int i) {   // i in [0, 18): 16 components + the two coefficients
    float v = 0.f;
    if (i < MLP_MAXA) {
      if (a.log_std && i < a.A) v = a.log_std[i];
    } else if (i < 2 * MLP_MAXA) {
      if (a.ac_scale && i - MLP_MAXA < a.A) v = a.ac_scale[i - MLP_MAXA];
    } else if (i == 2 * MLP_MAXA) {
      if (a.kl_coef) v = *a.kl_coef;
    } else if (i == 2 * MLP_MAXA + 1) {
      if (a.ent_coef) v = *a.ent_coef;
    }
    return v;
  };
  auto head_params_store = [&](int i, float v) {
    if (i < MLP_MAXA) S.hls[i] = v;
    else if (i < 2 * MLP_MAXA) S.hsc[i - MLP_MAXA] = v;
    else if (i < 2 * MLP_MAXA + 2) S.hco[i - 2 * MLP_MAXA] = v;
  };
  if (!SP && tid >= 128 && tid < 128 + 2 * MLP_MAXA + 2) head_params_store(tid - 128, head_params(tid - 128));
  if (!SP && tid >= 96 && tid < 96 + nl) {
    const int l = tid - 96;
    S.in[l] = (int)T.in[l];
    S.out[l] = (int)T.out[l];
    S.act[l] = (int)T.act[l];
    S.F[l] = T.F[l];
    S.b[l] = T.b[l];
    S.G[l] = T.G[l];
    S.xs[l] = T.xs[l];
    S.dp[l] = T.dp[l];
  }
  // ---- row gather: explicit index list, the keyed minibatch permutation (PPO), or identity
  auto gather_rows = [&]() {
    if (tid < MLP_BM) {
      const int lrow = min(row0 + tid, a.B - 1);
      int64_t g = lrow;
      if (a.idx) g = a.idx[lrow];
      else if (a.perm_uc)
        g = prp_index((uint32_t)(a.perm_off + lrow), (uint32_t)a.perm_n,
                      minibatch_key(a.perm_seed, *a.perm_uc, a.perm_ep));
      S.grow[tid] = g;
    }
  };
  // ---- train: the loss head's per-row inputs loaded now, consumed after the forward (issued behind the forward's
  // first weight loads they were a dependent global round trip in the middle of the chain): gaussian-phase thread
  // (r, j) the action component, row thread r the old log-prob and advantage (policy) or return and old value
  // (critic) -- the same threads that read them below
  // this row tile's blocks of a workspace array of width w (blk_out layout)
  auto wsp = [&](int64_t base, int w) { return P_<float>(base) + (size_t)blockIdx.x * ((w + 15) >> 4) * 256; };
  const bool policy = (t == 0);
  float e_act = 0.f, e_lo = 0.f, e_adv = 0.f, e_ret = 0.f, e_vo = 0.f;
  int e_ai = 0;
  // (SPEC: wave 0 loads them all, ahead of its input tile and weights; the action components go through LDS)
  auto head_rows = [&]() {
    if (tid < rows) {
      const int64_t grow = S.grow[tid];
      if (policy) {
        e_lo = a.logp_old[grow];
        e_adv = a.adv[grow];
        if (a.head != 2) e_ai = a.act_i_in[grow];
      } else {
        e_ret = a.ret[grow];
        if (a.v_old && a.v_clip > 0.f) e_vo = a.v_old[grow];
      }
    }
  };
  auto head_inputs = [&]() {
    const int r = tid / MLP_MAXA, j = tid % MLP_MAXA;
    if (policy && a.head == 2 && tid < MLP_BM * MLP_MAXA && j < a.A && r < rows) e_act = a.act_f_in[S.grow[r] * a.A + j];
    head_rows();
  };
  Regs R;
  // SPEC wave 0: Gaussian action components, head parameter, row inputs (raw loads, selected when staged)
  float ea[4] = {0.f, 0.f, 0.f, 0.f}, hp = 0.f, hx[2] = {0.f, 0.f};
  int32_t hxi = 0;
  constexpr int NG0 = SP ? SPEC : 1;
  float xa[NG0][4];   // SPEC: this lane's layer-0 A operands (row r, columns 16 g + 4 q + s) straight from memory
  if constexpr (SP) {
    // SPEC: every wave requests its layer-0 input operands first, then ALL of its weight fragments for the whole
    // forward + data-gradient chain (216 / 304 KB per actor / critic workgroup, which the L2 -> CU path delivers at
    // ~60 B/clk in ~1.5 / 2.1 us), with no barrier in between: the CU's memory pipeline serves requests in order,
    // so the inputs land first and layer 0 starts while the later layers' weights stream in. (Staging the input
    // tile through one wave queued it behind the weight stream: the first layer started ~2.6 us into the launch.)
    const int r = lane & 15, q = lane >> 4;
    const int lrow = min(row0 + r, a.B - 1);
    int64_t grow = lrow;
    if (a.idx) grow = a.idx[lrow];
    else if (a.perm_uc)
      grow = prp_index((uint32_t)(a.perm_off + lrow), (uint32_t)a.perm_n,
                       minibatch_key(a.perm_seed, *a.perm_uc, a.perm_ep));
#pragma unroll
    for (int g = 0; g < NG0; ++g)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int col = 16 * g + 4 * q + s2;
        xa[g][s2] = (col < a.D && row0 + r < a.B) ? a.obs[grow * a.ld_obs + col] : 0.f;
      }
    if (wave == 0 && lane < MLP_BM) S.grow[lane] = grow;
    spec_load<SPEC>(R, a.htw[TW], wave, lane, tid);
    // the loss head's inputs behind the weights (consumed after the forward, staged through LDS by then). Every
    // load unconditional from a valid address, values selected afterwards: a register loaded on one side of a
    // divergent branch and zeroed on the other makes the waitcnt pass drain the whole weight stream at the join.
    if (wave == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int64_t gr = S.grow[lane & 15];
      const bool vclip = a.v_old && a.v_clip > 0.f;
      const float* p0 = policy ? a.logp_old : a.ret;
      const float* p1 = policy ? a.adv : (vclip ? a.v_old : a.ret);
      const int32_t* p2 = (policy && a.head != 2) ? a.act_i_in : reinterpret_cast<const int32_t*>(a.ret);
      hx[0] = p0[gr];
      hx[1] = p1[gr];
      hxi = p2[gr];
      // head parameters: lane i < 16 log-std, < 32 action scale, 32 / 33 the kl / entropy coefficients
      const bool gs = a.log_std && a.ac_scale;
      const float* ph = (lane < MLP_MAXA && gs) ? a.log_std + min(lane, max(a.A - 1, 0))
                        : (lane < 2 * MLP_MAXA && gs) ? a.ac_scale + min(lane - MLP_MAXA, max(a.A - 1, 0))
                        : (lane == 2 * MLP_MAXA && a.kl_coef) ? a.kl_coef
                        : (lane == 2 * MLP_MAXA + 1 && a.ent_coef) ? a.ent_coef : a.ret;
      hp = *ph;   // (the raw values: selected where they are staged, after the forward -- a use here would wait)
      if (policy && a.head == 2) {
        const int n = max(rows * a.A, 1);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = min(lane + 64 * u, n - 1);
          ea[u] = a.act_f_in[S.grow[e / a.A] * a.A + e % a.A];
        }
      }
    }
    stamp(1);
  } else {
    gather_rows();
    __syncthreads();
    if (a.mode == 2) head_inputs();
    stamp(1);
    // ---- input tile (gathered rows; padded rows / columns are zero)
    for (int e = tid; e < MLP_BM * ld0; e += MLP_THREADS) {
      const int r = e / ld0, c = e - r * ld0;
      float v = 0.f;
      if (r < rows && c < a.D) v = a.obs[S.grow[r] * a.ld_obs + c];
      X0[e] = v;
    }
  }
  __syncthreads();
  stamp(2);
  cstamp(12);
  // ---- forward
  if constexpr (SP) {
    // (the layer inputs X_l for the weight gradients are stored after the forward: a store loop between the weight
    // loads and their MFMAs would make the waitcnt pass drain the whole weight stream)
    float* P1 = sm + YO(nl - 1) + MLP_BM * LDY(nl - 1) + MLP_BM * (MLP_MAXW + 4);   // head split-K scratch
    auto next = [&](int l) {
      __syncthreads();
      stamp(3 + l);
    };
    // layer 0 from the A operands in registers; wave 0 then keeps the tile in LDS (workspace store below)
    wset_fwd_rega(R.f0, xa, OUTW(0), act_slope(ACT(0)), sm + YO(0), LDY(0), wave, lane);
    if (wave == 0) {
      const int r = lane & 15, q = lane >> 4;
#pragma unroll
      for (int g = 0; g < NG0; ++g)
        *reinterpret_cast<floatx4*>(X0 + r * ld0 + 16 * g + 4 * q) = floatx4{xa[g][0], xa[g][1], xa[g][2], xa[g][3]};
    }
    if (TW == 1 || a.head == 2) {   // the loss head's top-gradient tile (value / fused Gaussian head), zeroed off the head's chain
      float* dz = sm + YO(nl - 1) + MLP_BM * LDY(nl - 1);
      for (int e = tid; e < MLP_BM * (MLP_MAXW + 4); e += MLP_THREADS) dz[e] = 0.f;
    }
    auto stage_head_inputs = [&]() {   // wave 0, before the last forward barrier (the loads landed long before)
      if (wave != 0) return;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = lane + 64 * u;
        if (policy && a.head == 2 && e < rows * a.A) S.hd[e / a.A][e % a.A] = ea[u];   // (read as e_act)
      }
      if (lane < MLP_BM) {
        const bool vclip = a.v_old && a.v_clip > 0.f;
        S.er[0][lane] = policy ? hx[0] : 0.f;                                    // log-prob
        S.er[1][lane] = policy ? hx[1] : 0.f;                                    // advantage
        S.er[2][lane] = policy ? 0.f : hx[0];                                    // return
        S.er[3][lane] = (!policy && vclip) ? hx[1] : 0.f;                        // old value
        S.er[4][lane] = __int_as_float((policy && a.head != 2) ? hxi : 0);       // action index
      }
      const bool gs = a.log_std && a.ac_scale;
      const bool hok = (lane < MLP_MAXA && gs && lane < a.A) ||
                       (lane >= MLP_MAXA && lane < 2 * MLP_MAXA && gs && lane - MLP_MAXA < a.A) ||
                       (lane == 2 * MLP_MAXA && a.kl_coef) || (lane == 2 * MLP_MAXA + 1 && a.ent_coef);
      head_params_store(lane, hok ? hp : 0.f);
    };
    next(0);
    const int64_t G1 = a.htw[TW == 0 ? 0 : 1].G[1];
    if constexpr (TW == 0) {
      // W1 [128][128]: g1 = WSet<8, 8> (one slot, 8 groups), one load per k-group of layer 1 (8 groups)
      wset_fwd_side(R.f1, sm + YO(0), LDY(0), OUTW(1), act_slope(ACT(1)), sm + YO(1), LDY(1), wave, lane,
                    [&](int g) { wset_load_one(R.g1, G1, 0, g, wave, lane); });
      next(1);
      wset_fwd(R.f2, sm + YO(1), LDY(1), OUTW(2), act_slope(ACT(2)), sm + YO(2), LDY(2), wave, lane);
      next(2);
      whead_fwd(R.f3, sm + YO(2), LDY(2), OUTW(3), act_slope(ACT(3)), sm + YO(3), LDY(3), P1, wave, lane, tid);
      stage_head_inputs();
      next(3);
    } else {
      // W1 [256][128]: g1 = WSet<8, 16> (two slots x 8 groups), one load per k-group of layer 1 (16 groups)
      wset_fwd_side(R.f1, sm + YO(0), LDY(0), OUTW(1), act_slope(ACT(1)), sm + YO(1), LDY(1), wave, lane,
                    [&](int g) { wset_load_one(R.g1, G1, g >> 3, g & 7, wave, lane); });
      next(1);
      whead_fwd(R.f2, sm + YO(1), LDY(1), OUTW(2), act_slope(ACT(2)), sm + YO(2), LDY(2), P1, wave, lane, tid);
      stage_head_inputs();
      next(2);
    }
    if (policy && a.head == 2 && tid < MLP_BM * MLP_MAXA) {
      const int r = tid / MLP_MAXA, j = tid % MLP_MAXA;
      if (j < a.A && r < rows) e_act = S.hd[r][j];
    }
    if (tid < MLP_BM) {
      e_lo = S.er[0][tid];
      e_adv = S.er[1][tid];
      e_ret = S.er[2][tid];
      e_vo = S.er[3][tid];
      e_ai = __float_as_int(S.er[4][tid]);
    }
  } else {
    const float* X = X0;
    int ldx = ld0;
    for (int l = 0; l < nl; ++l) {
      float* Yl = sm + S.yo[l];
      const int ldl = S.ld[l];
      layer_fwd(X, ldx, S.in[l], P_<const float>(S.F[l]), P_<const float>(S.b[l]), S.out[l], S.act[l], Yl, ldl);
      __syncthreads();
      stamp(3 + l);
      if (a.mode == 2 && l == 0) blk_out(X0, ld0, wsp(S.xs[0], a.D), a.D);   // inputs of each layer for its
      if (a.mode == 2 && l + 1 < nl) blk_out(Yl, ldl, wsp(S.xs[l + 1], S.out[l]), S.out[l]);   // weight gradient
      X = Yl;
      ldx = ldl;
    }
  }
  const int L = nl - 1;
  const float* Yo = sm + YO(L);
  const int ldo = LDY(L);
  // ---- heads: one thread per row
  float* dPtop = sm + YO(L) + MLP_BM * LDY(L);   // P0
  float* P1 = dPtop + MLP_BM * (MLP_MAXW + 4);
  const int ldP = MLP_MAXW + 4;
  // SPEC actor with the Gaussian head: the whole loss head in ONE barrier-free phase (fused_gauss_head below)
  const bool fgh = SP && TW == 0 && a.head == 2;
  if (a.mode == 2 && !(SP && (TW == 1 || fgh))) {   // zero the top dP tile (the head writes only valid columns)
    for (int e = tid; e < MLP_BM * ldP; e += MLP_THREADS) dPtop[e] = 0.f;
    __syncthreads();
  }
  if (fgh) {
    // Thread (r, j) = (tid >> 4, tid & 15) of waves 0-3: component j of row r -- mean, log-prob term, then the row's
    // log-prob and entropy as 16-lane xor trees (every lane of the row group gets the same bits), the PPO / A2C
    // surrogate and KL-proxy gradient redundantly per lane, d(loss)/d(pre-tanh mean) and the log-std term straight
    // from registers; the 4 rows of a wave meet through xor 16 / 32, the 4 waves through S.red in wave order.
    // (The generic head runs phase A, a 16-thread row section and phase C with a barrier between each.)
    if (tid < MLP_BM * MLP_MAXA) {
      const int r = tid >> 4, j = tid & 15;
      const bool comp = j < a.A, live = r < rows;
      float hl = 0.f, hc = 0.f, d = 0.f, th = 0.f, ivar = 0.f, lsc = 0.f, sc = 0.f, raw = 0.f;
      if (comp) {
        raw = S.hls[j];
        lsc = fminf(fmaxf(raw, -2.5f), 2.5f);
        sc = S.hsc[j];
        th = tanhf(Yo[r * ldo + j]);
        const float mu = th * sc;
        const float aj = live ? e_act : mu;
        const float zz = (aj - mu) * expf(-lsc);
        hl = -0.5f * zz * zz - lsc - HALF_LOG_2PI;
        hc = 0.5f + HALF_LOG_2PI + lsc;
        d = aj - mu;
        ivar = expf(-2.f * lsc);
      }
      float lp = hl, H = hc;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        lp += lane_xor(lp, o);
        H += lane_xor(H, o);
      }
      const float lo = S.er[0][r], adv = S.er[1][r];
      const float beta = S.hco[0];
      float st[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
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
      const float g = live ? a.inv_B * (-dsurr - 2.f * beta * (lo - lp)) : 0.f;
      if (comp) dPtop[r * ldP + j] = live ? g * d * ivar * sc * (1.f - th * th) : 0.f;
      const bool inr = raw >= -2.5f && raw <= 2.5f;
      float lsg = (comp && live && inr) ? g * (d * d * ivar - 1.f) - S.hco[1] * a.inv_B : 0.f;
      // the wave's 4 rows (lanes j, j + 16, j + 32, j + 48)
      lsg += lane_xor(lsg, 16);
      lsg += lane_xor(lsg, 32);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = live ? st[k] : 0.f;
        v += lane_xor(v, 16);
        v += lane_xor(v, 32);
        st[k] = v;
      }
      if (lane < MLP_MAXA) S.red[wave][lane] = lsg;
      if (lane == 0)
#pragma unroll
        for (int k = 0; k < 8; ++k) S.red[wave][MLP_MAXA + k] = st[k];
    }
    __syncthreads();
    stamp(8);
    if (tid < MLP_MAXA + 8) {   // partial row of this workgroup: 4 waves in order (summed by the weight-gradient kernel)
      const float v = ((S.red[0][tid] + S.red[1][tid]) + S.red[2][tid]) + S.red[3][tid];
      const int k = tid - MLP_MAXA;
      if (tid < MLP_MAXA) {
        if (tid < a.A) {
          if (a.mpart) a.mpart[(size_t)blockIdx.x * MPART_W + 8 + tid] = v;
          else atomicAdd(&a.g_log_std[tid], v);
        }
      } else if (k != 3) {
        if (a.mpart) a.mpart[(size_t)blockIdx.x * MPART_W + k] = v * a.inv_B;
        else if (k != 5 && v != 0.f) atomicAdd(&a.mstats[k], v * a.inv_B);
      }
    }
    stamp(14);
  } else {
  // Gaussian policy head, phase A: one thread per (row, action component) -- mean, sample (rollout) or given action,
  // the component's log-prob term (a per-row loop of tanh / hash / log / sqrt / cos / exp chains on 16 lanes would
  // idle 7 of 8 waves; the per-row sums below keep the sequential order, so the results do not change)
  const bool gauss = policy && a.head == 2;
  if (gauss) {
    if (tid < MLP_BM * MLP_MAXA) {
      const int r = tid / MLP_MAXA, j = tid % MLP_MAXA;
      if (j < a.A) {
        const bool live = r < rows;
        const int64_t grow = S.grow[r];
        const float ls = fminf(fmaxf(S.hls[j], -2.5f), 2.5f);
        const float th = tanhf(Yo[r * ldo + j]);
        const float mu = th * S.hsc[j];
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
        S.hl[r][j] = -0.5f * zz * zz - ls - HALF_LOG_2PI;
        S.ht[r][j] = th;
        S.hd[r][j] = aj - mu;
      }
    }
    __syncthreads();
    stamp(15);
  }
  if (tid < MLP_BM) {
    const int r = tid;
    const bool live = r < rows;
    const int64_t grow = S.grow[r];
    float st[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (!policy) {
      const float v = Yo[r * ldo];
      if (live && (a.mode == 0 || a.mode == 1) && a.v_out) a.v_out[grow] = v;
      if (live && a.mode == 2) {
        const float R_ = e_ret;
        float dv = 2.f * (v - R_), l2 = (v - R_) * (v - R_);
        if (a.v_old && a.v_clip > 0.f) {
          const float vo = e_vo;
          const float d = fminf(fmaxf(v - vo, -a.v_clip), a.v_clip);
          const float vc = vo + d;
          const float l2c = (vc - R_) * (vc - R_);
          const bool inr = (v - vo) >= -a.v_clip && (v - vo) <= a.v_clip;
          if (l2c > l2) { dv = inr ? 2.f * (vc - R_) : 0.f; l2 = l2c; }
          else if (l2c == l2) dv = 0.5f * dv + 0.5f * (inr ? 2.f * (vc - R_) : 0.f);
        }
        dPtop[r * ldP] = a.vf_coef * a.inv_B * dv;
        st[3] = l2;
      }
    } else if (a.head == 2) {   // diagonal Gaussian: per-component terms computed above, fixed-order sums here
      const int A = a.A;
      float lp = 0.f, H = 0.f;
      for (int j = 0; j < A; ++j) {
        lp += S.hl[r][j];
        H += 0.5f + HALF_LOG_2PI + fminf(fmaxf(S.hls[j], -2.5f), 2.5f);
      }
      if (live && a.mode != 2) {
        if (a.logp_out) a.logp_out[grow] = lp;
        if (a.ent_out) a.ent_out[grow] = H;
      }
      float g = 0.f;
      if (a.mode == 2 && live) {
        const float lo = e_lo, adv = e_adv;
        const float beta = S.hco[0];
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
      S.g[r] = g;
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
        const float beta = S.hco[0], ce = S.hco[1];
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
        const float raw = S.hls[j];
        const float ls = fminf(fmaxf(raw, -2.5f), 2.5f);
        const float ivar = expf(-2.f * ls);
        const float d = S.hd[r][j], th = S.ht[r][j], g = S.g[r];
        const float dmu = g * d * ivar;
        dPtop[r * ldP + j] = live ? dmu * S.hsc[j] * (1.f - th * th) : 0.f;
        const bool inr = raw >= -2.5f && raw <= 2.5f;
        S.red[r][j] = (live && inr) ? g * (d * d * ivar - 1.f) - S.hco[1] * a.inv_B : 0.f;
      }
    }
    __syncthreads();
  }
  // log-std gradient: column sums over the tile's rows, one atomic per column
  if (policy && a.head == 2 && tid < a.A) {
    float s = 0.f;
    for (int r = 0; r < MLP_BM; ++r) s += S.red[r][tid];
    if (a.mpart) a.mpart[(size_t)blockIdx.x * MPART_W + 8 + tid] = s;
    else atomicAdd(&a.g_log_std[tid], s);
  }
  stamp(14);   // head phase C + log-std sums (the data-gradient layers take slots 9 ..)
  }   // !fgh
  // ---- top layer dP: apply the head activation derivative (tanh applied above) and publish
  if constexpr (SP) {   // (no store loop ahead of the data-gradient MFMAs, see above; N <= 16: one block)
    // the layer inputs for the weight gradients, issued after the head (whose branch joins would otherwise wait for
    // them to land): they drain under the data-gradient chain
    blk_out_c<NG0>(X0, ld0, wsp(XS(0), a.D), a.D);
    if constexpr (TW == 0) {
      blk_out_c<8>(sm + YO(0), LDY(0), wsp(XS(1), OUTW(0)), OUTW(0));
      blk_out_c<8>(sm + YO(1), LDY(1), wsp(XS(2), OUTW(1)), OUTW(1));
      blk_out_c<4>(sm + YO(2), LDY(2), wsp(XS(3), OUTW(2)), OUTW(2));
    } else {
      blk_out_c<16>(sm + YO(0), LDY(0), wsp(XS(1), OUTW(0)), OUTW(0));
      blk_out_c<8>(sm + YO(1), LDY(1), wsp(XS(2), OUTW(1)), OUTW(1));
    }
    if (tid < 64) {
      const int c = tid >> 2, r4 = tid & 3;
      floatx4 v;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) v[s2] = dPtop[(4 * r4 + s2) * ldP + c];   // (columns >= N are zero)
      *(__attribute__((address_space(1))) floatx4*)(wsp(DPW(L), OUTW(L)) + c * 16 + 4 * r4) = v;
    }
  } else {
    blk_out(dPtop, ldP, wsp(S.dp[L], S.out[L]), S.out[L]);
  }
  // ---- data-gradient chain: dP_l -> dP_{l-1}
  if constexpr (SP) {
    auto gd = [&](int l) { return wsp(DPW(l - 1), INW(l)); };
    if constexpr (TW == 0) {
      wset_dgrad(R.g3, dPtop, ldP, INW(3), sm + YO(2), LDY(2), act_slope(ACT(2)), P1, ldP, gd(3), rows,
                 wave, lane);
      __syncthreads();
      stamp(9);
      wset_dgrad(R.g2, P1, ldP, INW(2), sm + YO(1), LDY(1), act_slope(ACT(1)), dPtop, ldP, gd(2), rows, wave,
                 lane);
      __syncthreads();
      stamp(10);
      wset_dgrad(R.g1, dPtop, ldP, INW(1), sm + YO(0), LDY(0), act_slope(ACT(0)), P1, ldP, gd(1), rows, wave,
                 lane);
      stamp(11);
    } else {
      wset_dgrad(R.g2, dPtop, ldP, INW(2), sm + YO(1), LDY(1), act_slope(ACT(1)), P1, ldP, gd(2), rows,
                 wave, lane);
      __syncthreads();
      stamp(9);
      wset_dgrad(R.g1, P1, ldP, INW(1), sm + YO(0), LDY(0), act_slope(ACT(0)), dPtop, ldP, gd(1), rows, wave,
                 lane);
      stamp(10);
    }
    if (a.stamps && blockIdx.x == 0) {
      cstamp(13);
      stamp(7);   // end of the data-gradient chain (stores issued)
      __syncthreads();
      if (tid < 16) a.stamps[blockIdx.y * 16 + tid] = S.ts[tid];
    }
    return;
  } else {
    float* cur = dPtop;
    float* nxt = P1;
    for (int l = L; l >= 1; --l) {
      const int K = S.in[l];
      gf32* gdst = wsp(S.dp[l - 1], K);
      layer_dgrad(cur, ldP, S.out[l], P_<const float>(S.G[l]), K, sm + S.yo[l - 1], S.ld[l - 1], S.act[l - 1], nxt,
                  ldP, gdst, rows);
      __syncthreads();
      stamp(9 + L - l);
      float* tmp = cur;
      cur = nxt;
      nxt = tmp;
    }
  }
  cstamp(13);
}

template <int SPEC>
__global__ void __launch_bounds__(MLP_THREADS) mlp_fwd_kernel(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];   // 16-byte base: the b128 LDS reads stay aligned
  __shared__ MlpShared S;
  const int t = blockIdx.y + a.tw_base;
  if constexpr (SPEC == 0) {
    mlp_tower<0, -1>(a, t, sm, S);
  } else {
    if (t == 0) mlp_tower<SPEC, 0>(a, 0, sm, S);
    else mlp_tower<SPEC, 1>(a, 1, sm, S);
  }
}

// ------------------------------------------------------------------------------------------------ weight grads

__device__ __forceinline__ float clipsq(float v, float c) {
  if (c > 0.f) v = fminf(fmaxf(v, -c), c);
  return v * v;
}

// One 4-wave workgroup per ITEM (a 16 x 16 tile of one dW_l = X_l^T dP_l, its bias column sums when it is in the first
// row of tiles, and its sum of squares for the global-norm clip), per batch split. The item record (8 int64, built by
// ops/mlp.py, read with one scalar load -- the tower / layer / tile search over the device descriptor was a chain of
// dependent round trips): X block base, dP block base, their row-tile strides (floats, low / high 32 bits),
// (valid dW rows | valid columns << 8 | N << 32), dW tile pointer, bias pointer (0: none), sum-of-squares slot (0:
// none), (clip as float bits | first parts slot to zero << 32, item 0 of a tower). The waves take interleaved row
// tiles, every operand of a wave's row tiles in flight before its MFMAs; the partial tiles are summed through LDS.
constexpr int WG_RT = 8;   // row tiles per wave per round (16 loads in flight per lane)

__global__ void __launch_bounds__(256) mlp_wgrad_kernel(WgradArgs a) {
  __shared__ float red[4][64][5];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (blockIdx.x == gridDim.x - 1) {
    // The bookkeeping workgroup (one past the items): the train kernel's per-workgroup partial rows summed in a fixed
    // order (deterministic) -- the loss statistics published and the log-std gradient finished with its sum of
    // squares in its own slot -- and the update counter advanced. Every load is issued up front (one round trip).
    if (wave != 0) return;
    const float kl = *a.kl_coef, ec = *a.ent_coef;
    float v[MPART_W];
#pragma unroll
    for (int c = 0; c < MPART_W; ++c) v[c] = 0.f;
    for (int row = lane; row < a.mpart_rows; row += 64) {
#pragma unroll
      for (int c = 0; c < MPART_W; ++c) v[c] += a.mpart[(size_t)row * MPART_W + c];
    }
#pragma unroll
    for (int c = 0; c < MPART_W; ++c) v[c] = wave_sum(v[c]);
    if (a.g_log_std) {
      float g = 0.f;   // v[8 + lane] with compile-time indices (a runtime index would put v in scratch)
#pragma unroll
      for (int j = 0; j < MLP_MAXA; ++j) g = lane == j ? v[8 + j] : g;
      // the gradient is STORED (like every other element of this launch): no zeroing between minibatches
      if (lane < a.A) a.g_log_std[lane] = g;
      if (a.ls_part) {
        const float ss = wave_sum(lane < a.A ? clipsq(g, a.ls_clip) : 0.f);
        if (lane == 0) *a.ls_part = ss;
      }
    }
    if (lane == 0) {
      if (a.stats) {
        float m[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) m[k] = v[k];
        m[5] = m[0] + kl * m[1] - ec * m[2];
#pragma unroll
        for (int k = 0; k < 7; ++k) a.stats[k] = m[k];
      }
      // the train kernel (the counter's only reader in this minibatch) has finished: stream order
      if (a.bump) __hip_atomic_fetch_add(a.bump, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  // XCD-grouped item order (common.h xcd_remap): each XCD takes one contiguous range of the item table, whose
  // neighbouring items (tiles of one layer) share their X / dP column blocks -- they meet in one L2
  const int bid = xcd_remap((int)blockIdx.x, (int)gridDim.x - 1);
  const int split = bid % a.nsplit;
  const int64_t* rec = a.items + (size_t)(bid / a.nsplit) * 8;
  gcf32* X = P_<const float>(rec[0]);
  gcf32* P = P_<const float>(rec[1]);
  const int sx = (int)(rec[2] & 0xFFFFFFFF), sp = (int)(rec[2] >> 32);
  const int ni = (int)(rec[3] & 0xFF), nj = (int)((rec[3] >> 8) & 0xFF), N = (int)(rec[3] >> 32);
  const int per = (a.nrt + a.nsplit - 1) / a.nsplit;
  const int rb = split * per, re = min(a.nrt, rb + per);
  const int r = lane & 15, q = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  for (int c0 = rb + wave; c0 < re; c0 += 4 * WG_RT) {
    floatx4 xa[WG_RT], pb[WG_RT];
#pragma unroll
    for (int u = 0; u < WG_RT; ++u) {
      const int rt = min(c0 + 4 * u, re - 1);   // (clamped: a duplicate load, not used)
      xa[u] = *(gcfx4*)(X + (size_t)rt * sx + r * 16 + 4 * q);
      pb[u] = *(gcfx4*)(P + (size_t)rt * sp + r * 16 + 4 * q);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < WG_RT; ++u) {
      if (c0 + 4 * u < re) {
        // lane (column r, quad q): rows 4q + s of the row tile, k-slot q of MFMA s (the same row mapping on both sides)
        acc = mfma4(xa[u][0], pb[u][0], acc);
        acc = mfma4(xa[u][1], pb[u][1], acc);
        acc = mfma4(xa[u][2], pb[u][2], acc);
        acc = mfma4(xa[u][3], pb[u][3], acc);
        bsum += (pb[u][0] + pb[u][1]) + (pb[u][2] + pb[u][3]);
      }
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
  const float c = __int_as_float((int)(rec[7] & 0xFFFFFFFF));
  gf32* gW = P_<float>(rec[4]);
  // C: col = lane&15 -> j, rows 4q+i -> i
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ii = 4 * q + i;
    if (ii < ni && r < nj) {
      gf32* dst = gW + (size_t)ii * N + r;
      if (a.nsplit > 1) atomicAdd((float*)dst, acc[i]);
      else {
        *dst = acc[i];
        ss += clipsq(acc[i], c);
      }
    }
  }
  if (rec[5]) {
    // lanes with equal (lane & 15) hold partial column sums over rows = q (mod 4)
    bsum += lane_xor(bsum, 16);
    bsum += lane_xor(bsum, 32);
    if (q == 0 && r < nj) {
      gf32* gb = P_<float>(rec[5]) + r;
      if (a.nsplit > 1) atomicAdd((float*)gb, bsum);
      else {
        *gb = bsum;
        ss += clipsq(bsum, c);
      }
    }
  }
  if (a.nsplit == 1 && rec[6]) {
    ss = wave_sum(ss);
    float* slot = reinterpret_cast<float*>(rec[6]);
    if (lane == 0) *slot = ss;
    const int zf = (int)(rec[7] >> 32);
    if (zf)   // item 0 of its tower: the unused slots are zero (the optimiser sums all MLP_PARTS in a fixed order)
      for (int k = zf + lane; k < MLP_PARTS; k += 64) slot[k] = 0.f;
  }
}

// PPO epoch gather: row i of every minibatch input (observation, action, old log-prob, advantage, return, old value)
// copied from row prp(i) of the batch -- the keyed epoch permutation (envs/rng.py prp; key from the device update
// counter) -- so the epoch's train launches read contiguous rows: no index or permutation round trip ahead of
// their input tiles. Actions are copied as 4-byte words (float components or the int32 index). One thread per row.
__global__ void __launch_bounds__(256) mlp_epoch_gather_kernel(EpochGatherArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const int64_t src = prp_index((uint32_t)i, (uint32_t)a.n, minibatch_key(a.seed, *a.uc, a.ep));
  // every load of a chunk issued before its stores (a load -> store loop per column waits out one round trip per
  // column: the row's D + aw + 4 words were ~D + aw dependent round trips)
  const float lp = a.logp[src], ad = a.adv[src], rt = a.ret[src], vv = a.v ? a.v[src] : 0.f;
  constexpr int CH = 8;
  for (int c0 = 0; c0 < a.D; c0 += CH) {
    float x[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) x[u] = c0 + u < a.D ? a.obs[src * a.ld_obs + c0 + u] : 0.f;
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (c0 + u < a.D) a.o_obs[(size_t)i * a.D + c0 + u] = x[u];
  }
  for (int c0 = 0; c0 < a.aw; c0 += CH) {
    uint32_t w[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) w[u] = c0 + u < a.aw ? a.act[src * a.aw + c0 + u] : 0u;
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (c0 + u < a.aw) a.o_act[(size_t)i * a.aw + c0 + u] = w[u];
  }
  a.o_logp[i] = lp;
  a.o_adv[i] = ad;
  a.o_ret[i] = rt;
  if (a.v) a.o_v[i] = vv;
}

// The fragment copies F (every layer) and G (layers >= 1) of every W of the launched towers (common.h mlp_frag_f /
// mlp_frag_g; the pads stay zero). One thread per weight element; the optimiser step writes them as it goes (optim.hip
// OptTrans ldt -3 / -4), this pass covers engine creation and parameter changes outside the optimiser.
__global__ void __launch_bounds__(256) mlp_tshadow_kernel(const MlpTower* __restrict__ tw, int ntw, int total) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  for (int t = 0; t < ntw; ++t) {
    const MlpTower& T = tw[t];
    for (int l = 0; l < (int)T.nl; ++l) {
      const int K = (int)T.in[l], N = (int)T.out[l];
      if (e < K * N) {
        const int k = e / N, c = e - k * N;
        const float w = P_<const float>(T.W[l])[e];
        P_<float>(T.F[l])[mlp_frag_f(k, c, K)] = w;
        if (T.G[l]) P_<float>(T.G[l])[mlp_frag_g(k, c, N)] = w;
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

// The rollout's tile is ROLL_RB = 4 envs: its per-step chain is bound by the f32 MFMA work of ONE CU (16 env rows on
// 16x16x4 tiles: 0.86 MFLOP = 3.4k clocks per step at the CU's 256 FLOP/clk, ~4.5 of 6.3 us measured), so 4-env
// workgroups on the 4x4x1 MFMA (16 blocks of 4 x 4, k = 1: one instruction = 4 env rows x 64 columns, no padded rows)
// spread the rollout over 4x the CUs. Lane 4 b + i supplies A[i][k] (env row i), lane 4 b + j B[k][j] (column
// 4 b + j of the 64-column group), and lane 4 b + j receives D[0..3][j] (scripts/probes/mfma4x4.hip).
constexpr int ROLL_RB = 4;
__device__ __forceinline__ floatx4 mfma4x4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

// One actor layer of the rollout step: Y[4][ldy] = act(X[4][ldx] W + b). The 8 waves split (64-column group cg, K
// range sp); each wave holds ITS slice of W -- column cg * 64 + lane, rows [sp * kper, (sp + 1) * kper), as kper / 4
// float4 -- in registers for the whole rollout (loaded once before the step loop: the step reads no weight bytes at
// all), reads its env rows' X float4s from LDS up front, and runs kper 4x4x1 MFMAs; the partial tiles meet in LDS
// (`red`) and the epilogue sums them in K order, adds the bias, applies the activation and writes the zero pad columns
// [N, 16 ngp2(N)) that the next layer's K pad reads.
template <int K_, int N_>   // K_ padded (16 ngp2(K)), N_ <= 256
struct RollLayer {
  static constexpr int CG = (N_ + 63) / 64;                                              // column groups
  static constexpr int S = MLP_THREADS / 64 / CG < K_ / 4 ? MLP_THREADS / 64 / CG : K_ / 4;   // K splits
  static constexpr int kper = K_ / S, NU = kper / 4;                                     // K rows / float4 per wave
};

template <class L>
__device__ __forceinline__ void roll_layer_load_w(float4 (&w)[L::NU], const float* __restrict__ W, int ldw, int N) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cg = wave % L::CG, sp = wave / L::CG;
  const int c = min(cg * 64 + lane, N - 1);
#pragma unroll
  for (int u = 0; u < L::NU; ++u) w[u] = *reinterpret_cast<const float4*>(W + c * ldw + sp * L::kper + 4 * u);
}

template <class L>
__device__ __forceinline__ void roll_layer_mfma(const float4 (&w)[L::NU], const float* __restrict__ X, int ldx,
                                                float* __restrict__ red) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave < L::CG * L::S) {
    const int sp = wave / L::CG;
    const float* xr = X + (lane & 3) * ldx + sp * L::kper;
    float4 x[L::NU];
#pragma unroll
    for (int u = 0; u < L::NU; ++u) x[u] = *reinterpret_cast<const float4*>(xr + 4 * u);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < L::NU; ++u) {
      acc = mfma4x4(x[u].x, w[u].x, acc);
      acc = mfma4x4(x[u].y, w[u].y, acc);
      acc = mfma4x4(x[u].z, w[u].z, acc);
      acc = mfma4x4(x[u].w, w[u].w, acc);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(wave * 4 + i) * 64 + lane] = acc[i];
  }
}

template <class L>
__device__ __forceinline__ void roll_layer_epilogue(const float* __restrict__ red, const float* __restrict__ bias,
                                                    int N, int act, float* __restrict__ Y, int ldy) {
  const float slope = act_slope(act);
  const int NP = 16 * ngp2(N);
  for (int e = threadIdx.x; e < ROLL_RB * NP; e += MLP_THREADS) {
    const int i = e / NP, c = e - i * NP;
    float v = 0.f;
    if (c < N) {
      const int cg = c >> 6, l = c & 63;
      float sum = 0.f;
#pragma unroll
      for (int sp = 0; sp < L::S; ++sp) sum += red[((sp * L::CG + cg) * 4 + i) * 64 + l];
      v = act_fwd(sum + bias[c], slope);
    }
    Y[i * ldy + c] = v;
  }
}

// The actor's weights and biases are staged in LDS once (the reference actor at D = 17 is ~120 KB, SURVEY §2.4 K01;
// ops/mlp.py takes this kernel only when they fit), so the step loop issues no global loads at all. That matters
// beyond the load latency: on gfx9 global stores count on vmcnt too, so every wait for a load issued after the
// previous step's stores (observations, actions, rewards) would first drain those stores. The descriptor, head
// parameters and env ids are staged as well.
// KP0: the padded observation width (32 / 64: frame stacks of 1 / 2-3); the actor is the reference's 128-128-64-A
// (ops/mlp.py supports_fused_rollout)
template <int KP0>
__global__ void __launch_bounds__(MLP_THREADS) mlp_rollout_kernel(RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];   // 16-byte base: the b128 LDS reads stay aligned
  __shared__ int64_t s_tg[ROLL_RB];
  __shared__ int64_t s_ids[ROLL_RB];
  __shared__ int s_t[ROLL_RB];
  __shared__ float s_er[ROLL_RB];
  __shared__ float s_ls[MLP_MAXA], s_sc[MLP_MAXA];
  __shared__ float s_hl[ROLL_RB * MLP_MAXA];
  // the NEXT step's Box-Muller factors sqrt(-2 log u1) and cos(2 pi u2) (computed a step ahead, by two waves)
  __shared__ float s_epa[ROLL_RB * MLP_MAXA], s_epb[ROLL_RB * MLP_MAXA];
  __shared__ float s_els[MLP_MAXA], s_eils[MLP_MAXA];   // exp(log_std), exp(-log_std): step-invariant
  __shared__ int s_in[MLP_MAXL], s_out[MLP_MAXL], s_actc[MLP_MAXL];
  __shared__ int64_t s_wt[MLP_MAXL], s_b[MLP_MAXL];
  __shared__ float s_red[MLP_THREADS / 64 * 4 * 64];   // the layers' partial tiles (roll_layer_mfma)
  const MlpTower& T = a.tw[0];
  const int nl = (int)T.nl;
  const int row0 = blockIdx.x * ROLL_RB;
  const int rows = min(ROLL_RB, a.N - row0);
  const int tid = threadIdx.x;
  const int A = a.A, D = a.D;
  const int ld0 = ld_of(D);
  if (tid < nl) {
    s_in[tid] = (int)T.in[tid];
    s_out[tid] = (int)T.out[tid];
    s_actc[tid] = (int)T.act[tid];
    s_wt[tid] = T.F[tid];
    s_b[tid] = T.b[tid];
  }
  if (tid < MLP_MAXA) {
    const float ls = tid < A ? fminf(fmaxf(a.log_std[tid], -2.5f), 2.5f) : 0.f;
    s_ls[tid] = ls;
    s_els[tid] = expf(ls);
    s_eils[tid] = expf(-ls);
    s_sc[tid] = tid < A ? a.ac_scale[tid] : 0.f;
  }
  if (tid < ROLL_RB) {
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
    int off = 2 * ROLL_RB * ld0;
    for (int j = 0; j < l; ++j) off += ROLL_RB * ldyf(j);
    return sm + off;
  };
  // LDS: obs tile x2 | Y_0 .. Y_{nl-1} | A | B | env state [4][17] | actions [4][16] | W_l, b_l per layer
  float* sA = Yp(nl);
  float* sB = sA + LIN_OBS * LIN_OBS;
  float* s_state = sB + LIN_OBS * LIN_ACT;
  float* s_act = s_state + ROLL_RB * LIN_OBS;
  float* s_w0 = sm + (((s_act - sm) + ROLL_RB * MLP_MAXA + 3) & ~3);   // 16-byte aligned (b128 reads)
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
  {   // W_l [out][16*ngp2(in) + 4] (transposed, from the zero-padded forward fragment copy), then b_l
    for (int l = 0; l < nl; ++l) {
      const int NG = ngp2(s_in[l]), K4 = 4 * NG, N = s_out[l], ldw = 16 * NG + 4;
      float* w = Wl(l);
      gcfx4* src = (gcfx4*)P_<const float>(s_wt[l]);
      for (int e = tid; e < N * K4; e += MLP_THREADS) {
        const int c = e / K4, k4 = e - c * K4;
        // W[4 k4 .. 4 k4 + 3][c] is one float4 of F (common.h mlp_frag_f with k % 4 == 0)
        *reinterpret_cast<floatx4*>(w + c * ldw + 4 * k4) = src[((c >> 4) * NG + (k4 >> 2)) * 64 + (k4 & 3) * 16 + (c & 15)];
      }
      float* b = w + N * ldw;
      gcf32* bsrc = P_<const float>(s_b[l]);
      for (int e = tid; e < 16 * ngp2(N); e += MLP_THREADS) b[e] = e < N ? bsrc[e] : 0.f;
    }
  }
  for (int e = tid; e < 2 * ROLL_RB * ld0; e += MLP_THREADS) {   // step-0 tile (+ a zeroed second buffer)
    const int r = e / ld0, c = e - r * ld0;
    float v = 0.f;
    if (r < rows && c < D) v = a.obs[(size_t)(row0 + r) * D + c];
    sm[e] = v;
  }
  for (int j = tid; j < LIN_OBS * LIN_OBS; j += MLP_THREADS) sA[j] = a.lin_A[j];
  for (int j = tid; j < LIN_OBS * LIN_ACT; j += MLP_THREADS) sB[j] = a.lin_B[j];
  for (int e = tid; e < ROLL_RB * LIN_OBS; e += MLP_THREADS)
    s_state[e] = e / LIN_OBS < rows ? a.state[(size_t)row0 * LIN_OBS + e] : 0.f;
  for (int e = tid; e < ROLL_RB * MLP_MAXA; e += MLP_THREADS) s_act[e] = 0.f;
  __syncthreads();
  // every wave's weight slices of the four layers, in registers for the whole rollout
  using L0 = RollLayer<KP0, 128>;
  using L1 = RollLayer<128, 128>;
  using L2 = RollLayer<128, 64>;
  using L3 = RollLayer<64, 16>;
  float4 w0[L0::NU], w1[L1::NU], w2[L2::NU], w3[L3::NU];
  roll_layer_load_w<L0>(w0, sm + s_wo[0], KP0 + 4, s_out[0]);
  roll_layer_load_w<L1>(w1, sm + s_wo[1], 132, s_out[1]);
  roll_layer_load_w<L2>(w2, sm + s_wo[2], 132, s_out[2]);
  roll_layer_load_w<L3>(w3, sm + s_wo[3], 68, s_out[3]);
  auto bias_of = [&](int l, int ldw) { return sm + s_wo[l] + s_out[l] * ldw; };
  // The policy noise of step t depends only on (seed, env counter, env id, component): waves 2 and 4 (idle during the
  // env step) compute step t + 1's two Box-Muller factors while waves 0-1 step the envs -- wave 2 sqrt(-2 log u1),
  // wave 4 cos(2 pi u2), multiplied in the head as before (bit-identical). The env counter advances by one per step
  // (the env step's tg + 1), so a register copy of the key follows it.
  const int nbase = tid < 256 ? 128 : 256;
  const bool nz_owner = (tid >= 128 && tid < 128 + ROLL_RB * MLP_MAXA) || (tid >= 256 && tid < 256 + ROLL_RB * MLP_MAXA);
  const bool nz_a = tid < 256;
  const int nr = (tid - nbase) / MLP_MAXA, nj = (tid - nbase) % MLP_MAXA;
  const bool nz_live = nz_owner && nr < rows && nj < A;
  int64_t nkey = nz_live ? s_tg[nr] * ((int64_t)1 << a.key_shift) + s_ids[nr] : 0;
  auto noise_ahead = [&]() {
    if (nz_owner) {
      float f = 0.f;
      if (nj < A) {
        if (nz_a) f = sqrtf(-2.0f * logf(uniform_open(a.policy_seed, nkey, 2 * nj)));
        else f = cosf(TWO_PI * uniform_open(a.policy_seed, nkey, 2 * nj + 1));
      }
      (nz_a ? s_epa : s_epb)[nr * MLP_MAXA + nj] = f;
      if (nz_live) nkey += (int64_t)1 << a.key_shift;
    }
  };
  noise_ahead();
  __syncthreads();
  // diagnostics only (stamps[255] == 1): the step loop runs the actor layers alone (no head, no env step)
  const bool layers_only = a.stamps && a.stamps[255] == 1;
  for (int step = 0; step < a.T; ++step) {
    float* Xc = sm + (step & 1) * ROLL_RB * ld0;
    float* Xn = sm + ((step & 1) ^ 1) * ROLL_RB * ld0;
    // ---- actor forward
    float* Y0 = sm + s_yo[0];
    float* Y1 = sm + s_yo[1];
    float* Y2 = sm + s_yo[2];
    float* Y3 = sm + s_yo[3];
    roll_layer_mfma<L0>(w0, Xc, ld0, s_red);
    __syncthreads();
    roll_layer_epilogue<L0>(s_red, bias_of(0, KP0 + 4), s_out[0], s_actc[0], Y0, 132);
    __syncthreads();
    stamp(step, 0);
    roll_layer_mfma<L1>(w1, Y0, 132, s_red);
    __syncthreads();
    roll_layer_epilogue<L1>(s_red, bias_of(1, 132), s_out[1], s_actc[1], Y1, 132);
    __syncthreads();
    stamp(step, 1);
    roll_layer_mfma<L2>(w2, Y1, 132, s_red);
    __syncthreads();
    roll_layer_epilogue<L2>(s_red, bias_of(2, 132), s_out[2], s_actc[2], Y2, 68);
    __syncthreads();
    stamp(step, 2);
    roll_layer_mfma<L3>(w3, Y2, 68, s_red);
    __syncthreads();
    roll_layer_epilogue<L3>(s_red, bias_of(3, 68), s_out[3], s_actc[3], Y3, 20);
    __syncthreads();
    stamp(step, 3);
    const float* X = Y3;
    const int ldx = 20;
    if (layers_only) {
      stamp(step, 6);
      continue;
    }
    // ---- Gaussian head, one thread per (env, action component): mean, Box-Muller sample and the component's
    // log-prob term in parallel (a serial per-env loop of hash + log/sqrt/cos/tanh/exp chains on 16 lanes would
    // leave 7 of 8 waves idle for most of the step), then fixed-order per-env sums: bit-identical to the
    // one-thread-per-row head of mlp_fwd_kernel mode 0
    if (tid < ROLL_RB * MLP_MAXA) {
      const int r = tid / MLP_MAXA, j = tid % MLP_MAXA;
      if (j < A) {
        const bool live = r < rows;
        const float* Yo = X + r * ldx;
        const float ls = s_ls[j];
        const float mu = tanhf(Yo[j]) * s_sc[j];
        const float eps = s_epa[r * MLP_MAXA + j] * s_epb[r * MLP_MAXA + j];   // (noise_ahead: the previous step)
        const float aj = mu + s_els[j] * eps;
        const float zz = (aj - mu) * s_eils[j];
        s_hl[r * MLP_MAXA + j] = -0.5f * zz * zz - ls - HALF_LOG_2PI;
        s_act[r * MLP_MAXA + j] = aj;
        if (live) a.act[((size_t)step * a.N + row0 + r) * A + j] = aj;
      }
    }
    __syncthreads();
    stamp(step, 5);
    // (the per-env log-prob / entropy sums run on wave 3, beside the env step of waves 0-1 and wave 2's noise)
    if (tid >= 192 && tid < 192 + rows) {
      const int r = tid - 192;
      float lp = 0.f, H = 0.f;
      for (int j = 0; j < A; ++j) {
        lp += s_hl[r * MLP_MAXA + j];
        H += 0.5f + HALF_LOG_2PI + s_ls[j];
      }
      a.logp[(size_t)step * a.N + row0 + r] = lp;
      a.ent[(size_t)step * a.N + row0 + r] = H;
    }
    noise_ahead();   // waves 2 and 4: step + 1's policy noise, beside the env step below
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
// spec: 0 = the generic kernel; 1 / 2 / 4 = the SPEC train path for the reference towers with ngp2(D) == spec (the
// binding checks the shapes against a->htw)
extern "C" hipError_t aca_mlp_fwd(const MlpArgs* a, int ntw, size_t lds, int spec, hipStream_t stream) {
  if (a->B <= 0) return hipSuccess;
  if (a->A > MLP_MAXA || a->D > MLP_MAXW || ntw < 1 || a->tw_base + ntw > 2 || !a->tw) return hipErrorInvalidValue;
  if (spec && (a->mode != 2 || a->tw_base != 0 || ntw != 2 || mlp_ngp2(a->D) != spec)) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    const void* ks[4] = {reinterpret_cast<const void*>(&mlp_fwd_kernel<0>),
                         reinterpret_cast<const void*>(&mlp_fwd_kernel<1>),
                         reinterpret_cast<const void*>(&mlp_fwd_kernel<2>),
                         reinterpret_cast<const void*>(&mlp_fwd_kernel<4>)};
    for (const void* k : ks)
      if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024) != hipSuccess)
        return hipErrorInvalidValue;
    attr = true;
  }
  if (lds > 140 * 1024) return hipErrorInvalidValue;
  dim3 grid((a->B + MLP_BM - 1) / MLP_BM, ntw);
  switch (spec) {
    case 0: mlp_fwd_kernel<0><<<grid, MLP_THREADS, lds, stream>>>(*a); break;
    case 1: mlp_fwd_kernel<1><<<grid, MLP_THREADS, lds, stream>>>(*a); break;
    case 2: mlp_fwd_kernel<2><<<grid, MLP_THREADS, lds, stream>>>(*a); break;
    case 4: mlp_fwd_kernel<4><<<grid, MLP_THREADS, lds, stream>>>(*a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t aca_mlp_wgrad(const WgradArgs* a, hipStream_t stream) {
  if (a->nrt <= 0) return hipSuccess;
  if (!a->items || a->nitems < 1 || a->nsplit < 1 || !a->mpart || !a->kl_coef || !a->ent_coef || a->A > MLP_MAXA)
    return hipErrorInvalidValue;
  // + the bookkeeping workgroup (statistics, log-std gradient, update counter)
  mlp_wgrad_kernel<<<a->nitems * a->nsplit + 1, 256, 0, stream>>>(*a);
  return hipGetLastError();
}

extern "C" hipError_t aca_mlp_epoch_gather(const EpochGatherArgs* a, hipStream_t stream) {
  if (a->n <= 0) return hipSuccess;
  if (!a->uc || a->D < 1 || a->aw < 1) return hipErrorInvalidValue;
  mlp_epoch_gather_kernel<<<(a->n + 255) / 256, 256, 0, stream>>>(*a);
  return hipGetLastError();
}

extern "C" hipError_t aca_mlp_tshadow(const MlpTower* tw, int ntw, int total, hipStream_t stream) {
  if (total <= 0) return hipSuccess;
  mlp_tshadow_kernel<<<(total + 255) / 256, 256, 0, stream>>>(tw, ntw, total);
  return hipGetLastError();
}

constexpr size_t ROLLOUT_MAX_LDS = 150 * 1024;   // + ~9 KB static (s_red): within the 160 KB of a CU

extern "C" hipError_t aca_mlp_rollout(const RolloutArgs* a, size_t lds, hipStream_t stream) {
  if (a->N <= 0 || a->T <= 0) return hipSuccess;
  if (!a->tw || a->head != 2 || a->A != LIN_ACT || a->k < 1 || a->k > 3 || a->D != LIN_OBS * a->k || !a->wlds)
    return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_rollout_kernel<32>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, ROLLOUT_MAX_LDS) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_rollout_kernel<64>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, ROLLOUT_MAX_LDS) != hipSuccess)
      return hipErrorInvalidValue;
    attr = true;
  }
  if (lds > ROLLOUT_MAX_LDS) return hipErrorInvalidValue;
  const dim3 grid((a->N + ROLL_RB - 1) / ROLL_RB);
  if (a->k == 1) mlp_rollout_kernel<32><<<grid, MLP_THREADS, lds, stream>>>(*a);
  else mlp_rollout_kernel<64><<<grid, MLP_THREADS, lds, stream>>>(*a);
  return hipGetLastError();
}
