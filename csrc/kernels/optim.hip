// Fused optimisers over flat fp32 parameter slabs.
//
// The reference runs clip_by_value + ApplyAdam per variable (17 TF ops for Pendulum, Basic_AC/policies.py:79-82).
// Here one launch updates a whole slab segment:  g = clip(g, +-c) ; g *= min(1, max_norm / ||g||) ;
// Adam (TF1 "epsilon hat" form) or RMSprop (TF form, eps inside the sqrt) ; optional bf16 shadow write for the
// MFMA GEMMs. lr and the step count live in device memory, so the KL-adaptive lr controller and the schedules
// never sync with the host and the whole learner step can be captured in a hipGraph.
//
// The step counter t is read by every workgroup and advanced by the workgroup that finishes last (ticket), so no
// extra launch is needed. sumsq is deterministic: it only writes per-workgroup partials (fixed slots); every optimiser
// workgroup sums the same slots in the same order, so no in-kernel cross-workgroup hand-off (and no L2 write-back
// fence) is needed for the global norm.
#include "common.h"

namespace aca {

constexpr int OPT_THREADS = 256;
constexpr unsigned int OPT_TK_LINE = 32;   // Adam step ticket: 9 counters, one per 128-byte line (ops/optim.py)
constexpr int SUMSQ_U = 8;
constexpr int SUMSQ_PARTS = 256;   // max sumsq workgroups = partial slots the optimiser reduces

// Partial sums of squares of x over `nblk` workgroups (this one: `bid`), one partial slot each; slot `nblk` .. are
// zeroed by workgroup 0 so the consumer always sums SUMSQ_PARTS entries in a fixed order.
// four consecutive elements of an fp32 or a bf16 (u16) array as a float4 (group i)
__device__ __forceinline__ float4 ld4(const float* __restrict__ x, size_t i) {
  return reinterpret_cast<const float4*>(x)[i];
}
__device__ __forceinline__ float4 ld4(const u16* __restrict__ x, size_t i) {
  const uint2 w = reinterpret_cast<const uint2*>(x)[i];
  return make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xFFFF0000u), __uint_as_float(w.y << 16),
                     __uint_as_float(w.y & 0xFFFF0000u));
}
__device__ __forceinline__ float ld1(const float* __restrict__ x, size_t i) { return x[i]; }
__device__ __forceinline__ float ld1(const u16* __restrict__ x, size_t i) { return bf2f(x[i]); }

template <int U = SUMSQ_U, typename T = float>
__device__ __forceinline__ void sumsq_body(const T* __restrict__ x, size_t n, float* __restrict__ partial,
                                           int nblk, int bid, float* sh) {
  float s = 0.f;
  const size_t n4 = n / 4;
  // SUMSQ_U independent 16-byte loads in flight per thread before any use: the grid is capped at one workgroup
  // per CU, so latency (not bandwidth) bounds a one-load-at-a-time loop
  const size_t step = (size_t)nblk * blockDim.x * U;
  for (size_t i0 = bid * (size_t)blockDim.x * U + threadIdx.x; i0 < n4; i0 += step) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = i0 + (size_t)u * blockDim.x;
      v[u] = i < n4 ? ld4(x, i) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u].x * v[u].x + v[u].y * v[u].y + v[u].z * v[u].z + v[u].w * v[u].w;
  }
  if (bid == 0) {
    for (size_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) s += ld1(x, i) * ld1(x, i);
    for (int b = nblk + threadIdx.x; b < SUMSQ_PARTS; b += blockDim.x) partial[b] = 0.f;
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) partial[bid] = s;
}

template <typename T>
__global__ void __launch_bounds__(OPT_THREADS) sumsq_kernel(const T* __restrict__ x, size_t n,
                                                             float* __restrict__ partial) {
  __shared__ float sh[16];
  sumsq_body<SUMSQ_U, T>(x, n, partial, gridDim.x, blockIdx.x, sh);
}

// Several independent sums of squares in ONE launch (the separate actor / critic norms of a data-parallel MLP
// update, per minibatch: tens of thousands of elements): blockIdx.y = segment, SUMSQ_MU float4 per thread -- one
// memory round trip over more workgroups instead of the 8-deep loop over 5 (4.8 -> ~2 us, profiles/r6_dp_world1.txt).
constexpr int SUMSQ_MU = 2;
struct SumsqSegs {
  const float* x[4];
  float* partial[4];
  size_t n[4];
  int nblk[4];
};
__global__ void __launch_bounds__(OPT_THREADS) sumsq_multi_kernel(SumsqSegs a) {
  __shared__ float sh[16];
  const int g = blockIdx.y;
  if ((int)blockIdx.x >= a.nblk[g]) return;
  sumsq_body<SUMSQ_MU>(a.x[g], a.n[g], a.partial[g], a.nblk[g], blockIdx.x, sh);
}

// Global squared norm from the sumsq partials, reduced by every consumer workgroup in the same fixed order
// (deterministic, and no in-kernel cross-workgroup hand-off: the kernel boundary publishes the partials).
__device__ __forceinline__ float partial_total(const float* __restrict__ parts, float* sh) {
  float v = 0.f;
  for (int i = threadIdx.x; i < SUMSQ_PARTS; i += blockDim.x) v += parts[i];
  return block_sum(v, sh);
}


// One optimiser segment (a parameter group of the flat slab) with its own lr / step / clip / norm settings.
// Optional copies of [K][N] weight matrices inside the segment, written by the update itself (no pass of their own):
//   ldt >= 0: transposed fp32 Wt[N][ldt];
//   ldt -1:   a FRAGMENT-ORDERED bf16 copy (the CNN engine's MFMA weight operands, cnn_fused.hip frag_w1..3): element
//             (k, c) goes to u16 ((((k / 16) * (N / 32) + c / 32) * 64 + (c / 8 % 4) * 16 + k % 16) * 8 + c % 8), so a
//             wave's 16-byte-per-lane fragment load is one contiguous 1 KB read;
//   (the MLP engine's fp32 fragment copies F / G are written by the item path below, not through this table)
constexpr int OPT_MAXT = 8;
struct OptTrans {
  int64_t off;   // element offset of W within the segment
  int K, N, ldt;
  float* dst;
};
constexpr int BLK_LD = 68;   // row stride (floats) of the workgroup's 16 x 64 LDS tile (item path)

struct OptSeg {
  float* p; float* g; float* m; float* v; size_t n;
  const float* lr; float* t;
  const float* parts; float* gnorm_out; u16* shadow;
  float clip, max_norm, gmul, norm_mul;
  unsigned int* ticket;
  int nblocks;
  int ntrans;
  OptTrans tr[OPT_MAXT];
  // >= 0: this launch is Adam step *t + t_off + 1 of a captured sequence whose counter the host advances once per
  // update (the launch-time step is known), so no workgroup publishes t + 1 and the ticket is skipped; -1: ticket
  int t_off = -1;
  // optional k-contiguous FRAGMENT-ORDERED bf16 copy of one row-major [K][N] weight inside the segment (the rollout
  // fc product's B operand, fc_rollout.hip): element (k, n) at u16 ((k/16 * N/32 + n/32) * 64 + (k/8 % 2) * 32 +
  // n % 32) * 8 + k % 8. Its region is updated by a separate wave-item loop (see opt_body); kc_K == 0: none.
  int64_t kc_off = 0;
  int kc_K = 0, kc_N = 0;
  u16* kc_dst = nullptr;
  // optional device gate: the launch is skipped (no parameter, moment or step-count change) while *gate == 0 (lag-1
  // data parallelism before its first all-reduced gradient, trainer.py _update_body_lag1)
  const int* gate = nullptr;
  // optional ITEM TABLE (device, OPT_ITEM_WORDS int64 per item, built by ops/optim.py FusedGroupStep): the segment is
  // updated by one workgroup per item instead of the float4 sweep -- element ranges, 16-row x 64-column blocks of
  // MLP weights that also write the weight's fp32 fragment copies F / G (common.h) as whole 1 KB wave stores, and
  // small MLP weights whose copies are written per element. A workgroup reads its item with ONE scalar load; the
  // copy tables of the sweep path (write_trans) are searched per element through kernel-argument reads, which cost
  // more than the update itself at the MLP sizes (~4 us of a 9 us launch, profiles/r6_mlp_opt.txt).
  const int64_t* items = nullptr;
  int nitems = 0;
  // optional bf16 gradient read in place of g (the all-reduced comm buffer of bf16 DP buckets: no cast back to the
  // fp32 slab; zero_grad still clears g). The plain launch only (opt_kernel G16).
  const u16* g16 = nullptr;
  int64_t* stamps = nullptr;   // diagnostics: [global workgroup][8] s_memrealtime phase stamps (aca_opt_set_stamps)
  int wg0 = 0;                 // global index of the segment's first workgroup (stamps row)
};
constexpr int OPT_ITEM_WORDS = 8;   // type, e0, n / rows / K, N, F, G, F column-tile stride, unused

// element o (< K * N) of one copy entry
__device__ __forceinline__ bool write_one(const OptTrans& T, uint32_t o, float v) {
  // 32-bit division (a 64-bit one is a ~100-instruction software sequence per element)
  const uint32_t n = (uint32_t)T.N;
  const uint32_t k = o / n, c = o - k * n;
  if (T.ldt < 0) {
    const uint32_t f = (((k >> 4) * (n >> 5) + (c >> 5)) * 64u + ((c >> 3) & 3u) * 16u + (k & 15u)) * 8u + (c & 7u);
    reinterpret_cast<u16*>(T.dst)[f] = f2bf(v);
  } else {
    T.dst[(size_t)c * T.ldt + k] = v;
  }
  return true;
}

// (runtime-bound entry loops: the pong / breakout segments carry 1-4 entries; the MLP segments, whose per-element
// search through the kernel-argument table cost more than their update, take the item path instead)
__device__ __forceinline__ void write_trans(const OptSeg& S, size_t i, float v) {
  for (int e = 0; e < S.ntrans; ++e) {
    const OptTrans& T = S.tr[e];
    const int64_t o = (int64_t)i - T.off;
    if (o >= 0 && o < (int64_t)T.K * T.N) {
      write_one(T, (uint32_t)o, v);
      return;
    }
  }
}

// The four consecutive elements 4 * i4 .. + 3 of a float4 group: for a fragment-ordered copy (ldt -1, offset and N
// multiples of 4) they are 4 consecutive u16 of one lane's 8 -> ONE 8-byte store (one 32-bit index computation)
// instead of four 2-byte stores; other copies per element.
__device__ __forceinline__ void write_trans4(const OptSeg& S, size_t i4, float4 p4) {
  const size_t i = 4 * i4;
  for (int e = 0; e < S.ntrans; ++e) {
    const OptTrans& T = S.tr[e];
    const int64_t o = (int64_t)i - T.off;
    if (o + 3 >= 0 && o < (int64_t)T.K * T.N) {
      if (T.ldt < 0 && o >= 0 && o + 3 < (int64_t)T.K * T.N && ((o | T.N) & 3) == 0) {
        const uint32_t ou = (uint32_t)o, n = (uint32_t)T.N;
        const uint32_t k = ou / n, c = ou - k * n;
        const uint32_t f = (((k >> 4) * (n >> 5) + (c >> 5)) * 64u + ((c >> 3) & 3u) * 16u + (k & 15u)) * 8u + (c & 7u);
        uint2 pk;
        pk.x = (uint32_t)f2bf(p4.x) | ((uint32_t)f2bf(p4.y) << 16);
        pk.y = (uint32_t)f2bf(p4.z) | ((uint32_t)f2bf(p4.w) << 16);
        *reinterpret_cast<uint2*>(reinterpret_cast<u16*>(T.dst) + f) = pk;
        return;
      }
      write_trans(S, i, p4.x);
      write_trans(S, i + 1, p4.y);
      write_trans(S, i + 2, p4.z);
      write_trans(S, i + 3, p4.w);
      return;
    }
  }
}

// Adam step ticket (t_off < 0):
__device__ __forceinline__ void opt_ticket(const OptSeg& S, int vblk, int vgrid, float t) {
    // The last workgroup to finish publishes t + 1. Only a COUNT is needed (no data hand-off), so the ticket is a
    // relaxed atomic with no release fence: a fenced last-arriver ticket (last_block_arrival) costs every workgroup
    // an agent-scope release -- an L2 write-back on this multi-XCD part -- which was 60 us of a 70 us step over a
    // 1.7M-parameter slab. The barrier orders this workgroup's reads of *S.t (every wave, at its start) before its
    // ticket, so the final write cannot overtake a reader.
    // The ticket is sharded by workgroup % 8 (each shard counter on its own 128-byte line): one counter took ~12 ns
    // per arrival serialised in memory -- ~20 us over the 1650 workgroups of a 1.7M-parameter Adam step. A shard's
    // last arriver (told by the returned count) resets its counter and adds to the top counter; the last shard
    // publishes t + 1 and resets the top. Words: [x * OPT_TK_LINE] shards, [8 * OPT_TK_LINE] top.
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned int x = (unsigned int)vblk & 7u, G = (unsigned int)vgrid;
      const unsigned int nsh = G < 8u ? G : 8u, nx = (G - x + 7u) / 8u;
      const unsigned int prev =
          __hip_atomic_fetch_add(S.ticket + x * OPT_TK_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == nx - 1u) {
        __hip_atomic_store(S.ticket + x * OPT_TK_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned int done =
            __hip_atomic_fetch_add(S.ticket + 8 * OPT_TK_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done == nsh - 1u) {
          *S.t = t;
          __hip_atomic_store(S.ticket + 8 * OPT_TK_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
}

// ---- item path (OptSeg::items): one workgroup per item record of OPT_ITEM_WORDS int64:
//   type 0: elements [e0, e0 + n) (n <= 4 * OPT_THREADS; thread t: e0 + t + OPT_THREADS j, coalesced)
//   type 1: rows [0, w2) of the 16-row x 64-column block at element e0 of a [K][N] weight (N = w3, N % 64 == 0): wave
//           w updates rows 4 w + (lane >> 4), columns 4 (lane & 15) .. + 3 (whole 256-byte row runs), the new values
//           go through the workgroup's LDS tile, then wave w stores the 1 KB F block of column tile w (at
//           F = w4 + w * w6 floats) and the 1 KB G block (at G = w5 + 256 w floats, w5 = 0: none)
//   type 2: a whole small [K][N] weight at e0 (K = w2, N = w3, K * N <= 4 * OPT_THREADS), F / G written per element
template <bool ADAM>
__device__ __forceinline__ void opt_items(const OptSeg& S, float b1, float b2, float eps, int zero_grad, int vblk,
                                          int vgrid, float* shr, float* blks) {
  auto stamp = [&](int k) {
    if (S.stamps && threadIdx.x == 0) S.stamps[(size_t)(S.wg0 + vblk) * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  float* __restrict__ p = S.p;
  float* __restrict__ g = S.g;
  float* __restrict__ m = S.m;
  float* __restrict__ v = S.v;
  const int64_t* rec = S.items + (size_t)vblk * OPT_ITEM_WORDS;
  const int type = (int)rec[0];
  const int64_t e0 = rec[1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // ---- operands requested before the global-norm reduction
  float4 x4[4][4];   // [array g, v, p, m][j]: type 0 / 2 element j (scalars in .x), type 1 the thread's float4 in [0]
  const int n = (int)rec[2], N = (int)rec[3];
  int cnt = 0;       // elements (types 0, 2) or float4 (type 1) this thread owns
  auto elem = [&](int j) -> int64_t { return e0 + tid + (int64_t)OPT_THREADS * j; };
  if (type == 1) {
    const int r = 4 * w + (lane >> 4);
    if (r < n) {
      cnt = 1;
      const size_t i = (size_t)(e0 + (int64_t)r * N + 4 * (lane & 15)) / 4;
      x4[0][0] = reinterpret_cast<const float4*>(g)[i];
      x4[1][0] = reinterpret_cast<const float4*>(v)[i];
      x4[2][0] = reinterpret_cast<const float4*>(p)[i];
      x4[3][0] = ADAM ? reinterpret_cast<const float4*>(m)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  } else {
    const int tot = type == 0 ? n : n * N;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (tid + OPT_THREADS * j < tot) {
        cnt = j + 1;
        const int64_t i = elem(j);
        x4[0][j].x = g[i];
        x4[1][j].x = v[i];
        x4[2][j].x = p[i];
        x4[3][j].x = ADAM ? m[i] : 0.f;
      }
    }
  }
  stamp(1);
  const float lr = *S.lr;
  const float t = ADAM ? (*S.t + 1.0f + (S.t_off > 0 ? (float)S.t_off : 0.f)) : 0.f;
  float scale = 1.f;
  if (S.parts) {
    const float gsq = partial_total(S.parts, shr) * S.norm_mul;
    scale = grad_scale(gsq, S.max_norm);
    if (S.gnorm_out && vblk == 0 && tid == 0) *S.gnorm_out = gsq;
  }
  stamp(2);
  const float clip = S.clip, gmul = S.gmul;
  float lr_t = lr;
  if (ADAM) lr_t = lr * sqrtf(1.0f - powf(b2, t)) / (1.0f - powf(b1, t));
  // (the update arithmetic of opt_body, term for term: the two paths give bit-identical parameters)
  auto upd = [&](float gi, float& vi, float& mi, float& pi) {
    gi *= gmul;
    if (clip > 0.f) gi = fminf(fmaxf(gi, -clip), clip);
    gi *= scale;
    vi = __builtin_fmaf(1.0f - b2, gi * gi, b2 * vi);
    if (ADAM) {
      mi = __builtin_fmaf(1.0f - b1, gi, b1 * mi);
      pi = __builtin_fmaf(-lr_t, mi / (sqrtf(vi) + eps), pi);
    } else {
      pi = __builtin_fmaf(-lr, gi / sqrtf(vi + eps), pi);
    }
  };
  u16* shadow = S.shadow;
  if (type == 1) {
    float4 w4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const int r = 4 * w + (lane >> 4);
    if (cnt) {
      float4 &g4 = x4[0][0], &v4 = x4[1][0], &p4 = x4[2][0], &m4 = x4[3][0];
      const size_t i = (size_t)(e0 + (int64_t)r * N + 4 * (lane & 15)) / 4;
      if (zero_grad) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      upd(g4.x, v4.x, m4.x, p4.x);
      upd(g4.y, v4.y, m4.y, p4.y);
      upd(g4.z, v4.z, m4.z, p4.z);
      upd(g4.w, v4.w, m4.w, p4.w);
      reinterpret_cast<float4*>(v)[i] = v4;
      if (ADAM) reinterpret_cast<float4*>(m)[i] = m4;
      reinterpret_cast<float4*>(p)[i] = p4;
      if (shadow) {
        uint2 sv;
        sv.x = (uint32_t)f2bf(p4.x) | ((uint32_t)f2bf(p4.y) << 16);
        sv.y = (uint32_t)f2bf(p4.z) | ((uint32_t)f2bf(p4.w) << 16);
        reinterpret_cast<uint2*>(shadow)[i] = sv;
      }
      w4 = p4;
    }
    // (rows past K are zero: the fragment pads)
    *reinterpret_cast<float4*>(blks + r * BLK_LD + 4 * (lane & 15)) = w4;
    __syncthreads();
    const int rr = lane & 15, q = lane >> 4;
    float* G = reinterpret_cast<float*>(rec[5]);
    // G block of column tile w, lane (q, rr): W[rr][16 w + 4 q .. + 3]
    if (G)
      *reinterpret_cast<float4*>(G + 256 * w + 4 * lane) =
          *reinterpret_cast<const float4*>(blks + rr * BLK_LD + 16 * w + 4 * q);
    // F block of column tile w, lane (q, rr): W[4 q + s][16 w + rr], s = 0..3
    float4 f4;
    f4.x = blks[(4 * q + 0) * BLK_LD + 16 * w + rr];
    f4.y = blks[(4 * q + 1) * BLK_LD + 16 * w + rr];
    f4.z = blks[(4 * q + 2) * BLK_LD + 16 * w + rr];
    f4.w = blks[(4 * q + 3) * BLK_LD + 16 * w + rr];
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(rec[4]) + rec[6] * w + 4 * lane) = f4;
  } else {
    float* F = reinterpret_cast<float*>(rec[4]);
    float* G = reinterpret_cast<float*>(rec[5]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < cnt) {
        const int64_t i = elem(j);
        float &gi = x4[0][j].x, &vi = x4[1][j].x, &pi = x4[2][j].x, &mi = x4[3][j].x;
        if (zero_grad) g[i] = 0.f;
        upd(gi, vi, mi, pi);
        v[i] = vi;
        if (ADAM) m[i] = mi;
        p[i] = pi;
        if (shadow) shadow[i] = f2bf(pi);
        if (type == 2) {
          const uint32_t o = (uint32_t)(tid + OPT_THREADS * j), k = o / (uint32_t)N, c = o - k * (uint32_t)N;
          F[mlp_frag_f(k, c, n)] = pi;
          if (G) G[mlp_frag_g(k, c, N)] = pi;
        }
      }
    }
  }
  stamp(4);
  if (S.stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(5);
  }
  if (ADAM && S.t_off < 0) opt_ticket(S, vblk, vgrid, t);
}

// U float4 groups per thread per round; the first round's operands are requested BEFORE the global-norm reduction
// (its partial loads + block sum would otherwise be a dependent round trip ahead of every element load).
// ITEMS: the item path is compiled in (the grouped launch of the MLP optimisers); the plain launch leaves it out --
// its code and LDS tile raised the sweep's registers and cost the headline RMSprop step ~30 % (12.5 -> 16.3 us).
template <bool ADAM, int U, bool ITEMS, bool G16 = false>
__device__ __forceinline__ void opt_body(const OptSeg& S, float b1, float b2, float eps, int zero_grad, int vblk,
                                         int vgrid, int* flag, float* shr, u16* kcs, float* blks) {
  if (S.gate && *S.gate == 0) return;   // uniform over the launch
  if constexpr (ITEMS) {
    if (S.items) {
      opt_items<ADAM>(S, b1, b2, eps, zero_grad, vblk, vgrid, shr, blks);
      return;
    }
  }
  auto stamp = [&](int k) {
    if (S.stamps && threadIdx.x == 0) S.stamps[(size_t)(S.wg0 + vblk) * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  float* __restrict__ p = S.p;
  float* __restrict__ g = S.g;
  float* __restrict__ m = S.m;
  float* __restrict__ v = S.v;
  const size_t n = S.n;
  const float lr = *S.lr;
  const float t = ADAM ? (*S.t + 1.0f + (S.t_off > 0 ? (float)S.t_off : 0.f)) : 0.f;
  const size_t n4 = n / 4;
  const size_t stride = (size_t)vgrid * blockDim.x * U;
  // the k-contiguous fragment region [kc0, kc1) in float4 groups is left to the wave-item loop below
  const size_t kc0 = S.kc_K ? (size_t)S.kc_off / 4 : 0, kc1 = S.kc_K ? kc0 + (size_t)S.kc_K * S.kc_N / 4 : 0;
  auto in_kc = [&](size_t i) { return i >= kc0 && i < kc1; };
  float4 g4[U], v4[U], p4[U], m4[U];
  auto load = [&](size_t i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = i0 + (size_t)u * blockDim.x;
      if (i < n4 && !in_kc(i)) {
        g4[u] = G16 ? ld4(S.g16, i) : reinterpret_cast<const float4*>(g)[i];
        v4[u] = reinterpret_cast<const float4*>(v)[i];
        p4[u] = reinterpret_cast<const float4*>(p)[i];
        m4[u] = ADAM ? reinterpret_cast<const float4*>(m)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  size_t i0 = vblk * (size_t)blockDim.x * U + threadIdx.x;
  if (i0 < n4) load(i0);
  // wave items of the fragment region: (k octet kq, 32-column block nb); lane -> row kq * 8 + (lane & 7), columns
  // nb * 32 + 4 (lane >> 3) .. + 3 (a wave load: 8 rows x 128 bytes)
  const int lane = threadIdx.x & 63, nwv = blockDim.x >> 6;
  const int kNB = S.kc_N >> 5;
  const int kItems = S.kc_K ? (S.kc_K >> 3) * kNB : 0;
  const int gw0 = vblk * nwv + (threadIdx.x >> 6), GW = vgrid * nwv;
  auto kc_index = [&](int it) {
    const int kq = it / kNB, nb = it - kq * kNB;
    return kc0 + ((size_t)(kq * 8 + (lane & 7)) * S.kc_N + nb * 32 + 4 * (lane >> 3)) / 4;
  };
  float4 kg, kv, kp, km;
  auto kc_load = [&](int it) {
    const size_t i = kc_index(it);
    kg = G16 ? ld4(S.g16, i) : reinterpret_cast<const float4*>(g)[i];
    kv = reinterpret_cast<const float4*>(v)[i];
    kp = reinterpret_cast<const float4*>(p)[i];
    km = ADAM ? reinterpret_cast<const float4*>(m)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  if (gw0 < kItems) kc_load(gw0);
  stamp(1);
  float scale = 1.f;
  if (S.parts) {
    const float gsq = partial_total(S.parts, shr) * S.norm_mul;
    scale = grad_scale(gsq, S.max_norm);
    if (S.gnorm_out && vblk == 0 && threadIdx.x == 0) *S.gnorm_out = gsq;
  }
  stamp(2);
  const float clip = S.clip, gmul = S.gmul;
  float lr_t = lr;
  if (ADAM) lr_t = lr * sqrtf(1.0f - powf(b2, t)) / (1.0f - powf(b1, t));
  auto upd = [&](float gi, float& vi, float& mi, float& pi) {
    gi *= gmul;   // data parallelism: 1/world averaging of the summed gradient, folded in (no extra pass)
    if (clip > 0.f) gi = fminf(fmaxf(gi, -clip), clip);
    gi *= scale;
    // explicit fused multiply-adds: the rounding of the update is fixed by the source, not by how the compiler
    // contracts it around the surrounding loads (which moved with the load order and changed the last ulp)
    vi = __builtin_fmaf(1.0f - b2, gi * gi, b2 * vi);
    if (ADAM) {
      mi = __builtin_fmaf(1.0f - b1, gi, b1 * mi);
      pi = __builtin_fmaf(-lr_t, mi / (sqrtf(vi) + eps), pi);
    } else {
      pi = __builtin_fmaf(-lr, gi / sqrtf(vi + eps), pi);
    }
  };
  u16* shadow = S.shadow;
  // float4 body: all operand loads of a round are issued together (one memory round trip per round)
  for (; i0 < n4; i0 += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = i0 + (size_t)u * blockDim.x;
      if (i >= n4) break;
      if (in_kc(i)) continue;
      if (zero_grad) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      upd(g4[u].x, v4[u].x, m4[u].x, p4[u].x);
      upd(g4[u].y, v4[u].y, m4[u].y, p4[u].y);
      upd(g4[u].z, v4[u].z, m4[u].z, p4[u].z);
      upd(g4[u].w, v4[u].w, m4[u].w, p4[u].w);
      reinterpret_cast<float4*>(v)[i] = v4[u];
      if (ADAM) reinterpret_cast<float4*>(m)[i] = m4[u];
      reinterpret_cast<float4*>(p)[i] = p4[u];
      if (shadow) {
        uint2 sv;
        sv.x = (uint32_t)f2bf(p4[u].x) | ((uint32_t)f2bf(p4[u].y) << 16);
        sv.y = (uint32_t)f2bf(p4[u].z) | ((uint32_t)f2bf(p4[u].w) << 16);
        reinterpret_cast<uint2*>(shadow)[i] = sv;
      }
      if (S.ntrans) write_trans4(S, i, p4[u]);
    }
    if (i0 + stride < n4) load(i0 + stride);
  }
  stamp(3);
  // fragment region: the same update per element, then the bf16 copy transposed through a 512-byte per-wave LDS
  // scratch laid out exactly as the destination run ([32 columns][8 k]) -> one contiguous 512-byte wave store
  for (int it = gw0; it < kItems; it += GW) {
    const size_t i = kc_index(it);
    if (zero_grad) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    upd(kg.x, kv.x, km.x, kp.x);
    upd(kg.y, kv.y, km.y, kp.y);
    upd(kg.z, kv.z, km.z, kp.z);
    upd(kg.w, kv.w, km.w, kp.w);
    reinterpret_cast<float4*>(v)[i] = kv;
    if (ADAM) reinterpret_cast<float4*>(m)[i] = km;
    reinterpret_cast<float4*>(p)[i] = kp;
    const u16 h0 = f2bf(kp.x), h1 = f2bf(kp.y), h2 = f2bf(kp.z), h3 = f2bf(kp.w);
    if (shadow) {
      uint2 sv;
      sv.x = (uint32_t)h0 | ((uint32_t)h1 << 16);
      sv.y = (uint32_t)h2 | ((uint32_t)h3 << 16);
      reinterpret_cast<uint2*>(shadow)[i] = sv;
    }
    u16* ws = kcs + (threadIdx.x >> 6) * 256;
    const int r = lane & 7, c4 = lane >> 3;
    ws[(4 * c4 + 0) * 8 + r] = h0;
    ws[(4 * c4 + 1) * 8 + r] = h1;
    ws[(4 * c4 + 2) * 8 + r] = h2;
    ws[(4 * c4 + 3) * 8 + r] = h3;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint2 o = reinterpret_cast<const uint2*>(ws)[lane];
    const int kq = it / kNB, nb = it - kq * kNB;
    reinterpret_cast<uint2*>(S.kc_dst + ((size_t)(kq >> 1) * kNB + nb) * 512 + (kq & 1) * 256)[lane] = o;
    __builtin_amdgcn_wave_barrier();   // the scratch is rewritten by the next item
    if (it + GW < kItems) kc_load(it + GW);
  }
  stamp(4);
  if (vblk == 0) {   // scalar tail
    for (size_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) {
      float gi = G16 ? bf2f(S.g16[i]) : g[i], vi = v[i], pi = p[i], mi = ADAM ? m[i] : 0.f;
      if (zero_grad) g[i] = 0.f;
      upd(gi, vi, mi, pi);
      v[i] = vi;
      if (ADAM) m[i] = mi;
      p[i] = pi;
      if (shadow) shadow[i] = f2bf(pi);
      if (S.ntrans) write_trans(S, i, pi);
    }
  }
  if (S.stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(5);
  }
  if (ADAM && S.t_off < 0) opt_ticket(S, vblk, vgrid, t);
}

template <bool ADAM, int U, bool G16 = false>
__global__ void __launch_bounds__(OPT_THREADS) opt_kernel(OptSeg S, float b1, float b2, float eps, int zero_grad) {
  __shared__ int flag;
  __shared__ float shr[16];
  __shared__ __attribute__((aligned(16))) u16 kcs[OPT_THREADS / 64 * 256];
  opt_body<ADAM, U, false, G16>(S, b1, b2, eps, zero_grad, blockIdx.x, gridDim.x, &flag, shr, kcs, nullptr);
}

// Several parameter groups (e.g. the reference's separate actor and critic optimisers) in ONE launch: the grid is
// the concatenation of the groups' grids.
constexpr int OPT_MAXSEG = 4;
struct OptMulti {
  OptSeg seg[OPT_MAXSEG];
  int nseg;
};

template <bool ADAM>
__global__ void __launch_bounds__(OPT_THREADS) opt_multi_kernel(OptMulti M, float b1, float b2, float eps,
                                                                int zero_grad) {
  __shared__ int flag;
  __shared__ float shr[16];
  __shared__ __attribute__((aligned(16))) u16 kcs[OPT_THREADS / 64 * 256];
  __shared__ __attribute__((aligned(16))) float blks[16 * BLK_LD];
  int b = blockIdx.x, k = 0;
  while (k + 1 < M.nseg && b >= M.seg[k].nblocks) b -= M.seg[k++].nblocks;
  opt_body<ADAM, 1, true>(M.seg[k], b1, b2, eps, zero_grad, b, M.seg[k].nblocks, &flag, shr, kcs, blks);
}

// Gradient finaliser: the last step of a backward pass before the optimiser. Gradient segments are either
// already final (src == null: read for the norm only) or reductions of S partial planes in plane order -- split-K
// weight-gradient planes, per-sample bias-gradient rows -- dst[i] = sum_{z < S} src[z * stride + i]
// (deterministic: fixed order, no atomics). The host cuts the segments into at most SUMSQ_PARTS jobs (one per
// workgroup, sized so that no thread walks a long dependent chain of loads); every workgroup writes the sum of
// squares of its share of the final gradient into its own partial slot (the unused slots zeroed), which the
// optimiser reduces in a fixed order: the global-norm clip needs no separate sum-of-squares pass.
// Job record (8 int64 words): dst, src, n, stride, S, (unused x3). dst / src / stride are float4-aligned when the
// job's flag word 5 is 1 (host-checked). src = 0, S = -1: dst holds n presummed sums of squares (added, not squared).
constexpr int FIN_WORDS = 8;
constexpr int FIN_RND = 32;        // 16-byte loads per thread in flight in the many-plane reductions (was 16)
constexpr int FIN_RND_ROWS = 16;   // ... in the bias-row reduction (256 rows per round: one round for the headline's
                                   // 160 rows and for the 256 per-workgroup rows of the persistent backward)

// One finaliser job (record w) by the whole workgroup; returns this thread's share of the sum of squares of the
// final gradient. FUSED (the finaliser + optimiser kernel below): the final values go to `out` (LDS, job-local
// index) instead of the slab, and read-only segments are zeroed after the read (the optimiser's zero-after-use).
template <bool FUSED>
__device__ __forceinline__ float fin_job(const int64_t* __restrict__ w, float* __restrict__ out, float* red) {
  float* dst = reinterpret_cast<float*>(w[0]);
  const float* src = reinterpret_cast<const float*>(w[1]);
  const int n = (int)w[2], S = (int)w[4], vec = (int)w[5];
  const int64_t stride = w[3];
  const int tid = threadIdx.x;
  float s = 0.f;
  if (!src && S < 0) {
    // presummed: n sums of squares a producer already formed (fc_bwd's per-tile partials), added as they are
    for (int i = tid; i < n; i += OPT_THREADS) s += dst[i];
  } else if (!src) {
    if (vec) {   // read-only, 8 independent 16-byte loads per thread in flight
      const int n4 = n >> 2;
      for (int i0 = tid; i0 < n4; i0 += OPT_THREADS * 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + OPT_THREADS * u;
          v[u] = reinterpret_cast<const float4*>(dst)[i < n4 ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (i0 + OPT_THREADS * u < n4) {
            s += v[u].x * v[u].x + v[u].y * v[u].y + v[u].z * v[u].z + v[u].w * v[u].w;
            if constexpr (FUSED) {
              reinterpret_cast<float4*>(out)[i0 + OPT_THREADS * u] = v[u];
              reinterpret_cast<float4*>(dst)[i0 + OPT_THREADS * u] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
          }
      }
      for (int i = 4 * n4 + tid; i < n; i += OPT_THREADS) {
        const float v = dst[i];
        s += v * v;
        if constexpr (FUSED) { out[i] = v; dst[i] = 0.f; }
      }
    } else {
      for (int i = tid; i < n; i += OPT_THREADS) {
        const float v = dst[i];
        s += v * v;
        if constexpr (FUSED) { out[i] = v; dst[i] = 0.f; }
      }
    }
  } else if (n <= 64 && vec && (n & 3) == 0) {
    // few elements, many planes (per-sample bias rows, up to one per learner sample): 16 float4 columns x 16 plane
    // groups, FIN_RND_ROWS 16-byte loads in flight per thread (this reduction is latency-bound: one workgroup walks
    // B planes in B / (16 FIN_RND_ROWS) dependent rounds), groups combined in LDS in group order
    const int c4 = tid & 15, pg = tid >> 4, n4 = n >> 2;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 < n4) {
      for (int z0 = pg; z0 < S; z0 += 16 * FIN_RND_ROWS) {
        float4 v[FIN_RND_ROWS];
#pragma unroll
        for (int u = 0; u < FIN_RND_ROWS; ++u) {
          const int z = z0 + 16 * u;
          v[u] = *reinterpret_cast<const float4*>(src + (int64_t)(z < S ? z : pg) * stride + 4 * c4);
        }
#pragma unroll
        for (int u = 0; u < FIN_RND_ROWS; ++u)
          if (z0 + 16 * u < S) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
      }
    }
    float* red4 = red;   // [16 groups][64 elements]
    __syncthreads();
    if (c4 < n4) {
      red4[pg * 64 + 4 * c4] = acc.x;
      red4[pg * 64 + 4 * c4 + 1] = acc.y;
      red4[pg * 64 + 4 * c4 + 2] = acc.z;
      red4[pg * 64 + 4 * c4 + 3] = acc.w;
    }
    __syncthreads();
    if (tid < n) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) v += red4[g * 64 + tid];
      if constexpr (FUSED) out[tid] = v; else dst[tid] = v;
      s = v * v;
    }
  } else if (n <= 64) {
    // few elements, many planes (per-sample bias rows): 64 elements x 4 plane groups, 16 loads in flight per
    // thread, the groups combined in LDS in group order
    const int el = tid & 63, pg = tid >> 6;
    float acc = 0.f;
    if (el < n) {
      for (int z0 = pg; z0 < S; z0 += 64) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int z = z0 + 4 * u;
          v[u] = src[(int64_t)(z < S ? z : pg) * stride + el];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += (z0 + 4 * u < S) ? v[u] : 0.f;
      }
    }
    red[tid] = acc;
    __syncthreads();
    if (tid < n) {
      const float v = (red[tid] + red[64 + tid]) + (red[128 + tid] + red[192 + tid]);
      if constexpr (FUSED) out[tid] = v; else dst[tid] = v;
      s = v * v;
    }
  } else if (vec && S <= 4) {
    // few planes of many elements (a two-split fc weight gradient): 8 float4 elements x S planes per thread in
    // flight per round (one element at a time would be a dependent round trip per 2 loads); plane order per element
    const int n4 = n >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    const int64_t st4 = stride >> 2;
    for (int i0 = tid; i0 < n4; i0 += OPT_THREADS * 8) {
      float4 v[4][8];
#pragma unroll
      for (int z = 0; z < 4; ++z)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + OPT_THREADS * u;
          if (z < S) v[z][u] = s4[z * st4 + (i < n4 ? i : 0)];
        }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + OPT_THREADS * u;
        if (i < n4) {
          float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int z = 0; z < 4; ++z)
            if (z < S) { acc.x += v[z][u].x; acc.y += v[z][u].y; acc.z += v[z][u].z; acc.w += v[z][u].w; }
          if constexpr (FUSED) reinterpret_cast<float4*>(out)[i] = acc; else reinterpret_cast<float4*>(dst)[i] = acc;
          s += acc.x * acc.x + acc.y * acc.y + acc.z * acc.z + acc.w * acc.w;
        }
      }
    }
    for (int i = 4 * n4 + tid; i < n; i += OPT_THREADS) {
      float v = 0.f;
      for (int z = 0; z < S; ++z) v += src[(int64_t)z * stride + i];
      if constexpr (FUSED) out[i] = v; else dst[i] = v;
      s += v * v;
    }
  } else if (vec && S >= 16 && n <= 512 && (n & 3) == 0) {
    // many planes of a short chunk (the conv weight-gradient jobs cut at 256 / 512 elements so that more workgroups
    // stream the planes): the planes split into G contiguous ranges, one per thread group (G = 4 of 64 float4
    // columns, or 2 of 128), each walked in plane order with FIN_RND loads in flight, the G partial columns added in
    // group order through LDS
    const int n4 = n >> 2, G = n4 <= 64 ? 4 : 2, cols = OPT_THREADS / G;
    const int c4 = tid % cols, g = tid / cols;
    const int z_lo = (int)((int64_t)S * g / G), z_hi = (int)((int64_t)S * (g + 1) / G);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 < n4) {
      for (int z0 = z_lo; z0 < z_hi; z0 += FIN_RND) {
        float4 v[FIN_RND];
#pragma unroll
        for (int u = 0; u < FIN_RND; ++u) {
          const int z = z0 + u < z_hi ? z0 + u : z_lo;
          v[u] = *reinterpret_cast<const float4*>(src + (int64_t)z * stride + 4 * (int64_t)c4);
        }
#pragma unroll
        for (int u = 0; u < FIN_RND; ++u)
          if (z0 + u < z_hi) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
      }
    }
    float4* red4 = reinterpret_cast<float4*>(red);   // [G][cols] float4 (256 x 16 bytes)
    __syncthreads();
    red4[g * cols + c4] = acc;
    __syncthreads();
    if (tid < n4) {
      float4 v = red4[tid];
      for (int k = 1; k < G; ++k) {
        const float4 w = red4[k * cols + tid];
        v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
      }
      if constexpr (FUSED) reinterpret_cast<float4*>(out)[tid] = v; else reinterpret_cast<float4*>(dst)[tid] = v;
      s = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
  } else if (vec) {
    // planes, float4 elements: FIN_RND planes per round in flight (the rounds are dependent memory round trips: 8 of
    // them for a 256-plane conv weight gradient), elements striding over the workgroup; the adds run in plane order
    // whatever the round size
    constexpr int RND = FIN_RND;
    const int n4 = n >> 2;
    for (int i = tid; i < n4; i += OPT_THREADS) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int z0 = 0; z0 < S; z0 += RND) {
        float4 v[RND];
#pragma unroll
        for (int u = 0; u < RND; ++u) {
          const int z = z0 + u < S ? z0 + u : 0;
          v[u] = *reinterpret_cast<const float4*>(src + (int64_t)z * stride + 4 * (int64_t)i);
        }
#pragma unroll
        for (int u = 0; u < RND; ++u)
          if (z0 + u < S) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
      }
      if constexpr (FUSED) reinterpret_cast<float4*>(out)[i] = acc; else reinterpret_cast<float4*>(dst)[i] = acc;
      s += acc.x * acc.x + acc.y * acc.y + acc.z * acc.z + acc.w * acc.w;
    }
    for (int i = 4 * n4 + tid; i < n; i += OPT_THREADS) {
      float v = 0.f;
      for (int z = 0; z < S; ++z) v += src[(int64_t)z * stride + i];
      if constexpr (FUSED) out[i] = v; else dst[i] = v;
      s += v * v;
    }
  } else {
    for (int i = tid; i < n; i += OPT_THREADS) {
      float v = 0.f;
      for (int z = 0; z < S; ++z) v += src[(int64_t)z * stride + i];
      if constexpr (FUSED) out[i] = v; else dst[i] = v;
      s += v * v;
    }
  }
  return s;
}


// Statistics duty of the finaliser (one extra workgroup past the jobs): the per-env A2C statistics rows written by
// loss.hip a2c_head_env_kernel ([N][A2C_STATS] fp64 sums) combined in env order into stats[0..7] -- the same slots
// and formulas as a2c_head_kernel's (pg, kl, entropy, value loss, clip fraction 0, actor loss, ratio 1, EV-before).
struct StatsDuty {
  const double* part; int N, B;
  const float* ent_coef; const float* kl_coef;
  float* stats;
  int ppo;   // 1: the PPO head's records (ppo_head.hip, PH_NSTAT doubles per workgroup), else a2c_head_env's rows
};

// The large-batch PPO head's per-workgroup statistics records [N][PH_NSTAT] (pg, kl, entropy, value loss, clip
// fraction, ratio sums) -> stats[0..6], the head kernel's own formulas; taken here instead of by the head's
// last-arriving workgroup (whose ticket cost every head workgroup an agent-scope release). 32 lanes per statistic
// stride over the records, then lane order (fixed: deterministic).
constexpr int PPO_NSTAT = 6;
__device__ __forceinline__ void ppo_stats_duty(const StatsDuty& d) {
  __shared__ double part[PPO_NSTAT * 32];
  __shared__ double tot[PPO_NSTAT];
  const int tid = threadIdx.x, q = tid >> 5, l = tid & 31;
  if (q < PPO_NSTAT) {
    double v = 0.0;
    int e = l;
    for (; e + 96 < d.N; e += 128) {   // 4 loads in flight per lane
      const double a0 = d.part[(int64_t)e * PPO_NSTAT + q], a1 = d.part[(int64_t)(e + 32) * PPO_NSTAT + q];
      const double a2 = d.part[(int64_t)(e + 64) * PPO_NSTAT + q], a3 = d.part[(int64_t)(e + 96) * PPO_NSTAT + q];
      v += a0;
      v += a1;
      v += a2;
      v += a3;
    }
    for (; e < d.N; e += 32) v += d.part[(int64_t)e * PPO_NSTAT + q];
    part[q * 32 + l] = v;
  }
  __syncthreads();
  if (tid < PPO_NSTAT) {
    double v = 0.0;
    for (int j = 0; j < 32; ++j) v += part[tid * 32 + j];
    tot[tid] = v;
  }
  __syncthreads();
  if (tid == 0) {
    const double inv = 1.0 / d.B;
    const float beta = *d.kl_coef, c_ent = *d.ent_coef;
    const double pg = tot[0] * inv, kl = tot[1] * inv, H = tot[2] * inv;
    d.stats[0] = (float)pg;
    d.stats[1] = (float)kl;
    d.stats[2] = (float)H;
    d.stats[3] = (float)(tot[3] * inv);
    d.stats[4] = (float)(tot[4] * inv);
    d.stats[5] = (float)(pg + beta * kl - c_ent * H);
    d.stats[6] = (float)(tot[5] * inv);
  }
}

__device__ __forceinline__ void a2c_stats_duty(const StatsDuty& d) {
  // 9 statistics x 16 lanes (thread 16 q + l: records l, l + 16, ...; all of a lane's loads in flight together), then
  // the 16 lane partials in lane order (fixed: deterministic)
  __shared__ double part[9 * 16];
  __shared__ double tot[A2C_STATS];
  const int tid = threadIdx.x, q = tid >> 4, l = tid & 15;
  if (q < 9) {
    double v = 0.0;
    int e = l;
    for (; e + 48 < d.N; e += 64) {
      const double a0 = d.part[(int64_t)e * A2C_STATS + q], a1 = d.part[(int64_t)(e + 16) * A2C_STATS + q];
      const double a2 = d.part[(int64_t)(e + 32) * A2C_STATS + q], a3 = d.part[(int64_t)(e + 48) * A2C_STATS + q];
      v += a0;
      v += a1;
      v += a2;
      v += a3;
    }
    for (; e < d.N; e += 16) v += d.part[(int64_t)e * A2C_STATS + q];
    part[q * 16 + l] = v;
  }
  __syncthreads();
  if (tid < 9) {
    double v = 0.0;
    for (int j = 0; j < 16; ++j) v += part[tid * 16 + j];
    tot[tid] = v;
  }
  __syncthreads();
  if (tid == 0) {
    const double inv = 1.0 / d.B;
    const float beta = *d.kl_coef, c_ent = *d.ent_coef;
    d.stats[0] = (float)(tot[0] * inv);
    d.stats[1] = (float)(tot[1] * inv);
    d.stats[2] = (float)(tot[2] * inv);
    d.stats[3] = (float)(tot[3] * inv);
    d.stats[4] = 0.f;
    d.stats[5] = (float)(tot[0] * inv + beta * tot[1] * inv - c_ent * tot[2] * inv);
    d.stats[6] = 1.f;
    const double mr = tot[4] * inv, mv = tot[6] * inv;
    const double vr = fmax(tot[5] * inv - mr * mr, 0.0), vv = fmax(tot[7] * inv - mv * mv, 0.0);
    d.stats[7] = (float)((tot[8] * inv - mr * mv) / sqrt(vr * vv));
  }
}

__global__ void __launch_bounds__(OPT_THREADS) grad_finalize_kernel(const int64_t* __restrict__ jobs, int njobs,
                                                                    float* __restrict__ partial, StatsDuty sd) {
  __shared__ float sh[16];
  __shared__ __attribute__((aligned(16))) float red[16 * 64];
  if ((int)blockIdx.x == njobs) {   // past the jobs: the statistics duty (its partial slot is zeroed by workgroup 0)
    if (sd.ppo) ppo_stats_duty(sd);
    else a2c_stats_duty(sd);
    return;
  }
  float s = fin_job<false>(jobs + (int64_t)blockIdx.x * FIN_WORDS, nullptr, red);
  if (blockIdx.x == 0)
    for (int b = njobs + threadIdx.x; b < SUMSQ_PARTS; b += OPT_THREADS) partial[b] = 0.f;
  s = block_sum(s, sh);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// lag-1 data parallelism: dst <- src, src <- 0 in one pass (the next backward accumulates into a clean slab while
// dst is all-reduced and consumed by the next optimiser step)
// lag-1 data parallelism: C <- G, G <- 0; `gate` (optional) is set to 1 -- C now holds a gradient the next
// optimiser launch gated on it may apply (OptSeg::gate)
// zero: clear src behind the copy (off when the next backward STORES every gradient element)
__global__ void __launch_bounds__(OPT_THREADS) grad_move_kernel(float* __restrict__ src, float* __restrict__ dst,
                                                                size_t n, int* __restrict__ gate, int zero) {
  if (gate && blockIdx.x == 0 && threadIdx.x == 0) *gate = 1;
  const size_t n4 = n / 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(src)[i];
    if (zero) reinterpret_cast<float4*>(src)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    reinterpret_cast<float4*>(dst)[i] = v;
  }
  if (blockIdx.x == 0)
    for (size_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) {
      dst[i] = src[i];
      if (zero) src[i] = 0.f;
    }
}

// fp32 -> bf16 (the comm buffer of bf16 DP buckets): one thread per 4 elements (a 16-byte load, an 8-byte store) when
// both ends are aligned, else one per element -- a single memory round trip per thread (a grid-stride loop of
// 4-byte loads was one dependent round trip per element)
__global__ void cast_bf16_kernel(const float* __restrict__ x, u16* __restrict__ y, size_t n, int vec) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (vec) {
    const size_t n4 = n / 4;
    if (t < n4) {
      const float4 v = reinterpret_cast<const float4*>(x)[t];
      uint2 o;
      o.x = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
      o.y = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
      reinterpret_cast<uint2*>(y)[t] = o;
    }
    if (t < n - n4 * 4) y[n4 * 4 + t] = f2bf(x[n4 * 4 + t]);
  } else if (t < n) {
    y[t] = f2bf(x[t]);
  }
}

static int opt_grid(size_t n, int unroll = 1) {   // `unroll` float4 groups per thread (up to 16M parameters per pass)
  size_t b = (n / 4 + (size_t)OPT_THREADS * unroll - 1) / ((size_t)OPT_THREADS * unroll);
  if (b < 1) b = 1;
  if (b > 16384) b = 16384;
  return (int)b;
}

// float4 groups per thread of the single-segment optimiser launches (a diagnostic knob, aca_opt_set_unroll)
static int g_opt_unroll = 1;
static int64_t* g_opt_stamps = nullptr;

template <bool ADAM>
static void launch_opt(OptSeg& S, float b1, float b2, float eps, int zero_grad, hipStream_t stream) {
  const int U = g_opt_unroll;
  S.nblocks = opt_grid(S.n, U);
  if (S.g16) {
    S.nblocks = opt_grid(S.n, 1);
    opt_kernel<ADAM, 1, true><<<S.nblocks, OPT_THREADS, 0, stream>>>(S, b1, b2, eps, zero_grad);
    return;
  }
  switch (U) {
    case 2: opt_kernel<ADAM, 2><<<S.nblocks, OPT_THREADS, 0, stream>>>(S, b1, b2, eps, zero_grad); break;
    case 4: opt_kernel<ADAM, 4><<<S.nblocks, OPT_THREADS, 0, stream>>>(S, b1, b2, eps, zero_grad); break;
    default: opt_kernel<ADAM, 1><<<S.nblocks, OPT_THREADS, 0, stream>>>(S, b1, b2, eps, zero_grad); break;
  }
}

}  // namespace aca

using namespace aca;

// x: fp32, or bf16 (the all-reduced comm buffer of bf16 gradient buckets) when bf16 != 0
extern "C" hipError_t aca_sumsq(const void* x, size_t n, float* partial, int bf16, hipStream_t stream) {
  if (reinterpret_cast<uintptr_t>(x) % (bf16 ? 8 : 16)) return hipErrorInvalidValue;
  int grid = (int)((n / 4 + OPT_THREADS * SUMSQ_U - 1) / (OPT_THREADS * SUMSQ_U));
  if (grid < 1) grid = 1;
  if (grid > SUMSQ_PARTS) grid = SUMSQ_PARTS;
  if (bf16) sumsq_kernel<u16><<<grid, OPT_THREADS, 0, stream>>>(static_cast<const u16*>(x), n, partial);
  else sumsq_kernel<float><<<grid, OPT_THREADS, 0, stream>>>(static_cast<const float*>(x), n, partial);
  return hipGetLastError();
}

extern "C" int aca_sumsq_parts() { return SUMSQ_PARTS; }

extern "C" hipError_t aca_sumsq_multi(const float* const* xs, const size_t* ns, float* const* partials, int nseg,
                                      hipStream_t stream) {
  if (nseg < 1 || nseg > 4) return hipErrorInvalidValue;
  SumsqSegs a{};
  int gx = 1;
  for (int g = 0; g < nseg; ++g) {
    if (reinterpret_cast<uintptr_t>(xs[g]) % 16) return hipErrorInvalidValue;
    int grid = (int)((ns[g] / 4 + OPT_THREADS * SUMSQ_MU - 1) / (OPT_THREADS * SUMSQ_MU));
    if (grid < 1) grid = 1;
    if (grid > SUMSQ_PARTS) grid = SUMSQ_PARTS;
    a.x[g] = xs[g];
    a.n[g] = ns[g];
    a.partial[g] = partials[g];
    a.nblk[g] = grid;
    gx = grid > gx ? grid : gx;
  }
  sumsq_multi_kernel<<<dim3(gx, nseg), OPT_THREADS, 0, stream>>>(a);
  return hipGetLastError();
}

// jobs: device int64 [njobs, FIN_WORDS] (built by the host, ops/optim.py finalize_jobs); partial: SUMSQ_PARTS floats
extern "C" hipError_t aca_grad_finalize(const int64_t* jobs, int njobs, float* partial, const double* spart, int sN,
                                        int sB, const float* ent_coef, const float* kl_coef, float* stats, int sppo,
                                        hipStream_t stream) {
  if (njobs < 1 || njobs > SUMSQ_PARTS) return hipErrorInvalidValue;
  if (spart && (sN < 1 || sB < 1 || !ent_coef || !kl_coef || !stats)) return hipErrorInvalidValue;
  const StatsDuty sd{spart, sN, sB, ent_coef, kl_coef, stats, sppo};
  grad_finalize_kernel<<<njobs + (spart ? 1 : 0), OPT_THREADS, 0, stream>>>(jobs, njobs, partial, sd);
  return hipGetLastError();
}

// trans: host table [OPT_MAXT][5] = (offset, K, N, ldt, dst) of one segment; K == 0 ends the list. ldt -1: the
// conv kernels' fragment order (write_trans); ldt -2: the k-contiguous fragment region (at most one; opt_body);
// ldt -9 (K = N = 1, at most one): dst is the launch's gate (const int*, OptSeg::gate). (The MLP engine's fragment
// copies go through the item table, OptSeg::items.)
static bool opt_load_trans(OptSeg& S, const int64_t* tw0) {
  S.ntrans = 0;
  S.kc_K = 0;
  S.gate = nullptr;
  if (!tw0) return true;
  for (int e = 0; e < OPT_MAXT; ++e) {
    const int64_t* tw = tw0 + (int64_t)e * 5;
    if (tw[1] <= 0) break;
    const int64_t ldt = tw[3];
    if (ldt == -9) {
      if (S.gate || !tw[4] || tw[4] % 4) return false;
      S.gate = reinterpret_cast<const int*>(tw[4]);
      continue;
    }
    if ((ldt == -1 || ldt == -2) && (tw[1] % 16 || tw[2] % 32)) return false;   // 16-row tiles, 32-wide k-steps
    if (ldt < -2 || ldt == 0 || tw[0] < 0 || (size_t)(tw[0] + tw[1] * tw[2]) > S.n || tw[2] <= 0) return false;
    if (ldt == -2) {
      if (S.kc_K || tw[0] % 4 || tw[4] % 16) return false;
      S.kc_off = tw[0];
      S.kc_K = (int)tw[1];
      S.kc_N = (int)tw[2];
      S.kc_dst = reinterpret_cast<u16*>(tw[4]);
      continue;
    }
    S.tr[S.ntrans++] = OptTrans{tw[0], (int)tw[1], (int)tw[2], (int)ldt, reinterpret_cast<float*>(tw[4])};
  }
  return true;
}

static bool opt_aligned(const float* p, const float* g, const float* m, const float* v, const uint16_t* shadow) {
  return !((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
            reinterpret_cast<uintptr_t>(v)) % 16 || reinterpret_cast<uintptr_t>(shadow) % 8);
}

extern "C" hipError_t aca_adam_step(float* p, float* g, float* m, float* v, size_t n, const float* lr,
                                    float* t, const float* gnorm_parts, float* gnorm_out, uint16_t* shadow, float b1, float b2, float eps,
                                    float clip, float max_norm, unsigned int* ticket, int zero_grad,
                                    float gmul, float norm_mul, const int64_t* trans, const uint16_t* g16,
                                    hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (!opt_aligned(p, g, m, v, shadow) || reinterpret_cast<uintptr_t>(g16) % 8) return hipErrorInvalidValue;
  OptSeg S{p, g, m, v, n, lr, t, gnorm_parts, gnorm_out, shadow, clip, max_norm, gmul, norm_mul, ticket, opt_grid(n),
           0, {}};
  S.g16 = g16;
  if (!ticket || !t) return hipErrorInvalidValue;
  if (!opt_load_trans(S, trans)) return hipErrorInvalidValue;
  launch_opt<true>(S, b1, b2, eps, zero_grad, stream);
  return hipGetLastError();
}

extern "C" hipError_t aca_rmsprop_step(float* p, float* g, float* v, size_t n, const float* lr,
                                       const float* gnorm_parts, float* gnorm_out, uint16_t* shadow, float alpha, float eps, float clip,
                                       float max_norm, int zero_grad, float gmul, float norm_mul,
                                       const int64_t* trans, const uint16_t* g16, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (!opt_aligned(p, g, v, v, shadow) || reinterpret_cast<uintptr_t>(g16) % 8) return hipErrorInvalidValue;
  OptSeg S{p, g, nullptr, v, n, lr, nullptr, gnorm_parts, gnorm_out, shadow, clip, max_norm, gmul, norm_mul, nullptr,
           opt_grid(n), 0, {}};
  S.g16 = g16;
  if (!opt_load_trans(S, trans)) return hipErrorInvalidValue;
  launch_opt<false>(S, 0.f, alpha, eps, zero_grad, stream);
  return hipGetLastError();
}

// Multi-group step. words: nseg records of OPT_MULTI_WORDS (see ops/optim.py FusedGroupStep): p, g, m, v, n, lr, t,
// parts, gnorm_out, shadow, ticket, items, nitems (pointers / sizes as 64-bit words); fvals: clip, max_norm, gmul,
// norm_mul (floats). The item tables (OptSeg::items) are the caller's, validated where they are built.
constexpr int OPT_MULTI_WORDS = 13;
extern "C" hipError_t aca_opt_multi(const int64_t* words, const float* fvals, const int64_t* trans, int nseg,
                                    int adam, float b1, float b2, float eps, int zero_grad, int t_off,
                                    hipStream_t stream) {
  if (nseg < 1 || nseg > OPT_MAXSEG) return hipErrorInvalidValue;
  OptMulti M{};
  M.nseg = nseg;
  int total = 0;
  for (int k = 0; k < nseg; ++k) {
    const int64_t* w = words + OPT_MULTI_WORDS * k;
    const float* f = fvals + 4 * k;
    OptSeg& S = M.seg[k];
    S.p = reinterpret_cast<float*>(w[0]);
    S.g = reinterpret_cast<float*>(w[1]);
    S.m = reinterpret_cast<float*>(w[2]);
    S.v = reinterpret_cast<float*>(w[3]);
    S.n = (size_t)w[4];
    S.lr = reinterpret_cast<const float*>(w[5]);
    S.t = reinterpret_cast<float*>(w[6]);
    S.parts = reinterpret_cast<const float*>(w[7]);
    S.gnorm_out = reinterpret_cast<float*>(w[8]);
    S.shadow = reinterpret_cast<u16*>(w[9]);
    S.ticket = reinterpret_cast<unsigned int*>(w[10]);
    S.clip = f[0];
    S.max_norm = f[1];
    S.gmul = f[2];
    S.norm_mul = f[3];
    S.t_off = t_off < 0 ? -1 : t_off;
    S.stamps = g_opt_stamps;
    S.items = reinterpret_cast<const int64_t*>(w[11]);
    S.nitems = (int)w[12];
    if ((S.items != nullptr) != (S.nitems > 0) || S.nitems > 4096) return hipErrorInvalidValue;
    if (S.n == 0 || !opt_aligned(S.p, S.g, adam ? S.m : S.v, S.v, S.shadow)) return hipErrorInvalidValue;
    if (adam && (!S.m || !S.t || !S.ticket)) return hipErrorInvalidValue;
    // trans: [nseg][OPT_MAXT][5]
    if (!opt_load_trans(S, trans ? trans + (int64_t)k * OPT_MAXT * 5 : nullptr)) return hipErrorInvalidValue;
    S.nblocks = S.items ? S.nitems : opt_grid(S.n);   // item path: one workgroup per item
    S.wg0 = total;
    total += S.nblocks;
  }
  if (adam) opt_multi_kernel<true><<<total, OPT_THREADS, 0, stream>>>(M, b1, b2, eps, zero_grad);
  else opt_multi_kernel<false><<<total, OPT_THREADS, 0, stream>>>(M, 0.f, b2, eps, zero_grad);
  return hipGetLastError();
}

extern "C" void aca_opt_set_stamps(int64_t* p) { g_opt_stamps = p; }

extern "C" int aca_opt_set_unroll(int u) {
  if (u == 1 || u == 2 || u == 4) g_opt_unroll = u;
  return g_opt_unroll;
}

extern "C" hipError_t aca_grad_move(float* src, float* dst, size_t n, int* gate, int zero, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) % 16) return hipErrorInvalidValue;
  grad_move_kernel<<<opt_grid(n), OPT_THREADS, 0, stream>>>(src, dst, n, gate, zero);
  return hipGetLastError();
}

extern "C" hipError_t aca_cast_bf16(const float* x, uint16_t* y, size_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const int vec = (reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(y) % 8 == 0) ? 1 : 0;
  const size_t threads = vec ? (n / 4 > 0 ? n / 4 : 1) : n;
  cast_bf16_kernel<<<(unsigned)((threads + OPT_THREADS - 1) / OPT_THREADS), OPT_THREADS, 0, stream>>>(x, y, n, vec);
  return hipGetLastError();
}
