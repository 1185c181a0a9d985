// Atari-shaped env bank (Pong-like game rendered to 84x84 uint8), BASELINE.json headline config.
//
// One 256-thread workgroup per env: thread 0 advances the 4 physics sub-steps (frameskip 4) and handles the
// auto-reset, then the whole workgroup renders the new 84x84 frame straight into the output stack with 16-byte
// stores and shifts the previous 3 frames in (frame stack [N, k, 84, 84]); finished envs get k copies of their
// first frame (Framer padding rule, Basic_AC/run_AC.py:37-40). Oracle: envs/atari.py (compiled with
// -ffp-contract=off so the physics rounds exactly like the PyTorch oracle).
#include "common.h"
#include "cnn_head.h"

namespace aca {

constexpr int PH = 84, PW = 84, FRAME = PH * PW;  // 7056 bytes = 441 x 16 B
constexpr float FIELD_TOP = 10.0f, FIELD_BOT = 74.0f, BALL = 2.0f, PADDLE_H = 8.0f, PADDLE_W = 2.0f;
constexpr float AGENT_X = 74.0f, OPP_X = 8.0f, AGENT_SPEED = 2.0f, OPP_SPEED = 1.25f, BALL_VX = 1.5f;
constexpr float WIN_SCORE = 21.0f;
constexpr uint8_t BG = 87, WALL = 236, OPP_C = 130, AGENT_C = 200, BALL_C = 255;

struct PongState {
  float bx, by, vx, vy, pa, po, sa, so;
};

__device__ __forceinline__ void serve(PongState& s, uint32_t seed, uint32_t id, uint32_t st, uint32_t stream0) {
  float u0 = uniform01(seed, id, st, stream0);
  float u1 = uniform01(seed, id, st, stream0 + 1);
  float u2 = uniform01(seed, id, st, stream0 + 2);
  s.bx = 41.0f;
  s.by = 30.0f + u0 * 24.0f;
  s.vx = (u1 < 0.5f) ? BALL_VX : -BALL_VX;
  s.vy = (u2 - 0.5f) * 2.0f;
}

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// optional phase timestamps (s_memrealtime, 100 MHz), [gridDim.x, 16]; null in production
__device__ __forceinline__ void stamp_if(uint64_t* st, int slot, bool who) {
  if (st && who) st[(size_t)blockIdx.x * 16 + slot] = __builtin_amdgcn_s_memrealtime();
}

struct PongIO {
  float* state; int32_t* tsteps; int64_t* tglob; float* ep_ret; float* ep_stats; const int64_t* env_ids;
  const uint8_t* prev; uint8_t* out; float* reward; uint8_t* done_out; uint8_t* trunc_out;
  uint32_t seed; int max_steps; int k;
};

// Result of advancing env `e` by one agent step (4 physics sub-steps) -- computed from global state without writing
// anything, so the fused rollout kernel can evaluate all three paddle directions while the policy is still sampling.
struct PongOut {
  PongState s;
  float rew, er;
  int t, done, trunc;
};

__device__ __forceinline__ int pong_dir_index(int a) {  // 0: up, 1: stay, 2: down (dirn = index - 1)
  return (a == 2 || a == 4) ? 0 : ((a == 3 || a == 5) ? 2 : 1);
}

__device__ __forceinline__ PongOut pong_advance(const PongIO& io, int e, float dirn) {
  const float* sp = io.state + (size_t)e * 8;
  PongState s{sp[0], sp[1], sp[2], sp[3], sp[4], sp[5], sp[6], sp[7]};
  const int64_t tg = io.tglob[e] + 1;
  const uint32_t id = (uint32_t)io.env_ids[e], st = (uint32_t)tg;
  float rew = 0.0f;
  const float lo = FIELD_TOP + PADDLE_H / 2, hi = FIELD_BOT - PADDLE_H / 2;
  for (int sub = 0; sub < 4; ++sub) {
    float bx = s.bx, by = s.by, vx = s.vx, vy = s.vy, pa = s.pa, po = s.po;
    pa = clampf(pa + dirn * AGENT_SPEED, lo, hi);
    po = clampf(po + clampf(by + 1.0f - po, -OPP_SPEED, OPP_SPEED), lo, hi);
    bx = bx + vx;
    by = by + vy;
    if (by < FIELD_TOP) { by = 2 * FIELD_TOP - by; vy = -vy; }
    if (by > FIELD_BOT - BALL) { by = 2 * (FIELD_BOT - BALL) - by; vy = -vy; }
    bool hit_a = (vx > 0) && (bx + BALL >= AGENT_X) && (bx + BALL - vx < AGENT_X) &&
                 (fabsf(by + 1.0f - pa) <= PADDLE_H / 2 + 1.0f);
    if (hit_a) { vy = clampf(vy + 0.25f * (by + 1.0f - pa), -2.0f, 2.0f); bx = AGENT_X - BALL; vx = -vx; }
    const float edge = OPP_X + PADDLE_W;
    bool hit_o = (vx < 0) && (bx <= edge) && (bx - vx > edge) && (fabsf(by + 1.0f - po) <= PADDLE_H / 2 + 1.0f);
    if (hit_o) { vy = clampf(vy + 0.25f * (by + 1.0f - po), -2.0f, 2.0f); bx = edge; vx = -vx; }
    bool miss_a = bx > (float)PW;
    bool miss_o = bx < -BALL;
    rew = rew + (miss_o ? 1.0f : 0.0f) - (miss_a ? 1.0f : 0.0f);
    s.sa = s.sa + (miss_o ? 1.0f : 0.0f);
    s.so = s.so + (miss_a ? 1.0f : 0.0f);
    s.bx = bx; s.by = by; s.vx = vx; s.vy = vy; s.pa = pa; s.po = po;
    if (miss_a || miss_o) serve(s, io.seed, id, st, 200 + 4 * sub);
  }
  PongOut r;
  const bool term = (s.sa >= WIN_SCORE) || (s.so >= WIN_SCORE);
  r.t = io.tsteps[e] + 1;
  r.trunc = (r.t >= io.max_steps) && !term;
  r.done = term || r.trunc;
  r.rew = rew;
  r.er = io.ep_ret[e] + rew;
  if (r.done) {
    const float mid = 0.5f * (FIELD_TOP + FIELD_BOT);
    s.pa = mid; s.po = mid; s.sa = 0.0f; s.so = 0.0f;
    serve(s, io.seed, id, st, 100);
  }
  r.s = s;
  return r;
}

// Writes the chosen outcome back (one thread). tg_old: the env's global step counter, when the caller already holds
// it (saves a dependent load round trip at the end of the fused step).
__device__ __forceinline__ void pong_commit(const PongIO& io, int e, const PongOut& r, int64_t tg_old = -1) {
  io.tglob[e] = (tg_old >= 0 ? tg_old : io.tglob[e]) + 1;
  io.reward[e] = r.rew;
  io.done_out[e] = r.done;
  io.trunc_out[e] = r.trunc;
  if (r.done) {
    atomicAdd(&io.ep_stats[0], r.er);
    atomicAdd(&io.ep_stats[1], 1.0f);
    atomicAdd(&io.ep_stats[2], (float)r.t);
  }
  io.tsteps[e] = r.done ? 0 : r.t;
  io.ep_ret[e] = r.done ? 0.0f : r.er;
  float* sp = io.state + (size_t)e * 8;
  const PongState& s = r.s;
  sp[0] = s.bx; sp[1] = s.by; sp[2] = s.vx; sp[3] = s.vy; sp[4] = s.pa; sp[5] = s.po; sp[6] = s.sa; sp[7] = s.so;
}

// Frame-stack shift out[0..k-2] = prev[1..k-1] by threads [t0, t0 + nt): independent of the action, so the fused
// kernel overlaps it with the policy head. The 4 loads of a round are issued (clamped addresses, unconditional)
// before its guarded stores. Named registers, not a guarded uint4 array: hipcc put that array in scratch (144 B/lane).
__device__ __forceinline__ void pong_shift(const PongIO& io, int e, int t0, int nt) {
  const int k = io.k;
  const uint4* src = reinterpret_cast<const uint4*>(io.prev + (size_t)e * k * FRAME + FRAME);
  uint4* dst = reinterpret_cast<uint4*>(io.out + (size_t)e * k * FRAME);
  const int n16 = (k - 1) * FRAME / 16;
  const int tid = threadIdx.x - t0;
  for (int j0 = tid; j0 < n16; j0 += 4 * nt) {
    const int j1 = j0 + nt, j2 = j0 + 2 * nt, j3 = j0 + 3 * nt;
    const uint4 v0 = src[j0];
    const uint4 v1 = src[min(j1, n16 - 1)];
    const uint4 v2 = src[min(j2, n16 - 1)];
    const uint4 v3 = src[min(j3, n16 - 1)];
    dst[j0] = v0;
    if (j1 < n16) dst[j1] = v1;
    if (j2 < n16) dst[j2] = v2;
    if (j3 < n16) dst[j3] = v3;
  }
}

// Render the newest frame (441 chunks of 16 pixels); a finished env gets k copies of its first frame (Framer padding,
// Basic_AC/run_AC.py:37-40) -- these stores overwrite the shifted frames, so call after a barrier that follows
// pong_shift.
__device__ __forceinline__ void pong_render(const PongIO& io, int e, const PongState& s, bool done) {
  // 4-pixel words, 21 per row: wall rows are uniform, and only the words that overlap a paddle or the ball need
  // per-pixel tests (one 4-byte store per word, consecutive lanes -> consecutive words)
  constexpr int WPR = PW / 4, NWORDS = PH * WPR;   // 21, 1764
  const int k = io.k;
  const int pa0 = (int)floorf(s.pa - PADDLE_H / 2), po0 = (int)floorf(s.po - PADDLE_H / 2);
  const int bx0 = (int)floorf(s.bx), by0 = (int)floorf(s.by);
  uint32_t* ov = reinterpret_cast<uint32_t*>(io.out + (size_t)e * k * FRAME);
  for (int w = threadIdx.x; w < NWORDS; w += blockDim.x) {
    const int y = w / WPR, x0 = (w - y * WPR) * 4;
    uint32_t word;
    if (y < (int)FIELD_TOP || y >= (int)FIELD_BOT) {
      word = WALL * 0x01010101u;
    } else {
      const bool agent = y >= pa0 && y < pa0 + (int)PADDLE_H && x0 + 4 > (int)AGENT_X &&
                         x0 < (int)(AGENT_X + PADDLE_W);
      const bool opp = y >= po0 && y < po0 + (int)PADDLE_H && x0 + 4 > (int)OPP_X && x0 < (int)(OPP_X + PADDLE_W);
      const bool ball = y >= by0 && y < by0 + (int)BALL && x0 + 4 > bx0 && x0 < bx0 + (int)BALL;
      word = BG * 0x01010101u;
      if (agent || opp || ball) {
        word = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int x = x0 + q;
          uint32_t v = BG;
          if (agent && x >= (int)AGENT_X && x < (int)(AGENT_X + PADDLE_W)) v = AGENT_C;
          if (opp && x >= (int)OPP_X && x < (int)(OPP_X + PADDLE_W)) v = OPP_C;
          if (ball && x >= bx0 && x < bx0 + (int)BALL) v = BALL_C;
          word |= v << (8 * q);
        }
      }
    }
    ov[(size_t)(k - 1) * NWORDS + w] = word;
    if (done)
      for (int s2 = 0; s2 < k - 1; ++s2) ov[(size_t)s2 * NWORDS + w] = word;
  }
}

// One env step per workgroup with known actions: thread 0 runs the physics while the others shift the stack.
__global__ void __launch_bounds__(256) pong_step_kernel(PongIO io, const int32_t* __restrict__ actions) {
  const int e = blockIdx.x;
  __shared__ PongOut sh;
  if (threadIdx.x == 0) {
    const int a = actions[e];
    sh = pong_advance(io, e, (float)(pong_dir_index(a) - 1));
    pong_commit(io, e, sh);
  }
  pong_shift(io, e, 0, blockDim.x);
  __syncthreads();
  const PongOut r = sh;
  pong_render(io, e, r.s, r.done != 0);
}

constexpr int HEAD_HDIM = 512;                       // hidden width of the Nature-CNN trunk

// Rollout step of the native engine fused with the env: the policy/value head (z = h.Wh + bh, 512 -> A+1) of
// env e, Gumbel-max sampling with the env-counter RNG key, logp / entropy / value, then the env step with the
// sampled action -- one launch instead of head GEMM + sampling + env kernels. The head uses the whole workgroup:
// thread t owns hidden units 2t, 2t+1 (reduced from the fc GEMM's split-K partial planes, every plane's load in
// flight at once), multiplies them into its two rows of Wh (register-resident, A1 = A + 1 a template parameter so
// the GEMV has no data-dependent branch), and the A1 partial sums meet through wave shuffles + one LDS row per
// wave (fixed order). Meanwhile threads 64..66 advance the physics for all three paddle directions. Wave 0 then
// samples; after one barrier the sampled direction's outcome is committed and the newest frame rendered.
struct FcParts {        // optional: h comes from the fc GEMM's split-K partial planes (cnn_head.h)
  const float* hpart;    // null: h is read as a finished bf16 row
  int S;
  int64_t plane_stride;
  const float* bfc;
};

template <int A1>
__global__ void __launch_bounds__(256) pong_policy_step_kernel(PongIO io, FcParts fc, u16* __restrict__ h,
                                                               const u16* __restrict__ Wh,
                                                               const float* __restrict__ bh,
                                                               float* __restrict__ z_out, int32_t* __restrict__ act,
                                                               float* __restrict__ logp, float* __restrict__ ent,
                                                               float* __restrict__ vout, int key_shift,
                                                               uint32_t pseed, int pre_shifted,
                                                               uint64_t* __restrict__ stamps) {
  constexpr int A = A1 - 1;
  const int e = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ int sh_act;
  __shared__ PongOut cand[3];
  __shared__ float s_acc[4][A1];
  stamp_if(stamps, 0, tid == 0);
  // operands of the sampling wave and the commit, requested first (they were dependent round trips after the
  // head's barrier): the RNG key's counters and the head bias
  const int64_t tg0 = io.tglob[e], id0 = io.env_ids[e];
  const float bhj = bh[lane < A1 ? lane : 0];
  // this thread's two Wh rows (2 * A1 bf16 = A1 32-bit words at byte offset 4 * A1 * tid)
  uint32_t wv[A1];
#pragma unroll
  for (int u = 0; u < A1; ++u) wv[u] = reinterpret_cast<const uint32_t*>(Wh)[A1 * tid + u];
  float hf[2];
  if (fc.hpart) {
    // h = relu(sum of the fc partial planes + bias), rounded to bf16 and stored for the learner
    fc_h2_from_parts(fc.hpart, fc.S, fc.plane_stride, fc.bfc, e, tid, h, hf);
  } else {
    const uint32_t hw = reinterpret_cast<const uint32_t*>(h + (size_t)e * HEAD_HDIM)[tid];
    hf[0] = __uint_as_float(hw << 16);
    hf[1] = __uint_as_float(hw & 0xFFFF0000u);
  }
  if (tid >= 64 && tid < 67) cand[tid - 64] = pong_advance(io, e, (float)(tid - 65));
  stamp_if(stamps, 8, tid == 0);
  float acc[A1];
#pragma unroll
  for (int j = 0; j < A1; ++j) {
    // Wh[2t][j] and Wh[2t+1][j] are elements j and A1 + j of the thread's 2 * A1 bf16
    const uint32_t w0 = wv[j >> 1], w1 = wv[(A1 + j) >> 1];
    const float a0 = __uint_as_float((j & 1) ? (w0 & 0xFFFF0000u) : (w0 << 16));
    const float a1 = __uint_as_float(((A1 + j) & 1) ? (w1 & 0xFFFF0000u) : (w1 << 16));
    acc[j] = wave_sum(hf[0] * a0 + hf[1] * a1);
  }
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < A1; ++j) s_acc[wid][j] = acc[j];
  __syncthreads();
  stamp_if(stamps, 9, tid == 0);
  if (wid == 0) {
    const int64_t key = tg0 * ((int64_t)1 << key_shift) + id0;  // pre-step counter
    const int jj = lane < A1 ? lane : 0;
    float zj = ((s_acc[0][jj] + s_acc[1][jj]) + (s_acc[2][jj] + s_acc[3][jj])) + bhj;
    if (lane < A1) z_out[(size_t)e * A1 + lane] = zj;
    const float value = __shfl(zj, A, 64);
    stamp_if(stamps, 10, lane == 0);
    // categorical head over lanes 0..A-1 (same maths as categorical_sample_kernel)
    const bool on = lane < A;
    const float z = on ? zj : -INFINITY;
    const float m = wave_max(z);
    const float ex = on ? expf(z - m) : 0.f;
    const float lse = m + logf(wave_sum(ex));
    const float lp = z - lse;
    const float H = wave_sum(on ? -expf(lp) * lp : 0.f);
    float g = -INFINITY;
    if (on) g = z + (-logf(-logf(uniform_open(pseed, key, (uint32_t)lane))));
    float best = g;
    int bi = on ? lane : 1 << 30;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    const float lpa = __shfl(lp, bi, 64);
    if (lane == 0) {
      act[e] = bi;
      logp[e] = lpa;
      ent[e] = H;
      vout[e] = value;
      sh_act = bi;
    }
    stamp_if(stamps, 1, lane == 0);
  } else if (!pre_shifted) {
    pong_shift(io, e, 64, blockDim.x - 64);   // else the trunk kernel already shifted the stack
  }
  stamp_if(stamps, 2, tid == 64);
  stamp_if(stamps, 3, tid == 64);
  __syncthreads();
  stamp_if(stamps, 4, tid == 0);
  const PongOut& r = cand[pong_dir_index(sh_act)];
  if (tid == 0) pong_commit(io, e, r, tg0);
  pong_render(io, e, r.s, r.done != 0);
  if (stamps) {
    stamp_if(stamps, 5, tid == 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp_if(stamps, 6, tid == 0);
  }
}

}  // namespace aca

static aca::PongIO make_pong_io(float* state, int32_t* t, int64_t* tg, float* ep_ret, float* ep_stats,
                                const int64_t* ids, const uint8_t* prev, uint8_t* out, float* reward, uint8_t* done,
                                uint8_t* trunc, uint32_t seed, int max_steps, int k) {
  aca::PongIO io;
  io.state = state; io.tsteps = t; io.tglob = tg; io.ep_ret = ep_ret; io.ep_stats = ep_stats; io.env_ids = ids;
  io.prev = prev; io.out = out; io.reward = reward; io.done_out = done; io.trunc_out = trunc; io.seed = seed;
  io.max_steps = max_steps; io.k = k;
  return io;
}

extern "C" hipError_t aca_env_step_pong(float* state, int32_t* t, int64_t* tg, float* ep_ret, float* ep_stats,
                                        const int64_t* ids, const int32_t* actions, const uint8_t* prev,
                                        uint8_t* out, float* reward, uint8_t* done, uint8_t* trunc, uint32_t seed,
                                        int max_steps, int k, int N, hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  aca::PongIO io = make_pong_io(state, t, tg, ep_ret, ep_stats, ids, prev, out, reward, done, trunc, seed, max_steps,
                                k);
  aca::pong_step_kernel<<<N, 256, 0, stream>>>(io, actions);
  return hipGetLastError();
}

extern "C" hipError_t aca_env_policy_step_pong(uint16_t* h, const float* hpart, int S, int64_t plane_stride,
                                               const float* bfc, int hdim, const uint16_t* Wh, const float* bh,
                                               int A, float* z, int32_t* act, float* logp, float* ent, float* value,
                                               int key_shift, uint32_t pseed, float* state, int32_t* t, int64_t* tg,
                                               float* ep_ret, float* ep_stats, const int64_t* ids,
                                               const uint8_t* prev, uint8_t* out, float* reward, uint8_t* done,
                                               uint8_t* trunc, uint32_t seed, int max_steps, int k, int N,
                                               int pre_shifted, uint64_t* stamps, hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  if (hdim != aca::HEAD_HDIM || reinterpret_cast<uintptr_t>(Wh) % 16 || reinterpret_cast<uintptr_t>(h) % 16)
    return hipErrorInvalidValue;
  if (hpart && (S < 1 || S > aca::FC_MAX_PLANES || !bfc || reinterpret_cast<uintptr_t>(hpart) % 16 ||
                reinterpret_cast<uintptr_t>(bfc) % 16 || plane_stride % 4))
    return hipErrorInvalidValue;
  const aca::FcParts fc{hpart, S, plane_stride, bfc};
  aca::PongIO io = make_pong_io(state, t, tg, ep_ret, ep_stats, ids, prev, out, reward, done, trunc, seed, max_steps,
                                k);
  switch (A + 1) {
#define ACA_POLICY_CASE(A1)                                                                                         \
  case A1:                                                                                                          \
    aca::pong_policy_step_kernel<A1><<<N, 256, 0, stream>>>(io, fc, h, Wh, bh, z, act, logp, ent, value, key_shift,\
                                                            pseed, pre_shifted, stamps);                            \
    break;
    ACA_POLICY_CASE(3) ACA_POLICY_CASE(4) ACA_POLICY_CASE(5) ACA_POLICY_CASE(6) ACA_POLICY_CASE(7)
    ACA_POLICY_CASE(8) ACA_POLICY_CASE(9) ACA_POLICY_CASE(10) ACA_POLICY_CASE(11) ACA_POLICY_CASE(12)
    ACA_POLICY_CASE(13) ACA_POLICY_CASE(14) ACA_POLICY_CASE(15) ACA_POLICY_CASE(16) ACA_POLICY_CASE(17)
    ACA_POLICY_CASE(18) ACA_POLICY_CASE(19) ACA_POLICY_CASE(20)
#undef ACA_POLICY_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
