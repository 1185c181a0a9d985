// Pong-shaped env bank: state, physics, frame rendering (device side). Shared by the env kernels
// (env_atari.hip) and the fused policy/env + trunk kernel (cnn_fused.hip). The physics carries its own
// `fp contract(off)`: it must round exactly like the PyTorch oracle (envs/atari.py) in every including file.
#pragma once
#include "common.h"

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
#pragma clang fp contract(off)
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

// The env's state as advance reads it: loaded by pong_load so that a kernel can request it before its other loads and
// run the physics later (pong_advance_in), without a round trip in between.
struct PongIn {
  PongState s;
  int64_t tg;
  int64_t id;
  int32_t t;
  float ep_ret;
};

__device__ __forceinline__ PongIn pong_load(const PongIO& io, int e) {
  const float* sp = io.state + (size_t)e * 8;
  return PongIn{PongState{sp[0], sp[1], sp[2], sp[3], sp[4], sp[5], sp[6], sp[7]}, io.tglob[e], io.env_ids[e],
                io.tsteps[e], io.ep_ret[e]};
}

__device__ __forceinline__ PongOut pong_advance_in(const PongIO& io, const PongIn& in, float dirn) {
#pragma clang fp contract(off)   // rounds exactly like the PyTorch oracle, whatever the including file's flags
  PongState s = in.s;
  const int64_t tg = in.tg + 1;
  const uint32_t id = (uint32_t)in.id, st = (uint32_t)tg;
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
  r.t = in.t + 1;
  r.trunc = (r.t >= io.max_steps) && !term;
  r.done = term || r.trunc;
  r.rew = rew;
  r.er = in.ep_ret + rew;
  if (r.done) {
    const float mid = 0.5f * (FIELD_TOP + FIELD_BOT);
    s.pa = mid; s.po = mid; s.sa = 0.0f; s.so = 0.0f;
    serve(s, io.seed, id, st, 100);
  }
  r.s = s;
  return r;
}

__device__ __forceinline__ PongOut pong_advance(const PongIO& io, int e, float dirn) {
  return pong_advance_in(io, pong_load(io, e), dirn);
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
// One 4-pixel word (row y, pixels x0..x0+3) of the frame of state s: wall rows are uniform, and only the words that
// overlap a paddle or the ball need per-pixel tests.
struct PongGeom {
  int pa0, po0, bx0, by0;
};
__device__ __forceinline__ PongGeom pong_geom(const PongState& s) {
  return PongGeom{(int)floorf(s.pa - PADDLE_H / 2), (int)floorf(s.po - PADDLE_H / 2), (int)floorf(s.bx),
                  (int)floorf(s.by)};
}
__device__ __forceinline__ uint32_t pong_word(const PongGeom& g, int y, int x0) {
  if (y < (int)FIELD_TOP || y >= (int)FIELD_BOT) return WALL * 0x01010101u;
  const bool agent = y >= g.pa0 && y < g.pa0 + (int)PADDLE_H && x0 + 4 > (int)AGENT_X &&
                     x0 < (int)(AGENT_X + PADDLE_W);
  const bool opp = y >= g.po0 && y < g.po0 + (int)PADDLE_H && x0 + 4 > (int)OPP_X && x0 < (int)(OPP_X + PADDLE_W);
  const bool ball = y >= g.by0 && y < g.by0 + (int)BALL && x0 + 4 > g.bx0 && x0 < g.bx0 + (int)BALL;
  uint32_t word = BG * 0x01010101u;
  if (agent || opp || ball) {
    word = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int x = x0 + q;
      uint32_t v = BG;
      if (agent && x >= (int)AGENT_X && x < (int)(AGENT_X + PADDLE_W)) v = AGENT_C;
      if (opp && x >= (int)OPP_X && x < (int)(OPP_X + PADDLE_W)) v = OPP_C;
      if (ball && x >= g.bx0 && x < g.bx0 + (int)BALL) v = BALL_C;
      word |= v << (8 * q);
    }
  }
  return word;
}

__device__ __forceinline__ void pong_render(const PongIO& io, int e, const PongState& s, bool done) {
  // 4-pixel words, 21 per row (one 4-byte store per word, consecutive lanes -> consecutive words)
  constexpr int WPR = PW / 4, NWORDS = PH * WPR;   // 21, 1764
  const int k = io.k;
  const PongGeom g = pong_geom(s);
  uint32_t* ov = reinterpret_cast<uint32_t*>(io.out + (size_t)e * k * FRAME);
  for (int w = threadIdx.x; w < NWORDS; w += blockDim.x) {
    const int y = w / WPR, x0 = (w - y * WPR) * 4;
    const uint32_t word = pong_word(g, y, x0);
    ov[(size_t)(k - 1) * NWORDS + w] = word;
    if (done)
      for (int s2 = 0; s2 < k - 1; ++s2) ov[(size_t)s2 * NWORDS + w] = word;
  }
}

}  // namespace aca
