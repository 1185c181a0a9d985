// Atari-shaped env bank (Pong-like game rendered to 84x84 uint8), BASELINE.json headline config.
//
// One 256-thread workgroup per env: thread 0 advances the 4 physics sub-steps (frameskip 4) and handles the
// auto-reset, then the whole workgroup renders the new 84x84 frame straight into the output stack with 16-byte
// stores and shifts the previous 3 frames in (frame stack [N, k, 84, 84]); finished envs get k copies of their
// first frame (Framer padding rule, Basic_AC/run_AC.py:37-40). Oracle: envs/atari.py (compiled with
// -ffp-contract=off so the physics rounds exactly like the PyTorch oracle).
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
  float u0 = uniform01(seed, id, st, stream0);
  float u1 = uniform01(seed, id, st, stream0 + 1);
  float u2 = uniform01(seed, id, st, stream0 + 2);
  s.bx = 41.0f;
  s.by = 30.0f + u0 * 24.0f;
  s.vx = (u1 < 0.5f) ? BALL_VX : -BALL_VX;
  s.vy = (u2 - 0.5f) * 2.0f;
}

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

__global__ void __launch_bounds__(256) pong_step_kernel(float* __restrict__ state, int32_t* __restrict__ tsteps,
                                                        int64_t* __restrict__ tglob, float* __restrict__ ep_ret,
                                                        float* __restrict__ ep_stats,
                                                        const int64_t* __restrict__ env_ids,
                                                        const int32_t* __restrict__ actions,
                                                        const uint8_t* __restrict__ prev, uint8_t* __restrict__ out,
                                                        float* __restrict__ reward, uint8_t* __restrict__ done_out,
                                                        uint8_t* __restrict__ trunc_out, uint32_t seed, int max_steps,
                                                        int k) {
  const int e = blockIdx.x;
  __shared__ PongState sh;
  __shared__ int sh_done;
  if (threadIdx.x == 0) {
    float* sp = state + (size_t)e * 8;
    PongState s{sp[0], sp[1], sp[2], sp[3], sp[4], sp[5], sp[6], sp[7]};
    const int64_t tg = tglob[e] + 1;
    tglob[e] = tg;
    const uint32_t id = (uint32_t)env_ids[e], st = (uint32_t)tg;
    const int a = actions[e];
    float dirn = 0.0f;
    if (a == 2 || a == 4) dirn = -1.0f;
    if (a == 3 || a == 5) dirn = 1.0f;
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
      if (miss_a || miss_o) serve(s, seed, id, st, 200 + 4 * sub);
    }
    bool term = (s.sa >= WIN_SCORE) || (s.so >= WIN_SCORE);
    int t = tsteps[e] + 1;
    bool trunc = (t >= max_steps) && !term;
    bool done = term || trunc;
    float er = ep_ret[e] + rew;
    reward[e] = rew;
    done_out[e] = done;
    trunc_out[e] = trunc;
    if (done) {
      atomicAdd(&ep_stats[0], er);
      atomicAdd(&ep_stats[1], 1.0f);
      atomicAdd(&ep_stats[2], (float)t);
      const float mid = 0.5f * (FIELD_TOP + FIELD_BOT);
      s.pa = mid; s.po = mid; s.sa = 0.0f; s.so = 0.0f;
      serve(s, seed, id, st, 100);
      t = 0;
      er = 0.0f;
    }
    tsteps[e] = t;
    ep_ret[e] = er;
    sp[0] = s.bx; sp[1] = s.by; sp[2] = s.vx; sp[3] = s.vy; sp[4] = s.pa; sp[5] = s.po; sp[6] = s.sa; sp[7] = s.so;
    sh = s;
    sh_done = done;
  }
  __syncthreads();
  const PongState s = sh;
  const bool done = sh_done != 0;
  const int pa0 = (int)floorf(s.pa - PADDLE_H / 2), po0 = (int)floorf(s.po - PADDLE_H / 2);
  const int bx0 = (int)floorf(s.bx), by0 = (int)floorf(s.by);
  const uint8_t* pv = prev + (size_t)e * k * FRAME;
  uint8_t* ov = out + (size_t)e * k * FRAME;
  // shift the older frames (16-byte copies); a reset stack is rewritten below
  if (!done) {
    const uint4* src = reinterpret_cast<const uint4*>(pv + FRAME);
    uint4* dst = reinterpret_cast<uint4*>(ov);
    const int n16 = (k - 1) * FRAME / 16;
    for (int j = threadIdx.x; j < n16; j += blockDim.x) dst[j] = src[j];
  }
  // render the newest frame: 441 chunks of 16 pixels
  for (int c = threadIdx.x; c < FRAME / 16; c += blockDim.x) {
    union { uint4 v; uint8_t b[16]; } px;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int p = c * 16 + q, y = p / PW, x = p % PW;
      uint8_t v = BG;
      if (y < (int)FIELD_TOP || y >= (int)FIELD_BOT) v = WALL;
      if (x >= (int)AGENT_X && x < (int)(AGENT_X + PADDLE_W) && y >= pa0 && y < pa0 + (int)PADDLE_H) v = AGENT_C;
      if (x >= (int)OPP_X && x < (int)(OPP_X + PADDLE_W) && y >= po0 && y < po0 + (int)PADDLE_H) v = OPP_C;
      if (x >= bx0 && x < bx0 + (int)BALL && y >= by0 && y < by0 + (int)BALL) v = BALL_C;
      px.b[q] = v;
    }
    uint4* dst = reinterpret_cast<uint4*>(ov + (size_t)(k - 1) * FRAME);
    dst[c] = px.v;
    if (done)
      for (int s2 = 0; s2 < k - 1; ++s2) reinterpret_cast<uint4*>(ov + (size_t)s2 * FRAME)[c] = px.v;
  }
}

}  // namespace aca

extern "C" hipError_t aca_env_step_pong(float* state, int32_t* t, int64_t* tg, float* ep_ret, float* ep_stats,
                                        const int64_t* ids, const int32_t* actions, const uint8_t* prev,
                                        uint8_t* out, float* reward, uint8_t* done, uint8_t* trunc, uint32_t seed,
                                        int max_steps, int k, int N, hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  aca::pong_step_kernel<<<N, 256, 0, stream>>>(state, t, tg, ep_ret, ep_stats, ids, actions, prev, out, reward, done,
                                               trunc, seed, max_steps, k);
  return hipGetLastError();
}
