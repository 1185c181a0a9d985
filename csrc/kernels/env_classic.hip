// Vector-observation env banks: CartPole (gym equations), Pendulum-v0 (gym equations) and the MuJoCo-shaped
// linear-Gaussian system. One thread per env; each launch advances the whole bank one step, auto-resets finished
// envs, pushes the new observation into the frame stack (Framer semantics, Basic_AC/run_AC.py:24-53) and
// accumulates episode statistics -- no host round trip, so a rollout step is hipGraph-capturable.
//
// Oracles: actor_critic_algs_on_tensorflow_amd/envs/classic.py and mujoco.py. This file is compiled with
// -ffp-contract=off so that fp32 arithmetic rounds exactly like the PyTorch oracle (separately rounded mul/add).
#include "common.h"

namespace aca {

struct EnvIO {
  float* state;
  int32_t* t;
  int64_t* tg;
  float* ep_ret;
  float* ep_stats;  // [sum_ret, count, sum_len]
  const int64_t* env_ids;
  const float* prev;  // [N, k*D] frame stack in
  float* out;         // [N, k*D] frame stack out
  float* reward;
  uint8_t* done;
  uint8_t* truncated;
  float* final_out;   // optional [N, k*D]: the stack with the transition's new frame BEFORE any auto-reset (the
                      // terminal observation of a finished episode; time-limit bootstrapping values it)
  uint32_t seed;
  int max_steps;
  int k;
  int N;
};

template <int D>
__device__ __forceinline__ void push_frame_to(const EnvIO& io, float* dst, int i, const float* frame, bool reset) {
  const int k = io.k;
  const float* p = io.prev + (size_t)i * k * D;
  float* o = dst + (size_t)i * k * D;
  if (reset) {
    for (int s = 0; s < k; ++s)
      for (int j = 0; j < D; ++j) o[s * D + j] = frame[j];
  } else {
    for (int s = 0; s < k - 1; ++s)
      for (int j = 0; j < D; ++j) o[s * D + j] = p[(s + 1) * D + j];
    for (int j = 0; j < D; ++j) o[(k - 1) * D + j] = frame[j];
  }
}

template <int D>
__device__ __forceinline__ void push_frame(const EnvIO& io, int i, const float* frame, bool reset) {
  push_frame_to<D>(io, io.out, i, frame, reset);
}

// ------------------------------------------------------------------------------------------------ CartPole
__global__ void cartpole_step_kernel(EnvIO io, const int32_t* __restrict__ actions) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i < io.N;
  bool done = false;
  float ret = 0.f, len = 0.f;
  if (active) {
    const float GRAVITY = 9.8f, MASSPOLE = 0.1f, TOTAL = 1.1f, LENGTH = 0.5f, PML = 0.05f, FORCE = 10.0f;
    const float TAU = 0.02f, THETA = (float)(12 * 2 * 3.141592653589793 / 360), XLIM = 2.4f;
    const float FOUR_THIRDS = (float)(4.0 / 3.0);
    float* s = io.state + (size_t)i * 4;
    const int64_t tg = io.tg[i] + 1;
    io.tg[i] = tg;
    float x = s[0], x_dot = s[1], th = s[2], th_dot = s[3];
    float force = actions[i] == 1 ? FORCE : -FORCE;
    float c = cosf(th), sn = sinf(th);
    float temp = (force + PML * th_dot * th_dot * sn) / TOTAL;
    float thacc = (GRAVITY * sn - c * temp) / (LENGTH * (FOUR_THIRDS - MASSPOLE * c * c / TOTAL));
    float xacc = temp - PML * thacc * c / TOTAL;
    x = x + TAU * x_dot;
    x_dot = x_dot + TAU * xacc;
    th = th + TAU * th_dot;
    th_dot = th_dot + TAU * thacc;
    bool term = (x < -XLIM) || (x > XLIM) || (th < -THETA) || (th > THETA);
    int t = io.t[i] + 1;
    bool trunc = (t >= io.max_steps) && !term;
    done = term || trunc;
    float er = io.ep_ret[i] + 1.0f;
    ret = er;
    len = (float)t;
    io.reward[i] = 1.0f;
    io.done[i] = done;
    io.truncated[i] = trunc;
    if (io.final_out) {
      const float fin[4] = {x, x_dot, th, th_dot};
      push_frame_to<4>(io, io.final_out, i, fin, false);
    }
    if (done) {
      const uint32_t id = (uint32_t)io.env_ids[i], st = (uint32_t)tg;
      x = uniform01(io.seed, id, st, 100) * 0.1f - 0.05f;
      x_dot = uniform01(io.seed, id, st, 101) * 0.1f - 0.05f;
      th = uniform01(io.seed, id, st, 102) * 0.1f - 0.05f;
      th_dot = uniform01(io.seed, id, st, 103) * 0.1f - 0.05f;
      t = 0;
      er = 0.f;
    }
    s[0] = x; s[1] = x_dot; s[2] = th; s[3] = th_dot;
    io.t[i] = t;
    io.ep_ret[i] = er;
    float frame[4] = {x, x_dot, th, th_dot};
    push_frame<4>(io, i, frame, done);
  }
  add_ep_stats(io.ep_stats, active, done, ret, len);
}

// ------------------------------------------------------------------------------------------------ Pendulum
__device__ __forceinline__ float angle_normalize(float x) {
  const float PI = 3.14159265358979323846f, TWO_PI = (float)(2 * 3.141592653589793);
  float y = x + PI;
  // torch.remainder (python-style modulo): y - floor(y / m) * m
  float r = y - floorf(y / TWO_PI) * TWO_PI;
  return r - PI;
}

__global__ void pendulum_step_kernel(EnvIO io, const float* __restrict__ actions, int act_dim) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i < io.N;
  bool done = false;
  float ret = 0.f, len = 0.f;
  if (active) {
    const float PI = 3.14159265358979323846f, TWO_PI = (float)(2 * 3.141592653589793);
    float* s = io.state + (size_t)i * 2;
    const int64_t tg = io.tg[i] + 1;
    io.tg[i] = tg;
    float th = s[0], thdot = s[1];
    float u = fminf(fmaxf(actions[(size_t)i * act_dim], -2.0f), 2.0f);
    float an = angle_normalize(th);
    float costs = an * an + 0.1f * (thdot * thdot) + 0.001f * (u * u);
    float newthdot = thdot + (-15.0f * sinf(th + PI) + 3.0f * u) * 0.05f;
    float newth = th + newthdot * 0.05f;
    newthdot = fminf(fmaxf(newthdot, -8.0f), 8.0f);
    th = newth;
    thdot = newthdot;
    int t = io.t[i] + 1;
    bool trunc = t >= io.max_steps;
    done = trunc;
    float rew = -costs;
    float er = io.ep_ret[i] + rew;
    ret = er;
    len = (float)t;
    io.reward[i] = rew;
    io.done[i] = done;
    io.truncated[i] = trunc;
    if (io.final_out) {
      const float fin[3] = {cosf(th), sinf(th), thdot};
      push_frame_to<3>(io, io.final_out, i, fin, false);
    }
    if (done) {
      const uint32_t id = (uint32_t)io.env_ids[i], st = (uint32_t)tg;
      th = uniform01(io.seed, id, st, 100) * TWO_PI - PI;
      thdot = uniform01(io.seed, id, st, 101) * 2.0f - 1.0f;
      t = 0;
      er = 0.f;
    }
    s[0] = th;
    s[1] = thdot;
    io.t[i] = t;
    io.ep_ret[i] = er;
    float frame[3] = {cosf(th), sinf(th), thdot};
    push_frame<3>(io, i, frame, done);
  }
  add_ep_stats(io.ep_stats, active, done, ret, len);
}

// ------------------------------------------------------------------------------------------------ linear (MuJoCo-shape)
constexpr int LIN_OBS = 17, LIN_ACT = 6;

// 32 lanes per env, lane r < 17 owns state row r: the matrix-vector products, the noise hash and the frame write are
// spread over the lanes (each row's sum keeps the sequential column order of the oracle); lane 0 owns the scalar
// episode bookkeeping. The env's previous state / actions are read by every lane of its group (broadcast loads).
constexpr int LIN_LANES = 32;

__global__ void __launch_bounds__(256) linear_step_kernel(EnvIO io, const float* __restrict__ actions,
                                                          const float* __restrict__ A, const float* __restrict__ B) {
  __shared__ float sA[LIN_OBS * LIN_OBS], sB[LIN_OBS * LIN_ACT];
  for (int j = threadIdx.x; j < LIN_OBS * LIN_OBS; j += blockDim.x) sA[j] = A[j];
  for (int j = threadIdx.x; j < LIN_OBS * LIN_ACT; j += blockDim.x) sB[j] = B[j];
  __syncthreads();
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) / LIN_LANES;
  const int r = threadIdx.x % LIN_LANES;
  const bool active = i < io.N;
  const bool owner = active && r == 0;
  bool done = false;
  float ret = 0.f, len = 0.f;
  if (active) {
    float* s = io.state + (size_t)i * LIN_OBS;
    const int64_t tg = io.tg[i] + 1;
    const uint32_t id = (uint32_t)io.env_ids[i], st = (uint32_t)tg;
    float a[LIN_ACT];
    float asq = 0.f;
    for (int j = 0; j < LIN_ACT; ++j) {
      a[j] = fminf(fmaxf(actions[(size_t)i * LIN_ACT + j], -1.0f), 1.0f);
      asq += a[j] * a[j];
    }
    float y = 0.f;
    if (r < LIN_OBS) {
      float acc = 0.f, acc2 = 0.f;
      for (int c = 0; c < LIN_OBS; ++c) acc += s[c] * sA[r * LIN_OBS + c];
      for (int c = 0; c < LIN_ACT; ++c) acc2 += a[c] * sB[r * LIN_ACT + c];
      const float nz = uniform01(io.seed, id, st, 300 + r);
      y = acc + acc2 + (nz - 0.5f) * 0.02f;
    }
    // reward reads row 8 (lane 8 of the group)
    const float y8 = __shfl(y, (threadIdx.x & 63 & ~(LIN_LANES - 1)) + 8, 64);
    const float rew = y8 - 0.1f * asq;
    const int t = io.t[i] + 1;
    const bool trunc = t >= io.max_steps;
    done = trunc;
    const float er = io.ep_ret[i] + rew;
    ret = er;
    len = (float)t;
    if (io.final_out && r < LIN_OBS) {   // terminal observation (before the reset below)
      const int k = io.k;
      const float* pv = io.prev + (size_t)i * k * LIN_OBS;
      float* fo = io.final_out + (size_t)i * k * LIN_OBS;
      for (int f = 0; f < k - 1; ++f) fo[f * LIN_OBS + r] = pv[(f + 1) * LIN_OBS + r];
      fo[(k - 1) * LIN_OBS + r] = y;
    }
    if (done && r < LIN_OBS) y = (uniform01(io.seed, id, st, 100 + r) - 0.5f) * 0.2f;
    if (r < LIN_OBS) {
      s[r] = y;
      // frame stack: shift the k-1 newest frames down, append y (reset: k copies of y)
      const int k = io.k;
      const float* pv = io.prev + (size_t)i * k * LIN_OBS;
      float* o = io.out + (size_t)i * k * LIN_OBS;
      for (int f = 0; f < k - 1; ++f) o[f * LIN_OBS + r] = done ? y : pv[(f + 1) * LIN_OBS + r];
      o[(k - 1) * LIN_OBS + r] = y;
    }
    if (owner) {
      io.tg[i] = tg;
      io.reward[i] = rew;
      io.done[i] = done;
      io.truncated[i] = trunc;
      io.t[i] = done ? 0 : t;
      io.ep_ret[i] = done ? 0.f : er;
    }
  }
  add_ep_stats(io.ep_stats, owner, done, ret, len);
}

}  // namespace aca

using namespace aca;

static EnvIO make_io(float* state, int32_t* t, int64_t* tg, float* ep_ret, float* ep_stats, const int64_t* ids,
                     const float* prev, float* out, float* reward, uint8_t* done, uint8_t* trunc, uint32_t seed,
                     int max_steps, int k, int N, float* final_out = nullptr) {
  EnvIO io;
  io.final_out = final_out;
  io.state = state; io.t = t; io.tg = tg; io.ep_ret = ep_ret; io.ep_stats = ep_stats; io.env_ids = ids;
  io.prev = prev; io.out = out; io.reward = reward; io.done = done; io.truncated = trunc; io.seed = seed;
  io.max_steps = max_steps; io.k = k; io.N = N;
  return io;
}

extern "C" hipError_t aca_env_step_cartpole(float* state, int32_t* t, int64_t* tg, float* ep_ret, float* ep_stats,
                                            const int64_t* ids, const int32_t* actions, const float* prev,
                                            float* out, float* reward, uint8_t* done, uint8_t* trunc,
                                            uint32_t seed, int max_steps, int k, int N, float* final_out,
                                            hipStream_t stream) {
  EnvIO io = make_io(state, t, tg, ep_ret, ep_stats, ids, prev, out, reward, done, trunc, seed, max_steps, k, N,
                     final_out);
  const int bs = 256;
  cartpole_step_kernel<<<(N + bs - 1) / bs, bs, 0, stream>>>(io, actions);
  return hipGetLastError();
}

extern "C" hipError_t aca_env_step_pendulum(float* state, int32_t* t, int64_t* tg, float* ep_ret, float* ep_stats,
                                            const int64_t* ids, const float* actions, int act_dim,
                                            const float* prev, float* out, float* reward, uint8_t* done,
                                            uint8_t* trunc, uint32_t seed, int max_steps, int k, int N,
                                            float* final_out, hipStream_t stream) {
  EnvIO io = make_io(state, t, tg, ep_ret, ep_stats, ids, prev, out, reward, done, trunc, seed, max_steps, k, N,
                     final_out);
  const int bs = 256;
  pendulum_step_kernel<<<(N + bs - 1) / bs, bs, 0, stream>>>(io, actions, act_dim);
  return hipGetLastError();
}

extern "C" hipError_t aca_env_step_linear(float* state, int32_t* t, int64_t* tg, float* ep_ret, float* ep_stats,
                                          const int64_t* ids, const float* actions, const float* A, const float* B,
                                          const float* prev, float* out, float* reward, uint8_t* done,
                                          uint8_t* trunc, uint32_t seed, int max_steps, int k, int N,
                                          float* final_out, hipStream_t stream) {
  EnvIO io = make_io(state, t, tg, ep_ret, ep_stats, ids, prev, out, reward, done, trunc, seed, max_steps, k, N,
                     final_out);
  const int bs = 256;
  linear_step_kernel<<<(N * LIN_LANES + bs - 1) / bs, bs, 0, stream>>>(io, actions, A, B);
  return hipGetLastError();
}
