// Atari-shaped env bank (Pong-like game rendered to 84x84 uint8), BASELINE.json headline config.
//
// One 256-thread workgroup per env: thread 0 advances the 4 physics sub-steps (frameskip 4) and handles the
// auto-reset, then the whole workgroup renders the new 84x84 frame straight into the output stack with 16-byte
// stores and shifts the previous 3 frames in (frame stack [N, k, 84, 84]); finished envs get k copies of their
// first frame (Framer padding rule, Basic_AC/run_AC.py:37-40). Oracle: envs/atari.py (compiled with
// -ffp-contract=off so the physics rounds exactly like the PyTorch oracle).
#include "common.h"
#include "cnn_head.h"
#include "pong_env.h"

namespace aca {

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
    const float value = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(zj), A));
    stamp_if(stamps, 10, lane == 0);
    // categorical head over lanes 0..A-1 (same maths as categorical_sample_kernel; A1 <= 7: the 8-lane trees)
    const CatSample cs = cat_sample<8>(zj, A, lane, pseed, key);
    const int bi = cs.act;
    const float lpa = cs.lpa, H = cs.H;
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
