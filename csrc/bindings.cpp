// torch.ops.acamd.* registrations for the gfx950 kernels in csrc/kernels/*.hip.
//
// The kernels are compiled by hipcc without torch headers and export plain C launchers taking raw pointers and a
// hipStream_t; this file (the only one that includes torch) validates tensors, resolves the current HIP stream of
// torch.cuda (so ops are hipGraph-capturable) and forwards. Every op mutates its output arguments in place and
// returns nothing: the Python layer owns all buffers (static addresses for graph capture).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <vector>

#include "gemm_desc.h"
#include "mlp_desc.h"
#include "ppo_head.h"

extern "C" {
hipError_t aca_seg_stats(const float*, const int64_t*, int, float*, hipStream_t);
hipError_t aca_colsum_reduce(const float*, int, int, float*, int, hipStream_t);
hipError_t aca_mlp_tshadow(const aca::MlpTower*, int, int, hipStream_t);
hipError_t aca_opt_multi(const int64_t*, const float*, const int64_t*, int, int, float, float, float, int, int,
                         hipStream_t);
hipError_t aca_prp_perm(int64_t*, int, uint32_t, const int64_t*, int, hipStream_t);
hipError_t aca_mlp_fwd(const aca::MlpArgs*, int, size_t, int, hipStream_t);
hipError_t aca_mlp_wgrad(const aca::WgradArgs*, hipStream_t);
hipError_t aca_mlp_epoch_gather(const aca::EpochGatherArgs*, hipStream_t);
hipError_t aca_ppo_head(const aca::PpoHeadArgs*, int, hipStream_t);
int aca_ppo_head_planes(int);
int aca_opt_set_unroll(int);
void aca_opt_set_stamps(int64_t*);
hipError_t aca_fc_bwd(const uint16_t*, const uint16_t*, const uint16_t*, uint16_t*, float*, int, float*, uint64_t*,
                      hipStream_t);
hipError_t aca_fc_rollout(const uint16_t*, int64_t, int, const uint16_t*, int, int, float*, int64_t, int, int, int*,
                          unsigned long long*, int, hipStream_t);
hipError_t aca_mlp_rollout(const aca::RolloutArgs*, size_t, hipStream_t);
hipError_t aca_env_step_cartpole(float*, int32_t*, int64_t*, float*, float*, const int64_t*, const int32_t*,
                                 const float*, float*, float*, uint8_t*, uint8_t*, uint32_t, int, int, int, float*,
                                 hipStream_t);
hipError_t aca_env_step_pendulum(float*, int32_t*, int64_t*, float*, float*, const int64_t*, const float*, int,
                                 const float*, float*, float*, uint8_t*, uint8_t*, uint32_t, int, int, int, float*,
                                 hipStream_t);
hipError_t aca_env_step_linear(float*, int32_t*, int64_t*, float*, float*, const int64_t*, const float*,
                               const float*, const float*, const float*, float*, float*, uint8_t*, uint8_t*,
                               uint32_t, int, int, int, float*, hipStream_t);
hipError_t aca_env_step_pong(float*, int32_t*, int64_t*, float*, float*, const int64_t*, const int32_t*,
                             const uint8_t*, uint8_t*, float*, uint8_t*, uint8_t*, uint32_t, int, int, int,
                             hipStream_t);
hipError_t aca_fc_value(const float*, int, int64_t, const float*, const uint16_t*, int, const float*, float*,
                        uint16_t*, int, hipStream_t);
hipError_t aca_env_policy_step_pong(uint16_t*, const float*, int, int64_t, const float*, int, const uint16_t*,
                                    const float*, int, float*, int32_t*,
                                    float*, float*, float*, int, uint32_t, float*, int32_t*, int64_t*, float*, float*,
                                    const int64_t*, const uint8_t*, uint8_t*, float*, uint8_t*, uint8_t*, uint32_t,
                                    int, int, int, int, uint64_t*, hipStream_t);
hipError_t aca_pong_fused_step(uint16_t*, const float*, int, int64_t, const float*, const uint16_t*, const float*, int,
                               float*, int32_t*, float*, float*, float*, int, uint32_t, float*, int32_t*, int64_t*,
                               float*, float*, int32_t*, int64_t*, float*, float*, const int64_t*, const uint8_t*,
                               uint8_t*, float*, uint8_t*, uint8_t*, uint32_t, int, const uint16_t*, const float*,
                               const uint16_t*, const float*, const uint16_t*, const float*, uint16_t*, uint16_t*,
                               uint16_t*, float, uint8_t*, uint64_t*, int, int, hipStream_t);
hipError_t aca_pong_fused_env_step(uint16_t*, const float*, int, int64_t, const float*, const uint16_t*, const float*,
                                   int, float*, int32_t*, float*, float*, float*, int, uint32_t, float*, int32_t*,
                                   int64_t*, float*, float*, const int64_t*, uint8_t*, float*, uint8_t*, uint8_t*,
                                   uint32_t, int, const uint16_t*, const float*, const uint16_t*, const float*,
                                   const uint16_t*, const float*, uint16_t*, uint16_t*, uint16_t*, float, uint8_t*,
                                   float*, int32_t*, int64_t*, float*, uint64_t*, int, int, hipStream_t);
hipError_t aca_wave_reduce_check(const float*, float*, int, hipStream_t);
hipError_t aca_categorical_sample(const float*, int, int, int, const int64_t*, const int64_t*, const int64_t*, int,
                                  uint32_t, int32_t*, float*, float*, float*, hipStream_t);
hipError_t aca_ev(const float*, const float*, float*, int, hipStream_t);
hipError_t aca_gaussian_sample(const float*, int, int, int, const float*, const int64_t*, uint32_t, float*, float*,
                               float*, hipStream_t);
hipError_t aca_gae(const float*, const float*, const uint8_t*, float*, float*, int, int, float, float, hipStream_t);
hipError_t aca_nstep(const float*, const float*, const uint8_t*, float*, float*, int, int, float, int, hipStream_t);
hipError_t aca_normalize(const float*, float*, int, float, hipStream_t);
hipError_t aca_moments(const float*, const float*, float*, int, hipStream_t);
void aca_returns_scan_geometry(int, int, int*, int*, int*, int*);
hipError_t aca_returns_scan(const float*, const float*, const uint8_t*, float*, float*, double*, double*, unsigned int*,
                            double*, float*, int, int, int, int, int, float, float, float, hipStream_t);
hipError_t aca_normalize_mom(const float*, float*, const double*, int, float, hipStream_t);
int aca_ev_multi_blocks(int);
hipError_t aca_gemm_group_run(const AcaGemmDesc*, int, hipStream_t, int*);
hipError_t aca_mb_gather(const uint8_t*, int64_t, const int*, const float*, const float*, const float*, const float*,
                         uint8_t*, int*, float*, float*, float*, float*, int, int, uint32_t, int64_t*, int, int,
                         const double*, float, unsigned int*, int64_t*, hipStream_t);
hipError_t aca_ev_multi(const float*, const float*, float*, int, double*, unsigned int*, hipStream_t);
hipError_t aca_conv1_wgrad2(const uint8_t*, const uint16_t*, float*, int, int, float, const int64_t*, hipStream_t);
hipError_t aca_conv_wgrad_gemm(int, const uint16_t*, const uint16_t*, float*, int, int, hipStream_t);
hipError_t aca_gemm_big(const AcaGemmDesc*, hipStream_t);
int64_t aca_gemm_big_ws(int, int, int);
hipError_t aca_sumsq(const void*, size_t, float*, int, hipStream_t);
hipError_t aca_sumsq_multi(const float* const*, const size_t*, float* const*, int, hipStream_t);
int aca_sumsq_parts();
hipError_t aca_adam_step(float*, float*, float*, float*, size_t, const float*, float*, const float*, float*, uint16_t*,
                         float, float, float, float, float, unsigned int*, int, float, float, const int64_t*,
                         const uint16_t*, hipStream_t);
hipError_t aca_rmsprop_step(float*, float*, float*, size_t, const float*, const float*, float*, uint16_t*, float, float,
                            float, float, int, float, float, const int64_t*, const uint16_t*, hipStream_t);
hipError_t aca_cast_bf16(const float*, uint16_t*, size_t, hipStream_t);
hipError_t aca_grad_move(float*, float*, size_t, int*, int, hipStream_t);
hipError_t aca_gemm_run(const AcaGemmDesc*, hipStream_t);
int aca_gemm_effective_splits(int, int, int);
int aca_gemm_tile_dims(int, int*, int*);
int aca_gemm_supported(int, int);
hipError_t aca_im2col_u8_nchw(const uint8_t*, uint16_t*, int, int, int, int, int, int, int, float, hipStream_t);
hipError_t aca_im2col_nhwc(const uint16_t*, uint16_t*, int, int, int, int, int, int, int, hipStream_t);
hipError_t aca_col2im_nhwc(const uint16_t*, const uint16_t*, uint16_t*, float*, int, int, int, int, int, int, int,
                           hipStream_t);
hipError_t aca_colsum_bf16(const uint16_t*, int64_t, int, int64_t, float*, hipStream_t);
hipError_t aca_ac_loss(const float*, int64_t, const float*, int64_t, const int32_t*, const float*, const float*,
                       const float*, const float*, const float*, const float*, const float*, const float*, float, float,
                       float, uint16_t*, int64_t, uint16_t*, int64_t, float*, float*, int, int, int, int,
                       const float*, const float*, const uint8_t*, int, int, int, float, float, int, float*, float*,
                       float*, int, hipStream_t);
hipError_t aca_cnn_trunk_fwd_s16(const uint8_t*, const uint16_t*, const float*, const uint16_t*, const float*,
                                 const uint16_t*, const float*, uint16_t*, uint16_t*, uint16_t*, int, float, uint8_t*,
                                 const int64_t*, int, hipStream_t);
hipError_t aca_grad_finalize(const int64_t*, int, float*, const double*, int, int, const float*, const float*, float*,
                             int, hipStream_t);
hipError_t aca_a2c_head_env(const float*, const int32_t*, const float*, const float*, const float*, float,
                            const float*, float*, const uint8_t*, int, int, int, int, float, float, float*, float*,
                            const uint16_t*, const uint16_t*, uint16_t*, int, const float*, int, int64_t,
                            const float*, const float*, float*, float*, float*, double*, uint64_t*, hipStream_t);
hipError_t aca_head_bwd(const float*, const int32_t*, const float*, const float*, const float*, float, const float*,
                        const float*, const uint8_t*, int, int, int, int, int, float, float, float*, float*,
                        const uint16_t*, const uint16_t*, uint16_t*, float*, float*, float*, float*, int,
                        uint64_t*, hipStream_t);
hipError_t aca_a2c_head(const float*, const int32_t*, const float*, const float*, const float*, float, const float*,
                        float*, const uint8_t*, int, int, int, int, int, float, float, float*, float*,
                        const uint16_t*, const uint16_t*, uint16_t*, float*, float*, float*, float*, int,
                        const float*, int, int64_t, const float*, const float*, unsigned int*, uint64_t*, hipStream_t);
hipError_t aca_cnn_trunk_bwd(const uint16_t*, const uint16_t*, const uint16_t*, const uint16_t*, const uint16_t*,
                             uint16_t*, uint16_t*, float*, int, uint64_t*, int, const uint8_t*, const int64_t*, float*,
                             float, int, hipStream_t);
hipError_t aca_cnn_trunk_rows(const uint8_t*, const uint16_t*, const float*, const uint16_t*, const float*,
                              const uint16_t*, const float*, uint16_t*, uint16_t*, uint16_t*, int, float, uint8_t*,
                              uint8_t*, uint64_t*, int, int, hipStream_t);
}

namespace {

using at::Tensor;

hipStream_t cur_stream(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "acamd::", what, " launch failed: ", hipGetErrorString(e));
}

void need(const Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), "acamd: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, "acamd: ", name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), "acamd: ", name, " must be contiguous");
}

template <typename T>
T* ptr(const Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

// optional per-workgroup phase timestamps [nblocks, 16] int64 (diagnostics; s_memrealtime ticks at 100 MHz)
uint64_t* stamps_ptr(const c10::optional<Tensor>& st, int64_t nblocks) {
  if (!(st.has_value() && st->defined())) return nullptr;
  need(*st, at::kLong, "stamps");
  TORCH_CHECK(st->numel() >= nblocks * 16, "stamps: needs [nblocks, 16]");
  return ptr<uint64_t>(*st);
}


template <typename T>
T* optr(const c10::optional<Tensor>& t) { return (t.has_value() && t->defined()) ? ptr<T>(*t) : nullptr; }

// ---------------------------------------------------------------------------------------------- env banks
void check_env(const Tensor& state, const Tensor& t, const Tensor& tg, const Tensor& ep_ret, const Tensor& ep_stats,
               const Tensor& ids, const Tensor& reward, const Tensor& done, const Tensor& trunc) {
  need(state, at::kFloat, "state");
  need(t, at::kInt, "t");
  need(tg, at::kLong, "tg");
  need(ep_ret, at::kFloat, "ep_ret");
  need(ep_stats, at::kFloat, "ep_stats");
  need(ids, at::kLong, "env_ids");
  need(reward, at::kFloat, "reward");
  need(done, at::kByte, "done");
  need(trunc, at::kByte, "truncated");
}

// optional terminal-observation output of the classic env kernels: same [N, k*D] stack shape as `out`
float* final_out_ptr(const c10::optional<Tensor>& f, const Tensor& out) {
  if (!(f.has_value() && f->defined())) return nullptr;
  need(*f, at::kFloat, "final_out");
  TORCH_CHECK(f->numel() == out.numel(), "final_out: must match the observation stack");
  return ptr<float>(*f);
}

void env_step_cartpole(Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, Tensor ids, Tensor actions,
                       Tensor prev, Tensor out, Tensor reward, Tensor done, Tensor trunc, int64_t seed,
                       int64_t max_steps, int64_t k, c10::optional<Tensor> final_out) {
  check_env(state, t, tg, ep_ret, ep_stats, ids, reward, done, trunc);
  need(actions, at::kInt, "actions");
  need(prev, at::kFloat, "prev");
  need(out, at::kFloat, "out");
  const int N = state.size(0);
  TORCH_CHECK(prev.numel() == (int64_t)N * 4 * k && out.numel() == prev.numel(), "cartpole: bad stack shape");
  check(aca_env_step_cartpole(ptr<float>(state), ptr<int32_t>(t), ptr<int64_t>(tg), ptr<float>(ep_ret),
                              ptr<float>(ep_stats), ptr<int64_t>(ids), ptr<int32_t>(actions), ptr<float>(prev),
                              ptr<float>(out), ptr<float>(reward), ptr<uint8_t>(done), ptr<uint8_t>(trunc),
                              (uint32_t)seed, (int)max_steps, (int)k, N, final_out_ptr(final_out, out),
                              cur_stream(state)),
        "env_step_cartpole");
}

void env_step_pendulum(Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, Tensor ids, Tensor actions,
                       Tensor prev, Tensor out, Tensor reward, Tensor done, Tensor trunc, int64_t seed,
                       int64_t max_steps, int64_t k, c10::optional<Tensor> final_out) {
  check_env(state, t, tg, ep_ret, ep_stats, ids, reward, done, trunc);
  need(actions, at::kFloat, "actions");
  need(prev, at::kFloat, "prev");
  need(out, at::kFloat, "out");
  const int N = state.size(0);
  TORCH_CHECK(prev.numel() == (int64_t)N * 3 * k && out.numel() == prev.numel(), "pendulum: bad stack shape");
  const int act_dim = actions.numel() / N;
  check(aca_env_step_pendulum(ptr<float>(state), ptr<int32_t>(t), ptr<int64_t>(tg), ptr<float>(ep_ret),
                              ptr<float>(ep_stats), ptr<int64_t>(ids), ptr<float>(actions), act_dim, ptr<float>(prev),
                              ptr<float>(out), ptr<float>(reward), ptr<uint8_t>(done), ptr<uint8_t>(trunc),
                              (uint32_t)seed, (int)max_steps, (int)k, N, final_out_ptr(final_out, out),
                              cur_stream(state)),
        "env_step_pendulum");
}

void env_step_linear(Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, Tensor ids, Tensor actions,
                     Tensor A, Tensor B, Tensor prev, Tensor out, Tensor reward, Tensor done, Tensor trunc,
                     int64_t seed, int64_t max_steps, int64_t k, c10::optional<Tensor> final_out) {
  check_env(state, t, tg, ep_ret, ep_stats, ids, reward, done, trunc);
  need(actions, at::kFloat, "actions");
  need(A, at::kFloat, "A");
  need(B, at::kFloat, "B");
  need(prev, at::kFloat, "prev");
  need(out, at::kFloat, "out");
  const int N = state.size(0);
  TORCH_CHECK(state.size(1) == 17 && A.numel() == 17 * 17 && B.numel() == 17 * 6 && actions.numel() == N * 6,
              "linear env: bad shapes");
  TORCH_CHECK(prev.numel() == (int64_t)N * 17 * k && out.numel() == prev.numel(), "linear: bad stack shape");
  check(aca_env_step_linear(ptr<float>(state), ptr<int32_t>(t), ptr<int64_t>(tg), ptr<float>(ep_ret),
                            ptr<float>(ep_stats), ptr<int64_t>(ids), ptr<float>(actions), ptr<float>(A),
                            ptr<float>(B), ptr<float>(prev), ptr<float>(out), ptr<float>(reward),
                            ptr<uint8_t>(done), ptr<uint8_t>(trunc), (uint32_t)seed, (int)max_steps, (int)k, N,
                            final_out_ptr(final_out, out), cur_stream(state)),
        "env_step_linear");
}

void env_step_pong(Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, Tensor ids, Tensor actions,
                   Tensor prev, Tensor out, Tensor reward, Tensor done, Tensor trunc, int64_t seed, int64_t max_steps,
                   int64_t k) {
  check_env(state, t, tg, ep_ret, ep_stats, ids, reward, done, trunc);
  need(actions, at::kInt, "actions");
  need(prev, at::kByte, "prev");
  need(out, at::kByte, "out");
  const int N = state.size(0);
  TORCH_CHECK(state.size(1) == 8, "pong: state must be [N, 8]");
  TORCH_CHECK(prev.numel() == (int64_t)N * k * 84 * 84 && out.numel() == prev.numel(), "pong: bad stack shape");
  TORCH_CHECK(prev.data_ptr() != out.data_ptr(), "pong: prev and out must not alias");
  check(aca_env_step_pong(ptr<float>(state), ptr<int32_t>(t), ptr<int64_t>(tg), ptr<float>(ep_ret),
                          ptr<float>(ep_stats), ptr<int64_t>(ids), ptr<int32_t>(actions), ptr<uint8_t>(prev),
                          ptr<uint8_t>(out), ptr<float>(reward), ptr<uint8_t>(done), ptr<uint8_t>(trunc),
                          (uint32_t)seed, (int)max_steps, (int)k, N, cur_stream(state)),
        "env_step_pong");
}

// fused rollout step: policy/value head + sampling + env step (native engine, Pong/Breakout-shaped banks)
void env_policy_step_pong(Tensor h, Tensor Wh, Tensor bh, Tensor z, Tensor act, Tensor logp, Tensor ent,
                          Tensor value, int64_t key_shift, int64_t pseed, Tensor state, Tensor t, Tensor tg,
                          Tensor ep_ret, Tensor ep_stats, Tensor ids, Tensor prev, Tensor out, Tensor reward,
                          Tensor done, Tensor trunc, int64_t seed, int64_t max_steps, int64_t k, bool pre_shifted,
                          c10::optional<Tensor> hpart, int64_t planes, c10::optional<Tensor> bfc,
                          c10::optional<Tensor> stamps) {
  check_env(state, t, tg, ep_ret, ep_stats, ids, reward, done, trunc);
  need(h, at::kBFloat16, "h");
  need(Wh, at::kBFloat16, "Wh");
  need(bh, at::kFloat, "bh");
  need(z, at::kFloat, "z");
  need(act, at::kInt, "act");
  need(logp, at::kFloat, "logp");
  need(ent, at::kFloat, "ent");
  need(value, at::kFloat, "value");
  need(prev, at::kByte, "prev");
  need(out, at::kByte, "out");
  const int N = state.size(0);
  const int A1 = bh.numel(), A = A1 - 1;
  const int hdim = h.numel() / N;
  TORCH_CHECK(state.size(1) == 8 && h.numel() == (int64_t)N * hdim && Wh.numel() == (int64_t)hdim * A1 &&
                  z.numel() >= (int64_t)N * A1 && act.numel() >= N && value.numel() >= N,
              "env_policy_step_pong: bad shapes");
  TORCH_CHECK(A1 >= 3 && A1 <= 20 && hdim == 512 && reinterpret_cast<uintptr_t>(Wh.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(h.data_ptr()) % 16 == 0,
              "env_policy_step_pong: 2..19 actions, hidden size 512, h and Wh 16-byte aligned");
  TORCH_CHECK(prev.numel() == (int64_t)N * k * 84 * 84 && out.numel() == prev.numel(), "pong: bad stack shape");
  TORCH_CHECK(prev.data_ptr() != out.data_ptr(), "pong: prev and out must not alias");
  const float* hp = nullptr;
  const float* bf = nullptr;
  int64_t pstride = 0;
  if (hpart.has_value() && hpart->defined()) {
    need(*hpart, at::kFloat, "hpart");
    TORCH_CHECK(bfc.has_value() && bfc->defined() && bfc->numel() == hdim, "env_policy_step_pong: hpart needs bfc");
    need(*bfc, at::kFloat, "bfc");
    TORCH_CHECK(planes >= 1 && planes <= 32 && hpart->numel() % 32 == 0, "env_policy_step_pong: 1..32 planes");
    pstride = hpart->numel() / 32;   // buffer holds 32 planes of equal size (engine.py FC_PLANES)
    TORCH_CHECK(pstride >= (int64_t)N * hdim, "env_policy_step_pong: hpart planes too small");
    hp = ptr<float>(*hpart);
    bf = ptr<float>(*bfc);
  }
  check(aca_env_policy_step_pong(ptr<uint16_t>(h), hp, (int)planes, pstride, bf, hdim, ptr<uint16_t>(Wh),
                                 ptr<float>(bh), A, ptr<float>(z),
                                 ptr<int32_t>(act), ptr<float>(logp), ptr<float>(ent), ptr<float>(value),
                                 (int)key_shift, (uint32_t)pseed, ptr<float>(state), ptr<int32_t>(t),
                                 ptr<int64_t>(tg), ptr<float>(ep_ret), ptr<float>(ep_stats), ptr<int64_t>(ids),
                                 ptr<uint8_t>(prev), ptr<uint8_t>(out), ptr<float>(reward), ptr<uint8_t>(done),
                                 ptr<uint8_t>(trunc), (uint32_t)seed, (int)max_steps, (int)k, N, pre_shifted ? 1 : 0,
                                 stamps_ptr(stamps, N), cur_stream(state)),
        "env_policy_step_pong");
}

// Rollout step t of the Pong bank fused with the row-split trunk of the observation it produces (cnn_fused.hip
// pong_fused_step_kernel): env state read from (state, t, tg, ep_ret), committed to the other parity buffers
// (state_n, t_n, tg_n, ep_ret_n); prev = obs[t], out = obs[t+1] (frames 0..2 already shifted in), shift_out =
// obs[t+2] or None; y1..y3 = the trunk activations of obs[t+1].
void pong_fused_step(Tensor h, Tensor Wh, Tensor bh, Tensor z, Tensor act, Tensor logp, Tensor ent, Tensor value,
                     int64_t key_shift, int64_t pseed, Tensor state, Tensor t, Tensor tg, Tensor ep_ret,
                     Tensor state_n, Tensor t_n, Tensor tg_n, Tensor ep_ret_n, Tensor ep_stats, Tensor ids,
                     Tensor prev, Tensor out, Tensor reward, Tensor done, Tensor trunc, int64_t seed,
                     int64_t max_steps, Tensor hpart, int64_t planes, Tensor bfc, Tensor W1, Tensor b1, Tensor W2,
                     Tensor b2, Tensor W3, Tensor b3, Tensor y1, Tensor y2, Tensor y3, double scale,
                     c10::optional<Tensor> shift_out, c10::optional<Tensor> stamps, bool frag) {
  // frag: W2 / W3 are the fragment-ordered copies (ops/optim.py frag_order); W1 row-major
  check_env(state, t, tg, ep_ret, ep_stats, ids, reward, done, trunc);
  check_env(state_n, t_n, tg_n, ep_ret_n, ep_stats, ids, reward, done, trunc);
  for (auto* x : {&h, &Wh, &W1, &W2, &W3, &y1, &y2, &y3}) need(*x, at::kBFloat16, "pong_fused_step bf16");
  for (auto* x : {&bh, &z, &logp, &ent, &value, &hpart, &bfc, &b1, &b2, &b3}) need(*x, at::kFloat, "pong_fused_step f32");
  need(act, at::kInt, "act");
  need(prev, at::kByte, "prev");
  need(out, at::kByte, "out");
  const int N = state.size(0);
  const int A1 = bh.numel(), A = A1 - 1;
  TORCH_CHECK(A1 >= 3 && A1 <= 7, "pong_fused_step: 2..6 actions");
  TORCH_CHECK(state.size(1) == 8 && h.numel() == (int64_t)N * 512 && Wh.numel() == 512 * A1 &&
                  z.numel() >= (int64_t)N * A1 && act.numel() >= N && value.numel() >= N,
              "pong_fused_step: bad head shapes");
  TORCH_CHECK(prev.numel() == (int64_t)N * 4 * 84 * 84 && out.numel() == prev.numel() &&
                  prev.data_ptr() != out.data_ptr(), "pong_fused_step: frame stacks [N, 4, 84, 84], not aliased");
  TORCH_CHECK(state.data_ptr() != state_n.data_ptr() && t.data_ptr() != t_n.data_ptr() &&
                  tg.data_ptr() != tg_n.data_ptr() && ep_ret.data_ptr() != ep_ret_n.data_ptr(),
              "pong_fused_step: the next-parity env state must be separate buffers");
  TORCH_CHECK(W1.numel() == 32 * 256 && W2.numel() == 64 * 512 && W3.numel() == 64 * 576 && b1.numel() == 32 &&
                  b2.numel() == 64 && b3.numel() == 64 && y1.numel() == (int64_t)N * 400 * 32 &&
                  y2.numel() == (int64_t)N * 81 * 64 && y3.numel() == (int64_t)N * 49 * 64,
              "pong_fused_step: trunk shapes");
  for (const Tensor* x : {&prev, &out, &W1, &W2, &W3, &y1, &y2, &y3, &h, &Wh})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x->data_ptr()) % 16 == 0, "pong_fused_step: 16-byte aligned buffers");
  TORCH_CHECK(planes >= 1 && planes <= 32 && hpart.numel() % 32 == 0 && bfc.numel() == 512,
              "pong_fused_step: 1..32 fc planes");
  const int64_t pstride = hpart.numel() / 32;
  TORCH_CHECK(pstride >= (int64_t)N * 512, "pong_fused_step: hpart planes too small");
  uint8_t* so = nullptr;
  if (shift_out.has_value() && shift_out->defined()) {
    need(*shift_out, at::kByte, "shift_out");
    TORCH_CHECK(shift_out->numel() == prev.numel() && reinterpret_cast<uintptr_t>(shift_out->data_ptr()) % 16 == 0 &&
                    shift_out->data_ptr() != out.data_ptr(), "pong_fused_step: shift_out shape / aliasing");
    so = shift_out->data_ptr<uint8_t>();
  }
  check(aca_pong_fused_step(ptr<uint16_t>(h), ptr<float>(hpart), (int)planes, pstride, ptr<float>(bfc),
                            ptr<uint16_t>(Wh), ptr<float>(bh), A, ptr<float>(z), ptr<int32_t>(act), ptr<float>(logp),
                            ptr<float>(ent), ptr<float>(value), (int)key_shift, (uint32_t)pseed, ptr<float>(state),
                            ptr<int32_t>(t), ptr<int64_t>(tg), ptr<float>(ep_ret), ptr<float>(state_n),
                            ptr<int32_t>(t_n), ptr<int64_t>(tg_n), ptr<float>(ep_ret_n), ptr<float>(ep_stats),
                            ptr<int64_t>(ids), ptr<uint8_t>(prev), ptr<uint8_t>(out), ptr<float>(reward),
                            ptr<uint8_t>(done), ptr<uint8_t>(trunc), (uint32_t)seed, (int)max_steps,
                            ptr<uint16_t>(W1), ptr<float>(b1), ptr<uint16_t>(W2), ptr<float>(b2), ptr<uint16_t>(W3),
                            ptr<float>(b3), ptr<uint16_t>(y1), ptr<uint16_t>(y2), ptr<uint16_t>(y3), (float)scale,
                            so, stamps_ptr(stamps, N * 7), frag ? 1 : 0, N, cur_stream(state)),
        "pong_fused_step");
}

// Per-env fused rollout step (cnn_fused.hip pong_fused_env_step_kernel): policy/env step t of env e (fc planes of
// obs t -> h, head, sample, physics, commit into (state, t, tg, ep_ret)) + the new frame rendered into obs t+1 (out,
// frames 0..2 already shifted in) + frames 1..3 of obs t+1 shifted into shift_out (obs t+2, or None) + conv1..conv3
// of obs t+1 into y1..y3. One workgroup per env; with next_state = [state_n, t_n, tg_n, ep_ret_n] (the other parity's
// env state) two workgroups per env, the state committed there (the caller flips parity after the launch).
void pong_fused_env_step(Tensor h, Tensor Wh, Tensor bh, Tensor z, Tensor act, Tensor logp, Tensor ent, Tensor value,
                         int64_t key_shift, int64_t pseed, Tensor state, Tensor t, Tensor tg, Tensor ep_ret,
                         Tensor ep_stats, Tensor ids, Tensor out, Tensor reward, Tensor done, Tensor trunc,
                         int64_t seed, int64_t max_steps, Tensor hpart, int64_t planes, Tensor bfc, Tensor W1,
                         Tensor b1, Tensor W2, Tensor b2, Tensor W3, Tensor b3, Tensor y1, Tensor y2, Tensor y3,
                         double scale, c10::optional<Tensor> shift_out, c10::optional<std::vector<Tensor>> next_state,
                         c10::optional<Tensor> stamps, bool frag) {
  // frag: W2 / W3 are the fragment-ordered copies (ops/optim.py frag_order); W1 row-major
  check_env(state, t, tg, ep_ret, ep_stats, ids, reward, done, trunc);
  float* sn = nullptr; int32_t* tn = nullptr; int64_t* tgn = nullptr; float* ern = nullptr;
  if (next_state.has_value()) {
    const auto& v = *next_state;
    TORCH_CHECK(v.size() == 4, "pong_fused_env_step: next_state = [state, t, tg, ep_ret]");
    check_env(v[0], v[1], v[2], v[3], ep_stats, ids, reward, done, trunc);
    TORCH_CHECK(v[0].sizes() == state.sizes() && v[0].data_ptr() != state.data_ptr() &&
                    v[1].data_ptr() != t.data_ptr() && v[2].data_ptr() != tg.data_ptr() &&
                    v[3].data_ptr() != ep_ret.data_ptr(),
                "pong_fused_env_step: the next-parity env state must be separate buffers of the same shape");
    sn = ptr<float>(v[0]); tn = ptr<int32_t>(v[1]); tgn = ptr<int64_t>(v[2]); ern = ptr<float>(v[3]);
  }
  for (auto* x : {&h, &Wh, &W1, &W2, &W3, &y1, &y2, &y3}) need(*x, at::kBFloat16, "pong_fused_env_step bf16");
  for (auto* x : {&bh, &z, &logp, &ent, &value, &hpart, &bfc, &b1, &b2, &b3})
    need(*x, at::kFloat, "pong_fused_env_step f32");
  need(act, at::kInt, "act");
  need(out, at::kByte, "out");
  const int N = state.size(0);
  const int A1 = bh.numel();
  TORCH_CHECK(A1 >= 3 && A1 <= 7, "pong_fused_env_step: 2..6 actions");
  TORCH_CHECK(state.size(1) == 8 && h.numel() == (int64_t)N * 512 && Wh.numel() == 512 * A1 &&
                  z.numel() >= (int64_t)N * A1 && act.numel() >= N && value.numel() >= N,
              "pong_fused_env_step: bad head shapes");
  TORCH_CHECK(out.numel() == (int64_t)N * 4 * 84 * 84, "pong_fused_env_step: frame stack [N, 4, 84, 84]");
  TORCH_CHECK(W1.numel() == 32 * 256 && W2.numel() == 64 * 512 && W3.numel() == 64 * 576 && b1.numel() == 32 &&
                  b2.numel() == 64 && b3.numel() == 64 && y1.numel() == (int64_t)N * 400 * 32 &&
                  y2.numel() == (int64_t)N * 81 * 64 && y3.numel() == (int64_t)N * 49 * 64,
              "pong_fused_env_step: trunk shapes");
  for (const Tensor* x : {&out, &W1, &W2, &W3, &y1, &y2, &y3, &h, &Wh, &hpart, &bfc})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x->data_ptr()) % 16 == 0, "pong_fused_env_step: 16-byte aligned buffers");
  TORCH_CHECK(planes >= 1 && planes <= 32 && hpart.numel() % 32 == 0 && bfc.numel() == 512,
              "pong_fused_env_step: 1..32 fc planes");
  const int64_t pstride = hpart.numel() / 32;
  TORCH_CHECK(pstride >= (int64_t)N * 512, "pong_fused_env_step: hpart planes too small");
  uint8_t* so = nullptr;
  if (shift_out.has_value() && shift_out->defined()) {
    need(*shift_out, at::kByte, "shift_out");
    TORCH_CHECK(shift_out->numel() == out.numel() && reinterpret_cast<uintptr_t>(shift_out->data_ptr()) % 16 == 0 &&
                    shift_out->data_ptr() != out.data_ptr(), "pong_fused_env_step: shift_out shape / aliasing");
    so = shift_out->data_ptr<uint8_t>();
  }
  check(aca_pong_fused_env_step(ptr<uint16_t>(h), ptr<float>(hpart), (int)planes, pstride, ptr<float>(bfc),
                                ptr<uint16_t>(Wh), ptr<float>(bh), A1 - 1, ptr<float>(z), ptr<int32_t>(act),
                                ptr<float>(logp), ptr<float>(ent), ptr<float>(value), (int)key_shift, (uint32_t)pseed,
                                ptr<float>(state), ptr<int32_t>(t), ptr<int64_t>(tg), ptr<float>(ep_ret),
                                ptr<float>(ep_stats), ptr<int64_t>(ids), ptr<uint8_t>(out), ptr<float>(reward),
                                ptr<uint8_t>(done), ptr<uint8_t>(trunc), (uint32_t)seed, (int)max_steps,
                                ptr<uint16_t>(W1), ptr<float>(b1), ptr<uint16_t>(W2), ptr<float>(b2),
                                ptr<uint16_t>(W3), ptr<float>(b3), ptr<uint16_t>(y1), ptr<uint16_t>(y2),
                                ptr<uint16_t>(y3), (float)scale, so, sn, tn, tgn, ern, stamps_ptr(stamps, sn ? 2 * N : N),
                                frag ? 1 : 0, N, cur_stream(state)),
        "pong_fused_env_step");
}

// learner fc backward at B <= 256 rows (fc_bwd.hip): dy3 = (dh Wfc^T) * (y3 > 0) bf16, dW = y3^T dh fp32 (stored)
// sq (optional, fp32 >= 1568): per (dWfc tile, wave) sums of squares for the finaliser's norm partials
void fc_bwd(Tensor dh, Tensor W, Tensor y3, Tensor dy3, Tensor dW, c10::optional<Tensor> stamps,
            c10::optional<Tensor> sq) {
  for (auto* x : {&dh, &W, &y3, &dy3}) need(*x, at::kBFloat16, "fc_bwd bf16");
  need(dW, at::kFloat, "fc_bwd dW");
  const int64_t B = dh.numel() / 512;
  TORCH_CHECK(B >= 1 && B <= 256 && dh.numel() == B * 512 && y3.numel() == B * 3136 && dy3.numel() == B * 3136 &&
                  W.numel() == 3136 * 512 && dW.numel() == 3136 * 512,
              "fc_bwd: dh [B <= 256, 512], y3 / dy3 [B, 3136], W / dW [3136, 512]");
  for (const Tensor* x : {&dh, &W, &y3, &dy3, &dW})
    TORCH_CHECK(x->is_contiguous() && reinterpret_cast<uintptr_t>(x->data_ptr()) % 16 == 0,
                "fc_bwd: contiguous 16-byte aligned buffers");
  const int64_t nwg = 392 + ((B + 31) / 32) * 49;
  float* sqp = nullptr;
  if (sq.has_value() && sq->defined()) {
    need(*sq, at::kFloat, "fc_bwd sq");
    TORCH_CHECK(sq->numel() >= 392 * 4, "fc_bwd: sq needs 1568 floats");
    sqp = ptr<float>(*sq);
  }
  check(aca_fc_bwd(ptr<uint16_t>(dh), ptr<uint16_t>(W), ptr<uint16_t>(y3), ptr<uint16_t>(dy3), ptr<float>(dW), (int)B,
                   sqp, stamps_ptr(stamps, nwg / 4 + 1), cur_stream(dh)),
        "fc_bwd");
}

// rollout fc product as split-K partial planes on the fragment-ordered Wfc copy (fc_rollout.hip); hpart holds 32
// equal planes of [M, 512]; returns the number of planes written
// variant >= 16: variant - 16 with the 32-row blocks split over workgroups (gridDim.y) instead of looped per wave
int64_t fc_rollout(Tensor X, Tensor Wf, Tensor hpart, int64_t variant, c10::optional<Tensor> stamps) {
  need(X, at::kBFloat16, "X");
  need(Wf, at::kBFloat16, "Wf");
  need(hpart, at::kFloat, "hpart");
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1 && X.size(1) == 3136 && X.size(0) >= 1 && X.size(0) <= 128,
              "fc_rollout: X must be [M <= 128, 3136] row-major");
  TORCH_CHECK(Wf.numel() == 3136 * 512 && Wf.is_contiguous(), "fc_rollout: Wf must be the [3136 x 512] fragment copy");
  TORCH_CHECK(hpart.numel() % 32 == 0 && hpart.numel() / 32 >= X.size(0) * 512, "fc_rollout: hpart must hold 32 planes");
  int S = 0;
  check(aca_fc_rollout(ptr<uint16_t>(X), X.stride(0), (int)X.size(0), ptr<uint16_t>(Wf), 3136, 512, ptr<float>(hpart),
                       hpart.numel() / 32, (int)(variant & 15), 32, &S,
                       reinterpret_cast<unsigned long long*>(stamps_ptr(stamps, 1)), variant >= 16 ? 1 : 0,
                       cur_stream(X)),
        "fc_rollout");
  return S;
}

// bootstrap value from the fc partial planes (cnn_fused.hip); hpart holds 32 equal planes of [N, 512]
void fc_value(Tensor hpart, int64_t planes, Tensor bfc, Tensor Wh, Tensor bh, Tensor out, c10::optional<Tensor> h_out) {
  need(hpart, at::kFloat, "hpart");
  need(bfc, at::kFloat, "bfc");
  need(Wh, at::kBFloat16, "Wh");
  need(bh, at::kFloat, "bh");
  need(out, at::kFloat, "out");
  const int N = out.numel(), A1 = bh.numel();
  const int64_t pstride = hpart.numel() / 32;
  TORCH_CHECK(hpart.numel() % 32 == 0 && pstride >= (int64_t)N * 512 && planes >= 1 && planes <= 32,
              "fc_value: hpart must hold 32 planes of [N, 512]");
  TORCH_CHECK(bfc.numel() == 512 && Wh.numel() == 512 * A1, "fc_value: bad head shapes");
  uint16_t* ho = nullptr;
  if (h_out.has_value() && h_out->defined()) {
    need(*h_out, at::kBFloat16, "h_out");
    TORCH_CHECK(h_out->numel() >= (int64_t)N * 512, "fc_value: h_out too small");
    ho = ptr<uint16_t>(*h_out);
  }
  check(aca_fc_value(ptr<float>(hpart), (int)planes, pstride, ptr<float>(bfc), ptr<uint16_t>(Wh), A1, ptr<float>(bh),
                     ptr<float>(out), ho, N, cur_stream(out)),
        "fc_value");
}

// ---------------------------------------------------------------------------------------------- heads
// diagnostics: x [rows, 64] fp32 -> out [rows, 4, 64] (heads.hip wave_reduce_check_kernel)
void wave_reduce_check(Tensor x, Tensor out) {
  need(x, at::kFloat, "x");
  need(out, at::kFloat, "out");
  TORCH_CHECK(x.numel() % 64 == 0 && out.numel() == x.numel() * 4, "wave_reduce_check: x [rows, 64], out [rows, 4, 64]");
  check(aca_wave_reduce_check(ptr<float>(x), ptr<float>(out), (int)(x.numel() / 64), cur_stream(x)), "wave_reduce_check");
}

void categorical_sample(Tensor logits, Tensor keys, int64_t seed, Tensor act, Tensor logp, Tensor ent) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kFloat && logits.dim() == 2 && logits.stride(1) == 1,
              "categorical_sample: logits must be fp32 [B, A] with unit column stride");
  need(keys, at::kLong, "keys");
  need(act, at::kInt, "act");
  need(logp, at::kFloat, "logp");
  need(ent, at::kFloat, "ent");
  const int B = logits.size(0), A = logits.size(1);
  TORCH_CHECK(A <= 64, "categorical_sample: at most 64 actions");
  TORCH_CHECK(keys.numel() >= B && act.numel() >= B && logp.numel() >= B && ent.numel() >= B, "bad sizes");
  check(aca_categorical_sample(ptr<float>(logits), (int)logits.stride(0), B, A, ptr<int64_t>(keys), nullptr, nullptr, 0,
                               (uint32_t)seed, ptr<int32_t>(act), ptr<float>(logp), ptr<float>(ent), nullptr,
                               cur_stream(logits)),
        "categorical_sample");
}

// rollout form: keys from the env bank counters, optional copy of the fused head's value column (logits[:, A])
void categorical_sample_env(Tensor logits, Tensor tg, Tensor env_ids, int64_t key_shift, int64_t seed, Tensor act,
                            Tensor logp, Tensor ent, c10::optional<Tensor> vout) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kFloat && logits.dim() == 2 && logits.stride(1) == 1,
              "categorical_sample_env: logits must be fp32 [B, A] with unit column stride");
  need(tg, at::kLong, "tg");
  need(env_ids, at::kLong, "env_ids");
  need(act, at::kInt, "act");
  need(logp, at::kFloat, "logp");
  need(ent, at::kFloat, "ent");
  const int B = logits.size(0), A = logits.size(1);
  TORCH_CHECK(A <= 64, "categorical_sample_env: at most 64 actions");
  TORCH_CHECK(tg.numel() >= B && env_ids.numel() >= B && act.numel() >= B && logp.numel() >= B && ent.numel() >= B,
              "bad sizes");
  float* vo = nullptr;
  if (vout.has_value() && vout->defined()) {
    need(*vout, at::kFloat, "vout");
    TORCH_CHECK(vout->numel() >= B && logits.stride(0) > A, "vout needs a value column after the logits");
    vo = ptr<float>(*vout);
  }
  check(aca_categorical_sample(ptr<float>(logits), (int)logits.stride(0), B, A, nullptr, ptr<int64_t>(tg),
                               ptr<int64_t>(env_ids), (int)key_shift, (uint32_t)seed, ptr<int32_t>(act),
                               ptr<float>(logp), ptr<float>(ent), vo, cur_stream(logits)),
        "categorical_sample_env");
}

void gaussian_sample(Tensor mu, Tensor log_std, Tensor keys, int64_t seed, Tensor act, Tensor logp, Tensor ent) {
  TORCH_CHECK(mu.is_cuda() && mu.scalar_type() == at::kFloat && mu.dim() == 2 && mu.stride(1) == 1,
              "gaussian_sample: mu must be fp32 [B, A] with unit column stride");
  need(log_std, at::kFloat, "log_std");
  need(keys, at::kLong, "keys");
  need(act, at::kFloat, "act");
  need(logp, at::kFloat, "logp");
  need(ent, at::kFloat, "ent");
  const int B = mu.size(0), A = mu.size(1);
  TORCH_CHECK(log_std.numel() == A && act.numel() >= (int64_t)B * A, "gaussian_sample: bad sizes");
  check(aca_gaussian_sample(ptr<float>(mu), (int)mu.stride(0), B, A, ptr<float>(log_std), ptr<int64_t>(keys),
                            (uint32_t)seed, ptr<float>(act), ptr<float>(logp), ptr<float>(ent), cur_stream(mu)),
        "gaussian_sample");
}

// ---------------------------------------------------------------------------------------------- returns / stats
void check_returns(const Tensor& r, const Tensor& v, const Tensor& d, const Tensor& o1, const Tensor& o2) {
  need(r, at::kFloat, "rewards");
  need(v, at::kFloat, "values");
  need(d, at::kByte, "dones");
  need(o1, at::kFloat, "out1");
  need(o2, at::kFloat, "out2");
  TORCH_CHECK(r.dim() == 2 && v.dim() == 2 && v.size(0) == r.size(0) + 1 && v.size(1) == r.size(1) &&
                  d.sizes() == r.sizes() && o1.sizes() == r.sizes() && o2.sizes() == r.sizes(),
              "returns: expected rewards/dones [T, N], values [T+1, N]");
}

void gae(Tensor r, Tensor v, Tensor d, Tensor ret, Tensor adv, double gamma, double lam) {
  check_returns(r, v, d, ret, adv);
  check(aca_gae(ptr<float>(r), ptr<float>(v), ptr<uint8_t>(d), ptr<float>(ret), ptr<float>(adv), r.size(0), r.size(1),
                (float)gamma, (float)lam, cur_stream(r)),
        "gae");
}

void nstep_returns(Tensor r, Tensor v, Tensor d, Tensor tgt, Tensor adv, double gamma, int64_t L) {
  check_returns(r, v, d, tgt, adv);
  check(aca_nstep(ptr<float>(r), ptr<float>(v), ptr<uint8_t>(d), ptr<float>(tgt), ptr<float>(adv), r.size(0),
                  r.size(1), (float)gamma, (int)L, cur_stream(r)),
        "nstep_returns");
}

void normalize(Tensor a, Tensor out, double eps) {
  need(a, at::kFloat, "a");
  need(out, at::kFloat, "out");
  TORCH_CHECK(a.numel() == out.numel(), "normalize: size mismatch");
  check(aca_normalize(ptr<float>(a), ptr<float>(out), a.numel(), (float)eps, cur_stream(a)), "normalize");
}

// ev(x, y, out[, part, ticket]): with a workspace (part fp64 [>= ev_blocks(n) * 8], ticket int32 zeroed once) the
// many-workgroup form runs; without, the one-workgroup kernel.
void ev(Tensor x, Tensor y, Tensor out, c10::optional<Tensor> part, c10::optional<Tensor> ticket) {
  need(x, at::kFloat, "x");
  need(y, at::kFloat, "y");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.numel() >= 1, "ev: out must be fp32");
  TORCH_CHECK(x.numel() == y.numel(), "ev: size mismatch");
  if (part.has_value() && part->defined()) {
    need(*part, at::kDouble, "part");
    TORCH_CHECK(ticket.has_value() && ticket->is_cuda() && ticket->scalar_type() == at::kInt, "ev: ticket int32");
    TORCH_CHECK(part->numel() >= aca_ev_multi_blocks(x.numel()) * 8, "ev: part too small");
    check(aca_ev_multi(ptr<float>(x), ptr<float>(y), ptr<float>(out), x.numel(), ptr<double>(*part),
                       reinterpret_cast<unsigned int*>(ticket->data_ptr<int>()), cur_stream(x)),
          "ev_multi");
    return;
  }
  check(aca_ev(ptr<float>(x), ptr<float>(y), ptr<float>(out), x.numel(), cur_stream(x)), "ev");
}

int64_t ev_blocks(int64_t n) { return aca_ev_multi_blocks((int)n); }

std::vector<int64_t> returns_scan_geometry(int64_t T, int64_t N) {
  int E, CH, K, blocks;
  aca_returns_scan_geometry((int)T, (int)N, &E, &CH, &K, &blocks);
  return {E, CH, K, blocks};
}

// Chunked-scan returns (mode 1 n-step window L, 2 GAE) + moments + EV + optional in-place adv normalisation.
void returns_scan(Tensor r, Tensor v, Tensor d, Tensor ret, Tensor adv, int64_t mode, double gamma, double lam,
                  int64_t L, bool norm, double eps, Tensor part, Tensor ticket, Tensor mom,
                  c10::optional<Tensor> ev_out, c10::optional<Tensor> gz) {
  check_returns(r, v, d, ret, adv);
  const int T = r.size(0), N = r.size(1);
  TORCH_CHECK(mode == 1 || mode == 2, "returns_scan: mode 1 (n-step) or 2 (GAE)");
  int E, CH, K, blocks;
  aca_returns_scan_geometry(T, N, &E, &CH, &K, &blocks);
  need(part, at::kDouble, "part");
  need(mom, at::kDouble, "mom");
  TORCH_CHECK(part.numel() >= (int64_t)blocks * 8 && mom.numel() >= 8, "returns_scan: workspace too small");
  TORCH_CHECK(ticket.is_cuda() && ticket.scalar_type() == at::kInt, "returns_scan: ticket int32");
  double* gzp = nullptr;
  if (mode == 1 && L < T) {
    TORCH_CHECK(gz.has_value() && gz->defined(), "returns_scan: truncated n-step needs a gz workspace");
    need(*gz, at::kDouble, "gz");
    TORCH_CHECK(gz->numel() >= (int64_t)T * N, "returns_scan: gz too small");
    gzp = ptr<double>(*gz);
  }
  float* evp = nullptr;
  if (ev_out.has_value() && ev_out->defined()) {
    need(*ev_out, at::kFloat, "ev_out");
    evp = ptr<float>(*ev_out);
  }
  check(aca_returns_scan(ptr<float>(r), ptr<float>(v), ptr<uint8_t>(d), ptr<float>(ret), ptr<float>(adv), gzp,
                         ptr<double>(part), reinterpret_cast<unsigned int*>(ticket.data_ptr<int>()), ptr<double>(mom),
                         evp, T, N, (int)mode, (int)L, norm ? 1 : 0, (float)gamma, (float)lam, (float)eps,
                         cur_stream(r)),
        "returns_scan");
}

// conv1 weight gradient as P partial planes [P][32][256] (conv_wgrad.hip): obs uint8 [B, 4, 84, 84], dy1 bf16
// [B * 400, 32]; plane g holds samples [g B / P, (g + 1) B / P).
// obs_idx (optional int64 [B]): sample b's frames are row obs_idx[b] of obs (a PPO minibatch gathered by index)
// (conv1_wgrad2_kernel: all four channels per workgroup, 32x32x16 MFMAs, grid P)
void conv1_wgrad(Tensor obs, Tensor dy1, Tensor planes, int64_t P, double scale, c10::optional<Tensor> obs_idx) {
  TORCH_CHECK(obs.is_cuda() && obs.is_contiguous() && obs.scalar_type() == at::kByte, "conv1_wgrad: obs uint8");
  need(dy1, at::kBFloat16, "conv1_wgrad dy1");
  need(planes, at::kFloat, "conv1_wgrad planes");
  const int64_t rows = obs.numel() / (4 * 84 * 84);
  TORCH_CHECK(rows >= 1 && obs.numel() == rows * 4 * 84 * 84, "conv1_wgrad: obs [n, 4, 84, 84]");
  const int64_t* idx = nullptr;
  int64_t B = rows;
  if (obs_idx.has_value() && obs_idx->defined()) {
    need(*obs_idx, at::kLong, "obs_idx");
    B = obs_idx->numel();
    idx = obs_idx->data_ptr<int64_t>();
  }
  TORCH_CHECK(B >= 1 && dy1.numel() == B * 400 * 32, "conv1_wgrad: dy1 [B * 400, 32]");
  TORCH_CHECK(P >= 1 && P <= 1024 && planes.numel() >= P * 32 * 256, "conv1_wgrad: planes too small");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(obs.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dy1.data_ptr()) % 16 == 0,
              "conv1_wgrad: 16-byte aligned operands");
  check(aca_conv1_wgrad2(obs.data_ptr<uint8_t>(), ptr<uint16_t>(dy1), ptr<float>(planes), (int)B, (int)P,
                         (float)scale, idx, cur_stream(obs)),
        "conv1_wgrad");
}

// conv2 / conv3 weight gradient as P partial planes [P][64][KS KS C] from the batched-position MFMA 32x32x16 kernel
// (conv_wgrad.hip conv_wgrad_gemm_kernel): grid P, every workgroup owns its whole plane. layer 2: img = y1
// [B * 400, 32], dy = dy2 [B * 81, 64]; layer 3: img = y2 [B * 81, 64], dy = dy3 [B * 49, 64].
void conv_wgrad_gemm(int64_t layer, Tensor img, Tensor dy, Tensor planes, int64_t P) {
  need(img, at::kBFloat16, "conv_wgrad_gemm img");
  need(dy, at::kBFloat16, "conv_wgrad_gemm dy");
  need(planes, at::kFloat, "conv_wgrad_gemm planes");
  TORCH_CHECK(layer == 2 || layer == 3, "conv_wgrad_gemm: layer 2 or 3");
  const int64_t img_per = layer == 2 ? 400 * 32 : 81 * 64, dy_per = layer == 2 ? 81 * 64 : 49 * 64;
  const int64_t ncol = layer == 2 ? 512 : 576;
  const int64_t B = dy.numel() / dy_per;
  TORCH_CHECK(B >= 1 && dy.numel() == B * dy_per && img.numel() == B * img_per, "conv_wgrad_gemm: shapes");
  TORCH_CHECK(P >= 1 && P <= 1024 && planes.numel() >= P * 64 * ncol, "conv_wgrad_gemm: planes too small");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(img.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0,
              "conv_wgrad_gemm: 16-byte aligned operands");
  check(aca_conv_wgrad_gemm((int)layer, ptr<uint16_t>(img), ptr<uint16_t>(dy), ptr<float>(planes), (int)B, (int)P,
                            cur_stream(img)),
        "conv_wgrad_gemm");
}

// PPO minibatch k of epoch ep: rows prp_index(off + i, n, key(seed, *uc, ep)) of the rollout gathered in one launch.
// o_obs None + o_idx (int64 [mb]): index mode -- the source row of every minibatch row is written instead of a copy
// of its observation (the minibatch's trunk forward and conv1 weight gradient read through it)
void mb_gather(Tensor obs, Tensor act, Tensor logp, Tensor adv, Tensor ret, Tensor v, c10::optional<Tensor> o_obs_opt,
               Tensor o_act, Tensor o_logp, Tensor o_adv, Tensor o_ret, Tensor o_v, int64_t seed, Tensor uc,
               int64_t ep, int64_t off, c10::optional<Tensor> mom, double eps, c10::optional<Tensor> bump_ticket,
               c10::optional<Tensor> o_idx) {
  const double* momp = nullptr;
  unsigned int* tk = nullptr;
  if (bump_ticket.has_value() && bump_ticket->defined()) {
    need(*bump_ticket, at::kInt, "bump_ticket");
    tk = reinterpret_cast<unsigned int*>(bump_ticket->data_ptr<int32_t>());
  }
  if (mom.has_value() && mom->defined()) {
    need(*mom, at::kDouble, "mom");
    TORCH_CHECK(mom->numel() >= 3, "mb_gather: mom needs [count, sum, sum of squares]");
    momp = ptr<double>(*mom);
  }
  TORCH_CHECK(obs.is_cuda() && obs.is_contiguous() && obs.scalar_type() == at::kByte, "mb_gather: obs uint8");
  const bool by_index = o_idx.has_value() && o_idx->defined();
  TORCH_CHECK(by_index != (o_obs_opt.has_value() && o_obs_opt->defined()), "mb_gather: exactly one of o_obs, o_idx");
  int64_t* idxp = nullptr;
  uint8_t* oobs = nullptr;
  int64_t mb = 0;
  if (by_index) {
    need(*o_idx, at::kLong, "o_idx");
    idxp = o_idx->data_ptr<int64_t>();
    mb = o_idx->numel();
  } else {
    const Tensor& o_obs = *o_obs_opt;
    TORCH_CHECK(o_obs.is_cuda() && o_obs.is_contiguous() && o_obs.scalar_type() == at::kByte, "mb_gather: o_obs");
    oobs = o_obs.data_ptr<uint8_t>();
    mb = o_obs.size(0);
  }
  need(act, at::kInt, "act");
  need(o_act, at::kInt, "o_act");
  for (auto* t : {&logp, &adv, &ret, &v, &o_logp, &o_adv, &o_ret, &o_v}) need(*t, at::kFloat, "mb_gather f32");
  TORCH_CHECK(uc.is_cuda() && uc.scalar_type() == at::kLong, "mb_gather: update counter int64");
  const int64_t n = obs.size(0);
  const int64_t R = obs.numel() / n;
  TORCH_CHECK(by_index || o_obs_opt->numel() == mb * R, "mb_gather: o_obs shape");
  TORCH_CHECK(act.numel() == n && logp.numel() == n && adv.numel() == n && ret.numel() == n && v.numel() == n,
              "mb_gather: per-row inputs must have n rows");
  TORCH_CHECK(o_act.numel() == mb && o_logp.numel() == mb && o_adv.numel() == mb && o_ret.numel() == mb &&
                  o_v.numel() == mb, "mb_gather: per-row outputs must have mb rows");
  TORCH_CHECK(off >= 0 && off + mb <= n, "mb_gather: minibatch out of range");
  check(aca_mb_gather(obs.data_ptr<uint8_t>(), R, ptr<int>(act), ptr<float>(logp), ptr<float>(adv), ptr<float>(ret),
                      ptr<float>(v), oobs, ptr<int>(o_act), ptr<float>(o_logp),
                      ptr<float>(o_adv), ptr<float>(o_ret), ptr<float>(o_v), (int)mb, (int)n, (uint32_t)seed,
                      uc.data_ptr<int64_t>(), (int)ep, (int)off, momp, (float)eps, tk, idxp, cur_stream(obs)),
        "mb_gather");
}

void normalize_mom(Tensor a, Tensor out, Tensor mom, double eps) {
  need(a, at::kFloat, "a");
  need(out, at::kFloat, "out");
  need(mom, at::kDouble, "mom");
  TORCH_CHECK(a.numel() == out.numel() && mom.numel() >= 3, "normalize_mom: bad sizes");
  check(aca_normalize_mom(ptr<float>(a), ptr<float>(out), ptr<double>(mom), a.numel(), (float)eps, cur_stream(a)),
        "normalize_mom");
}

void moments(Tensor x, Tensor y, Tensor out) {
  need(x, at::kFloat, "x");
  need(y, at::kFloat, "y");
  need(out, at::kFloat, "out");
  TORCH_CHECK(x.numel() == y.numel() && out.numel() >= 5, "moments: bad sizes");
  check(aca_moments(ptr<float>(x), ptr<float>(y), ptr<float>(out), x.numel(), cur_stream(x)), "moments");
}

// ---------------------------------------------------------------------------------------------- optimisers
// Writes aca_sumsq_parts() partial sums of squares (unused slots zeroed); the optimisers reduce them.
void sumsq(Tensor x, Tensor partial) {
  const bool bf16 = x.scalar_type() == at::kBFloat16;
  need(x, bf16 ? at::kBFloat16 : at::kFloat, "x");
  need(partial, at::kFloat, "partial");
  TORCH_CHECK(partial.numel() >= aca_sumsq_parts(), "sumsq: partial needs ", aca_sumsq_parts(), " slots");
  check(aca_sumsq(x.data_ptr(), x.numel(), ptr<float>(partial), bf16 ? 1 : 0, cur_stream(x)), "sumsq");
}

// optional bf16 gradient the optimiser reads in place of g (the all-reduced bf16 comm buffer of the same group)
const uint16_t* g16_ptr(const c10::optional<Tensor>& g16, const Tensor& p, const char* who) {
  if (!(g16.has_value() && g16->defined())) return nullptr;
  need(*g16, at::kBFloat16, "g16");
  TORCH_CHECK(g16->numel() == p.numel(), who, ": g16 size mismatch");
  return ptr<uint16_t>(*g16);
}

// several sums of squares (one partial set each) in one launch: the per-group norms of a multi-group optimiser step
void sumsq_multi(std::vector<Tensor> xs, std::vector<Tensor> partials) {
  TORCH_CHECK(!xs.empty() && xs.size() <= 4 && xs.size() == partials.size(), "sumsq_multi: 1..4 (x, partial) pairs");
  const float* xp[4];
  float* pp[4];
  size_t ns[4];
  for (size_t g = 0; g < xs.size(); ++g) {
    need(xs[g], at::kFloat, "x");
    need(partials[g], at::kFloat, "partial");
    TORCH_CHECK(partials[g].numel() >= aca_sumsq_parts(), "sumsq_multi: partial needs ", aca_sumsq_parts(), " slots");
    xp[g] = ptr<float>(xs[g]);
    pp[g] = ptr<float>(partials[g]);
    ns[g] = xs[g].numel();
  }
  check(aca_sumsq_multi(xp, ns, pp, (int)xs.size(), cur_stream(xs[0])), "sumsq_multi");
}

const float* gnorm_parts_ptr(const c10::optional<Tensor>& parts, double max_norm, const char* who) {
  if (max_norm <= 0) return nullptr;
  TORCH_CHECK(parts.has_value() && parts->defined(), who, ": max_norm needs the sumsq partials");
  need(*parts, at::kFloat, "gnorm_parts");
  TORCH_CHECK(parts->numel() >= aca_sumsq_parts(), who, ": gnorm_parts too small");
  return ptr<float>(*parts);
}

uint16_t* shadow_ptr(const c10::optional<Tensor>& shadow, const Tensor& p, const char* who) {
  if (!(shadow.has_value() && shadow->defined() && shadow->numel() > 0)) return nullptr;
  need(*shadow, at::kBFloat16, "shadow");
  TORCH_CHECK(shadow->numel() == p.numel(), who, ": shadow size mismatch");
  return ptr<uint16_t>(*shadow);
}

// trans: optional CPU int64 [6, 5] table of weight copies the update writes as it goes (optim.hip OptTrans)
static const int64_t* trans_table(const c10::optional<Tensor>& trans, const char* who) {
  if (!(trans.has_value() && trans->defined())) return nullptr;
  TORCH_CHECK(!trans->is_cuda() && trans->scalar_type() == at::kLong && trans->is_contiguous() &&
                  trans->numel() == 8 * 5, who, ": trans must be CPU int64 [8, 5]");
  return ptr<int64_t>(*trans);
}

void adam_step(Tensor p, Tensor g, Tensor m, Tensor v, Tensor lr, Tensor t, c10::optional<Tensor> gnorm_parts,
               c10::optional<Tensor> gnorm_out, c10::optional<Tensor> shadow, double b1, double b2, double eps,
               double clip, double max_norm, Tensor ticket, bool zero_grad, double gmul, double norm_mul,
               c10::optional<Tensor> trans, c10::optional<Tensor> g16) {
  need(p, at::kFloat, "p");
  need(g, at::kFloat, "g");
  need(m, at::kFloat, "m");
  need(v, at::kFloat, "v");
  need(lr, at::kFloat, "lr");
  need(t, at::kFloat, "t");
  TORCH_CHECK(ticket.numel() >= 9 * 32, "adam_step: the step ticket needs 9 x 32 words (8 shards + top)");
  TORCH_CHECK(g.numel() == p.numel() && m.numel() == p.numel() && v.numel() == p.numel(), "adam: size mismatch");
  check(aca_adam_step(ptr<float>(p), ptr<float>(g), ptr<float>(m), ptr<float>(v), p.numel(), ptr<float>(lr),
                      ptr<float>(t), gnorm_parts_ptr(gnorm_parts, max_norm, "adam"), optr<float>(gnorm_out),
                      shadow_ptr(shadow, p, "adam"), (float)b1, (float)b2, (float)eps, (float)clip, (float)max_norm,
                      ptr<unsigned int>(ticket), zero_grad ? 1 : 0, (float)gmul, (float)norm_mul,
                      trans_table(trans, "adam_step"), g16_ptr(g16, p, "adam_step"), cur_stream(p)),
        "adam_step");
}

void rmsprop_step(Tensor p, Tensor g, Tensor v, Tensor lr, c10::optional<Tensor> gnorm_parts,
                  c10::optional<Tensor> gnorm_out, c10::optional<Tensor> shadow, double alpha, double eps,
                  double clip, double max_norm, bool zero_grad, double gmul, double norm_mul,
                  c10::optional<Tensor> trans, c10::optional<Tensor> g16) {
  need(p, at::kFloat, "p");
  need(g, at::kFloat, "g");
  need(v, at::kFloat, "v");
  need(lr, at::kFloat, "lr");
  TORCH_CHECK(g.numel() == p.numel() && v.numel() == p.numel(), "rmsprop: size mismatch");
  check(aca_rmsprop_step(ptr<float>(p), ptr<float>(g), ptr<float>(v), p.numel(), ptr<float>(lr),
                         gnorm_parts_ptr(gnorm_parts, max_norm, "rmsprop"), optr<float>(gnorm_out),
                         shadow_ptr(shadow, p, "rmsprop"), (float)alpha, (float)eps, (float)clip, (float)max_norm,
                         zero_grad ? 1 : 0, (float)gmul, (float)norm_mul, trans_table(trans, "rmsprop_step"),
                         g16_ptr(g16, p, "rmsprop_step"), cur_stream(p)),
        "rmsprop_step");
}

// ---------------------------------------------------------------------------------------------- MLP engine
// desc: device int64 [2 * sizeof(MlpTower) / 8] built by ops/mlp.py (pointers into the parameter / gradient slabs
// and the training workspace); lds: dynamic LDS bytes computed there for (desc, mode).
template <typename T>
const T* copt(const c10::optional<Tensor>& t, at::ScalarType dt, const char* name) {
  if (!(t.has_value() && t->defined())) return nullptr;
  need(*t, dt, name);
  return ptr<T>(*t);
}

// Large-batch learner head (ppo_head.hip): z = h Wh + bh, the PPO-clip / A2C loss, dz, dh = (h > 0) dz Wh^T and
// per-workgroup partial planes of dWh [P, 512 * A1], dbh [P, A1], dbfc [P, 512] (P = ppo_head_planes(B), reduced in
// plane order by the gradient finaliser); stats[0..6] written by the last workgroup (pstats: double [P, 6] scratch,
// ticket: int32 zero-initialised, self-cleaning).
void ppo_head(Tensor h, Tensor Wh, Tensor bh, Tensor act, Tensor logp_old, Tensor adv, Tensor ret,
              c10::optional<Tensor> v_old, Tensor ent_coef, Tensor kl_coef, double vf_coef, double ppo_clip,
              double v_clip, Tensor dh, c10::optional<Tensor> z_out, Tensor pWh, Tensor pbh, Tensor pbfc,
              Tensor pstats, c10::optional<Tensor> ticket, Tensor stats, c10::optional<Tensor> hp, int64_t hp_planes,
              c10::optional<Tensor> hbias) {
  need(h, at::kBFloat16, "h");
  need(Wh, at::kBFloat16, "Wh");
  need(dh, at::kBFloat16, "dh");
  for (auto* x : {&bh, &logp_old, &adv, &ret, &ent_coef, &kl_coef, &pWh, &pbh, &pbfc, &stats})
    need(*x, at::kFloat, "ppo_head f32 operand");
  need(act, at::kInt, "act");
  need(pstats, at::kDouble, "pstats");
  const int64_t B = act.numel(), A1 = bh.numel();
  TORCH_CHECK(A1 >= 3 && A1 <= 8, "ppo_head: 2..7 actions + value");
  TORCH_CHECK(h.is_contiguous() && h.numel() == B * 512 && dh.is_contiguous() && dh.numel() == B * 512,
              "ppo_head: h / dh must be contiguous [B, 512]");
  TORCH_CHECK(Wh.is_contiguous() && Wh.numel() == 512 * A1, "ppo_head: Wh must be contiguous [512, A1]");
  TORCH_CHECK(logp_old.numel() >= B && adv.numel() >= B && ret.numel() >= B, "ppo_head: row operands too small");
  const int64_t P = aca_ppo_head_planes((int)B);
  TORCH_CHECK(pWh.numel() >= P * 512 * A1 && pbh.numel() >= P * A1 && pbfc.numel() >= P * 512 &&
                  pstats.numel() >= P * aca::PH_NSTAT && stats.numel() >= 7,
              "ppo_head: plane / scratch buffers too small");
  aca::PpoHeadArgs a{};
  a.h = ptr<uint16_t>(h);
  a.Wh = ptr<uint16_t>(Wh);
  a.bh = ptr<float>(bh);
  a.act = ptr<int32_t>(act);
  a.logp_old = ptr<float>(logp_old);
  a.adv = ptr<float>(adv);
  a.ret = ptr<float>(ret);
  a.v_old = copt<float>(v_old, at::kFloat, "v_old");
  TORCH_CHECK(v_clip <= 0.0 || a.v_old, "ppo_head: value clipping needs v_old");
  a.ent_coef = ptr<float>(ent_coef);
  a.kl_coef = ptr<float>(kl_coef);
  a.vf_coef = (float)vf_coef;
  a.ppo_clip = (float)ppo_clip;
  a.v_clip = (float)v_clip;
  a.dh = ptr<uint16_t>(dh);
  a.z_out = const_cast<float*>(copt<float>(z_out, at::kFloat, "z_out"));
  if (a.z_out) TORCH_CHECK(z_out->numel() >= B * A1, "ppo_head: z_out too small");
  a.pWh = ptr<float>(pWh);
  a.pbh = ptr<float>(pbh);
  a.pbfc = ptr<float>(pbfc);
  a.pstats = ptr<double>(pstats);
  // (no ticket: the statistics records are summed by the gradient finaliser's duty, grad_finalize)
  a.ticket = reinterpret_cast<unsigned int*>(const_cast<int32_t*>(copt<int32_t>(ticket, at::kInt, "ticket")));
  a.stats = ptr<float>(stats);
  a.B = (int)B;
  if (hp.has_value() && hp->defined()) {
    need(*hp, at::kFloat, "hp");
    TORCH_CHECK(hp_planes >= 1 && hp_planes <= 4 && hp->numel() >= hp_planes * B * 512,
                "ppo_head: hp must hold hp_planes (1..4) planes of [B, 512]");
    TORCH_CHECK(hbias.has_value() && hbias->defined() && hbias->scalar_type() == at::kFloat && hbias->numel() >= 512,
                "ppo_head: hp needs the fp32 fc bias");
    a.hp = ptr<float>(*hp);
    a.hbias = ptr<float>(*hbias);
    a.hp_stride = B * 512;
    a.hp_planes = (int)hp_planes;
  }
  check(aca_ppo_head(&a, (int)A1, cur_stream(h)), "ppo_head");
}

int64_t ppo_head_planes(int64_t B) { return aca_ppo_head_planes((int)B); }
// float4 groups per thread of the single-segment optimiser launches (1, 2 or 4; A/B diagnostics); returns the value
int64_t opt_set_unroll(int64_t u) { return aca_opt_set_unroll((int)u); }
// diagnostics: optimiser launches write s_memtime phase stamps of every workgroup ([workgroup][8] int64) into buf
// (None: off); see optim.hip opt_body
void opt_set_stamps(c10::optional<Tensor> buf) {
  int64_t* p = nullptr;
  if (buf.has_value() && buf->defined()) {
    need(*buf, at::kLong, "buf");
    p = buf->data_ptr<int64_t>();
  }
  aca_opt_set_stamps(p);
}

void prp_perm(Tensor out, int64_t seed, Tensor uc, int64_t epoch) {
  need(out, at::kLong, "out");
  need(uc, at::kLong, "uc");
  check(aca_prp_perm(ptr<int64_t>(out), (int)out.numel(), (uint32_t)seed, ptr<int64_t>(uc), (int)epoch,
                     cur_stream(out)),
        "prp_perm");
}

void mlp_fwd(Tensor desc, int64_t tw_base, int64_t ntw, int64_t mode, int64_t lds, Tensor obs,
             c10::optional<Tensor> idx, c10::optional<Tensor> perm_uc, int64_t perm_ep, int64_t perm_off,
             int64_t perm_n, int64_t perm_seed, int64_t B, int64_t head, int64_t A, c10::optional<Tensor> log_std,
             c10::optional<Tensor> ac_scale, c10::optional<Tensor> tg, c10::optional<Tensor> env_ids,
             int64_t key_shift, int64_t seed, c10::optional<Tensor> act_out, c10::optional<Tensor> logp_out,
             c10::optional<Tensor> ent_out, c10::optional<Tensor> v_out, c10::optional<Tensor> act_in,
             c10::optional<Tensor> logp_old, c10::optional<Tensor> adv, c10::optional<Tensor> ret,
             c10::optional<Tensor> v_old, c10::optional<Tensor> ent_coef, c10::optional<Tensor> kl_coef,
             double vf_coef, double ppo_clip, double v_clip, bool ppo, c10::optional<Tensor> g_log_std,
             c10::optional<Tensor> mstats, c10::optional<Tensor> mpart, c10::optional<Tensor> stamps,
             c10::optional<Tensor> hdesc) {
  need(desc, at::kLong, "desc");
  TORCH_CHECK(desc.numel() * 8 >= (int64_t)(2 * sizeof(aca::MlpTower)), "mlp_fwd: desc too small");
  TORCH_CHECK(obs.is_cuda() && obs.scalar_type() == at::kFloat && obs.dim() == 2 && obs.stride(1) == 1,
              "mlp_fwd: obs must be fp32 [rows, D] with unit column stride");
  aca::MlpArgs a{};
  a.tw = reinterpret_cast<const aca::MlpTower*>(desc.data_ptr());
  a.tw_base = (int)tw_base;
  a.B = (int)B;
  a.D = (int)obs.size(1);
  a.obs = ptr<float>(obs);
  a.ld_obs = obs.stride(0);
  a.idx = copt<int64_t>(idx, at::kLong, "idx");
  a.perm_uc = copt<int64_t>(perm_uc, at::kLong, "perm_uc");
  a.perm_ep = (int)perm_ep;
  a.perm_off = (int)perm_off;
  a.perm_n = (int)perm_n;
  a.perm_seed = (uint32_t)perm_seed;
  if (a.perm_uc) TORCH_CHECK(perm_n > 0 && perm_off + B <= perm_n && obs.size(0) >= perm_n,
                             "mlp_fwd: minibatch permutation out of range");
  if (!a.idx && !a.perm_uc) TORCH_CHECK(obs.size(0) >= B, "mlp_fwd: obs has fewer rows than B");
  a.mode = (int)mode;
  a.head = (int)head;
  a.A = (int)A;
  a.log_std = copt<float>(log_std, at::kFloat, "log_std");
  a.ac_scale = copt<float>(ac_scale, at::kFloat, "ac_scale");
  a.tg = copt<int64_t>(tg, at::kLong, "tg");
  a.env_ids = copt<int64_t>(env_ids, at::kLong, "env_ids");
  a.key_shift = (int)key_shift;
  a.seed = (uint32_t)seed;
  const bool gauss = head == 2;
  if (act_out.has_value() && act_out->defined()) {
    if (gauss) a.act_f_out = const_cast<float*>(copt<float>(act_out, at::kFloat, "act_out"));
    else a.act_i_out = const_cast<int32_t*>(copt<int32_t>(act_out, at::kInt, "act_out"));
  }
  if (act_in.has_value() && act_in->defined()) {
    if (gauss) a.act_f_in = copt<float>(act_in, at::kFloat, "act_in");
    else a.act_i_in = copt<int32_t>(act_in, at::kInt, "act_in");
  }
  a.logp_out = const_cast<float*>(copt<float>(logp_out, at::kFloat, "logp_out"));
  a.ent_out = const_cast<float*>(copt<float>(ent_out, at::kFloat, "ent_out"));
  a.v_out = const_cast<float*>(copt<float>(v_out, at::kFloat, "v_out"));
  a.logp_old = copt<float>(logp_old, at::kFloat, "logp_old");
  a.adv = copt<float>(adv, at::kFloat, "adv");
  a.ret = copt<float>(ret, at::kFloat, "ret");
  a.v_old = copt<float>(v_old, at::kFloat, "v_old");
  a.ent_coef = copt<float>(ent_coef, at::kFloat, "ent_coef");
  a.kl_coef = copt<float>(kl_coef, at::kFloat, "kl_coef");
  a.vf_coef = (float)vf_coef;
  a.ppo_clip = (float)ppo_clip;
  a.v_clip = (float)v_clip;
  a.ppo = ppo ? 1 : 0;
  a.g_log_std = const_cast<float*>(copt<float>(g_log_std, at::kFloat, "g_log_std"));
  a.mstats = const_cast<float*>(copt<float>(mstats, at::kFloat, "mstats"));
  a.mpart = const_cast<float*>(copt<float>(mpart, at::kFloat, "mpart"));
  if (a.mpart) TORCH_CHECK(mode == 2 && mpart->numel() >= (B + 15) / 16 * aca::MPART_W,
                           "mlp_fwd: mpart must hold ceil(B/16) rows of ", aca::MPART_W, " (train mode)");
  a.inv_B = B > 0 ? 1.0f / (float)B : 0.f;
  a.stamps = reinterpret_cast<int64_t*>(stamps_ptr(stamps, 2));   // [2 towers][16 phases]
  // SPEC train path (mlp.hip): hdesc = the CPU copy of desc; taken when both towers have the reference shapes
  int spec = 0;
  if (hdesc.has_value() && hdesc->defined() && mode == 2 && tw_base == 0 && ntw == 2) {
    TORCH_CHECK(!hdesc->is_cuda() && hdesc->scalar_type() == at::kLong && hdesc->is_contiguous() &&
                    hdesc->numel() * 8 >= (int64_t)(2 * sizeof(aca::MlpTower)), "mlp_fwd: hdesc must be the CPU desc");
    std::memcpy(a.htw, hdesc->data_ptr(), sizeof(a.htw));
    const aca::MlpTower& P = a.htw[0];
    const aca::MlpTower& C = a.htw[1];
    const int D = (int)obs.size(1);
    const int g0 = D <= 16 ? 1 : D <= 32 ? 2 : D <= 64 ? 4 : 0;
    const bool ok = g0 && P.nl == 4 && P.in[0] == D && P.out[0] == 128 && P.out[1] == 128 && P.out[2] == 64 &&
                    P.out[3] >= 1 && P.out[3] <= 16 && P.out[3] == A && C.nl == 3 && C.in[0] == D &&
                    C.out[0] == 256 && C.out[1] == 128 && C.out[2] == 1;
    if (ok) {
      for (int t = 0; t < 2; ++t)
        for (int l = 0; l < (int)a.htw[t].nl; ++l)
          TORCH_CHECK(a.htw[t].F[l] && (l == 0 || a.htw[t].G[l]) && a.htw[t].xs[l] && a.htw[t].dp[l],
                      "mlp_fwd: hdesc lacks fragment copies / workspace");
      spec = g0;
    }
  }
  const bool policy = tw_base == 0;
  if (policy) {
    TORCH_CHECK(head == 1 || head == 2, "mlp_fwd: policy tower needs head 1 (categorical) or 2 (gaussian)");
    if (gauss) TORCH_CHECK(a.log_std && a.ac_scale, "mlp_fwd: gaussian head needs log_std and ac_scale");
    if (mode == 0) TORCH_CHECK((gauss ? (void*)a.act_f_out : (void*)a.act_i_out) && a.tg && a.env_ids,
                               "mlp_fwd: rollout needs act_out, tg, env_ids");
    if (mode == 1) TORCH_CHECK(gauss ? (bool)a.act_f_in : (bool)a.act_i_in, "mlp_fwd: evaluate needs act_in");
  }
  if (mode == 2) {
    TORCH_CHECK(a.mstats && a.ret && a.ent_coef && a.kl_coef, "mlp_fwd: train needs mstats, ret, coefficients");
    if (policy) TORCH_CHECK(a.logp_old && a.adv && (gauss ? (bool)a.act_f_in : (bool)a.act_i_in) &&
                                (!gauss || a.g_log_std), "mlp_fwd: train needs actions, logp_old, adv (+ g_log_std)");
    if (ppo && v_clip > 0) TORCH_CHECK(a.v_old, "mlp_fwd: clipped value loss needs v_old");
  }
  check(aca_mlp_fwd(&a, (int)ntw, (size_t)lds, spec, cur_stream(obs)), "mlp_fwd");
}

void mlp_tshadow(Tensor desc, int64_t ntw, int64_t total) {
  need(desc, at::kLong, "desc");
  check(aca_mlp_tshadow(reinterpret_cast<const aca::MlpTower*>(desc.data_ptr()), (int)ntw, (int)total,
                        cur_stream(desc)),
        "mlp_tshadow");
}

// items: device int64 [nitems, 8] (ops/mlp.py MLPEngine.wgrad_items); nrt: 16-row tiles of the batch
void mlp_wgrad(Tensor items, int64_t nrt, int64_t nsplit, c10::optional<Tensor> g_log_std, int64_t A,
               c10::optional<Tensor> ls_part, double ls_clip, c10::optional<Tensor> stats, Tensor ent_coef,
               Tensor kl_coef, Tensor mpart, int64_t mpart_rows, c10::optional<Tensor> bump) {
  need(items, at::kLong, "items");
  TORCH_CHECK(items.dim() == 2 && items.size(1) == 8 && items.size(0) >= 1, "mlp_wgrad: items must be [n, 8]");
  aca::WgradArgs a{};
  if (bump.has_value() && bump->defined()) {
    need(*bump, at::kLong, "bump");
    a.bump = bump->data_ptr<int64_t>();
  }
  need(mpart, at::kFloat, "mpart");
  TORCH_CHECK(mpart_rows >= 0 && mpart.numel() >= mpart_rows * aca::MPART_W && A <= 16, "mlp_wgrad: mpart too small");
  a.items = items.data_ptr<int64_t>();
  a.nitems = (int)items.size(0);
  a.nrt = (int)nrt;
  a.nsplit = (int)nsplit;
  a.g_log_std = const_cast<float*>(copt<float>(g_log_std, at::kFloat, "g_log_std"));
  a.A = (int)A;
  a.ls_part = const_cast<float*>(copt<float>(ls_part, at::kFloat, "ls_part"));
  a.ls_clip = (float)ls_clip;
  a.stats = const_cast<float*>(copt<float>(stats, at::kFloat, "stats"));
  need(ent_coef, at::kFloat, "ent_coef");
  need(kl_coef, at::kFloat, "kl_coef");
  a.ent_coef = ent_coef.data_ptr<float>();
  a.kl_coef = kl_coef.data_ptr<float>();
  a.mpart = mpart.data_ptr<float>();
  a.mpart_rows = (int)mpart_rows;
  check(aca_mlp_wgrad(&a, cur_stream(items)), "mlp_wgrad");
}

// PPO epoch gather for the MLP engine: out rows i = in rows prp(i) (keyed by the device update counter uc, epoch ep)
void mlp_epoch_gather(Tensor obs, Tensor act, Tensor logp, Tensor adv, Tensor ret, c10::optional<Tensor> v,
                      Tensor o_obs, Tensor o_act, Tensor o_logp, Tensor o_adv, Tensor o_ret, c10::optional<Tensor> o_v,
                      Tensor uc, int64_t ep, int64_t seed) {
  TORCH_CHECK(obs.is_cuda() && obs.scalar_type() == at::kFloat && obs.dim() == 2 && obs.stride(1) == 1,
              "mlp_epoch_gather: obs must be fp32 [n, D] with unit column stride");
  const int64_t n = obs.size(0), D = obs.size(1);
  TORCH_CHECK(act.is_cuda() && act.is_contiguous() && act.element_size() == 4 && act.size(0) == n,
              "mlp_epoch_gather: act must be [n] int32 or [n, A] fp32");
  const int64_t aw = act.numel() / n;
  for (const Tensor* t : {&logp, &adv, &ret, &o_logp, &o_adv, &o_ret}) {
    need(*t, at::kFloat, "mlp_epoch_gather row value");
    TORCH_CHECK(t->numel() == n, "mlp_epoch_gather: per-row values must have n elements");
  }
  need(o_obs, at::kFloat, "o_obs");
  TORCH_CHECK(o_obs.numel() == n * D && o_act.is_contiguous() && o_act.numel() == n * aw &&
                  o_act.element_size() == 4, "mlp_epoch_gather: output shapes");
  need(uc, at::kLong, "uc");
  aca::EpochGatherArgs a{};
  a.n = (int)n;
  a.D = (int)D;
  a.aw = (int)aw;
  a.obs = ptr<float>(obs);
  a.ld_obs = obs.stride(0);
  a.act = reinterpret_cast<const uint32_t*>(act.data_ptr());
  a.logp = ptr<float>(logp);
  a.adv = ptr<float>(adv);
  a.ret = ptr<float>(ret);
  a.v = copt<float>(v, at::kFloat, "v");
  a.o_obs = ptr<float>(o_obs);
  a.o_act = reinterpret_cast<uint32_t*>(o_act.data_ptr());
  a.o_logp = ptr<float>(o_logp);
  a.o_adv = ptr<float>(o_adv);
  a.o_ret = ptr<float>(o_ret);
  a.o_v = const_cast<float*>(copt<float>(o_v, at::kFloat, "o_v"));
  TORCH_CHECK((a.v != nullptr) == (a.o_v != nullptr), "mlp_epoch_gather: v and o_v go together");
  if (a.v) TORCH_CHECK(v->numel() == n && o_v->numel() == n, "mlp_epoch_gather: v shapes");
  a.uc = uc.data_ptr<int64_t>();
  a.ep = (int)ep;
  a.seed = (uint32_t)seed;
  check(aca_mlp_epoch_gather(&a, cur_stream(obs)), "mlp_epoch_gather");
}

void mlp_rollout(Tensor desc, int64_t lds, Tensor obs, Tensor act, Tensor logp, Tensor ent, Tensor reward,
                 Tensor done, Tensor trunc, Tensor log_std, Tensor ac_scale, int64_t key_shift, int64_t policy_seed,
                 Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, Tensor env_ids, Tensor lin_A,
                 Tensor lin_B, int64_t env_seed, int64_t max_steps, int64_t k, bool wlds,
                 c10::optional<Tensor> stamps) {
  need(desc, at::kLong, "desc");
  TORCH_CHECK(desc.numel() * 8 >= (int64_t)sizeof(aca::MlpTower), "mlp_rollout: desc too small");
  need(obs, at::kFloat, "obs");
  check_env(state, t, tg, ep_ret, ep_stats, env_ids, reward, done, trunc);
  need(act, at::kFloat, "act");
  need(logp, at::kFloat, "logp");
  need(ent, at::kFloat, "ent");
  need(log_std, at::kFloat, "log_std");
  need(ac_scale, at::kFloat, "ac_scale");
  need(lin_A, at::kFloat, "lin_A");
  need(lin_B, at::kFloat, "lin_B");
  TORCH_CHECK(obs.dim() == 3, "mlp_rollout: obs must be [T+1, N, D]");
  const int64_t T = obs.size(0) - 1, N = obs.size(1), D = obs.size(2);
  TORCH_CHECK(T >= 1 && k >= 1 && D == 17 * k && state.numel() == N * 17, "mlp_rollout: bad obs / state shapes");
  TORCH_CHECK(act.numel() == T * N * 6 && logp.numel() == T * N && ent.numel() == T * N && reward.numel() == T * N &&
                  done.numel() == T * N && trunc.numel() == T * N,
              "mlp_rollout: rollout buffers must be [T, N] / [T, N, 6]");
  TORCH_CHECK(t.numel() == N && tg.numel() == N && ep_ret.numel() == N && env_ids.numel() == N &&
                  ep_stats.numel() >= 3, "mlp_rollout: env bank buffers must be [N]");
  TORCH_CHECK(log_std.numel() == 6 && ac_scale.numel() == 6 && lin_A.numel() == 17 * 17 && lin_B.numel() == 17 * 6,
              "mlp_rollout: bad head / dynamics shapes");
  aca::RolloutArgs a{};
  a.tw = reinterpret_cast<const aca::MlpTower*>(desc.data_ptr());
  a.N = (int)N;
  a.T = (int)T;
  a.D = (int)D;
  a.A = 6;
  a.head = 2;
  a.k = (int)k;
  a.log_std = ptr<float>(log_std);
  a.ac_scale = ptr<float>(ac_scale);
  a.key_shift = (int)key_shift;
  a.policy_seed = (uint32_t)policy_seed;
  a.obs = ptr<float>(obs);
  a.act = ptr<float>(act);
  a.logp = ptr<float>(logp);
  a.ent = ptr<float>(ent);
  a.reward = ptr<float>(reward);
  a.done = ptr<uint8_t>(done);
  a.trunc = ptr<uint8_t>(trunc);
  a.state = ptr<float>(state);
  a.t = ptr<int32_t>(t);
  a.tg = ptr<int64_t>(tg);
  a.ep_ret = ptr<float>(ep_ret);
  a.ep_stats = ptr<float>(ep_stats);
  a.env_ids = ptr<int64_t>(env_ids);
  a.lin_A = ptr<float>(lin_A);
  a.lin_B = ptr<float>(lin_B);
  a.env_seed = (uint32_t)env_seed;
  a.max_steps = (int)max_steps;
  a.wlds = wlds ? 1 : 0;
  a.stamps = reinterpret_cast<int64_t*>(stamps_ptr(stamps, 16));   // [16 steps][8 phases] + per-wave layer stamps + flag
  check(aca_mlp_rollout(&a, (size_t)lds, cur_stream(obs)), "mlp_rollout");
}

// words: CPU int64 [nseg, 13], fvals: CPU float [nseg, 4] (built once by ops/optim.py FusedGroupStep)
void opt_multi(Tensor words, Tensor fvals, c10::optional<Tensor> trans, bool adam, double b1, double b2, double eps,
               bool zero_grad, Tensor stream_ref, int64_t t_off) {
  TORCH_CHECK(!words.is_cuda() && words.scalar_type() == at::kLong && words.is_contiguous() && words.dim() == 2 &&
                  words.size(1) == 13, "opt_multi: words must be CPU int64 [nseg, 13]");
  TORCH_CHECK(!fvals.is_cuda() && fvals.scalar_type() == at::kFloat && fvals.is_contiguous() &&
                  fvals.numel() == words.size(0) * 4, "opt_multi: fvals must be CPU float [nseg, 4]");
  const int64_t* tp = nullptr;
  if (trans.has_value() && trans->defined()) {
    TORCH_CHECK(!trans->is_cuda() && trans->scalar_type() == at::kLong && trans->is_contiguous() &&
                    trans->numel() == words.size(0) * 8 * 5, "opt_multi: trans must be CPU int64 [nseg, 8, 5]");
    tp = ptr<int64_t>(*trans);
  }
  check(aca_opt_multi(ptr<int64_t>(words), ptr<float>(fvals), tp, (int)words.size(0), adam ? 1 : 0, (float)b1,
                      (float)b2, (float)eps, zero_grad ? 1 : 0, (int)t_off, cur_stream(stream_ref)),
        "opt_multi");
}

// In-place SUM all-reduce of a contiguous fp32 / bf16 / fp64 device tensor through an RCCL communicator (the one torch's
// ProcessGroupNCCL owns, passed as its address: ProcessGroupNCCL._comm_ptr()) ON THE CALLER'S STREAM. A torch
// collective runs on the process group's internal stream joined by two events to the compute stream; inside a captured
// update those cross-stream edges cost more than the all-reduce itself at the MLP engine's gradient sizes
// (profiles/r6_dp_world1.txt). Issued in program order on every rank, like the process group's own collectives.
void rccl_allreduce(Tensor buf, int64_t comm) {
  TORCH_CHECK(buf.is_cuda() && buf.is_contiguous(), "rccl_allreduce: contiguous device tensor");
  TORCH_CHECK(comm != 0, "rccl_allreduce: no communicator");
  ncclDataType_t dt;
  if (buf.scalar_type() == at::kFloat) dt = ncclFloat32;
  else if (buf.scalar_type() == at::kBFloat16) dt = ncclBfloat16;
  else if (buf.scalar_type() == at::kDouble) dt = ncclFloat64;
  else TORCH_CHECK(false, "rccl_allreduce: fp32, bf16 or fp64");
  const ncclResult_t r = ncclAllReduce(buf.data_ptr(), buf.data_ptr(), (size_t)buf.numel(), dt, ncclSum,
                                       reinterpret_cast<ncclComm_t>(comm), cur_stream(buf));
  TORCH_CHECK(r == ncclSuccess, "rccl_allreduce: ", ncclGetErrorString(r));
}

void grad_move(Tensor src, Tensor dst, c10::optional<Tensor> gate, bool zero) {
  need(src, at::kFloat, "src");
  need(dst, at::kFloat, "dst");
  TORCH_CHECK(src.numel() == dst.numel(), "grad_move: size mismatch");
  int* gp = const_cast<int*>(copt<int32_t>(gate, at::kInt, "gate"));
  check(aca_grad_move(ptr<float>(src), ptr<float>(dst), src.numel(), gp, zero ? 1 : 0, cur_stream(src)), "grad_move");
}

void cast_bf16(Tensor x, Tensor y) {
  need(x, at::kFloat, "x");
  need(y, at::kBFloat16, "y");
  TORCH_CHECK(x.numel() == y.numel(), "cast_bf16: size mismatch");
  check(aca_cast_bf16(ptr<float>(x), ptr<uint16_t>(y), x.numel(), cur_stream(x)), "cast_bf16");
}

// ---------------------------------------------------------------------------------------------- GEMM / conv
// A/B/C/mask are addressed through data_ptr (views with offsets are fine); the caller passes leading dimensions.
// Bounds are validated against the tensors' storage extents so a bad call fails here instead of faulting the GPU.
void check_extent(const Tensor& t, int64_t rows, int64_t cols, int64_t ld, const char* name) {
  TORCH_CHECK(t.is_cuda(), "gemm: ", name, " must be on the GPU");
  if (rows <= 0 || cols <= 0) return;
  const int64_t need_elems = (rows - 1) * ld + cols;
  const int64_t have = (int64_t)(t.storage().nbytes() / t.element_size()) - t.storage_offset();
  TORCH_CHECK(need_elems <= have, "gemm: ", name, " too small: needs ", need_elems, " elements, has ", have);
}

// gather spec: [mode, B, C, H, W, KH, KW, S] (mode 0 = plain operand); the gather source is the operand tensor
AcaConvGather make_gather(const Tensor& src, const std::vector<int64_t>& spec, double scale, const char* name) {
  AcaConvGather g{};
  g.mode = spec.empty() ? 0 : (int)spec[0];
  if (!g.mode) return g;
  TORCH_CHECK(spec.size() == 8, "gemm: gather spec for ", name, " must be [mode, B, C, H, W, KH, KW, S]");
  g.src = src.data_ptr();
  g.B = spec[1]; g.C = spec[2]; g.H = spec[3]; g.W = spec[4]; g.KH = spec[5]; g.KW = spec[6]; g.S = spec[7];
  g.OH = (g.H - g.KH) / g.S + 1;
  g.OW = (g.W - g.KW) / g.S + 1;
  g.scale = (float)scale;
  aca_gather_prepare(&g);
  TORCH_CHECK(src.is_contiguous(), "gemm: gather source ", name, " must be contiguous");
  if (g.mode == 3 || g.mode == 5) {
    TORCH_CHECK(g.OH > 0 && g.OW > 0, "gemm: gather mode 3/5 bad geometry");
    if (g.mode == 5)
      TORCH_CHECK(g.S > 0 && g.KH % g.S == 0 && g.KW % g.S == 0 && g.H % g.S == 0 && g.W % g.S == 0,
                  "gemm: sub-pixel gather needs KH, KW, H, W divisible by the stride");
    TORCH_CHECK(src.numel() >= (int64_t)g.B * g.OH * g.OW * g.C, "gemm: gather source ", name, " too small");
  } else if (g.mode == 4 || g.mode == 6) {
    TORCH_CHECK(src.numel() >= (int64_t)g.C * g.KH * g.KW * g.W, "gemm: gather source ", name, " too small");
  } else {
    TORCH_CHECK(src.numel() >= (int64_t)g.B * g.C * g.H * g.W, "gemm: gather source ", name, " too small");
  }
  if (g.mode == 1) {
    TORCH_CHECK(src.scalar_type() == at::kByte, "gemm: gather mode 1 needs a uint8 source");
    TORCH_CHECK(g.KW % 8 == 0 && g.S % 4 == 0 && g.W % 4 == 0, "gemm: gather mode 1 needs KW%8, S%4, W%4 == 0");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(g.src) % 4 == 0, "gemm: gather source must be 4-byte aligned");
  } else if (g.mode == 2) {
    TORCH_CHECK(src.scalar_type() == at::kBFloat16, "gemm: gather mode 2 needs a bf16 source");
    TORCH_CHECK(g.C % 8 == 0, "gemm: gather mode 2 needs C % 8 == 0");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(g.src) % 16 == 0, "gemm: gather source must be 16-byte aligned");
  } else if (g.mode >= 3 && g.mode <= 6) {
    TORCH_CHECK(src.scalar_type() == at::kBFloat16, "gemm: gather modes 3-6 need a bf16 source");
    TORCH_CHECK((g.mode == 3 || g.mode == 5 ? g.C : g.W) % 8 == 0,
                "gemm: gather modes 3-6 need 8-aligned contiguous channels");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(g.src) % 16 == 0, "gemm: gather source must be 16-byte aligned");
  } else {
    TORCH_CHECK(false, "gemm: unknown gather mode ", g.mode);
  }
  return g;
}

struct GemmGroupState {
  bool active = false, paused = false;
  std::vector<AcaGemmDesc> descs;
  hipStream_t stream = nullptr;
};
static thread_local GemmGroupState g_gemm_group;

// Large plain bf16 products on 128 x 128 tiles of the 32x32x16 MFMA with LDS-DMA staging (gemm_big.hip): epilogue
// alpha / bias / relu / mask, store fp32 (out_mode 0) or bf16 (1); splits > 1: slab split-K (ws >= gemm_big_ws
// floats, tickets >= tiles int32 zeros, self-cleaning), reduced in split order by the last-arriving split.
void gemm_big(Tensor A, int64_t lda, bool a_k, Tensor B, int64_t ldb, bool b_k, Tensor C, int64_t ldc,
              int64_t out_mode, int64_t M, int64_t N, int64_t K, double alpha, c10::optional<Tensor> bias, bool relu,
              c10::optional<Tensor> mask, int64_t ldm, int64_t splits, c10::optional<Tensor> ws,
              c10::optional<Tensor> tickets, c10::optional<Tensor> stamps, int64_t variant) {
  TORCH_CHECK(out_mode == 0 || out_mode == 1 || out_mode == 3, "gemm_big: out_mode 0 / 1 / 3 (partial planes)");
  TORCH_CHECK(variant >= 0 && variant < 16, "gemm_big: variant 0..15");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "gemm_big: bf16 operands");
  TORCH_CHECK(C.scalar_type() == (out_mode == 1 ? at::kBFloat16 : at::kFloat), "gemm_big: C dtype mismatch");
  check_extent(A, a_k ? M : K, a_k ? K : M, lda, "A");
  check_extent(B, b_k ? N : K, b_k ? K : N, ldb, "B");
  check_extent(C, M, N, ldc, "C");
  if (out_mode == 3) {
    TORCH_CHECK(C.is_contiguous() && C.numel() >= std::max<int64_t>(splits, 1) * M * ldc,
                "gemm_big: out_mode 3 needs splits planes of [M, ldc]");
    TORCH_CHECK(!(bias.has_value() && bias->defined()) && !relu && !(mask.has_value() && mask->defined()) &&
                    alpha == 1.0, "gemm_big: partial planes take no epilogue");
  }
  AcaGemmDesc d{};
  d.A = A.data_ptr();
  d.B = B.data_ptr();
  d.C = C.data_ptr();
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= N, "gemm_big: bias must be fp32 [N]");
    d.bias = ptr<float>(*bias);
  }
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->scalar_type() == at::kBFloat16, "gemm_big: mask must be bf16");
    check_extent(*mask, M, N, ldm, "mask");
    d.mask = mask->data_ptr();
  }
  if (splits > 1 && out_mode != 3) {
    TORCH_CHECK(ws.has_value() && ws->defined() && tickets.has_value() && tickets->defined(),
                "gemm_big: split-K needs ws and tickets");
    TORCH_CHECK(ws->scalar_type() == at::kFloat && ws->numel() >= aca_gemm_big_ws((int)M, (int)N, (int)splits),
                "gemm_big: ws too small");
    TORCH_CHECK(tickets->scalar_type() == at::kInt &&
                    tickets->numel() >= ((M + 127) / 128) * ((N + 127) / 128), "gemm_big: tickets too small");
    d.ws = ptr<float>(*ws);
    d.tickets = reinterpret_cast<unsigned int*>(tickets->data_ptr<int32_t>());
  }
  d.lda = lda; d.ldb = ldb; d.ldc = ldc; d.ldm = ldm;
  d.M = (int)M; d.N = (int)N; d.K = (int)K;
  d.a_k = a_k; d.b_k = b_k;
  d.out_mode = (int)out_mode;
  d.relu = relu;
  d.alpha = (float)alpha;
  d.splits = (int)splits;
  d.tile = (int)variant;
  if (stamps.has_value() && stamps->defined()) {
    const int64_t grid = ((M + 127) / 128) * ((N + 127) / 128) * std::max<int64_t>(splits, 1);
    TORCH_CHECK(stamps->scalar_type() == at::kLong && stamps->numel() >= grid * 8, "gemm_big: stamps [grid, 8] int64");
    d.stamps = reinterpret_cast<unsigned long long*>(stamps->data_ptr<int64_t>());
  }
  check(aca_gemm_big(&d, cur_stream(C)), "gemm_big");
}

int64_t gemm_big_ws(int64_t M, int64_t N, int64_t splits) { return aca_gemm_big_ws((int)M, (int)N, (int)splits); }

void gemm(Tensor A, int64_t lda, bool a_k, Tensor B, int64_t ldb, bool b_k, Tensor C, int64_t ldc, int64_t out_mode,
          int64_t M, int64_t N, int64_t K, double alpha, c10::optional<Tensor> bias, bool relu,
          c10::optional<Tensor> mask, int64_t ldm, c10::optional<Tensor> colsum, int64_t colsum_mod, int64_t tile,
          int64_t bk, int64_t splits, c10::optional<Tensor> ws, c10::optional<Tensor> tickets,
          std::vector<int64_t> ga, double ga_scale, std::vector<int64_t> gb, double gb_scale,
          c10::optional<Tensor> stamps, c10::optional<Tensor> colsum_part) {
  TORCH_CHECK(out_mode >= 0 && out_mode <= 3, "gemm: bad out_mode");
  if (out_mode == 3)
    TORCH_CHECK(!(bias.has_value() && bias->defined()) && !relu && !(mask.has_value() && mask->defined()) &&
                    !(colsum.has_value() && colsum->defined()),
                "gemm: out_mode 3 (partial planes) takes no bias / relu / mask / colsum");
  TORCH_CHECK(aca_gemm_supported((int)tile, (int)bk), "gemm: unsupported tile ", tile, " / bk ", bk);
  TORCH_CHECK(C.scalar_type() == (out_mode == 1 ? at::kBFloat16 : at::kFloat), "gemm: C dtype mismatch");
  AcaGemmDesc d{};
  d.ga = make_gather(A, ga, ga_scale, "A");
  d.gb = make_gather(B, gb, gb_scale, "B");
  TORCH_CHECK(d.ga.mode != 4 && d.gb.mode != 3 && d.ga.mode != 6 && d.gb.mode != 5,
              "gemm: gather modes 3/5 are A-only, 4/6 B-only");
  TORCH_CHECK((d.ga.mode == 3) == (d.gb.mode == 4), "gemm: gather modes 3 and 4 go together (data gradient)");
  TORCH_CHECK((d.ga.mode == 5) == (d.gb.mode == 6), "gemm: gather modes 5 and 6 go together (sub-pixel dgrad)");
  if (d.ga.mode == 5) {
    TORCH_CHECK(a_k, "gemm: A gather needs a_k");
    TORCH_CHECK(M == (int64_t)d.ga.B * d.ga.H * d.ga.W && K == (int64_t)d.ga.C * d.ga.KHS * d.ga.KWS,
                "gemm: sub-pixel gather shape does not match M/K");
    TORCH_CHECK(d.gb.S == d.ga.S && d.gb.KH == d.ga.KH && d.gb.KW == d.ga.KW && d.gb.C == d.ga.C,
                "gemm: sub-pixel A/B gather geometry mismatch");
    int bm, bn;
    aca_gemm_tile_dims((int)tile, &bm, &bn);
    TORCH_CHECK(((int64_t)d.ga.B * d.ga.HS * d.ga.WS) % bm == 0, "gemm: sub-pixel rows per phase must be a multiple "
                "of the tile height");
  } else if (d.ga.mode == 3) {
    TORCH_CHECK(a_k, "gemm: A gather needs a_k");
    TORCH_CHECK(M == (int64_t)d.ga.B * d.ga.H * d.ga.W && K == (int64_t)d.ga.C * d.ga.KH * d.ga.KW,
                "gemm: transposed-conv gather shape does not match M/K");
  } else if (d.ga.mode) {
    TORCH_CHECK(a_k, "gemm: A gather needs a_k");
    TORCH_CHECK(M == (int64_t)d.ga.B * d.ga.OH * d.ga.OW && K == (int64_t)d.ga.C * d.ga.KH * d.ga.KW,
                "gemm: A gather shape does not match M/K");
  } else {
    TORCH_CHECK(A.scalar_type() == at::kBFloat16, "gemm: A must be bf16");
    check_extent(A, a_k ? M : K, a_k ? K : M, lda, "A");
  }
  if (d.gb.mode == 6) {
    TORCH_CHECK(!b_k, "gemm: B gather needs !b_k");
    TORCH_CHECK(K == (int64_t)d.gb.C * d.gb.KHS * d.gb.KWS && N == d.gb.W, "gemm: phase weight gather shape");
  } else if (d.gb.mode == 4) {
    TORCH_CHECK(!b_k, "gemm: B gather needs !b_k");
    TORCH_CHECK(K == (int64_t)d.gb.C * d.gb.KH * d.gb.KW && N == d.gb.W, "gemm: weight-transpose gather shape");
  } else if (d.gb.mode) {
    TORCH_CHECK(!b_k, "gemm: B gather needs !b_k");
    TORCH_CHECK(K == (int64_t)d.gb.B * d.gb.OH * d.gb.OW && N == (int64_t)d.gb.C * d.gb.KH * d.gb.KW,
                "gemm: B gather shape does not match K/N");
  } else {
    TORCH_CHECK(B.scalar_type() == at::kBFloat16, "gemm: B must be bf16");
    check_extent(B, b_k ? N : K, b_k ? K : N, ldb, "B");
  }
  if (out_mode == 3) check_extent(C, aca_gemm_effective_splits((int)K, (int)bk, (int)splits) * M, N, ldc, "C");
  else check_extent(C, M, N, ldc, "C");
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= N, "gemm: bias must be fp32 [N]");
  }
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->scalar_type() == at::kBFloat16, "gemm: mask must be bf16");
    check_extent(*mask, M, N, ldm, "mask");
  }
  if (colsum.has_value() && colsum->defined()) {
    TORCH_CHECK(colsum->scalar_type() == at::kFloat && colsum->numel() >= (colsum_mod > 0 ? colsum_mod : N),
                "gemm: colsum too small");
  }
  const int eff = aca_gemm_effective_splits((int)K, (int)bk, (int)splits);
  if (eff > 1 && out_mode < 2) {
    TORCH_CHECK(ws.has_value() && ws->defined() && tickets.has_value() && tickets->defined(),
                "gemm: slab split-K needs ws and tickets");
    int bm, bn;
    aca_gemm_tile_dims((int)tile, &bm, &bn);
    const int64_t tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    TORCH_CHECK(ws->scalar_type() == at::kFloat && ws->numel() >= tiles * eff * bm * bn, "gemm: ws too small (need ",
                tiles * eff * bm * bn, ")");
    TORCH_CHECK(tickets->scalar_type() == at::kInt && tickets->numel() >= tiles, "gemm: tickets too small");
    d.ws = ptr<float>(*ws);
    d.tickets = ptr<unsigned int>(*tickets);
  }
  d.A = A.data_ptr(); d.B = B.data_ptr(); d.C = C.data_ptr();
  d.bias = optr<float>(bias);
  d.mask = (mask.has_value() && mask->defined()) ? mask->data_ptr() : nullptr;
  d.colsum = optr<float>(colsum);
  d.lda = lda; d.ldb = ldb; d.ldc = ldc; d.ldm = ldm;
  d.M = (int)M; d.N = (int)N; d.K = (int)K;
  d.a_k = a_k; d.b_k = b_k;
  d.out_mode = (int)out_mode; d.relu = relu ? 1 : 0; d.colsum_mod = (int)colsum_mod;
  d.alpha = (float)alpha;
  if (stamps.has_value() && stamps->defined()) {   // diagnostics: [tiles * splits, 4] int64 per workgroup
    int bm, bn;
    aca_gemm_tile_dims((int)tile, &bm, &bn);
    const int64_t wgs = ((M + bm - 1) / bm) * ((N + bn - 1) / bn) * aca_gemm_effective_splits((int)K, (int)bk, (int)splits);
    need(*stamps, at::kLong, "stamps");
    TORCH_CHECK(stamps->numel() >= wgs * 4, "gemm: stamps needs [workgroups, 4]");
    d.stamps = ptr<unsigned long long>(*stamps);
  }
  d.tile = (int)tile; d.bk = (int)bk; d.splits = (int)splits;
  if (colsum_part.has_value() && colsum_part->defined()) {
    TORCH_CHECK(d.colsum && eff == 1 && out_mode != 3, "gemm: colsum partials need colsum and no split-K");
    int bm, bn;
    aca_gemm_tile_dims((int)tile, &bm, &bn);
    need(*colsum_part, at::kFloat, "colsum_part");
    TORCH_CHECK(colsum_part->numel() >= ((M + bm - 1) / bm) * N, "gemm: colsum_part needs [M tiles, N]");
    d.colsum_part = ptr<float>(*colsum_part);
  }
  if (g_gemm_group.active) {   // grouped launch being collected: run at gemm_group_end
    TORCH_CHECK(g_gemm_group.descs.empty() || g_gemm_group.stream == cur_stream(C),
                "gemm group: every product must be issued on the same stream");
    g_gemm_group.stream = cur_stream(C);
    g_gemm_group.descs.push_back(d);
    return;
  }
  check(aca_gemm_run(&d, cur_stream(C)), "gemm");
}

// Grouped GEMM launches: between gemm_group_begin() and gemm_group_end() every gemm() call is collected instead of
// launched; the end runs them as ONE grouped kernel when an instantiation covers their tile configurations
// (csrc/kernels/gemm_group.hip), else one launch each, in issue order. Returns 1 if the grouped kernel ran.
void gemm_group_begin() {
  TORCH_CHECK(!g_gemm_group.active, "gemm group already open");
  g_gemm_group.active = true;
  g_gemm_group.descs.clear();
}

int64_t gemm_group_end() {
  TORCH_CHECK(g_gemm_group.active, "gemm group not open");
  g_gemm_group.active = false;
  if (g_gemm_group.descs.empty()) return 0;
  int grouped = 0;
  const hipError_t err = aca_gemm_group_run(g_gemm_group.descs.data(), (int)g_gemm_group.descs.size(),
                                            g_gemm_group.stream, &grouped);
  g_gemm_group.descs.clear();
  check(err, "gemm_group");
  return grouped;
}

void gemm_group_pause(bool paused) {   // autotuning inside an open group launches its trials directly
  if (paused && g_gemm_group.active) {
    g_gemm_group.active = false;
    g_gemm_group.paused = true;
  } else if (!paused && g_gemm_group.paused) {
    g_gemm_group.active = true;
    g_gemm_group.paused = false;
  }
}

int64_t gemm_effective_splits(int64_t K, int64_t bk, int64_t splits) {
  return aca_gemm_effective_splits((int)K, (int)bk, (int)splits);
}

// Fused Nature-CNN trunk (conv1..conv3 of one env per workgroup, csrc/kernels/cnn_fused.hip). Shapes are fixed by
// the kernel: obs [B, 4, 84, 84] uint8, W1 [32, 256] (OIHW), W2 [64, 512] / W3 [64, 576] (OHWI), y1 [B*400, 32],
// y2 [B*81, 64], y3 [B*49, 64]; all 16-byte aligned (the kernel uses 16-byte vector accesses).
// mode 0: one workgroup per env; mode 1: 7 row workgroups per env (cnn_trunk_rows_kernel). copy_out (mode 1 only):
// also copy the whole observation there (rollover of the last observation into slot 0 of the next rollout).
void cnn_trunk_fwd(Tensor obs, Tensor W1, Tensor b1, Tensor W2, Tensor b2, Tensor W3, Tensor b3, Tensor y1,
                   Tensor y2, Tensor y3, double scale, c10::optional<Tensor> shift_out,
                   c10::optional<Tensor> stamps, int64_t mode, c10::optional<Tensor> copy_out,
                   c10::optional<Tensor> obs_idx) {
  need(obs, at::kByte, "obs");
  for (auto* w : {&W1, &W2, &W3, &y1, &y2, &y3}) need(*w, at::kBFloat16, "trunk bf16 operand");
  for (auto* b : {&b1, &b2, &b3}) need(*b, at::kFloat, "trunk bias");
  TORCH_CHECK(obs.numel() % (4 * 84 * 84) == 0, "cnn_trunk_fwd: obs must be [B, 4, 84, 84]");
  int64_t B = obs.numel() / (4 * 84 * 84);
  const int64_t* idxp = nullptr;
  if (obs_idx.has_value() && obs_idx->defined()) {   // sample b = row obs_idx[b] of obs (per-env modes 3 / 5)
    need(*obs_idx, at::kLong, "obs_idx");
    TORCH_CHECK(mode == 3 || mode == 5, "cnn_trunk_fwd: obs_idx needs a per-env mode");
    B = obs_idx->numel();
    idxp = obs_idx->data_ptr<int64_t>();
  }
  TORCH_CHECK(W1.numel() == 32 * 256 && W2.numel() == 64 * 512 && W3.numel() == 64 * 576,
              "cnn_trunk_fwd: weights must be Nature-CNN conv1..3");
  TORCH_CHECK(b1.numel() == 32 && b2.numel() == 64 && b3.numel() == 64, "cnn_trunk_fwd: bias sizes");
  TORCH_CHECK(y1.numel() >= B * 400 * 32 && y2.numel() >= B * 81 * 64 && y3.numel() >= B * 49 * 64,
              "cnn_trunk_fwd: activation buffers too small");
  for (auto* t : {&obs, &W1, &W2, &W3, &y1, &y2, &y3})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "cnn_trunk_fwd: operands must be 16B aligned");
  uint8_t* so = nullptr;
  if (shift_out.has_value() && shift_out->defined()) {
    need(*shift_out, at::kByte, "shift_out");
    TORCH_CHECK(shift_out->numel() == obs.numel() && reinterpret_cast<uintptr_t>(shift_out->data_ptr()) % 16 == 0 &&
                    shift_out->data_ptr() != obs.data_ptr(),
                "cnn_trunk_fwd: shift_out must be a distinct, aligned [B, 4, 84, 84] uint8 buffer");
    so = ptr<uint8_t>(*shift_out);
  }
  uint8_t* co = nullptr;
  if (copy_out.has_value() && copy_out->defined()) {
    TORCH_CHECK(mode == 1 || mode == 2 || mode == 6 || mode == 7, "cnn_trunk_fwd: copy_out needs a row-split mode");
    need(*copy_out, at::kByte, "copy_out");
    TORCH_CHECK(copy_out->numel() == obs.numel() && reinterpret_cast<uintptr_t>(copy_out->data_ptr()) % 16 == 0 &&
                    copy_out->data_ptr() != obs.data_ptr(),
                "cnn_trunk_fwd: copy_out must be a distinct, aligned [B, 4, 84, 84] uint8 buffer");
    co = ptr<uint8_t>(*copy_out);
  }
  if (mode == 1 || mode == 2 || mode == 6 || mode == 7) {
    // 2: the row kernel with its conv2/conv3 weight loads issued after conv1; 6 / 7: modes 1 / 2 reading
    // fragment-ordered W2 / W3 copies (W1 row-major)
    check(aca_cnn_trunk_rows(ptr<uint8_t>(obs), ptr<uint16_t>(W1), ptr<float>(b1), ptr<uint16_t>(W2),
                             ptr<float>(b2), ptr<uint16_t>(W3), ptr<float>(b3), ptr<uint16_t>(y1), ptr<uint16_t>(y2),
                             ptr<uint16_t>(y3), (int)B, (float)scale, so, co, stamps_ptr(stamps, B * 7),
                             (mode == 2 || mode == 7) ? 1 : 0, mode >= 6 ? 1 : 0, cur_stream(obs)),
          "cnn_trunk_rows");
    return;
  }
  if (mode == 3 || mode == 5) {   // the per-env bf16-staged kernel (one byte conversion per pixel); mode 5: W1..W3
    // are the fragment-ordered copies (frag_weights)
    TORCH_CHECK(!stamps.has_value() || !stamps->defined(), "cnn_trunk_fwd: mode 3 has no phase stamps");
    check(aca_cnn_trunk_fwd_s16(ptr<uint8_t>(obs), ptr<uint16_t>(W1), ptr<float>(b1), ptr<uint16_t>(W2),
                                ptr<float>(b2), ptr<uint16_t>(W3), ptr<float>(b3), ptr<uint16_t>(y1),
                                ptr<uint16_t>(y2), ptr<uint16_t>(y3), (int)B, (float)scale, so, idxp,
                                mode == 5 ? 1 : 0, cur_stream(obs)),
          "cnn_trunk_fwd_s16");
    return;
  }
  TORCH_CHECK(false, "cnn_trunk_fwd: mode must be 1, 2, 3, 5, 6 or 7");
}

// Fused data-gradient chain dy3 -> dy2 -> dy1 of the Nature-CNN trunk, one workgroup per sample
// (cnn_fused.hip cnn_trunk_bwd_kernel), or ``persist`` > 0 workgroups walking the samples with the weight fragments
// held in registers (cnn_trunk_bwd_persist_kernel, bit-identical): dy3 [B*49, 64] (already masked by y3 > 0), W3 [64, 576] / W2 [64, 512]
// (OHWI bf16 shadows), masks y2 [B*81, 64] / y1 [B*400, 32]; writes dy2, dy1 (masked) and the per-sample bias
// gradient partials biasp [B, 160] = (sum dy3 | sum dy2 | sum dy1).
// bias_acc (persistent kernel only): biasp gets min(persist, B) rows, each the sum of its workgroup's samples' rows.
// w1_obs / w1_planes: the conv1 weight gradient folded in -- one [32][256] fp32 plane per sample (per-sample
// kernel) or per workgroup (persistent kernel), times w1_scale; frames of sample b = w1_obs row w1_obs_idx[b] (or b).
// skip_dy1 (persistent fold): dy1 is not stored (its only consumer is the folded weight gradient).
void cnn_trunk_bwd(Tensor dy3, Tensor W3, Tensor y2, Tensor W2, Tensor y1, Tensor dy2, Tensor dy1, Tensor biasp,
                   c10::optional<Tensor> stamps, int64_t persist, c10::optional<Tensor> w1_obs,
                   c10::optional<Tensor> w1_obs_idx, c10::optional<Tensor> w1_planes, double w1_scale,
                   bool bias_acc, bool skip_dy1) {
  for (auto* t : {&dy3, &W3, &y2, &W2, &y1, &dy2, &dy1}) need(*t, at::kBFloat16, "trunk_bwd bf16 operand");
  need(biasp, at::kFloat, "biasp");
  TORCH_CHECK(dy3.numel() % (49 * 64) == 0, "cnn_trunk_bwd: dy3 must be [B*49, 64]");
  const int64_t B = dy3.numel() / (49 * 64);
  TORCH_CHECK(W3.numel() == 64 * 576 && W2.numel() == 64 * 512, "cnn_trunk_bwd: weights must be conv3 / conv2");
  TORCH_CHECK(y2.numel() >= B * 81 * 64 && y1.numel() >= B * 400 * 32 && dy2.numel() >= B * 81 * 64 &&
                  dy1.numel() >= B * 400 * 32 && biasp.numel() >= B * 160,
              "cnn_trunk_bwd: buffers too small");
  TORCH_CHECK(!bias_acc || persist > 0, "cnn_trunk_bwd: bias_acc needs the persistent kernel");
  const uint8_t* wo = nullptr;
  const int64_t* wi = nullptr;
  float* wp = nullptr;
  if (w1_obs.has_value() && w1_obs->defined()) {
    need(*w1_obs, at::kByte, "w1_obs");
    TORCH_CHECK(w1_obs->is_contiguous() && w1_obs->numel() % (4 * 84 * 84) == 0, "cnn_trunk_bwd: w1_obs [*, 4, 84, 84]");
    TORCH_CHECK(w1_planes.has_value() && w1_planes->defined(), "cnn_trunk_bwd: w1_obs needs w1_planes");
    need(*w1_planes, at::kFloat, "w1_planes");
    const int64_t np = persist > 0 ? std::min<int64_t>(persist, B) : B;   // one plane per workgroup
    TORCH_CHECK(w1_planes->numel() >= np * 32 * 256, "cnn_trunk_bwd: w1_planes needs a [32][256] plane per workgroup");
    if (w1_obs_idx.has_value() && w1_obs_idx->defined()) {
      need(*w1_obs_idx, at::kLong, "w1_obs_idx");
      TORCH_CHECK(w1_obs_idx->numel() >= B, "cnn_trunk_bwd: w1_obs_idx needs B rows");
      wi = ptr<int64_t>(*w1_obs_idx);
    } else {
      TORCH_CHECK(w1_obs->numel() >= B * 4 * 84 * 84, "cnn_trunk_bwd: w1_obs needs B samples");
    }
    wo = ptr<uint8_t>(*w1_obs);
    wp = ptr<float>(*w1_planes);
  }
  TORCH_CHECK(!skip_dy1 || (wo && persist > 0), "cnn_trunk_bwd: skip_dy1 needs the persistent conv1 fold");
  check(aca_cnn_trunk_bwd(ptr<uint16_t>(dy3), ptr<uint16_t>(W3), ptr<uint16_t>(y2), ptr<uint16_t>(W2),
                          ptr<uint16_t>(y1), ptr<uint16_t>(dy2), skip_dy1 ? nullptr : ptr<uint16_t>(dy1),
                          ptr<float>(biasp), (int)B,
                          stamps_ptr(stamps, B), (int)persist, wo, wi, wp, (float)w1_scale, bias_acc ? 1 : 0,
                          cur_stream(dy3)),
        "cnn_trunk_bwd");
}

// Gradient finaliser (optim.hip grad_finalize_kernel): jobs = device int64 [njobs, 8] (dst, src, n, stride, S,
// vec, 0, 0) built by ops/optim.py finalize_jobs; writes dst = sum of S planes where src != 0 and the
// SUMSQ_PARTS sum-of-squares partials.
// Optional statistics duty (one extra workgroup): spart [N, 10] fp64 per-env A2C statistics rows (a2c_head_env)
// combined into stats[0..7] over B = T * N rows.
void grad_finalize(Tensor jobs, Tensor partial, c10::optional<Tensor> spart, int64_t B, c10::optional<Tensor> ent_coef,
                   c10::optional<Tensor> kl_coef, c10::optional<Tensor> stats) {
  need(jobs, at::kLong, "jobs");
  TORCH_CHECK(jobs.dim() == 2 && jobs.size(1) == 8 && jobs.is_contiguous(), "grad_finalize: jobs must be [njobs, 8]");
  need(partial, at::kFloat, "partial");
  TORCH_CHECK(partial.numel() >= aca_sumsq_parts() && jobs.size(0) <= aca_sumsq_parts(),
              "grad_finalize: partial too small / too many jobs");
  const double* sp = nullptr;
  int sN = 0, sppo = 0;
  if (spart.has_value() && spart->defined()) {
    need(*spart, at::kDouble, "spart");
    TORCH_CHECK(spart->dim() == 2 && (spart->size(1) == 10 || spart->size(1) == aca::PH_NSTAT) && B >= 1 &&
                    ent_coef.has_value() && kl_coef.has_value() && stats.has_value() && stats->numel() >= 8,
                "grad_finalize: statistics duty needs spart [N, 10] (a2c_head_env) or [N, 6] (ppo_head), B, "
                "ent_coef, kl_coef and stats[8]");
    need(*ent_coef, at::kFloat, "ent_coef");
    need(*kl_coef, at::kFloat, "kl_coef");
    need(*stats, at::kFloat, "stats");
    sp = spart->data_ptr<double>();
    sN = (int)spart->size(0);
    sppo = spart->size(1) == aca::PH_NSTAT ? 1 : 0;
  }
  check(aca_grad_finalize(jobs.data_ptr<int64_t>(), (int)jobs.size(0), ptr<float>(partial), sp, sN, (int)B,
                          optr<float>(ent_coef), optr<float>(kl_coef), optr<float>(stats), sppo, cur_stream(partial)),
        "grad_finalize");
}

// A2C learner head, one workgroup per env (loss.hip a2c_head_env_kernel; A2C without advantage normalisation): the
// bootstrap value V(s_T) from the rollout's last fc planes (written into val[T]), returns, loss, dz, dh, and per-env
// partial planes of dWh [N, 512 * A1], dbfc [N, 512], dbh [N, A1] + statistics rows spart [N, 10] (reduced by the
// gradient finaliser).
void a2c_head_env(Tensor z, Tensor act, Tensor logp_old, Tensor ent_coef, Tensor kl_coef, double vf_coef, Tensor rew,
                  Tensor val, Tensor dones, int64_t L, int64_t returns_mode, double gamma, double lam, Tensor ret_w,
                  Tensor adv_w, Tensor h, Tensor Wh, Tensor dh, c10::optional<Tensor> hpart, int64_t S,
                  c10::optional<Tensor> bfc, c10::optional<Tensor> bh, Tensor pWh, Tensor pbfc, Tensor pbh,
                  Tensor spart, c10::optional<Tensor> stamps) {
  TORCH_CHECK(rew.dim() == 2, "a2c_head_env: rewards must be [T, N]");
  const int T = rew.size(0), N = rew.size(1), B = T * N;
  TORCH_CHECK(z.dim() == 2 && z.size(0) >= B, "a2c_head_env: z must be [B, A + 1]");
  const int A = z.size(1) - 1, A1 = A + 1;
  need(z, at::kFloat, "z");
  need(act, at::kInt, "act");
  need(dones, at::kByte, "dones");
  for (auto* t : {&logp_old, &ent_coef, &kl_coef, &rew, &val, &ret_w, &adv_w, &pWh, &pbfc, &pbh})
    need(*t, at::kFloat, "a2c_head_env fp32 operand");
  need(spart, at::kDouble, "spart");
  for (auto* t : {&h, &Wh, &dh}) need(*t, at::kBFloat16, "a2c_head_env bf16 operand");
  TORCH_CHECK(z.is_contiguous() && z.stride(0) == A1, "a2c_head_env: z must be contiguous [B, A + 1]");
  TORCH_CHECK(act.numel() >= B && logp_old.numel() >= B && val.numel() >= (int64_t)(T + 1) * N &&
                  dones.numel() >= B && ret_w.numel() >= B && adv_w.numel() >= B && h.numel() >= (int64_t)B * 512 &&
                  dh.numel() >= (int64_t)B * 512 && Wh.numel() == 512 * A1,
              "a2c_head_env: shape mismatch");
  TORCH_CHECK(pWh.numel() >= (int64_t)N * 512 * A1 && pbfc.numel() >= (int64_t)N * 512 && pbh.numel() >= (int64_t)N * A1 &&
                  spart.numel() >= (int64_t)N * 10,
              "a2c_head_env: partial planes too small");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(pbfc.data_ptr()) % 8 == 0, "a2c_head_env: pbfc must be 8-byte aligned");
  const float* hp = nullptr;
  int64_t pstride = 0;
  if (hpart.has_value() && hpart->defined()) {
    need(*hpart, at::kFloat, "hpart");
    TORCH_CHECK(bfc.has_value() && bh.has_value(), "a2c_head_env: hpart needs bfc and bh");
    need(*bfc, at::kFloat, "bfc");
    need(*bh, at::kFloat, "bh");
    pstride = hpart->numel() / 32;
    TORCH_CHECK(hpart->numel() % 32 == 0 && pstride >= (int64_t)N * 512 && S >= 1 && S <= 32,
                "a2c_head_env: hpart must hold 32 planes of [N, 512]");
    TORCH_CHECK(bfc->numel() == 512 && bh->numel() == A1, "a2c_head_env: bad bootstrap operands");
    hp = ptr<float>(*hpart);
  }
  check(aca_a2c_head_env(ptr<float>(z), ptr<int32_t>(act), ptr<float>(logp_old), ptr<float>(ent_coef),
                         ptr<float>(kl_coef), (float)vf_coef, ptr<float>(rew), ptr<float>(val), ptr<uint8_t>(dones), T,
                         N, (int)L, (int)returns_mode, (float)gamma, (float)lam, ptr<float>(ret_w), ptr<float>(adv_w),
                         ptr<uint16_t>(h), ptr<uint16_t>(Wh), ptr<uint16_t>(dh), A, hp, (int)S, pstride,
                         optr<float>(bfc), optr<float>(bh), ptr<float>(pWh), ptr<float>(pbfc), ptr<float>(pbh),
                         spart.data_ptr<double>(), stamps_ptr(stamps, N), cur_stream(z)),
        "a2c_head_env");
}

// A2C learner head in one launch (loss.hip head_bwd_kernel): returns + EV + advantage normalisation + loss + dz,
// then dh = (h > 0) * dz Wh^T, dbfc, dWh, dbh written straight into their gradient slots (deterministic).
void head_bwd(Tensor z, Tensor act, Tensor logp_old, Tensor ent_coef, Tensor kl_coef, double vf_coef, Tensor rew,
              Tensor val, Tensor dones, int64_t L, int64_t returns_mode, bool norm_adv, double gamma, double lam,
              Tensor ret_w, Tensor adv_w, Tensor h, Tensor Wh, Tensor dh, Tensor gWh, Tensor gbh, Tensor gbfc,
              Tensor stats, c10::optional<Tensor> stamps) {
  TORCH_CHECK(rew.dim() == 2, "head_bwd: rewards must be [T, N]");
  const int T = rew.size(0), N = rew.size(1), B = T * N;
  TORCH_CHECK(z.dim() == 2 && z.size(0) >= B, "head_bwd: z must be [B, A + 1]");
  const int A = z.size(1) - 1;
  need(z, at::kFloat, "z");
  need(act, at::kInt, "act");
  for (auto* t : {&logp_old, &ent_coef, &kl_coef, &rew, &val, &ret_w, &adv_w, &gWh, &gbh, &gbfc, &stats})
    need(*t, at::kFloat, "head_bwd fp32 operand");
  need(dones, at::kByte, "dones");
  for (auto* t : {&h, &Wh, &dh}) need(*t, at::kBFloat16, "head_bwd bf16 operand");
  TORCH_CHECK(z.is_contiguous() && z.stride(0) == A + 1, "head_bwd: z must be contiguous [B, A + 1]");
  TORCH_CHECK(act.numel() >= B && logp_old.numel() >= B && val.numel() == (int64_t)(T + 1) * N &&
                  dones.numel() == B && ret_w.numel() >= B && adv_w.numel() >= B && h.numel() >= (int64_t)B * 512 &&
                  dh.numel() >= (int64_t)B * 512 && Wh.numel() == 512 * (A + 1) && gWh.numel() == 512 * (A + 1) &&
                  gbh.numel() == A + 1 && gbfc.numel() == 512 && stats.numel() >= 8,
              "head_bwd: shape mismatch");
  check(aca_head_bwd(ptr<float>(z), ptr<int32_t>(act), ptr<float>(logp_old), ptr<float>(ent_coef),
                     ptr<float>(kl_coef), (float)vf_coef, ptr<float>(rew), ptr<float>(val), ptr<uint8_t>(dones), T, N,
                     (int)L, (int)returns_mode, norm_adv ? 1 : 0, (float)gamma, (float)lam, ptr<float>(ret_w),
                     ptr<float>(adv_w), ptr<uint16_t>(h), ptr<uint16_t>(Wh), ptr<uint16_t>(dh), ptr<float>(gWh),
                     ptr<float>(gbh), ptr<float>(gbfc), ptr<float>(stats), A, stamps_ptr(stamps, 8), cur_stream(z)),
        "head_bwd");
}

// A2C learner head v2 (loss.hip a2c_head_kernel): the bootstrap value V(s_T) from the rollout's last fc partial planes
// (written into val[T]) + everything head_bwd does, in one launch of 32 narrow workgroups meeting at a bounded grid
// barrier (bar: int32[3] zeros; bar[2] != 0 after a launch = the barrier timed out). hpart = None: val[T] is given.
void a2c_head(Tensor z, Tensor act, Tensor logp_old, Tensor ent_coef, Tensor kl_coef, double vf_coef, Tensor rew,
              Tensor val, Tensor dones, int64_t L, int64_t returns_mode, bool norm_adv, double gamma, double lam,
              Tensor ret_w, Tensor adv_w, Tensor h, Tensor Wh, Tensor dh, Tensor gWh, Tensor gbh, Tensor gbfc,
              Tensor stats, c10::optional<Tensor> hpart, int64_t planes, c10::optional<Tensor> bfc,
              c10::optional<Tensor> bh, c10::optional<Tensor> bar, c10::optional<Tensor> stamps) {
  TORCH_CHECK(rew.dim() == 2, "a2c_head: rewards must be [T, N]");
  const int T = rew.size(0), N = rew.size(1), B = T * N;
  TORCH_CHECK(z.dim() == 2 && z.size(0) >= B, "a2c_head: z must be [B, A + 1]");
  const int A = z.size(1) - 1;
  need(z, at::kFloat, "z");
  need(act, at::kInt, "act");
  for (auto* t : {&logp_old, &ent_coef, &kl_coef, &rew, &val, &ret_w, &adv_w, &gWh, &gbh, &gbfc, &stats})
    need(*t, at::kFloat, "a2c_head fp32 operand");
  need(dones, at::kByte, "dones");
  for (auto* t : {&h, &Wh, &dh}) need(*t, at::kBFloat16, "a2c_head bf16 operand");
  TORCH_CHECK(z.is_contiguous() && z.stride(0) == A + 1, "a2c_head: z must be contiguous [B, A + 1]");
  TORCH_CHECK(act.numel() >= B && logp_old.numel() >= B && val.numel() == (int64_t)(T + 1) * N &&
                  dones.numel() == B && ret_w.numel() >= B && adv_w.numel() >= B && h.numel() >= (int64_t)B * 512 &&
                  dh.numel() >= (int64_t)B * 512 && Wh.numel() == 512 * (A + 1) && gWh.numel() == 512 * (A + 1) &&
                  gbh.numel() == A + 1 && gbfc.numel() == 512 && stats.numel() >= 8,
              "a2c_head: shape mismatch");
  const float* hp = nullptr;
  int64_t pstride = 0;
  unsigned int* barp = nullptr;
  if (hpart.has_value() && hpart->defined()) {
    need(*hpart, at::kFloat, "hpart");
    TORCH_CHECK(bfc.has_value() && bh.has_value() && bar.has_value(), "a2c_head: hpart needs bfc, bh and bar");
    need(*bfc, at::kFloat, "bfc");
    need(*bh, at::kFloat, "bh");
    need(*bar, at::kInt, "bar");
    pstride = hpart->numel() / 32;
    TORCH_CHECK(hpart->numel() % 32 == 0 && pstride >= (int64_t)N * 512 && planes >= 1 && planes <= 32,
                "a2c_head: hpart must hold 32 planes of [N, 512]");
    TORCH_CHECK(bfc->numel() == 512 && bh->numel() == A + 1 && bar->numel() >= 3, "a2c_head: bad bootstrap operands");
    hp = ptr<float>(*hpart);
    barp = reinterpret_cast<unsigned int*>(bar->data_ptr<int32_t>());
  }
  check(aca_a2c_head(ptr<float>(z), ptr<int32_t>(act), ptr<float>(logp_old), ptr<float>(ent_coef),
                     ptr<float>(kl_coef), (float)vf_coef, ptr<float>(rew), ptr<float>(val), ptr<uint8_t>(dones), T, N,
                     (int)L, (int)returns_mode, norm_adv ? 1 : 0, (float)gamma, (float)lam, ptr<float>(ret_w),
                     ptr<float>(adv_w), ptr<uint16_t>(h), ptr<uint16_t>(Wh), ptr<uint16_t>(dh), ptr<float>(gWh),
                     ptr<float>(gbh), ptr<float>(gbfc), ptr<float>(stats), A, hp, (int)planes, pstride,
                     hp ? ptr<float>(*bfc) : nullptr, hp ? ptr<float>(*bh) : nullptr, barp, stamps_ptr(stamps, 32),
                     cur_stream(z)),
        "a2c_head");
}

void im2col_u8(Tensor x, Tensor col, int64_t kh, int64_t kw, int64_t s, double scale) {
  need(x, at::kByte, "x");
  need(col, at::kBFloat16, "col");
  TORCH_CHECK(x.dim() == 4, "im2col_u8: x must be [B, C, H, W]");
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int OH = (H - kh) / s + 1, OW = (W - kw) / s + 1;
  TORCH_CHECK(col.numel() == (int64_t)B * OH * OW * C * kh * kw, "im2col_u8: col size mismatch");
  check(aca_im2col_u8_nchw(ptr<uint8_t>(x), ptr<uint16_t>(col), B, C, H, W, kh, kw, s, (float)scale, cur_stream(x)),
        "im2col_u8");
}

void im2col_nhwc(Tensor x, Tensor col, int64_t B, int64_t H, int64_t W, int64_t C, int64_t kh, int64_t kw,
                 int64_t s) {
  need(x, at::kBFloat16, "x");
  need(col, at::kBFloat16, "col");
  const int OH = (H - kh) / s + 1, OW = (W - kw) / s + 1;
  TORCH_CHECK(x.numel() >= B * H * W * C, "im2col_nhwc: x too small");
  TORCH_CHECK(col.numel() >= (int64_t)B * OH * OW * C * kh * kw, "im2col_nhwc: col too small");
  check(aca_im2col_nhwc(ptr<uint16_t>(x), ptr<uint16_t>(col), B, C, H, W, kh, kw, s, cur_stream(x)), "im2col_nhwc");
}

void col2im_nhwc(Tensor dcol, Tensor ymask, Tensor dx, c10::optional<Tensor> colsum, int64_t B, int64_t H, int64_t W,
                 int64_t C, int64_t kh, int64_t kw, int64_t s) {
  need(dcol, at::kBFloat16, "dcol");
  need(ymask, at::kBFloat16, "ymask");
  need(dx, at::kBFloat16, "dx");
  const int OH = (H - kh) / s + 1, OW = (W - kw) / s + 1;
  TORCH_CHECK(dcol.numel() >= (int64_t)B * OH * OW * C * kh * kw, "col2im: dcol too small");
  TORCH_CHECK(ymask.numel() >= B * H * W * C && dx.numel() >= B * H * W * C, "col2im: dx/ymask too small");
  if (colsum.has_value() && colsum->defined())
    TORCH_CHECK(colsum->scalar_type() == at::kFloat && colsum->numel() >= C, "col2im: colsum must be fp32 [C]");
  check(aca_col2im_nhwc(ptr<uint16_t>(dcol), ptr<uint16_t>(ymask), ptr<uint16_t>(dx), optr<float>(colsum), B, C, H, W,
                        kh, kw, s, cur_stream(dcol)),
        "col2im_nhwc");
}

void seg_stats(Tensor x, Tensor segs, Tensor out) {
  need(x, at::kFloat, "x");
  need(segs, at::kLong, "segs");
  need(out, at::kFloat, "out");
  const int64_t nv = segs.numel() / 2;
  TORCH_CHECK(out.numel() >= 4 * nv, "seg_stats: out needs [nvars, 4]");
  check(aca_seg_stats(ptr<float>(x), ptr<int64_t>(segs), (int)nv, ptr<float>(out), cur_stream(x)), "seg_stats");
}

void colsum_reduce(Tensor part, int64_t R, int64_t N, Tensor out, int64_t mod) {
  need(part, at::kFloat, "part");
  need(out, at::kFloat, "out");
  TORCH_CHECK(part.numel() >= R * N && out.numel() >= (mod > 0 ? mod : N), "colsum_reduce: size mismatch");
  check(aca_colsum_reduce(ptr<float>(part), (int)R, (int)N, ptr<float>(out), (int)mod, cur_stream(part)),
        "colsum_reduce");
}

void colsum_bf16(Tensor x, int64_t M, int64_t N, int64_t ld, Tensor out) {
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "colsum: x must be bf16");
  check_extent(x, M, N, ld, "x");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= N, "colsum: out must be fp32 [N]");
  check(aca_colsum_bf16(ptr<uint16_t>(x), M, N, ld, ptr<float>(out), cur_stream(x)), "colsum_bf16");
}

// ---------------------------------------------------------------------------------------------- loss
void ac_loss(Tensor logits, int64_t ldl, c10::optional<Tensor> value, int64_t ldv, c10::optional<Tensor> act_i,
             c10::optional<Tensor> act_f, c10::optional<Tensor> log_std, Tensor logp_old, c10::optional<Tensor> adv,
             c10::optional<Tensor> ret, c10::optional<Tensor> v_old, c10::optional<Tensor> ent_coef,
             c10::optional<Tensor> kl_coef, double vf_coef, double ppo_clip, double v_clip, Tensor dlogits,
             int64_t lddl, c10::optional<Tensor> dvalue, int64_t lddv, c10::optional<Tensor> dlog_std, Tensor stats,
             int64_t B, int64_t A, bool gaussian, int64_t returns_mode, c10::optional<Tensor> rew,
             c10::optional<Tensor> val, c10::optional<Tensor> dones, int64_t L, double gamma, double lam,
             bool norm_adv, c10::optional<Tensor> ret_w, c10::optional<Tensor> adv_w, c10::optional<Tensor> dbias) {
  TORCH_CHECK(logits.scalar_type() == at::kFloat && dlogits.scalar_type() == at::kBFloat16, "ac_loss: dtypes");
  check_extent(logits, B, A, ldl, "logits");
  check_extent(dlogits, B, A, lddl, "dlogits");
  need(logp_old, at::kFloat, "logp_old");
  need(stats, at::kFloat, "stats");
  TORCH_CHECK(logp_old.numel() >= B && stats.numel() >= 8, "ac_loss: sizes");
  int T = 0, N = 0;
  if (returns_mode) {
    TORCH_CHECK(rew.has_value() && val.has_value() && dones.has_value() && ret_w.has_value() && adv_w.has_value(),
                "ac_loss: fused returns need rew, val, dones, ret_w, adv_w");
    need(*rew, at::kFloat, "rew");
    need(*val, at::kFloat, "val");
    need(*dones, at::kByte, "dones");
    need(*ret_w, at::kFloat, "ret_w");
    need(*adv_w, at::kFloat, "adv_w");
    TORCH_CHECK(rew->dim() == 2, "ac_loss: rewards must be [T, N]");
    T = rew->size(0);
    N = rew->size(1);
    TORCH_CHECK((int64_t)T * N == B && val->numel() == (int64_t)(T + 1) * N && dones->numel() == B &&
                    ret_w->numel() >= B && adv_w->numel() >= B,
                "ac_loss: fused returns shape mismatch");
  } else {
    TORCH_CHECK(adv.has_value() && ret.has_value(), "ac_loss: adv and ret needed");
    need(*adv, at::kFloat, "adv");
    need(*ret, at::kFloat, "ret");
    TORCH_CHECK(adv->numel() >= B && ret->numel() >= B, "ac_loss: sizes");
  }
  if (gaussian) {
    TORCH_CHECK(act_f.has_value() && log_std.has_value(), "ac_loss: gaussian needs act_f and log_std");
  } else {
    TORCH_CHECK(act_i.has_value(), "ac_loss: categorical needs act_i");
  }
  if (value.has_value() && value->defined()) {
    TORCH_CHECK(dvalue.has_value() && dvalue->defined(), "ac_loss: value needs dvalue");
    check_extent(*value, B, 1, ldv, "value");
    check_extent(*dvalue, B, 1, lddv, "dvalue");
  }
  int dbn = 0;
  if (dbias.has_value() && dbias->defined()) {
    TORCH_CHECK(dbias->scalar_type() == at::kFloat && dbias->numel() >= A + 1, "ac_loss: dbias must be fp32 [A+1]");
    dbn = A + 1;
  }
  check(aca_ac_loss(ptr<float>(logits), ldl, optr<float>(value), ldv, optr<int32_t>(act_i), optr<float>(act_f),
                    optr<float>(log_std), ptr<float>(logp_old), optr<float>(adv), optr<float>(ret), optr<float>(v_old),
                    optr<float>(ent_coef), optr<float>(kl_coef), (float)vf_coef, (float)ppo_clip, (float)v_clip,
                    ptr<uint16_t>(dlogits), lddl, optr<uint16_t>(dvalue), lddv, optr<float>(dlog_std),
                    ptr<float>(stats), (int)B, (int)A, gaussian ? 1 : 0, (int)returns_mode, optr<float>(rew),
                    optr<float>(val), optr<uint8_t>(dones), T, N, (int)L, (float)gamma, (float)lam, norm_adv ? 1 : 0,
                    optr<float>(ret_w), optr<float>(adv_w), optr<float>(dbias), dbn, cur_stream(logits)),
        "ac_loss");
}

int64_t ping() { return 355; }

}  // namespace

TORCH_LIBRARY(acamd, m) {
  m.def("ping() -> int", &ping);
  m.def("env_step_cartpole(Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, Tensor env_ids, "
        "Tensor actions, Tensor prev, Tensor out, Tensor reward, Tensor done, Tensor truncated, int seed, "
        "int max_steps, int k, Tensor? final_out=None) -> ()");
  m.def("env_step_pendulum(Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, Tensor env_ids, "
        "Tensor actions, Tensor prev, Tensor out, Tensor reward, Tensor done, Tensor truncated, int seed, "
        "int max_steps, int k, Tensor? final_out=None) -> ()");
  m.def("env_step_linear(Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, Tensor env_ids, "
        "Tensor actions, Tensor A, Tensor B, Tensor prev, Tensor out, Tensor reward, Tensor done, Tensor truncated, "
        "int seed, int max_steps, int k, Tensor? final_out=None) -> ()");
  m.def("env_step_pong(Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, Tensor env_ids, "
        "Tensor actions, Tensor prev, Tensor out, Tensor reward, Tensor done, Tensor truncated, int seed, "
        "int max_steps, int k) -> ()");
  m.def("env_policy_step_pong(Tensor h, Tensor Wh, Tensor bh, Tensor z, Tensor act, Tensor logp, Tensor ent, "
        "Tensor value, int key_shift, int pseed, Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, "
        "Tensor env_ids, Tensor prev, Tensor out, Tensor reward, Tensor done, Tensor truncated, int seed, "
        "int max_steps, int k, bool pre_shifted=False, Tensor? hpart=None, int planes=0, Tensor? bfc=None, "
        "Tensor? stamps=None) -> ()");
  m.def("fc_value(Tensor hpart, int planes, Tensor bfc, Tensor Wh, Tensor bh, Tensor out, Tensor? h_out) -> ()");
  m.def("pong_fused_step(Tensor h, Tensor Wh, Tensor bh, Tensor z, Tensor act, Tensor logp, Tensor ent, "
        "Tensor value, int key_shift, int pseed, Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor state_n, "
        "Tensor t_n, Tensor tg_n, Tensor ep_ret_n, Tensor ep_stats, Tensor env_ids, Tensor prev, Tensor out, "
        "Tensor reward, Tensor done, Tensor truncated, int seed, int max_steps, Tensor hpart, int planes, "
        "Tensor bfc, Tensor W1, Tensor b1, Tensor W2, Tensor b2, Tensor W3, Tensor b3, Tensor y1, Tensor y2, "
        "Tensor y3, float scale, Tensor? shift_out=None, Tensor? stamps=None, bool frag=False) -> ()");
  m.def("pong_fused_env_step(Tensor h, Tensor Wh, Tensor bh, Tensor z, Tensor act, Tensor logp, Tensor ent, "
        "Tensor value, int key_shift, int pseed, Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, "
        "Tensor env_ids, Tensor out, Tensor reward, Tensor done, Tensor truncated, int seed, int max_steps, "
        "Tensor hpart, int planes, Tensor bfc, Tensor W1, Tensor b1, Tensor W2, Tensor b2, Tensor W3, Tensor b3, "
        "Tensor y1, Tensor y2, Tensor y3, float scale, Tensor? shift_out=None, Tensor[]? next_state=None, "
        "Tensor? stamps=None, bool frag=False) -> ()");
  m.def("categorical_sample(Tensor logits, Tensor keys, int seed, Tensor act, Tensor logp, Tensor ent) -> ()");
  m.def("wave_reduce_check(Tensor x, Tensor out) -> ()");
  m.def("categorical_sample_env(Tensor logits, Tensor tg, Tensor env_ids, int key_shift, int seed, Tensor act, "
        "Tensor logp, Tensor ent, Tensor? vout) -> ()");
  m.def("ev(Tensor x, Tensor y, Tensor out, Tensor? part=None, Tensor? ticket=None) -> ()");
  m.def("ev_blocks(int n) -> int", &ev_blocks);
  m.def("returns_scan_geometry(int T, int N) -> int[]", &returns_scan_geometry);
  m.def("returns_scan(Tensor r, Tensor v, Tensor d, Tensor ret, Tensor adv, int mode, float gamma, float lam, int L, "
        "bool norm, float eps, Tensor part, Tensor ticket, Tensor mom, Tensor? ev_out=None, Tensor? gz=None) -> ()");
  m.def("normalize_mom(Tensor a, Tensor out, Tensor mom, float eps) -> ()");
  m.def("gemm_group_begin() -> ()", &gemm_group_begin);
  m.def("gemm_group_end() -> int", &gemm_group_end);
  m.def("gemm_group_pause(bool paused) -> ()", &gemm_group_pause);
  m.def("conv1_wgrad(Tensor obs, Tensor dy1, Tensor planes, int P, float scale, Tensor? obs_idx=None) -> ()");
  m.def("conv_wgrad_gemm(int layer, Tensor img, Tensor dy, Tensor planes, int P) -> ()");
  m.def("mb_gather(Tensor obs, Tensor act, Tensor logp, Tensor adv, Tensor ret, Tensor v, Tensor? o_obs, "
        "Tensor o_act, Tensor o_logp, Tensor o_adv, Tensor o_ret, Tensor o_v, int seed, Tensor uc, int ep, "
        "int off, Tensor? mom=None, float eps=1e-8, Tensor? bump_ticket=None, Tensor? o_idx=None) -> ()");
  m.def("gaussian_sample(Tensor mu, Tensor log_std, Tensor keys, int seed, Tensor act, Tensor logp, Tensor ent) -> ()");
  m.def("gae(Tensor r, Tensor v, Tensor d, Tensor ret, Tensor adv, float gamma, float lam) -> ()");
  m.def("nstep_returns(Tensor r, Tensor v, Tensor d, Tensor tgt, Tensor adv, float gamma, int L) -> ()");
  m.def("normalize(Tensor a, Tensor out, float eps) -> ()");
  m.def("moments(Tensor x, Tensor y, Tensor out) -> ()");
  m.def("sumsq(Tensor x, Tensor partial) -> ()");
  m.def("sumsq_multi(Tensor[] xs, Tensor[] partials) -> ()");
  m.def("adam_step(Tensor p, Tensor g, Tensor m, Tensor v, Tensor lr, Tensor t, Tensor? gnorm_parts, "
        "Tensor? gnorm_out, Tensor? shadow, float b1, float b2, float eps, float clip, float max_norm, Tensor ticket, "
        "bool zero_grad=False, float gmul=1.0, float norm_mul=1.0, Tensor? trans=None, Tensor? g16=None) -> ()");
  m.def("rmsprop_step(Tensor p, Tensor g, Tensor v, Tensor lr, Tensor? gnorm_parts, Tensor? gnorm_out, "
        "Tensor? shadow, float alpha, float eps, float clip, float max_norm, bool zero_grad=False, float gmul=1.0, "
        "float norm_mul=1.0, Tensor? trans=None, Tensor? g16=None) -> ()");
  m.def("cast_bf16(Tensor x, Tensor y) -> ()");
  m.def("grad_move(Tensor src, Tensor dst, Tensor? gate=None, bool zero=True) -> ()");
  m.def("rccl_allreduce(Tensor buf, int comm) -> ()");
  m.def("opt_multi(Tensor words, Tensor fvals, Tensor? trans, bool adam, float b1, float b2, float eps, bool zero_grad, "
        "Tensor stream_ref, int t_off=-1) -> ()");
  m.def("prp_perm(Tensor out, int seed, Tensor uc, int epoch) -> ()");
  m.def("mlp_tshadow(Tensor desc, int ntw, int total) -> ()");
  m.def("mlp_fwd(Tensor desc, int tw_base, int ntw, int mode, int lds, Tensor obs, Tensor? idx, Tensor? perm_uc, "
        "int perm_ep, int perm_off, int perm_n, int perm_seed, int B, int head, "
        "int A, Tensor? log_std, Tensor? ac_scale, Tensor? tg, Tensor? env_ids, int key_shift, int seed, "
        "Tensor? act_out, Tensor? logp_out, Tensor? ent_out, Tensor? v_out, Tensor? act_in, Tensor? logp_old, "
        "Tensor? adv, Tensor? ret, Tensor? v_old, Tensor? ent_coef, Tensor? kl_coef, float vf_coef, float ppo_clip, "
        "float v_clip, bool ppo, Tensor? g_log_std, Tensor? mstats, Tensor? mpart=None, Tensor? stamps=None, Tensor? hdesc=None) -> ()");
  m.def("mlp_wgrad(Tensor items, int nrt, int nsplit, Tensor? g_log_std, int A, Tensor? ls_part, float ls_clip, "
        "Tensor? stats, Tensor ent_coef, Tensor kl_coef, Tensor mpart, int mpart_rows, Tensor? bump) -> ()");
  m.def("mlp_epoch_gather(Tensor obs, Tensor act, Tensor logp, Tensor adv, Tensor ret, Tensor? v, Tensor o_obs, "
        "Tensor o_act, Tensor o_logp, Tensor o_adv, Tensor o_ret, Tensor? o_v, Tensor uc, int ep, int seed) -> ()");
  m.def("mlp_rollout(Tensor desc, int lds, Tensor obs, Tensor act, Tensor logp, Tensor ent, Tensor reward, "
        "Tensor done, Tensor truncated, Tensor log_std, Tensor ac_scale, int key_shift, int policy_seed, "
        "Tensor state, Tensor t, Tensor tg, Tensor ep_ret, Tensor ep_stats, Tensor env_ids, Tensor lin_A, "
        "Tensor lin_B, int env_seed, int max_steps, int k, bool wlds, Tensor? stamps=None) -> ()");
  m.def("gemm(Tensor A, int lda, bool a_k, Tensor B, int ldb, bool b_k, Tensor C, int ldc, int out_mode, int M, "
        "int N, int K, float alpha, Tensor? bias, bool relu, Tensor? mask, int ldm, Tensor? colsum, int colsum_mod, "
        "int tile, int bk, int splits, Tensor? ws, Tensor? tickets, int[] ga, float ga_scale, int[] gb, "
        "float gb_scale, Tensor? stamps=None, Tensor? colsum_part=None) -> ()");
  m.def("colsum_reduce(Tensor part, int R, int N, Tensor out, int mod) -> ()");
  m.def("gemm_big(Tensor A, int lda, bool a_k, Tensor B, int ldb, bool b_k, Tensor C, int ldc, int out_mode, int M, "
        "int N, int K, float alpha, Tensor? bias, bool relu, Tensor? mask, int ldm, int splits, Tensor? ws=None, "
        "Tensor? tickets=None, Tensor? stamps=None, int variant=0) -> ()");
  m.def("gemm_big_ws(int M, int N, int splits) -> int", &gemm_big_ws);
  m.def("seg_stats(Tensor x, Tensor segs, Tensor out) -> ()");
  m.def("gemm_effective_splits(int K, int bk, int splits) -> int", &gemm_effective_splits);
  m.def("cnn_trunk_fwd(Tensor obs, Tensor W1, Tensor b1, Tensor W2, Tensor b2, Tensor W3, Tensor b3, Tensor y1, "
        "Tensor y2, Tensor y3, float scale, Tensor? shift_out=None, Tensor? stamps=None, int mode=3, "
        "Tensor? copy_out=None, Tensor? obs_idx=None) -> ()");
  m.def("cnn_trunk_bwd(Tensor dy3, Tensor W3, Tensor y2, Tensor W2, Tensor y1, Tensor dy2, Tensor dy1, "
        "Tensor biasp, Tensor? stamps=None, int persist=0, Tensor? w1_obs=None, Tensor? w1_obs_idx=None, "
        "Tensor? w1_planes=None, float w1_scale=1.0, bool bias_acc=False, bool skip_dy1=False) -> ()");
  m.def("grad_finalize(Tensor jobs, Tensor partial, Tensor? spart=None, int B=0, Tensor? ent_coef=None, "
        "Tensor? kl_coef=None, Tensor? stats=None) -> ()");
  m.def("a2c_head_env(Tensor z, Tensor act, Tensor logp_old, Tensor ent_coef, Tensor kl_coef, float vf_coef, "
        "Tensor rew, Tensor val, Tensor dones, int L, int returns_mode, float gamma, float lam, Tensor ret_w, "
        "Tensor adv_w, Tensor h, Tensor Wh, Tensor dh, Tensor? hpart, int S, Tensor? bfc, Tensor? bh, Tensor pWh, "
        "Tensor pbfc, Tensor pbh, Tensor spart, Tensor? stamps=None) -> ()");
  m.def("ppo_head(Tensor h, Tensor Wh, Tensor bh, Tensor act, Tensor logp_old, Tensor adv, Tensor ret, Tensor? v_old, "
        "Tensor ent_coef, Tensor kl_coef, float vf_coef, float ppo_clip, float v_clip, Tensor dh, Tensor? z_out, "
        "Tensor pWh, Tensor pbh, Tensor pbfc, Tensor pstats, Tensor? ticket, Tensor stats, Tensor? hp=None, "
        "int hp_planes=0, Tensor? hbias=None) -> ()");
  m.def("ppo_head_planes(int B) -> int", &ppo_head_planes);
  m.def("opt_set_unroll(int u) -> int", &opt_set_unroll);
  m.def("opt_set_stamps(Tensor? buf) -> ()", &opt_set_stamps);
  m.def("fc_rollout(Tensor X, Tensor Wf, Tensor hpart, int variant, Tensor? stamps=None) -> int");
  m.def("fc_bwd(Tensor dh, Tensor W, Tensor y3, Tensor dy3, Tensor dW, Tensor? stamps=None, Tensor? sq=None) -> ()");
  m.def("head_bwd(Tensor z, Tensor act, Tensor logp_old, Tensor ent_coef, Tensor kl_coef, float vf_coef, Tensor rew, "
        "Tensor val, Tensor dones, int L, int returns_mode, bool norm_adv, float gamma, float lam, Tensor ret_w, "
        "Tensor adv_w, Tensor h, Tensor Wh, Tensor dh, Tensor gWh, Tensor gbh, Tensor gbfc, Tensor stats, "
        "Tensor? stamps=None) -> ()");
  m.def("a2c_head(Tensor z, Tensor act, Tensor logp_old, Tensor ent_coef, Tensor kl_coef, float vf_coef, Tensor rew, "
        "Tensor val, Tensor dones, int L, int returns_mode, bool norm_adv, float gamma, float lam, Tensor ret_w, "
        "Tensor adv_w, Tensor h, Tensor Wh, Tensor dh, Tensor gWh, Tensor gbh, Tensor gbfc, Tensor stats, "
        "Tensor? hpart, int planes, Tensor? bfc, Tensor? bh, Tensor? bar, Tensor? stamps=None) -> ()");
  m.def("im2col_u8(Tensor x, Tensor col, int kh, int kw, int s, float scale) -> ()");
  m.def("im2col_nhwc(Tensor x, Tensor col, int B, int H, int W, int C, int kh, int kw, int s) -> ()");
  m.def("col2im_nhwc(Tensor dcol, Tensor ymask, Tensor dx, Tensor? colsum, int B, int H, int W, int C, int kh, "
        "int kw, int s) -> ()");
  m.def("colsum_bf16(Tensor x, int M, int N, int ld, Tensor out) -> ()");
  m.def("ac_loss(Tensor logits, int ldl, Tensor? value, int ldv, Tensor? act_i, Tensor? act_f, Tensor? log_std, "
        "Tensor logp_old, Tensor? adv, Tensor? ret, Tensor? v_old, Tensor? ent_coef, Tensor? kl_coef, float vf_coef, "
        "float ppo_clip, float v_clip, Tensor dlogits, int lddl, Tensor? dvalue, int lddv, Tensor? dlog_std, "
        "Tensor stats, int B, int A, bool gaussian, int returns_mode=0, Tensor? rew=None, Tensor? val=None, "
        "Tensor? dones=None, int L=0, float gamma=0.99, float lam=0.95, bool norm_adv=False, Tensor? ret_w=None, "
        "Tensor? adv_w=None, Tensor? dbias=None) -> ()");
}

TORCH_LIBRARY_IMPL(acamd, CUDA, m) {
  m.impl("env_step_cartpole", &env_step_cartpole);
  m.impl("env_step_pendulum", &env_step_pendulum);
  m.impl("env_step_linear", &env_step_linear);
  m.impl("env_step_pong", &env_step_pong);
  m.impl("env_policy_step_pong", &env_policy_step_pong);
  m.impl("pong_fused_step", &pong_fused_step);
  m.impl("categorical_sample", &categorical_sample);
  m.impl("gaussian_sample", &gaussian_sample);
  m.impl("categorical_sample_env", &categorical_sample_env);
  m.impl("ev", &ev);
  m.impl("gae", &gae);
  m.impl("nstep_returns", &nstep_returns);
  m.impl("normalize", &normalize);
  m.impl("returns_scan", &returns_scan);
  m.impl("normalize_mom", &normalize_mom);
  m.impl("mb_gather", &mb_gather);
  m.impl("conv1_wgrad", &conv1_wgrad);
  m.impl("conv_wgrad_gemm", &conv_wgrad_gemm);
  m.impl("moments", &moments);
  m.impl("sumsq", &sumsq);
  m.impl("sumsq_multi", &sumsq_multi);
  m.impl("adam_step", &adam_step);
  m.impl("rmsprop_step", &rmsprop_step);
  m.impl("cast_bf16", &cast_bf16);
  m.impl("grad_move", &grad_move);
  m.impl("rccl_allreduce", &rccl_allreduce);
  m.impl("opt_multi", &opt_multi);
  m.impl("mlp_fwd", &mlp_fwd);
  m.impl("prp_perm", &prp_perm);
  m.impl("mlp_tshadow", &mlp_tshadow);
  m.impl("mlp_wgrad", &mlp_wgrad);
  m.impl("mlp_rollout", &mlp_rollout);
  m.impl("mlp_epoch_gather", &mlp_epoch_gather);
  m.impl("gemm", &gemm);
  m.impl("cnn_trunk_fwd", &cnn_trunk_fwd);
  m.impl("fc_value", &fc_value);
  m.impl("fc_rollout", &fc_rollout);
  m.impl("fc_bwd", &fc_bwd);
  m.impl("cnn_trunk_bwd", &cnn_trunk_bwd);
  m.impl("grad_finalize", &grad_finalize);
  m.impl("a2c_head_env", &a2c_head_env);
  m.impl("ppo_head", &ppo_head);
  m.impl("gemm_big", &gemm_big);
  m.impl("pong_fused_env_step", &pong_fused_env_step);
  m.impl("wave_reduce_check", &wave_reduce_check);
  m.impl("head_bwd", &head_bwd);
  m.impl("a2c_head", &a2c_head);
  m.impl("im2col_u8", &im2col_u8);
  m.impl("im2col_nhwc", &im2col_nhwc);
  m.impl("col2im_nhwc", &col2im_nhwc);
  m.impl("colsum_bf16", &colsum_bf16);
  m.impl("colsum_reduce", &colsum_reduce);
  m.impl("seg_stats", &seg_stats);
  m.impl("ac_loss", &ac_loss);
}
