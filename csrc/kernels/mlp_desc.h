// Descriptors shared by the MLP engine kernels (mlp.hip) and the torch-op bindings (bindings.cpp): plain C types
// only, so both hipcc and g++ compile this header.
#pragma once
#include <stdint.h>

namespace aca {

constexpr int MLP_MAXL = 5;
constexpr int MPART_W = 24;   // per-workgroup partial row of the train kernel: 8 loss statistics + 16 log-std grads

// Tower descriptor, device-resident (built once per engine and batch size by ops/mlp.py, every field 64-bit so the
// host packs it as an int64 tensor). Read with uniform (scalar) loads; a by-value kernel argument indexed by a
// runtime layer number would be spilled to scratch instead.
struct MlpTower {
  int64_t nl, pad;
  int64_t in[MLP_MAXL], out[MLP_MAXL], act[MLP_MAXL];
  int64_t W[MLP_MAXL];        // const float* [in][out]
  int64_t b[MLP_MAXL];
  int64_t gW[MLP_MAXL];
  int64_t gb[MLP_MAXL];
  int64_t xs[MLP_MAXL];       // train workspace: layer inputs [B][in], 16 x 16 blocks (mlp.hip blk_out)
  int64_t dp[MLP_MAXL];       // train workspace: dL/d(pre-activation) [B][out], 16 x 16 blocks
  int64_t F[MLP_MAXL];        // forward operand: fp32 FRAGMENT copy of W (common.h mlp_frag_f), zero pad
  int64_t G[MLP_MAXL];        // data-gradient operand: fp32 fragment copy of W (mlp_frag_g; layers >= 1), zero pad
};

struct MlpArgs {
  const MlpTower* tw;         // [2] device: 0 = actor (policy head), 1 = critic (value)
  int tw_base;
  int B, D;
  const float* obs; int64_t ld_obs;
  const int64_t* idx;         // optional row gather (explicit index list)
  const int64_t* perm_uc;     // optional row gather: rows prp(perm_off + r) of a keyed permutation of [0, perm_n)
  int perm_ep, perm_off, perm_n;   // (PPO minibatch: key = minibatch_key(perm_seed, *perm_uc, perm_ep))
  uint32_t perm_seed;
  int mode;                   // 0 rollout, 1 evaluate, 2 train
  int head;                   // tower 0's head: 1 categorical, 2 gaussian
  int A;
  const float* log_std;
  const float* ac_scale;
  const int64_t* tg; const int64_t* env_ids; int key_shift; uint32_t seed;
  int32_t* act_i_out; float* act_f_out; float* logp_out; float* ent_out; float* v_out;
  const int32_t* act_i_in; const float* act_f_in;
  const float* logp_old; const float* adv; const float* ret; const float* v_old;
  const float* ent_coef; const float* kl_coef;
  float vf_coef, ppo_clip, v_clip;
  int ppo;
  float* g_log_std;
  float* mstats;              // [8] sums (atomics): pg, kl, ent, vloss, clipfrac, -, ratio
  float* mpart;               // optional [ceil(B/16)][MPART_W]: per-workgroup partials instead of the atomics above
  float inv_B;
  int64_t* stamps;            // optional diagnostics: [2 towers][16] s_memrealtime at phase ends of workgroup (0, tower)
  // train launches of the reference towers (mlp.hip SPEC path): a by-value copy of both tower descriptors, so the
  // weight-fragment pointers are kernel-argument (scalar) reads at entry, before any other memory round trip
  MlpTower htw[2];
};

struct WgradArgs {
  const int64_t* items;       // device item table (mlp.hip mlp_wgrad_kernel; ops/mlp.py MLPEngine.wgrad_items)
  int nitems;
  int nrt;                    // 16-row tiles of the batch
  int nsplit;                 // > 1: the row tiles are split over workgroups, results added atomically (no sumsq)
  float* g_log_std; int A;    // the log-std gradient (summed from the train kernel's partial rows)
  float* ls_part; float ls_clip;   // its sum of squares slot (tower 0's slot after its tiles; null: none)
  float* stats; const float* ent_coef; const float* kl_coef;
  const float* mpart; int mpart_rows;   // the train kernel's partial rows (reduced here in a fixed order)
  int64_t* bump;              // optional counter advanced once (PPO update counter after the update's last minibatch)
};

// PPO epoch gather (mlp_epoch_gather_kernel): row i of the outputs = row prp(i) of the inputs
struct EpochGatherArgs {
  int n, D, aw;               // rows, observation width, action words per row (A floats or 1 int32)
  const float* obs; int64_t ld_obs;
  const uint32_t* act; const float* logp; const float* adv; const float* ret; const float* v;   // v optional
  float* o_obs; uint32_t* o_act; float* o_logp; float* o_adv; float* o_ret; float* o_v;
  const int64_t* uc; int ep; uint32_t seed;
};

// Fused rollout of the MuJoCo-shaped linear bank (mlp_rollout_kernel): T steps of actor + Gaussian sample + env step.
struct RolloutArgs {
  const MlpTower* tw;         // tower 0 (actor) of the engine descriptor
  int N, T, D, A, head, k;
  const float* log_std; const float* ac_scale;
  int key_shift; uint32_t policy_seed;
  float* obs;                 // [T+1][N][D]: block 0 read, blocks 1..T written
  float* act; float* logp; float* ent;        // [T][N][A], [T][N], [T][N]
  float* reward; uint8_t* done; uint8_t* trunc;   // [T][N]
  float* state; int32_t* t; int64_t* tg; float* ep_ret; float* ep_stats; const int64_t* env_ids;
  const float* lin_A; const float* lin_B;
  uint32_t env_seed; int max_steps;
  int wlds;                   // actor weights staged in LDS (host decides from the LDS budget)
  int64_t* stamps;            // optional diagnostics: s_memrealtime per phase of the first 16 steps (workgroup 0)
};

}  // namespace aca
