// Argument block of the large-batch learner head launch (ppo_head.hip), shared with csrc/bindings.cpp.
#pragma once
#include <stdint.h>

namespace aca {

constexpr int PH_THREADS = 256;
constexpr int PH_ROWS_PER_WAVE = 4;
constexpr int PH_ROWS = PH_ROWS_PER_WAVE * PH_THREADS / 64;   // 16 rows per workgroup
constexpr int PH_H = 512;
constexpr int PH_NSTAT = 6;   // pg, kl, entropy, value loss, clip count, ratio

struct PpoHeadArgs {
  const uint16_t* h;            // [B, 512] bf16 (unless hp)
  const float* hp;              // optional: fc split-K partial planes [hp_planes][B, 512] fp32; h = bf16(relu(sum + hbias))
  const float* hbias;           // [512] fc bias (with hp)
  int64_t hp_stride;            // floats between planes
  int hp_planes;                // 1..4
  const uint16_t* Wh;           // [512, A1] bf16 (k-major, TF [in, out] layout)
  const float* bh;         // [A1]
  const int32_t* act;      // [B]
  const float* logp_old;   // [B]
  const float* adv;        // [B] (already normalised)
  const float* ret;        // [B]
  const float* v_old;      // [B] or null (value clipping only)
  const float* ent_coef;   // device scalar
  const float* kl_coef;    // device scalar
  float vf_coef, ppo_clip, v_clip;
  uint16_t* dh;                 // [B, 512] bf16
  float* z_out;            // optional [B, A1] fp32
  float* pWh;              // [P][512 * A1] per-workgroup partial planes
  float* pbh;              // [P][A1]
  float* pbfc;             // [P][512]
  double* pstats;          // [P][PH_NSTAT]
  unsigned int* ticket;    // zero between launches (self-cleaning)
  float* stats;            // [7] pg, kl, entropy, value loss, clip fraction, actor loss, mean ratio
  int B;
};

}  // namespace aca
