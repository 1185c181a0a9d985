// Grouped launches of independent MFMA GEMMs (gemm_impl.h gemm_group_kernel): the learner's independent products
// (fc weight gradient || fc data gradient; the three conv weight gradients) in ONE launch each instead of products
// on two streams joined by events -- inside a captured hipGraph every cross-stream edge costs several microseconds
// of inter-queue synchronisation, more than the products themselves on the critical path. Instantiated for the
// tile configurations the autotuner picks for those products (up to two configurations per launch); any other
// combination falls back to one launch per product (aca_gemm_group_run).
#include "gemm_impl.h"

extern "C" int aca_gemm_tile_dims(int tile, int* bm, int* bn);
extern "C" hipError_t aca_gemm_run(const AcaGemmDesc* d, hipStream_t stream);
extern "C" int aca_gemm_effective_splits(int K, int bk, int splits);

namespace aca {

constexpr int cfg_key(int bm, int bn, int bk, bool ak, bool bkk, int ag, int bg, bool vec) {
  return ((((((bm / 32) * 8 + bn / 32) * 8 + bk / 64) * 2 + (ak ? 1 : 0)) * 2 + (bkk ? 1 : 0)) * 8 + ag) * 16 +
         bg * 2 + (vec ? 1 : 0);
}

template <int BM, int BN, int BK, bool A_K, bool B_K, int AG, int BG, bool VEC>
struct KCfg : GemmCfg<BM, BN, BK, A_K, B_K, AG, BG, VEC> {
  static constexpr int key = cfg_key(BM, BN, BK, A_K, B_K, AG, BG, VEC);
};

// fc weight gradient (A = y3 [B, 3136] k-major, B = dh) || fc data gradient (dh x Wfc^T)
using FcW32 = KCfg<32, 32, 64, false, false, 0, 0, true>;
using FcW64x32 = KCfg<64, 32, 64, false, false, 0, 0, true>;
using FcW64 = KCfg<64, 64, 64, false, false, 0, 0, true>;
using FcW32k128 = KCfg<32, 32, 128, false, false, 0, 0, true>;
using FcD32 = KCfg<32, 32, 64, true, true, 0, 0, true>;
using FcD64 = KCfg<64, 64, 64, true, true, 0, 0, true>;
using FcD32x64 = KCfg<32, 64, 64, true, true, 0, 0, true>;
using FcD32x64k128 = KCfg<32, 64, 128, true, true, 0, 0, true>;
using FcD32k128 = KCfg<32, 32, 128, true, true, 0, 0, true>;
using FcD64x32 = KCfg<64, 32, 64, true, true, 0, 0, true>;
// conv weight gradients: B gathered from the bf16 NHWC activations (conv2 / conv3) or the uint8 frames (conv1)
using Wg64x32 = KCfg<64, 32, 64, false, false, 0, 2, true>;
using Wg32x64k128 = KCfg<32, 64, 128, false, false, 0, 2, true>;
using Wg64 = KCfg<64, 64, 64, false, false, 0, 2, true>;
using Wg64x32k128 = KCfg<64, 32, 128, false, false, 0, 2, true>;
using Wu32k256 = KCfg<32, 32, 256, false, false, 0, 1, true>;
using Wu32k128 = KCfg<32, 32, 128, false, false, 0, 1, true>;

struct GroupEntry {
  int ka, kb;
  hipError_t (*fn)(GemmGroupArgs&, hipStream_t);
};

template <class A, class B>
constexpr GroupEntry entry() { return GroupEntry{A::key, B::key, &gemm_group_launch<A, B>}; }

#define FC_ROW(W)                                                                                           \
  entry<W, FcD32>(), entry<W, FcD64>(), entry<W, FcD32x64>(), entry<W, FcD32x64k128>(), entry<W, FcD32k128>(), \
      entry<W, FcD64x32>()

static const GroupEntry kGroups[] = {
    FC_ROW(FcW32), FC_ROW(FcW64x32), FC_ROW(FcW64), FC_ROW(FcW32k128),
    entry<Wg64x32, Wu32k256>(), entry<Wg64x32, Wu32k128>(), entry<Wg32x64k128, Wu32k256>(),
    entry<Wg32x64k128, Wu32k128>(), entry<Wg64, Wu32k256>(), entry<Wg64, Wu32k128>(),
    entry<Wg64x32k128, Wu32k256>(), entry<Wg64x32k128, Wu32k128>(),
};

static int desc_key(const AcaGemmDesc& d) {
  int bm, bn;
  aca_gemm_tile_dims(d.tile, &bm, &bn);
  bool vec = true;
  if (!d.ga.mode && !d.gb.mode)
    vec = gemm_operand_vec(d.A, d.lda, d.a_k ? d.K : d.M) && gemm_operand_vec(d.B, d.ldb, d.b_k ? d.K : d.N);
  return cfg_key(bm, bn, d.bk, d.a_k, d.b_k, d.ga.mode, d.gb.mode, vec);
}

}  // namespace aca

using namespace aca;

// Runs n independent products (descriptors as for aca_gemm_run) as one grouped launch when an instantiation covers
// their tile configurations, else one launch each. *grouped = 1 if the grouped kernel ran.
extern "C" hipError_t aca_gemm_group_run(const AcaGemmDesc* ds, int n, hipStream_t stream, int* grouped) {
  *grouped = 0;
  if (n < 1) return hipSuccess;
  bool ok = n <= GEMM_GROUP_MAX;
  int keys[GEMM_GROUP_MAX] = {0, 0, 0};
  for (int k = 0; ok && k < n; ++k) {
    const AcaGemmDesc& d = ds[k];
    if (d.M <= 0 || d.N <= 0 || d.colsum_part || d.stamps || d.ga.mode >= 3 || d.gb.mode >= 3) ok = false;
    else keys[k] = desc_key(d);
  }
  const GroupEntry* e = nullptr;
  if (ok && n > 1) {
    for (const GroupEntry& g : kGroups) {
      bool all = true;
      for (int k = 0; k < n; ++k) all = all && (keys[k] == g.ka || keys[k] == g.kb);
      if (all) { e = &g; break; }
    }
  }
  if (!e) {
    for (int k = 0; k < n; ++k) {
      const hipError_t err = aca_gemm_run(&ds[k], stream);
      if (err != hipSuccess) return err;
    }
    return hipSuccess;
  }
  GemmGroupArgs G{};
  G.n = n;
  for (int k = 0; k < n; ++k) {
    const AcaGemmDesc& d = ds[k];
    GemmParams& P = G.p[k];
    P.d = d;
    const int kt = (d.K + d.bk - 1) / d.bk;
    P.splits = aca_gemm_effective_splits(d.K, d.bk, d.splits);
    P.k_tiles_per_split = kt > 0 ? (kt + P.splits - 1) / P.splits : 0;
    if (P.splits > 1 && d.out_mode < 2 && (d.ws == nullptr || d.tickets == nullptr)) return hipErrorInvalidValue;
    G.cfg[k] = keys[k] == e->ka ? 0 : 1;
  }
  *grouped = 1;
  return e->fn(G, stream);
}
