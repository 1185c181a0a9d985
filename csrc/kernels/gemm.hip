// Host-side entry of the MFMA GEMM (kernel: gemm_impl.h; instantiations: gemm_plain.hip, gemm_conv.hip).
#include "gemm_impl.h"

namespace aca {
hipError_t gemm_plain(const GemmParams& P, hipStream_t s);
hipError_t gemm_conv(const GemmParams& P, hipStream_t s);
}  // namespace aca

using namespace aca;

extern "C" int aca_gemm_tile_dims(int tile, int* bm, int* bn) {
  switch (tile) {
    case 1: *bm = 32; *bn = 64; break;
    case 2: *bm = 64; *bn = 32; break;
    case 3: *bm = 128; *bn = 64; break;
    case 4: *bm = 32; *bn = 32; break;
    case 5: *bm = 64; *bn = 256; break;
    case 6: *bm = 32; *bn = 256; break;
    case 7: *bm = 128; *bn = 128; break;
    default: *bm = 64; *bn = 64; break;
  }
  return 0;
}

extern "C" int aca_gemm_supported(int tile, int bk) {
  if (bk == 64) return tile >= 0 && tile <= 7;
  if (bk == 128) return tile == 0 || tile == 1 || tile == 2 || tile == 4;
  if (bk == 256) return tile == 4;
  return 0;
}

// effective split count actually launched (every split gets >= 1 k-step)
extern "C" int aca_gemm_effective_splits(int K, int bk, int splits) {
  const int kt = (K + bk - 1) / bk;
  if (splits < 1) splits = 1;
  if (splits > kt) splits = kt > 0 ? kt : 1;
  const int per = (kt + splits - 1) / splits;
  return kt > 0 ? (kt + per - 1) / per : 1;
}

extern "C" hipError_t aca_gemm_run(const AcaGemmDesc* d, hipStream_t stream) {
  if (d->M <= 0 || d->N <= 0) return hipSuccess;
  if (!aca_gemm_supported(d->tile, d->bk)) return hipErrorInvalidValue;
  GemmParams P;
  P.d = *d;
  const int kt = (d->K + d->bk - 1) / d->bk;
  P.splits = aca_gemm_effective_splits(d->K, d->bk, d->splits);
  P.k_tiles_per_split = kt > 0 ? (kt + P.splits - 1) / P.splits : 0;
  if (P.splits > 1 && d->out_mode < 2 && (d->ws == nullptr || d->tickets == nullptr)) return hipErrorInvalidValue;
  if (d->out_mode == 3 && (d->bias || d->relu || d->mask || d->colsum)) return hipErrorInvalidValue;
  if (d->ga.mode || d->gb.mode) return gemm_conv(P, stream);
  return gemm_plain(P, stream);
}
