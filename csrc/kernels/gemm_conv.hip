// Instantiations of the MFMA GEMM with implicit-im2col operand gathers (convolution forward: A gathered from the
// input image; weight gradient: B gathered from the input image; data gradient: A gathered from the output gradient
// as a transposed conv, B = the OHWI weight read transposed).
#include "gemm_impl.h"

extern "C" int aca_gemm_tile_dims(int tile, int* bm, int* bn);

namespace aca {
hipError_t gemm_conv(const GemmParams& P, hipStream_t s) {
  // the non-gathered operand of a conv product must be vector-loadable (weights / output gradients always are)
  const AcaGemmDesc& d = P.d;
  const int ag = d.ga.mode, bg = d.gb.mode;
  if (!ag && !gemm_operand_vec(d.A, d.lda, d.a_k ? d.K : d.M)) return hipErrorInvalidValue;
  if (!bg && !gemm_operand_vec(d.B, d.ldb, d.b_k ? d.K : d.N)) return hipErrorInvalidValue;
  if (ag == 1 && !bg && d.a_k && d.b_k) return gemm_dispatch_tiles<true, true, 1, 0, true>(P, s);
  if (ag == 2 && !bg && d.a_k && d.b_k) return gemm_dispatch_tiles<true, true, 2, 0, true>(P, s);
  if (!ag && bg == 1 && !d.a_k && !d.b_k) return gemm_dispatch_tiles<false, false, 0, 1, true>(P, s);
  if (!ag && bg == 2 && !d.a_k && !d.b_k) return gemm_dispatch_tiles<false, false, 0, 2, true>(P, s);
  if (ag == 3 && bg == 4 && d.a_k && !d.b_k) return gemm_dispatch_tiles<true, false, 3, 4, true>(P, s);
  if (ag == 5 && bg == 6 && d.a_k && !d.b_k) {
    int bm, bn;
    aca_gemm_tile_dims(d.tile, &bm, &bn);
    if ((d.ga.B * d.ga.HS * d.ga.WS) % bm) return hipErrorInvalidValue;   // tiles must not straddle phases
    return gemm_dispatch_tiles<true, false, 5, 6, true>(P, s);
  }
  return hipErrorInvalidValue;
}
}  // namespace aca
