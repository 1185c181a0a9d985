// Instantiations of the MFMA GEMM with implicit-im2col operand gathers (convolution forward: A gathered from the
// input image; weight gradient: B gathered from the input image; data gradient: A gathered from the output gradient
// as a transposed conv, B = the OHWI weight read transposed).
#include "gemm_impl.h"

namespace aca {
hipError_t gemm_conv(const GemmParams& P, hipStream_t s) {
  const int ag = P.d.ga.mode, bg = P.d.gb.mode;
  if (ag == 1 && !bg && P.d.a_k && P.d.b_k) return gemm_dispatch_tiles<true, true, 1, 0>(P, s);
  if (ag == 2 && !bg && P.d.a_k && P.d.b_k) return gemm_dispatch_tiles<true, true, 2, 0>(P, s);
  if (!ag && bg == 1 && !P.d.a_k && !P.d.b_k) return gemm_dispatch_tiles<false, false, 0, 1>(P, s);
  if (!ag && bg == 2 && !P.d.a_k && !P.d.b_k) return gemm_dispatch_tiles<false, false, 0, 2>(P, s);
  if (ag == 3 && bg == 4 && P.d.a_k && !P.d.b_k) return gemm_dispatch_tiles<true, false, 3, 4>(P, s);
  return hipErrorInvalidValue;
}
}  // namespace aca
