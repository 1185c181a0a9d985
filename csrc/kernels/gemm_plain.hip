// Instantiations of the MFMA GEMM for plain strided operands (all four storage layouts).
#include "gemm_impl.h"

namespace aca {
hipError_t gemm_plain(const GemmParams& P, hipStream_t s) {
  const bool a = P.d.a_k, b = P.d.b_k;
  if (a && b) return gemm_dispatch_tiles<true, true, 0, 0>(P, s);
  if (a && !b) return gemm_dispatch_tiles<true, false, 0, 0>(P, s);
  if (!a && b) return gemm_dispatch_tiles<false, true, 0, 0>(P, s);
  return gemm_dispatch_tiles<false, false, 0, 0>(P, s);
}
}  // namespace aca
