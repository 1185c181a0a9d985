// Instantiations of the MFMA GEMM for plain strided operands (all four storage layouts).
#include "gemm_impl.h"

namespace aca {
hipError_t gemm_plain(const GemmParams& P, hipStream_t s) {
  const AcaGemmDesc& d = P.d;
  const bool a = d.a_k, b = d.b_k;
  const bool vec = gemm_operand_vec(d.A, d.lda, a ? d.K : d.M) && gemm_operand_vec(d.B, d.ldb, b ? d.K : d.N);
  if (vec) {
    if (a && b) return gemm_dispatch_tiles<true, true, 0, 0, true>(P, s);
    if (a && !b) return gemm_dispatch_tiles<true, false, 0, 0, true>(P, s);
    if (!a && b) return gemm_dispatch_tiles<false, true, 0, 0, true>(P, s);
    return gemm_dispatch_tiles<false, false, 0, 0, true>(P, s);
  }
  if (a && b) return gemm_dispatch_tiles<true, true, 0, 0, false>(P, s);
  if (a && !b) return gemm_dispatch_tiles<true, false, 0, 0, false>(P, s);
  if (!a && b) return gemm_dispatch_tiles<false, true, 0, 0, false>(P, s);
  return gemm_dispatch_tiles<false, false, 0, 0, false>(P, s);
}
}  // namespace aca
