// DMA-engine conv tiles with MT = 1 (see conv3d_impl.h); a translation unit
// per MT keeps the ~60 instantiations compiling in parallel.
#include "conv3d_impl.h"

namespace lea {
LEA_DMA_TU(1)

int run_dma_dp(const Plan& p, const ConvArgs& a, int B, hipStream_t st) {
  LEA_DMA_DP_LIST(LEA_DMA_DP_RUN_CASE)
  set_error("lea_conv3d: no depth-paired tile <1, %d, %d>", p.nt, p.tw);
  return LEA_E_UNSUPPORTED;
}
}  // namespace lea
