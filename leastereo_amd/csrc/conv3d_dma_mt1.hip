// DMA-engine conv tiles with MT = 1 (see conv3d_impl.h); a translation unit
// per MT keeps the ~60 instantiations compiling in parallel.
#include "conv3d_impl.h"

namespace lea {
LEA_DMA_TU(1)
}  // namespace lea
