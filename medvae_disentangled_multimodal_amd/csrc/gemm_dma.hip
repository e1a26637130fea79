// GEMM launches of the bf16-stored operand path (PREC 4, LDS-DMA main loop of gemm3x_kernel): conv fwd / dgrad
// gathers and plain row-major products over packed bf16 operands (bf16-mixed mode).
#include "gemm_core.h"

namespace mvae {

void conv_dma(int ak, GemmArgs& a, hipStream_t st, int cfg) {
  switch (ak) {
    case A_CONV_FWD: launch_dma<A_CONV_FWD>(a, st, cfg); break;
    case A_CONV_DGRAD: launch_dma<A_CONV_DGRAD>(a, st, cfg); break;
    case A_CONV_SUBPIX: launch_dma<A_CONV_SUBPIX>(a, st, cfg); break;
    default: launch_dma<A_ROWK>(a, st, cfg); break;
  }
}

template <int BKIND>
static void wgrad_dma_cfg(GemmArgs& a, hipStream_t st, int cfg) {
  switch (cfg) {
    case T256x256: launch_cfg<T256x256, A_COLM, 4, BKIND, 4, 4>(a, st); break;
    case T256x128: launch_cfg<T256x128, A_COLM, 4, BKIND, 4, 4>(a, st); break;
    case T128x256: launch_cfg<T128x256, A_COLM, 4, BKIND, 4, 4>(a, st); break;
    case T128x128: launch_cfg<T128x128, A_COLM, 4, BKIND, 4, 4>(a, st); break;
    default: launch_cfg<T64x64, A_COLM, 4, BKIND, 4, 4>(a, st); break;
  }
}

void wgrad_dma(int bkind, GemmArgs& a, hipStream_t st, int cfg) {
  if (bkind == B_WGRAD_SUBPIX) wgrad_dma_cfg<B_WGRAD_SUBPIX>(a, st, cfg);
  else wgrad_dma_cfg<B_WGRAD_FWD>(a, st, cfg);
}

}  // namespace mvae
