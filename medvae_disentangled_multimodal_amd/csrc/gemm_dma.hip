// GEMM launches of the LDS-DMA staged operand paths of gemm3x_kernel: PREC 4 (packed bf16 operands, bf16-mixed mode)
// and PREC 5 (planar 3xBF16 operands, fp32-class mode) -- conv fwd / dgrad gathers, plain row-major products and the
// weight gradient.
#include "gemm_core.h"

namespace mvae {

template <int P>
static void conv_dma_p(int ak, GemmArgs& a, hipStream_t st, int cfg) {
  switch (ak) {
    case A_CONV_FWD: launch_dma<A_CONV_FWD, P>(a, st, cfg); break;
    case A_CONV_DGRAD: launch_dma<A_CONV_DGRAD, P>(a, st, cfg); break;
    case A_CONV_SUBPIX: launch_dma<A_CONV_SUBPIX, P>(a, st, cfg); break;
    default: launch_dma<A_ROWK, P>(a, st, cfg); break;
  }
}

void conv_dma(int ak, GemmArgs& a, hipStream_t st, int cfg, int prec) {
  if (prec == 5) conv_dma_p<5>(ak, a, st, cfg);
  else conv_dma_p<4>(ak, a, st, cfg);
}

template <int BKIND, int P>
static void wgrad_dma_cfg(GemmArgs& a, hipStream_t st, int cfg) {
  switch (cfg) {
    case T256x256: launch_cfg<T256x256, A_COLM, 4, BKIND, 4, P>(a, st); break;
    case T256x128: launch_cfg<T256x128, A_COLM, 4, BKIND, 4, P>(a, st); break;
    case T128x256: launch_cfg<T128x256, A_COLM, 4, BKIND, 4, P>(a, st); break;
    case T128x128: launch_cfg<T128x128, A_COLM, 4, BKIND, 4, P>(a, st); break;
    default: launch_cfg<T64x64, A_COLM, 4, BKIND, 4, P>(a, st); break;
  }
}

void wgrad_dma(int bkind, GemmArgs& a, hipStream_t st, int cfg, int prec) {
  if (prec == 5) {
    if (bkind == B_WGRAD_SUBPIX) wgrad_dma_cfg<B_WGRAD_SUBPIX, 5>(a, st, cfg);
    else if (bkind == B_WGRAD_P2) wgrad_dma_cfg<B_WGRAD_P2, 5>(a, st, cfg);
    else wgrad_dma_cfg<B_WGRAD_FWD, 5>(a, st, cfg);
  } else {
    if (bkind == B_COLN) wgrad_dma_cfg<B_COLN, 4>(a, st, cfg);
    else if (bkind == B_WGRAD_SUBPIX) wgrad_dma_cfg<B_WGRAD_SUBPIX, 4>(a, st, cfg);
    else if (bkind == B_WGRAD_P2) wgrad_dma_cfg<B_WGRAD_P2, 4>(a, st, cfg);
    else wgrad_dma_cfg<B_WGRAD_FWD, 4>(a, st, cfg);
  }
}

}  // namespace mvae

