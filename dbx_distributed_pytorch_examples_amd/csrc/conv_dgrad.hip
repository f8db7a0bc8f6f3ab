// Data-gradient instantiations of igemm_kernel (conv_igemm_kernel.h): its own translation unit.
#include "conv_igemm_kernel.h"

using namespace dbx;

template <int BM, int BN>
static int dispatch_dgrad(const IGemmArgs& a, bool accum, int epi, int dma, hipStream_t st) {
  if (a.res) {  // BN-backward apply prologue (1x1 stride-1 dgrads of the bottleneck)
    constexpr int TM = BM, TN = BN;  // (128 x 256 fits since the half-split tail prologue: no remap)
    if (accum) {
      if (epi == 1) DBX_DMA_PRO(launch_igemm_t, TM, TN, DGRAD, true, false, true, 1, true);
      if (epi == 0) DBX_DMA_PRO(launch_igemm_t, TM, TN, DGRAD, true, false, true, 0, true);
      return -11;
    }
    if (epi == 2) DBX_DMA_PRO(launch_igemm_t, TM, TN, DGRAD, true, false, false, 2, true);
    if (epi == 0) DBX_DMA_PRO(launch_igemm_t, TM, TN, DGRAD, true, false, false, 0, true);
    return -11;
  }
  if (accum) {
    if (epi == 1) DBX_DMA_PLAIN(launch_igemm_t, BM, BN, DGRAD, false, false, true, 1, false);
    if (epi == 2) DBX_DMA_PLAIN(launch_igemm_t, BM, BN, DGRAD, false, false, true, 2, false);
    DBX_DMA_PLAIN(launch_igemm_t, BM, BN, DGRAD, false, false, true, 0, false);
  }
  if (epi == 1) DBX_DMA_PLAIN(launch_igemm_t, BM, BN, DGRAD, false, false, false, 1, false);
  if (epi == 2) DBX_DMA_PLAIN(launch_igemm_t, BM, BN, DGRAD, false, false, false, 2, false);
  DBX_DMA_PLAIN(launch_igemm_t, BM, BN, DGRAD, false, false, false, 0, false);
}

int dbx_dispatch_dgrad(int bm, int bn, const IGemmArgs& a, bool accum, int epi, int dma, hipStream_t st) {
  DBX_TILES(dispatch_dgrad, a, accum, epi, dma, st)
  return -3;
}
