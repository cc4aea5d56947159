// GEMM tile config 6: 256x192 block tile, 2x4 waves (128x48 per wave), pipelined main loop.
// 192 = 768 / 4: GPT-2-small's N = 768 / 2304 / 3072 / 50304 GEMMs tile the 256 CUs with no
// wave-quantisation tail (e.g. 16384x768 -> exactly 256 blocks).
#include "gemm_impl.h"

void rn_gemm_launch_cfg6(rn_gemm_detail::GemmArgs& a, bool ak, bool bk, int act, hipStream_t st) {
    rn_gemm_detail::launch_cfg<256, 192, 2, 4, true>(a, ak, bk, act, st);
}
