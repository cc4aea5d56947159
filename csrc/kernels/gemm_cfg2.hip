// GEMM tile config 2: 256x128 block tile, 4x2 waves, pipelined main loop.
#include "gemm_impl.h"

void rn_gemm_launch_cfg2(rn_gemm_detail::GemmArgs& a, bool ak, bool bk, int act, hipStream_t st) {
    rn_gemm_detail::launch_cfg<256, 128, 4, 2, true>(a, ak, bk, act, st);
}
