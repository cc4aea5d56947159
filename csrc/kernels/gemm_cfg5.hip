// GEMM tile config 5: 128x128 block tile, 2x2 waves, pipelined main loop.
#include "gemm_impl.h"

void rn_gemm_launch_cfg5(rn_gemm_detail::GemmArgs& a, bool ak, bool bk, int act, hipStream_t st) {
    rn_gemm_detail::launch_cfg<128, 128, 2, 2, true>(a, ak, bk, act, st);
}
