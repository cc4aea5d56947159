// GEMM tile config 0: 128x128 block tile, 2x2 waves, simple main loop.
#include "gemm_impl.h"

void rn_gemm_launch_cfg0(rn_gemm_detail::GemmArgs& a, bool ak, bool bk, int act, hipStream_t st) {
    rn_gemm_detail::launch_cfg<128, 128, 2, 2, false>(a, ak, bk, act, st);
}
