// GEMM tile config 3: 128x256 block tile, 2x4 waves, simple main loop.
#include "gemm_impl.h"

void rn_gemm_launch_cfg3(rn_gemm_detail::GemmArgs& a, bool ak, bool bk, int act, hipStream_t st) {
    rn_gemm_detail::launch_cfg<128, 256, 2, 4, false>(a, ak, bk, act, st);
}
