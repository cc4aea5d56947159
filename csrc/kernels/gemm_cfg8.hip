// GEMM tile config 8: 256x128 block tile, 4x2 waves, 3-stage LDS ring (2 tiles in flight).
#include "gemm_impl.h"

void rn_gemm_launch_cfg8(rn_gemm_detail::GemmArgs& a, bool ak, bool bk, int act, hipStream_t st) {
    rn_gemm_detail::launch_cfg<256, 128, 4, 2, true, 3>(a, ak, bk, act, st);
}
