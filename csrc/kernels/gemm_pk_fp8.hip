// Persistent 256x256 GEMM (tile config 9, csrc/include/gemm_pk.h) on e4m3 operands: the fp8
// forward GEMM x8 · W8ᵀ (both K-contiguous) with the bf16 kernel's fused epilogues.
#include "gemm_pk.h"

using namespace rn_gemm_detail;

void rn_gemm_launch_pk_fp8(GemmArgs& a, int act, hipStream_t st) {
    switch (act) {
        case ACT_GELU: launch_pk_t<true, true, ACT_GELU, false, false, 0, true>(a, st); break;
        case ACT_GELU_D: launch_pk_t<true, true, ACT_GELU_D, false, false, 0, true>(a, st); break;
        case ACT_RELU: launch_pk_t<true, true, ACT_RELU, false, false, 0, true>(a, st); break;
        default: launch_pk_t<true, true, ACT_NONE, false, false, 0, true>(a, st); break;
    }
}
