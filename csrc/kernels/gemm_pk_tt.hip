// Persistent 256x256 GEMM (tile config 9, csrc/include/gemm_pk.h) for operand layout
// A K-contiguous, B K-contiguous.
#include "gemm_pk.h"

using namespace rn_gemm_detail;

void rn_gemm_launch_pk_tt(GemmArgs& a, int act, hipStream_t st) {
    if (a.split > 1) {
        launch_pk_t<true, true, ACT_NONE, true, true>(a, st);
        const long total4 = ((long)a.M * a.N + 3) / 4;
        const int g = (int)std::min<long>((total4 + 255) / 256, 4096);
        if (act == ACT_GELU) splitk_reduce_k<ACT_GELU><<<g, 256, 0, st>>>(a);
        else if (act == ACT_GELU_D) splitk_reduce_k<ACT_GELU_D><<<g, 256, 0, st>>>(a);
        else if (act == ACT_RELU) splitk_reduce_k<ACT_RELU><<<g, 256, 0, st>>>(a);
        else if (act == ACT_GELU_BWD) splitk_reduce_k<ACT_GELU_BWD><<<g, 256, 0, st>>>(a);
        else if (act == ACT_RELU_BWD) splitk_reduce_k<ACT_RELU_BWD><<<g, 256, 0, st>>>(a);
        else splitk_reduce_k<ACT_NONE><<<g, 256, 0, st>>>(a);
        return;
    }
    if (a.out_f32) { launch_pk_t<true, true, ACT_NONE, false, true>(a, st); return; }
    switch (act) {
        case ACT_GELU: launch_pk_t<true, true, ACT_GELU, false, false>(a, st); break;
        case ACT_GELU_D: launch_pk_t<true, true, ACT_GELU_D, false, false>(a, st); break;
        case ACT_RELU: launch_pk_t<true, true, ACT_RELU, false, false>(a, st); break;

        default: launch_pk_t<true, true, ACT_NONE, false, false>(a, st); break;
    }
}
