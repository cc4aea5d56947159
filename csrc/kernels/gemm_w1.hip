// One-wave-per-SIMD persistent GEMM (tile config 11, csrc/include/gemm_w1.h): the forward x·Wᵀ on
// bf16 or e4m3 operands with the bias / plain epilogue interleaved into the next tile.
#include "gemm_w1.h"

using namespace rn_gemm_detail;

// a: A K-contiguous, B K-contiguous ([N][K], bmn false) or MN-contiguous ([K][N], bmn true: bf16 only);
// K, lda, ldb in BYTES (K % 128 == 0, K >= 256); ldc in elements; N % 8 == 0
int rn_gemm_launch_w1(GemmArgs& a, int fp8, int act, hipStream_t st, bool bmn) {
    if (a.K % 128 || a.K < 256 || a.N % 8 || a.ldc % 8 || a.lda % 16 || a.ldb % 16) return -1;
    if (act != ACT_NONE) return -1;
    if (a.alpha && a.bias) return -1;
    if (bmn && fp8) return -1;
    a.tiles_m = (a.M + 255) / 256;
    a.tiles_n = (a.N + 255) / 256;
    if (fp8) launch_w1_t<1, ACT_NONE, false, true>(a, st);
    else if (bmn) {
        if (a.alpha) launch_w1_t<0, ACT_NONE, true, false>(a, st);
        else launch_w1_t<0, ACT_NONE, false, false>(a, st);
    } else if (a.alpha) launch_w1_t<0, ACT_NONE, true, true>(a, st);
    else launch_w1_t<0, ACT_NONE, false, true>(a, st);
    return 0;
}
