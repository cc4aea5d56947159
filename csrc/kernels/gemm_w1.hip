// One-wave-per-SIMD persistent GEMM (tile config 11, csrc/include/gemm_w1.h): the forward x·Wᵀ on
// bf16 or e4m3 operands with the bias / plain epilogue interleaved into the next tile.
#include <cstdlib>

#include "gemm_w1.h"

using namespace rn_gemm_detail;

// a.res: + residual (row stride ldc; x·Wᵀ layout, K >= 6 K-tiles).
// a: A K-contiguous, B K-contiguous ([N][K], bmn false) or MN-contiguous ([K][N], bmn true: bf16 only);
// K, lda, ldb in BYTES (K % 128 == 0, K >= 256); ldc in elements; N % 8 == 0
int rn_gemm_launch_w1(GemmArgs& a, int fp8, int act, hipStream_t st, bool bmn) {
    if (a.K % 128 || a.K < 256 || a.N % 8 || a.ldc % 8 || a.lda % 16 || a.ldb % 16) return -1;
    if (act != ACT_NONE) return -1;
    if (a.alpha && a.bias) return -1;
    if (bmn && fp8) return -1;
    if (a.res && (bmn || a.alpha || a.K / 128 < 6)) return -1;  // residual bodies: K-tiles 1-4 of >= 6
    a.tiles_m = (a.M + 255) / 256;
    a.tiles_n = (a.N + 255) / 256;
    static const int dbg = [] {
        const char* e = std::getenv("REPLICANN_W1_DBG");
        return e ? std::atoi(e) : 0;
    }();
    if (dbg && !bmn && !a.alpha && !a.res) {  // timing ablations (wrong outputs): see gemm_w1.h DBG
        if (fp8) {
            if (dbg == 1) launch_w1_t<1, ACT_NONE, false, true, 1>(a, st);
            else if (dbg == 2) launch_w1_t<1, ACT_NONE, false, true, 2>(a, st);
            else launch_w1_t<1, ACT_NONE, false, true, 3>(a, st);
        } else {
            if (dbg == 1) launch_w1_t<0, ACT_NONE, false, true, 1>(a, st);
            else if (dbg == 2) launch_w1_t<0, ACT_NONE, false, true, 2>(a, st);
            else launch_w1_t<0, ACT_NONE, false, true, 3>(a, st);
        }
        return 0;
    }
    if (a.res) {
        if (fp8) launch_w1_t<1, ACT_NONE, false, true, 0, true>(a, st);
        else launch_w1_t<0, ACT_NONE, false, true, 0, true>(a, st);
        return 0;
    }
    if (fp8) launch_w1_t<1, ACT_NONE, false, true>(a, st);
    else if (bmn) {
        if (a.alpha) launch_w1_t<0, ACT_NONE, true, false>(a, st);
        else launch_w1_t<0, ACT_NONE, false, false>(a, st);
    } else if (a.alpha) launch_w1_t<0, ACT_NONE, true, true>(a, st);
    else launch_w1_t<0, ACT_NONE, false, true>(a, st);
    return 0;
}
