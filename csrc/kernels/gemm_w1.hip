// One-wave-per-SIMD persistent GEMM (tile config 11, csrc/include/gemm_w1.h): the forward x·Wᵀ on
// bf16 or e4m3 operands with the bias / plain epilogue interleaved into the next tile.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "gemm_w1.h"

using namespace rn_gemm_detail;

// a.res: + residual (row stride ldc; x·Wᵀ layout, K >= 6 K-tiles).
// a: A K-contiguous, B K-contiguous ([N][K], bmn false) or MN-contiguous ([K][N], bmn true; fp8: plain
// epilogue, N % 16 == 0; fp8 == 2: A in e5m2);
// K, lda, ldb in BYTES (K % 128 == 0, K >= 256); ldc in elements; N % 8 == 0
int rn_gemm_launch_w1(GemmArgs& a, int fp8, int act, hipStream_t st, bool bmn) {
    a.group_m = GROUP_M;
    if (a.K % 128 || a.K < 256 || a.N % 8 || a.ldc % 8 || a.lda % 16 || a.ldb % 16) return -1;
    if (act != ACT_NONE) return -1;
    if (a.alpha && a.bias) return -1;
    if (bmn && fp8 && (a.N % 16 || a.bias || a.res)) return -1;  // fp8 MN-contiguous B: plain / alpha epilogue
    if (fp8 && !bmn && a.alpha) return -1;
    if (a.res && (bmn || a.alpha || a.K / 128 < 6)) return -1;  // residual bodies: K-tiles 1-4 of >= 6
    a.tiles_m = (a.M + 255) / 256;
    a.tiles_n = (a.N + 255) / 256;
#ifdef REPLICANN_DEV
    // timing ablations (WRONG outputs by design, see gemm_w1.h DBG): developer builds only
    static const int dbg = [] {
        const char* e = std::getenv("REPLICANN_W1_DBG");
        return e ? std::atoi(e) : 0;
    }();
    if (dbg && !bmn && !a.alpha && !a.res) {
        if (fp8) {
            if (dbg == 1) launch_w1_t<1, ACT_NONE, false, true, 1>(a, st);
            else if (dbg == 2) launch_w1_t<1, ACT_NONE, false, true, 2>(a, st);
            else if (dbg == 4) launch_w1_t<1, ACT_NONE, false, true, 4>(a, st);
            else if (dbg == 8) launch_w1_t<1, ACT_NONE, false, true, 8>(a, st);
            else launch_w1_t<1, ACT_NONE, false, true, 3>(a, st);
        } else {
            if (dbg == 1) launch_w1_t<0, ACT_NONE, false, true, 1>(a, st);
            else if (dbg == 2) launch_w1_t<0, ACT_NONE, false, true, 2>(a, st);
            else if (dbg == 4) launch_w1_t<0, ACT_NONE, false, true, 4>(a, st);
            else if (dbg == 8) launch_w1_t<0, ACT_NONE, false, true, 8>(a, st);
            else launch_w1_t<0, ACT_NONE, false, true, 3>(a, st);
        }
        return 0;
    }
#else
    // a release build has no ablation kernels: a stray REPLICANN_W1_DBG must not pass silently
    static const bool dbg_set = std::getenv("REPLICANN_W1_DBG") != nullptr;
    if (dbg_set) {
        std::fprintf(stderr, "REPLICANN_W1_DBG is set but this _C.so is a release build (REPLICANN_DEV=0)\n");
        std::abort();
    }
#endif
    if (a.res) {
        if (fp8) launch_w1_t<1, ACT_NONE, false, true, 0, true>(a, st);
        else launch_w1_t<0, ACT_NONE, false, true, 0, true>(a, st);
        return 0;
    }
    if (fp8 && bmn) {  // the fp8 data gradient (A e4m3 or, fp8 == 2, e5m2; alpha: the fp8 LM head's g / n)
        if (fp8 == 2 && a.alpha) launch_w1_t<2, ACT_NONE, true, false>(a, st);
        else if (fp8 == 2) launch_w1_t<2, ACT_NONE, false, false>(a, st);
        else if (a.alpha) launch_w1_t<1, ACT_NONE, true, false>(a, st);
        else launch_w1_t<1, ACT_NONE, false, false>(a, st);
    } else if (fp8) launch_w1_t<1, ACT_NONE, false, true>(a, st);
    else if (bmn) {
        if (a.alpha) launch_w1_t<0, ACT_NONE, true, false>(a, st);
        else launch_w1_t<0, ACT_NONE, false, false>(a, st);
    } else if (a.alpha) launch_w1_t<0, ACT_NONE, true, true>(a, st);
    else launch_w1_t<0, ACT_NONE, false, true>(a, st);
    return 0;
}

// The fp8 weight gradient dW = dYᵀ·X on the one-wave-per-SIMD kernel: A = dY [K = tokens][M = out] (e5m2 if
// fp8 == 2), B = X [K][N = in] (e4m3), both MN-contiguous as stored; split-K fp32 slabs in ws (split × M × N
// floats) summed by splitk_reduce_k into C (bf16 or fp32, accumulate or not).  K, lda, ldb in bytes;
// M, N % 16; K / 128 divisible by split with >= 2 K-tiles per slab.  a.reduce_alpha (optional device scalar)
// multiplies the slab sum.
int rn_gemm_launch_w1_wgrad(GemmArgs& a, int fp8, int split, hipStream_t st) {
    a.group_m = GROUP_M;
    const int kt = a.K / 128;
    if (a.K % 128 || a.M % 16 || a.N % 16 || a.lda % 16 || a.ldb % 16 || split < 1 || kt % split || kt / split < 2)
        return -1;
    a.tiles_m = (a.M + 255) / 256;
    a.tiles_n = (a.N + 255) / 256;
    a.split = split;
    a.k_per_split = kt / split;
    a.slab_step = 1;
    if (fp8 == 2) launch_w1_t<2, ACT_NONE, false, false, 0, false, false, true>(a, st);
    else launch_w1_t<1, ACT_NONE, false, false, 0, false, false, true>(a, st);
    const long total4 = ((long)a.M * a.N + 3) / 4;
    const int g = (int)std::min<long>((total4 + 255) / 256, 4096);
    splitk_reduce_k<ACT_NONE><<<g, 256, 0, st>>>(a);
    return 0;
}
