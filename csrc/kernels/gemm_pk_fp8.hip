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

// fp8 weight gradient dW = dYᵀ·X on MN-contiguous operands (gemm_pk.h, F8MN): A = dY [K][M] in e5m2
// (a_bf8) or e4m3, B = X [K][N] in e4m3, fp32 split-K slabs, then the fixed-order slab reduction
// (bf16 or fp32 output, accumulate or overwrite): deterministic.
void rn_gemm_launch_pk_fp8_wgrad(GemmArgs& a, int a_bf8, hipStream_t st) {
    if (a_bf8) launch_pk_t<false, false, ACT_NONE, true, true, 0, 2>(a, st);
    else launch_pk_t<false, false, ACT_NONE, true, true, 0, 1>(a, st);
    const long total4 = ((long)a.M * a.N + 3) / 4;
    const int g = (int)std::min<long>((total4 + 255) / 256, 4096);
    splitk_reduce_k<ACT_NONE><<<g, 256, 0, st>>>(a);
}

// fp8 data gradient dX = dY·W: A = dY [M][K] (e5m2 if a_bf8, else e4m3; K-contiguous, as produced),
// B = W [K][N] (the weight as stored, [out][in] = [K][N]: MN-contiguous, read transposed), bf16 out.
void rn_gemm_launch_pk_fp8_dgrad(GemmArgs& a, int a_bf8, hipStream_t st) {
    if (a_bf8) launch_pk_t<true, false, ACT_NONE, false, false, 0, 2>(a, st);
    else launch_pk_t<true, false, ACT_NONE, false, false, 0, 1>(a, st);
}
