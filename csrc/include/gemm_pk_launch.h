// Per-layout launch of the persistent GEMM (config 9, gemm_pk.h): the epilogue switch shared by the
// static-walk instantiations (gemm_pk_{tt,tf,ft,ff}.hip) and the dynamic-queue ones
// (gemm_pk_{tt,tf,ft,ff}_dyn.hip, separate units so both compile in parallel).  The split-K slab
// reduction that follows a split launch is issued by the static unit's entry point.
#pragma once
#include "gemm_pk.h"


namespace rn_gemm_detail {


template <bool AK, bool BKC, bool DYN>
void pk_launch_layout(GemmArgs& a, int act, hipStream_t st) {
    constexpr bool dgrad = AK && !BKC;  // activation-backward epilogues: dY·W layout only
    constexpr bool fwd = AK && BKC;     // saved-derivative GELU: x·Wᵀ layout only
    if (a.split > 1) {
        launch_pk_t<AK, BKC, ACT_NONE, true, true, 0, false, DYN>(a, st);
        return;
    }
    if (a.out_f32) {
        launch_pk_t<AK, BKC, ACT_NONE, false, true, 0, false, DYN>(a, st);
        return;
    }
    switch (act) {
        case ACT_GELU: launch_pk_t<AK, BKC, ACT_GELU, false, false, 0, false, DYN>(a, st); return;
        case ACT_RELU: launch_pk_t<AK, BKC, ACT_RELU, false, false, 0, false, DYN>(a, st); return;
        case ACT_GELU_D:
            if constexpr (fwd) { launch_pk_t<AK, BKC, ACT_GELU_D, false, false, 0, false, DYN>(a, st); return; }
            break;
        case ACT_GELU_BWD:
            if constexpr (dgrad) { launch_pk_t<AK, BKC, ACT_GELU_BWD, false, false, 0, false, DYN>(a, st); return; }
            break;
        case ACT_MUL_BWD:
            if constexpr (dgrad) { launch_pk_t<AK, BKC, ACT_MUL_BWD, false, false, 0, false, DYN>(a, st); return; }
            break;
        case ACT_RELU_BWD:
            if constexpr (dgrad) { launch_pk_t<AK, BKC, ACT_RELU_BWD, false, false, 0, false, DYN>(a, st); return; }
            break;
        default: break;
    }
    launch_pk_t<AK, BKC, ACT_NONE, false, false, 0, false, DYN>(a, st);
}

// the split-K slab reduction + epilogue after a split launch (fixed slab order: deterministic)
inline void pk_splitk_reduce(GemmArgs& a, int act, hipStream_t st) {
    const long total4 = ((long)a.M * a.N + 3) / 4;
    const int g = (int)std::min<long>((total4 + 255) / 256, 4096);
    switch (act) {
        case ACT_GELU: splitk_reduce_k<ACT_GELU><<<g, 256, 0, st>>>(a); break;
        case ACT_GELU_D: splitk_reduce_k<ACT_GELU_D><<<g, 256, 0, st>>>(a); break;
        case ACT_RELU: splitk_reduce_k<ACT_RELU><<<g, 256, 0, st>>>(a); break;
        case ACT_GELU_BWD: splitk_reduce_k<ACT_GELU_BWD><<<g, 256, 0, st>>>(a); break;
        case ACT_MUL_BWD: splitk_reduce_k<ACT_MUL_BWD><<<g, 256, 0, st>>>(a); break;
        case ACT_RELU_BWD: splitk_reduce_k<ACT_RELU_BWD><<<g, 256, 0, st>>>(a); break;
        default:
            splitk_reduce_k<ACT_NONE><<<g, 256, 0, st>>>(a);
            break;
    }
}

}  // namespace rn_gemm_detail

// entry point of one layout: dynamic-queue launch when a counter slot is available (see
// pk_sched_slot), else the static walk; then the split-K reduction
#define RN_PK_ENTRY(NAME, AK, BKC)                                                        \
    void NAME##_dyn(rn_gemm_detail::GemmArgs& a, int act, hipStream_t st);               \
    void NAME(rn_gemm_detail::GemmArgs& a, int act, hipStream_t st) {                    \
        using namespace rn_gemm_detail;                                                   \
        int* slot = pk_sched_slot(a, st);                                                  \
        if (slot) {                                                                       \
            a.sched = slot;                                                               \
            NAME##_dyn(a, act, st);                                                       \
        } else {                                                                          \
            a.sched = nullptr;                                                            \
            pk_launch_layout<AK, BKC, false>(a, act, st);                                 \
        }                                                                                 \
        if (a.split > 1) pk_splitk_reduce(a, act, st);                                    \
    }
#define RN_PK_ENTRY_DYN(NAME, AK, BKC)                                                    \
    void NAME##_dyn(rn_gemm_detail::GemmArgs& a, int act, hipStream_t st) {               \
        rn_gemm_detail::pk_launch_layout<AK, BKC, true>(a, act, st);                      \
    }
