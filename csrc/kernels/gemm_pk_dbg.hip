// Timing-only ablation builds of the persistent GEMM (cfg 90 + DBG, see gemm_pk.h): plain
// bf16 NT / NN with parts of the kernel removed.  Outputs are WRONG; used by scripts only.
#include "gemm_pk.h"

using namespace rn_gemm_detail;

template <int DBG>
static void launch_dbg(GemmArgs& a, bool ak, bool bk, hipStream_t st) {
    if (ak && bk) launch_pk_t<true, true, ACT_NONE, false, false, DBG>(a, st);
    else launch_pk_t<true, false, ACT_NONE, false, false, DBG>(a, st);
}

int rn_gemm_launch_pk_dbg(GemmArgs& a, bool ak, bool bk, int dbg, hipStream_t st) {
    if (!ak || a.split > 1) return -1;
    switch (dbg) {
        case 1: launch_dbg<1>(a, ak, bk, st); break;
        case 2: launch_dbg<2>(a, ak, bk, st); break;
        case 3: launch_dbg<3>(a, ak, bk, st); break;
        case 4: launch_dbg<4>(a, ak, bk, st); break;
        case 5: launch_dbg<5>(a, ak, bk, st); break;
        case 8: launch_dbg<8>(a, ak, bk, st); break;
        case 9: launch_dbg<9>(a, ak, bk, st); break;
        case 16: launch_dbg<16>(a, ak, bk, st); break;
        case 32: launch_dbg<32>(a, ak, bk, st); break;
        case 64: launch_dbg<64>(a, ak, bk, st); break;
        default: return -1;
    }
    return 0;
}
