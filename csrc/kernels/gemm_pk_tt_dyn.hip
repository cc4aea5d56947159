// Persistent 256x256 GEMM, operand layout tt: the dynamic-tile-queue instantiations
// (gemm_pk.h "Tile schedule"), a unit of their own so they compile beside the static ones.
#include "gemm_pk_launch.h"

RN_PK_ENTRY_DYN(rn_gemm_launch_pk_tt, true, true)
