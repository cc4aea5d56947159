// Persistent 256x256 GEMM (tile config 9, csrc/include/gemm_pk.h), operand layout ft
// (A M-contiguous, B K-contiguous): static-walk instantiations and the entry point.
#include "gemm_pk_launch.h"

RN_PK_ENTRY(rn_gemm_launch_pk_ft, false, true)
