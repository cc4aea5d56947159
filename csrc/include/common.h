// Shared device helpers for the replicann gfx950 kernels.
//
// Everything here is written for CDNA4 directly: 64-lane waves, bf16 moved as
// 16-byte vectors (8 elements per lane), fp32 math, hardware bf16 converts.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

typedef __bf16 bf16;
typedef short  s16x8 __attribute__((ext_vector_type(8)));
typedef short  s16x4 __attribute__((ext_vector_type(4)));
typedef float  f32x4 __attribute__((ext_vector_type(4)));
typedef float  f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

#define RN_WAVE 64
#define RN_DEV __device__ __forceinline__

// Debug build (REPLICANN_CHECK=1 python -m replicann_amd._build): device-side
// bounds checks on data-dependent indices (token ids, targets) trap the wave
// instead of reading/writing out of bounds.  Compiled out otherwise.
#ifdef REPLICANN_CHECK
#define RN_CHECK(c) do { if (!(c)) __builtin_trap(); } while (0)
#else
#define RN_CHECK(c) do { } while (0)
#endif

RN_DEV float bf2f(bf16 x) { return (float)x; }
RN_DEV bf16 f2bf(float x) { return (bf16)x; }

// 8 bf16 <-> 8 float
RN_DEV void load8(const bf16* p, float* f) {
    bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
}
RN_DEV void store8(bf16* p, const float* f) {
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (bf16)f[i];
    *reinterpret_cast<bf16x8*>(p) = v;
}

RN_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
RN_DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Block-wide sum for blockDim.x <= 1024 (scratch: >= 16 floats of LDS).
RN_DEV float block_sum(float v, float* scratch) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    float t = 0.f;
    for (int i = 0; i < nw; ++i) t += scratch[i];
    return t;
}
RN_DEV float block_max(float v, float* scratch) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    float t = -INFINITY;
    for (int i = 0; i < nw; ++i) t = fmaxf(t, scratch[i]);
    return t;
}

// Counter-based RNG (splitmix64 finaliser): uniform in [0,1) from (seed, index).
// Stateless, so dropout masks are regenerated in the backward instead of stored.
RN_DEV float hash_uniform(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);
}

// tanh-approximate GELU and its derivative, via the identity
//   0.5·x·(1 + tanh(u)) = x·σ(2u),  u = √(2/π)(x + 0.044715x³)
// → one v_exp_f32 + one v_rcp_f32 per element (no libm tanhf).
RN_DEV float fast_sigmoid(float z) { return __builtin_amdgcn_rcpf(1.f + __expf(-z)); }
// s = σ(2u) with the constants folded into the exp2 argument: 2u·log2e = x·(B + A·x²), so the
// argument is one FMA + one multiply and exp2 is the raw v_exp_f32 (its argument range is the
// whole line, but σ saturates correctly: exp2(+big) = inf → rcp(inf) = 0, exp2(-big) = 0 → 1).
RN_DEV float gelu_sig(float x, float x2) {
    constexpr float c = 0.7978845608028654f, L2E = 1.4426950408889634f;
    constexpr float B = -2.f * c * L2E, A = -2.f * c * 0.044715f * L2E;
    return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * __builtin_fmaf(x2, A, B)));
}
RN_DEV float gelu_f(float x) { return x * gelu_sig(x, x * x); }
// d/dx x·σ(2u) = s + s(1-s)·k,  k = 2x·u'(x)/… = x·(2c + 2c·3·0.044715·x²)  →  d = s·(1 + (1-s)·k)
RN_DEV float gelu_dk(float x, float x2) {
    constexpr float c = 0.7978845608028654f;
    return x * __builtin_fmaf(x2, 2.f * c * 0.134145f, 2.f * c);
}
RN_DEV float gelu_grad_f(float x) {
    const float x2 = x * x;
    const float s = gelu_sig(x, x2);
    const float k = gelu_dk(x, x2);
    return __builtin_fmaf(s, __builtin_fmaf(-s, k, k), s);
}

// gelu(x) and gelu'(x) sharing one exp + rcp
RN_DEV float gelu_and_grad_f(float x, float& d) {
    const float x2 = x * x;
    const float s = gelu_sig(x, x2);
    const float k = gelu_dk(x, x2);
    d = __builtin_fmaf(s, __builtin_fmaf(-s, k, k), s);
    return x * s;
}

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_RELU_BWD = 3, ACT_GELU_BWD = 4, ACT_GELU_D = 5, ACT_MUL_BWD = 6 };
// *_BWD (GEMM epilogue only): out = acc · act'(aux) with aux = the saved pre-activation,
// i.e. the activation backward fused into the dgrad GEMM that produces dY·W.
// ACT_GELU_D: GELU whose forward epilogue saves gelu'(h) instead of h (computed with the same
// exp / rcp as gelu(h)); its backward ACT_MUL_BWD is then one multiply per element, out = acc · aux,
// instead of re-deriving gelu'(h) (exp, rcp and ~10 FMAs) in the dgrad epilogue.
constexpr bool act_fwd(int a) { return a == ACT_RELU || a == ACT_GELU || a == ACT_GELU_D; }
constexpr bool act_bwd(int a) { return a == ACT_RELU_BWD || a == ACT_GELU_BWD || a == ACT_MUL_BWD; }

template <int ACT>
RN_DEV float act_f(float x) {
    if constexpr (ACT == ACT_RELU) return fmaxf(x, 0.f);
    else if constexpr (ACT == ACT_GELU || ACT == ACT_GELU_D) return gelu_f(x);
    else return x;
}
template <int ACT>
RN_DEV float act_grad_f(float x) {
    if constexpr (ACT == ACT_RELU || ACT == ACT_RELU_BWD) return x > 0.f ? 1.f : 0.f;
    else if constexpr (ACT == ACT_GELU || ACT == ACT_GELU_BWD) return gelu_grad_f(x);
    else if constexpr (ACT == ACT_MUL_BWD) return x;
    else return 1.f;
}
// forward epilogue with a pre-activation buffer: returns act(h), *pre = what the buffer stores
template <int ACT>
RN_DEV float act_fwd_pre(float h, float& pre) {
    if constexpr (ACT == ACT_GELU_D) return gelu_and_grad_f(h, pre);
    else {
        pre = h;
        return act_f<ACT>(h);
    }
}

#define HIP_CHECK_LAUNCH() (void)hipGetLastError()

static inline int rn_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------------------
// Deterministic parallel column reduction of an fp32 [R][C] partial matrix:
// stage 1 grid (ceil(C/64), S) — each wave sums a strided subset of rows for 64
// columns (256-B coalesced rows), 4 waves combine in LDS → tmp[S][C];
// stage 2 one thread per column sums the S stage-1 rows in fixed order and
// writes fp32 and/or bf16.  Fixed summation order → bitwise reproducible.
// ---------------------------------------------------------------------------
constexpr int RN_COLRED_S = 32;

namespace {  // internal linkage: every TU gets its own copy

__global__ void __launch_bounds__(256) rn_colred1_k(const float* __restrict__ in, int R, int C,
                                                    float* __restrict__ tmp) {
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    const int S = gridDim.y;
    const int r0 = (int)((long)R * blockIdx.y / S), r1 = (int)((long)R * (blockIdx.y + 1) / S);
    float s = 0.f;
    if (c < C)
        for (int r = r0 + w; r < r1; r += 4) s += in[(long)r * C + c];
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && c < C) tmp[(long)blockIdx.y * C + c] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

__global__ void rn_colred2_k(const float* __restrict__ tmp, int S, int C, long ld, float* __restrict__ out32,
                             __bf16* __restrict__ out16, int accum) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float s = 0.f;
    for (int i = 0; i < S; ++i) s += tmp[(long)i * ld + c];
    if (out32) out32[c] = s + (accum == 1 ? out32[c] : 0.f);
    if (out16) out16[c] = (__bf16)(s + (accum ? (float)out16[c] : 0.f));
}

// ---------------------------------------------------------------------------
// Single-launch version: grid (ceil(C/64), S); every block writes its stage-1
// row of tmp, bumps a per-column-chunk arrival counter, and the LAST arriving
// block of a chunk sums the S rows in fixed order and writes the outputs, then
// re-arms the counter.  One launch instead of two, still bitwise reproducible.
// Hand-off without fences (MI355X guide §6 G16, R1): the slab values are stored
// write-through (sc1, agent-scope atomic stores) and drained before the ticket,
// and the last arriver reads them with sc1 loads — an agent-scope release fence
// per block (buffer_wbl2, ≈1.7 µs each) made this kernel ~4× slower.  Outputs may
// be split into segments of `seg` columns (e.g. [dw | db] of LayerNorm in one pass).
// ---------------------------------------------------------------------------
constexpr int RN_COLSUM_MAXCB = 4096;
__device__ unsigned int rn_colsum_cnt[RN_COLSUM_MAXCB];  // zero at load, self-resetting

struct RnColOut {
    float* o32[3];
    __bf16* o16[3];
    int seg;
    int accum[3];  // per segment: 1 = add into both outputs, 2 = add into the bf16 output only
};

__global__ void __launch_bounds__(256) rn_colsum_k(const float* __restrict__ in, int R, int C,
                                                   float* tmp, RnColOut out) {
    __shared__ float red[4][64];
    __shared__ int is_last;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    const int S = gridDim.y;
    const int r0 = (int)((long)R * blockIdx.y / S), r1 = (int)((long)R * (blockIdx.y + 1) / S);
    // Batches of 8 independent loads per lane (one L2/HBM round trip per batch instead of one
    // per row); the adds stay in row order, so the result does not depend on the batching.
    float s = 0.f;
    if (c < C) {
        for (int rb = r0 + w; rb < r1; rb += 32) {
            float t[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {  // clamped row, no per-load branch (each would wait vmcnt(0))
                const int r = min(rb + 4 * u, r1 - 1);
                t[u] = in[(long)r * C + c];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) s += (rb + 4 * u < r1) ? t[u] : 0.f;
        }
    }
    red[w][lane] = s;
    __syncthreads();
    if (w == 0) {
        if (c < C)
            __hip_atomic_store(tmp + (long)blockIdx.y * C + c, red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1 write-through
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores drained
        if (lane == 0) {
            unsigned t = __hip_atomic_fetch_add(&rn_colsum_cnt[blockIdx.x], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
            is_last = (t == (unsigned)S - 1);
        }
    }
    __syncthreads();
    if (!is_last || w != 0) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
    if (c < C) {
        // all S (≤ RN_COLRED_S) slab values in flight at once (sc1 loads), summed in fixed order
        float t[RN_COLRED_S];
#pragma unroll
        for (int i = 0; i < RN_COLRED_S; ++i)
            t[i] = __hip_atomic_load(tmp + (long)min(i, S - 1) * C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < RN_COLRED_S; ++i) acc += i < S ? t[i] : 0.f;
        const int k = c / out.seg, o = c - k * out.seg;
        if (out.o32[k]) out.o32[k][o] = acc + (out.accum[k] == 1 ? out.o32[k][o] : 0.f);
        if (out.o16[k]) out.o16[k][o] = (__bf16)(acc + (out.accum[k] ? (float)out.o16[k][o] : 0.f));
    }
    if (lane == 0) __hip_atomic_store(&rn_colsum_cnt[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Short inputs (R <= RN_COLSUM1_R rows, e.g. the GEMM epilogue's 256 per-tile-row bias partials or
// the attention backward's 1024 per-block qkv-bias partials):
// ONE block of 16 waves per 64 columns sums all rows — each wave a strided row subset in 16-deep
// load batches (adds in row order), the 16 wave sums combined in fixed order through LDS.  No
// second stage, no arrival ticket: one load round trip per 16 rows per wave instead of the
// two-stage kernel's slab write + ticket + slab read.  Bitwise reproducible (fixed order).
// (gpt2-small step: 49 column sums 0.448 -> 0.344 ms at R <= 512, profiles/r3s_resume_xent_gelu.txt)
constexpr int RN_COLSUM1_R = 1024;

__global__ void __launch_bounds__(1024) rn_colsum1_k(const float* __restrict__ in, int R, int C, RnColOut out) {
    __shared__ float red[16][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    float s = 0.f;
    if (c < C) {
        for (int rb = w; rb < R; rb += 256) {
            float t[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) t[u] = in[(long)min(rb + 16 * u, R - 1) * C + c];
#pragma unroll
            for (int u = 0; u < 16; ++u) s += (rb + 16 * u < R) ? t[u] : 0.f;
        }
    }
    red[w][lane] = s;
    __syncthreads();
    if (w != 0 || c >= C) return;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += red[i][lane];
    const int k = c / out.seg, o = c - k * out.seg;
    if (out.o32[k]) out.o32[k][o] = acc + (out.accum[k] == 1 ? out.o32[k][o] : 0.f);
    if (out.o16[k]) out.o16[k][o] = (__bf16)(acc + (out.accum[k] ? (float)out.o16[k][o] : 0.f));
}

// Segmented column reduction: out.seg columns per output segment (≤ 3 segments).
// tmp must hold RN_COLRED_S * C floats.
static inline void rn_colreduce_seg(const float* in, int R, int C, float* tmp, const RnColOut& out,
                                    hipStream_t st) {
    if (R <= RN_COLSUM1_R) {
        rn_colsum1_k<<<(C + 63) / 64, 1024, 0, st>>>(in, R, C, out);
        return;
    }
    // >= 32 rows per block (8-deep load batches for each of its 4 waves), at most RN_COLRED_S blocks
    int S = (R + 31) / 32;
    S = S < 1 ? 1 : (S > RN_COLRED_S ? RN_COLRED_S : S);
    const int cb = (C + 63) / 64;
    if (cb <= RN_COLSUM_MAXCB) {
        rn_colsum_k<<<dim3(cb, S), 256, 0, st>>>(in, R, C, tmp, out);
        return;
    }
    rn_colred1_k<<<dim3(cb, S), 256, 0, st>>>(in, R, C, tmp);
    for (int k = 0; k * out.seg < C; ++k)
        rn_colred2_k<<<(out.seg + 255) / 256, 256, 0, st>>>(
            tmp + (long)k * out.seg, S, out.seg < C - k * out.seg ? out.seg : C - k * out.seg, C, out.o32[k],
            out.o16[k], out.accum[k]);
}

// tmp must hold RN_COLRED_S * C floats.  accum: add into the outputs (gradient accumulation).
static inline void rn_colreduce(const float* in, int R, int C, float* tmp, float* out32, __bf16* out16,
                                hipStream_t st, int accum = 0) {
    RnColOut o{{out32, nullptr, nullptr}, {out16, nullptr, nullptr}, C, {accum, 0, 0}};
    rn_colreduce_seg(in, R, C, tmp, o, st);
}

}  // namespace
