// Shared device helpers for the replicann gfx950 kernels.
//
// Everything here is written for CDNA4 directly: 64-lane waves, bf16 moved as
// 16-byte vectors (8 elements per lane), fp32 math, hardware bf16 converts.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

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
RN_DEV float gelu_f(float x) {
    const float c2 = 2.f * 0.7978845608028654f;
    return x * fast_sigmoid(c2 * (x + 0.044715f * x * x * x));
}
RN_DEV float gelu_grad_f(float x) {
    const float c = 0.7978845608028654f;
    const float x2 = x * x;
    const float s = fast_sigmoid(2.f * c * (x + 0.044715f * x2 * x));
    // d/dx = s + 2·x·s·(1-s)·c·(1 + 3·0.044715·x²)
    return s + 2.f * x * s * (1.f - s) * c * (1.f + 0.134145f * x2);
}

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2 };

template <int ACT>
RN_DEV float act_f(float x) {
    if constexpr (ACT == ACT_RELU) return fmaxf(x, 0.f);
    else if constexpr (ACT == ACT_GELU) return gelu_f(x);
    else return x;
}
template <int ACT>
RN_DEV float act_grad_f(float x) {
    if constexpr (ACT == ACT_RELU) return x > 0.f ? 1.f : 0.f;
    else if constexpr (ACT == ACT_GELU) return gelu_grad_f(x);
    else return 1.f;
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

__global__ void rn_colred2_k(const float* __restrict__ tmp, int S, int C, float* __restrict__ out32,
                             __bf16* __restrict__ out16, int accum) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float s = 0.f;
    for (int i = 0; i < S; ++i) s += tmp[(long)i * C + c];
    if (out32) out32[c] = s + (accum ? out32[c] : 0.f);
    if (out16) out16[c] = (__bf16)(s + (accum ? (float)out16[c] : 0.f));
}

// tmp must hold RN_COLRED_S * C floats.  accum: add into the outputs (gradient accumulation).
static inline void rn_colreduce(const float* in, int R, int C, float* tmp, float* out32, __bf16* out16,
                                hipStream_t st, int accum = 0) {
    int S = R < RN_COLRED_S ? (R > 0 ? R : 1) : RN_COLRED_S;
    dim3 g((C + 63) / 64, S);
    rn_colred1_k<<<g, 256, 0, st>>>(in, R, C, tmp);
    rn_colred2_k<<<(C + 255) / 256, 256, 0, st>>>(tmp, S, C, out32, out16, accum);
}

}  // namespace
