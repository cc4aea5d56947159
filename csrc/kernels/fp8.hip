// FP8 (OCP e4m3fn — gfx950's format, not the MI300 fnuz variant) support — N3.
//
// * amax / quantise kernels with per-tensor "current" scaling: scale = amax/448,
//   the quantised tensor q satisfies x ≈ q · scale; amax is reduced on device
//   (block max → one atomicMax per block on the float bits, non-negative so
//   integer order == float order); the quantise kernel derives the scale from
//   the device amax itself, so the whole sequence is graph-capturable.
// * the GEMM runs on v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales:
//   2x the bf16 MFMA rate per clock (MI355X_MICROARCH.md §Matrix cores), with the
//   product of the two tensor scales applied as the epilogue alpha.
#include <algorithm>
#include <cstdlib>

#include "gemm_impl.h"

namespace {

constexpr float E4M3_MAX = 448.f;

// Every per-tensor scale is rounded UP to a power of two (never more clipping than the exact scale:
// q = x / s stays within the format's range), so that a scale is an exact E8M0 exponent: the
// one-wave-per-SIMD GEMM (gemm_w1.h) feeds the two tensors' exponents to the scaled MFMA's block-
// scale operands instead of multiplying every output by sa·sb (the same bits as the multiply: a
// product of powers of two is exact).
__device__ inline float pow2_ceil(float s) {
    if (!(s > 0.f)) return 1.f;
    uint32_t u = __float_as_uint(s);
    const uint32_t e = u & 0x7F800000u;
    if (e == 0x7F800000u) return s;  // inf / nan pass through
    u = (u & 0x007FFFFFu) ? e + 0x00800000u : e;
    return __uint_as_float(u ? u : 0x00800000u);  // (subnormal: the smallest normal)
}

__global__ void __launch_bounds__(256) amax_k(const bf16* __restrict__ x, long n, float* __restrict__ state) {
    __shared__ float sm[16];
    float m = 0.f;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n / 8; i += (long)gridDim.x * 256) {
        float f[8];
        load8(x + i * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(f[j]));
    }
    for (long i = (n / 8) * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        m = fmaxf(m, fabsf(bf2f(x[i])));
    m = block_max(m, sm);
    if (threadIdx.x == 0) atomicMax(reinterpret_cast<int*>(state + 1), __float_as_int(m));
}

// state: [scale, amax, ...]; writes scale = amax/448 (1 if amax == 0) and q = x/scale as e4m3
__global__ void __launch_bounds__(256) quant_k(const bf16* __restrict__ x, long n, uint8_t* __restrict__ q,
                                               float* __restrict__ state) {
    const float amax = state[1];
    const float scale = amax > 0.f ? pow2_ceil(amax / E4M3_MAX) : 1.f;
    const float inv = 1.f / scale;
    if (blockIdx.x == 0 && threadIdx.x == 0) state[0] = scale;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n / 8; i += (long)gridDim.x * 256) {
        float f[8];
        load8(x + i * 8, f);
        int w0 = 0, w1 = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(f[j] * inv, -E4M3_MAX), E4M3_MAX);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], w0, false);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w0, true);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], w1, false);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], w1, true);
        *reinterpret_cast<int2*>(q + i * 8) = make_int2(w0, w1);
    }
    for (long i = (n / 8) * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const float f = fminf(fmaxf(bf2f(x[i]) * inv, -E4M3_MAX), E4M3_MAX);
        q[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(f, 0.f, 0, false) & 0xFF);
    }
}

// Delayed scaling (one pass over x): the scale comes from the amax recorded by the PREVIOUS
// quantisation of this tensor (x2 headroom), and this pass records the current amax for the
// next one.  state: [0] scale used, [1] amax of the last pass, [2] amax the scale came from.
// delayed-scaling headroom: scale = pow2_ceil(2 · previous amax / max) for the e4m3 (activations,
// weights) and e5m2 (gradients) slots (headroom 4 / 8 measured in round 5: profiles/fp8_headroom_proj_r5x.txt)
static float fp8_hr() { return 2.f; }
static float fp8_ghr() { return 2.f; }
__device__ inline void fp8_roll_k_body(float* __restrict__ state, float hr) {
    const float a = state[1];
    state[2] = a;
    state[0] = a > 0.f ? pow2_ceil(hr * a / E4M3_MAX) : 1.f;
    state[1] = 0.f;
}
__global__ void fp8_roll_k(float* __restrict__ state, float hr) { fp8_roll_k_body(state, hr); }

__global__ void __launch_bounds__(256) quant_delayed_k(const bf16* __restrict__ x, long n, uint8_t* __restrict__ q,
                                                       float* __restrict__ state) {
    __shared__ float sm[16];
    const float inv = 1.f / state[0];
    float m = 0.f;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n / 8; i += (long)gridDim.x * 256) {
        float f[8];
        load8(x + i * 8, f);
        int w0 = 0, w1 = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            m = fmaxf(m, fabsf(f[j]));
            f[j] = fminf(fmaxf(f[j] * inv, -E4M3_MAX), E4M3_MAX);
        }
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], w0, false);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w0, true);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], w1, false);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], w1, true);
        *reinterpret_cast<int2*>(q + i * 8) = make_int2(w0, w1);
    }
    for (long i = (n / 8) * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const float v = bf2f(x[i]);
        m = fmaxf(m, fabsf(v));
        const float f = fminf(fmaxf(v * inv, -E4M3_MAX), E4M3_MAX);
        q[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(f, 0.f, 0, false) & 0xFF);
    }
    m = block_max(m, sm);
    if (threadIdx.x == 0) atomicMax(reinterpret_cast<int*>(state + 1), __float_as_int(m));
}

// Gradient operands of the fp8 weight-gradient GEMM: OCP e5m2 ("bf8": 2 more exponent bits, the
// range gradients need) with the same one-pass delayed scaling (scale from the previous pass's amax,
// x2 headroom, this pass records the new amax).  state as quant_delayed_k; the roll is folded in
// (block 0 rolls nothing: the host launches fp8_roll_fmt_k first).
constexpr float E5M2_MAX = 57344.f;
__global__ void fp8_roll_bf8_k(float* __restrict__ state, float hr) {
    const float a = state[1];
    state[2] = a;
    state[0] = a > 0.f ? pow2_ceil(hr * a / E5M2_MAX) : 1.f;
    state[1] = 0.f;
}
__global__ void __launch_bounds__(256) quant_delayed_bf8_k(const bf16* __restrict__ x, long n, uint8_t* __restrict__ q,
                                                           float* __restrict__ state) {
    __shared__ float sm[16];
    const float inv = 1.f / state[0];
    float m = 0.f;
    auto one = [&](long i, float* f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            m = fmaxf(m, fabsf(f[j]));
            f[j] = fminf(fmaxf(f[j] * inv, -E5M2_MAX), E5M2_MAX);
        }
        int w0 = 0, w1 = 0;
        w0 = __builtin_amdgcn_cvt_pk_bf8_f32(f[0], f[1], w0, false);
        w0 = __builtin_amdgcn_cvt_pk_bf8_f32(f[2], f[3], w0, true);
        w1 = __builtin_amdgcn_cvt_pk_bf8_f32(f[4], f[5], w1, false);
        w1 = __builtin_amdgcn_cvt_pk_bf8_f32(f[6], f[7], w1, true);
        *reinterpret_cast<int2*>(q + i * 8) = make_int2(w0, w1);
    };
    // 4 chunks in flight per thread (one at a time left a grid-capped launch latency-bound)
    const long S = (long)gridDim.x * 256, n8 = n / 8;
    long i = blockIdx.x * 256L + threadIdx.x;
    for (; i + 3 * S < n8; i += 4 * S) {
        float f[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) load8(x + (i + u * S) * 8, f[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) one(i + u * S, f[u]);
    }
    for (; i < n8; i += S) {
        float f[8];
        load8(x + i * 8, f);
        one(i, f);
    }
    for (long i = (n / 8) * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const float v = bf2f(x[i]);
        m = fmaxf(m, fabsf(v));
        const float f = fminf(fmaxf(v * inv, -E5M2_MAX), E5M2_MAX);
        q[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_bf8_f32(f, 0.f, 0, false) & 0xFF);
    }
    m = block_max(m, sm);
    if (threadIdx.x == 0) atomicMax(reinterpret_cast<int*>(state + 1), __float_as_int(m));
}
// first (current-scaling) pass of a gradient slot: amax, then scale = amax / E5M2_MAX
__global__ void __launch_bounds__(256) quant_bf8_k(const bf16* __restrict__ x, long n, uint8_t* __restrict__ q,
                                                   float* __restrict__ state) {
    const float amax = state[1];
    const float scale = amax > 0.f ? pow2_ceil(amax / E5M2_MAX) : 1.f;
    const float inv = 1.f / scale;
    if (blockIdx.x == 0 && threadIdx.x == 0) state[0] = scale;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n / 8; i += (long)gridDim.x * 256) {
        float f[8];
        load8(x + i * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(f[j] * inv, -E5M2_MAX), E5M2_MAX);
        int w0 = 0, w1 = 0;
        w0 = __builtin_amdgcn_cvt_pk_bf8_f32(f[0], f[1], w0, false);
        w0 = __builtin_amdgcn_cvt_pk_bf8_f32(f[2], f[3], w0, true);
        w1 = __builtin_amdgcn_cvt_pk_bf8_f32(f[4], f[5], w1, false);
        w1 = __builtin_amdgcn_cvt_pk_bf8_f32(f[6], f[7], w1, true);
        *reinterpret_cast<int2*>(q + i * 8) = make_int2(w0, w1);
    }
    for (long i = (n / 8) * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const float f = fminf(fmaxf(bf2f(x[i]) * inv, -E5M2_MAX), E5M2_MAX);
        q[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_bf8_f32(f, 0.f, 0, false) & 0xFF);
    }
}

// The GELU backward of the fp8 MLP fused with the e5m2 quantisation of its result: dH = dU ⊙ gelu'(h)
// (dU = the MLP c_proj's fp8 data gradient, gelu'(h) saved by c_fc's forward epilogue), written ONLY as
// e5m2 for c_fc's fp8 data / weight gradients, plus per-row-group column partial sums of dH (c_fc's
// bias gradient, reduced by rn_colsum_f32).  Thread t owns 16-B column chunk t % (N/8) of rows
// t / (N/8), + G, + 2G, ...  MODE 0: amax of dH only (a slot's first, current-scaling pass); 1: quantise
// with the scale from that amax (as quant_bf8_k); 2: delayed (scale rolled by fp8_roll_bf8_k, this
// pass records the new amax).
template <int MODE, bool FROM_H>
__global__ void __launch_bounds__(256) act_mul_bf8_k(const bf16* __restrict__ du, const bf16* __restrict__ dd, long M,
                                                     int N, uint8_t* __restrict__ q, float* __restrict__ state,
                                                     float* __restrict__ colpart, int G) {
    __shared__ float sm[16];
    const int nc = N / 8;
    const long t = blockIdx.x * 256L + threadIdx.x;
    const bool live = t < (long)G * nc;
    const int c = (int)(t % nc), g = (int)(t / nc);
    float inv = 1.f;
    if constexpr (MODE == 1) {
        const float amax = state[1];
        const float scale = amax > 0.f ? pow2_ceil(amax / E5M2_MAX) : 1.f;
        inv = 1.f / scale;
        if (t == 0) state[0] = scale;
    } else if constexpr (MODE == 2) {
        inv = 1.f / state[0];
    }
    float m = 0.f, cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto one = [&](long off, float* a, const float* b) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float h = a[j] * (FROM_H ? gelu_grad_f(b[j]) : b[j]);
            m = fmaxf(m, fabsf(h));
            cs[j] += h;
            a[j] = fminf(fmaxf(h * inv, -E5M2_MAX), E5M2_MAX);
        }
        if constexpr (MODE != 0) {
            int w0 = 0, w1 = 0;
            w0 = __builtin_amdgcn_cvt_pk_bf8_f32(a[0], a[1], w0, false);
            w0 = __builtin_amdgcn_cvt_pk_bf8_f32(a[2], a[3], w0, true);
            w1 = __builtin_amdgcn_cvt_pk_bf8_f32(a[4], a[5], w1, false);
            w1 = __builtin_amdgcn_cvt_pk_bf8_f32(a[6], a[7], w1, true);
            *reinterpret_cast<int2*>(q + off) = make_int2(w0, w1);
        }
    };
    if (live) {
        // 4 rows per iteration, their 8 loads issued before any math (one row at a time left a
        // thread with a single dependent 16-B pair in flight: 3.7 TB/s)
        long r = g;
        for (; r + 3L * G < M; r += 4L * G) {
            float a[4][8], b[4][8];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                load8(du + (r + u * (long)G) * N + c * 8, a[u]);
                load8(dd + (r + u * (long)G) * N + c * 8, b[u]);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) one((r + u * (long)G) * N + c * 8, a[u], b[u]);
        }
        for (; r < M; r += G) {
            float a[8], b[8];
            load8(du + r * N + c * 8, a);
            load8(dd + r * N + c * 8, b);
            one(r * N + c * 8, a, b);
        }
        if (MODE != 0 && colpart) {
            float4* cp = reinterpret_cast<float4*>(colpart + (long)g * N + c * 8);
            cp[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
            cp[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
        }
    }
    if constexpr (MODE != 1) {
        m = block_max(m, sm);
        if (threadIdx.x == 0) atomicMax(reinterpret_cast<int*>(state + 1), __float_as_int(m));
    }
}

__global__ void dequant_bf8_k(const uint8_t* __restrict__ q, long n, const float* __restrict__ state,
                              bf16* __restrict__ y) {
    const float scale = state[0];
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        y[i] = (bf16)(__builtin_amdgcn_cvt_f32_bf8((int)q[i], 0) * scale);
}

__global__ void dequant_k(const uint8_t* __restrict__ q, long n, const float* __restrict__ state,
                          bf16* __restrict__ y) {
    const float scale = state[0];
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        y[i] = (bf16)(__builtin_amdgcn_cvt_f32_fp8((int)q[i], 0) * scale);
}

// ---- e4m3 weight cache (ops/fp8.py Fp8WeightCache): every fp8 weight of the model re-quantised
// right after the optimizer step, in two launches for the whole model.  segs: int64 [nseg][4] =
// (element offset in the flat bf16 parameter buffer, numel, byte offset in the e4m3 buffer,
// address of the weight's Fp8State slot).  Delayed scaling as fp8_roll_k / quant_delayed_k.
__global__ void fp8_roll_many_k(const long* __restrict__ segs, int nseg, float hr) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nseg) fp8_roll_k_body(reinterpret_cast<float*>(segs[i * 4 + 3]), hr);
}

__global__ void __launch_bounds__(256) fp8_quant_many_k(const bf16* __restrict__ flat, const long* __restrict__ segs,
                                                        uint8_t* __restrict__ qbuf) {
    __shared__ float sm[16];
    const long* sg = segs + blockIdx.y * 4;
    const bf16* x = flat + sg[0];
    const long n = sg[1];
    uint8_t* q = qbuf + sg[2];
    float* state = reinterpret_cast<float*>(sg[3]);
    const float inv = 1.f / state[0];
    float m = 0.f;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n / 8; i += (long)gridDim.x * 256) {
        float f[8];
        load8(x + i * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            m = fmaxf(m, fabsf(f[j]));
            f[j] = fminf(fmaxf(f[j] * inv, -E4M3_MAX), E4M3_MAX);
        }
        int w0 = 0, w1 = 0;
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], w0, false);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w0, true);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], w1, false);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], w1, true);
        *reinterpret_cast<int2*>(q + i * 8) = make_int2(w0, w1);
    }
    for (long i = (n / 8) * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const float v = bf2f(x[i]);
        m = fmaxf(m, fabsf(v));
        const float f = fminf(fmaxf(v * inv, -E4M3_MAX), E4M3_MAX);
        q[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(f, 0.f, 0, false) & 0xFF);
    }
    m = block_max(m, sm);
    if (threadIdx.x == 0) atomicMax(reinterpret_cast<int*>(state + 1), __float_as_int(m));
}

// alpha = sa * sb on device
__global__ void scale_mul_k(const float* __restrict__ sa, const float* __restrict__ sb, float* __restrict__ alpha,
                            const float* __restrict__ post = nullptr) {
    alpha[0] = sa[0] * sb[0] * (post ? post[0] : 1.f);
}

inline int gridn(long n) {
    long g = (n + 255) / 256;
    return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

// REPLICANN_FP8_GEMM: unset = by shape, 0 = one-tile-per-block 256x192, 9 = persistent 256x256,
// 11 = one-wave-per-SIMD persistent 256x256 (gemm_w1.h)
int fp8_gemm_kernel() {
    const char* e = std::getenv("REPLICANN_FP8_GEMM");
    if (!e || !e[0]) return -1;  // by shape
    const int v = std::atoi(e);
    return v == 0 ? 0 : (v == 11 ? 11 : 9);
}

}  // namespace

void rn_gemm_launch_pk_fp8(rn_gemm_detail::GemmArgs& a, int act, hipStream_t st);
int rn_gemm_launch_w1(rn_gemm_detail::GemmArgs& a, int fp8, int act, hipStream_t st, bool bmn);
int rn_gemm_launch_w1_wgrad(rn_gemm_detail::GemmArgs& a, int fp8, int split, hipStream_t st);
void rn_gemm_launch_pk_fp8_wgrad(rn_gemm_detail::GemmArgs& a, int a_bf8, hipStream_t st);
void rn_gemm_launch_pk_fp8_dgrad(rn_gemm_detail::GemmArgs& a, int a_bf8, hipStream_t st);

extern "C" {

// state must hold >= 2 floats; it is (re)initialised here (memset node + 2 kernels).
void rn_fp8_quantize(const void* x, long n, void* q, float* state, hipStream_t st) {
    // all 4 slot floats: a first (current-scaling) quantisation is copied whole into a training slot,
    // whose [2] / [3] must not carry uninitialised bytes (run-to-run bitwise state_dicts)
    (void)hipMemsetAsync(state, 0, 4 * sizeof(float), st);
    amax_k<<<gridn(n / 8 + 1), 256, 0, st>>>((const bf16*)x, n, state);
    quant_k<<<gridn(n / 8 + 1), 256, 0, st>>>((const bf16*)x, n, (uint8_t*)q, state);
}

// One-pass delayed-scaling quantisation (state as fp8_roll_k / quant_delayed_k); graph-capturable.
void rn_fp8_quantize_delayed(const void* x, long n, void* q, float* state, hipStream_t st) {
    fp8_roll_k<<<1, 1, 0, st>>>(state, fp8_hr());
    quant_delayed_k<<<gridn(n / 8 + 1), 256, 0, st>>>((const bf16*)x, n, (uint8_t*)q, state);
}

// Re-quantise every cached fp8 weight (segs: device int64 [nseg][4], see fp8_quant_many_k).
// roll = 0: keep the scales already in the slots (rebuilding the cache after a checkpoint load: the
// bytes and the recorded amax are then exactly those of the saving run's last refresh).
void rn_fp8_quant_many(const void* flat, const long* segs, int nseg, long max_n, void* qbuf, int roll,
                       hipStream_t st) {
    if (nseg <= 0) return;
    if (roll) fp8_roll_many_k<<<(nseg + 255) / 256, 256, 0, st>>>(segs, nseg, fp8_hr());
    long per = (max_n / 8 + 255) / 256;  // blocks that cover the largest weight in one sweep
    const int bx = (int)(per < 1 ? 1 : (per > 64 ? 64 : per));
    fp8_quant_many_k<<<dim3(bx, nseg), 256, 0, st>>>((const bf16*)flat, segs, (uint8_t*)qbuf);
}

// The delayed-scaling roll alone (for producers that quantise inside their own kernel).
void rn_fp8_roll(float* state, hipStream_t st) { fp8_roll_k<<<1, 1, 0, st>>>(state, fp8_hr()); }

void rn_fp8_dequantize(const void* q, long n, const float* state, void* y, hipStream_t st) {
    dequant_k<<<gridn(n), 256, 0, st>>>((const uint8_t*)q, n, state, (bf16*)y);
}

// e5m2 gradient quantisation: delayed (roll + one pass) or, for a slot without a scale yet,
// current scaling (memset + amax + quantise); state as rn_fp8_quantize_delayed
void rn_bf8_quantize(const void* x, long n, void* q, float* state, int delayed, hipStream_t st) {
    if (delayed) {
        fp8_roll_bf8_k<<<1, 1, 0, st>>>(state, fp8_ghr());
        quant_delayed_bf8_k<<<gridn(n / 8 + 1), 256, 0, st>>>((const bf16*)x, n, (uint8_t*)q, state);
        return;
    }
    (void)hipMemsetAsync(state, 0, 2 * sizeof(float), st);
    amax_k<<<gridn(n / 8 + 1), 256, 0, st>>>((const bf16*)x, n, state);
    quant_bf8_k<<<gridn(n / 8 + 1), 256, 0, st>>>((const bf16*)x, n, (uint8_t*)q, state);
}
void rn_fp8_roll_bf8(float* state, hipStream_t st) { fp8_roll_bf8_k<<<1, 1, 0, st>>>(state, fp8_ghr()); }

// dH = dU ⊙ d in e5m2 (+ column partials [G][N] of dH when colpart): see act_mul_bf8_k.  N % 8 == 0.
int rn_act_mul_bf8_groups(long M, int N) {
    const long nc = N / 8;
    long g = (262144 + nc - 1) / nc;  // ~256 k threads, 4 rows in flight each
    if (g > M) g = M;
    return (int)(g < 1 ? 1 : g);
}
extern "C++" template <bool FROM_H>
static void act_mul_bf8_run(const void* du, const void* d, long M, int N, void* q, float* state, int delayed,
                            float* colpart, hipStream_t st) {
    const int G = rn_act_mul_bf8_groups(M, N);
    const long threads = (long)G * (N / 8);
    const int blocks = (int)((threads + 255) / 256);
    const bf16 *a = (const bf16*)du, *b = (const bf16*)d;
    if (delayed) {
        fp8_roll_bf8_k<<<1, 1, 0, st>>>(state, fp8_ghr());
        act_mul_bf8_k<2, FROM_H><<<blocks, 256, 0, st>>>(a, b, M, N, (uint8_t*)q, state, colpart, G);
        return;
    }
    (void)hipMemsetAsync(state, 0, 2 * sizeof(float), st);
    act_mul_bf8_k<0, FROM_H><<<blocks, 256, 0, st>>>(a, b, M, N, (uint8_t*)q, state, nullptr, G);
    act_mul_bf8_k<1, FROM_H><<<blocks, 256, 0, st>>>(a, b, M, N, (uint8_t*)q, state, colpart, G);
}
// from_h: d holds the pre-activation h and the kernel takes gelu'(h) itself (the fp8 MLP whose forward kept
// h instead of gelu'(h), rn_gelu_q8)
void rn_act_mul_bf8(const void* du, const void* d, long M, int N, void* q, float* state, int delayed, float* colpart,
                    int from_h, hipStream_t st) {
    if (from_h) act_mul_bf8_run<true>(du, d, M, N, q, state, delayed, colpart, st);
    else act_mul_bf8_run<false>(du, d, M, N, q, state, delayed, colpart, st);
}

// The fp8 MLP's activation as its own pass: q8 = e4m3(bf16(gelu(h))) with the consumer's delayed scale
// (rolled here; this pass records amax(|gelu(h)|)), from the bf16 pre-activation h the c_fc GEMM wrote on the
// one-wave-per-SIMD kernel.  The MLP then keeps h for the backward (gelu'(h) is re-derived inside
// act_mul_bf8_k) and never writes gelu(h) or gelu'(h) in bf16: 2 B/element less than the fused-epilogue
// GEMM's three outputs.
__global__ void __launch_bounds__(256) gelu_q8_k(const bf16* __restrict__ h, long n, uint8_t* __restrict__ q,
                                                 float* __restrict__ state) {
    __shared__ float sm[16];
    const float inv = 1.f / state[0];
    float m = 0.f;
    auto one = [&](long i, float* f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float u = (float)(bf16)gelu_f(f[j]);
            m = fmaxf(m, fabsf(u));
            f[j] = fminf(fmaxf(u * inv, -E4M3_MAX), E4M3_MAX);
        }
        int w0 = 0, w1 = 0;
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], w0, false);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w0, true);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], w1, false);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], w1, true);
        *reinterpret_cast<int2*>(q + i * 8) = make_int2(w0, w1);
    };
    // one chunk per iteration over a large grid (the 4-chunk unroll measured slower here: 225 vs 179 us)
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n / 8; i += (long)gridDim.x * 256) {
        float f[8];
        load8(h + i * 8, f);
        one(i, f);
    }
    m = block_max(m, sm);
    if (threadIdx.x == 0) atomicMax(reinterpret_cast<int*>(state + 1), __float_as_int(m));
}
void rn_gelu_q8(const void* h, long n, void* q, float* state, hipStream_t st) {
    fp8_roll_k<<<1, 1, 0, st>>>(state, fp8_hr());
    const long blocks = (n / 8 + 255) / 256;
    gelu_q8_k<<<(int)std::min<long>(std::max<long>(blocks, 1), 8192), 256, 0, st>>>((const bf16*)h, n, (uint8_t*)q, state);
}

void rn_bf8_dequantize(const void* q, long n, const float* state, void* y, hipStream_t st) {
    dequant_bf8_k<<<gridn(n), 256, 0, st>>>((const uint8_t*)q, n, state, (bf16*)y);
}

// C[M,N] (bf16) = act(sa·sb · A8[M,K] · B8[N,K]ᵀ + bias) + res ; K % 16 == 0, lda/ldb in bytes % 16 == 0
// q8 / q8st (optional, activation-forward with a saved pre-activation only): also write the output
// in e4m3 for the next fp8 GEMM (q8st rolled here; the tile kernel's epilogue quantises and records amax)
int rn_gemm_fp8(const void* A8, const void* B8, void* C, const void* bias, const void* res, void* pre,
                const float* sa, const float* sb, float* alpha_ws, int M, int N, int K, long lda, long ldb, long ldc,
                int act, hipStream_t st, void* q8, float* q8st) {
    if (K % 16 || lda % 16 || ldb % 16) return -1;
    if (q8 && (!pre || (act != ACT_GELU && act != ACT_GELU_D && act != ACT_RELU) || N % 8 || ldc % 8)) return -2;
    // the one-wave-per-SIMD persistent kernel (gemm_w1.h, default; REPLICANN_FP8_GEMM=11 forces it where it
    // applies, 0 / 9 select the older kernels): plain / bias / residual epilogues, the power-of-two tensor
    // scales riding the scaled MFMA (no alpha pass).  profiles/w1_ab_r5a.txt: 1.67-2.30 PF/s on the
    // GPT-2-medium shapes against 1.39-1.94 for the best older kernel
    const int kern = fp8_gemm_kernel();
    if ((kern == 11 || kern < 0) && !q8 && act == ACT_NONE) {
        rn_gemm_detail::GemmArgs w = {};
        w.A = (const bf16*)A8; w.B = (const bf16*)B8; w.C = C; w.bias = (const bf16*)bias; w.res = (const bf16*)res;
        w.M = M; w.N = N; w.K = K; w.lda = lda; w.ldb = ldb; w.ldc = ldc; w.sa = sa; w.sb = sb;
        if (rn_gemm_launch_w1(w, 1, ACT_NONE, st, false) == 0) return 0;
    }
    scale_mul_k<<<1, 1, 0, st>>>(sa, sb, alpha_ws);
    if (q8) fp8_roll_k<<<1, 1, 0, st>>>(q8st, fp8_hr());
    rn_gemm_detail::GemmArgs a = {};
    a.A = (const bf16*)A8; a.B = (const bf16*)B8; a.C = C; a.bias = (const bf16*)bias; a.res = (const bf16*)res;
    a.pre = (bf16*)pre; a.ws = nullptr; a.alpha = alpha_ws;
    a.M = M; a.N = N; a.K = K / 2; a.lda = lda / 2; a.ldb = ldb / 2; a.ldc = ldc;
    a.split = 1; a.k_per_split = ((K / 2) + 63) / 64 * 64; a.out_f32 = 0; a.accumulate = 0;
    a.q8 = (uint8_t*)q8; a.q8st = q8st;
    using namespace rn_gemm_detail;
    // persistent 256x256 half-tile stream (gemm_pk<.., FP8>): its epilogue stores 8 contiguous
    // columns per lane, so it takes N % 8 == 0 and ldc % 8 == 0 only.  Measured on the GPT-2-medium
    // b64 shapes (profiles/fp8_gemm_ab_r2r.txt): it wins at K = 4096 (1.94 vs 1.85 PF/s) and loses
    // at K = 1024 (1.32 vs 1.59 PF/s: 8 K-tiles per output tile, the per-tile epilogue dominates),
    // so by default it takes K >= 2048 only; REPLICANN_FP8_GEMM=9 forces it, =0 never.
    if (!q8 && N % 8 == 0 && ldc % 8 == 0 && (kern == 9 || (kern < 0 && K >= 2048))) {
        a.tiles_m = (M + 255) / 256;
        a.tiles_n = (N + 255) / 256;
        rn_gemm_launch_pk_fp8(a, act, st);
        return 0;
    }
    if (act == ACT_GELU) launch_fp8_t<256, 192, 2, 4, ACT_GELU>(a, st);
    else if (act == ACT_GELU_D) launch_fp8_t<256, 192, 2, 4, ACT_GELU_D>(a, st);
    else if (act == ACT_RELU) launch_fp8_t<256, 192, 2, 4, ACT_RELU>(a, st);
    else launch_fp8_t<256, 192, 2, 4, ACT_NONE>(a, st);
    return 0;
}

// dW[M,N] (+)= sa·sb · Σ_k A8[k][m] · B8[k][n]  — the fp8 weight gradient with both operands as the
// forward / backward produced them (token-major: A8 = dY [K][lda] e5m2 or e4m3, B8 = X [K][ldb]
// e4m3; lda / ldb in bytes), K = tokens.  C: bf16 (out_f32 = 0) or fp32, accumulated into when
// `accumulate`.  ws: split · M · N floats (rn_gemm_fp8_wgrad_ws).  Requirements: M, N, lda, ldb
// multiples of 16, K a multiple of 128.
long rn_gemm_fp8_wgrad_split(int M, int N, int K) {
    // K slices of whole 128-deep K-tiles, an exact division of the K-tiles (the one-wave-per-SIMD kernel's
    // split-K walk) with >= 2 per slice: the divisor with the shortest makespan over 256 CUs, each item
    // costed as its K-tiles + 2 for its epilogue / pipeline fill (ties: fewer slabs)
    const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
    const long kt = K / 128;
    long best = 1, best_cost = -1;
    for (long d = 1; d <= kt / 2; ++d) {
        if (kt % d) continue;
        const long rounds = (tiles * d + 255) / 256;
        const long cost = rounds * (kt / d + 2);
        if (best_cost < 0 || cost < best_cost) {
            best = d;
            best_cost = cost;
        }
    }
    return best;
}
long rn_gemm_fp8_wgrad_ws(int M, int N, int K) { return rn_gemm_fp8_wgrad_split(M, N, K) * (long)M * N; }
int rn_gemm_fp8_wgrad(const void* A8, const void* B8, void* C, const float* sa, const float* sb, float* alpha_ws,
                      float* ws, int M, int N, int K, long lda, long ldb, long ldc, int accumulate, int out_f32,
                      int a_bf8, hipStream_t st, const float* post) {
    if (M % 16 || N % 16 || lda % 16 || ldb % 16 || K % 128 || M <= 0 || N <= 0) return -1;
    const int split = (int)rn_gemm_fp8_wgrad_split(M, N, K);
    const int kern = fp8_gemm_kernel();
    if (kern == 11 || kern < 0) {
        // the one-wave-per-SIMD kernel: both operands MN-contiguous (tr_b8 reads), split-K fp32 slabs, the
        // power-of-two scales on the scaled MFMA; then the fixed-order slab sum
        rn_gemm_detail::GemmArgs w = {};
        w.A = (const bf16*)A8; w.B = (const bf16*)B8; w.C = C; w.ws = ws;
        w.M = M; w.N = N; w.K = K; w.lda = lda; w.ldb = ldb; w.ldc = ldc; w.sa = sa; w.sb = sb;
        w.out_f32 = out_f32; w.accumulate = accumulate; w.reduce_alpha = post;
        if (rn_gemm_launch_w1_wgrad(w, a_bf8 ? 2 : 1, split, st) == 0) return 0;
    }
    scale_mul_k<<<1, 1, 0, st>>>(sa, sb, alpha_ws, post);
    const int kt = K / 128, per = (kt + split - 1) / split;
    rn_gemm_detail::GemmArgs a = {};
    a.A = (const bf16*)A8; a.B = (const bf16*)B8; a.C = C; a.ws = ws; a.alpha = alpha_ws;
    a.M = M; a.N = N; a.K = K / 2; a.lda = lda; a.ldb = ldb; a.ldc = ldc;  // MN-contiguous fp8: ld in bytes
    a.tiles_m = (M + 255) / 256;
    a.tiles_n = (N + 255) / 256;
    a.split = split; a.k_per_split = per * 64; a.out_f32 = out_f32; a.accumulate = accumulate;
    a.slab_step = 1;
    rn_gemm_launch_pk_fp8_wgrad(a, a_bf8, st);
    return 0;
}

// C[M,N] (bf16) = sa·sb · A8[M][K] · B8[K][N]: the fp8 data gradient dX = dY·W with dY (A8, e5m2 if
// a_bf8) K-contiguous and the weight W [out = K][in = N] as stored (the forward's e4m3 weight copy),
// read transposed.  K, N, lda, ldb, ldc multiples of 16 (bytes for the fp8 operands).
// post (optional device scalar): one more output multiplier (the fp8 LM head's g / n)
int rn_gemm_fp8_dgrad(const void* A8, const void* B8, void* C, const float* sa, const float* sb, float* alpha_ws,
                      int M, int N, int K, long lda, long ldb, long ldc, int a_bf8, hipStream_t st, const float* post) {
    if (K % 16 || N % 16 || lda % 16 || ldb % 16 || ldc % 8 || M <= 0) return -1;
    const int kern = fp8_gemm_kernel();
    if ((kern == 11 || kern < 0) && K % 128 == 0 && K >= 256) {
        // the one-wave-per-SIMD kernel with its fp8 MN-contiguous B path (tr_b8 reads of W as stored; the
        // power-of-two scales ride the scaled MFMA, no alpha pass)
        rn_gemm_detail::GemmArgs w = {};
        w.A = (const bf16*)A8; w.B = (const bf16*)B8; w.C = C;
        w.M = M; w.N = N; w.K = K; w.lda = lda; w.ldb = ldb; w.ldc = ldc; w.sa = sa; w.sb = sb; w.alpha = post;
        if (rn_gemm_launch_w1(w, a_bf8 ? 2 : 1, ACT_NONE, st, true) == 0) return 0;
    }
    scale_mul_k<<<1, 1, 0, st>>>(sa, sb, alpha_ws, post);
    rn_gemm_detail::GemmArgs a = {};
    a.A = (const bf16*)A8; a.B = (const bf16*)B8; a.C = C; a.alpha = alpha_ws;
    a.M = M; a.N = N; a.K = K / 2;
    a.lda = lda / 2;  // K-contiguous fp8: bf16-pair units
    a.ldb = ldb;      // MN-contiguous fp8: bytes
    a.ldc = ldc;
    a.tiles_m = (M + 255) / 256;
    a.tiles_n = (N + 255) / 256;
    a.split = 1; a.k_per_split = ((K / 2) + 63) / 64 * 64; a.out_f32 = 0; a.accumulate = 0;
    rn_gemm_launch_pk_fp8_dgrad(a, a_bf8, st);
    return 0;
}

}  // extern "C"
