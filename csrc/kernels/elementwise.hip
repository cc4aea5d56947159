// Elementwise kernels: activations, dropout, fused activation-backward + bias-grad,
// add(+relu).  Memory-bound: every kernel moves bf16 as 16-byte vectors
// (8 elements / lane), grid-strides over at most 256 CUs x 8 blocks.
#include "common.h"

namespace {

constexpr int TPB = 256;

inline int ew_grid(long n8) {
    long g = (n8 + TPB - 1) / TPB;
    return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

template <int ACT>
__global__ void __launch_bounds__(TPB) act_fwd_k(const bf16* __restrict__ x, bf16* __restrict__ y, long n) {
    long n8 = n / 8;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n8; i += (long)gridDim.x * TPB) {
        float f[8];
        load8(x + i * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = act_f<ACT>(f[j]);
        store8(y + i * 8, f);
    }
    for (long i = n8 * 8 + blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB)
        y[i] = f2bf(act_f<ACT>(bf2f(x[i])));
}

template <int ACT>
__global__ void __launch_bounds__(TPB) act_bwd_k(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                 bf16* __restrict__ dx, long n) {
    long n8 = n / 8;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n8; i += (long)gridDim.x * TPB) {
        float g[8], f[8];
        load8(dy + i * 8, g);
        load8(x + i * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] *= act_grad_f<ACT>(f[j]);
        store8(dx + i * 8, g);
    }
    for (long i = n8 * 8 + blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB)
        dx[i] = f2bf(bf2f(dy[i]) * act_grad_f<ACT>(bf2f(x[i])));
}

__global__ void __launch_bounds__(TPB) dropout_k(const bf16* __restrict__ x, bf16* __restrict__ y, long n,
                                                 float p, uint64_t seed, const uint64_t* __restrict__ seed_ptr) {
    if (seed_ptr) seed = *seed_ptr;  // device-drawn seed (graph-capturable dropout)
    const float keep = 1.f / (1.f - p);
    long n8 = n / 8;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n8; i += (long)gridDim.x * TPB) {
        float f[8];
        load8(x + i * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = hash_uniform(seed, i * 8 + j) >= p ? f[j] * keep : 0.f;
        store8(y + i * 8, f);
    }
    for (long i = n8 * 8 + blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB)
        y[i] = f2bf(hash_uniform(seed, i) >= p ? bf2f(x[i]) * keep : 0.f);
}

// out = relu?(a + b)
template <bool RELU>
__global__ void __launch_bounds__(TPB) add_k(const bf16* __restrict__ a, const bf16* __restrict__ b,
                                             bf16* __restrict__ y, long n) {
    long n8 = n / 8;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n8; i += (long)gridDim.x * TPB) {
        float f[8], g[8];
        load8(a + i * 8, f);
        load8(b + i * 8, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = RELU ? fmaxf(f[j] + g[j], 0.f) : f[j] + g[j];
        store8(y + i * 8, f);
    }
    for (long i = n8 * 8 + blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB) {
        float v = bf2f(a[i]) + bf2f(b[i]);
        y[i] = f2bf(RELU ? fmaxf(v, 0.f) : v);
    }
}

// dH = dY * act'(H) (written only when ACT != NONE) and partial column sums of dH.
// Grid: (col_blocks of 512 columns, row_splits).  Each lane owns 8 columns; the
// block's 4 waves split the rows, partials combine through LDS and land in
// part[row_split][N] (fp32), summed in fixed order by colsum_finish_k.
template <int ACT, bool WANT_BIAS>
__global__ void __launch_bounds__(TPB) bias_act_grad_k(const bf16* __restrict__ dy, const bf16* __restrict__ h,
                                                       bf16* __restrict__ dh, float* __restrict__ part,
                                                       int M, int N, int rows_per_split) {
    __shared__ float red[4][512];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int col = blockIdx.x * 512 + lane * 8;
    const int r0 = blockIdx.y * rows_per_split;
    const int r1 = min(M, r0 + rows_per_split);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bool vec = (N % 8 == 0);
    if (vec && col < N) {
        for (int r = r0 + wid; r < r1; r += 4) {
            float g[8];
            long off = (long)r * N + col;
            load8(dy + off, g);
            if constexpr (ACT != ACT_NONE) {
                float f[8];
                load8(h + off, f);
#pragma unroll
                for (int j = 0; j < 8; ++j) g[j] *= act_grad_f<ACT>(f[j]);
                store8(dh + off, g);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] += g[j];
        }
    } else if (!vec) {
        for (int r = r0 + wid; r < r1; r += 4) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                int c = col + j;
                if (c < N) {
                    long off = (long)r * N + c;
                    float g = bf2f(dy[off]);
                    if constexpr (ACT != ACT_NONE) {
                        g *= act_grad_f<ACT>(bf2f(h[off]));
                        dh[off] = f2bf(g);
                    }
                    acc[j] += g;
                }
            }
        }
    }
    if constexpr (WANT_BIAS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wid][lane * 8 + j] = acc[j];
        __syncthreads();
        for (int c = threadIdx.x; c < 512; c += TPB) {
            int gc = blockIdx.x * 512 + c;
            if (gc < N) part[(long)blockIdx.y * N + gc] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
        }
    }
}

}  // namespace

// fp32 -> bf16 (round to nearest even), 8 elements per lane: the narrowing step of the data-parallel
// reducer's reduce-scatter (fp32) -> all-gather (bf16) path, run on the communicator's stream
__global__ void __launch_bounds__(256) cast_f32_bf16_k(const float* __restrict__ in, bf16* __restrict__ out, long n) {
    const long n8 = n / 8;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
        const float4 a = reinterpret_cast<const float4*>(in)[2 * i], b = reinterpret_cast<const float4*>(in)[2 * i + 1];
        const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        store8(out + i * 8, f);
    }
    for (long i = n8 * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) out[i] = (bf16)in[i];
}

extern "C" {

void rn_cast_f32_bf16(const float* in, void* out, long n, hipStream_t st) {
    if (n <= 0) return;
    long g = (n / 8 + 255) / 256;
    g = g < 1 ? 1 : (g > 2048 ? 2048 : g);
    cast_f32_bf16_k<<<(int)g, 256, 0, st>>>(in, (bf16*)out, n);
}

void rn_act_fwd(const void* x, void* y, long n, int kind, hipStream_t st) {
    int g = ew_grid(n / 8 + 1);
    if (kind == ACT_GELU) act_fwd_k<ACT_GELU><<<g, TPB, 0, st>>>((const bf16*)x, (bf16*)y, n);
    else act_fwd_k<ACT_RELU><<<g, TPB, 0, st>>>((const bf16*)x, (bf16*)y, n);
}

void rn_act_bwd(const void* dy, const void* x, void* dx, long n, int kind, hipStream_t st) {
    int g = ew_grid(n / 8 + 1);
    if (kind == ACT_GELU) act_bwd_k<ACT_GELU><<<g, TPB, 0, st>>>((const bf16*)dy, (const bf16*)x, (bf16*)dx, n);
    else act_bwd_k<ACT_RELU><<<g, TPB, 0, st>>>((const bf16*)dy, (const bf16*)x, (bf16*)dx, n);
}

void rn_dropout(const void* x, void* y, long n, float p, uint64_t seed, const uint64_t* seed_ptr, hipStream_t st) {
    dropout_k<<<ew_grid(n / 8 + 1), TPB, 0, st>>>((const bf16*)x, (bf16*)y, n, p, seed, seed_ptr);
}

// Device RNG stream for dropout seeds (ops/rng.py): out[0] = splitmix64(state[0]); state[0] += γ.
// One thread; stream-ordered, so a captured hipGraph draws a fresh seed at every replay.
__global__ void rng_next_k(uint64_t* __restrict__ state, uint64_t* __restrict__ out) {
    uint64_t z = state[0] + 0x9E3779B97F4A7C15ull;
    state[0] = z;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    out[0] = z ^ (z >> 31);
}

void rn_rng_next(void* state, void* out, hipStream_t st) {
    rng_next_k<<<1, 1, 0, st>>>((uint64_t*)state, (uint64_t*)out);
}

void rn_add(const void* a, const void* b, void* y, long n, int relu, hipStream_t st) {
    int g = ew_grid(n / 8 + 1);
    if (relu) add_k<true><<<g, TPB, 0, st>>>((const bf16*)a, (const bf16*)b, (bf16*)y, n);
    else add_k<false><<<g, TPB, 0, st>>>((const bf16*)a, (const bf16*)b, (bf16*)y, n);
}

// part: workspace of >= (splits + RN_COLRED_S) * N floats.  db (fp32) / db16 (bf16) written if want_bias.
void rn_bias_act_grad(const void* dy, const void* h, void* dh, float* db, void* db16, float* part, int M, int N,
                      int act, int want_bias, int accum, hipStream_t st) {
    int cblocks = (N + 511) / 512;
    int splits = 1;
    while (cblocks * splits < 512 && M / (splits * 2) >= 32) splits *= 2;
    int rps = (M + splits - 1) / splits;
    dim3 grid(cblocks, splits);
#define RN_BAG(A, W) bias_act_grad_k<A, W><<<grid, TPB, 0, st>>>((const bf16*)dy, (const bf16*)h, (bf16*)dh, part, M, N, rps)
    if (act == ACT_GELU) { if (want_bias) RN_BAG(ACT_GELU, true); else RN_BAG(ACT_GELU, false); }
    else if (act == ACT_RELU) { if (want_bias) RN_BAG(ACT_RELU, true); else RN_BAG(ACT_RELU, false); }
    else { if (want_bias) RN_BAG(ACT_NONE, true); else return; }
#undef RN_BAG
    if (want_bias) rn_colreduce(part, splits, N, part + (long)splits * N, db, (bf16*)db16, st, accum);
}

// out16[c] (+)= Σ_r in[r][c] for an fp32 [R][C] partial matrix (tmp: RN_COLRED_S * C floats).
void rn_colsum_f32(const float* in, int R, int C, float* tmp, void* out16, int accum, hipStream_t st) {
    rn_colreduce(in, R, C, tmp, nullptr, (bf16*)out16, st, accum);
}
int rn_colsum_ws(int C) { return RN_COLRED_S * C; }

int rn_bias_act_grad_splits(int M, int N) {
    int cblocks = (N + 511) / 512;
    int splits = 1;
    while (cblocks * splits < 512 && M / (splits * 2) >= 32) splits *= 2;
    return splits;
}

}  // extern "C"
