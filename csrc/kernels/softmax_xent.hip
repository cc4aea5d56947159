// Row softmax (N8) and fused softmax cross-entropy (N9).
//
// Softmax: one 256-thread block per row, online (max, sum) in one pass over
// 16-byte vectors, normalised write in a second pass.
// Cross-entropy: forward reads each logits row ONCE (online log-sum-exp with
// one rescale per 8 elements) and stores only the per-row lse + NLL; backward
// writes (softmax - onehot) * g / n in place over the logits, zero in the
// padded columns [n_valid, V).
#include <cstdlib>

#include "common.h"

namespace {

constexpr int TPB = 256;

RN_DEV void online_update(float& m, float& s, const float* f, int cnt) {
    float lm = f[0];
    for (int j = 1; j < cnt; ++j) lm = fmaxf(lm, f[j]);
    float nm = fmaxf(m, lm);
    float acc = (m == -INFINITY) ? 0.f : s * __expf(m - nm);
    for (int j = 0; j < cnt; ++j) acc += __expf(f[j] - nm);
    m = nm;
    s = acc;
}

// reduce (m, s) pairs across the block
RN_DEV void block_reduce_ms(float& m, float& s, float* sm) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
        float nm = fmaxf(m, om);
        float a = (m == -INFINITY) ? 0.f : s * __expf(m - nm);
        float b = (om == -INFINITY) ? 0.f : os * __expf(om - nm);
        m = nm;
        s = a + b;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) { sm[wid] = m; sm[8 + wid] = s; }
    __syncthreads();
    float M = -INFINITY;
    for (int i = 0; i < TPB / 64; ++i) M = fmaxf(M, sm[i]);
    float S = 0.f;
    for (int i = 0; i < TPB / 64; ++i) S += (sm[i] == -INFINITY) ? 0.f : sm[8 + i] * __expf(sm[i] - M);
    m = M;
    s = S;
}

// row statistics over columns [0, n) of a row (scaled by `scale`)
RN_DEV void row_ms(const bf16* row, int n, float scale, float& m, float& s, float* sm) {
    m = -INFINITY;
    s = 0.f;
    const bool vec = ((reinterpret_cast<uintptr_t>(row) & 15) == 0);
    int n8 = vec ? n / 8 : 0;
    for (int i = threadIdx.x; i < n8; i += TPB) {
        float f[8];
        load8(row + i * 8, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= scale;
        online_update(m, s, f, 8);
    }
    for (int i = n8 * 8 + threadIdx.x; i < n; i += TPB) {
        float f = bf2f(row[i]) * scale;
        online_update(m, s, &f, 1);
    }
    block_reduce_ms(m, s, sm);
}

__global__ void __launch_bounds__(TPB) softmax_fwd_k(const bf16* __restrict__ x, bf16* __restrict__ y, int N,
                                                     float scale) {
    __shared__ float sm[16];
    const bf16* xr = x + (long)blockIdx.x * N;
    bf16* yr = y + (long)blockIdx.x * N;
    float m, s;
    row_ms(xr, N, scale, m, s, sm);
    const float inv = 1.f / s;
    for (int i = threadIdx.x; i < N; i += TPB) yr[i] = f2bf(__expf(bf2f(xr[i]) * scale - m) * inv);
}

__global__ void __launch_bounds__(TPB) softmax_bwd_k(const bf16* __restrict__ dy, const bf16* __restrict__ y,
                                                     bf16* __restrict__ dx, int N, float scale) {
    __shared__ float sm[16];
    const long base = (long)blockIdx.x * N;
    float d = 0.f;
    for (int i = threadIdx.x; i < N; i += TPB) d += bf2f(dy[base + i]) * bf2f(y[base + i]);
    d = block_sum(d, sm);
    for (int i = threadIdx.x; i < N; i += TPB)
        dx[base + i] = f2bf(scale * bf2f(y[base + i]) * (bf2f(dy[base + i]) - d));
}

// GRAD: also overwrite the row with the UNSCALED gradient softmax - onehot (0 in
// padded columns / ignored rows); the caller folds g/n into the consumers (the
// LM-head GEMM epilogues' alpha), so the logits are read from HBM once per step.
template <bool GRAD>
__global__ void __launch_bounds__(TPB) xent_fwd_k(bf16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                  float* __restrict__ loss, float* __restrict__ lse_out, int V,
                                                  int nvalid, long ignore) {
    __shared__ float sm[16];
    bf16* row = logits + (long)blockIdx.x * V;
    float m, s;
    row_ms(row, nvalid, 1.f, m, s, sm);
    const float lse = m + __logf(s);
    const long t = tgt[blockIdx.x];
    const bool ign = (t == ignore || t < 0 || t >= nvalid);
    if (threadIdx.x == 0) {
        lse_out[blockIdx.x] = lse;
        loss[blockIdx.x] = ign ? 0.f : lse - bf2f(row[t]);
    }
    if constexpr (GRAD) {
        __syncthreads();  // the target logit was read above before anyone overwrites it
        const float z = ign ? 0.f : 1.f;
        if (V % 8 == 0) {
            for (int i = threadIdx.x; i < V / 8; i += TPB) {
                float f[8];
                load8(row + i * 8, f);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int c = i * 8 + j;
                    f[j] = (c < nvalid ? __expf(f[j] - lse) - (c == t ? 1.f : 0.f) : 0.f) * z;
                }
                store8(row + i * 8, f);
            }
        } else {
            for (int c = threadIdx.x; c < V; c += TPB) {
                const float p = c < nvalid ? __expf(bf2f(row[c]) - lse) - (c == t ? 1.f : 0.f) : 0.f;
                row[c] = f2bf(p * z);
            }
        }
    }
}

// Loss-only single-pass row kernel (evaluation) for V % 8 == 0, V <= 8 * 1024 * CH: the 1024-thread
// block keeps its whole row in registers (CH 16-byte chunks per thread), so the row is read from HBM
// once.  Same outputs and the same fixed reduction order for every launch.  (Its round-1 gradient
// form was replaced by xent_row2_k and removed in round 4.)
template <int CH>
__global__ void __launch_bounds__(1024) xent_row_k(bf16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                   float* __restrict__ loss, float* __restrict__ lse_out, int V,
                                                   int nvalid, long ignore) {
    __shared__ float sm[16];
    bf16* row = logits + (long)blockIdx.x * V;
    const int n8 = V / 8;
    const long t = tgt[blockIdx.x];
    const bool ign = (t == ignore || t < 0 || t >= nvalid);
    RN_CHECK(t == ignore || (t >= 0 && t < nvalid));
    const float xt = ign ? 0.f : bf2f(row[t]);
    bf16x8 v[CH];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        const int i = threadIdx.x + k * 1024;
        if (i < n8) {
            v[k] = *reinterpret_cast<const bf16x8*>(row + i * 8);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (i * 8 + j < nvalid) m = fmaxf(m, (float)v[k][j]);
        }
    }
    m = block_max(m, sm);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        const int i = threadIdx.x + k * 1024;
        if (i < n8) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (i * 8 + j < nvalid) s += __expf((float)v[k][j] - m);
        }
    }
    s = block_sum(s, sm);
    const float lse = m + __logf(s);
    if (threadIdx.x == 0) {
        lse_out[blockIdx.x] = lse;
        loss[blockIdx.x] = ign ? 0.f : lse - xt;
    }
}

// Fused-gradient row kernel, v2 (the default for V % 8 == 0, V <= 8·1024·CH, write_grad):
//   * ONE block reduction: each thread reduces its registers to a local (max, Σ exp) pair first,
//     the pairs are merged across the block (m, s) ⊕ (m', s') = (M, s·2^(m-M) + s'·2^(m'-M));
//   * ONE exponential per element: the exp2 of the local pass is kept (as bf16, over the logits
//     in registers) and the gradient is e · 2^(m_local - lse): a multiply, not a second exp;
//   * base-2 throughout (x·log2e folded into one FMA with the max), padded-column and target
//     masks only where a chunk straddles them.
// Output differs from xent_row_k by the extra bf16 rounding of e (≤ 1 bf16 ulp of the gradient).
// The logits are loaded non-temporally (the 6.6 GB GPT-2 logits stream cannot stay in any cache
// between the LM-head GEMM, this pass and the backward GEMMs: 2.42 -> 2.38 ms); the gradient stores
// stay plain (non-temporal stores measured 1.5x slower, 3.54-3.68 ms, gpu_r3zt).
// Q8: the gradient goes to q8 (row stride V bytes) as e5m2 of (softmax - onehot) · 2^15 instead of bf16 over
// the logits — the fp8 LM head's backward operand (ops/loss.py _LinearXentFp8Fn).  |softmax - onehot| <= 1, so the
// fixed power-of-two scale XQ8_SCALE keeps every value below e5m2's 57344 and puts probabilities down to 2^-31 in
// its range: no amax pass, no delayed-scaling slot.
constexpr float XQ8_SCALE = 32768.f;
template <int CH, bool Q8 = false>
__global__ void __launch_bounds__(1024) xent_row2_k(bf16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                    float* __restrict__ loss, float* __restrict__ lse_out, int V,
                                                    int nvalid, long ignore, uint8_t* __restrict__ q8 = nullptr) {
    constexpr float L2E = 1.4426950408889634f;
    __shared__ float sm_m[16], sm_s[16];
    bf16* row = logits + (long)blockIdx.x * V;
    const int n8 = V / 8;
    const long t = tgt[blockIdx.x];
    const bool ign = (t == ignore || t < 0 || t >= nvalid);
    RN_CHECK(t == ignore || (t >= 0 && t < nvalid));
    const float xt = ign ? 0.f : bf2f(row[t]);
    bf16x8 v[CH];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        const int i = threadIdx.x + k * 1024;
        if (i < n8) {
            v[k] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(row + i * 8));
            if (i * 8 + 8 <= nvalid) {
#pragma unroll
                for (int j = 0; j < 8; ++j) m = fmaxf(m, (float)v[k][j]);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (i * 8 + j < nvalid) m = fmaxf(m, (float)v[k][j]);
            }
        }
    }
    const float mL = (m == -INFINITY) ? 0.f : m * L2E;
    const float m_own = m;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        const int i = threadIdx.x + k * 1024;
        if (i < n8) {
            bf16x8 e;
            // raw v_exp_f32 (arguments <= 0: no overflow; results below 2^-126 flush to 0, which the
            // bf16 e could not hold anyway) -- exp2f's denormal range reduction was 4 extra VALU per
            // element; the padded-column mask only in the one chunk that straddles nvalid
            if (i * 8 + 8 <= nvalid) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float x = __builtin_amdgcn_exp2f(fmaf((float)v[k][j], L2E, -mL));
                    s += x;
                    e[j] = (bf16)x;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float x = (i * 8 + j < nvalid) ? __builtin_amdgcn_exp2f(fmaf((float)v[k][j], L2E, -mL)) : 0.f;
                    s += x;
                    e[j] = (bf16)x;
                }
            }
            v[k] = e;
        }
    }
    // block merge of (m, s): wave butterfly, then the 16 wave results (every thread, same order)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
        const float M = fmaxf(m, m2);
        s = (M == -INFINITY) ? 0.f : s * __builtin_amdgcn_exp2f((m - M) * L2E) + s2 * __builtin_amdgcn_exp2f((m2 - M) * L2E);
        m = M;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        sm_m[wid] = m;
        sm_s[wid] = s;
    }
    __syncthreads();
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 16; ++w) M = fmaxf(M, sm_m[w]);
    float S = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) S += sm_s[w] * __builtin_amdgcn_exp2f((sm_m[w] - M) * L2E);
    const float lse = M + __logf(S);
    if (threadIdx.x == 0) {
        lse_out[blockIdx.x] = lse;
        loss[blockIdx.x] = ign ? 0.f : lse - xt;
    }
    // this thread's e values were taken relative to ITS local max (mL): rescale to the row's lse
    // (a thread without a valid column has e = 0 and m = -inf: f = 0, never 0 · inf)
    const float f = (ign || m_own == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(mL - lse * L2E);
    if constexpr (Q8) {
        uint8_t* qrow = q8 + (long)blockIdx.x * V;
        const float fq = f * XQ8_SCALE;
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int i = threadIdx.x + k * 1024;
            if (i < n8) {
                float g[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) g[j] = (float)v[k][j] * fq;
                int w0 = 0, w1 = 0;
                w0 = __builtin_amdgcn_cvt_pk_bf8_f32(g[0], g[1], w0, false);
                w0 = __builtin_amdgcn_cvt_pk_bf8_f32(g[2], g[3], w0, true);
                w1 = __builtin_amdgcn_cvt_pk_bf8_f32(g[4], g[5], w1, false);
                w1 = __builtin_amdgcn_cvt_pk_bf8_f32(g[6], g[7], w1, true);
                *reinterpret_cast<uint2*>(qrow + i * 8) = make_uint2((uint32_t)w0, (uint32_t)w1);
            }
        }
        if (!ign && threadIdx.x == (int)((t >> 3) & 1023)) {  // the one-hot term, as below
            const float et = (float)(bf16)__builtin_amdgcn_exp2f(fmaf(xt, L2E, -mL));
            qrow[t] = (uint8_t)(__builtin_amdgcn_cvt_pk_bf8_f32((et * f - 1.f) * XQ8_SCALE, 0.f, 0, false) & 0xFF);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        const int i = threadIdx.x + k * 1024;
        if (i < n8) {
            float g[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) g[j] = (float)v[k][j] * f;
            store8(row + i * 8, g);
        }
    }
    // the one-hot term: the thread that owns column t rewrites it (a runtime index into g[] was a
    // compare + select per element); its e is recomputed bit-identically from xt
    if (!ign && threadIdx.x == (int)((t >> 3) & 1023)) {
        const float et = (float)(bf16)__builtin_amdgcn_exp2f(fmaf(xt, L2E, -mL));
        row[t] = (bf16)(et * f - 1.f);
    }
}

__global__ void __launch_bounds__(TPB) xent_bwd_k(const bf16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                  const float* __restrict__ lse, const float* __restrict__ gscale,
                                                  bf16* __restrict__ grad, int V, int nvalid, long ignore) {
    const long base = (long)blockIdx.x * V;
    const long t = tgt[blockIdx.x];
    const bool ign = (t == ignore);
    const float L = lse[blockIdx.x];
    const float g = ign ? 0.f : gscale[0];
    const bool vec = (V % 8 == 0);
    if (vec) {
        for (int i = threadIdx.x; i < V / 8; i += TPB) {
            float f[8];
            load8(logits + base + i * 8, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                int c = i * 8 + j;
                float p = c < nvalid ? __expf(f[j] - L) : 0.f;
                f[j] = (p - (c == t ? 1.f : 0.f)) * g;
            }
            store8(grad + base + i * 8, f);
        }
    } else {
        for (int c = threadIdx.x; c < V; c += TPB) {
            float p = c < nvalid ? __expf(bf2f(logits[base + c]) - L) : 0.f;
            grad[base + c] = f2bf((p - (c == t ? 1.f : 0.f)) * g);
        }
    }
}

}  // namespace

extern "C" {

void rn_softmax_fwd(const void* x, void* y, int M, int N, float scale, hipStream_t st) {
    softmax_fwd_k<<<M, TPB, 0, st>>>((const bf16*)x, (bf16*)y, N, scale);
}
void rn_softmax_bwd(const void* dy, const void* y, void* dx, int M, int N, float scale, hipStream_t st) {
    softmax_bwd_k<<<M, TPB, 0, st>>>((const bf16*)dy, (const bf16*)y, (bf16*)dx, N, scale);
}
void rn_xent_fwd(void* logits, const int64_t* tgt, float* loss, float* lse, int M, int V, int nvalid, long ignore,
                 int write_grad, hipStream_t st) {
    if (V % 8 == 0 && V <= 8 * 1024 * 8) {
        const int ch = (V / 8 + 1023) / 1024;
#define RN_XR(C) { if (write_grad) xent_row2_k<C><<<M, 1024, 0, st>>>((bf16*)logits, tgt, loss, lse, V, nvalid, ignore); \
                   else xent_row_k<C><<<M, 1024, 0, st>>>((bf16*)logits, tgt, loss, lse, V, nvalid, ignore); }
        if (ch <= 1) RN_XR(1) else if (ch <= 2) RN_XR(2) else if (ch <= 4) RN_XR(4) else if (ch <= 7) RN_XR(7)
        else RN_XR(8)
#undef RN_XR
        return;
    }
    if (write_grad) xent_fwd_k<true><<<M, TPB, 0, st>>>((bf16*)logits, tgt, loss, lse, V, nvalid, ignore);
    else xent_fwd_k<false><<<M, TPB, 0, st>>>((bf16*)logits, tgt, loss, lse, V, nvalid, ignore);
}
// the fp8 LM head's loss: rn_xent_fwd with write_grad, the gradient to q8 as e5m2 · 2^15 (xent_row2_k<.., true>);
// -1 if V is outside the row kernel's range (the caller keeps the bf16 path)
int rn_xent_fwd_q8(void* logits, const int64_t* tgt, float* loss, float* lse, int M, int V, int nvalid, long ignore,
                   void* q8, hipStream_t st) {
    if (V % 8 || V > 8 * 1024 * 8) return -1;
    const int ch = (V / 8 + 1023) / 1024;
#define RN_XQ(C) xent_row2_k<C, true><<<M, 1024, 0, st>>>((bf16*)logits, tgt, loss, lse, V, nvalid, ignore, (uint8_t*)q8)
    if (ch <= 1) RN_XQ(1); else if (ch <= 2) RN_XQ(2); else if (ch <= 4) RN_XQ(4); else if (ch <= 7) RN_XQ(7);
    else RN_XQ(8);
#undef RN_XQ
    return 0;
}
void rn_xent_bwd(const void* logits, const int64_t* tgt, const float* lse, const float* gscale, void* grad, int M,
                 int V, int nvalid, long ignore, hipStream_t st) {
    xent_bwd_k<<<M, TPB, 0, st>>>((const bf16*)logits, tgt, lse, gscale, (bf16*)grad, V, nvalid, ignore);
}

}  // extern "C"
