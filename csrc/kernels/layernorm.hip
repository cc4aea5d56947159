// LayerNorm forward / backward (N6), optional fused residual add.
//
// One row per wave (4 rows per 256-thread block).  Each lane holds up to NV
// 16-byte vectors (8 bf16) of its row in registers, so the row is read from
// HBM exactly once per pass; statistics in fp32 with wave shuffles (no LDS).
//   fwd:  h = x (+ r);  y = (h - mu) * rstd * w + b;  saves mu, rstd (fp32)
//   bwd:  dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) (+ gh),  g = dy * w
//         dw, db: per-wave fp32 partial rows, reduced in fixed order (deterministic).
#include <cstdlib>

#include "common.h"

namespace {

// Q8: also write the output as OCP e4m3 (q8 = y / st8[0], saturating) for the consumer's fp8
// GEMM and record amax(|y|) in st8[1] (delayed scaling, ops/fp8.py: the scale was rolled from the
// previous amax just before this launch) — the consumer's separate quantisation pass (read y,
// write q) is gone.  Rows are grid-strided so the amax costs one atomic per block.
template <int NV, bool RES, bool BIAS, bool Q8 = false>
__global__ void __launch_bounds__(256) ln_fwd_k(const bf16* __restrict__ x, const bf16* __restrict__ r,
                                                const bf16* __restrict__ w, const bf16* __restrict__ b,
                                                bf16* __restrict__ y, bf16* __restrict__ hout,
                                                float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                int M, int E, float eps, uint8_t* __restrict__ q8 = nullptr,
                                                float* __restrict__ st8 = nullptr) {
    constexpr float E4M3_MAX = 448.f;
    const int lane = threadIdx.x & 63;
    const int nvec = E / 8;
    [[maybe_unused]] float amax = 0.f, inv8 = 0.f;
    if constexpr (Q8) inv8 = 1.f / st8[0];
    // gamma / beta chunks loaded once, before the row's loads and reductions (not after them:
    // that was a second memory round trip per row)
    bf16x8 wv[NV];
    [[maybe_unused]] bf16x8 bv[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = lane + i * 64;
        if (c < nvec) {
            wv[i] = *reinterpret_cast<const bf16x8*>(w + c * 8);
            if constexpr (BIAS) bv[i] = *reinterpret_cast<const bf16x8*>(b + c * 8);
        }
    }
    // grid-strided rows with a one-row software prefetch: the next row's x (and r) loads are in
    // flight while this row is reduced, normalised and stored (one HBM round trip per row was the
    // limiter of the one-row-per-wave version: ~4.6 TB/s)
    const int rstride = gridDim.x * 4;
    bf16x8 xn[NV];
    [[maybe_unused]] bf16x8 rn[NV];
    auto fetch = [&](int rr) {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = lane + i * 64;
            if (c < nvec) {
                xn[i] = *reinterpret_cast<const bf16x8*>(x + (long)rr * E + c * 8);
                if constexpr (RES) rn[i] = *reinterpret_cast<const bf16x8*>(r + (long)rr * E + c * 8);
            }
        }
    };
    int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row < M) fetch(row);
    for (; row < M; row += rstride) {
        float v[NV][8];
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = (lane + i * 64);
            if (c < nvec) {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[i][j] = (float)xn[i][j];
                if constexpr (RES) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[i][j] += (float)rn[i][j];
                }
            }
        }
        if (row + rstride < M) fetch(row + rstride);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = (lane + i * 64);
            if (c < nvec) {
                if constexpr (RES) store8(hout + (long)row * E + c * 8, v[i]);
#pragma unroll
                for (int j = 0; j < 8; ++j) s += v[i][j];
            }
        }
        const float mu = wave_sum(s) / E;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = lane + i * 64;
            if (c < nvec) {
#pragma unroll
                for (int j = 0; j < 8; ++j) { float d = v[i][j] - mu; q += d * d; }
            }
        }
        const float rs = rsqrtf(wave_sum(q) / E + eps);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = lane + i * 64;
            if (c < nvec) {
                float o[8];
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    o[j] = (v[i][j] - mu) * rs * (float)wv[i][j] + (BIAS ? (float)bv[i][j] : 0.f);
                store8(y + (long)row * E + c * 8, o);
                if constexpr (Q8) {
                    float f[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {  // from the stored bf16 y: same bytes as a separate pass
                        const float yb = bf2f(f2bf(o[j]));
                        amax = fmaxf(amax, fabsf(yb));
                        f[j] = fminf(fmaxf(yb * inv8, -E4M3_MAX), E4M3_MAX);
                    }
                    int w0 = 0, w1 = 0;
                    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], w0, false);
                    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w0, true);
                    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], w1, false);
                    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], w1, true);
                    *reinterpret_cast<int2*>(q8 + (long)row * E + c * 8) = make_int2(w0, w1);
                }
            }
        }
        if (lane == 0) { mean_out[row] = mu; rstd_out[row] = rs; }
    }
    if constexpr (Q8) {
        __shared__ float am[4];
        amax = wave_max(amax);
        if (lane == 0) am[threadIdx.x >> 6] = amax;
        __syncthreads();
        if (threadIdx.x == 0)
            atomicMax(reinterpret_cast<int*>(st8 + 1),
                      __float_as_int(fmaxf(fmaxf(am[0], am[1]), fmaxf(am[2], am[3]))));
    }
}

// One row per wave; each block folds its 4 waves' column partials in LDS and
// writes ONE partial row [dw | db | Σdx] (Q = 2 or 3 segments of E floats), so
// the column reduction reads 4× fewer partials and runs as a single launch.
// Σdx (DXS) is the bias gradient of the linear layer whose output fed this
// LayerNorm (x = x_prev + a·Wᵀ + b ⇒ db = Σ_rows dx): computed here for free
// instead of a separate pass over dx.
// Q8: dx also as e5m2 with the delayed scale q8st[0] (rolled by the host) — the bytes the consumer's delayed
// quantisation pass would write from the stored bf16 dx — and amax(|dx|) recorded into q8st[1] (one atomic per
// block): the fp8 linear that produced this LayerNorm's input takes its dY operand from here
template <int NV, bool GH, bool DXS, bool Q8 = false>
__global__ void __launch_bounds__(256) ln_bwd_k(const bf16* __restrict__ dy, const bf16* __restrict__ gh,
                                                const bf16* __restrict__ h, const bf16* __restrict__ w,
                                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                                bf16* __restrict__ dx, float* __restrict__ part, int M, int E,
                                                uint8_t* __restrict__ q8 = nullptr, float* __restrict__ q8st = nullptr) {
    constexpr int Q = DXS ? 3 : 2;
    __shared__ float red[3][NV * 512];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wave = blockIdx.x * 4 + wv;
    const int nwaves = gridDim.x * 4;
    const int nvec = E / 8;
    float acc[Q][NV][8], wf[NV][8];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int c = lane + i * 64;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
            for (int q = 0; q < Q; ++q) acc[q][i][j] = 0.f;
        }
        if (c < nvec) load8(w + c * 8, wf[i]);
    }
    // one-row software prefetch (as the forward): the next row's dy / h / gh loads and its mean /
    // rstd are in flight while this row is reduced and dx stored
    bf16x8 hn[NV], dn[NV];
    [[maybe_unused]] bf16x8 gn[NV];
    float mun = 0.f, rsn = 0.f;
    auto fetch = [&](int rr) {
        mun = mean[rr];
        rsn = rstd[rr];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = lane + i * 64;
            if (c < nvec) {
                if constexpr (GH) gn[i] = *reinterpret_cast<const bf16x8*>(gh + (long)rr * E + c * 8);
                hn[i] = *reinterpret_cast<const bf16x8*>(h + (long)rr * E + c * 8);
                dn[i] = *reinterpret_cast<const bf16x8*>(dy + (long)rr * E + c * 8);
            }
        }
    };
    [[maybe_unused]] const float q8inv = Q8 ? 1.f / q8st[0] : 1.f;
    [[maybe_unused]] float q8m = 0.f;
    if (wave < M) fetch(wave);
    for (int row = wave; row < M; row += nwaves) {
        const float mu = mun, rs = rsn;
        float xh[NV][8], g[NV][8];
        float s1 = 0.f, s2 = 0.f;
        [[maybe_unused]] bf16x8 ghv[NV];
        float d[NV][8];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            if constexpr (GH) ghv[i] = gn[i];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                xh[i][j] = (float)hn[i][j];
                d[i][j] = (float)dn[i][j];
            }
        }
        if (row + nwaves < M) fetch(row + nwaves);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = lane + i * 64;
            if (c < nvec) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    xh[i][j] = (xh[i][j] - mu) * rs;
                    g[i][j] = d[i][j] * wf[i][j];
                    s1 += g[i][j];
                    s2 += g[i][j] * xh[i][j];
                    acc[0][i][j] += d[i][j] * xh[i][j];
                    acc[1][i][j] += d[i][j];
                }
            }
        }
        s1 = wave_sum(s1) / E;
        s2 = wave_sum(s2) / E;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = lane + i * 64;
            if (c < nvec) {
                float o[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = rs * (g[i][j] - s1 - xh[i][j] * s2);
                if constexpr (GH) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) o[j] += (float)ghv[i][j];
                }
                store8(dx + (long)row * E + c * 8, o);
                if constexpr (Q8) {
                    constexpr float LIM = 57344.f;
                    float f[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float v = (float)(bf16)o[j];
                        q8m = fmaxf(q8m, fabsf(v));
                        f[j] = fminf(fmaxf(v * q8inv, -LIM), LIM);
                    }
                    int w0 = 0, w1 = 0;
                    w0 = __builtin_amdgcn_cvt_pk_bf8_f32(f[0], f[1], w0, false);
                    w0 = __builtin_amdgcn_cvt_pk_bf8_f32(f[2], f[3], w0, true);
                    w1 = __builtin_amdgcn_cvt_pk_bf8_f32(f[4], f[5], w1, false);
                    w1 = __builtin_amdgcn_cvt_pk_bf8_f32(f[6], f[7], w1, true);
                    *reinterpret_cast<int2*>(q8 + (long)row * E + c * 8) = make_int2(w0, w1);
                }
                if constexpr (DXS) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc[Q - 1][i][j] += (float)(bf16)o[j];  // Σ of the stored dx
                }
            }
        }
    }
    if constexpr (Q8) {  // block amax → one atomic (max is order-independent: bitwise repeatable)
        __shared__ float qm[4];
        q8m = wave_max(q8m);
        if (lane == 0) qm[wv] = q8m;
        __syncthreads();
        if (threadIdx.x == 0)
            atomicMax(reinterpret_cast<int*>(q8st + 1), __float_as_int(fmaxf(fmaxf(qm[0], qm[1]), fmaxf(qm[2], qm[3]))));
    }
    // fold the 4 waves: waves 1..3 park their partials in LDS, wave 0 adds (fixed order)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        if (wv > 0) {
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                int c = lane + i * 64;
                if (c < nvec) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) red[wv - 1][c * 8 + j] = acc[q][i][j];
                }
            }
        }
        __syncthreads();
        if (wv == 0) {
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                int c = lane + i * 64;
                if (c < nvec) {
                    float o[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        o[j] = acc[q][i][j] + red[0][c * 8 + j] + red[1][c * 8 + j] + red[2][c * 8 + j];
                    float* dst = part + (long)blockIdx.x * Q * E + (long)q * E + c * 8;
                    *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
                    *reinterpret_cast<float4*>(dst + 4) = make_float4(o[4], o[5], o[6], o[7]);
                }
            }
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" {

int rn_ln_nv(int E) { return (E / 8 + 63) / 64; }

// q8 / st8 (optional): fused e4m3 output with delayed scaling (st8 already rolled by the caller)
int rn_ln_fwd(const void* x, const void* r, const void* w, const void* b, void* y, void* h, float* mean,
              float* rstd, int M, int E, float eps, hipStream_t st, void* q8, float* st8) {
    if (E % 8 != 0 || E > 8192) return -1;
    int nv = rn_ln_nv(E);
    if (q8) {
        // 4096 blocks (16 per CU): enough rows in flight for HBM, one amax atomic per block
        dim3 grid((M + 3) / 4 < 4096 ? (M + 3) / 4 : 4096);
#define RN_LNF(NV, R, B) ln_fwd_k<NV, R, B, true><<<grid, 256, 0, st>>>((const bf16*)x, (const bf16*)r, (const bf16*)w, (const bf16*)b, (bf16*)y, (bf16*)h, mean, rstd, M, E, eps, (uint8_t*)q8, st8)
#define RN_LNF2(NV) { if (r) { if (b) RN_LNF(NV, true, true); else RN_LNF(NV, true, false); } \
                      else { if (b) RN_LNF(NV, false, true); else RN_LNF(NV, false, false); } }
        if (nv <= 1) RN_LNF2(1) else if (nv <= 2) RN_LNF2(2) else if (nv <= 4) RN_LNF2(4) else if (nv <= 8) RN_LNF2(8)
        else RN_LNF2(16)
#undef RN_LNF2
#undef RN_LNF
        return 0;
    }
    // 2048 blocks = 8192 waves (32 per CU): each wave walks M / 8192 rows with the prefetch
    constexpr int fwd_cap = 2048;
    dim3 grid((M + 3) / 4 < fwd_cap ? (M + 3) / 4 : fwd_cap);
#define RN_LNF(NV, R, B) ln_fwd_k<NV, R, B><<<grid, 256, 0, st>>>((const bf16*)x, (const bf16*)r, (const bf16*)w, (const bf16*)b, (bf16*)y, (bf16*)h, mean, rstd, M, E, eps)
#define RN_LNF2(NV) { if (r) { if (b) RN_LNF(NV, true, true); else RN_LNF(NV, true, false); } \
                      else { if (b) RN_LNF(NV, false, true); else RN_LNF(NV, false, false); } }
    if (nv <= 1) RN_LNF2(1) else if (nv <= 2) RN_LNF2(2) else if (nv <= 4) RN_LNF2(4) else if (nv <= 8) RN_LNF2(8)
    else RN_LNF2(16)
#undef RN_LNF2
#undef RN_LNF
    return 0;
}

// waves of the backward grid (each loops over rows with a one-row prefetch): 2048 (8 per CU): with the prefetch this keeps HBM as busy as 8192 did and writes
// 4x fewer column-partial rows for the reduction that follows (GPT-2-small step -0.3 ms, call gpu_r3zn)
int rn_ln_bwd_blocks(int M) {
    constexpr int cap = 2048;
    int W = M < cap ? M : cap;
    return (W + 3) / 4;
}
int rn_ln_bwd_waves(int M) { return 4 * rn_ln_bwd_blocks(M); }

// workspace floats: partial rows [blocks][3E] + the reduction's [RN_COLRED_S][3E] scratch
long rn_ln_bwd_ws(int M, int E) { return 3L * (rn_ln_bwd_blocks(M) + RN_COLRED_S) * E; }

// ws: rn_ln_bwd_ws(M, E) floats.  dw/db (fp32) and dw16/db16 (bf16) outputs, any may be null.
// dxs16 (optional, bf16, always accumulated into): Σ_rows dx — the bias gradient of the layer
// that produced this LayerNorm's input.
void rn_fp8_roll_bf8(float* state, hipStream_t st);  // fp8.hip
// q8 / q8st (optional): dx also in e5m2 with the consumer's delayed scale (q8st rolled here), see ln_bwd_k
int rn_ln_bwd(const void* dy, const void* gh, const void* h, const void* w, const float* mean, const float* rstd,
              void* dx, float* dw, float* db, void* dw16, void* db16, void* dxs16, float* ws, int M, int E,
              int accum, hipStream_t st, void* q8, float* q8st) {
    if (E % 8 != 0 || E > 8192) return -1;
    const int nv = rn_ln_nv(E);
    const int B = rn_ln_bwd_blocks(M);
    const int Q = dxs16 ? 3 : 2;
    float* part = ws;
    float* tmp = ws + (long)B * Q * E;
    if (q8) rn_fp8_roll_bf8(q8st, st);
#define RN_LNB(NV, G, D) do { if (q8) ln_bwd_k<NV, G, D, true><<<B, 256, 0, st>>>((const bf16*)dy, (const bf16*)gh, (const bf16*)h, (const bf16*)w, mean, rstd, (bf16*)dx, part, M, E, (uint8_t*)q8, q8st); \
                           else ln_bwd_k<NV, G, D><<<B, 256, 0, st>>>((const bf16*)dy, (const bf16*)gh, (const bf16*)h, (const bf16*)w, mean, rstd, (bf16*)dx, part, M, E); } while (0)
#define RN_LNB2(NV) { if (gh) { if (dxs16) RN_LNB(NV, true, true); else RN_LNB(NV, true, false); } \
                      else { if (dxs16) RN_LNB(NV, false, true); else RN_LNB(NV, false, false); } }
    if (nv <= 1) RN_LNB2(1) else if (nv <= 2) RN_LNB2(2) else if (nv <= 4) RN_LNB2(4) else if (nv <= 8) RN_LNB2(8)
    else RN_LNB2(16)
#undef RN_LNB2
#undef RN_LNB
    RnColOut o{{dw, db, nullptr}, {(bf16*)dw16, (bf16*)db16, (bf16*)dxs16}, E, {accum, accum, 1}};
    rn_colreduce_seg(part, B, Q * E, tmp, o, st);
    return 0;
}

}  // extern "C"
