// LayerNorm forward / backward (N6), optional fused residual add.
//
// One row per wave (4 rows per 256-thread block).  Each lane holds up to NV
// 16-byte vectors (8 bf16) of its row in registers, so the row is read from
// HBM exactly once per pass; statistics in fp32 with wave shuffles (no LDS).
//   fwd:  h = x (+ r);  y = (h - mu) * rstd * w + b;  saves mu, rstd (fp32)
//   bwd:  dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) (+ gh),  g = dy * w
//         dw, db: per-wave fp32 partial rows, reduced in fixed order (deterministic).
#include "common.h"

namespace {

template <int NV, bool RES, bool BIAS>
__global__ void __launch_bounds__(256) ln_fwd_k(const bf16* __restrict__ x, const bf16* __restrict__ r,
                                                const bf16* __restrict__ w, const bf16* __restrict__ b,
                                                bf16* __restrict__ y, bf16* __restrict__ hout,
                                                float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                int M, int E, float eps) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int nvec = E / 8;
    const bf16* xr = x + (long)row * E;
    float v[NV][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int c = (lane + i * 64);
        if (c < nvec) {
            load8(xr + c * 8, v[i]);
            if constexpr (RES) {
                float t[8];
                load8(r + (long)row * E + c * 8, t);
#pragma unroll
                for (int j = 0; j < 8; ++j) v[i][j] += t[j];
                store8(hout + (long)row * E + c * 8, v[i]);
            }
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
            float wf[8], bfv[8], o[8];
            load8(w + c * 8, wf);
            if constexpr (BIAS) load8(b + c * 8, bfv);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mu) * rs * wf[j] + (BIAS ? bfv[j] : 0.f);
            store8(y + (long)row * E + c * 8, o);
        }
    }
    if (lane == 0) { mean_out[row] = mu; rstd_out[row] = rs; }
}

template <int NV, bool GH>
__global__ void __launch_bounds__(256) ln_bwd_k(const bf16* __restrict__ dy, const bf16* __restrict__ gh,
                                                const bf16* __restrict__ h, const bf16* __restrict__ w,
                                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                                bf16* __restrict__ dx, float* __restrict__ pdw,
                                                float* __restrict__ pdb, int M, int E) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nwaves = gridDim.x * 4;
    const int nvec = E / 8;
    float adw[NV][8], adb[NV][8], wf[NV][8];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int c = lane + i * 64;
#pragma unroll
        for (int j = 0; j < 8; ++j) { adw[i][j] = 0.f; adb[i][j] = 0.f; }
        if (c < nvec) load8(w + c * 8, wf[i]);
    }
    for (int row = wave; row < M; row += nwaves) {
        const float mu = mean[row], rs = rstd[row];
        float xh[NV][8], g[NV][8];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = lane + i * 64;
            if (c < nvec) {
                float d[8];
                load8(h + (long)row * E + c * 8, xh[i]);
                load8(dy + (long)row * E + c * 8, d);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    xh[i][j] = (xh[i][j] - mu) * rs;
                    g[i][j] = d[j] * wf[i][j];
                    s1 += g[i][j];
                    s2 += g[i][j] * xh[i][j];
                    adw[i][j] += d[j] * xh[i][j];
                    adb[i][j] += d[j];
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
                    float t[8];
                    load8(gh + (long)row * E + c * 8, t);
#pragma unroll
                    for (int j = 0; j < 8; ++j) o[j] += t[j];
                }
                store8(dx + (long)row * E + c * 8, o);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int c = lane + i * 64;
        if (c < nvec) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                pdw[(long)wave * E + c * 8 + j] = adw[i][j];
                pdb[(long)wave * E + c * 8 + j] = adb[i][j];
            }
        }
    }
}

}  // namespace

extern "C" {

int rn_ln_nv(int E) { return (E / 8 + 63) / 64; }

int rn_ln_fwd(const void* x, const void* r, const void* w, const void* b, void* y, void* h, float* mean,
              float* rstd, int M, int E, float eps, hipStream_t st) {
    if (E % 8 != 0 || E > 8192) return -1;
    int nv = rn_ln_nv(E);
    dim3 grid((M + 3) / 4);
#define RN_LNF(NV, R, B) ln_fwd_k<NV, R, B><<<grid, 256, 0, st>>>((const bf16*)x, (const bf16*)r, (const bf16*)w, (const bf16*)b, (bf16*)y, (bf16*)h, mean, rstd, M, E, eps)
#define RN_LNF2(NV) { if (r) { if (b) RN_LNF(NV, true, true); else RN_LNF(NV, true, false); } \
                      else { if (b) RN_LNF(NV, false, true); else RN_LNF(NV, false, false); } }
    if (nv <= 1) RN_LNF2(1) else if (nv <= 2) RN_LNF2(2) else if (nv <= 4) RN_LNF2(4) else if (nv <= 8) RN_LNF2(8)
    else RN_LNF2(16)
#undef RN_LNF2
#undef RN_LNF
    return 0;
}

int rn_ln_bwd_waves(int M) { int W = M < 2048 ? M : 2048; return ((W + 3) / 4) * 4; }

// pdw/pdb workspace: rn_ln_bwd_waves(M) * E floats each.
long rn_ln_bwd_ws(int M, int E) { return 2L * rn_ln_bwd_waves(M) * E + 2L * RN_COLRED_S * E; }

// ws: rn_ln_bwd_ws(M, E) floats.  dw/db (fp32) and dw16/db16 (bf16) outputs, any may be null.
int rn_ln_bwd(const void* dy, const void* gh, const void* h, const void* w, const float* mean, const float* rstd,
              void* dx, float* dw, float* db, void* dw16, void* db16, float* ws, int M, int E, int accum,
              hipStream_t st) {
    float* pdw = ws;
    float* pdb = ws + (long)rn_ln_bwd_waves(M) * E;
    if (E % 8 != 0 || E > 8192) return -1;
    int nv = rn_ln_nv(E);
    int W = rn_ln_bwd_waves(M);
    dim3 grid(W / 4);
#define RN_LNB(NV, G) ln_bwd_k<NV, G><<<grid, 256, 0, st>>>((const bf16*)dy, (const bf16*)gh, (const bf16*)h, (const bf16*)w, mean, rstd, (bf16*)dx, pdw, pdb, M, E)
#define RN_LNB2(NV) { if (gh) RN_LNB(NV, true); else RN_LNB(NV, false); }
    if (nv <= 1) RN_LNB2(1) else if (nv <= 2) RN_LNB2(2) else if (nv <= 4) RN_LNB2(4) else if (nv <= 8) RN_LNB2(8)
    else RN_LNB2(16)
#undef RN_LNB2
#undef RN_LNB
    // pdw/pdb are followed by 2 * RN_COLRED_S * E floats of scratch (see rn_ln_bwd_ws)
    float* tmp = pdb + (long)W * E;
    rn_colreduce(pdw, W, E, tmp, dw, (bf16*)dw16, st, accum);
    rn_colreduce(pdb, W, E, tmp + RN_COLRED_S * E, db, (bf16*)db16, st, accum);
    return 0;
}

}  // extern "C"
