// Convolution support for NHWC bf16 (N10/N11): im2col / col2im for the MFMA
// GEMM, BatchNorm (training statistics, fused ReLU) and pooling.
//
// im2col writes cols[(n,oh,ow)][(kh,kw,c)] with K zero-padded to Kp (multiple
// of 8) so every GEMM row is 16-B aligned; when C % 8 == 0 each lane moves one
// 16-byte channel chunk.  col2im is a gather (each input pixel sums the column
// entries that read it): deterministic, no atomics.
#include "common.h"

namespace {

__global__ void __launch_bounds__(256) im2col_k(const bf16* __restrict__ x, bf16* __restrict__ cols, int N, int H,
                                                int W, int C, int KH, int KW, int S, int P, int OH, int OW, int Kp,
                                                int vec) {
    const int cw = vec ? C / 8 : C;           // channel work items per (kh, kw)
    const long per_row = (long)KH * KW * cw;
    const long rowsK = (long)N * OH * OW;
    const long total = rowsK * per_row;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const long row = i / per_row;
        const int rem = i % per_row;
        const int kk = rem / cw, cc = rem % cw;
        const int kh = kk / KW, kw = kk % KW;
        const int ow = row % OW;
        const long t = row / OW;
        const int oh = t % OH, n = t / OH;
        const int ih = oh * S - P + kh, iw = ow * S - P + kw;
        const bool ok = ih >= 0 && ih < H && iw >= 0 && iw < W;
        bf16* dst = cols + row * Kp + (long)kk * C;
        if (vec) {
            s16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
            if (ok) v = *reinterpret_cast<const s16x8*>(x + (((long)n * H + ih) * W + iw) * C + cc * 8);
            *reinterpret_cast<s16x8*>(dst + cc * 8) = v;
        } else {
            dst[cc] = ok ? x[(((long)n * H + ih) * W + iw) * C + cc] : (bf16)0.f;
        }
    }
    // zero the K padding columns
    const int pad = Kp - KH * KW * C;
    if (pad > 0) {
        for (long i = blockIdx.x * 256L + threadIdx.x; i < rowsK * pad; i += (long)gridDim.x * 256)
            cols[(i / pad) * Kp + KH * KW * C + (i % pad)] = (bf16)0.f;
    }
}

__global__ void __launch_bounds__(256) col2im_k(const bf16* __restrict__ dcols, bf16* __restrict__ dx, int N, int H,
                                                int W, int C, int KH, int KW, int S, int P, int OH, int OW, int Kp) {
    const long total = (long)N * H * W * C;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c = i % C;
        long t = i / C;
        const int w = t % W;
        t /= W;
        const int h = t % H, n = t / H;
        float acc = 0.f;
        for (int kh = 0; kh < KH; ++kh) {
            const int oh_s = h + P - kh;
            if (oh_s < 0 || oh_s % S) continue;
            const int oh = oh_s / S;
            if (oh >= OH) continue;
            for (int kw = 0; kw < KW; ++kw) {
                const int ow_s = w + P - kw;
                if (ow_s < 0 || ow_s % S) continue;
                const int ow = ow_s / S;
                if (ow >= OW) continue;
                acc += bf2f(dcols[(((long)n * OH + oh) * OW + ow) * Kp + (kh * KW + kw) * C + c]);
            }
        }
        dx[i] = f2bf(acc);
    }
}

__global__ void __launch_bounds__(256) maxpool_fwd_k(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int H,
                                                     int W, int C, int K, int S, int P, int OH, int OW) {
    const long total = (long)N * OH * OW * C;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c = i % C;
        long t = i / C;
        const int ow = t % OW;
        t /= OW;
        const int oh = t % OH, n = t / OH;
        float m = -INFINITY;
        for (int kh = 0; kh < K; ++kh)
            for (int kw = 0; kw < K; ++kw) {
                const int ih = oh * S - P + kh, iw = ow * S - P + kw;
                if (ih >= 0 && ih < H && iw >= 0 && iw < W) m = fmaxf(m, bf2f(x[(((long)n * H + ih) * W + iw) * C + c]));
            }
        y[i] = f2bf(m);
    }
}

// gradient goes to the FIRST maximum of each window in scan order (matches ATen)
__global__ void __launch_bounds__(256) maxpool_bwd_k(const bf16* __restrict__ gy, const bf16* __restrict__ x,
                                                     const bf16* __restrict__ y, bf16* __restrict__ dx, int N, int H,
                                                     int W, int C, int K, int S, int P, int OH, int OW) {
    const long total = (long)N * H * W * C;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c = i % C;
        long t = i / C;
        const int w = t % W;
        t /= W;
        const int h = t % H, n = t / H;
        float acc = 0.f;
        for (int oh = max(0, (h + P - K + S) / S); oh <= min(OH - 1, (h + P) / S); ++oh)
            for (int ow = max(0, (w + P - K + S) / S); ow <= min(OW - 1, (w + P) / S); ++ow) {
                const long oi = (((long)n * OH + oh) * OW + ow) * C + c;
                const float ym = bf2f(y[oi]);
                // first argmax in the window
                int fh = -1, fw = -1;
                for (int kh = 0; kh < K && fh < 0; ++kh)
                    for (int kw = 0; kw < K; ++kw) {
                        const int ih = oh * S - P + kh, iw = ow * S - P + kw;
                        if (ih >= 0 && ih < H && iw >= 0 && iw < W && bf2f(x[(((long)n * H + ih) * W + iw) * C + c]) == ym) {
                            fh = ih; fw = iw;
                            break;
                        }
                    }
                if (fh == h && fw == w) acc += bf2f(gy[oi]);
            }
        dx[i] = f2bf(acc);
    }
}

__global__ void __launch_bounds__(256) avgpool_fwd_k(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int HW,
                                                     int C) {
    const long total = (long)N * C;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c = i % C, n = i / C;
        float s = 0.f;
        for (int p = 0; p < HW; ++p) s += bf2f(x[((long)n * HW + p) * C + c]);
        y[i] = f2bf(s / HW);
    }
}

__global__ void __launch_bounds__(256) avgpool_bwd_k(const bf16* __restrict__ gy, bf16* __restrict__ dx, int N, int HW,
                                                     int C) {
    const long total = (long)N * HW * C;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c = i % C;
        const long n = i / ((long)HW * C);
        dx[i] = f2bf(bf2f(gy[n * C + c]) / HW);
    }
}

// ---- BatchNorm on [M rows][C channels] ----
// column partial sums of f(row, c) over row splits.  MODE 0: (x, x^2)
// MODE 1: (dy', dy' * xhat) with dy' = dy * relu'(y)
template <int MODE>
__global__ void __launch_bounds__(256) bn_colsum_k(const bf16* __restrict__ a, const bf16* __restrict__ b,
                                                  const bf16* __restrict__ yv, const float* __restrict__ mean,
                                                  const float* __restrict__ rstd, float* __restrict__ p0,
                                                  float* __restrict__ p1, int M, int C, int rps, int relu) {
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int wv = threadIdx.x >> 6;
    const int r0 = blockIdx.y * rps, r1 = min(M, r0 + rps);
    __shared__ float s0[4][64], s1[4][64];
    float a0 = 0.f, a1 = 0.f;
    if (c < C) {
        const float mu = MODE ? mean[c] : 0.f, rs = MODE ? rstd[c] : 0.f;
        for (int r = r0 + wv; r < r1; r += 4) {
            const long e = (long)r * C + c;
            if (MODE == 0) {
                const float v = bf2f(a[e]);
                a0 += v;
                a1 += v * v;
            } else {
                float g = bf2f(a[e]);
                if (relu && bf2f(yv[e]) <= 0.f) g = 0.f;
                a0 += g;
                a1 += g * (bf2f(b[e]) - mu) * rs;
            }
        }
    }
    s0[wv][threadIdx.x & 63] = a0;
    s1[wv][threadIdx.x & 63] = a1;
    __syncthreads();
    if (wv == 0 && c < C) {
        p0[(long)blockIdx.y * C + c] = s0[0][threadIdx.x] + s0[1][threadIdx.x] + s0[2][threadIdx.x] + s0[3][threadIdx.x];
        p1[(long)blockIdx.y * C + c] = s1[0][threadIdx.x] + s1[1][threadIdx.x] + s1[2][threadIdx.x] + s1[3][threadIdx.x];
    }
}

__global__ void bn_stats_k(const float* __restrict__ p0, const float* __restrict__ p1, int S, int C, int M,
                           float eps, float mom, float* __restrict__ mean, float* __restrict__ rstd,
                           float* __restrict__ rmean, float* __restrict__ rvar) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float s = 0.f, q = 0.f;
    for (int i = 0; i < S; ++i) { s += p0[(long)i * C + c]; q += p1[(long)i * C + c]; }
    const float mu = s / M;
    const float var = fmaxf(q / M - mu * mu, 0.f);
    mean[c] = mu;
    rstd[c] = rsqrtf(var + eps);
    if (rmean) {
        rmean[c] = (1.f - mom) * rmean[c] + mom * mu;
        rvar[c] = (1.f - mom) * rvar[c] + mom * var * (M > 1 ? (float)M / (M - 1) : 1.f);
    }
}

__global__ void bn_gsum_k(const float* __restrict__ p0, const float* __restrict__ p1, int S, int C,
                          float* __restrict__ db, float* __restrict__ dw) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float s = 0.f, q = 0.f;
    for (int i = 0; i < S; ++i) { s += p0[(long)i * C + c]; q += p1[(long)i * C + c]; }
    db[c] = s;
    dw[c] = q;
}

__global__ void __launch_bounds__(256) bn_apply_k(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                  const bf16* __restrict__ b, const float* __restrict__ mean,
                                                  const float* __restrict__ rstd, bf16* __restrict__ y, long total,
                                                  int C, int relu) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c = i % C;
        float v = (bf2f(x[i]) - mean[c]) * rstd[c] * bf2f(w[c]) + bf2f(b[c]);
        if (relu) v = fmaxf(v, 0.f);
        y[i] = f2bf(v);
    }
}

// eval mode: running statistics
__global__ void __launch_bounds__(256) bn_eval_k(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                 const bf16* __restrict__ b, const float* __restrict__ rm,
                                                 const float* __restrict__ rv, bf16* __restrict__ y, long total, int C,
                                                 float eps, int relu) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c = i % C;
        float v = (bf2f(x[i]) - rm[c]) * rsqrtf(rv[c] + eps) * bf2f(w[c]) + bf2f(b[c]);
        if (relu) v = fmaxf(v, 0.f);
        y[i] = f2bf(v);
    }
}

__global__ void __launch_bounds__(256) bn_bwd_apply_k(const bf16* __restrict__ gy, const bf16* __restrict__ x,
                                                      const bf16* __restrict__ yv, const bf16* __restrict__ w,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      const float* __restrict__ db, const float* __restrict__ dw,
                                                      bf16* __restrict__ dx, long total, int C, int M, int relu) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c = i % C;
        float g = bf2f(gy[i]);
        if (relu && bf2f(yv[i]) <= 0.f) g = 0.f;
        const float xh = (bf2f(x[i]) - mean[c]) * rstd[c];
        const float v = bf2f(w[c]) * rstd[c] * (g - db[c] / M - xh * dw[c] / M);
        dx[i] = f2bf(v);
    }
}

inline int gridn(long n) {
    long g = (n + 255) / 256;
    return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

inline int bn_splits(int M, int C) {
    int cb = (C + 63) / 64, s = 1;
    while (cb * s < 1024 && M / (s * 2) >= 64) s *= 2;
    return s;
}

}  // namespace

extern "C" {

void rn_im2col(const void* x, void* cols, int N, int H, int W, int C, int KH, int KW, int S, int P, int OH, int OW,
               int Kp, hipStream_t st) {
    const int vec = (C % 8 == 0);
    long total = (long)N * OH * OW * KH * KW * (vec ? C / 8 : C);
    im2col_k<<<gridn(total), 256, 0, st>>>((const bf16*)x, (bf16*)cols, N, H, W, C, KH, KW, S, P, OH, OW, Kp, vec);
}

void rn_col2im(const void* dcols, void* dx, int N, int H, int W, int C, int KH, int KW, int S, int P, int OH, int OW,
               int Kp, hipStream_t st) {
    col2im_k<<<gridn((long)N * H * W * C), 256, 0, st>>>((const bf16*)dcols, (bf16*)dx, N, H, W, C, KH, KW, S, P, OH, OW, Kp);
}

void rn_maxpool_fwd(const void* x, void* y, int N, int H, int W, int C, int K, int S, int P, int OH, int OW,
                    hipStream_t st) {
    maxpool_fwd_k<<<gridn((long)N * OH * OW * C), 256, 0, st>>>((const bf16*)x, (bf16*)y, N, H, W, C, K, S, P, OH, OW);
}

void rn_maxpool_bwd(const void* gy, const void* x, const void* y, void* dx, int N, int H, int W, int C, int K, int S,
                    int P, int OH, int OW, hipStream_t st) {
    maxpool_bwd_k<<<gridn((long)N * H * W * C), 256, 0, st>>>((const bf16*)gy, (const bf16*)x, (const bf16*)y,
                                                               (bf16*)dx, N, H, W, C, K, S, P, OH, OW);
}

void rn_avgpool_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st) {
    avgpool_fwd_k<<<gridn((long)N * C), 256, 0, st>>>((const bf16*)x, (bf16*)y, N, HW, C);
}

void rn_avgpool_bwd(const void* gy, void* dx, int N, int HW, int C, hipStream_t st) {
    avgpool_bwd_k<<<gridn((long)N * HW * C), 256, 0, st>>>((const bf16*)gy, (bf16*)dx, N, HW, C);
}

long rn_bn_ws_floats(int M, int C) { return 2L * bn_splits(M, C) * C; }

void rn_bn_fwd(const void* x, const void* w, const void* b, float* rmean, float* rvar, void* y, float* mean,
               float* rstd, float* ws, int M, int C, float mom, float eps, int relu, hipStream_t st) {
    const int S = bn_splits(M, C);
    const int rps = (M + S - 1) / S;
    dim3 g((C + 63) / 64, S);
    bn_colsum_k<0><<<g, 256, 0, st>>>((const bf16*)x, nullptr, nullptr, nullptr, nullptr, ws, ws + (long)S * C, M, C,
                                      rps, 0);
    bn_stats_k<<<(C + 255) / 256, 256, 0, st>>>(ws, ws + (long)S * C, S, C, M, eps, mom, mean, rstd, rmean, rvar);
    bn_apply_k<<<gridn((long)M * C), 256, 0, st>>>((const bf16*)x, (const bf16*)w, (const bf16*)b, mean, rstd,
                                                    (bf16*)y, (long)M * C, C, relu);
}

void rn_bn_eval(const void* x, const void* w, const void* b, const float* rmean, const float* rvar, void* y, int M,
                int C, float eps, int relu, hipStream_t st) {
    bn_eval_k<<<gridn((long)M * C), 256, 0, st>>>((const bf16*)x, (const bf16*)w, (const bf16*)b, rmean, rvar,
                                                   (bf16*)y, (long)M * C, C, eps, relu);
}

// dw/db: fp32 outputs [C]
void rn_bn_bwd(const void* gy, const void* x, const void* y, const void* w, const float* mean, const float* rstd,
               void* dx, float* dw, float* db, float* ws, int M, int C, int relu, hipStream_t st) {
    const int S = bn_splits(M, C);
    const int rps = (M + S - 1) / S;
    dim3 g((C + 63) / 64, S);
    bn_colsum_k<1><<<g, 256, 0, st>>>((const bf16*)gy, (const bf16*)x, (const bf16*)y, mean, rstd, ws,
                                      ws + (long)S * C, M, C, rps, relu);
    bn_gsum_k<<<(C + 255) / 256, 256, 0, st>>>(ws, ws + (long)S * C, S, C, db, dw);
    bn_bwd_apply_k<<<gridn((long)M * C), 256, 0, st>>>((const bf16*)gy, (const bf16*)x, (const bf16*)y,
                                                        (const bf16*)w, mean, rstd, db, dw, (bf16*)dx, (long)M * C, C,
                                                        M, relu);
}

}  // extern "C"
