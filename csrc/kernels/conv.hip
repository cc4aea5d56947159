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

// im2col for C % 8 != 0 (the 7×7×3 stem): one lane per 16-B chunk (8 consecutive k) of a
// cols row, so every store is a whole 16 B and the row index is decoded once per chunk instead
// of per element; the 8 taps of a chunk are walked incrementally (c, then kw, then kh).
__global__ void __launch_bounds__(256) im2col_chunk_k(const bf16* __restrict__ x, bf16* __restrict__ cols, int N,
                                                      int H, int W, int C, int KH, int KW, int S, int P, int OH,
                                                      int OW, int Kp) {
    const int chunks = Kp / 8, K = KH * KW * C;
    const long total = (long)N * OH * OW * chunks;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const long row = i / chunks;
        const int k0 = (int)(i - row * chunks) * 8;
        const int ow = row % OW;
        const long t = row / OW;
        const int oh = t % OH, n = t / OH;
        int kk = k0 / C, c = k0 - kk * C;
        int kh = kk / KW, kw = kk - kh * KW;
        const bf16* xn = x + (long)n * H * W * C;
        s16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            short val = 0;
            const int ih = oh * S - P + kh, iw = ow * S - P + kw;
            if (k0 + e < K && ih >= 0 && ih < H && iw >= 0 && iw < W)
                val = __builtin_bit_cast(short, xn[((long)ih * W + iw) * C + c]);
            v[e] = val;
            if (++c == C) {
                c = 0;
                if (++kw == KW) kw = 0, ++kh;
            }
        }
        *reinterpret_cast<s16x8*>(cols + row * Kp + k0) = v;
    }
}

// im2col for C % 8 != 0 with the KH input rows of one output row staged in LDS (the 7×7×3 stem):
// block = (image, output row).  The KH rows (W + 2P pixels incl. the zero border, C channels) are
// read once with coalesced loads; each lane then writes whole 16-B chunks of a cols row from LDS
// (k = (kh·KW + kw)·C + c reads row kh at pixel ow·S + kw, i.e. a contiguous run of KW·C elements
// per kh).  The per-chunk gather of im2col_chunk_k issued 8 dependent 2-byte global loads instead.
__global__ void __launch_bounds__(256) im2col_rows_k(const bf16* __restrict__ x, bf16* __restrict__ cols, int N,
                                                     int H, int W, int C, int KH, int KW, int S, int P, int OH,
                                                     int OW, int Kp) {
    // [KH][RS] rows: padded row element r at lead + r, with lead chosen so the unpadded part starts
    // 16-B aligned (its fill is 16-B loads / ds_write_b128 when W·C % 8 == 0)
    extern __shared__ __attribute__((aligned(16))) short srow[];
    const int oh = blockIdx.x % OH, n = blockIdx.x / OH;
    const int WPC = (W + 2 * P) * C, PC = P * C, WC = W * C;
    const int lead = (8 - PC % 8) % 8, RS = (lead + WPC + 7) / 8 * 8;
    const bool vec = WC % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    const bf16* xn = x + (long)n * H * W * C;
    for (int kh = 0; kh < KH; ++kh) {
        const int ih = oh * S - P + kh;
        short* dst = srow + kh * RS + lead;
        if (ih < 0 || ih >= H) {
            for (int r = threadIdx.x; r < WPC; r += 256) dst[r] = 0;
            continue;
        }
        const bf16* xr = xn + (long)ih * W * C;
        for (int r = threadIdx.x; r < PC; r += 256) {
            dst[r] = 0;
            dst[PC + WC + r] = 0;
        }
        if (vec) {
            for (int q = threadIdx.x; q < WC / 8; q += 256)
                *reinterpret_cast<s16x8*>(dst + PC + 8 * q) = *reinterpret_cast<const s16x8*>(xr + 8 * q);
        } else {
            for (int e = threadIdx.x; e < WC; e += 256) dst[PC + e] = __builtin_bit_cast(short, xr[e]);
        }
    }
    __syncthreads();
    const int chunks = Kp / 8, K = KH * KW * C, KWC = KW * C;
    bf16* crow = cols + (long)(n * OH + oh) * OW * Kp;
    for (int i = threadIdx.x; i < OW * chunks; i += 256) {
        const int ow = i / chunks;
        const int k0 = (i - ow * chunks) * 8;
        int kh = k0 / KWC, j = k0 - kh * KWC;
        const int base = ow * S * C;
        s16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            v[e] = (k0 + e < K) ? srow[kh * RS + lead + base + j] : (short)0;
            if (++j == KWC) j = 0, ++kh;
        }
        *reinterpret_cast<s16x8*>(crow + (long)ow * Kp + k0) = v;
    }
}

// col2im gather for C % 8 == 0: one lane per (pixel, 8-channel chunk), 16-B loads/stores, only
// the taps whose output position exists (stride-aligned) are visited.
// accumulate: dx += the gathered sum (the other gradient of a tensor read by two ops, e.g. ResNet's
// shortcut, added in this pass instead of by a separate add kernel).
__global__ void __launch_bounds__(256) col2im_vec_k(const bf16* __restrict__ dcols, bf16* __restrict__ dx, int N,
                                                    int H, int W, int C, int KH, int KW, int S, int P, int OH,
                                                    int OW, int Kp, int accumulate) {
    const int CV = C / 8;
    const long total = (long)N * H * W * CV;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int cv = i % CV;
        long t = i / CV;
        const int w = t % W;
        t /= W;
        const int h = t % H, n = t / H;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (accumulate) load8(dx + i * 8, acc);
        // first kh with (h + P - kh) % S == 0, then every S-th
        for (int kh = (h + P) % S; kh < KH; kh += S) {
            const int oh = (h + P - kh) / S;
            if (h + P - kh < 0) break;
            if (oh >= OH) continue;
            for (int kw = (w + P) % S; kw < KW; kw += S) {
                if (w + P - kw < 0) break;
                const int ow = (w + P - kw) / S;
                if (ow >= OW) continue;
                float v[8];
                load8(dcols + (((long)n * OH + oh) * OW + ow) * Kp + (kh * KW + kw) * C + cv * 8, v);
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[e] += v[e];
            }
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16)acc[e];
        *reinterpret_cast<bf16x8*>(dx + i * 8) = o;
    }
}

__global__ void __launch_bounds__(256) col2im_k(const bf16* __restrict__ dcols, bf16* __restrict__ dx, int N, int H,
                                                int W, int C, int KH, int KW, int S, int P, int OH, int OW, int Kp,
                                                int accumulate) {
    const long total = (long)N * H * W * C;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int c = i % C;
        long t = i / C;
        const int w = t % W;
        t /= W;
        const int h = t % H, n = t / H;
        float acc = accumulate ? bf2f(dx[i]) : 0.f;
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

// Max-pool, NHWC, V channels per thread (V = 8: one 16-B load per window tap; V = 1 for C % 8 != 0).
// The forward also writes the window position (kh·K + kw, one byte per output element) of the
// FIRST maximum in scan order (ATen's tie rule), so the backward is a gather of at most
// ceil(K/S)² gradient values per input element — no window re-scan, no atomics.
template <int V>
__global__ void __launch_bounds__(256) maxpool_fwd_k(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                     uint8_t* __restrict__ idx, int N, int H, int W, int C, int K,
                                                     int S, int P, int OH, int OW) {
    const int CV = C / V;
    const long total = (long)N * OH * OW * CV;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int cv = i % CV;
        long t = i / CV;
        const int ow = t % OW;
        t /= OW;
        const int oh = t % OH, n = t / OH;
        float m[V];
        int am[V];
#pragma unroll
        for (int j = 0; j < V; ++j) { m[j] = -INFINITY; am[j] = 0; }
        for (int kh = 0; kh < K; ++kh) {
            const int ih = oh * S - P + kh;
            if (ih < 0 || ih >= H) continue;
            for (int kw = 0; kw < K; ++kw) {
                const int iw = ow * S - P + kw;
                if (iw < 0 || iw >= W) continue;
                const bf16* src = x + (((long)n * H + ih) * W + iw) * C + cv * V;
                float v[V];
                if constexpr (V == 8) load8(src, v);
                else v[0] = bf2f(src[0]);
#pragma unroll
                for (int j = 0; j < V; ++j)
                    if (v[j] > m[j]) { m[j] = v[j]; am[j] = kh * K + kw; }
            }
        }
        const long o = (((long)n * OH + oh) * OW + ow) * C + cv * V;
        if constexpr (V == 8) {
            store8(y + o, m);
            uint2 packed;
            packed.x = (uint32_t)am[0] | ((uint32_t)am[1] << 8) | ((uint32_t)am[2] << 16) | ((uint32_t)am[3] << 24);
            packed.y = (uint32_t)am[4] | ((uint32_t)am[5] << 8) | ((uint32_t)am[6] << 16) | ((uint32_t)am[7] << 24);
            *reinterpret_cast<uint2*>(idx + o) = packed;
        } else {
            y[o] = f2bf(m[0]);
            idx[o] = (uint8_t)am[0];
        }
    }
}

template <int V>
__global__ void __launch_bounds__(256) maxpool_bwd_k(const bf16* __restrict__ gy, const uint8_t* __restrict__ idx,
                                                     bf16* __restrict__ dx, int N, int H, int W, int C, int K, int S,
                                                     int P, int OH, int OW) {
    const int CV = C / V;
    const long total = (long)N * H * W * CV;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int cv = i % CV;
        long t = i / CV;
        const int w = t % W;
        t /= W;
        const int h = t % H, n = t / H;
        float acc[V];
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = 0.f;
        for (int oh = max(0, (h + P - K + S) / S); oh <= min(OH - 1, (h + P) / S); ++oh)
            for (int ow = max(0, (w + P - K + S) / S); ow <= min(OW - 1, (w + P) / S); ++ow) {
                const int pos = (h + P - oh * S) * K + (w + P - ow * S);  // this input's place in the window
                const long oi = (((long)n * OH + oh) * OW + ow) * C + cv * V;
                if constexpr (V == 8) {
                    const uint2 a = *reinterpret_cast<const uint2*>(idx + oi);
                    float g[8];
                    load8(gy + oi, g);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint32_t b = ((j < 4 ? a.x : a.y) >> (8 * (j & 3))) & 0xFF;
                        if ((int)b == pos) acc[j] += g[j];
                    }
                } else {
                    if ((int)idx[oi] == pos) acc[0] += bf2f(gy[oi]);
                }
            }
        const long o = (((long)n * H + h) * W + w) * C + cv * V;
        if constexpr (V == 8) store8(dx + o, acc);
        else dx[o] = f2bf(acc[0]);
    }
}

// Max-pool backward, 8 channels per lane, one input row per grid row: blockIdx.y = (n, h), so the
// output-row window of the row (oh range) is uniform across the block and the per-lane index math is
// one division by the channel-chunk count (was four runtime divisions per chunk in maxpool_bwd_k).
__global__ void __launch_bounds__(256) maxpool_bwd_rows_k(const bf16* __restrict__ gy, const uint8_t* __restrict__ idx,
                                                          bf16* __restrict__ dx, int H, int W, int C, int K, int S,
                                                          int P, int OH, int OW) {
    const int CV = C / 8;
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= W * CV) return;
    const int w = j / CV, cv = j - w * CV;
    const int n = blockIdx.y / H, h = blockIdx.y - n * H;
    const int oh0 = max(0, (h + P - K + S) / S), oh1 = min(OH - 1, (h + P) / S);
    const int ow0 = max(0, (w + P - K + S) / S), ow1 = min(OW - 1, (w + P) / S);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int oh = oh0; oh <= oh1; ++oh)
        for (int ow = ow0; ow <= ow1; ++ow) {
            const int pos = (h + P - oh * S) * K + (w + P - ow * S);  // this input's place in the window
            const long oi = (((long)n * OH + oh) * OW + ow) * C + cv * 8;
            const uint2 a = *reinterpret_cast<const uint2*>(idx + oi);
            float g[8];
            load8(gy + oi, g);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const uint32_t b = ((e < 4 ? a.x : a.y) >> (8 * (e & 3))) & 0xFF;
                if ((int)b == pos) acc[e] += g[e];
            }
        }
    store8(dx + (((long)n * H + h) * W + w) * C + cv * 8, acc);
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

// ---- BatchNorm on [M rows][C channels] (NHWC flattened) ----
// Training statistics in two deterministic steps:
//   bn_part_k    grid S row-splits × 256 threads; thread t owns channel group t % (C/8) (8 channels,
//                16-B loads) and rows t / (C/8) + k·(256·8/C); per-split partials → part[S][2C]
//                (MODE 0: Σx | Σx² ; MODE 1: Σg' | Σg'·x̂ with g' = dy masked by the fused ReLU)
//   rn_colreduce_seg (common.h) sums the S partial rows in fixed order → [2C] fp32,
//   bn_finalize_k turns the forward sums into mean / rstd / running statistics.
// Apply kernels are 8 channels per thread.  An optional residual input is fused into the forward
// apply (y = relu(BN(x) + res)); the backward then also returns g' = dy ⊙ relu'(y), the residual
// branch's gradient.  With ReLU the training forward also writes relu'(y) as a bit mask (one byte
// per 8 channels of a row, 1/16 of y's bytes), which both backward passes read instead of y.
// C % 8 == 0 and C ≤ 2048 (all of ResNet-18).
constexpr int BN_T = 256;

template <int MODE>
__global__ void __launch_bounds__(BN_T) bn_part_k(const bf16* __restrict__ a, const bf16* __restrict__ xin,
                                                  const uint8_t* __restrict__ mk, const float* __restrict__ mean,
                                                  const float* __restrict__ rstd, float* __restrict__ part, int M,
                                                  int C, int rps, int relu) {
    __shared__ float red[2][BN_T * 8];
    const int CG = C / 8;
    const int t = threadIdx.x;
    const int cg = t % CG, ro = t / CG, rpi = BN_T / CG;  // threads t >= rpi*CG idle (CG ∤ 256)
    const int r0 = blockIdx.x * rps, r1 = min(M, r0 + rps);
    float s0[8], s1[8], mu[8], rs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { s0[j] = 0.f; s1[j] = 0.f; mu[j] = 0.f; rs[j] = 0.f; }
    const bool active = ro < rpi;
    if (MODE == 1 && active) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { mu[j] = mean[cg * 8 + j]; rs[j] = rstd[cg * 8 + j]; }
    }
    if (active) {
        // rows in batches of U: all U rows' loads are issued before any is accumulated (one memory
        // round trip per batch instead of per row: the loop was latency-bound at ~3 TB/s); the adds
        // stay in row order, so the sums do not depend on the batching
        constexpr int U = 4;
        for (int rb = r0 + ro; rb < r1; rb += U * rpi) {
            bf16x8 av[U], xvv[U];
            unsigned mm[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = min(rb + u * rpi, r1 - 1);  // clamped: no per-load branch
                const long e = (long)r * C + cg * 8;
                av[u] = *reinterpret_cast<const bf16x8*>(a + e);
                if (MODE == 1) {
                    xvv[u] = *reinterpret_cast<const bf16x8*>(xin + e);
                    mm[u] = relu ? (unsigned)mk[e >> 3] : 0xFFu;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (rb + u * rpi >= r1) break;
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (float)av[u][j];
                if (MODE == 0) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) { s0[j] += v[j]; s1[j] += v[j] * v[j]; }
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float g = ((mm[u] >> j) & 1u) ? v[j] : 0.f;
                        s0[j] += g;
                        s1[j] += g * ((float)xvv[u][j] - mu[j]) * rs[j];
                    }
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[0][t * 8 + j] = s0[j]; red[1][t * 8 + j] = s1[j]; }
    __syncthreads();
    // thread c < C: fixed-order sum over the row groups of its channel
    for (int c = t; c < C; c += BN_T) {
        const int g = c / 8, j = c % 8;
        float u0 = 0.f, u1 = 0.f;
        for (int k = 0; k < rpi; ++k) {
            u0 += red[0][(k * CG + g) * 8 + j];
            u1 += red[1][(k * CG + g) * 8 + j];
        }
        part[(long)blockIdx.x * 2 * C + c] = u0;
        part[(long)blockIdx.x * 2 * C + C + c] = u1;
    }
}

__global__ void bn_finalize_k(const float* __restrict__ sums, int C, int M, float eps, float mom,
                              float* __restrict__ mean, float* __restrict__ rstd, float* __restrict__ rmean,
                              float* __restrict__ rvar) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float mu = sums[c] / M;
    const float var = fmaxf(sums[C + c] / M - mu * mu, 0.f);
    mean[c] = mu;
    rstd[c] = rsqrtf(var + eps);
    if (rmean) {
        rmean[c] = (1.f - mom) * rmean[c] + mom * mu;
        rvar[c] = (1.f - mom) * rvar[c] + mom * var * (M > 1 ? (float)M / (M - 1) : 1.f);
    }
}

// y = [relu](BN(x) [+ res]); per-channel affine from (mean, rstd, w, b) or, in eval mode, running stats.
// The grid stride is a multiple of C/8 for every launch of ResNet-18 (powers of two), so a thread's
// channel group never changes: its 8 scale / shift pairs are computed once (recomputed only if the
// group does change) and each element costs one FMA; two grid-stride iterations are loaded together.
template <bool EVAL>
__global__ void __launch_bounds__(256) bn_apply_k(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                  const bf16* __restrict__ b, const float* __restrict__ mean,
                                                  const float* __restrict__ rstd, const bf16* __restrict__ res,
                                                  bf16* __restrict__ y, uint8_t* __restrict__ mk, long total8, int C,
                                                  float eps, int relu) {
    const int CG = C / 8;
    const long stride = (long)gridDim.x * 256;
    int cprev = -1;
    float sc[8], sh[8];
    auto affine = [&](int c0) {
        if (c0 == cprev) return;
        cprev = c0;
        float wf[8], bf[8];
        load8(w + c0, wf);
        load8(b + c0, bf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float r = EVAL ? rsqrtf(rstd[c0 + j] + eps) : rstd[c0 + j];  // eval: rstd holds running var
            sc[j] = r * wf[j];
            sh[j] = bf[j] - mean[c0 + j] * sc[j];
        }
    };
    auto out = [&](long i, const bf16x8& xv, const bf16x8& rv) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float o = __builtin_fmaf((float)xv[j], sc[j], sh[j]);
            if (res) o += (float)rv[j];
            v[j] = relu ? fmaxf(o, 0.f) : o;
        }
        store8(y + i * 8, v);
        if (mk) {  // relu'(y) of the stored (bf16) values
            unsigned m = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) m |= ((float)(bf16)v[j] > 0.f ? 1u : 0u) << j;
            mk[i] = (uint8_t)m;
        }
    };
    long i = blockIdx.x * 256L + threadIdx.x;
    for (; i + stride < total8; i += 2 * stride) {
        const long i2 = i + stride;
        const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(x + i * 8), x2 = *reinterpret_cast<const bf16x8*>(x + i2 * 8);
        bf16x8 r1 = x1, r2 = x2;
        if (res) {
            r1 = *reinterpret_cast<const bf16x8*>(res + i * 8);
            r2 = *reinterpret_cast<const bf16x8*>(res + i2 * 8);
        }
        affine((int)(i % CG) * 8);
        out(i, x1, r1);
        affine((int)(i2 % CG) * 8);
        out(i2, x2, r2);
    }
    if (i < total8) {
        const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(x + i * 8);
        const bf16x8 r1 = res ? *reinterpret_cast<const bf16x8*>(res + i * 8) : x1;
        affine((int)(i % CG) * 8);
        out(i, x1, r1);
    }
}

// dx = w·rstd·(g' − Σg'/M − x̂·Σ(g'x̂)/M), g' = dy ⊙ relu'(y); optionally g' itself (residual branch).
// Per channel that is dx = a·g' + k1·x + k0 (a = w·rstd, k1 = −a·rstd·Σ(g'x̂)/M,
// k0 = −a·Σg'/M − k1·mean): hoisted like the forward apply, two FMAs per element.
__global__ void __launch_bounds__(256) bn_bwd_apply_k(const bf16* __restrict__ gy, const bf16* __restrict__ x,
                                                      const uint8_t* __restrict__ mk, const bf16* __restrict__ w,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      const float* __restrict__ sums, bf16* __restrict__ dx,
                                                      bf16* __restrict__ gres, long total8, int C, int M, int relu) {
    const int CG = C / 8;
    const float invM = 1.f / M;
    const long stride = (long)gridDim.x * 256;
    int cprev = -1;
    float ka[8], k1[8], k0[8];
    auto coef = [&](int c0) {
        if (c0 == cprev) return;
        cprev = c0;
        float wf[8];
        load8(w + c0, wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = c0 + j;
            ka[j] = wf[j] * rstd[c];
            k1[j] = -ka[j] * rstd[c] * (sums[C + c] * invM);
            k0[j] = -ka[j] * (sums[c] * invM) - k1[j] * mean[c];
        }
    };
    auto out = [&](long i, const bf16x8& gv, const bf16x8& xv, unsigned m) {
        float g[8], o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            g[j] = (float)gv[j];
            if (relu) g[j] = ((m >> j) & 1u) ? g[j] : 0.f;
            o[j] = __builtin_fmaf(ka[j], g[j], __builtin_fmaf(k1[j], (float)xv[j], k0[j]));
        }
        if (gres) store8(gres + i * 8, g);
        store8(dx + i * 8, o);
    };
    long i = blockIdx.x * 256L + threadIdx.x;
    for (; i + stride < total8; i += 2 * stride) {
        const long i2 = i + stride;
        const bf16x8 g1 = *reinterpret_cast<const bf16x8*>(gy + i * 8), g2 = *reinterpret_cast<const bf16x8*>(gy + i2 * 8);
        const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(x + i * 8), x2 = *reinterpret_cast<const bf16x8*>(x + i2 * 8);
        const unsigned m1 = relu ? mk[i] : 0u, m2 = relu ? mk[i2] : 0u;
        coef((int)(i % CG) * 8);
        out(i, g1, x1, m1);
        coef((int)(i2 % CG) * 8);
        out(i2, g2, x2, m2);
    }
    if (i < total8) {
        const bf16x8 g1 = *reinterpret_cast<const bf16x8*>(gy + i * 8);
        const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(x + i * 8);
        coef((int)(i % CG) * 8);
        out(i, g1, x1, relu ? mk[i] : 0u);
    }
}

inline int gridn(long n) {
    long g = (n + 255) / 256;
    return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

inline int bn_splits(int M) {
    // >= 64 rows per split: the small late-layer tensors (12.5 k rows at layer 4) still fill the chip (M / 256
    // gave layer 4 only 49 workgroups: 19 us for 25 MB, profiles/resnet_vit_r5r.txt trace)
    int S = M / 64;
    return S < 1 ? 1 : (S > 1024 ? 1024 : S);
}

}  // namespace

extern "C" {

void rn_im2col(const void* x, void* cols, int N, int H, int W, int C, int KH, int KW, int S, int P, int OH, int OW,
               int Kp, hipStream_t st) {
    const int vec = (C % 8 == 0);
    const long rs = ((8 - (P * C) % 8) % 8 + (long)(W + 2 * P) * C + 7) / 8 * 8;  // im2col_rows_k's RS
    if (!vec && KH * rs * 2 <= 32768) {  // the KH input rows of one output row fit in LDS
        im2col_rows_k<<<N * OH, 256, KH * rs * 2, st>>>((const bf16*)x, (bf16*)cols, N, H, W, C, KH, KW,
                                                                      S, P, OH, OW, Kp);
        return;
    }
    if (!vec) {
        im2col_chunk_k<<<gridn((long)N * OH * OW * (Kp / 8)), 256, 0, st>>>((const bf16*)x, (bf16*)cols, N, H, W, C,
                                                                            KH, KW, S, P, OH, OW, Kp);
        return;
    }
    long total = (long)N * OH * OW * KH * KW * (C / 8);
    im2col_k<<<gridn(total), 256, 0, st>>>((const bf16*)x, (bf16*)cols, N, H, W, C, KH, KW, S, P, OH, OW, Kp, vec);
}

void rn_col2im(const void* dcols, void* dx, int N, int H, int W, int C, int KH, int KW, int S, int P, int OH, int OW,
               int Kp, int accumulate, hipStream_t st) {
    if (C % 8 == 0 && Kp % 8 == 0) {
        col2im_vec_k<<<gridn((long)N * H * W * C / 8), 256, 0, st>>>((const bf16*)dcols, (bf16*)dx, N, H, W, C, KH, KW,
                                                                      S, P, OH, OW, Kp, accumulate);
        return;
    }
    col2im_k<<<gridn((long)N * H * W * C), 256, 0, st>>>((const bf16*)dcols, (bf16*)dx, N, H, W, C, KH, KW, S, P, OH, OW,
                                                          Kp, accumulate);
}

// idx: one byte per output element (window position of the first maximum); K*K <= 256
void rn_maxpool_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int K, int S, int P, int OH,
                    int OW, hipStream_t st) {
    if (C % 8 == 0)
        maxpool_fwd_k<8><<<gridn((long)N * OH * OW * C / 8), 256, 0, st>>>((const bf16*)x, (bf16*)y, (uint8_t*)idx, N,
                                                                             H, W, C, K, S, P, OH, OW);
    else
        maxpool_fwd_k<1><<<gridn((long)N * OH * OW * C), 256, 0, st>>>((const bf16*)x, (bf16*)y, (uint8_t*)idx, N, H,
                                                                         W, C, K, S, P, OH, OW);
}

void rn_maxpool_bwd(const void* gy, const void* idx, void* dx, int N, int H, int W, int C, int K, int S, int P,
                    int OH, int OW, hipStream_t st) {
    if (C % 8 == 0 && (long)N * H < 65536) {
        maxpool_bwd_rows_k<<<dim3((W * (C / 8) + 255) / 256, N * H), 256, 0, st>>>(
            (const bf16*)gy, (const uint8_t*)idx, (bf16*)dx, H, W, C, K, S, P, OH, OW);
        return;
    }
    if (C % 8 == 0)
        maxpool_bwd_k<8><<<gridn((long)N * H * W * C / 8), 256, 0, st>>>((const bf16*)gy, (const uint8_t*)idx,
                                                                           (bf16*)dx, N, H, W, C, K, S, P, OH, OW);
    else
        maxpool_bwd_k<1><<<gridn((long)N * H * W * C), 256, 0, st>>>((const bf16*)gy, (const uint8_t*)idx, (bf16*)dx,
                                                                       N, H, W, C, K, S, P, OH, OW);
}

void rn_avgpool_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st) {
    avgpool_fwd_k<<<gridn((long)N * C), 256, 0, st>>>((const bf16*)x, (bf16*)y, N, HW, C);
}

void rn_avgpool_bwd(const void* gy, void* dx, int N, int HW, int C, hipStream_t st) {
    avgpool_bwd_k<<<gridn((long)N * HW * C), 256, 0, st>>>((const bf16*)gy, (bf16*)dx, N, HW, C);
}

// workspace floats: partials [S][2C] + reduced sums [2C] + the column reduction's scratch
long rn_bn_ws_floats(int M, int C) { return 2L * C * (bn_splits(M) + 1) + (long)RN_COLRED_S * 2 * C; }

static void bn_stats(int mode, const void* a, const void* xin, const uint8_t* mk, const float* mean, const float* rstd,
                     float* ws, int M, int C, int relu, void* db16, void* dw16, hipStream_t st, int accum16 = 0) {
    const int S = bn_splits(M);
    const int rps = (M + S - 1) / S;
    float* part = ws;
    float* sums = ws + 2L * C * S;
    float* tmp = sums + 2L * C;
    if (mode == 0)
        bn_part_k<0><<<S, BN_T, 0, st>>>((const bf16*)a, nullptr, nullptr, nullptr, nullptr, part, M, C, rps, 0);
    else
        bn_part_k<1><<<S, BN_T, 0, st>>>((const bf16*)a, (const bf16*)xin, mk, mean, rstd, part, M, C,
                                         rps, relu);
    const int a16 = accum16 ? 2 : 0;  // direct gradient accumulation: add into db16/dw16, never into sums
    RnColOut o{{sums, sums + C, nullptr}, {(__bf16*)db16, (__bf16*)dw16, nullptr}, C, {a16, a16, 0}};
    rn_colreduce_seg(part, S, 2 * C, tmp, o, st);
}

int rn_bn_supported(int C) { return C % 8 == 0 && C <= 2048; }

// res (optional): y = relu(BN(x) + res).  partials (optional): [prows][2C] Σx | Σx² row-block partials
// from x's producer (the implicit-conv GEMM epilogue): only their fixed-order column reduction runs,
// not a statistics pass over x.  mask (optional, with relu): [M·C/8] bytes of relu'(y) bits.
void rn_bn_fwd(const void* x, const void* w, const void* b, float* rmean, float* rvar, void* y, float* mean,
               float* rstd, float* ws, int M, int C, float mom, float eps, int relu, const void* res,
               const float* partials, int prows, void* mask, hipStream_t st) {
    if (partials) {
        float* sums = ws + 2L * C * bn_splits(M);
        RnColOut o{{sums, sums + C, nullptr}, {nullptr, nullptr, nullptr}, C, {0, 0, 0}};
        rn_colreduce_seg(partials, prows, 2 * C, sums + 2L * C, o, st);
    } else {
        bn_stats(0, x, nullptr, nullptr, nullptr, nullptr, ws, M, C, 0, nullptr, nullptr, st);
    }
    const float* sums = ws + 2L * C * bn_splits(M);
    bn_finalize_k<<<(C + 255) / 256, 256, 0, st>>>(sums, C, M, eps, mom, mean, rstd, rmean, rvar);
    const long t8 = (long)M * C / 8;
    bn_apply_k<false><<<gridn(t8), 256, 0, st>>>((const bf16*)x, (const bf16*)w, (const bf16*)b, mean, rstd,
                                                  (const bf16*)res, (bf16*)y, relu ? (uint8_t*)mask : nullptr, t8,
                                                  C, eps, relu);
}

void rn_bn_eval(const void* x, const void* w, const void* b, const float* rmean, const float* rvar, void* y, int M,
                int C, float eps, int relu, const void* res, hipStream_t st) {
    const long t8 = (long)M * C / 8;
    bn_apply_k<true><<<gridn(t8), 256, 0, st>>>((const bf16*)x, (const bf16*)w, (const bf16*)b, rmean, rvar,
                                                 (const bf16*)res, (bf16*)y, nullptr, t8, C, eps, relu);
}

// dw/db: bf16 outputs [C] (the parameter dtype, written by the reduction itself; with `accum` ADDED
// into them: the flat gradient buffer's views, no AccumulateGrad pass); gres (optional):
// dy ⊙ relu'(y), the gradient of a fused residual input; mask: the forward's relu'(y) bits (relu only)
void rn_bn_bwd(const void* gy, const void* x, const void* mask, const void* w, const float* mean, const float* rstd,
               void* dx, void* dw, void* db, float* ws, int M, int C, int relu, void* gres, int accum,
               hipStream_t st) {
    bn_stats(1, gy, x, (const uint8_t*)mask, mean, rstd, ws, M, C, relu, db, dw, st, accum);
    const float* sums = ws + 2L * C * bn_splits(M);
    const long t8 = (long)M * C / 8;
    bn_bwd_apply_k<<<gridn(t8), 256, 0, st>>>((const bf16*)gy, (const bf16*)x, (const uint8_t*)mask, (const bf16*)w, mean,
                                               rstd, sums, (bf16*)dx, (bf16*)gres, t8, C, M, relu);
}

}  // extern "C"
