// GEMM config 10: skinny-M forward GEMM for incremental decoding (M <= 64 token rows).
//
//   C[M][N] = epilogue(A[M][K] · W[N][K]ᵀ)      (the Linear forward layout: A and W K-contiguous)
//
// At decode sizes (M = batch rows, one new token each) the 256²/128² tile kernels leave almost the
// whole chip idle (GPT-2-small c_proj: 768 output columns = 6 tiles of 128) and walk K serially
// through LDS, so each launch is a chain of K/64 DMA round trips (≈ 25 µs measured per decode GEMM,
// profiles/decode_r4s.txt).  Here the work is cut along N AND K:
//   * one workgroup = 16 output columns × one K range; its 4 waves take interleaved 32-deep k-steps
//     of that range, so a launch has N/16 × S workgroups (S = K splits, picked by the autotuner);
//   * no LDS staging: for v_mfma_f32_16x16x32_bf16 lane l holds row (l & 15), k-run 8·(l >> 4) of
//     each operand — a 16-byte load straight from K-contiguous rows of A and W — so a k-step is
//     1 + MB global loads per lane and MB MFMAs (MB = ceil(M / 16) row blocks);
//   * the 4 waves' accumulators are summed through LDS in a fixed order; S = 1 applies the epilogue
//     right there, S > 1 writes fp32 partials [S][M][N] and skinny_fin_k sums them in split order
//     and applies it: deterministic, no atomics.
// Epilogue order as the tile kernels': ·alpha, +bias, activation (with the optional
// pre-activation / gelu' store of the bf16-rounded h), +residual.
//
// LN variant (rn_ln_gemm_skinny, the decode step's LayerNorm → projection pairs): A = LN(x) is never
// written — each workgroup first reduces its rows' mean / rstd (two passes over the row, as the
// LayerNorm kernel), then normalises every A fragment as it is loaded ((x − μ)·rstd·γ + β, rounded
// to bf16 like the stored LayerNorm output).  Saves one launch per LayerNorm of a decode step.
#include "common.h"

namespace {

struct SkArgs {
    const bf16* A;
    const bf16* W;
    void* C;
    const bf16* bias;
    const bf16* res;
    bf16* pre;
    float* ws;
    const float* alpha;
    int M, N, K, S, kc;  // kc: K range per split (multiple of 32)
    long lda, ldw, ldc;
    int out_f32;
    const bf16* ln_w;  // LN variant: γ, β (β optional), eps
    const bf16* ln_b;
    float eps;
};

template <int ACT>
RN_DEV void sk_store(const SkArgs& p, int m, int n, float v) {
    if (p.alpha) v *= *p.alpha;
    if (p.bias) v += (float)p.bias[n];
    if constexpr (act_fwd(ACT)) {
        if (p.pre) {
            float pv;
            v = act_fwd_pre<ACT>((float)(bf16)v, pv);
            p.pre[(long)m * p.ldc + n] = (bf16)pv;
        } else {
            v = act_f<ACT>(v);
        }
    }
    if (p.res) v += (float)p.res[(long)m * p.ldc + n];
    if (p.out_f32) reinterpret_cast<float*>(p.C)[(long)m * p.ldc + n] = v;
    else reinterpret_cast<bf16*>(p.C)[(long)m * p.ldc + n] = (bf16)v;
}

RN_DEV s16x8 sk_load(const bf16* base, long row_off, int k, int K, bool row_ok) {
    if (row_ok && k < K) return *reinterpret_cast<const s16x8*>(base + row_off + k);
    return (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
}

// LN(x) fragment: 8 consecutive k of one row, normalised with the row's (μ, rstd), rounded to bf16
RN_DEV s16x8 sk_load_ln(const SkArgs& p, long row_off, int k, int K, bool row_ok, float mu, float rs) {
    if (!(row_ok && k < K)) return (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
    float x[8], g[8], b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    load8(p.A + row_off + k, x);
    load8(p.ln_w + k, g);
    if (p.ln_b) load8(p.ln_b + k, b);
    s16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = __builtin_bit_cast(short, (bf16)((x[j] - mu) * rs * g[j] + b[j]));
    return o;
}

template <int MB, int ACT, bool LN = false>
__global__ void __launch_bounds__(256) skinny_k(SkArgs p) {
    __shared__ f32x4 red[4][MB][64];
    [[maybe_unused]] __shared__ float st_mu[64], st_rs[64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if constexpr (LN) {  // row statistics over the full K: 4 lanes per row, two passes (mean, then Σ(x−μ)²)
        const int row = threadIdx.x >> 2, part = threadIdx.x & 3, nch = p.K / 8;
        const bool ok = row < p.M;
        const bf16* xr = p.A + (long)(ok ? row : 0) * p.lda;
        float s = 0.f, f[8];
        for (int c = part; ok && c < nch; c += 4) {
            load8(xr + c * 8, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) s += f[j];
        }
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        const float mu = s / p.K;
        float q = 0.f;
        for (int c = part; ok && c < nch; c += 4) {
            load8(xr + c * 8, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) { const float d = f[j] - mu; q += d * d; }
        }
        q += __shfl_xor(q, 1, 64);
        q += __shfl_xor(q, 2, 64);
        if (part == 0) { st_mu[row] = mu; st_rs[row] = rsqrtf(q / p.K + p.eps); }
        __syncthreads();
    }
    const int n0 = blockIdx.x * 16, split = blockIdx.y;
    const int r = lane & 15, kg = 8 * (lane >> 4);
    const int k_lo = split * p.kc, k_hi = min(p.K, k_lo + p.kc);
    const int n = n0 + r;
    const long w_off = (long)min(n, p.N - 1) * p.ldw;
    long a_off[MB];
    bool a_ok[MB];
    [[maybe_unused]] float a_mu[MB], a_rs[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
        const int m = mb * 16 + r;
        a_ok[mb] = m < p.M;
        a_off[mb] = (long)min(m, p.M - 1) * p.lda;
        if constexpr (LN) { a_mu[mb] = st_mu[min(m, 63)]; a_rs[mb] = st_rs[min(m, 63)]; }
    }
    auto load_a = [&](int mb, int kk) -> s16x8 {
        if constexpr (LN) return sk_load_ln(p, a_off[mb], kk, k_hi, a_ok[mb], a_mu[mb], a_rs[mb]);
        else return sk_load(p.A, a_off[mb], kk, k_hi, a_ok[mb]);
    };
    f32x4 acc[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // k-steps k_lo + 32·(wave + 4·i): two steps' loads in flight before their MFMAs
    int k = k_lo + 32 * wave;
#pragma unroll 1
    for (; k + 128 < k_hi; k += 256) {
        s16x8 w0 = sk_load(p.W, w_off, k + kg, k_hi, n < p.N), w1 = sk_load(p.W, w_off, k + 128 + kg, k_hi, n < p.N);
        s16x8 a0[MB], a1[MB];
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
            a0[mb] = load_a(mb, k + kg);
            a1[mb] = load_a(mb, k + 128 + kg);
        }
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[mb], w0, acc[mb], 0, 0, 0);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[mb], w1, acc[mb], 0, 0, 0);
    }
    if (k < k_hi) {
        const s16x8 w0 = sk_load(p.W, w_off, k + kg, k_hi, n < p.N);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
            acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(load_a(mb, k + kg), w0, acc[mb], 0, 0, 0);
    }
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) red[wave][mb][lane] = acc[mb];
    __syncthreads();
    if (wave != 0) return;
    // lane holds D[row 4·(lane >> 4) + i][col lane & 15] of each 16-row block
    const int cn = n0 + (lane & 15);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
        f32x4 s = red[0][mb][lane];
#pragma unroll
        for (int w = 1; w < 4; ++w) s += red[w][mb][lane];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = mb * 16 + 4 * (lane >> 4) + i;
            if (m >= p.M || cn >= p.N) continue;
            if (p.S > 1) p.ws[((long)split * p.M + m) * p.N + cn] = s[i];
            else sk_store<ACT>(p, m, cn, s[i]);
        }
    }
}

// S > 1: sum the split partials in split order, then the epilogue
template <int ACT>
__global__ void __launch_bounds__(256) skinny_fin_k(SkArgs p) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    if (i >= (long)p.M * p.N) return;
    const int m = (int)(i / p.N), n = (int)(i % p.N);
    float v = 0.f;
    for (int s = 0; s < p.S; ++s) v += p.ws[(long)s * p.M * p.N + i];
    sk_store<ACT>(p, m, n, v);
}

template <int ACT, bool LN = false>
void sk_launch(const SkArgs& a, int mb, hipStream_t st) {
    const dim3 grid((a.N + 15) / 16, a.S);
    switch (mb) {
        case 1: skinny_k<1, ACT, LN><<<grid, 256, 0, st>>>(a); break;
        case 2: skinny_k<2, ACT, LN><<<grid, 256, 0, st>>>(a); break;
        case 3: skinny_k<3, ACT, LN><<<grid, 256, 0, st>>>(a); break;
        default: skinny_k<4, ACT, LN><<<grid, 256, 0, st>>>(a); break;
    }
    if (a.S > 1) skinny_fin_k<ACT><<<rn_cdiv((long)a.M * a.N, 256), 256, 0, st>>>(a);
}

}  // namespace

// Returns -1 for what this config does not take (the caller's autotuner then skips it): a
// transposed operand, M > 64, accumulate, activation backward, column partials, split without a
// workspace.  ``split``: K ranges (>= 1); each is a multiple of 32 deep.
extern "C" int rn_gemm_skinny(const void* A, const void* W, void* C, const void* bias, const void* res, void* pre, float* ws,
                   const float* alpha, int M, int N, int K, long lda, long ldw, long ldc, int trans_a, int trans_b,
                   int act, int split, int out_f32, int accumulate, const float* colpart, hipStream_t st) {
    if (trans_a || !trans_b || M < 1 || M > 64 || accumulate || act_bwd(act) || colpart) return -1;
    if (K % 8 != 0 || lda % 8 != 0 || ldw % 8 != 0) return -1;
    if (act != ACT_NONE && act != ACT_RELU && act != ACT_GELU && act != ACT_GELU_D) return -1;
    SkArgs a = {};
    a.A = (const bf16*)A; a.W = (const bf16*)W; a.C = C; a.bias = (const bf16*)bias; a.res = (const bf16*)res;
    a.pre = (bf16*)pre; a.ws = ws; a.alpha = alpha; a.M = M; a.N = N; a.K = K;
    a.lda = lda; a.ldw = ldw; a.ldc = ldc; a.out_f32 = out_f32;
    const int ksteps = (K + 31) / 32;
    int S = split < 1 ? 1 : split;
    S = S > ksteps ? ksteps : S;
    a.kc = (ksteps + S - 1) / S * 32;
    a.S = (K + a.kc - 1) / a.kc;
    if (a.S > 1 && !ws) return -1;
    const int mb = (M + 15) / 16;
    switch (act) {
        case ACT_RELU: sk_launch<ACT_RELU>(a, mb, st); break;
        case ACT_GELU: sk_launch<ACT_GELU>(a, mb, st); break;
        case ACT_GELU_D: sk_launch<ACT_GELU_D>(a, mb, st); break;
        default: sk_launch<ACT_NONE>(a, mb, st); break;
    }
    return 0;
}

// out[M][N] = act(LN(x)·Wᵀ + bias), LN over K with γ (ln_w), β (ln_b, optional), eps; M <= 64, one K
// range per workgroup (the row statistics need the whole row anyway).  Returns -1 if not taken.
extern "C" int rn_ln_gemm_skinny(const void* x, const void* ln_w, const void* ln_b, float eps, const void* W,
                                 const void* bias, void* C, int M, int N, int K, long ldx, long ldw, long ldc, int act,
                                 hipStream_t st) {
    if (M < 1 || M > 64 || K % 8 != 0 || ldx % 8 != 0 || ldw % 8 != 0) return -1;
    if (act != ACT_NONE && act != ACT_RELU && act != ACT_GELU) return -1;
    SkArgs a = {};
    a.A = (const bf16*)x; a.W = (const bf16*)W; a.C = C; a.bias = (const bf16*)bias;
    a.M = M; a.N = N; a.K = K; a.lda = ldx; a.ldw = ldw; a.ldc = ldc;
    a.ln_w = (const bf16*)ln_w; a.ln_b = (const bf16*)ln_b; a.eps = eps;
    a.S = 1;
    a.kc = (K + 31) / 32 * 32;
    const int mb = (M + 15) / 16;
    switch (act) {
        case ACT_RELU: sk_launch<ACT_RELU, true>(a, mb, st); break;
        case ACT_GELU: sk_launch<ACT_GELU, true>(a, mb, st); break;
        default: sk_launch<ACT_NONE, true>(a, mb, st); break;
    }
    return 0;
}
