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
    // K|V append (rn_gemm_skinny_kv, the decode step's QKV projection): output columns >= kv_c0 are
    // also stored into the KV cache row *kv_pos of batch row m: kvd[m·kv_sb + pos·kv_row + n − kv_c0]
    bf16* kvd;
    const int64_t* kv_pos;
    long kv_sb, kv_row;
    int kv_c0;
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
    if (p.kvd && n >= p.kv_c0) p.kvd[(long)m * p.kv_sb + (long)*p.kv_pos * p.kv_row + (n - p.kv_c0)] = (bf16)v;
}

RN_DEV s16x8 sk_load(const bf16* base, long row_off, int k, int K, bool row_ok) {
    if (row_ok && k < K) return *reinterpret_cast<const s16x8*>(base + row_off + k);
    return (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
}

template <int MB, int ACT>
__global__ void __launch_bounds__(256) skinny_k(SkArgs p) {
    __shared__ f32x4 red[4][MB][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = blockIdx.x * 16, split = blockIdx.y;
    const int r = lane & 15, kg = 8 * (lane >> 4);
    const int k_lo = split * p.kc, k_hi = min(p.K, k_lo + p.kc);
    const int n = n0 + r;
    const long w_off = (long)min(n, p.N - 1) * p.ldw;
    long a_off[MB];
    bool a_ok[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
        const int m = mb * 16 + r;
        a_ok[mb] = m < p.M;
        a_off[mb] = (long)min(m, p.M - 1) * p.lda;
    }
    f32x4 acc[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // k-steps k_lo + 32·(wave + 4·i): FOUR steps' loads in flight before their MFMAs (a decode GEMM's
    // wave has only a handful of k-steps, so the launch costs about one memory round trip per
    // iteration); a step past the range loads zeros (its MFMAs add nothing)
    int k = k_lo + 32 * wave;
#pragma unroll 1
    for (; k < k_hi; k += 512) {
        s16x8 wf[4], af[4][MB];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int kk = k + 128 * u + kg;
            wf[u] = sk_load(p.W, w_off, kk, k_hi, n < p.N);
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) af[u][mb] = sk_load(p.A, a_off[mb], kk, k_hi, a_ok[mb]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
                acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u][mb], wf[u], acc[mb], 0, 0, 0);
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

template <int ACT>
void sk_launch(const SkArgs& a, int mb, hipStream_t st) {
    const dim3 grid((a.N + 15) / 16, a.S);
    switch (mb) {
        case 1: skinny_k<1, ACT><<<grid, 256, 0, st>>>(a); break;
        case 2: skinny_k<2, ACT><<<grid, 256, 0, st>>>(a); break;
        case 3: skinny_k<3, ACT><<<grid, 256, 0, st>>>(a); break;
        default: skinny_k<4, ACT><<<grid, 256, 0, st>>>(a); break;
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

// Decode step QKV projection with the K|V append fused: out = x·Wᵀ + bias (M <= 64 rows = batch
// rows, one new token each) and its columns >= kv_c0 (keys, values) also written into the KV cache
// at the device-side row *kv_pos — the separate index_copy of every layer's keys / values is gone.
extern "C" int rn_gemm_skinny_kv(const void* x, const void* W, const void* bias, void* C, int M, int N, int K,
                                 long ldx, long ldw, long ldc, void* kvd, const int64_t* kv_pos, long kv_sb,
                                 long kv_row, int kv_c0, hipStream_t st) {
    if (M < 1 || M > 64 || K % 8 != 0 || ldx % 8 != 0 || ldw % 8 != 0 || kv_c0 < 0 || kv_c0 > N) return -1;
    SkArgs a = {};
    a.A = (const bf16*)x; a.W = (const bf16*)W; a.C = C; a.bias = (const bf16*)bias;
    a.M = M; a.N = N; a.K = K; a.lda = ldx; a.ldw = ldw; a.ldc = ldc;
    a.S = 1;
    a.kc = (K + 31) / 32 * 32;
    a.kvd = (bf16*)kvd; a.kv_pos = kv_pos; a.kv_sb = kv_sb; a.kv_row = kv_row; a.kv_c0 = kv_c0;
    sk_launch<ACT_NONE>(a, (M + 15) / 16, st);
    return 0;
}
