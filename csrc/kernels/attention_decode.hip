// One-query attention for incremental decoding: o[b, h] = softmax(q·Kᵀ·scale + mask) · V over a KV
// cache of Tk rows, head size 64 (GPT-2).  Used by the captured decode step (GPT2.generate), where
// the key mask (fp32, one row shared by the batch: 0 = written, −inf = not yet) carries causality
// and the shapes are fixed at the cache length.
//
// The tiled flash kernels spend a 256-thread block with one live query row per (b, h) here and walk
// the keys 64 at a time through LDS (≈ 9 µs per layer, profiles/decode_steady_r4w.txt).  This kernel
// is shaped for one query: one workgroup per (b, h); scores with one key per thread (the q vector in
// registers, 8 × 16-byte loads of the key row), a block max / sum, then P·V with thread (8-column
// chunk, key group) = (t % 8, t / 8): 16-byte value loads, ≤ Tk / 32 independent iterations per
// thread, the 32 key groups merged in LDS in a fixed order.  Deterministic, no atomics.
// Tk <= 4 · 256 = 1024 keys (GPT-2's context).
#include "common.h"

namespace {

constexpr int DEC_T = 256, DEC_KPT = 4;  // threads, keys per thread in the score phase

__global__ void __launch_bounds__(DEC_T) attn_decode64_k(const bf16* __restrict__ q, const bf16* __restrict__ k,
                                                         const bf16* __restrict__ v, const float* __restrict__ mask,
                                                         bf16* __restrict__ o, int H, int Tk, long q_sb, long q_sh,
                                                         long k_sb, long k_st, long k_sh, long v_sb, long v_st,
                                                         long v_sh, long o_sb, long o_sh, float scale) {
    __shared__ float p_s[DEC_T * DEC_KPT];
    __shared__ float red[DEC_T / 64];
    __shared__ float part[32][64];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int b = blockIdx.x / H, h = blockIdx.x % H;
    const float sl2 = scale * 1.4426950408889634f;
    // q (64 elements) in every thread's registers
    float qf[64];
    const bf16* qp = q + b * q_sb + h * q_sh;
#pragma unroll
    for (int c = 0; c < 8; ++c) load8(qp + c * 8, qf + c * 8);
    const bf16* kb = k + b * k_sb + h * k_sh;
    float m = -INFINITY;
    float sc[DEC_KPT];
#pragma unroll
    for (int i = 0; i < DEC_KPT; ++i) {
        const int j = t + i * DEC_T;
        sc[i] = -INFINITY;
        if (j < Tk) {
            const bf16* kr = kb + (long)j * k_st;
            float s = 0.f, kf[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                load8(kr + c * 8, kf);
#pragma unroll
                for (int e = 0; e < 8; ++e) s = fmaf(qf[c * 8 + e], kf[e], s);
            }
            sc[i] = s * sl2 + (mask ? mask[j] * 1.4426950408889634f : 0.f);  // log2 units
        }
        m = fmaxf(m, sc[i]);
    }
    m = wave_max(m);
    if (lane == 0) red[wave] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < DEC_KPT; ++i) {
        const float pv = (sc[i] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(sc[i] - m);
        p_s[t + i * DEC_T] = pv;
        l += pv;
    }
    l = wave_sum(l);
    __syncthreads();  // red[] read by every thread above; p_s complete
    if (lane == 0) red[wave] = l;
    __syncthreads();
    l = red[0] + red[1] + red[2] + red[3];
    // P·V: thread (8-column chunk t % 8, key group t / 8) over keys t/8, t/8 + 32, ...: 16-byte value
    // loads, at most Tk / 32 independent iterations per thread; the 32 groups are summed in order
    const int dc = t & 7, kgp = t >> 3;
    const bf16* vb = v + b * v_sb + h * v_sh + dc * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int j = kgp; j < Tk; j += 32) {
        float vf[8];
        load8(vb + (long)j * v_st, vf);
        const float pj = p_s[j];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(pj, vf[e], acc[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) part[kgp][dc * 8 + e] = acc[e];
    __syncthreads();
    if (t < 64) {
        float tot = 0.f;
        for (int g = 0; g < 32; ++g) tot += part[g][t];
        o[b * o_sb + h * o_sh + t] = (bf16)(l > 0.f ? tot / l : 0.f);
    }
}

}  // namespace

// q, o: (B, 1, H, 64); k, v: (B, Tk, H, 64) with the given element strides (unit D stride);
// mask: Tk fp32 additive (or null).  Returns -1 for shapes this kernel does not take.
extern "C" int rn_attn_decode(const void* q, const void* k, const void* v, const float* mask, void* o, int B, int H,
                              int Tk, int D, const long* s, float scale, hipStream_t st) {
    if (D != 64 || Tk < 1 || Tk > DEC_T * DEC_KPT) return -1;
    for (int i = 0; i < 8; ++i)
        if (s[i] % 8 != 0) return -1;  // 16-byte row loads
    attn_decode64_k<<<B * H, DEC_T, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, mask, (bf16*)o, H, Tk, s[0],
                                             s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9], scale);
    return 0;
}
