// Fused scaled-dot-product attention, forward + backward (N4/N5).
//
// Layout: q/k/v/o are [B][T][H][D] with arbitrary batch/token/head strides
// (q, k, v are usually views into one packed QKV GEMM output).  LSE is saved as
// [B][H][Tq] fp32 (natural log).
//
// MFMA path, head size D ∈ {32, 64, 128} (D = 64: GPT-2 small/medium, ViT-B/16; 32 / 128: the
// reference blocks' E // n_heads at e.g. 256/8 and 512/4), all v_mfma_f32_16x16x32_bf16:
//   * every product is arranged so that the softmax row index (the query for
//     fwd / dQ, the key for dK/dV) sits on lane&15 and the reduced index sits in
//     accumulator registers: the accumulator tile is then directly the next
//     MFMA's B operand (no LDS round trip, no lane shuffles for P or dS);
//     the k-order inside each 32-wide k-step is permuted identically on both
//     operands ({4g..4g+3} ∪ {16+4g..16+4g+3} for lane group g);
//   * the other operand of those products is a column slice of a row-major LDS
//     tile, read with ds_read_b64_tr_b16 (hardware transpose);
//   * LDS tiles are [64 rows][D bf16] staged by LDS-DMA (buffer_load … lds) with a
//     per-D 16-B chunk XOR swizzle (swz<D>) that is conflict-free for BOTH the
//     ds_read_b128 row reads and the transposed reads (one image serves both);
//   * online softmax in exp2 domain; causal tiles above the diagonal are
//     skipped, diagonal tiles masked; heaviest causal blocks launch first;
//   * dropout on P by a stateless counter hash, regenerated in the backward;
//   * backward = dQ kernel (one workgroup per 64 queries, loops over keys; also
//     emits delta = rowsum(dO·O) from registers) + dK/dV kernel (one workgroup
//     per 64 keys, loops over queries): no atomics, bitwise deterministic.
// D = 64 has extra tuned variants (split-loop forward with MFMA row sums, two query / key
// groups per wave in the backward); D = 32 / 128 use the single-loop forward and one group.
// Generic path (odd head sizes ≤ 256 only): per-query-row kernels with fp32 scores in LDS; the
// backward is dQ per query row, then dK/dV per key row (no atomics).
// Round 6 (D = 64): the 32×32×16 forward (causal: 8 waves / 256 queries per workgroup), and for
// Tq, Tk ≤ 256 whole-head-resident forward / backward kernels (docs/DESIGN.md §4 has the selection table).
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) const s16x8 lds_s16x8;
typedef __attribute__((address_space(3))) const f32x4 lds_f32x4;

struct AttnArgs {
    const bf16* q; const bf16* k; const bf16* v; bf16* o; float* lse; const float* bias;
    const bf16* dout; bf16* dq; bf16* dk; bf16* dv; const float* delta;
    long q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, o_sb, o_st, o_sh;
    long do_sb, do_st, do_sh, dq_sb, dq_st, dq_sh, dk_sb, dk_st, dk_sh, dv_sb, dv_st, dv_sh;
    int B, H, Tq, Tk, D;
    int causal, bias_b;
    float scale, p_drop;
    uint64_t seed;
    // optional device seed (graph-capturable dropout: drawn on the device per call, see ops/rng.py);
    // replaces `seed` when set
    const uint64_t* seed_ptr;
    float* dk32; float* dv32;  // generic bwd scratch
    // optional [B * ceil(T/64)][3 * H * 64] fp32: per-64-row-block column sums of dQ | dK | dV
    // (the packed-QKV projection's bias gradient, reduced later) — fast path, self-attention
    float* bsum;
    // lse units: the D = 64 forward kernels store log2(Σ exp) in base-2 units (the backward then
    // needs one FMA per score, exp2(s·scale·log2e − lse2)); the generic forward stores natural log.
    int lse_log2;
    // optional (D = 64 fast path): dQ | dK | dV also — or, q8_only, only — as OCP e5m2 at q8 (same element
    // offsets as dq / dk / dv: the packed dQKV's byte image) with the fp8 consumer's delayed scale q8st[0]
    // (rolled before the launch); amax(|dQKV|) recorded into q8st[1].  The c_attn projection's fp8 data /
    // weight gradients then need no quantisation pass over dQKV.
    uint8_t* q8;   // dQ's e5m2 base (dK / dV: q8k / q8v, the same element offsets as dk / dv)
    uint8_t* q8k;
    uint8_t* q8v;
    float* q8st;
    int q8_only;
    // per-wave amax partials (no same-address atomics: one per wave serialised 32 k atomics per launch
    // and tripled the kernels' time): dQ kernel at q8part[4·block + wave], dK/dV kernel at q8part2[...]
    float* q8part;
    float* q8part2;
};

// 4 values of a gradient row as e5m2 (one 4-B store) with the delayed scale, their amax folded into m
RN_DEV void attn_q8_store4(uint8_t* dst, float a, float b, float c, float d, float inv, float& m) {
    m = fmaxf(m, fmaxf(fmaxf(fabsf(a), fabsf(b)), fmaxf(fabsf(c), fabsf(d))));
    const float lim = 57344.f;
    int w = 0;
    w = __builtin_amdgcn_cvt_pk_bf8_f32(fminf(fmaxf(a * inv, -lim), lim), fminf(fmaxf(b * inv, -lim), lim), w, false);
    w = __builtin_amdgcn_cvt_pk_bf8_f32(fminf(fmaxf(c * inv, -lim), lim), fminf(fmaxf(d * inv, -lim), lim), w, true);
    *reinterpret_cast<int*>(dst) = w;
}
RN_DEV void attn_q8_amax(float* part, float m) {
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) part[blockIdx.x * 4 + (threadIdx.x >> 6)] = m;
}
// the partials of both kernels -> the slot's amax (state[1], zeroed by the roll): a grid-strided max, one
// atomic per block (a single block took 86 us for the 262 k partials of a GPT-2-medium step)
__global__ void __launch_bounds__(256) attn_amax_reduce_k(const float* __restrict__ part, int n, float* __restrict__ st) {
    __shared__ float red[4];
    float m = 0.f;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) m = fmaxf(m, part[i]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)
        atomicMax(reinterpret_cast<int*>(st + 1), __float_as_int(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// (bh, block) of this workgroup; `reverse`: the head's heaviest (last) causal block first
RN_DEV void blk_map(const AttnArgs& p, int nblk, bool reverse, int& bh, int& blk) {
    // head-interleaved 1-D grid of B·H·nblk blocks: block L works on head L % (B·H), so the
    // heaviest causal blocks of every head are dispatched first
    const int BH = p.B * p.H, L = blockIdx.x;
    const int i = L / BH;
    bh = L % BH;
    blk = reverse ? nblk - 1 - i : i;
}

// LDS tile geometry for head size D ∈ {32, 64, 128}: [64 rows][D bf16] = RB-byte rows, 16-B chunks
// XOR-swizzled per row.  Each swizzle is a permutation of the row's chunks that (a) makes the
// 16 rows of a ds_read_b128 row fragment (same logical chunk) land in 16 distinct 16-B bank slots
// and (b) keeps the 32-B chunk pairs of a ds_read_b64_tr_b16 column fragment (8 rows per pass) in
// 8 distinct 32-B slots; all three repeat with period 16 in the row, which FragOff relies on.
//   D = 64  (128-B rows, 2 per bank line): c ^ (((r>>1)&3)<<1)
//   D = 128 (256-B rows):                  c ^ (((r&7)<<1) | ((r>>3)&1))
//   D = 32  (64-B rows, 4 per bank line):  c ^ ((((r>>2)&1)<<1) | ((r>>3)&1))
template <int D = 64>
RN_DEV int swz(int r) {
    if constexpr (D == 64) return ((r >> 1) & 3) << 1;
    else if constexpr (D == 128) return ((r & 7) << 1) | ((r >> 3) & 1);
    else return (((r >> 2) & 1) << 1) | ((r >> 3) & 1);
}
template <int D> constexpr int kRB = 2 * D;        // bytes per tile row
template <int D> constexpr int kTB = 64 * 2 * D;   // bytes per 64-row tile
template <int D> constexpr int kNS = D / 32;       // 32-wide k-steps over the head dim
template <int D> constexpr int kNJ = D / 16;       // 16-wide output column blocks over the head dim

// Sum a wave-tile's [16 rows][D cols] accumulator (lane holds row lane&15, cols 16jd+4g+r)
// over the 64 rows of the 4 waves via LDS and write one partial row: out[col].
template <int D = 64>
RN_DEV void block_colsum64(const f32x4 (&acc)[kNJ<D>], float mul, float* lds, float* out, int wave, int lane) {
    const int g = lane >> 4, c = lane & 15;
    __syncthreads();  // LDS tiles no longer read by any wave
#pragma unroll
    for (int jd = 0; jd < kNJ<D>; ++jd)
#pragma unroll
        for (int r = 0; r < 4; ++r) lds[(wave * 16 + c) * (D + 1) + jd * 16 + 4 * g + r] = acc[jd][r] * mul;
    __syncthreads();
    if (threadIdx.x < D) {
        float t = 0.f;
        for (int row = 0; row < 64; ++row) t += lds[row * (D + 1) + threadIdx.x];
        out[threadIdx.x] = t;
    }
}

RN_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
    const uint64_t bp = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 0x7FFFFFF0, 0x00020000);
}

// row fragment: 8 bf16 of row `row`, columns 32*s + 8*(lane>>4) .. +7
template <int D = 64>
RN_DEV s16x8 rowfrag(const char* t, int row, int s, int lane) {
    const int chunk = s * 4 + (lane >> 4);
    return *reinterpret_cast<const s16x8*>(t + row * kRB<D> + ((chunk ^ swz<D>(row)) << 4));
}

// column fragment: column c0 + (lane&15), rows {rb + 4g + 0..3} ∪ {rb + 16 + 4g + 0..3}
template <int D = 64>
RN_DEV s16x8 colfrag(const char* t, int rb, int c0, int lane) {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
    const int ch = (c0 >> 3) + (p >> 1);
    const int r0 = rb + 4 * g + qq, r1 = r0 + 16;
    const char* a0 = t + r0 * kRB<D> + ((ch ^ swz<D>(r0)) << 4) + (p & 1) * 8;
    const char* a1 = t + r1 * kRB<D> + ((ch ^ swz<D>(r1)) << 4) + (p & 1) * 8;
    s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
    s16x8 r;
    r[0] = v0[0]; r[1] = v0[1]; r[2] = v0[2]; r[3] = v0[3];
    r[4] = v1[0]; r[5] = v1[1]; r[6] = v1[2]; r[7] = v1[3];
    return r;
}

// Per-lane parts of the rowfrag / colfrag LDS addresses, computed once per kernel.  Every call
// site reads row X*16 + (lane&15) (rowfrag) or rows 32*ks + … / columns 16*jd + … (colfrag) with
// X, ks, jd compile-time: the XOR swizzle then depends on the lane only, so the address is
// base + per-lane offset + an immediate, instead of ~50 recomputed VALU address ops per tile.
template <int D = 64>
struct FragOffT {
    uint32_t rf[kNS<D>];  // rowfrag, k-step s
    uint32_t cf[kNJ<D>];  // colfrag, column block jd
};
using FragOff = FragOffT<64>;
template <int D = 64>
RN_DEV FragOffT<D> make_fragoff(int lane) {
    FragOffT<D> f;
    const int g = lane >> 4, c = lane & 15;
    const int swc = swz<D>(c);
#pragma unroll
    for (int s = 0; s < kNS<D>; ++s) f.rf[s] = c * kRB<D> + ((((4 * s) + g) ^ swc) << 4);
    const int qq = c >> 2, pp = c & 3;
    const int r0 = 4 * g + qq;
    const int swr = swz<D>(r0);
#pragma unroll
    for (int jd = 0; jd < kNJ<D>; ++jd) f.cf[jd] = r0 * kRB<D> + (((2 * jd + (pp >> 1)) ^ swr) << 4) + (pp & 1) * 8;
    return f;
}
// == rowfrag<D>(t, X * 16 + (lane & 15), s, lane)
template <int D>
RN_DEV s16x8 rowfragx(const char* t, int X, int s, const FragOffT<D>& f) {
    return *reinterpret_cast<const s16x8*>(t + X * 16 * kRB<D> + f.rf[s]);
}
// == colfrag<D>(t, 32 * ks, 16 * jd, lane)
template <int D>
RN_DEV s16x8 colfragx(const char* t, int ks, int jd, const FragOffT<D>& f) {
    const char* a0 = t + ks * 32 * kRB<D> + f.cf[jd];
    s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 16 * kRB<D>));
    s16x8 r;
    r[0] = v0[0]; r[1] = v0[1]; r[2] = v0[2]; r[3] = v0[3];
    r[4] = v1[0]; r[5] = v1[1]; r[6] = v1[2]; r[7] = v1[3];
    return r;
}

RN_DEV s16x8 gload16(const bf16* p, bool ok) {
    if (!ok) return (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
    return *reinterpret_cast<const s16x8*>(p);
}

RN_DEV short bfbits(float f) { return __builtin_bit_cast(short, (bf16)f); }

RN_DEV s16x8 pack_p(const f32x4& a, const f32x4& b) {
    s16x8 r;
    r[0] = bfbits(a[0]); r[1] = bfbits(a[1]); r[2] = bfbits(a[2]); r[3] = bfbits(a[3]);
    r[4] = bfbits(b[0]); r[5] = bfbits(b[1]); r[6] = bfbits(b[2]); r[7] = bfbits(b[3]);
    return r;
}

RN_DEV uint64_t drop_idx(const AttnArgs& p, int b, int h, int qi, int kj) {
    return (((uint64_t)(b * p.H + h) * p.Tq + qi) * (uint64_t)p.Tk) + kj;
}

#define MFMA __builtin_amdgcn_mfma_f32_16x16x32_bf16

// ============================== forward, D = 64 ==============================
// grid: (ceil(Tq/128), B*H); 4 waves x 32 query rows.
// LDS-DMA issued through inline asm: the compiler then does not know a DMA is in
// flight, so it does not drain it (s_waitcnt vmcnt(0)) in front of every LDS read
// of the OTHER buffer — hipcc (ROCm 7.2) cannot tell the two buffers apart.  The
// hand-off is explicit instead: `s_waitcnt vmcnt(0)` + barrier at the top of each
// tile.  M0 (the DMA's LDS base) is written here; nothing else in these kernels
// uses it.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

RN_DEV u32x4 make_rsrc_sgpr(const void* base, uint32_t bytes = 0x7FFFFFF0u) {
    const uint64_t bp = (uint64_t)base;
    u32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    r[2] = __builtin_amdgcn_readfirstlane(bytes);  // range-checked: dwords past it read as 0
    r[3] = 0x00020000u;
    return r;
}

RN_DEV uint32_t lds_addr(const char* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)p);
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is "reserved": declaring the clobber is still right
RN_DEV void dma16_async(const u32x4& rs_, uint32_t voff, uint32_t lds) {
    // re-assert uniformity: after the loop unrolling the divergence analysis can lose track of the
    // (readfirstlane-built) descriptor and hand the "s" constraint a VGPR tuple
    u32x4 rs;
#pragma unroll
    for (int i = 0; i < 4; ++i) rs[i] = __builtin_amdgcn_readfirstlane(rs_[i]);
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
                 "s"(__builtin_amdgcn_readfirstlane(lds))
                 : "memory", "m0");
}
#pragma clang diagnostic pop

// Stage rows [r0, r0+64) (valid < rlim) of a [T][stride] bf16 matrix (D cols at the resource's
// base) into a swizzled LDS tile, by compiler-invisible LDS-DMA: D/8 16-B instructions in all,
// D/32 per wave; instruction `ins` fills rows ins·(512/D) .. +512/D (1 KiB of LDS).
template <int D = 64>
RN_DEV void stage64_async(const u32x4& rs, long st, int r0, int rlim, const char* lds, int wave, int lane) {
    constexpr int CPR = D / 8, RPI = 64 / CPR;
#pragma unroll
    for (int i = 0; i < D / 32; ++i) {
        const int ins = wave * (D / 32) + i;
        const int r = ins * RPI + lane / CPR;
        const int cg = (lane % CPR) ^ swz<D>(r);
        const bool ok = (r0 + r) < rlim;
        const uint32_t voff = ok ? (uint32_t)((((long)(r0 + r)) * st + cg * 8) * 2) : 0xFFFFFFF0u;
        dma16_async(rs, voff, lds_addr(lds + ins * 1024));
    }
}

RN_DEV void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// max over lanes {l, l^16, l^32, l^48} (the 4 lane groups holding one softmax row)
// with the gfx950 permlane swaps (VALU) instead of two ds_bpermute round trips.
RN_DEV float max4groups(float x) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
RN_DEV float sum4groups(float x) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// D = 32 / 64 / 128 (template); at D = 64 the default for bias / dropout, D = 32 / 128 for everything.
// QI: 16-query fragments per wave (block = 64·QI queries); 1 at D = 128 to fit the O accumulators.
// The bias / dropout variants run at occupancy ≤ 2: the per-score loads / hash need the registers.
template <bool CAUSAL, bool BIAS, bool DROP, int D = 64, int OCC = 3, int QI = 2>
__global__ void __launch_bounds__(256, ((DROP || BIAS) && OCC > 2) ? 2 : OCC) attn_fwd64_k(AttnArgs p) {
    constexpr int NS = kNS<D>, NJ = kNJ<D>, TB = kTB<D>, QBLK = 64 * QI;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // grid (B*H, blocks): the block index varies SLOWEST, so under causal masking every head's
    // heaviest query block is dispatched before any lighter one (longest-first over the grid)
    int bh, qb;
    blk_map(p, (p.Tq + QBLK - 1) / QBLK, CAUSAL, bh, qb);
    const int b = bh / p.H, h = bh % p.H;
    const int q0 = qb * QBLK + wave * 16 * QI;
    const int off = p.Tk - p.Tq;  // causal: key j visible to query i iff j <= i + off
    const float sl2 = p.scale * LOG2E;
    const float xs = BIAS ? 1.f : sl2;  // units of the running max m: log2-scaled with bias, raw without

    const bf16* qbase = p.q + b * p.q_sb + h * p.q_sh;
    const u32x4 krs = make_rsrc_sgpr(p.k + b * p.k_sb + h * p.k_sh);
    const u32x4 vrs = make_rsrc_sgpr(p.v + b * p.v_sb + h * p.v_sh);

    int kv_end = p.Tk;
    if (CAUSAL) kv_end = min(p.Tk, qb * QBLK + QBLK + off);
    const int nkv = kv_end > 0 ? (kv_end + 63) / 64 : 0;
#define Kt(i) (smem + (i) * 2 * TB)
#define Vt(i) (smem + TB + (i) * 2 * TB)
    if (nkv > 0) {  // first tile in flight while Q is loaded
        stage64_async<D>(krs, p.k_st, 0, p.Tk, Kt(0), wave, lane);
        stage64_async<D>(vrs, p.v_st, 0, p.Tk, Vt(0), wave, lane);
    }

    s16x8 qf[QI][NS];
#pragma unroll
    for (int qi = 0; qi < QI; ++qi)
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int row = q0 + qi * 16 + c;
            qf[qi][s] = gload16(qbase + (long)row * p.q_st + s * 32 + g * 8, row < p.Tq);
        }
    // Re-define qf through an (empty) asm so the compiler's wait for these loads happens
    // here, once: otherwise it re-waits vmcnt(0) inside the loop at their first use,
    // which would also drain the in-flight K/V prefetch.
#pragma unroll
    for (int qi = 0; qi < QI; ++qi)
#pragma unroll
        for (int s = 0; s < NS; ++s) asm volatile("" : "+v"(qf[qi][s]));
    float m[QI], l[QI];
#pragma unroll
    for (int qi = 0; qi < QI; ++qi) { m[qi] = -INFINITY; l[qi] = 0.f; }
    f32x4 oacc[QI][NJ];
#pragma unroll
    for (int qi = 0; qi < QI; ++qi)
#pragma unroll
        for (int jd = 0; jd < NJ; ++jd) oacc[qi][jd] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const float rd = DROP ? 1.f / (1.f - p.p_drop) : 1.f;
    if (p.p_drop > 0.f && p.seed_ptr) p.seed = *p.seed_ptr;
    for (int t = 0; t < nkv; ++t) {
        vm_wait_all();   // this wave's DMA of tile t landed ...
        __syncthreads(); // ... and every wave's; every wave also finished tile t-1 (its buffer is free)
        const int cur = t & 1;
        if (t + 1 < nkv) {
            stage64_async<D>(krs, p.k_st, (t + 1) * 64, p.Tk, Kt(cur ^ 1), wave, lane);
            stage64_async<D>(vrs, p.v_st, (t + 1) * 64, p.Tk, Vt(cur ^ 1), wave, lane);
        }
        const int kv0 = t * 64;
        // wave-uniform skip: this wave's queries all precede the tile
        if (CAUSAL && kv0 > q0 + 16 * QI - 1 + off) continue;
        const char* kt = Kt(cur);
        const char* vt = Vt(cur);
        f32x4 sacc[QI][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            s16x8 a[NS];
#pragma unroll
            for (int s = 0; s < NS; ++s) a[s] = rowfrag<D>(kt, j * 16 + c, s, lane);
#pragma unroll
            for (int qi = 0; qi < QI; ++qi) {
                f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < NS; ++s) z = MFMA(a[s], qf[qi][s], z, 0, 0, 0);
                sacc[qi][j] = z;
            }
        }
        if constexpr (BIAS) {  // x = s·scale·log2e + bias·log2e
#pragma unroll
            for (int qi = 0; qi < QI; ++qi) {
                const int qg = q0 + qi * 16 + c;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int kvb = kv0 + j * 16 + 4 * g;
                    float bb[4] = {0.f, 0.f, 0.f, 0.f};
                    if (qg < p.Tq) {
                        const float* bp = p.bias + ((long)(p.bias_b > 1 ? b : 0) * p.Tq + qg) * p.Tk + kvb;
                        if (kvb + 3 < p.Tk && (p.Tk & 3) == 0) {
                            float4 t4 = *reinterpret_cast<const float4*>(bp);
                            bb[0] = t4.x; bb[1] = t4.y; bb[2] = t4.z; bb[3] = t4.w;
                        } else {
                            for (int r = 0; r < 4; ++r) bb[r] = (kvb + r < p.Tk) ? bp[r] : 0.f;
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) sacc[qi][j][r] = sacc[qi][j][r] * sl2 + bb[r] * LOG2E;
                }
            }
        }
        // masking only on diagonal / ragged tiles: a real (wave-uniform) branch — the
        // empty asm keeps hipcc from if-converting it into per-element selects on
        // every tile
        if ((kv0 + 64 > p.Tk) || (CAUSAL && kv0 + 63 > q0 + off)) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int qi = 0; qi < QI; ++qi) {
                const int qg = q0 + qi * 16 + c;
                const int lim = CAUSAL ? min(qg + off, p.Tk - 1) : p.Tk - 1;
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (kv0 + j * 16 + 4 * g + r > lim) sacc[qi][j][r] = -INFINITY;
            }
        }
#pragma unroll
        for (int qi = 0; qi < QI; ++qi) {
            const int qg = q0 + qi * 16 + c;
            float tmax = -INFINITY;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, sacc[qi][j][r]);
            tmax = max4groups(tmax);
            const float mn = fmaxf(m[qi], tmax);
            const float ms = (mn == -INFINITY) ? 0.f : mn;  // fully-masked rows stay at p = 0
            const float alpha = (m[qi] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f((m[qi] - ms) * xs);
            const float nms = -ms * xs;
            m[qi] = mn;
            float ls = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[qi][j][r], xs, nms));
                    ls += pv;
                    if constexpr (DROP) {
                        const int kvj = kv0 + j * 16 + 4 * g + r;
                        pv = (hash_uniform(p.seed, drop_idx(p, b, h, qg, kvj)) >= p.p_drop) ? pv * rd : 0.f;
                    }
                    sacc[qi][j][r] = pv;
                }
            l[qi] = l[qi] * alpha + ls;
#pragma unroll
            for (int jd = 0; jd < NJ; ++jd) oacc[qi][jd] *= alpha;
        }
        // O^T[d][q] += V^T[d][kv] * P^T[kv][q]
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            s16x8 pb[QI];
#pragma unroll
            for (int qi = 0; qi < QI; ++qi) pb[qi] = pack_p(sacc[qi][2 * s], sacc[qi][2 * s + 1]);
#pragma unroll
            for (int jd = 0; jd < NJ; ++jd) {
                s16x8 a = colfrag<D>(vt, 32 * s, 16 * jd, lane);
#pragma unroll
                for (int qi = 0; qi < QI; ++qi) oacc[qi][jd] = MFMA(a, pb[qi], oacc[qi][jd], 0, 0, 0);
            }
        }
    }
#undef Kt
#undef Vt
    // epilogue
    bf16* obase = p.o + b * p.o_sb + h * p.o_sh;
#pragma unroll
    for (int qi = 0; qi < QI; ++qi) {
        const float lt = sum4groups(l[qi]);
        const int qg = q0 + qi * 16 + c;
        const float inv = lt > 0.f ? 1.f / lt : 0.f;
        if (qg < p.Tq) {
#pragma unroll
            for (int jd = 0; jd < NJ; ++jd) {
                bf16x4 o4 = {(bf16)(oacc[qi][jd][0] * inv), (bf16)(oacc[qi][jd][1] * inv),
                             (bf16)(oacc[qi][jd][2] * inv), (bf16)(oacc[qi][jd][3] * inv)};
                *reinterpret_cast<bf16x4*>(obase + (long)qg * p.o_st + jd * 16 + 4 * g) = o4;
            }
            if (g == 0)
                p.lse[((long)b * p.H + h) * p.Tq + qg] = (lt > 0.f) ? (m[qi] * xs + log2f(lt)) : INFINITY;  // base 2
        }
    }
}

// ------------------------- forward v2 (no bias / dropout) -------------------------
// Same data layout and fragment algebra as attn_fwd64_k; the loop is restructured:
//   * two loops — tiles every wave of the block sees in full (no mask, no per-wave skip)
//     and the diagonal / ragged tail (masked).  The single loop's per-wave `continue`
//     made hipcc carry the accumulators through a phi and copy 34 VGPRs per tile.
//   * the 16 transposed V reads of a tile are issued right after its QKᵀ MFMAs, so they
//     land under the softmax VALU work instead of being waited for between PV MFMAs;
//   * QKᵀ issues the k-step-0 MFMAs of all 8 output tiles before the k-step-1 ones (no
//     back-to-back dependent MFMAs).
// LEAN (variant 3): (a) the O / l rescale by alpha = exp2(m_old - m_new) runs only when some row
// of the wave raised its running max this tile (a wave-uniform ballot; after the first tiles the
// max rarely moves), (b) the row sums of P come from the matrix cores — P·1 as two extra MFMAs
// per query fragment against an all-ones A operand — instead of 32 v_add_f32 per tile.  Both
// trade VALU issue slots, which bound this kernel at head_dim 64, for idle MFMA / scalar slots;
// l then sums the bf16-rounded P that also feeds P·V.
template <bool CAUSAL, int OCC, bool LEAN = false, int QI = 2>
__global__ void __launch_bounds__(256, OCC) attn_fwd64v2_k(AttnArgs p) {
    constexpr int QW = 16 * QI, QBLK = 64 * QI;  // queries per wave / per block
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const FragOff fo = make_fragoff(lane);
    // grid (B*H, blocks): the block index varies SLOWEST, so under causal masking every head's
    // heaviest query block is dispatched before any lighter one (longest-first over the grid)
    int bh, qb;
    blk_map(p, (p.Tq + QBLK - 1) / QBLK, CAUSAL, bh, qb);
    const int b = bh / p.H, h = bh % p.H;
    const int q0 = qb * QBLK + wave * QW;
    const int off = p.Tk - p.Tq;
    const float sl2 = p.scale * LOG2E;

    const bf16* qbase = p.q + b * p.q_sb + h * p.q_sh;
    const u32x4 krs = make_rsrc_sgpr(p.k + b * p.k_sb + h * p.k_sh);
    const u32x4 vrs = make_rsrc_sgpr(p.v + b * p.v_sb + h * p.v_sh);

    int kv_end = p.Tk;
    if (CAUSAL) kv_end = min(p.Tk, qb * QBLK + QBLK + off);
    const int nkv = kv_end > 0 ? (kv_end + 63) / 64 : 0;
    // tiles [0, nfull): every key visible to every query of the block (and Tk-complete)
    int nfull = p.Tk / 64;
    if (CAUSAL) nfull = min(nfull, max(0, (qb * QBLK + off + 1) / 64));
    nfull = min(nfull, nkv);
#define Kt(i) (smem + (i) * 16384)
#define Vt(i) (smem + 8192 + (i) * 16384)
    if (nkv > 0) {
        stage64_async(krs, p.k_st, 0, p.Tk, Kt(0), wave, lane);
        stage64_async(vrs, p.v_st, 0, p.Tk, Vt(0), wave, lane);
    }
    s16x8 qf[QI][2];
#pragma unroll
    for (int qi = 0; qi < QI; ++qi)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int row = q0 + qi * 16 + c;
            qf[qi][s] = gload16(qbase + (long)row * p.q_st + s * 32 + g * 8, row < p.Tq);
        }
#pragma unroll
    for (int qi = 0; qi < QI; ++qi) asm volatile("" : "+v"(qf[qi][0]), "+v"(qf[qi][1]));
    float m[QI], l[QI];
#pragma unroll
    for (int qi = 0; qi < QI; ++qi) { m[qi] = -INFINITY; l[qi] = 0.f; }
    f32x4 oacc[QI][4];
#pragma unroll
    for (int qi = 0; qi < QI; ++qi)
#pragma unroll
        for (int jd = 0; jd < 4; ++jd) oacc[qi][jd] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const short one = 0x3F80;  // bf16 1.0
    [[maybe_unused]] const s16x8 ones = {one, one, one, one, one, one, one, one};

    auto tile = [&](const int t, auto masked_c) {
        constexpr bool MASKED = decltype(masked_c)::value;
        const int cur = t & 1;
        const char* kt = Kt(cur);
        const char* vt = Vt(cur);
        const int kv0 = t * 64;
        f32x4 sacc[QI][4];
        s16x8 ka[4][2];
        [[maybe_unused]] bool moved = false;
        [[maybe_unused]] float alph[QI];
        // masked tiles: a (16-query fragment qi, 16-key block j) of this wave with no visible pair —
        // past Tq / Tk (the ragged tail of a T = 197 sequence) or wholly above the causal diagonal —
        // skips its QKᵀ and P·V MFMAs (wave-uniform; its scores are −inf, so P = 0 there)
        auto live = [&](int qi, int j) -> bool {
            if constexpr (!MASKED) return true;
            const int qa = q0 + qi * 16, k0 = kv0 + j * 16;
            if (qa >= p.Tq || k0 >= p.Tk) return false;
            return !(CAUSAL && k0 > min(qa + 15, p.Tq - 1) + off);
        };
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ka[j][0] = rowfragx(kt, j, 0, fo);
            ka[j][1] = rowfragx(kt, j, 1, fo);
        }
        if constexpr (MASKED) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int qi = 0; qi < QI; ++qi) {
                    if (live(qi, j)) {
                        sacc[qi][j] = MFMA(ka[j][0], qf[qi][0], ((f32x4){0.f, 0.f, 0.f, 0.f}), 0, 0, 0);
                        sacc[qi][j] = MFMA(ka[j][1], qf[qi][1], sacc[qi][j], 0, 0, 0);
                    } else {
                        sacc[qi][j] = (f32x4){-INFINITY, -INFINITY, -INFINITY, -INFINITY};
                    }
                }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int qi = 0; qi < QI; ++qi) sacc[qi][j] = MFMA(ka[j][0], qf[qi][0], ((f32x4){0.f, 0.f, 0.f, 0.f}), 0, 0, 0);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int qi = 0; qi < QI; ++qi) sacc[qi][j] = MFMA(ka[j][1], qf[qi][1], sacc[qi][j], 0, 0, 0);
        }
        // V^T fragments for the PV product, in flight during the softmax
        s16x8 va[2][4];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int jd = 0; jd < 4; ++jd) va[s][jd] = colfragx(vt, s, jd, fo);
        if constexpr (MASKED) {
#pragma unroll
            for (int qi = 0; qi < QI; ++qi) {
                const int qg = q0 + qi * 16 + c;
                const int lim = CAUSAL ? min(qg + off, p.Tk - 1) : p.Tk - 1;
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (kv0 + j * 16 + 4 * g + r > lim) sacc[qi][j][r] = -INFINITY;
            }
        }
#pragma unroll
        for (int qi = 0; qi < QI; ++qi) {
            float tmax = -INFINITY;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, sacc[qi][j][r]);
            tmax = max4groups(tmax);
            const float mn = fmaxf(m[qi], tmax);
            float alpha, nms;
            if constexpr (MASKED) {
                const float ms = (mn == -INFINITY) ? 0.f : mn;  // fully-masked rows stay at p = 0
                alpha = (m[qi] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f((m[qi] - ms) * sl2);
                nms = -ms * sl2;
            } else {  // an unmasked tile has a finite max in every row
                alpha = __builtin_amdgcn_exp2f((m[qi] - mn) * sl2);  // exp2(-inf) = 0 on the first tile
                nms = -mn * sl2;
            }
            if constexpr (LEAN) {
                moved |= (mn != m[qi]);
                alph[qi] = alpha;
            }
            m[qi] = mn;
            float ls = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[qi][j][r], sl2, nms));
                    if constexpr (!LEAN) ls += pv;
                    sacc[qi][j][r] = pv;
                }
            if constexpr (!LEAN) {
                l[qi] = l[qi] * alpha + ls;
#pragma unroll
                for (int jd = 0; jd < 4; ++jd) oacc[qi][jd] *= alpha;
            }
        }
        if constexpr (LEAN) {
            if (__builtin_amdgcn_ballot_w64(moved)) {  // wave-uniform
#pragma unroll
                for (int qi = 0; qi < QI; ++qi) {
                    l[qi] *= alph[qi];
#pragma unroll
                    for (int jd = 0; jd < 4; ++jd) oacc[qi][jd] *= alph[qi];
                }
            }
        }
        f32x4 lsum[QI];
#pragma unroll
        for (int qi = 0; qi < QI; ++qi) lsum[qi] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            s16x8 pb[QI];
#pragma unroll
            for (int qi = 0; qi < QI; ++qi) pb[qi] = pack_p(sacc[qi][2 * s], sacc[qi][2 * s + 1]);
            if constexpr (MASKED) {  // skip (qi, k-step) pairs whose 32 keys are all dead for qi
#pragma unroll
                for (int qi = 0; qi < QI; ++qi) {
                    if (!(live(qi, 2 * s) || live(qi, 2 * s + 1))) continue;
#pragma unroll
                    for (int jd = 0; jd < 4; ++jd) oacc[qi][jd] = MFMA(va[s][jd], pb[qi], oacc[qi][jd], 0, 0, 0);
                    if constexpr (LEAN) lsum[qi] = MFMA(ones, pb[qi], lsum[qi], 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int jd = 0; jd < 4; ++jd)
#pragma unroll
                    for (int qi = 0; qi < QI; ++qi) oacc[qi][jd] = MFMA(va[s][jd], pb[qi], oacc[qi][jd], 0, 0, 0);
                if constexpr (LEAN) {
#pragma unroll
                    for (int qi = 0; qi < QI; ++qi) lsum[qi] = MFMA(ones, pb[qi], lsum[qi], 0, 0, 0);
                }
            }
        }
        if constexpr (LEAN) {
#pragma unroll
            for (int qi = 0; qi < QI; ++qi) l[qi] += lsum[qi][0];  // every row of P·1 holds the sum
        }
    };
    auto sync_prefetch = [&](int t) {
        vm_wait_all();   // this wave's DMA of tile t landed ...
        __syncthreads(); // ... and every wave's; tile t-1's buffer is free
        if (t + 1 < nkv) {
            stage64_async(krs, p.k_st, (t + 1) * 64, p.Tk, Kt((t & 1) ^ 1), wave, lane);
            stage64_async(vrs, p.v_st, (t + 1) * 64, p.Tk, Vt((t & 1) ^ 1), wave, lane);
        }
    };
    // (not unrolled by buffer like the backward kernels: at occupancy 3 the unrolled loop spills)
    // A wave whose queries all lie past Tq (the padded rows of a T = 197 sequence's last block) skips
    // every tile's work; it still joins every tile's barrier and DMA issue.
    const int nf = q0 < p.Tq ? nfull : 0;  // wave-uniform trip count
    int t = 0;
    for (; t < nf; ++t) {
        sync_prefetch(t);
        tile(t, std::false_type{});
    }
    for (; t < nkv; ++t) {
        sync_prefetch(t);
        if (CAUSAL && t * 64 > q0 + QW - 1 + off) continue;  // wave-uniform: every query of this wave precedes the tile
        if (q0 >= p.Tq) continue;                            // wave-uniform: no live query in this wave
        tile(t, std::true_type{});
    }
#undef Kt
#undef Vt
    bf16* obase = p.o + b * p.o_sb + h * p.o_sh;
#pragma unroll
    for (int qi = 0; qi < QI; ++qi) {
        const float lt = LEAN ? l[qi] : sum4groups(l[qi]);  // LEAN: P·1 already summed over all 64 keys
        const int qg = q0 + qi * 16 + c;
        const float inv = lt > 0.f ? 1.f / lt : 0.f;
        if (qg < p.Tq) {
#pragma unroll
            for (int jd = 0; jd < 4; ++jd) {
                bf16x4 o4 = {(bf16)(oacc[qi][jd][0] * inv), (bf16)(oacc[qi][jd][1] * inv),
                             (bf16)(oacc[qi][jd][2] * inv), (bf16)(oacc[qi][jd][3] * inv)};
                *reinterpret_cast<bf16x4*>(obase + (long)qg * p.o_st + jd * 16 + 4 * g) = o4;
            }
            if (g == 0)
                p.lse[((long)b * p.H + h) * p.Tq + qg] = (lt > 0.f) ? (m[qi] * sl2 + log2f(lt)) : INFINITY;  // base 2
        }
    }
}

// ============================== backward, D = 64 ==============================
// dK, dV: grid (B*H, ceil(Tk/(64·KG))); key group u (< KG) of wave w owns keys
// kb·64·KG + 64·u + 16w + (lane&15).  KG = 2: every Q / dO fragment read from LDS feeds both key
// groups' MFMAs and each wave carries two independent S → P → dS chains (as in the dQ kernel).
template <bool CAUSAL, bool BIAS, bool DROP, int OCC = 3, int KG = 1, int D = 64>
__global__ void __launch_bounds__(256, ((DROP || BIAS) && OCC > 2) ? 2 : OCC) attn_bwd_dkdv64_k(AttnArgs p) {
    constexpr int NS = kNS<D>, NJ = kNJ<D>, TB = kTB<D>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const FragOffT<D> fo = make_fragoff<D>(lane);
    constexpr int KB = 64 * KG;  // keys per block
    // grid (B*H, key blocks): low key blocks see the most queries under causal and, with the block
    // index varying slowest, launch first across ALL heads (longest-first)
    int bh, kb;
    blk_map(p, (p.Tk + KB - 1) / KB, false, bh, kb);  // low key blocks see the most queries: first
    const int b = bh / p.H, h = bh % p.H;
    const int kvw = kb * KB + wave * 16;  // this wave's first key (group 0)
    int kvl[KG];
#pragma unroll
    for (int u = 0; u < KG; ++u) kvl[u] = kvw + 64 * u + c;
    const int off = p.Tk - p.Tq;
    const float sl2 = p.scale * LOG2E;

    const u32x4 qrs = make_rsrc_sgpr(p.q + b * p.q_sb + h * p.q_sh);
    const u32x4 ors = make_rsrc_sgpr(p.dout + b * p.do_sb + h * p.do_sh);
    // per-row softmax statistics ride along with each Q/dO tile (LDS-DMA, 64 floats each)
    const u32x4 lrs = make_rsrc_sgpr(p.lse + ((long)b * p.H + h) * p.Tq, (uint32_t)p.Tq * 4);
    const u32x4 drs = make_rsrc_sgpr(p.delta + ((long)b * p.H + h) * p.Tq, (uint32_t)p.Tq * 4);
    const bf16* kbase = p.k + b * p.k_sb + h * p.k_sh;
    const bf16* vbase = p.v + b * p.v_sb + h * p.v_sh;

    int qt0 = 0;
    if (CAUSAL) qt0 = max(0, (kb * KB - off)) / 64;
    const int nqt = (p.Tq + 63) / 64;
    // buffer i: Q tile [0, TB), dO tile [TB, 2TB), lse [2TB, 2TB + 1K), delta [2TB + 1K, 2TB + 2K)
#define Qt(i) (smem + (i) * (2 * TB + 2048))
#define Ot(i) (smem + TB + (i) * (2 * TB + 2048))
#define Lt(i) (smem + 2 * TB + (i) * (2 * TB + 2048))
#define Dt(i) (smem + 2 * TB + 1024 + (i) * (2 * TB + 2048))
    auto stage = [&](int qt, int buf) {
        stage64_async<D>(qrs, p.q_st, qt * 64, p.Tq, Qt(buf), wave, lane);
        stage64_async<D>(ors, p.do_st, qt * 64, p.Tq, Ot(buf), wave, lane);
        if (wave < 2) {  // lanes 0-15 carry 64 floats; the rest land as zeros past them
            const int r = qt * 64 + lane * 4;
            const uint32_t voff = (lane < 16 && r < p.Tq) ? (uint32_t)(r * 4) : 0xFFFFFFF0u;
            dma16_async(wave == 0 ? lrs : drs, voff, lds_addr(wave == 0 ? Lt(buf) : Dt(buf)));
        }
    };
    if (qt0 < nqt) stage(qt0, 0);

    s16x8 kf[KG][NS], vf[KG][NS];
#pragma unroll
    for (int u = 0; u < KG; ++u) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            kf[u][s] = gload16(kbase + (long)kvl[u] * p.k_st + s * 32 + g * 8, kvl[u] < p.Tk);
            vf[u][s] = gload16(vbase + (long)kvl[u] * p.v_st + s * 32 + g * 8, kvl[u] < p.Tk);
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) asm volatile("" : "+v"(kf[u][s]), "+v"(vf[u][s]));  // wait here, not in the loop
    }
    f32x4 dvacc[KG][NJ], dkacc[KG][NJ];
#pragma unroll
    for (int u = 0; u < KG; ++u)
#pragma unroll
        for (int jd = 0; jd < NJ; ++jd) { dvacc[u][jd] = (f32x4){0, 0, 0, 0}; dkacc[u][jd] = (f32x4){0, 0, 0, 0}; }

    const float rd = DROP ? 1.f / (1.f - p.p_drop) : 1.f;
    if (p.p_drop > 0.f && p.seed_ptr) p.seed = *p.seed_ptr;
    // Tiles split into masked (causal diagonal of this block's keys, ragged Tq / Tk) and unmasked
    // ones, each class in its own loop: a per-wave `continue` or a runtime mask branch inside one
    // loop makes hipcc carry the accumulators through a phi (a VGPR copy block every tile).
    auto masked_tile = [&](int qt) {
        return (qt * 64 + 64 > p.Tq) || (kb * KB + KB > p.Tk) || (CAUSAL && kb * KB + KB - 1 > qt * 64 + off);
    };
    auto sync_stage = [&](int qt) {
        vm_wait_all();
        __syncthreads();
        if (qt + 1 < nqt) stage(qt + 1, ((qt - qt0) & 1) ^ 1);
    };
    auto body = [&](int qt, auto masked_c, auto buf_c) {  // buf_c: compile-time buffer, see the forward
        constexpr bool MASKED = decltype(masked_c)::value;
        constexpr int cur = decltype(buf_c)::value;
        const int q0 = qt * 64;
        const char* qt_ = Qt(cur);
        const char* ot_ = Ot(cur);
        const float* lt_ = reinterpret_cast<const float*>(Lt(cur));
        const float* dt_ = reinterpret_cast<const float*>(Dt(cur));
        // masked tiles: a (key group u, 16-query fragment qi) block of this wave with no visible
        // (key, query) pair — past Tk / Tq, or wholly above the causal diagonal — skips its MFMAs and
        // VALU (wave-uniform; P = dS = 0 there).  The diagonal's upper blocks and the ragged tail of a
        // T = 197 sequence (ViT) are most of such a tile.
        auto live = [&](int u, int qi) -> bool {
            if constexpr (!MASKED) return true;
            const int k0 = kvw + 64 * u, qa = q0 + qi * 16;
            if (k0 >= p.Tk || qa >= p.Tq) return false;
            return !(CAUSAL && k0 > min(qa + 15, p.Tq - 1) + off);
        };
        f32x4 pq[KG][4], dsq[KG][4];
#pragma unroll
        for (int qi = 0; qi < 4; ++qi) {
            s16x8 af[NS], of[NS];
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                af[s] = rowfragx(qt_, qi, s, fo);
                of[s] = rowfragx(ot_, qi, s, fo);
            }
            // lane holds S[q = q0 + 16qi + 4g + r][kv]
            const int ql = qi * 16 + 4 * g;
            const float4 l4 = *reinterpret_cast<const float4*>(lt_ + ql);
            const float4 d4 = *reinterpret_cast<const float4*>(dt_ + ql);
            // the dQ kernel stored −δ: without dropout it is the dP accumulator's start value
            const float ls[4] = {l4.x, l4.y, l4.z, l4.w}, nd[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
            for (int u = 0; u < KG; ++u) {
                if (MASKED && !live(u, qi)) {
                    pq[u][qi] = (f32x4){0, 0, 0, 0};
                    dsq[u][qi] = (f32x4){0, 0, 0, 0};
                    continue;
                }
                f32x4 sa = {0, 0, 0, 0}, da = {0, 0, 0, 0};
                if constexpr (!DROP) da = (f32x4){nd[0], nd[1], nd[2], nd[3]};
#pragma unroll
                for (int s = 0; s < NS; ++s) sa = MFMA(af[s], kf[u][s], sa, 0, 0, 0);
#pragma unroll
                for (int s = 0; s < NS; ++s) da = MFMA(of[s], vf[u][s], da, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int qg = q0 + ql + r;
                    float x = __builtin_fmaf(sa[r], sl2, -ls[r]);  // lse in base-2 units: one FMA
                    if constexpr (BIAS) {
                        if (qg < p.Tq && kvl[u] < p.Tk)
                            x += p.bias[((long)(p.bias_b > 1 ? b : 0) * p.Tq + qg) * p.Tk + kvl[u]] * LOG2E;
                    }
                    // masked scores: exponent −inf, so P = 0 and dS = 0 follow (one select per element)
                    if constexpr (MASKED)
                        if (kvl[u] >= p.Tk || qg >= p.Tq || (CAUSAL && kvl[u] > qg + off)) x = -INFINITY;
                    float pv = __builtin_amdgcn_exp2f(x);
                    float dpv = da[r];
                    float pd = pv;
                    if constexpr (DROP) {
                        const bool keep = hash_uniform(p.seed, drop_idx(p, b, h, qg, kvl[u])) >= p.p_drop;
                        pd = keep ? pv * rd : 0.f;
                        dpv = keep ? dpv * rd : 0.f;
                    }
                    pq[u][qi][r] = pd;
                    dsq[u][qi][r] = DROP ? pv * (dpv + nd[r]) : pv * dpv;
                }
            }
        }
        // dV^T[d][kv] += dO^T[d][q] Pd[q][kv];  dK^T[d][kv] += Q^T[d][q] dS[q][kv]
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            if constexpr (MASKED) {  // both 16-query fragments of this k-step dead for every key group
                bool any = false;
#pragma unroll
                for (int u = 0; u < KG; ++u) any = any || live(u, 2 * ks) || live(u, 2 * ks + 1);
                if (!any) continue;
            }
            s16x8 pb[KG], sb[KG];
#pragma unroll
            for (int u = 0; u < KG; ++u) {
                pb[u] = pack_p(pq[u][2 * ks], pq[u][2 * ks + 1]);
                sb[u] = pack_p(dsq[u][2 * ks], dsq[u][2 * ks + 1]);
            }
#pragma unroll
            for (int jd = 0; jd < NJ; ++jd) {
                const s16x8 ao = colfragx(ot_, ks, jd, fo);
#pragma unroll
                for (int u = 0; u < KG; ++u) dvacc[u][jd] = MFMA(ao, pb[u], dvacc[u][jd], 0, 0, 0);
                const s16x8 aq = colfragx(qt_, ks, jd, fo);
#pragma unroll
                for (int u = 0; u < KG; ++u) dkacc[u][jd] = MFMA(aq, sb[u], dkacc[u][jd], 0, 0, 0);
            }
        }
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    auto step = [&](int qt, auto masked_c, auto buf_c) {
        sync_stage(qt);
        // wave-uniform skip: every query of the tile precedes this wave's first key
        if (decltype(masked_c)::value && CAUSAL && qt * 64 + 63 + off < kvw) return;
        [[clang::always_inline]] body(qt, masked_c, buf_c);
    };
    // tiles [qt, end) with buffer (qt - qt0) & 1 resolved at compile time (always_inline: see dQ)
    auto run = [&](int qt, int end, auto masked_c) {
        if (qt < end && ((qt - qt0) & 1)) [[clang::always_inline]] step(qt++, masked_c, B1{});
        for (; qt + 1 < end; qt += 2) {
            [[clang::always_inline]] step(qt, masked_c, B0{});
            [[clang::always_inline]] step(qt + 1, masked_c, B1{});
        }
        if (qt < end) [[clang::always_inline]] step(qt++, masked_c, B0{});
        return qt;
    };
    int qt = qt0, qe = qt0;
    while (qe < nqt && masked_tile(qe)) ++qe;
    qt = run(qt, qe, std::true_type{});  // diagonal head
    while (qe < nqt && !masked_tile(qe)) ++qe;
    qt = run(qt, qe, std::false_type{});
    run(qt, nqt, std::true_type{});  // ragged tail
#undef Qt
#undef Ot
#undef Lt
#undef Dt
    if (p.bsum) {  // dK / dV column partials for the QKV bias gradient; row = (b, 64-key block)
        const int E = p.H * D, nb64 = (p.Tk + 63) / 64;
#pragma unroll
        for (int u = 0; u < KG; ++u) {
            const int blk = kb * KG + u;
            if (blk < nb64) {  // block-uniform
                float* row = p.bsum + ((long)b * nb64 + blk) * 3 * E + h * D;
                block_colsum64<D>(dkacc[u], p.scale, reinterpret_cast<float*>(smem), row + E, wave, lane);
                block_colsum64<D>(dvacc[u], 1.f, reinterpret_cast<float*>(smem), row + 2 * E, wave, lane);
            }
        }
    }
    float q8m = 0.f;
    const float q8inv = p.q8 ? 1.f / p.q8st[0] : 0.f;
#pragma unroll
    for (int u = 0; u < KG; ++u) {
        if (kvl[u] < p.Tk) {
            const long ko = b * p.dk_sb + (long)kvl[u] * p.dk_st + h * p.dk_sh;
            const long vo = b * p.dv_sb + (long)kvl[u] * p.dv_st + h * p.dv_sh;
            bf16* dkp = p.dk + ko;
            bf16* dvp = p.dv + vo;
#pragma unroll
            for (int jd = 0; jd < NJ; ++jd) {
                const float k0 = dkacc[u][jd][0] * p.scale, k1 = dkacc[u][jd][1] * p.scale,
                            k2 = dkacc[u][jd][2] * p.scale, k3 = dkacc[u][jd][3] * p.scale;
                if (p.q8) {  // (the e5m2 of the bf16-rounded values a separate pass would quantise)
                    attn_q8_store4(p.q8k + ko + jd * 16 + 4 * g, (float)(bf16)k0, (float)(bf16)k1, (float)(bf16)k2,
                                   (float)(bf16)k3, q8inv, q8m);
                    attn_q8_store4(p.q8v + vo + jd * 16 + 4 * g, (float)(bf16)dvacc[u][jd][0], (float)(bf16)dvacc[u][jd][1],
                                   (float)(bf16)dvacc[u][jd][2], (float)(bf16)dvacc[u][jd][3], q8inv, q8m);
                }
                if (!p.q8_only) {
                    bf16x4 k4 = {(bf16)k0, (bf16)k1, (bf16)k2, (bf16)k3};
                    bf16x4 v4 = {(bf16)dvacc[u][jd][0], (bf16)dvacc[u][jd][1], (bf16)dvacc[u][jd][2],
                                 (bf16)dvacc[u][jd][3]};
                    *reinterpret_cast<bf16x4*>(dkp + jd * 16 + 4 * g) = k4;
                    *reinterpret_cast<bf16x4*>(dvp + jd * 16 + 4 * g) = v4;
                }
            }
        }
    }
    if (p.q8) attn_q8_amax(p.q8part2, q8m);
}

// dQ: grid (B*H, ceil(Tq/(64·QG))); query group qg (< QG) of wave w owns queries
// qb·64·QG + 64·qg + 16w + (lane&15).  With QG = 2 every K / V fragment read from LDS feeds
// the MFMAs of two query groups (half the LDS reads per MFMA) and each wave carries two
// independent dependency chains (S → P → dS → dQ) for the scheduler to interleave.
template <bool CAUSAL, bool BIAS, bool DROP, int OCC = 2, int QG = 1, int D = 64>
__global__ void __launch_bounds__(256, OCC) attn_bwd_dq64_k(AttnArgs p) {
    constexpr int NS = kNS<D>, NJ = kNJ<D>, TB = kTB<D>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const FragOffT<D> fo = make_fragoff<D>(lane);
    constexpr int QB = 64 * QG;  // queries per block
    int bh, qb;
    blk_map(p, (p.Tq + QB - 1) / QB, CAUSAL, bh, qb);  // heaviest blocks of every head first
    const int b = bh / p.H, h = bh % p.H;
    const int qw_last = qb * QB + 64 * (QG - 1) + wave * 16;  // this wave's first query of its LAST group
    const int off = p.Tk - p.Tq;
    const float sl2 = p.scale * LOG2E;

    const bf16* qbase = p.q + b * p.q_sb + h * p.q_sh;
    const bf16* dobase = p.dout + b * p.do_sb + h * p.do_sh;
    const u32x4 krs = make_rsrc_sgpr(p.k + b * p.k_sb + h * p.k_sh);
    const u32x4 vrs = make_rsrc_sgpr(p.v + b * p.v_sb + h * p.v_sh);
    int qgl[QG];
    bool qok[QG];
    s16x8 qf[QG][NS], df[QG][NS];
    float lse2[QG], dl[QG];
#pragma unroll
    for (int u = 0; u < QG; ++u) {
        qgl[u] = qb * QB + 64 * u + wave * 16 + c;
        qok[u] = qgl[u] < p.Tq;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            qf[u][s] = gload16(qbase + (long)qgl[u] * p.q_st + s * 32 + g * 8, qok[u]);
            df[u][s] = gload16(dobase + (long)qgl[u] * p.do_st + s * 32 + g * 8, qok[u]);
        }
        lse2[u] = qok[u] ? p.lse[((long)b * p.H + h) * p.Tq + qgl[u]] : INFINITY;  // base-2 units
        // delta = rowsum(dO ∘ O), computed here from the dO fragments already in
        // registers (no separate delta kernel); written out for the dK/dV kernel.
        const bf16* obase = p.o + b * p.o_sb + h * p.o_sh;
        float part = 0.f;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            s16x8 of = gload16(obase + (long)qgl[u] * p.o_st + s * 32 + g * 8, qok[u]);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                part += (float)__builtin_bit_cast(bf16, (short)of[j]) * (float)__builtin_bit_cast(bf16, (short)df[u][s][j]);
        }
        dl[u] = sum4groups(part);
        // stored NEGATED: the dK/dV kernel starts its dP accumulators at −δ (dP − δ from the MFMA)
        if (qok[u] && g == 0) const_cast<float*>(p.delta)[((long)b * p.H + h) * p.Tq + qgl[u]] = -dl[u];
#pragma unroll
        for (int s = 0; s < NS; ++s) asm volatile("" : "+v"(qf[u][s]), "+v"(df[u][s]));
        asm volatile("" : "+v"(dl[u]));  // loads retired here
    }
    f32x4 dqacc[QG][NJ];
#pragma unroll
    for (int u = 0; u < QG; ++u)
#pragma unroll
        for (int jd = 0; jd < NJ; ++jd) dqacc[u][jd] = (f32x4){0, 0, 0, 0};

    int kv_end = p.Tk;
    if (CAUSAL) kv_end = min(p.Tk, qb * QB + QB + off);
    const int nkv = kv_end > 0 ? (kv_end + 63) / 64 : 0;
#define Kt(i) (smem + (i) * 2 * TB)
#define Vt(i) (smem + TB + (i) * 2 * TB)
    if (nkv > 0) {
        stage64_async<D>(krs, p.k_st, 0, p.Tk, Kt(0), wave, lane);
        stage64_async<D>(vrs, p.v_st, 0, p.Tk, Vt(0), wave, lane);
    }
    const float rd = DROP ? 1.f / (1.f - p.p_drop) : 1.f;
    if (p.p_drop > 0.f && p.seed_ptr) p.seed = *p.seed_ptr;
    // masked (diagonal / ragged) and unmasked tiles in separate loops, see the dK/dV kernel
    auto masked_tile = [&](int t) {
        return (t * 64 + 64 > p.Tk) || (qb * QB + QB > p.Tq) || (CAUSAL && t * 64 + 63 > qb * QB + off);
    };
    auto sync_stage = [&](int t) {
        vm_wait_all();
        __syncthreads();
        if (t + 1 < nkv) {
            stage64_async<D>(krs, p.k_st, (t + 1) * 64, p.Tk, Kt((t & 1) ^ 1), wave, lane);
            stage64_async<D>(vrs, p.v_st, (t + 1) * 64, p.Tk, Vt((t & 1) ^ 1), wave, lane);
        }
    };
    auto body = [&](int t, auto masked_c, auto buf_c) {
        constexpr bool MASKED = decltype(masked_c)::value;
        constexpr int cur = decltype(buf_c)::value;  // compile-time buffer, see the dK/dV kernel
        const int kv0 = t * 64;
        const char* kt = Kt(cur);
        const char* vt = Vt(cur);
        // masked tiles: a (query group u, 16-key block j) of this wave with no visible pair skips
        // its MFMAs and VALU (wave-uniform; dS = 0 there), as in the dK/dV kernel
        auto live = [&](int u, int j) -> bool {
            if constexpr (!MASKED) return true;
            const int qa = qb * QB + 64 * u + wave * 16, k0 = kv0 + 16 * j;
            if (qa >= p.Tq || k0 >= p.Tk) return false;
            return !(CAUSAL && k0 > min(qa + 15, p.Tq - 1) + off);
        };
        f32x4 dsv[QG][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            s16x8 kr[NS], vr[NS];
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                kr[s] = rowfragx(kt, j, s, fo);
                vr[s] = rowfragx(vt, j, s, fo);
            }
#pragma unroll
            for (int u = 0; u < QG; ++u) {
                if (MASKED && !live(u, j)) {
                    dsv[u][j] = (f32x4){0, 0, 0, 0};
                    continue;
                }
                f32x4 sa = {0, 0, 0, 0}, da = {0, 0, 0, 0};
#pragma unroll
                for (int s = 0; s < NS; ++s) sa = MFMA(kr[s], qf[u][s], sa, 0, 0, 0);
#pragma unroll
                for (int s = 0; s < NS; ++s) da = MFMA(vr[s], df[u][s], da, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int kvj = kv0 + j * 16 + 4 * g + r;
                    float x = sa[r] * sl2;
                    if constexpr (BIAS) {
                        if (qok[u] && kvj < p.Tk)
                            x += p.bias[((long)(p.bias_b > 1 ? b : 0) * p.Tq + qgl[u]) * p.Tk + kvj] * LOG2E;
                    }
                    float pv = __builtin_amdgcn_exp2f(x - lse2[u]);
                    float dpv = da[r];
                    if constexpr (DROP) {
                        const bool keep = hash_uniform(p.seed, drop_idx(p, b, h, qgl[u], kvj)) >= p.p_drop;
                        dpv = keep ? dpv * rd : 0.f;
                    }
                    dsv[u][j][r] = pv * (dpv - dl[u]);  // (a −δ accumulator start here costs occupancy 3 → 2)
                }
            }
        }
        if constexpr (MASKED) {  // (the dK/dV kernel's −inf-exponent form costs this kernel occupancy 3 → 2)
#pragma unroll
            for (int u = 0; u < QG; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int kvj = kv0 + j * 16 + 4 * g + r;
                        if (kvj >= p.Tk || !qok[u] || (CAUSAL && kvj > qgl[u] + off)) dsv[u][j][r] = 0.f;
                    }
        }
        // dQ^T[d][q] += K^T[d][kv] dS^T[kv][q]
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            if constexpr (MASKED) {  // both 16-key blocks of this k-step dead for every query group
                bool any = false;
#pragma unroll
                for (int u = 0; u < QG; ++u) any = any || live(u, 2 * ks) || live(u, 2 * ks + 1);
                if (!any) continue;
            }
            s16x8 sb[QG];
#pragma unroll
            for (int u = 0; u < QG; ++u) sb[u] = pack_p(dsv[u][2 * ks], dsv[u][2 * ks + 1]);
#pragma unroll
            for (int jd = 0; jd < NJ; ++jd) {
                const s16x8 kc = colfragx(kt, ks, jd, fo);
#pragma unroll
                for (int u = 0; u < QG; ++u) dqacc[u][jd] = MFMA(kc, sb[u], dqacc[u][jd], 0, 0, 0);
            }
        }
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    auto step = [&](int t, auto masked_c, auto buf_c) {
        sync_stage(t);
        // wave-uniform skip: every query of this wave (its last group included) precedes the tile
        if (decltype(masked_c)::value && CAUSAL && t * 64 > qw_last + 15 + off) return;
        [[clang::always_inline]] body(t, masked_c, buf_c);
    };
    // (always_inline: with two query groups hipcc otherwise outlines the causal masked step into a
    // real call whose captured state round-trips through scratch)
    auto run = [&](int t, int end, auto masked_c) {
        if (t < end && (t & 1)) [[clang::always_inline]] step(t++, masked_c, B1{});
        for (; t + 1 < end; t += 2) {
            [[clang::always_inline]] step(t, masked_c, B0{});
            [[clang::always_inline]] step(t + 1, masked_c, B1{});
        }
        if (t < end) [[clang::always_inline]] step(t++, masked_c, B0{});
        return t;
    };
    int te = 0;
    while (te < nkv && !masked_tile(te)) ++te;
    const int t = run(0, te, std::false_type{});
    run(t, nkv, std::true_type{});  // diagonal / ragged tail
#undef Kt
#undef Vt
    if (p.bsum) {  // dQ column partials; row = (b, 64-query block) — the dK/dV kernel's row layout
        const int E = p.H * D, nb64 = (p.Tq + 63) / 64;
#pragma unroll
        for (int u = 0; u < QG; ++u) {
            const int blk = qb * QG + u;
            if (blk < nb64) {  // block-uniform
                float* row = p.bsum + ((long)b * nb64 + blk) * 3 * E + h * D;
                block_colsum64<D>(dqacc[u], p.scale, reinterpret_cast<float*>(smem), row, wave, lane);
            }
        }
    }
    float q8m = 0.f;
    const float q8inv = p.q8 ? 1.f / p.q8st[0] : 0.f;
#pragma unroll
    for (int u = 0; u < QG; ++u) {
        if (qok[u]) {
            const long qo = b * p.dq_sb + (long)qgl[u] * p.dq_st + h * p.dq_sh;
            bf16* dqp = p.dq + qo;
#pragma unroll
            for (int jd = 0; jd < NJ; ++jd) {
                bf16x4 q4 = {(bf16)(dqacc[u][jd][0] * p.scale), (bf16)(dqacc[u][jd][1] * p.scale),
                             (bf16)(dqacc[u][jd][2] * p.scale), (bf16)(dqacc[u][jd][3] * p.scale)};
                if (p.q8)
                    attn_q8_store4(p.q8 + qo + jd * 16 + 4 * g, (float)q4[0], (float)q4[1], (float)q4[2], (float)q4[3],
                                   q8inv, q8m);
                if (!p.q8_only) *reinterpret_cast<bf16x4*>(dqp + jd * 16 + 4 * g) = q4;
            }
        }
    }
    if (p.q8) attn_q8_amax(p.q8part, q8m);
}

// ======================= D = 64 on v_mfma_f32_32x32x16_bf16 (round 6) =======================
// The causal forward re-tiled for the 32×32×16 MFMA.  Why: the 16×16×32 kernels above run with the
// softmax VALU beside their MFMAs, and a 16×16×32 MFMA holds the SIMD's vector issue for 8 of its 16
// cycles while a 32×32×16 one holds it for 8 of 32 (MI355X_MICROARCH.md, 'vector-instruction ISSUE
// cost'): for the same FLOPs the larger shape issues half the MFMA instructions and leaves 3× the issue
// cycles between them.
//   * the softmax row (the query) is the accumulator COLUMN (lane & 31), the keys sit in the 16
//     accumulator registers: a 32×32 result is the next MFMA's B operand after pairwise bf16 packing
//     (registers 8s'..8s'+7 = k-step s', element j of lane half h = row 16s' + 8(j>>2) + 4h + (j&3):
//     cdna_hip_programming.md §3), and V's column read (ds_read_b64_tr_b16 from the row-major LDS tile)
//     takes the same rows, so P never crosses lanes or LDS; a row max is 16 v_max3 + one permlane32 swap;
//   * LDS tiles [64 rows][64 bf16], 16-B chunk c of row r at c ^ swz32(r): conflict-free for the
//     32×32×16 row fragments (ds_read_b128 lane groups of the §LDS table) AND the transposed fragments
//     (4 consecutive rows × 4 chunks per 32-lane half); one image serves both (SQ_LDS_BANK_CONFLICT 0);
//   * row sums from a P·1 MFMA, the O rescale deferred until a row max grows past 2^8 (T13), mask work
//     only on the 32-key blocks the diagonal / Tk tail cuts.
// Measured (profiles/attention_r6.txt, GPT-2-small b64 causal): forward 0.187 -> 0.179 ms per layer.  The
// same re-tiling of dQ and dK/dV (with the dP accumulators started at −δ straight from LDS) was built,
// fp32-tested and measured SLOWER (0.559 -> 0.594 ms: dQ 238 -> 258 us, dK/dV 347 -> 352 us; MFMA busy
// 0.31-0.32 either way, 254 VGPRs in dK/dV); as the non-causal ViT forward (T = 197: 0.205 -> 0.212 ms)
// — both removed.  A software-pipelined dK/dV (query block 1's S / dP MFMAs issued before block 0's softmax
// VALU, block 0's dV / dK before block 1's; 246 VGPRs) closed half the gap (+2 %), sched_group_barrier
// interleaving of those phases nothing more, occupancy 1 (122 VGPR + 160 AGPR) lost 33 %: removed too.  Their unmasked loops were already lean (per 32 MFMAs: 32 fma / exp / mul / cvt_pk),
// so the remaining gap is stall structure (WAIT_ANY ≈ 0.3-0.4), not instruction count.
typedef float f32x16 __attribute__((ext_vector_type(16)));
#define MFMA32 __builtin_amdgcn_mfma_f32_32x32x16_bf16

RN_DEV int swz32(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }

// rows [r0, r0+64) (valid < rlim) of a [T][stride] bf16 matrix (64 columns) into a swz32 tile
RN_DEV void stage32_async(const u32x4& rs, long st, int r0, int rlim, const char* lds, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ins = wave * 2 + i;
        const int r = ins * 8 + (lane >> 3);
        const int cg = (lane & 7) ^ swz32(r);
        const bool ok = (r0 + r) < rlim;
        const uint32_t voff = ok ? (uint32_t)((((long)(r0 + r)) * st + cg * 8) * 2) : 0xFFFFFFF0u;
        dma16_async(rs, voff, lds_addr(lds + ins * 1024));
    }
}

// per-lane LDS offsets of the 32×32×16 fragments in a swz32 tile (rows of a 32-row block r0 = 32·X):
//   row fragment (A operand, row r0 + (lane&31), k-step s = columns 16s + 8h .. +7): rf[s]
//   transposed fragment (A operand, row = column 32·jd + (lane&31) of the tile, k-step rows
//   r0 + 16s' + 8(j>>2) + 4h + (j&3)): two ds_read_b64_tr_b16 at cf[jd][0] / cf[jd][1]
struct Frag32 {
    uint32_t rf[4];
    uint32_t cf[2][2];
};
RN_DEV Frag32 make_frag32(int lane) {
    Frag32 f;
    const int r = lane & 31, h = lane >> 5;
    const int sw = swz32(r);
#pragma unroll
    for (int s = 0; s < 4; ++s) f.rf[s] = r * 128 + (((2 * s + h) ^ sw) << 4);
    const int i = lane & 15, qq = i >> 2, pp = i & 3, gp = (lane >> 4) & 1;
#pragma unroll
    for (int jd = 0; jd < 2; ++jd)
#pragma unroll
        for (int sec = 0; sec < 2; ++sec) {
            const int R = 4 * h + qq + 8 * sec;
            const int ch = 4 * jd + 2 * gp + (pp >> 1);
            f.cf[jd][sec] = R * 128 + ((ch ^ swz32(R)) << 4) + (pp & 1) * 8;
        }
    return f;
}
// row fragment of 32-row block X, k-step s
RN_DEV s16x8 rfrag32(const char* t, int X, int s, const Frag32& f) {
    return *reinterpret_cast<const s16x8*>(t + X * 32 * 128 + f.rf[s]);
}
// transposed fragment: tile rows 16·ks + … (ks = 0..3 over the 64-row tile), tile columns 32·jd + (lane&31)
RN_DEV s16x8 tfrag32(const char* t, int ks, int jd, const Frag32& f) {
    const char* a = t + ks * 16 * 128;
    s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + f.cf[jd][0]));
    s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + f.cf[jd][1]));
    s16x8 r;
    r[0] = v0[0]; r[1] = v0[1]; r[2] = v0[2]; r[3] = v0[3];
    r[4] = v1[0]; r[5] = v1[1]; r[6] = v1[2]; r[7] = v1[3];
    return r;
}
// registers 8s'..8s'+7 of a 32×32 accumulator as a bf16 B-operand fragment (k-step s')
RN_DEV s16x8 pack16(const f32x16& x, int s2) {
    s16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = bfbits(x[8 * s2 + j]);
    return r;
}
RN_DEV float swap_max(float x) {
    auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
}
RN_DEV float swap_sum(float x) {
    auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}
// accumulator row of register i for lane half h
RN_DEV constexpr int arow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// store a wave's [64 d][32 cols] accumulator pair as rows (col = this lane's row of the output):
// out[d] = x·mul in bf16 (and, q8, e5m2 of the bf16 value with the delayed scale)
RN_DEV void store_rows32(const f32x16 (&x)[2], float mul, bf16* dst, uint8_t* q8dst, bool bf, float q8inv, float& q8m,
                         int h) {
#pragma unroll
    for (int jd = 0; jd < 2; ++jd)
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
            const int d = 32 * jd + 8 * c4 + 4 * h;
            const bf16x4 v = {(bf16)(x[jd][4 * c4] * mul), (bf16)(x[jd][4 * c4 + 1] * mul), (bf16)(x[jd][4 * c4 + 2] * mul),
                              (bf16)(x[jd][4 * c4 + 3] * mul)};
            if (q8dst) attn_q8_store4(q8dst + d, (float)v[0], (float)v[1], (float)v[2], (float)v[3], q8inv, q8m);
            if (bf) *reinterpret_cast<bf16x4*>(dst + d) = v;
        }
}

// ---------------- forward: 4 waves × 32 queries, 64-key tiles ----------------
// RES (Tq, Tk <= 256, RES_T): one workgroup of 8 waves per (b, h) holds the head's whole K and V in LDS
// (staged once, 64 KiB, no barrier inside the key loop): K / V are read from HBM once per head instead
// of once per 128-query block.  At ViT-B/16's T = 197 the streaming kernel reads K and V twice and
// the forward is HBM-bound (Q + 2K + 2V + O per layer).
// W8 (streaming, round 6): 8 waves × 32 queries per workgroup instead of 4: every staged K / V tile serves 256
// queries, so a causal head fetches its K / V tiles 40 times instead of 72 (T = 1024).
constexpr int RES_T = 256;
template <bool CAUSAL, bool RES = false, bool W8 = false>
__global__ void __launch_bounds__(RES || W8 ? 512 : 256, RES || W8 ? 4 : 2) attn_fwd32_k(AttnArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Frag32 fo = make_frag32(lane);
    constexpr int QB = RES || W8 ? 256 : 128;  // queries per workgroup
    int bh, qb;
    if constexpr (RES) {
        bh = blockIdx.x;
        qb = 0;
    } else {
        blk_map(p, (p.Tq + QB - 1) / QB, CAUSAL, bh, qb);
    }
    const int b = bh / p.H, hh = bh % p.H;
    const int q0 = qb * QB + wave * 32;  // this wave's first query
    const int qg = q0 + r;               // this lane's query
    const int off = p.Tk - p.Tq;
    const float sl2 = p.scale * LOG2E;
    const bf16* qbase = p.q + b * p.q_sb + hh * p.q_sh;
    const u32x4 krs = make_rsrc_sgpr(p.k + b * p.k_sb + hh * p.k_sh);
    const u32x4 vrs = make_rsrc_sgpr(p.v + b * p.v_sb + hh * p.v_sh);
    int kv_end = p.Tk;
    if (CAUSAL) kv_end = min(p.Tk, qb * QB + QB + off);
    const int nkv = kv_end > 0 ? (kv_end + 63) / 64 : 0;
    int nfull = p.Tk / 64;  // tiles every key of which every query of the block sees
    if (CAUSAL) nfull = min(nfull, max(0, (qb * QB + off + 1) / 64));
    nfull = min(nfull, nkv);
    // streaming: double-buffered [K 64 rows | V 64 rows] pairs; RES: K rows [0, 256) then V rows [0, 256)
#define Kt(i) (RES ? smem + (i) * 8192 : smem + ((i) & 1) * 16384)
#define Vt(i) (RES ? smem + 32768 + (i) * 8192 : smem + 8192 + ((i) & 1) * 16384)
    // one 64-row K tile and V tile (streaming): 4 waves issue 2 pieces of each, 8 waves 1
    auto stage_kv = [&](int t) {
        if constexpr (W8) {
            const int row = wave * 8 + (lane >> 3);
            const int cg = (lane & 7) ^ swz32(row);
            const bool ok = t * 64 + row < p.Tk;
            dma16_async(krs, ok ? (uint32_t)((((long)(t * 64 + row)) * p.k_st + cg * 8) * 2) : 0xFFFFFFF0u,
                        lds_addr(Kt(t) + wave * 1024));
            dma16_async(vrs, ok ? (uint32_t)((((long)(t * 64 + row)) * p.v_st + cg * 8) * 2) : 0xFFFFFFF0u,
                        lds_addr(Vt(t) + wave * 1024));
        } else {
            stage32_async(krs, p.k_st, t * 64, p.Tk, Kt(t), wave, lane);
            stage32_async(vrs, p.v_st, t * 64, p.Tk, Vt(t), wave, lane);
        }
    };
    if constexpr (RES) {
        // every 8-row piece of the nkv tiles (rows past Tk read as zeros: V's padding rows must be finite)
        for (int ins = wave; ins < nkv * 8; ins += 8) {
            const int row = ins * 8 + (lane >> 3);
            const int cg = (lane & 7) ^ swz32(row);
            const bool ok = row < p.Tk;
            dma16_async(krs, ok ? (uint32_t)(((long)row * p.k_st + cg * 8) * 2) : 0xFFFFFFF0u, lds_addr(smem + ins * 1024));
            dma16_async(vrs, ok ? (uint32_t)(((long)row * p.v_st + cg * 8) * 2) : 0xFFFFFFF0u,
                        lds_addr(smem + 32768 + ins * 1024));
        }
    } else if (nkv > 0) {
        stage_kv(0);
    }
    s16x8 qf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = gload16(qbase + (long)qg * p.q_st + 16 * s + 8 * h, qg < p.Tq);
#pragma unroll
    for (int s = 0; s < 4; ++s) asm volatile("" : "+v"(qf[s]));
    // Online softmax in log2 units (ms = running row max × sl2) with a deferred rescale (cdna_hip_programming.md
    // T13): O and the row sum are rescaled only when some row's tile max exceeds ms by more than THR, so p ≤
    // 2^THR (exact in fp32, the usual relative error in the bf16 P operand).  Row sums come from a P·1 MFMA
    // (every register of lsum holds the running sum of its column; [0] is read): 2 MFMAs per 32 keys
    // instead of 32 adds, the VALU being this kernel's bound (PMC, profiles/attention_r6f.txt).
    constexpr float THR = 8.f;
    float ms = -INFINITY;
    f32x16 oacc[2], lsum;
#pragma unroll
    for (int i = 0; i < 16; ++i) { oacc[0][i] = 0.f; oacc[1][i] = 0.f; lsum[i] = 0.f; }
    const short one = 0x3F80;  // bf16 1.0
    const s16x8 ones = {one, one, one, one, one, one, one, one};

    auto tile = [&](const int t, auto masked_c) {
        constexpr bool MASKED = decltype(masked_c)::value;
        const char* kt = Kt(t);
        const char* vt = Vt(t);
        const int kv0 = t * 64;
        // 32-key block class (wave-uniform): 0 dead (past Tk / above every query of this wave), 1 every key
        // visible to every query, 2 partial (the causal diagonal, the ragged Tk tail): per-element mask
        auto cls = [&](int kb) -> int {
            if constexpr (!MASKED) return 1;
            const int k0 = kv0 + 32 * kb;
            if (k0 >= p.Tk) return 0;
            if (CAUSAL && k0 > min(q0 + 31, p.Tq - 1) + off) return 0;
            return (k0 + 31 >= p.Tk || (CAUSAL && k0 + 31 > q0 + off)) ? 2 : 1;
        };
        f32x16 sacc[2];
        float pm = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            const int c_ = cls(kb);
            if (MASKED && c_ == 0) continue;
            f32x16 a;
#pragma unroll
            for (int i = 0; i < 16; ++i) a[i] = 0.f;
#pragma unroll
            for (int s = 0; s < 4; ++s) a = MFMA32(rfrag32(kt, kb, s, fo), qf[s], a, 0, 0, 0);
            if (MASKED && c_ == 2) {
                const int lim = CAUSAL ? min(qg + off, p.Tk - 1) : p.Tk - 1;
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (kv0 + 32 * kb + arow(i, h) > lim) a[i] = -INFINITY;
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) pm = fmaxf(pm, a[i]);
            sacc[kb] = a;
        }
        pm = swap_max(pm) * sl2;
        if (__builtin_amdgcn_ballot_w64(pm > ms + THR)) {  // wave-uniform, rare after the first tile
            const float mn = fmaxf(ms, pm);
            const float alpha = (ms == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ms - mn);
            oacc[0] *= alpha;
            oacc[1] *= alpha;
            lsum[0] *= alpha;
            ms = mn;
        }
        // (masked tiles: a row with no visible key so far keeps ms = -inf and p = 0)
        const float nms = (MASKED && ms == -INFINITY) ? 0.f : -ms;
        // O^T[d][q] += V^T[d][key] P^T[key][q];  lsum += 1 · P^T
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            if (MASKED && cls(kb) == 0) continue;
#pragma unroll
            for (int i = 0; i < 16; ++i) sacc[kb][i] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[kb][i], sl2, nms));
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const s16x8 pb = pack16(sacc[kb], s2);
#pragma unroll
                for (int jd = 0; jd < 2; ++jd) oacc[jd] = MFMA32(tfrag32(vt, 2 * kb + s2, jd, fo), pb, oacc[jd], 0, 0, 0);
                lsum = MFMA32(ones, pb, lsum, 0, 0, 0);
            }
        }
    };
    auto sync_prefetch = [&](int t) {
        if constexpr (RES) {
            if (t == 0) {
                vm_wait_all();
                __syncthreads();
            }
            return;
        }
        vm_wait_all();
        __syncthreads();
        if (t + 1 < nkv) stage_kv(t + 1);
    };
    const int nf = q0 < p.Tq ? nfull : 0;
    int t = 0;
    for (; t < nf; ++t) {
        sync_prefetch(t);
        tile(t, std::false_type{});
    }
    for (; t < nkv; ++t) {
        sync_prefetch(t);
        if (CAUSAL && t * 64 > q0 + 31 + off) continue;  // wave-uniform: every query precedes the tile
        if (q0 >= p.Tq) continue;
        tile(t, std::true_type{});
    }
#undef Kt
#undef Vt
    const float lt = lsum[0];  // (the full sum over both lane halves' keys: the MFMA summed them)
    if (qg < p.Tq) {
        const float inv = lt > 0.f ? 1.f / lt : 0.f;
        float dummy = 0.f;
        store_rows32(oacc, inv, p.o + b * p.o_sb + (long)qg * p.o_st + hh * p.o_sh, nullptr, true, 0.f, dummy, h);
        if (h == 0) p.lse[((long)b * p.H + hh) * p.Tq + qg] = (lt > 0.f) ? (ms + log2f(lt)) : INFINITY;
    }
}

// ---------------- backward, whole head resident (Tq, Tk <= RES_T; non-causal, no bias / dropout / e5m2) ----------------
// ViT-B/16 (T = 197) is HBM-bound in the streaming backward: the dQ kernel re-reads K / V per 128-query
// block, the dK/dV kernel Q / dO per 128-key block, and δ makes a round trip.  Here one persistent 8-wave
// workgroup per CU walks the heads; a head's Q, dO, K, V tiles sit in LDS (128 KiB) and every operand is read
// from HBM once:
//   A   δ of the wave's 32 queries (O rows in registers · dO rows of the tile); lse, −δ -> LDS   (barrier B0)
//   P1  wave w owns keys [32w, 32w+32): K / V rows in registers (loaded at the end of the previous head),
//       loops over every query block of the Q / dO tiles: S, dP, P, dS; dV^T += dO^T P, dK^T += Q^T dS (B1)
//       -> the Q / dO tiles of the NEXT head stream in during P2
//   P2  wave w owns queries [32w, 32w+32): loops over every key block from the K / V tiles:
//       S^T, dP^T, dS^T; dQ^T += K^T dS^T                                             (barrier B2)
//       -> the K / V tiles of the next head stream in during the next A + P1
// The 32×32×16 orientation and fragment helpers are the forward's (accumulator column = the row that
// owns the result, reduced index in registers).  Rows past Tq / Tk are zero-filled by the DMA and lse = +inf
// there, so only the ragged key block of P2 needs a mask.
// QKV bias partials (bsum): Σ_rows dV = Σ_q dO (softmax rows sum to 1; dO^T·1 on the MFMA), Σ_rows dK = 0 (a key
// bias shifts all of a query's scores alike), Σ_rows dQ by an in-register reduce-scatter of each wave's dQ^T —
// all written into the head's first 64-row block (the consumer sums every block).
constexpr int RES_LDS = 4 * 32768 + 2 * 1024 + 2 * 8 * 64 * 4;  // tiles, lse | −δ, bias partials
__global__ void __launch_bounds__(512, 2) attn_bwd_res_k(AttnArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* const Qt = smem;
    char* const Dt = smem + 32768;
    char* const Kt = smem + 65536;
    char* const Vt = smem + 98304;
    float* const lseL = reinterpret_cast<float*>(smem + 131072);  // [256] −lse / (scale·log2 e) (−inf past Tq)
    float* const ndL = lseL + 256;                                 // [256] −δ
    float* const bpL = ndL + 256;                                  // [2][8][64] bias partials: dQ, dV
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Frag32 fo = make_frag32(lane);
    const float sl2 = p.scale * LOG2E;
    const int BH = p.B * p.H, E = p.H * 64;
    const int nqb = (p.Tq + 31) / 32, nkb = (p.Tk + 31) / 32;
    const int w0 = wave * 32;  // this wave's keys (P1) and queries (P2)
    const short one = 0x3F80;
    const s16x8 ones = {one, one, one, one, one, one, one, one};

    s16x8 kf[4], vf[4], orw[4];
    float lsel;
    // registers of head bh: K / V rows w0 + r (P1's B operands), O rows w0 + r (δ), lse
    auto issue_regs = [&](int bh) {
        const int b = bh / p.H, hh = bh % p.H;
        int row = w0 + r;
        asm volatile("" : "+v"(row));  // (as in issue_tiles)
        const bool kok = row < p.Tk, qok = row < p.Tq;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int c = 16 * s + 8 * h;
            kf[s] = gload16(p.k + b * p.k_sb + (long)row * p.k_st + hh * p.k_sh + c, kok);
            vf[s] = gload16(p.v + b * p.v_sb + (long)row * p.v_st + hh * p.v_sh + c, kok);
            orw[s] = gload16(p.o + b * p.o_sb + (long)row * p.o_st + hh * p.o_sh + c, qok);
        }
        lsel = qok ? p.lse[((long)b * p.H + hh) * p.Tq + row] : INFINITY;
    };
    // two [256][64] tiles by LDS-DMA, 4 + 4 pieces per wave whatever T (rows past `lim` zero-filled): the K / V
    // pair must be this wave's 8 youngest loads (s_waitcnt vmcnt(8) below)
    auto issue_tiles = [&](const bf16* x0, long st0, const bf16* x1, long st1, int lim, char* t0, char* t1) {
        const u32x4 rs0 = make_rsrc_sgpr(x0), rs1 = make_rsrc_sgpr(x1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ins = wave + 8 * i;
            int row = ins * 8 + (lane >> 3);
            asm volatile("" : "+v"(row));  // recomputed per head: hoisted out of the head loop they were spilled
            const int cg = (lane & 7) ^ swz32(row);
            const bool ok = row < lim;
            dma16_async(rs0, ok ? (uint32_t)(((long)row * st0 + cg * 8) * 2) : 0xFFFFFFF0u, lds_addr(t0 + ins * 1024));
            dma16_async(rs1, ok ? (uint32_t)(((long)row * st1 + cg * 8) * 2) : 0xFFFFFFF0u, lds_addr(t1 + ins * 1024));
        }
    };
    auto issue_qdo = [&](int bh) {
        const int b = bh / p.H, hh = bh % p.H;
        issue_tiles(p.q + b * p.q_sb + hh * p.q_sh, p.q_st, p.dout + b * p.do_sb + hh * p.do_sh, p.do_st, p.Tq, Qt, Dt);
    };
    auto issue_kv = [&](int bh) {
        const int b = bh / p.H, hh = bh % p.H;
        issue_tiles(p.k + b * p.k_sb + hh * p.k_sh, p.k_st, p.v + b * p.v_sb + hh * p.v_sh, p.v_st, p.Tk, Kt, Vt);
    };

    // LDS byte addresses held whole in one register (opaque to the compiler, which otherwise re-adds the
    // >64 KiB tile bases — beyond ds_read's 16-bit offset — to every address in the loops); the block /
    // tile / dO-V offsets then ride the instructions' immediates
    auto la = [](const void* ptr, uint32_t off) -> uint32_t {
        uint32_t x = (uint32_t)(uintptr_t)(lds_void*)ptr + off;
        asm volatile("" : "+v"(x));
        return x;
    };
    auto ld16 = [](uint32_t a) -> s16x8 { return *reinterpret_cast<const lds_s16x8*>((size_t)a); };
    auto trd = [](uint32_t a0, uint32_t a1) -> s16x8 {  // a transposed fragment's two ds_read_b64_tr_b16
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)a0);
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(size_t)a1);
        return (s16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    };
    auto ldf4 = [](uint32_t a) -> f32x4 { return *reinterpret_cast<const lds_f32x4*>((size_t)a); };

    int bh = blockIdx.x;
    if (bh < BH) {
        issue_qdo(bh);
        issue_regs(bh);
        issue_kv(bh);
    }
    for (; bh < BH; bh += gridDim.x) {
        const int b = bh / p.H, hh = bh % p.H;
        const int nxt = bh + gridDim.x;
        // ---- A ----
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // everything but this head's K / V pieces
        __syncthreads();  // (every wave's Q / dO pieces)
        float dsum = 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const s16x8 dr = rfrag32(Dt, wave, s, fo);  // dO row w0 + r, the columns orw[s] holds
#pragma unroll
            for (int j = 0; j < 8; ++j)
                dsum += __uint_as_float((uint32_t)(unsigned short)orw[s][j] << 16) *
                        __uint_as_float((uint32_t)(unsigned short)dr[j] << 16);
        }
        const float ndl = -swap_sum(dsum);  // −δ of query w0 + r (0 past Tq: zero rows)
        const float lse2 = lsel;
        if (h == 0) {
            lseL[w0 + r] = -lsel / sl2;  // P1 starts its S accumulators here: P = exp2(acc · sl2)
            ndL[w0 + r] = ndl;
        }
        __syncthreads();  // B0: lse, −δ
        if (p.bsum) {  // Σ_q dO[q][d] over this wave's 32 queries: dO^T · 1 on the MFMA (P1's dV product with P = 1)
            const Frag32 f2 = make_frag32(lane);
            f32x16 u[2];
#pragma unroll
            for (int i = 0; i < 16; ++i) { u[0][i] = 0.f; u[1][i] = 0.f; }
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int jd = 0; jd < 2; ++jd) u[jd] = MFMA32(tfrag32(Dt, 2 * wave + s2, jd, f2), ones, u[jd], 0, 0, 0);
            if (r == 0) {  // every column of u holds the sums: lanes 0 / 32 write rows arow(i, h)
#pragma unroll
                for (int jd = 0; jd < 2; ++jd)
#pragma unroll
                    for (int i = 0; i < 16; ++i) bpL[512 + wave * 64 + 32 * jd + arow(i, h)] = u[jd][i];
            }
        }
        // ---- P1: dK, dV of keys w0 .. w0+31 ----
        f32x16 dk[2], dv[2];
#pragma unroll
        for (int i = 0; i < 16; ++i) { dk[0][i] = dk[1][i] = dv[0][i] = dv[1][i] = 0.f; }
        if (w0 < p.Tk) {
            // per-lane LDS pointers into the Q tile (dO: +32768, block X: +4096·X — immediates / one add each)
            uint32_t qr[4], qc[2][2];
#pragma unroll
            for (int s = 0; s < 4; ++s) qr[s] = la(Qt, fo.rf[s]);
#pragma unroll
            for (int jd = 0; jd < 2; ++jd) {
                qc[jd][0] = la(Qt, fo.cf[jd][0]);
                qc[jd][1] = la(Qt, fo.cf[jd][1]);
            }
            const uint32_t nda = la(ndL, 16 * h), lsa = la(lseL, 16 * h);
            s16x8 qa[4], da[4];
#pragma unroll 1
            for (int X = 0; X < nqb; ++X) {
                const int xo = X * 4096;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    qa[s] = ld16(qr[s] + xo);
                    da[s] = ld16(qr[s] + xo + 32768);
                }
                f32x16 sa, dp;
#pragma unroll
                for (int c4 = 0; c4 < 4; ++c4) {
                    const f32x4 nd = ldf4(nda + 128 * X + 32 * c4);
                    const f32x4 nl = ldf4(lsa + 128 * X + 32 * c4);
#pragma unroll
                    for (int e = 0; e < 4; ++e) { dp[4 * c4 + e] = nd[e]; sa[4 * c4 + e] = nl[e]; }
                }
#pragma unroll
                for (int s = 0; s < 4; ++s) sa = MFMA32(qa[s], kf[s], sa, 0, 0, 0);
#pragma unroll
                for (int s = 0; s < 4; ++s) dp = MFMA32(da[s], vf[s], dp, 0, 0, 0);
                // dO^T / Q^T fragments of the dV / dK products read now: their latency hides under the softmax VALU
                s16x8 to[2][2], tq[2][2];
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                    for (int jd = 0; jd < 2; ++jd) {
                        const int o = xo + s2 * 2048;
                        to[s2][jd] = trd(qc[jd][0] + o + 32768, qc[jd][1] + o + 32768);
                        tq[s2][jd] = trd(qc[jd][0] + o, qc[jd][1] + o);
                    }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    sa[i] = __builtin_amdgcn_exp2f(sa[i] * sl2);  // P
                    dp[i] *= sa[i];                               // dS
                }
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const s16x8 pb = pack16(sa, s2);
#pragma unroll
                    for (int jd = 0; jd < 2; ++jd) dv[jd] = MFMA32(to[s2][jd], pb, dv[jd], 0, 0, 0);
                }
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const s16x8 db = pack16(dp, s2);
#pragma unroll
                    for (int jd = 0; jd < 2; ++jd) dk[jd] = MFMA32(tq[s2][jd], db, dk[jd], 0, 0, 0);
                }
            }
        }
        // P2's B operands (Q / dO rows w0 + r) while the tiles are resident
        s16x8 qf[4], df[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            qf[s] = rfrag32(Qt, wave, s, fo);
            df[s] = rfrag32(Dt, wave, s, fo);
        }
        vm_wait_all();  // this head's K / V tiles (issued before A)
        if (w0 + r < p.Tk) {
            float dummy = 0.f;
            store_rows32(dk, p.scale, p.dk + b * p.dk_sb + (long)(w0 + r) * p.dk_st + hh * p.dk_sh, nullptr, true, 0.f,
                         dummy, h);
            store_rows32(dv, 1.f, p.dv + b * p.dv_sb + (long)(w0 + r) * p.dv_st + hh * p.dv_sh, nullptr, true, 0.f,
                         dummy, h);
        }
        __syncthreads();  // B1: Q / dO tiles free; K / V tiles and Σ_q dS complete
        if (nxt < BH) {
            issue_qdo(nxt);
            issue_regs(nxt);
        }
        // ---- P2: dQ of queries w0 .. w0+31 ----
        f32x16 dq[2];
#pragma unroll
        for (int i = 0; i < 16; ++i) { dq[0][i] = dq[1][i] = 0.f; }
        if (w0 < p.Tq) {
            uint32_t kr[4], kc[2][2];  // per-lane addresses in the K tile (V: +32768)
#pragma unroll
            for (int s = 0; s < 4; ++s) kr[s] = la(Kt, fo.rf[s]);
#pragma unroll
            for (int jd = 0; jd < 2; ++jd) {
                kc[jd][0] = la(Kt, fo.cf[jd][0]);
                kc[jd][1] = la(Kt, fo.cf[jd][1]);
            }
            s16x8 ka[4], va[4];
#pragma unroll 1
            for (int kb = 0; kb < nkb; ++kb) {
                const int ko = kb * 4096;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    ka[s] = ld16(kr[s] + ko);
                    va[s] = ld16(kr[s] + ko + 32768);
                }
                f32x16 sa, dp;
#pragma unroll
                for (int i = 0; i < 16; ++i) { sa[i] = 0.f; dp[i] = ndl; }
#pragma unroll
                for (int s = 0; s < 4; ++s) sa = MFMA32(ka[s], qf[s], sa, 0, 0, 0);
#pragma unroll
                for (int s = 0; s < 4; ++s) dp = MFMA32(va[s], df[s], dp, 0, 0, 0);
                // both chains issued before the softmax VALU (which then overlaps the dP chain); left alone the
                // scheduler put the dP MFMAs after the exps, exposing both chains' latency
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < 16; ++i) sa[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(sa[i], sl2, -lse2));
                if (32 * kb + 32 > p.Tk) {  // the ragged key block (wave-uniform)
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        if (32 * kb + arow(i, h) >= p.Tk) sa[i] = 0.f;
                }
#pragma unroll
                for (int i = 0; i < 16; ++i) dp[i] *= sa[i];
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const s16x8 db = pack16(dp, s2);
                    const int o = ko + s2 * 2048;
#pragma unroll
                    for (int jd = 0; jd < 2; ++jd) dq[jd] = MFMA32(trd(kc[jd][0] + o, kc[jd][1] + o), db, dq[jd], 0, 0, 0);
                }
            }
        }
        if (w0 + r < p.Tq) {
            float dummy = 0.f;
            store_rows32(dq, p.scale, p.dq + b * p.dq_sb + (long)(w0 + r) * p.dq_st + hh * p.dq_sh, nullptr, true, 0.f,
                         dummy, h);
        }
        if (p.bsum) {
            // Σ_q dQ[q][d] over this wave's 32 queries: a reduce-scatter of the dQ^T accumulator across the 32
            // lanes of each half (5 levels of XOR partners; at each, a lane keeps the half of its values its
            // lane bit selects and adds the partner's copy of them), so lane r ends with value v = r: d = 32·(r>>4)
            // + arow(r & 15, h).  Rows past Tq hold zeros (P = 0 there).  No LDS round trip, no extra barrier.
            float cur[32];
#pragma unroll
            for (int v = 0; v < 32; ++v) cur[v] = dq[v >> 4][v & 15];
#pragma unroll
            for (int m = 16; m >= 1; m >>= 1) {
                const bool hi = (r & m) != 0;
#pragma unroll
                for (int k = 0; k < m; ++k) {
                    const float keep = hi ? cur[k + m] : cur[k];
                    const float send = hi ? cur[k] : cur[k + m];
                    cur[k] = keep + __shfl_xor(send, m, 64);
                }
            }
            bpL[wave * 64 + 32 * (r >> 4) + arow(r & 15, h)] = cur[0];
        }
        __syncthreads();  // B2: K / V tiles free, bias partials complete
        if (p.bsum && threadIdx.x < 128) {
            const int part = threadIdx.x >> 6, d = lane;  // 0: dQ (and dK), 1: dV
            float a = 0.f;
#pragma unroll
            for (int w = 0; w < 8; ++w) a += bpL[part * 512 + w * 64 + d];
            const int nb64 = (p.Tq + 63) / 64;
            float* row = p.bsum + (long)b * nb64 * 3 * E + hh * 64 + d;
            if (part == 0) {
                row[0] = a * p.scale;
                row[E] = 0.f;
            } else {
                row[2 * E] = a;
            }
            for (int blk = 1; blk < nb64; ++blk) {
                float* z = row + (long)blk * 3 * E;
                if (part == 0) {
                    z[0] = 0.f;
                    z[E] = 0.f;
                } else {
                    z[2 * E] = 0.f;
                }
            }
        }
        if (nxt < BH) issue_kv(nxt);
    }
}

#undef MFMA32

// ============================== generic path (any D <= 256) ==============================
RN_DEV float bias_at(const AttnArgs& p, int b, int qi, int kj) {
    return p.bias ? p.bias[((long)(p.bias_b > 1 ? b : 0) * p.Tq + qi) * p.Tk + kj] : 0.f;
}
RN_DEV bool visible(const AttnArgs& p, int qi, int kj) { return !(p.causal && kj > qi + (p.Tk - p.Tq)); }

// one block per (b, h, q); scores in LDS (Tk floats)
__global__ void __launch_bounds__(256) attn_fwd_generic_k(AttnArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* sc = reinterpret_cast<float*>(smem);
    float* qv = sc + p.Tk;
    __shared__ float red[16];
    const int qi = blockIdx.x, bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
    const bf16* qp = p.q + b * p.q_sb + (long)qi * p.q_st + h * p.q_sh;
    for (int d = threadIdx.x; d < p.D; d += 256) qv[d] = bf2f(qp[d]);
    __syncthreads();
    float mx = -INFINITY;
    for (int kj = threadIdx.x; kj < p.Tk; kj += 256) {
        const bf16* kp = p.k + b * p.k_sb + (long)kj * p.k_st + h * p.k_sh;
        float s = 0.f;
        for (int d = 0; d < p.D; ++d) s += qv[d] * bf2f(kp[d]);
        s = s * p.scale + bias_at(p, b, qi, kj);
        if (!visible(p, qi, kj)) s = -INFINITY;
        sc[kj] = s;
        mx = fmaxf(mx, s);
    }
    mx = block_max(mx, red);
    __syncthreads();
    float sum = 0.f;
    const float ms = mx == -INFINITY ? 0.f : mx;
    for (int kj = threadIdx.x; kj < p.Tk; kj += 256) {
        float e = __expf(sc[kj] - ms);
        sc[kj] = e;
        sum += e;
    }
    sum = block_sum(sum, red);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    const float rd = p.p_drop > 0.f ? 1.f / (1.f - p.p_drop) : 1.f;
    if (p.p_drop > 0.f && p.seed_ptr) p.seed = *p.seed_ptr;
    for (int kj = threadIdx.x; kj < p.Tk; kj += 256) {
        float pv = sc[kj] * inv;
        if (p.p_drop > 0.f) pv = hash_uniform(p.seed, drop_idx(p, b, h, qi, kj)) >= p.p_drop ? pv * rd : 0.f;
        sc[kj] = pv;
    }
    __syncthreads();
    bf16* op = p.o + b * p.o_sb + (long)qi * p.o_st + h * p.o_sh;
    for (int d = threadIdx.x; d < p.D; d += 256) {
        float acc = 0.f;
        for (int kj = 0; kj < p.Tk; ++kj) acc += sc[kj] * bf2f(p.v[b * p.v_sb + (long)kj * p.v_st + h * p.v_sh + d]);
        op[d] = f2bf(acc);
    }
    if (threadIdx.x == 0) p.lse[((long)b * p.H + h) * p.Tq + qi] = sum > 0.f ? ms + __logf(sum) : INFINITY;
}

__global__ void __launch_bounds__(256) attn_bwd_generic_k(AttnArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* pp = reinterpret_cast<float*>(smem);   // P (undropped)
    float* ds = pp + p.Tk;                          // dS
    float* qv = ds + p.Tk;                          // q row
    float* dov = qv + p.D;                          // dO row
    __shared__ float red[16];
    const int qi = blockIdx.x, bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
    const bf16* qp = p.q + b * p.q_sb + (long)qi * p.q_st + h * p.q_sh;
    const bf16* dop = p.dout + b * p.do_sb + (long)qi * p.do_st + h * p.do_sh;
    const bf16* op = p.o + b * p.o_sb + (long)qi * p.o_st + h * p.o_sh;
    float dl = 0.f;
    for (int d = threadIdx.x; d < p.D; d += 256) {
        qv[d] = bf2f(qp[d]);
        dov[d] = bf2f(dop[d]);
        dl += dov[d] * bf2f(op[d]);
    }
    dl = block_sum(dl, red);
    const float L = p.lse[((long)b * p.H + h) * p.Tq + qi] * (p.lse_log2 ? LN2 : 1.f);
    const float rd = p.p_drop > 0.f ? 1.f / (1.f - p.p_drop) : 1.f;
    if (p.p_drop > 0.f && p.seed_ptr) p.seed = *p.seed_ptr;
    for (int kj = threadIdx.x; kj < p.Tk; kj += 256) {
        const bf16* kp = p.k + b * p.k_sb + (long)kj * p.k_st + h * p.k_sh;
        const bf16* vp = p.v + b * p.v_sb + (long)kj * p.v_st + h * p.v_sh;
        float s = 0.f, dp = 0.f;
        for (int d = 0; d < p.D; ++d) { s += qv[d] * bf2f(kp[d]); dp += dov[d] * bf2f(vp[d]); }
        s = s * p.scale + bias_at(p, b, qi, kj);
        float pv = (visible(p, qi, kj) && L != INFINITY) ? __expf(s - L) : 0.f;
        float pd = pv;
        if (p.p_drop > 0.f) {
            bool keep = hash_uniform(p.seed, drop_idx(p, b, h, qi, kj)) >= p.p_drop;
            pd = keep ? pv * rd : 0.f;
            dp = keep ? dp * rd : 0.f;
        }
        pp[kj] = pd;
        ds[kj] = pv * (dp - dl);
    }
    __syncthreads();
    bf16* dqp = p.dq + b * p.dq_sb + (long)qi * p.dq_st + h * p.dq_sh;
    for (int d = threadIdx.x; d < p.D; d += 256) {
        float acc = 0.f;
        for (int kj = 0; kj < p.Tk; ++kj) acc += ds[kj] * bf2f(p.k[b * p.k_sb + (long)kj * p.k_st + h * p.k_sh + d]);
        dqp[d] = f2bf(acc * p.scale);
    }
    // delta for the dK/dV kernel (dK/dV are NOT accumulated here: that took fp32 atomics across
    // query rows, i.e. a run-to-run varying summation order)
    if (threadIdx.x == 0) const_cast<float*>(p.delta)[((long)b * p.H + h) * p.Tq + qi] = dl;
}

// Generic-head-size dK/dV, deterministic: one block per key row j sums over the query rows in a
// fixed order — dVⱼ = Σᵢ P̃ᵢⱼ dOᵢ, dKⱼ = scale · Σᵢ dSᵢⱼ qᵢ with P, dP recomputed from q, k, v, dO,
// the forward's lse and delta = rowsum(dO∘O) written by attn_bwd_generic_k (same dropout mask:
// the hash of the same (b, h, i, j) index).  Scalar (odd head sizes only; 32/64/128 run on MFMA).
__global__ void __launch_bounds__(256) attn_bwd_generic_kv_k(AttnArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* pd = reinterpret_cast<float*>(smem);  // P̃ (dropped, rescaled) per query row
    float* ds = pd + p.Tq;                       // dS per query row
    float* kv = ds + p.Tq;                       // k row
    float* vv = kv + p.D;                        // v row
    const int kj = blockIdx.x, bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
    const bf16* kp = p.k + b * p.k_sb + (long)kj * p.k_st + h * p.k_sh;
    const bf16* vp = p.v + b * p.v_sb + (long)kj * p.v_st + h * p.v_sh;
    for (int d = threadIdx.x; d < p.D; d += 256) {
        kv[d] = bf2f(kp[d]);
        vv[d] = bf2f(vp[d]);
    }
    __syncthreads();
    const float lsc = p.lse_log2 ? LN2 : 1.f;
    const float rd = p.p_drop > 0.f ? 1.f / (1.f - p.p_drop) : 1.f;
    if (p.p_drop > 0.f && p.seed_ptr) p.seed = *p.seed_ptr;
    for (int qi = threadIdx.x; qi < p.Tq; qi += 256) {
        const bf16* qp = p.q + b * p.q_sb + (long)qi * p.q_st + h * p.q_sh;
        const bf16* dop = p.dout + b * p.do_sb + (long)qi * p.do_st + h * p.do_sh;
        const float L = p.lse[((long)b * p.H + h) * p.Tq + qi] * lsc;
        float pv = 0.f, dp = 0.f;
        if (visible(p, qi, kj) && L != INFINITY) {
            float sc = 0.f;
            for (int d = 0; d < p.D; ++d) {
                sc += bf2f(qp[d]) * kv[d];
                dp += bf2f(dop[d]) * vv[d];
            }
            pv = __expf(sc * p.scale + bias_at(p, b, qi, kj) - L);
        }
        float pdv = pv;
        if (p.p_drop > 0.f) {
            const bool keep = hash_uniform(p.seed, drop_idx(p, b, h, qi, kj)) >= p.p_drop;
            pdv = keep ? pv * rd : 0.f;
            dp = keep ? dp * rd : 0.f;
        }
        pd[qi] = pdv;
        ds[qi] = pv * (dp - p.delta[((long)b * p.H + h) * p.Tq + qi]);
    }
    __syncthreads();
    bf16* dkp = p.dk + b * p.dk_sb + (long)kj * p.dk_st + h * p.dk_sh;
    bf16* dvp = p.dv + b * p.dv_sb + (long)kj * p.dv_st + h * p.dv_sh;
    for (int d = threadIdx.x; d < p.D; d += 256) {
        float ak = 0.f, av = 0.f;
        for (int qi = 0; qi < p.Tq; ++qi) {
            const float dsv = ds[qi], pdq = pd[qi];
            if (dsv == 0.f && pdq == 0.f) continue;  // masked (causal / dropped) pairs
            ak += dsv * bf2f(p.q[b * p.q_sb + (long)qi * p.q_st + h * p.q_sh + d]);
            av += pdq * bf2f(p.dout[b * p.do_sb + (long)qi * p.do_st + h * p.do_sh + d]);
        }
        dkp[d] = f2bf(ak * p.scale);
        dvp[d] = f2bf(av);
    }
}


#define RN_DISPATCH3(KERN, grid, lds, st, args)                                                       \
    do {                                                                                               \
        const bool c_ = args.causal, b_ = args.bias != nullptr, d_ = args.p_drop > 0.f;              \
        if (c_) {                                                                                      \
            if (b_) { if (d_) KERN<true, true, true><<<grid, 256, lds, st>>>(args); else KERN<true, true, false><<<grid, 256, lds, st>>>(args); } \
            else { if (d_) KERN<true, false, true><<<grid, 256, lds, st>>>(args); else KERN<true, false, false><<<grid, 256, lds, st>>>(args); } \
        } else {                                                                                       \
            if (b_) { if (d_) KERN<false, true, true><<<grid, 256, lds, st>>>(args); else KERN<false, true, false><<<grid, 256, lds, st>>>(args); } \
            else { if (d_) KERN<false, false, true><<<grid, 256, lds, st>>>(args); else KERN<false, false, false><<<grid, 256, lds, st>>>(args); } \
        }                                                                                              \
    } while (0)

// RN_DISPATCH3 with trailing template arguments after <CAUSAL, BIAS, DROP>; kernels above 64 KiB of
// dynamic LDS are opted in on every launch (D = 128 only; the call is a host-side attribute write)
#define RN_DISPATCH3V(KERN, grid, lds, st, args, ...)                                                 \
    do {                                                                                               \
        const bool c_ = args.causal, b_ = args.bias != nullptr, d_ = args.p_drop > 0.f;              \
        auto k_ = c_ ? (b_ ? (d_ ? KERN<true, true, true, __VA_ARGS__> : KERN<true, true, false, __VA_ARGS__>)      \
                           : (d_ ? KERN<true, false, true, __VA_ARGS__> : KERN<true, false, false, __VA_ARGS__>))    \
                     : (b_ ? (d_ ? KERN<false, true, true, __VA_ARGS__> : KERN<false, true, false, __VA_ARGS__>)    \
                           : (d_ ? KERN<false, false, true, __VA_ARGS__> : KERN<false, false, false, __VA_ARGS__>)); \
        if ((lds) > 65536) (void)hipFuncSetAttribute((const void*)k_, hipFuncAttributeMaxDynamicSharedMemorySize, (lds)); \
        k_<<<grid, 256, lds, st>>>(args);                                                              \
    } while (0)

// MFMA path for head sizes 32 / 128 (one kernel family, templated on D): forward = the bias/dropout
// capable single-loop kernel, backward = dQ (+delta) then dK/dV, one 64-row group per wave.
template <int D>
void attn_fwd_mfma(AttnArgs& a, hipStream_t st) {
    constexpr int QBLK = D == 128 ? 64 : 128;
    dim3 grid(a.B * a.H * ((a.Tq + QBLK - 1) / QBLK));
    RN_DISPATCH3V(attn_fwd64_k, grid, 4 * kTB<D>, st, a, D, (D == 128 ? 2 : 3), (D == 128 ? 1 : 2));
}
template <int D>
void attn_bwd_mfma(AttnArgs& a, hipStream_t st) {
    dim3 g2(a.B * a.H * ((a.Tq + 63) / 64));
    dim3 g1(a.B * a.H * ((a.Tk + 63) / 64));
    RN_DISPATCH3V(attn_bwd_dq64_k, g2, 4 * kTB<D>, st, a, 2, 1, D);
    RN_DISPATCH3V(attn_bwd_dkdv64_k, g1, 2 * (2 * kTB<D> + 2048), st, a, (D == 128 ? 1 : 3), 1, D);
}

// Block order: head-interleaved (blk_map).  An XCD-grouped order was measured slower (GPT-2-small
// causal B64: fwd 0.177 -> 0.199 ms, bwd 0.571 -> 0.597 ms: a head's 8 query blocks then read the
// same K/V tiles at the same moment) and was removed in round 4.

// the MFMA kernels' requirements: D ∈ {32, 64, 128} and 16-B aligned rows (strides in elements)
bool mfma_head(int D) { return D == 32 || D == 64 || D == 128; }

}  // namespace

extern "C" {

// strides in elements: [b, t, h] for q, k, v, o ; d is contiguous
int rn_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const float* bias, int bias_b,
                const long* strides, int B, int H, int Tq, int Tk, int D, float scale, int causal, float p_drop,
                uint64_t seed, const uint64_t* seed_ptr, hipStream_t st) {
    AttnArgs a = {};
    a.seed_ptr = seed_ptr;
    a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v; a.o = (bf16*)o; a.lse = lse; a.bias = bias;
    a.q_sb = strides[0]; a.q_st = strides[1]; a.q_sh = strides[2];
    a.k_sb = strides[3]; a.k_st = strides[4]; a.k_sh = strides[5];
    a.v_sb = strides[6]; a.v_st = strides[7]; a.v_sh = strides[8];
    a.o_sb = strides[9]; a.o_st = strides[10]; a.o_sh = strides[11];
    a.B = B; a.H = H; a.Tq = Tq; a.Tk = Tk; a.D = D; a.causal = causal; a.bias_b = bias_b;
    a.scale = scale; a.p_drop = p_drop; a.seed = seed;
    const bool fast = mfma_head(D) && (a.q_st % 8 == 0) && (a.k_st % 8 == 0) && (a.v_st % 8 == 0) && (a.o_st % 4 == 0);
    if (fast && D != 64) {
        if (D == 32) attn_fwd_mfma<32>(a, st);
        else attn_fwd_mfma<128>(a, st);
    } else if (fast) {
        dim3 grid(B * H * ((Tq + 127) / 128));
        // plain, Tq / Tk <= 256: the whole-head-resident 32×32×16 kernel (ViT-B/16 T = 197: 0.205 -> 0.165 ms per
        // layer, profiles/attention_resident_r6.txt); plain causal: the 32×32×16 kernel with 8 waves (256 queries) per
        // workgroup (GPT-2-small b64: 0.187 -> 0.179 -> 0.170 ms per layer, profiles/attention_r6.txt,
        // attention_memtraffic_r6.txt); plain non-causal: the 16×16×32 split-loop v2 kernel; additive bias or
        // dropout (the reference blocks): the single-loop kernel
        if (!bias && p_drop == 0.f && Tq <= RES_T && Tk <= RES_T) {
            // whole head resident (ViT-B/16, T = 197): one 8-wave workgroup per (b, h)
            if (causal) attn_fwd32_k<true, true><<<dim3(B * H), 512, 65536, st>>>(a);
            else attn_fwd32_k<false, true><<<dim3(B * H), 512, 65536, st>>>(a);
        } else if (!bias && p_drop == 0.f && causal) {
            attn_fwd32_k<true, false, true><<<dim3(B * H * ((Tq + 255) / 256)), 512, 32768, st>>>(a);
        } else if (!bias && p_drop == 0.f) {
            attn_fwd64v2_k<false, 3, true><<<grid, 256, 32768, st>>>(a);
        } else {
            RN_DISPATCH3(attn_fwd64_k, grid, 32768, st, a);
        }
    } else {
        if (D > 256 || Tk > 12000) return -1;
        dim3 grid(Tq, B * H);
        attn_fwd_generic_k<<<grid, 256, (Tk + D) * 4, st>>>(a);
    }
    return 0;
}

// strides: q,k,v,o,do,dq,dk,dv (each b,t,h).  delta: B*H*Tq floats workspace.
// dk32/dv32: generic path scratch (B*Tk*H*D floats each, zeroed by caller) or null.
void rn_fp8_roll_bf8(float* state, hipStream_t st);  // fp8.hip
long rn_attn_q8_part_floats(int B, int H, int Tq, int Tk);

int rn_attn_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o, const float* lse,
                const float* bias, int bias_b, void* dq, void* dk, void* dv, float* delta, float* dk32, float* dv32,
                const long* s, int B, int H, int Tq, int Tk, int D, float scale, int causal, float p_drop,
                uint64_t seed, const uint64_t* seed_ptr, float* bsum, void* q8, float* q8st, int q8_only, float* q8part,
                hipStream_t st) {
    AttnArgs a = {};
    // q8: the e5m2 twin of the buffer dq / dk / dv live in (same element offsets from dq)
    a.q8 = (uint8_t*)q8; a.q8st = q8st; a.q8_only = q8_only;
    if (q8) {
        a.q8k = (uint8_t*)q8 + ((const bf16*)dk - (const bf16*)dq);
        a.q8v = (uint8_t*)q8 + ((const bf16*)dv - (const bf16*)dq);
        // q8part: >= 8·B·H·ceil(T/64) floats (rn_attn_q8_part_floats): both kernels' per-wave partials
        a.q8part = q8part;
        a.q8part2 = q8part + 4L * B * H * ((Tq + 63) / 64);
    }
    a.seed_ptr = seed_ptr;
    a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v; a.o = (bf16*)o; a.lse = (float*)lse;
    a.bias = bias; a.dout = (const bf16*)dout; a.dq = (bf16*)dq; a.dk = (bf16*)dk; a.dv = (bf16*)dv; a.delta = delta;
    a.q_sb = s[0]; a.q_st = s[1]; a.q_sh = s[2]; a.k_sb = s[3]; a.k_st = s[4]; a.k_sh = s[5];
    a.v_sb = s[6]; a.v_st = s[7]; a.v_sh = s[8]; a.o_sb = s[9]; a.o_st = s[10]; a.o_sh = s[11];
    a.do_sb = s[12]; a.do_st = s[13]; a.do_sh = s[14]; a.dq_sb = s[15]; a.dq_st = s[16]; a.dq_sh = s[17];
    a.dk_sb = s[18]; a.dk_st = s[19]; a.dk_sh = s[20]; a.dv_sb = s[21]; a.dv_st = s[22]; a.dv_sh = s[23];
    a.B = B; a.H = H; a.Tq = Tq; a.Tk = Tk; a.D = D; a.causal = causal; a.bias_b = bias_b;
    a.scale = scale; a.p_drop = p_drop; a.seed = seed; a.dk32 = dk32; a.dv32 = dv32; a.bsum = bsum;
    const bool fast = mfma_head(D) && (a.q_st % 8 == 0) && (a.k_st % 8 == 0) && (a.v_st % 8 == 0) &&
                      (a.do_st % 8 == 0) && (a.o_st % 8 == 0) && (a.dq_st % 4 == 0) && (a.dk_st % 4 == 0) &&
                      (a.dv_st % 4 == 0) && (a.o_sh % 8 == 0) && (a.do_sh % 8 == 0);
    if (bsum && !(fast && Tq == Tk)) return -2;  // bias partials: fast self-attention path only
    // the forward chose its path with its own stride test: lse is base 2 iff that one was fast
    a.lse_log2 = mfma_head(D) && (a.q_st % 8 == 0) && (a.k_st % 8 == 0) && (a.v_st % 8 == 0) && (a.o_st % 4 == 0);
    if (fast && !a.lse_log2) return -1;  // cannot happen (the backward test is stricter); never mix units
    if (q8 && !(fast && D == 64)) return -3;  // e5m2 dQKV: the D = 64 kernels only (the caller quantises instead)
    if (q8) {
        rn_fp8_roll_bf8(q8st, st);  // the consumer's delayed e5m2 scale, before both kernels
        (void)hipMemsetAsync(q8part, 0, (size_t)rn_attn_q8_part_floats(B, H, Tq, Tk) * sizeof(float), st);
    }
    if (fast && D != 64) {
        if (D == 32) attn_bwd_mfma<32>(a, st);
        else attn_bwd_mfma<128>(a, st);
    } else if (fast) {
        // dQ first: it also produces delta = rowsum(dO∘O), which the dK/dV kernel reads
        dim3 g2(B * H * ((Tq + 63) / 64));
        dim3 g1(B * H * ((Tk + 63) / 64));
        // plain causal / non-causal: two 64-query groups per wave in dQ (bwd -11 % at GPT-2-small
        // shapes) and two 64-key groups per wave in dK/dV (-2.4 %, occupancy 2 at 240 VGPRs);
        // bias / dropout: one group per wave
        if (!bias && p_drop == 0.f && !causal && !q8 && Tq <= RES_T && Tk <= RES_T) {
            // whole head resident, persistent over the CUs (ViT-B/16, T = 197)
            static unsigned long long res_devs = 0;
            static int res_cus[64];
            int dev = 0;
            (void)hipGetDevice(&dev);
            const unsigned long long bit = 1ull << (dev & 63);
            if (!(res_devs & bit)) {
                (void)hipFuncSetAttribute((const void*)attn_bwd_res_k, hipFuncAttributeMaxDynamicSharedMemorySize, RES_LDS);
                int cus = 256;
                (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
                res_cus[dev & 63] = cus > 0 ? cus : 256;
                res_devs |= bit;
            }
            attn_bwd_res_k<<<std::min(B * H, res_cus[dev & 63]), 512, RES_LDS, st>>>(a);
            return 0;
        }
        if (!bias && p_drop == 0.f) {
            dim3 g2b(B * H * ((Tq + 127) / 128));
            if (causal) attn_bwd_dq64_k<true, false, false, 2, 2><<<g2b, 256, 32768, st>>>(a);
            else attn_bwd_dq64_k<false, false, false, 2, 2><<<g2b, 256, 32768, st>>>(a);
        } else {
            RN_DISPATCH3(attn_bwd_dq64_k, g2, 32768, st, a);
        }
        if (!bias && p_drop == 0.f) {
            dim3 g1b(B * H * ((Tk + 127) / 128));
            if (causal) attn_bwd_dkdv64_k<true, false, false, 2, 2><<<g1b, 256, 36864, st>>>(a);
            else attn_bwd_dkdv64_k<false, false, false, 2, 2><<<g1b, 256, 36864, st>>>(a);
        } else {
            RN_DISPATCH3(attn_bwd_dkdv64_k, g1, 36864, st, a);
        }
        if (q8) {  // (the buffer was zeroed before the launches: a wave that never reaches its store leaves 0)
            const int nk = (!bias && p_drop == 0.f) ? B * H * ((Tk + 127) / 128) : B * H * ((Tk + 63) / 64);
            const int n = (int)(a.q8part2 - a.q8part) + 4 * nk;
            attn_amax_reduce_k<<<std::min(256, (n + 4095) / 4096), 256, 0, st>>>(a.q8part, n, q8st);
        }
    } else {
        if (D > 256 || Tk > 12000 || Tq > 12000) return -1;
        // dQ + delta per query row, then dK/dV per key row: no atomics, bitwise repeatable
        dim3 grid(Tq, B * H);
        const int lds_q = (2 * Tk + 2 * D) * 4, lds_k = (2 * Tq + 2 * D) * 4;
        if (lds_q > 65536)
            (void)hipFuncSetAttribute((const void*)attn_bwd_generic_k, hipFuncAttributeMaxDynamicSharedMemorySize, lds_q);
        attn_bwd_generic_k<<<grid, 256, lds_q, st>>>(a);
        dim3 gkv(Tk, B * H);
        if (lds_k > 65536)
            (void)hipFuncSetAttribute((const void*)attn_bwd_generic_kv_k, hipFuncAttributeMaxDynamicSharedMemorySize, lds_k);
        attn_bwd_generic_kv_k<<<gkv, 256, lds_k, st>>>(a);
        (void)dk32;
        (void)dv32;
    }
    return 0;
}

int rn_attn_is_fast(int D) { return mfma_head(D); }
long rn_attn_q8_part_floats(int B, int H, int Tq, int Tk) {
    return 4L * B * H * ((Tq + 63) / 64) + 4L * B * H * ((Tk + 63) / 64);
}

}  // extern "C"
