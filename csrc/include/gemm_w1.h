// One-wave-per-SIMD persistent 256×256 GEMM (tile config 11): 4 waves × 512 registers per lane,
// the 256×256 fp32 accumulator (256 registers per lane) in the accumulator file, and the previous
// output tile's epilogue interleaved into the next tile's first K-tile.
//
// Why (round-5 redesign of the forward x·Wᵀ GEMM, bf16 and fp8; the 8-wave cfg-9 kernel stays for
// the other layouts and epilogues):
//   * cfg 9 (gemm_pk.h) runs 2 waves per SIMD at ≤ 256 registers each: its accumulators fill half the
//     register file, so an output tile's epilogue cannot overlap the next tile's MFMAs — the matrix
//     cores idle while the tile is converted and stored, and four phases later the counted waits
//     retire those stores too.  At K = 768 (bf16) / 1024 (fp8) that epilogue was 35-42 % of the GEMM
//     (profiles/gemm_k_sweep_r1d.txt, fp8_gemm_ab_r2r.txt: 11 µs per fp8 tile against 15 µs of main
//     loop), and the fp8 main loop moved the bf16 loop's bytes per MFMA;
//   * here one wave owns a 64×256 strip of the tile (4 A fragments × 16 B fragments = 64 MFMAs per
//     128-byte K-tile: 2048 MFMA cycles against 40 ds_read_b128), so per staged byte the wave issues
//     2× the MFMA work of cfg 9, and the freed registers hold the epilogue in flight: at the next
//     tile's first K-tile, right before the MFMAs of B-fragment pair p overwrite their accumulators,
//     pair p of the finished tile is converted and stored (4 × 16-B stores per lane) — the stores
//     drain under the MFMAs and the counted waits allow them a K-tile and a half to complete.
//
// Structure (per workgroup: one CU, 256 threads, 160 KiB LDS):
//   * the grid walks 256×256 output tiles persistently (XCD remap + GROUP_M grouping, cfg 9's order);
//   * operands arrive by LDS-DMA in 128-byte K-tiles (64 bf16 / 128 e4m3 k): A rows (32 KiB) into a
//     2-stage ring, B rows (32 KiB) into a 3-stage ring.  Wave w stages and reads A rows 64w..64w+63
//     only — A needs no barrier; every wave reads all of B: one barrier per K-tile;
//   * a K-tile is 16 blocks j (B fragment j × the 4 A fragments = 4 MFMAs): B fragment j + 3 is read
//     in block j, the DMA of K-tile t + 2 goes out in blocks 1-8 (two LDS-DMA per block: A(t+2) into
//     the A slot whose fragments are already in registers, B(t+2) into the slot the last barrier
//     freed), the counted wait for K-tile t + 1 + lgkmcnt(0) + s_barrier sit before block 13, after
//     which A(t+1) and B(t+1) fragments 0-2 are read under blocks 13-15's MFMAs;
//   * B fragments are row-permuted (pk_frag_b: pair p = columns 32p..32p+31) so each lane ends with 8
//     contiguous output columns per A fragment: one 16-B store per (A fragment, pair);
//   * bias is folded into the first K-tile as the MFMAs' C operand (no epilogue add); the next tile's
//     bias is loaded (8 × 16-B per lane, compiler-invisible, counted) at the start of the tile's last
//     K-tile.  fp8: the per-tensor scales are powers of two (ops/fp8.py) and ride the scaled MFMA's
//     E8M0 block-scale operands, so the fp8 epilogue is the bf16 one;
//   * vmcnt bookkeeping (every VMEM op is compiler-invisible asm): per K-tile the issue order is
//     [bias loads (last K-tile of a tile)] [16 DMA, blocks 1-8] [stores of the previous tile, blocks
//     1, 3, .., 15 (first K-tile)]; the wait before block 13 leaves the ops younger than K-tile t + 1's
//     DMA in flight: this K-tile's bias / DMA / stores issued so far plus the previous K-tile's stores
//     issued after its last DMA (w1_wait_count).
// Requirements (host-checked): both operands K-contiguous, K a multiple of 128 bytes with ≥ 2 K-tiles,
// N % 8 == 0, ldc % 8 == 0, 16-B aligned operands.
#pragma once
#include "gemm_pk.h"

namespace rn_gemm_detail {

constexpr int W1_STAGE = 32768;       // one operand stage: 256 rows × 128 B
constexpr int W1_A0 = 0;              // A ring: 2 stages
constexpr int W1_B0 = 2 * W1_STAGE;   // B ring: 3 stages
constexpr int W1_LDS = 5 * W1_STAGE;  // 160 KiB
constexpr int W1_WAIT_J = 13;         // block that opens with the end-of-K-tile wait + barrier

enum { W1_EPI = 1, W1_STEADY = 2, W1_LAST = 3, W1_RES0 = 4 };  // W1_RES0 + q, q = 0..3: residual bodies

// VMEM ops a K-tile issues before its end-of-K-tile wait (block 13): the wait for K-tile t + 1 (whose
// DMA went out in K-tile t - 1's blocks 1-8) leaves exactly these in flight.  Ops of K-tile t - 1
// issued after its DMA (an EPI's stores of blocks 9-15) are waited for too: conservative, no branch.
// (a residual body's 8 loads go out at its start, before its DMA: outside the allowance, so this wait
// retires them)
constexpr int w1_before_wait(int kind) { return (kind == W1_LAST ? 8 : 0) + 16 + (kind == W1_EPI ? 24 : 0); }
// names 8 registers as redefined here, after the wait that retired their loads (no consumer above it)
RN_DEV void w1_touch8(u32x4* v) {
    asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]));
}
static_assert(w1_before_wait(W1_EPI) <= 63, "vmcnt range");

struct W1Frag {
    s16x8 lo, hi;  // 16-B chunks g and g + 4 of the fragment row (k-steps 0 / 1 of bf16; one 32-B e4m3 operand)
};

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// 16-B load the compiler does not count (the next tile's bias): the caller retires it with a counted
// wait that names the destination (w1_pin8), so no consumer is scheduled above that wait
RN_DEV void w1_ld16(u32x4& v, const u32x4& rs, uint32_t voff) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(rs) : "memory");
}
template <int N>
RN_DEV void w1_pin8(u32x4* v) {
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
                 : "n"(N)
                 : "memory");
}
#pragma clang diagnostic pop

template <int FP8>
RN_DEV f32x4 w1_mma(const W1Frag& b, const W1Frag& a, f32x4 c, int eb, int ea) {
    if constexpr (FP8) {
        return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(pk_cat8(b.lo, b.hi), pk_cat8(a.lo, a.hi), c, 0, 0, 0,
                                                                eb, 0, ea);
    } else {
        (void)eb;
        (void)ea;
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b.lo, a.lo, c, 0, 0, 0);
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(b.hi, a.hi, c, 0, 0, 0);
    }
}

// buffer descriptor from wave-uniform values, every word through readfirstlane (so the compiler can
// prove it uniform and keep it in SGPRs: asm "s" operands)
RN_DEV u32x4 w1_rsrc(const void* base, uint32_t bytes) {
    const uint64_t bp = (uint64_t)base;
    u32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    r[2] = __builtin_amdgcn_readfirstlane(bytes);
    r[3] = 0x00020000u;
    return r;
}

// an opaque copy: offsets derived from it are recomputed where they are used instead of being
// hoisted out of the tile loop as dozens of lane constants (which the 256 arch VGPRs cannot hold
// next to the fragments: the MI355X guide's "lane-constant address hoisted to kernel entry" pitfall)
RN_DEV uint32_t w1_opq(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}
// the same for a wave-uniform value (SGPR): its products are recomputed per use, not kept as dozens of
// hoisted SGPR constants (which spill into VGPR lanes)
RN_DEV int w1_opq_s(int x) {
    asm volatile("" : "+s"(x));
    return x;
}

// E8M0 exponent of a power-of-two scale (its biased float exponent); 127 = 1.0
RN_DEV int w1_e8m0(const float* s) {
    if (!s) return 127;
    const uint32_t u = __builtin_bit_cast(uint32_t, *s);
    return (int)((u >> 23) & 0xFF);
}

// DBG (timing ablations, REPLICANN_W1_DBG; outputs wrong): bit 0 issues the epilogue stores out of range
// (same instructions, no traffic), bit 1 the operand DMA (no HBM/L2 traffic; the LDS is still written)
// RES: + residual (x·Wᵀ + b + r; p.res, row stride p.ldc) added by MFMA — see the residual bodies below
template <int FP8, int ACT, bool ALPHA, bool BKC, int DBG = 0, bool RES = false>
__global__ void __launch_bounds__(256, 1) gemm_w1(GemmArgs p) {
    static_assert(!RES || (BKC && !ALPHA), "w1 residual: x·Wᵀ layout, no alpha");
    static_assert(ACT == ACT_NONE, "w1: forward epilogues without activation (activations: cfg 9)");
    static_assert(!(FP8 && ALPHA), "fp8: the scales ride the MFMA");
    static_assert(BKC || !FP8, "w1: fp8 operands K-contiguous");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int G = lane >> 4;
    const int tiles = p.tiles_m * p.tiles_n;
    const int grid = gridDim.x;
    const int bid = xcd_remap(blockIdx.x, grid);
    const int nk = p.K >> 7;  // 128-byte K-tiles per output tile (host: nk >= 2)
    const int n_items = (tiles - bid + grid - 1) / grid;
    if (n_items <= 0) return;
    const long lda = p.lda, ldb = p.ldb;  // bytes (host); ldc in elements

    // scales: fp8 E8M0 exponents (src0 = B, src1 = A); bf16 alpha multiply
    const int eb = FP8 ? w1_e8m0(p.sb) : 127, ea = FP8 ? w1_e8m0(p.sa) : 127;
    float alpha = 1.f;
    if constexpr (ALPHA) alpha = *p.alpha;
    asm volatile("" ::"v"(alpha));

    auto clamp_u = [](long v) -> uint32_t { return v <= 0 ? 0u : (v > 0x7FFFFF00L ? 0x7FFFFF00u : (uint32_t)v); };
    // ---- tile walk: the tile being computed (m0, n0), the next one (m1, n1; has1), the one whose
    // epilogue is pending (pm0, pn0) ----
    auto item_mn = [&](int s, int& m0, int& n0) {
        int tm, tn;
        group_tile(bid + s * grid, p.tiles_m, p.tiles_n, tm, tn);
        m0 = tm * 256;
        n0 = tn * 256;
    };
    int m0 = 0, n0 = 0, m1 = 0, n1 = 0, pm0 = 0, pn0 = 0;
    bool has1 = false, pm_live = false;
    item_mn(0, m0, n0);
    auto set_next = [&](int s) {
        has1 = s < n_items;
        if (has1) item_mn(s, m1, n1);
    };
    set_next(1);

    // per-lane DMA source offsets: rows 64w + 8i + (lane>>3) of the stage, 16-B chunk (lane&7) ^ swizzle
    // (A: swz_kc, B: swz_kcp; both depend on i only through i & 1 / i & 3)
    const int dr = 64 * w + (lane >> 3);
    uint32_t a_off[2], b_off[4];
    [[maybe_unused]] int b_col[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int r = dr + 8 * q;
        a_off[q] = (uint32_t)((long)r * lda + (((lane & 7) ^ swz_kc(r)) << 4));
    }
    if constexpr (BKC) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r = dr + 8 * q;
            b_off[q] = (uint32_t)((long)r * ldb + (((lane & 7) ^ swz_kcp(r)) << 4));
        }
    } else {
        // MN-contiguous B ([k][n] rows, the data gradient dY·W): wave w stages sub-image w = columns
        // 64w..64w+63 of the 64 k rows, k row 8i + (lane>>3), 8-column chunk (lane&7) ^ swz_mnp(k)
        // (pk_stage<false, true>'s image); the swizzle depends on i only through i & 1
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int r = 8 * q + (lane >> 3);
            b_col[q] = 64 * w + (((lane & 7) ^ swz_mnp(r)) << 3);
            b_off[q] = (uint32_t)((long)r * ldb + b_col[q] * 2);
        }
        b_off[2] = b_off[3] = 0u;
    }
    // descriptors of K-tile d of the tile (d >= nk: K-tile d - nk of the next tile; past the block's
    // last tile: zero records, every lane out of range — the DMA zero-fills and moves nothing)
    auto dma_rs = [&](bool isA, int d) -> u32x4 {
        const bool nxt = d >= nk;
        const int dd = nxt ? d - nk : d;
        const bool live = !nxt || has1;
        const int r0 = isA ? (nxt ? m1 : m0) : (nxt ? n1 : n0);
        const long ld = isA ? lda : ldb;
        if (!BKC && !isA) {  // K-tile dd = k rows 64dd..64dd+63 (bf16), columns from r0; N tail per lane
            const char* base = (const char*)p.B + (long)(64 * dd) * ld + (long)r0 * 2;
            const long n = live ? (long)((p.K >> 1) - 64 * dd) * ld - (long)r0 * 2 : 0;
            return w1_rsrc(base, clamp_u(n));
        }
        const char* base = (const char*)(isA ? p.A : p.B) + (long)r0 * ld + dd * 128;
        const long n = live ? (long)((isA ? p.M : p.N) - r0) * ld - dd * 128 : 0;
        return w1_rsrc(base, clamp_u(n));
    };
    // columns of the tile K-tile d belongs to that exist (MN-contiguous B: the per-lane N-tail check)
    auto b_ncols = [&](int d) -> int { return p.N - (d >= nk ? n1 : n0); };
    auto dma_one = [&](const u32x4& rs, bool isA, int slot, int i, int ncols) {
        uint32_t off;
        if (isA) off = w1_opq(a_off[i & 1]) + (uint32_t)((i & ~1) * 8 * w1_opq_s((int)lda));
        else if constexpr (BKC) off = w1_opq(b_off[i & 3]) + (uint32_t)((i & ~3) * 8 * w1_opq_s((int)ldb));
        else {
            off = w1_opq(b_off[i & 1]) + (uint32_t)((i & ~1) * 8 * w1_opq_s((int)ldb));
            off = (int)w1_opq((uint32_t)b_col[i & 1]) < ncols ? off : 0xFFFFFFF0u;
        }
        const uint32_t dst = lds_addr(smem) + (isA ? W1_A0 : W1_B0) + slot * W1_STAGE + (uint32_t)((8 * w + i) * 1024);
        if constexpr ((DBG & 2) != 0) off = 0xFFFFFFF0u;
        dma16_at(rs, off, dst);
    };

    // ---- LDS fragment addresses (per lane; + slot base + immediates) ----
    // A fragment i: rows 16i + (lane & 15) of the wave's 64-row region, chunks G and G + 4
    const int ar = lane & 15;
    const uint32_t a_lo = (uint32_t)(w * 8192 + ar * 128 + ((G ^ swz_kc(ar)) << 4));
    const uint32_t a_hi = (uint32_t)(w * 8192 + ar * 128 + (((G + 4) ^ swz_kc(ar)) << 4));
    // B fragment jj (pair p = jj >> 1, half h = jj & 1): pk_frag_b's permuted rows
    //   32p + 8·(i>>2) + 4h + (i&3), i = lane & 15; the lane part is independent of p and h
    const int bi = lane & 15;
    const int brow = 8 * (bi >> 2) + (bi & 3);
    const uint32_t b_lo = (uint32_t)(brow * 128 + ((G ^ swz_kcp(brow)) << 4));
    const uint32_t b_hi = (uint32_t)(brow * 128 + (((G + 4) ^ swz_kcp(brow)) << 4));
    // MN-contiguous B (pk_frag_b<false> on the 4 sub-images of a stage): k row 8G + (bi>>2) (+4, +32 for
    // k-step 1), chunk (4·(pair & 1) + (bi&3)) ^ swz_mnp, 8-B half (jj & 1) ^ (bi & 1): four lane offsets
    [[maybe_unused]] uint32_t b_mn[2][2];
    if constexpr (!BKC) {
        const int k0 = 8 * G + (bi >> 2), pl = bi & 3;
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                b_mn[e][h] = (uint32_t)(k0 * 128 + (((4 * e + pl) ^ swz_mnp(k0)) << 4) + ((h ^ (pl & 1)) << 3));
    }
    auto rd_a = [&](int slot, int i) -> W1Frag {
        const char* base = smem + W1_A0 + slot * W1_STAGE + i * 2048;
        return {*reinterpret_cast<const s16x8*>(base + a_lo), *reinterpret_cast<const s16x8*>(base + a_hi)};
    };
    auto rd_b = [&](int slot, int jj) -> W1Frag {
        if constexpr (!BKC) {
            typedef __attribute__((address_space(3))) s16x4 lds4;
            const char* base = smem + W1_B0 + slot * W1_STAGE + (jj >> 2) * 8192 + w1_opq(b_mn[(jj >> 1) & 1][jj & 1]);
            s16x4 v[4];
#pragma unroll
            for (int t = 0; t < 4; ++t)  // (k-step t >> 1, rows +4 for t & 1)
                v[t] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(base + (t >> 1) * 4096 + (t & 1) * 512));
            W1Frag f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                f.lo[e] = v[0][e];
                f.lo[4 + e] = v[1][e];
                f.hi[e] = v[2][e];
                f.hi[4 + e] = v[3][e];
            }
            return f;
        }
        const char* base = smem + W1_B0 + slot * W1_STAGE + (jj >> 1) * 4096 + (jj & 1) * 512;
        return {*reinterpret_cast<const s16x8*>(base + b_lo), *reinterpret_cast<const s16x8*>(base + b_hi)};
    };

    f32x4 acc[4][16];
    W1Frag Acur[4], Bq[3];  // Bq: B fragments 0-2 of the next K-tile
    u32x4 braw[8];          // bias (8 bf16 columns per lane per pair) of the next tile to start

    // ---- epilogue: stores from the tile origin, rows past M out of range through the record count,
    // columns past N dropped per lane ----
    auto st_rs = [&](void* base, int tm0, int tn0) -> u32x4 {
        if (!base) return w1_rsrc(nullptr, 0u);
        return w1_rsrc((char*)base + ((long)tm0 * p.ldc + tn0) * 2, clamp_u(((long)(p.M - tm0) * p.ldc - tn0) * 2));
    };
    const uint32_t st_lane = (uint32_t)(((64 * w + (lane & 15)) * p.ldc + 8 * G) * 2);
    auto st_off = [&](int i, int pp, int tn0) -> uint32_t {
        const uint32_t o = w1_opq(st_lane) + (uint32_t)((16 * i * w1_opq_s((int)p.ldc) + 32 * pp) * 2);
        return ((int)w1_opq((uint32_t)(8 * G)) < p.N - tn0 - 32 * pp) ? o : 0xFFFFFFF0u;
    };
    auto bias_issue = [&](bool live, int tn0) {
        // bias of the tile at column tn0 (8 × 16 B per lane, columns tn0 + 32p + 8G ..); zero records = zeros
        live = live && p.bias;
        const u32x4 rs = w1_rsrc(live ? (const void*)(p.bias + tn0) : nullptr, live ? clamp_u((long)(p.N - tn0) * 2) : 0u);
#pragma unroll
        for (int pp = 0; pp < 8; ++pp) w1_ld16(braw[pp], rs, w1_opq((uint32_t)(16 * G)) + (uint32_t)(64 * pp));
    };
    // C operand of the first K-tile's MFMAs of B fragment jj: the bias of its 4 columns
    // (MN-contiguous B: odd lane groups hold a pair's fragment 1 columns first — pk_frag_b's a(g))
    const bool swp = !BKC && (G & 1);
    auto cinit = [&](int jj) -> f32x4 {
        if constexpr (ALPHA) return (f32x4){0.f, 0.f, 0.f, 0.f};  // (host: no bias with alpha)
        const u32x4 u = braw[jj >> 1];
        const bool second = (jj & 1) != (int)swp;
        const uint32_t lo = second ? u.z : u.x, hi = second ? u.w : u.y;
        return (f32x4){__builtin_bit_cast(float, lo << 16), __builtin_bit_cast(float, lo & 0xFFFF0000u),
                       __builtin_bit_cast(float, hi << 16), __builtin_bit_cast(float, hi & 0xFFFF0000u)};
    };
    // pair pp of the pending tile: bf16 rows (acc read before this block's MFMAs overwrite it).  In the
    // loop the reads are asm v_accvgpr_read with an AGPR operand: plain reads let the allocator move
    // accumulators into arch VGPRs (MFMA's either-file operand class) and spill; the asm form keeps
    // every accumulator in the AGPR file and copies on use.  (No hazard padding: the pending tile's
    // last MFMA on these registers was a full K-tile ago.)
    auto epi_convert = [&](int pp, u32x4* o, bool in_loop) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float v[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                if (in_loop) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v[c]) : "a"(acc[i][2 * pp + (c >> 2)][c & 3]));
                else v[c] = acc[i][2 * pp + (c >> 2)][c & 3];
                if constexpr (ALPHA) v[c] *= alpha;
            }
            o[i] = (u32x4){pk_pack2(v[0], v[1]), pk_pack2(v[2], v[3]), pk_pack2(v[4], v[5]), pk_pack2(v[6], v[7])};
            if constexpr (!BKC) {
                const u32x4 t = o[i];
                o[i] = swp ? (u32x4){t.z, t.w, t.x, t.y} : t;
            }
        }
    };
    // ---- residual (RES): the MFMAs add it.  For output pair pp the lane's 16-B residual chunk (row
    // 16i + (lane&15), columns 32pp + 8G ..; the chunk the lane stores) is the A-side operand of a bf16
    // 16x16x32 MFMA whose k runs over the pair's 32 columns, and the B side is a one-hot "permutation"
    // operand Pid[h]: output row n of fragment 2pp + h takes k = 8(n>>2) + 4h + (n&3) — the column the
    // permuted fragment put there — so acc[i][2pp+h] += r exactly (products r·1, fp32 sums with zeros).
    // Residual body q (K-tiles 1-4 of a tile) issues pairs 2q, 2q + 1 (8 × 16 B per lane) at its start,
    // its end-of-K-tile wait retires them (≈ 13 blocks of MFMAs later) and blocks 14-15 run the 16 extra
    // MFMAs: 4 % more MFMA work per tile, no epilogue VALU, 32 + 8 registers.  Rows past M / columns past
    // N load zeros. ----
    [[maybe_unused]] s16x8 pid[2];
    [[maybe_unused]] u32x4 rres[8];
    if constexpr (RES) {
        const int ni = lane & 15;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
            for (int c = 0; c < 8; ++c) pid[h][c] = (G == (ni >> 2) && c == 4 * h + (ni & 3)) ? (short)0x3F80 : (short)0;
            asm volatile("" : "+v"(pid[h]));
        }
    }
    auto res_issue = [&](int q) {  // pairs 2q, 2q + 1 of the current tile (m0, n0)
        const u32x4 rs = w1_rsrc(p.res + ((long)m0 * p.ldc + n0), clamp_u(((long)(p.M - m0) * p.ldc - n0) * 2));
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int i = 0; i < 4; ++i) w1_ld16(rres[e * 4 + i], rs, st_off(i, 2 * q + e, n0));
    };
    auto res_mma = [&](int q, int e) {  // pair 2q + e (its loads retired)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int jj = 2 * (2 * q + e) + h;
                acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pid[h], __builtin_bit_cast(s16x8, rres[e * 4 + i]),
                                                                     acc[i][jj], 0, 0, 0);
            }
    };
    auto epi_store = [&](const u32x4* o, int pp, const u32x4& crs, int tn0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) pk_st16(o[i], crs, (DBG & 1) ? 0xFFFFFFF0u : st_off(i, pp, tn0));
    };

    // ---- K-tile bodies.  Three straight-line bodies, no branch inside (a uniform branch per block made
    // hipcc sink every MFMA below the block's reads and DMA): EPI = a tile's first K-tile (bias as the
    // MFMAs' C operand) with the previous tile's epilogue interleaved (the block's first tile "stores"
    // zero-initialised accumulators through a zero-record descriptor: no traffic, same counts), STEADY,
    // LAST (issues the next tile's bias).  The end-of-K-tile waits are the counts of each body's own
    // ops plus, where a K-tile follows an EPI, nothing more: the EPI's late stores are simply waited
    // for a K-tile later (conservative, branch-free).  Ring slots: A t % 2, B t % 3. ----
    int aslot = 0, bslot = 0;
    auto ktile = [&](auto kc, int kt) {
        constexpr int KIND = decltype(kc)::value;
        constexpr bool K0 = KIND == W1_EPI;
        constexpr int RQ = KIND >= W1_RES0 ? KIND - W1_RES0 : -1;  // residual body q (or -1)
        [[maybe_unused]] u32x4 crs = {0u, 0u, 0u, 0u};
        if constexpr (K0) crs = st_rs(pm_live ? p.C : nullptr, pm0, pn0);
        if constexpr (KIND == W1_LAST) bias_issue(has1, n1);
        if constexpr (RQ >= 0) res_issue(RQ);
        if constexpr (K0) w1_pin8<16>(braw);  // this tile's bias (issued a K-tile ago; 16 DMA younger)
        constexpr int NW = w1_before_wait(KIND);
        const int an = aslot ^ 1, bn = bslot == 2 ? 0 : bslot + 1;
        const int bd = bslot == 0 ? 2 : bslot - 1;  // B slot of K-tile t + 2 (= t - 1's)
        const u32x4 rsA = dma_rs(true, kt + 2), rsB = dma_rs(false, kt + 2);
        const int ncB = BKC ? 0 : b_ncols(kt + 2);
        [[maybe_unused]] u32x4 pend[4];
        W1Frag Bf[16], An[4];
        Bf[0] = Bq[0];
        Bf[1] = Bq[1];
        Bf[2] = Bq[2];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            __builtin_amdgcn_sched_barrier(0);
            if (j == W1_WAIT_J) {
                // K-tile t + 1 staged (own DMA), every wave done reading B(t): barrier, then its first
                // fragments under blocks 13-15
                vm_wait<NW>();
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                if constexpr (RQ >= 0) w1_touch8(rres);  // this body's residual loads retired
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (RQ >= 0) {
                if (j == 14) res_mma(RQ, 0);
                if (j == 15) res_mma(RQ, 1);
            }
            // next K-tile's fragments spread over blocks 13-15 (lgkmcnt counts stay below 16)
            if (j == 13) {
                An[0] = rd_a(an, 0);
                An[1] = rd_a(an, 1);
                Bq[0] = rd_b(bn, 0);
            }
            if (j == 14) {
                An[2] = rd_a(an, 2);
                An[3] = rd_a(an, 3);
                Bq[1] = rd_b(bn, 1);
            }
            if (j == 15) Bq[2] = rd_b(bn, 2);
            if constexpr (K0) {
                if ((j & 1) == 0) epi_convert(j >> 1, pend, true);
                else epi_store(pend, j >> 1, crs, pn0);
            }
            if (j >= 1 && j <= 8) {
                const bool isA = j <= 4;
                const int i0 = ((j - 1) & 3) * 2;
                dma_one(isA ? rsA : rsB, isA, isA ? aslot : bd, i0, ncB);
                dma_one(isA ? rsA : rsB, isA, isA ? aslot : bd, i0 + 1, ncB);
            }
            if (j + 3 < 16) Bf[j + 3] = rd_b(bslot, j + 3);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i][j] = w1_mma<FP8>(Bf[j], Acur[i], K0 ? cinit(j) : acc[i][j], eb, ea);
        }
        __builtin_amdgcn_sched_barrier(0);
        // every accumulator lives in the AGPR file across the loops: without this the allocator gives
        // some loop-carried accumulators arch VGPRs and copies each MFMA result out (hazard nops)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 16; ++j) asm volatile("" : "+a"(acc[i][j]));
        if constexpr (KIND == W1_LAST) w1_pin8<16>(braw);  // the next tile's bias (16 DMA younger)
#pragma unroll
        for (int i = 0; i < 4; ++i) Acur[i] = An[i];
        aslot = an;
        bslot = bn;
    };
    using KEpi = std::integral_constant<int, W1_EPI>;
    using KSteady = std::integral_constant<int, W1_STEADY>;
    using KLast = std::integral_constant<int, W1_LAST>;

    // ---- prologue: bias of tile 0, its K-tiles 0 and 1 in flight, K-tile 0's first fragments ----
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    bias_issue(true, n0);
#pragma unroll
    for (int d = 0; d < 2; ++d) {
        const u32x4 rsA = dma_rs(true, d), rsB = dma_rs(false, d);
        const int ncB = BKC ? 0 : b_ncols(d);
#pragma unroll
        for (int i = 0; i < 8; ++i) dma_one(rsA, true, d, i, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) dma_one(rsB, false, d, i, ncB);
    }
    vm_wait<16>();  // K-tile 0 (own DMA) landed
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i) Acur[i] = rd_a(0, i);
    Bq[0] = rd_b(0, 0);
    Bq[1] = rd_b(0, 1);
    Bq[2] = rd_b(0, 2);

#pragma unroll 1
    for (int s = 0; s < n_items; ++s) {
        if (s > 0) {  // a new tile: the finished one's epilogue runs under its first K-tile
            pm0 = m0;
            pn0 = n0;
            m0 = m1;
            n0 = n1;
            set_next(s + 1);
        }
        pm_live = s > 0;
        ktile(KEpi{}, 0);
        int kt1 = 1;
        if constexpr (RES) {  // K-tiles 1-4 (host: nk >= 6)
            ktile(std::integral_constant<int, W1_RES0>{}, 1);
            ktile(std::integral_constant<int, W1_RES0 + 1>{}, 2);
            ktile(std::integral_constant<int, W1_RES0 + 2>{}, 3);
            ktile(std::integral_constant<int, W1_RES0 + 3>{}, 4);
            kt1 = 5;
        }
#pragma unroll 1
        for (int kt = kt1; kt < nk - 1; ++kt) ktile(KSteady{}, kt);
        ktile(KLast{}, nk - 1);
    }
    // ---- the last tile's epilogue (exposed; asm accumulator reads as in the loop, after enough wait
    // states for the last MFMAs' results: 4 × s_nop 7 > the longest MFMA write latency) ----
    {
        const u32x4 crs = st_rs(p.C, m0, n0);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
        for (int pp = 0; pp < 8; ++pp) {
            __builtin_amdgcn_sched_barrier(0);
            u32x4 o[4];
            epi_convert(pp, o, true);
            epi_store(o, pp, crs, n0);
        }
    }
}

// host: persistent grid of min(tiles, CUs) workgroups, 160 KiB LDS each
template <int FP8, int ACT, bool ALPHA, bool BKC, int DBG = 0, bool RES = false>
void launch_w1_t(GemmArgs& a, hipStream_t st) {
    auto kern = gemm_w1<FP8, ACT, ALPHA, BKC, DBG, RES>;
    static int attr_dev = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (attr_dev != dev) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, W1_LDS);
        attr_dev = dev;
    }
    static int cu_dev = -1, cu_n = 256;
    if (cu_dev != dev) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cu_n = prop.multiProcessorCount;
        cu_dev = dev;
    }
    const int tiles = a.tiles_m * a.tiles_n;
    const int grid = tiles < cu_n ? tiles : cu_n;
    kern<<<grid, 256, W1_LDS, st>>>(a);
}

}  // namespace rn_gemm_detail
