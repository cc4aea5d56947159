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

// W1_POST: the STEADY body right after an EPI; W1_RES0 + q, q = 0..3: residual bodies (RES0 follows the EPI)
enum { W1_EPI = 1, W1_STEADY = 2, W1_LAST = 3, W1_POST = 4, W1_RES0 = 5 };

// VMEM ops a K-tile issues before its end-of-K-tile wait (block 13): the wait for K-tile t + 1 (whose
// DMA went out in K-tile t - 1's blocks 1-8) leaves exactly these in flight.  Ops of K-tile t - 1
// issued after its DMA (an EPI's stores of blocks 9-15) are waited for too: conservative, no branch.
// The body after an EPI (POST / RES0) also leaves the EPI's 16 stores issued after its last DMA (blocks
// 9-15) in flight: they get until the next K-tile's wait.  (A residual body's 8 loads go out at its
// start, before its DMA: outside the allowance, so its own wait retires them.)
// With a residual, LAST also issues the next tile's residual cache prefetch (4 loads) after its DMA (the
// prologue: tile 0's): in flight at its own wait and at the EPI's, retired by RES0's.  RES0 gets no
// store allowance: its residual loads are younger than the EPI's DMA it waits for, so anything but its
// own DMA must retire there.  Every allowance is exact or short (never counts an op that was not
// issued: that would let the wait pass before the DMA it guards landed).
// spp: epilogue stores per output pair (4 × 16 B; 8 × 8 B for the fp8 MN-contiguous-B layout).  Counts
// past vmcnt's 63 are clamped (a short allowance only waits longer).
constexpr int w1_before_wait(int kind, bool res, int spp) {
    const int n = (kind == W1_LAST ? 8 : 0) + 16 + (kind == W1_EPI ? 6 * spp : 0) + (kind == W1_POST ? 4 * spp : 0) +
                  ((res && (kind == W1_LAST || kind == W1_EPI)) ? 4 : 0);
    return n > 63 ? 63 : n;
}
// names 8 registers as redefined here, after the wait that retired their loads (no consumer above it)
RN_DEV void w1_touch8(u32x4* v) {
    asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]));
}
static_assert(w1_before_wait(W1_EPI, true, 4) <= 63, "vmcnt range");

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

// FP8: 1 = e4m3 × e4m3, 2 = A (src1) e5m2 (a gradient) × B e4m3
template <int FP8>
RN_DEV f32x4 w1_mma(const W1Frag& b, const W1Frag& a, f32x4 c, int eb, int ea) {
    if constexpr (FP8) {
        return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(pk_cat8(b.lo, b.hi), pk_cat8(a.lo, a.hi), c, 0,
                                                                FP8 == 2 ? 1 : 0, 0, eb, 0, ea);
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

// fp8 MN-contiguous A image (64-B rows): row r's 16-B chunk c at c ^ swz_a8(r) — the 16 rows a 32-lane
// half of a transposing read covers (16g + 8t + q, g = 2h, 2h + 1) land on 16 distinct 16-B bank groups
RN_DEV int w1_swz_a8(int r) { return ((r >> 2) & 1) | (((r >> 4) & 1) << 1); }

// E8M0 exponent of a power-of-two scale (its biased float exponent); 127 = 1.0
RN_DEV int w1_e8m0(const float* s) {
    if (!s) return 127;
    const uint32_t u = __builtin_bit_cast(uint32_t, *s);
    return (int)((u >> 23) & 0xFF);
}

// DBG (timing ablations, REPLICANN_W1_DBG; outputs wrong except with bit 2 alone): bit 0 issues the
// epilogue stores out of range (same instructions, no traffic), bit 1 the operand DMA (no HBM/L2 traffic;
// the LDS is still written), bit 2 makes the epilogue stores non-temporal, bit 3 points every tile's
// operand DMA at tile (0, 0)'s rows (same traffic, all L2 hits after the first touch)
// RES: + residual (x·Wᵀ + b + r; p.res, row stride p.ldc) added by MFMA — see the residual bodies below.
// AKC false: A MN-contiguous too (fp8 only: the weight gradient dYᵀ·X, both operands read as stored);
// SPLIT: split-K items writing fp32 slabs (p.ws, slab s at ws + s·M·N, row stride N; p.split slabs of
// p.k_per_split K-tiles each, host: an exact division), summed by splitk_reduce_k
template <int FP8, int ACT, bool ALPHA, bool BKC, int DBG = 0, bool RES = false, bool AKC = true, bool SPLIT = false>
__global__ void __launch_bounds__(256, 1) gemm_w1(GemmArgs p) {
    static_assert(AKC || (FP8 && !BKC && SPLIT), "w1 MN-contiguous A: the fp8 weight gradient (split-K slabs)");
    static_assert(!RES || (BKC && !ALPHA), "w1 residual: x·Wᵀ layout, no alpha");
    static_assert(ACT == ACT_NONE, "w1: forward epilogues without activation (activations: cfg 9)");
    // fp8: the power-of-two tensor scales ride the MFMA; ALPHA (fp8 MN-contiguous B only: the fp8 LM head's data
    // gradient) multiplies in one more device scalar (the loss gradient's g / n)
    static_assert(!(FP8 && ALPHA) || !BKC, "fp8 alpha: MN-contiguous B only");
    // fp8 with an MN-contiguous B (the data gradient dY·W, W read as stored): transposing tr_b8 fragment
    // reads in plain column order, so a lane holds two 4-column runs per output pair (8-B stores)
    constexpr bool F8MN = FP8 && !BKC;
    static_assert(!F8MN || (!RES && !(ALPHA && SPLIT)), "w1 fp8 MN-contiguous B: plain / alpha epilogue");
    constexpr int SPP = F8MN ? 8 : 4;  // epilogue stores per output pair
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int G = lane >> 4;
    const int tiles = p.tiles_m * p.tiles_n;
    const int grid = gridDim.x;
    const int bid = xcd_remap(blockIdx.x, grid);
    // 128-byte K-tiles per item (host: >= 2); SPLIT: items = tiles × p.split, item i = split i / tiles
    const int nk = SPLIT ? p.k_per_split : (p.K >> 7);
    const int n_items = ((SPLIT ? tiles * p.split : tiles) - bid + grid - 1) / grid;
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
    // (SPLIT: k0 = the item's first K-tile; sd = its slab)
    auto item_mn = [&](int s, int& m0, int& n0, int& kt0, int& sd) {
        int tm, tn;
        int it = bid + s * grid;
        sd = 0;
        if constexpr (SPLIT) {
            sd = it / tiles;
            it -= sd * tiles;
        }
        if (!SPLIT && band_ok(grid, p.tiles_m, p.tiles_n))
            band_tile(it, grid, p.tiles_m, p.tiles_n, p.group_m > 0 ? p.group_m : GROUP_M, tm, tn);
        else group_tile_g(it, p.tiles_m, p.tiles_n, p.group_m > 0 ? p.group_m : GROUP_M, tm, tn);
        m0 = tm * 256;
        n0 = tn * 256;
        kt0 = sd * nk;
    };
    int m0 = 0, n0 = 0, m1 = 0, n1 = 0, pm0 = 0, pn0 = 0;
    [[maybe_unused]] int ik0 = 0, ik1 = 0, sd0 = 0, sd1 = 0, psd = 0;
    bool has1 = false, pm_live = false;
    item_mn(0, m0, n0, ik0, sd0);
    auto set_next = [&](int s) {
        has1 = s < n_items;
        if (has1) item_mn(s, m1, n1, ik1, sd1);
    };
    set_next(1);

    // per-lane DMA source offsets: rows 64w + 8i + (lane>>3) of the stage, 16-B chunk (lane&7) ^ swizzle
    // (A: swz_kc, B: swz_kcp; both depend on i only through i & 1 / i & 3)
    const int dr = 64 * w + (lane >> 3);
    uint32_t a_off[2], b_off[4];
    [[maybe_unused]] int b_col[2];
    [[maybe_unused]] int a_col[2];
    if constexpr (AKC) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int r = dr + 8 * q;
            a_off[q] = (uint32_t)((long)r * lda + (((lane & 7) ^ swz_kc(r)) << 4));
        }
    } else {
        // fp8 MN-contiguous A, wave-private image [128 k rows][64 mn bytes] (the wave's 64 output rows):
        // instruction i stages k rows 16i + (lane>>2), 16-B chunk (lane&3) ^ swz_a8(row); the swizzle
        // depends on i only through i & 1
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int r = 16 * q + (lane >> 2);
            a_col[q] = 64 * w + (((lane & 3) ^ w1_swz_a8(r)) << 4);
            a_off[q] = (uint32_t)((long)r * lda + a_col[q]);
        }
    }
    if constexpr (BKC) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r = dr + 8 * q;
            b_off[q] = (uint32_t)((long)r * ldb + (((lane & 7) ^ swz_kcp(r)) << 4));
        }
    } else if constexpr (F8MN) {
        // fp8 MN image ([128 k rows][128 mn bytes] × 2 sub-images, chunk c of row r at c ^ swz_f8(r)): wave w
        // stages sub-image w >> 1, rows 64(w & 1) + 8i + (lane>>3); instruction i = 4a + 2q + b adds
        // (32a + 8b) rows to lane offset q (the swizzle depends on i only through q)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int r = 64 * (w & 1) + 16 * q + (lane >> 3);
            b_col[q] = 128 * (w >> 1) + (((lane & 7) ^ swz_f8(r)) << 4);
            b_off[q] = (uint32_t)((long)r * ldb + b_col[q]);
        }
        b_off[2] = b_off[3] = 0u;
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
        const int dd = (nxt ? d - nk : d) + (SPLIT ? (nxt ? ik1 : ik0) : 0);  // K-tile within the whole K
        const bool live = !nxt || has1;
        const int r0 = (DBG & 8) ? 0 : (isA ? (nxt ? m1 : m0) : (nxt ? n1 : n0));
        const long ld = isA ? lda : ldb;
        if (!AKC && isA) {  // fp8 MN A: k rows 128dd.., columns (bytes) from r0; M tail per lane
            const char* base = (const char*)p.A + (long)(128 * dd) * ld + (long)r0;
            const long n = live ? (long)(p.K - 128 * dd) * ld - (long)r0 : 0;
            return w1_rsrc(base, clamp_u(n));
        }
        if (F8MN && !isA) {  // K-tile dd = k rows 128dd..128dd+127 (bytes), columns (bytes) from r0
            const char* base = (const char*)p.B + (long)(128 * dd) * ld + (long)r0;
            const long n = live ? (long)(p.K - 128 * dd) * ld - (long)r0 : 0;
            return w1_rsrc(base, clamp_u(n));
        }
        if (!BKC && !isA) {  // K-tile dd = k rows 64dd..64dd+63 (bf16), columns from r0; N tail per lane
            const char* base = (const char*)p.B + (long)(64 * dd) * ld + (long)r0 * 2;
            const long n = live ? (long)((p.K >> 1) - 64 * dd) * ld - (long)r0 * 2 : 0;
            return w1_rsrc(base, clamp_u(n));
        }
        const char* base = (const char*)(isA ? p.A : p.B) + (long)r0 * ld + dd * 128;
        const long n = live ? (long)((isA ? p.M : p.N) - r0) * ld - dd * 128 : 0;
        return w1_rsrc(base, clamp_u(n));
    };
    // columns of the tile K-tile d belongs to that exist (MN-contiguous B: the per-lane N-tail check;
    // MN-contiguous A: rows)
    auto b_ncols = [&](int d) -> int { return p.N - (d >= nk ? n1 : n0); };
    auto a_nrows = [&](int d) -> int { return p.M - (d >= nk ? m1 : m0); };
    auto dma_one = [&](const u32x4& rs, bool isA, int slot, int i, int ncols) {
        uint32_t off;
        if (isA && !AKC) {
            off = w1_opq(a_off[i & 1]) + (uint32_t)(16 * (i & ~1) * w1_opq_s((int)lda));
            off = (int)w1_opq((uint32_t)a_col[i & 1]) < ncols ? off : 0xFFFFFFF0u;
        } else if (isA) off = w1_opq(a_off[i & 1]) + (uint32_t)((i & ~1) * 8 * w1_opq_s((int)lda));
        else if constexpr (BKC) off = w1_opq(b_off[i & 3]) + (uint32_t)((i & ~3) * 8 * w1_opq_s((int)ldb));
        else if constexpr (F8MN) {
            off = w1_opq(b_off[(i >> 1) & 1]) + (uint32_t)((32 * (i >> 2) + 8 * (i & 1)) * w1_opq_s((int)ldb));
            off = (int)w1_opq((uint32_t)b_col[(i >> 1) & 1]) < ncols ? off : 0xFFFFFFF0u;
        } else {
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
    // fp8 MN (pk_frag8_mn): fragment jj = columns 32(jj>>1) + 16(jj&1) .. +15 = 16-B column chunk jj & 7 of
    // sub-image jj >> 3; row 64s + 16G + 8t + q (q = (lane&15)>>1) of the image, its swizzle independent of
    // s and t: one lane offset per chunk
    [[maybe_unused]] uint32_t b_f8[8];
    if constexpr (F8MN) {
        const int q = (lane & 15) >> 1;
        const int sw = ((q >> 1) & 3) | ((G & 1) << 2);  // swz_f8(16G + 8t + q)
#pragma unroll
        for (int c = 0; c < 8; ++c) b_f8[c] = (uint32_t)((16 * G + q) * 128 + ((c ^ sw) << 4) + 8 * (lane & 1));
    } else if constexpr (!BKC) {
        const int k0 = 8 * G + (bi >> 2), pl = bi & 3;
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                b_mn[e][h] = (uint32_t)(k0 * 128 + (((4 * e + pl) ^ swz_mnp(k0)) << 4) + ((h ^ (pl & 1)) << 3));
    }
    // fp8 MN A (the wave's [128][64 B] image): fragment i = 16-B column chunk i; rows 64s + 16G + 8t + q
    // (q = (lane&15)>>1), swizzle independent of s and t: one lane offset per fragment
    [[maybe_unused]] uint32_t a_f8[4];
    if constexpr (!AKC) {
        const int q = (lane & 15) >> 1;
        const int sw = ((q >> 2) & 1) | ((G & 1) << 1);  // w1_swz_a8(16G + 8t + q)
#pragma unroll
        for (int c = 0; c < 4; ++c) a_f8[c] = (uint32_t)(w * 8192 + (16 * G + q) * 64 + ((c ^ sw) << 4) + 8 * (lane & 1));
    }
    auto rd_a = [&](int slot, int i) -> W1Frag {
        if constexpr (!AKC) {
            typedef int i32x2v __attribute__((ext_vector_type(2)));
            typedef __attribute__((address_space(3))) i32x2v lds8;
            const char* base = smem + W1_A0 + slot * W1_STAGE + w1_opq(a_f8[i]);
            i32x2v v[4];
#pragma unroll
            for (int t = 0; t < 4; ++t)  // (k-step t >> 1: rows + 64; t & 1: rows + 8)
                v[t] = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds8*)(base + (t >> 1) * 4096 + (t & 1) * 512));
            return {__builtin_bit_cast(s16x8, (i32x4){v[0][0], v[0][1], v[1][0], v[1][1]}),
                    __builtin_bit_cast(s16x8, (i32x4){v[2][0], v[2][1], v[3][0], v[3][1]})};
        }
        const char* base = smem + W1_A0 + slot * W1_STAGE + i * 2048;
        return {*reinterpret_cast<const s16x8*>(base + a_lo), *reinterpret_cast<const s16x8*>(base + a_hi)};
    };
    auto rd_b = [&](int slot, int jj) -> W1Frag {
        if constexpr (F8MN) {
            typedef int i32x2v __attribute__((ext_vector_type(2)));
            typedef __attribute__((address_space(3))) i32x2v lds8;
            const char* base = smem + W1_B0 + slot * W1_STAGE + (jj >> 3) * 16384 + w1_opq(b_f8[jj & 7]);
            i32x2v v[4];
#pragma unroll
            for (int t = 0; t < 4; ++t)  // (k-step t >> 1: rows + 64; t & 1: rows + 8)
                v[t] = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds8*)(base + (t >> 1) * 8192 + (t & 1) * 1024));
            return {__builtin_bit_cast(s16x8, (i32x4){v[0][0], v[0][1], v[1][0], v[1][1]}),
                    __builtin_bit_cast(s16x8, (i32x4){v[2][0], v[2][1], v[3][0], v[3][1]})};
        } else if constexpr (!BKC) {
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
    // (SPLIT: the item's fp32 slab sd, row stride N)
    auto st_rs = [&](void* base, int tm0, int tn0, int sd) -> u32x4 {
        if (!base) return w1_rsrc(nullptr, 0u);
        if constexpr (SPLIT) {
            const long MN = (long)p.M * p.N;
            return w1_rsrc((char*)p.ws + (sd * MN + (long)tm0 * p.N + tn0) * 4, clamp_u(((long)(p.M - tm0) * p.N - tn0) * 4));
        }
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
    const bool swp = !BKC && !FP8 && (G & 1);
    auto cinit = [&](int jj) -> f32x4 {
        if constexpr (ALPHA || F8MN) return (f32x4){0.f, 0.f, 0.f, 0.f};  // (host: no bias with alpha / fp8 MN)
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
    // (SPLIT: the raw fp32 accumulators, o[2i + h] = fragment 2pp + h of A fragment i)
    auto epi_convert = [&](int pp, u32x4* o, bool in_loop) {
        if constexpr (SPLIT) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        float v;
                        if (in_loop) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(acc[i][2 * pp + h][c]));
                        else v = acc[i][2 * pp + h][c];
                        o[2 * i + h][c] = __builtin_bit_cast(uint32_t, v);
                    }
            return;
        }
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
            if constexpr (!BKC && !FP8) {
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
    // the NEXT tile's residual pulled into the L2 / Infinity Cache while this tile computes (one dword per
    // 128-B line: wave w rows 64w + lane, 4 lines each), so the residual bodies' loads hit a cache.  All 4
    // loads target ONE register (returns retire in order; the value is never read), named until the wait
    // that retires them (a late write into a register the allocator had reused would corrupt it)
    [[maybe_unused]] uint32_t pfr = 0u;
    auto res_prefetch = [&](bool live, int tm0, int tn0) {
        const u32x4 rs = w1_rsrc(live ? (const void*)(p.res + ((long)tm0 * p.ldc + tn0)) : nullptr,
                                 live ? clamp_u(((long)(p.M - tm0) * p.ldc - tn0) * 2) : 0u);
        const uint32_t row = w1_opq((uint32_t)((64 * w + lane) * p.ldc * 2));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t off = 64 * c < p.N - tn0 ? row + 128u * c : 0xFFFFFFF0u;
            asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "+v"(pfr) : "v"(off), "s"(rs) : "memory");
        }
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
    // fp8 MN: the lane's columns of pair pp are 32pp + 4G .. +3 (fragment 2pp) and 32pp + 16 + 4G .. +3
    const uint32_t st_lane8 = (uint32_t)(((64 * w + (lane & 15)) * p.ldc + 4 * G) * 2);
    auto st_off8 = [&](int i, int pp, int h, int tn0) -> uint32_t {
        const uint32_t o = w1_opq(st_lane8) + (uint32_t)((16 * i * w1_opq_s((int)p.ldc) + 32 * pp + 16 * h) * 2);
        return ((int)w1_opq((uint32_t)(4 * G)) < p.N - tn0 - 32 * pp - 16 * h) ? o : 0xFFFFFFF0u;
    };
    // SPLIT: fp32, the same 4-column runs, row stride N
    const uint32_t st_lane32 = (uint32_t)(((64 * w + (lane & 15)) * p.N + 4 * G) * 4);
    auto st_off32 = [&](int i, int pp, int h, int tn0) -> uint32_t {
        const uint32_t o = w1_opq(st_lane32) + (uint32_t)((16 * i * w1_opq_s(p.N) + 32 * pp + 16 * h) * 4);
        return ((int)w1_opq((uint32_t)(4 * G)) < p.N - tn0 - 32 * pp - 16 * h) ? o : 0xFFFFFFF0u;
    };
    auto epi_store = [&](const u32x4* o, int pp, const u32x4& crs, int tn0) {
        if constexpr (SPLIT) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) pk_st16(o[2 * i + h], crs, (DBG & 1) ? 0xFFFFFFF0u : st_off32(i, pp, h, tn0));
            return;
        }
        if constexpr (F8MN) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                pk_st8((u32x2v){o[i].x, o[i].y}, crs, (DBG & 1) ? 0xFFFFFFF0u : st_off8(i, pp, 0, tn0));
                pk_st8((u32x2v){o[i].z, o[i].w}, crs, (DBG & 1) ? 0xFFFFFFF0u : st_off8(i, pp, 1, tn0));
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr ((DBG & 4) != 0) pk_st16_nt(o[i], crs, (DBG & 1) ? 0xFFFFFFF0u : st_off(i, pp, tn0));
            else pk_st16(o[i], crs, (DBG & 1) ? 0xFFFFFFF0u : st_off(i, pp, tn0));
        }
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
        if constexpr (K0) crs = st_rs(pm_live ? p.C : nullptr, pm0, pn0, psd);
        if constexpr (KIND == W1_LAST) bias_issue(has1, n1);
        if constexpr (RQ >= 0) res_issue(RQ);
        if constexpr (K0) w1_pin8<16>(braw);  // this tile's bias (issued a K-tile ago; 16 DMA younger)
        constexpr int NW = w1_before_wait(KIND, RES, SPP);
        const int an = aslot ^ 1, bn = bslot == 2 ? 0 : bslot + 1;
        const int bd = bslot == 0 ? 2 : bslot - 1;  // B slot of K-tile t + 2 (= t - 1's)
        const u32x4 rsA = dma_rs(true, kt + 2), rsB = dma_rs(false, kt + 2);
        const int ncB = BKC ? 0 : b_ncols(kt + 2);
        const int ncA = AKC ? 0 : a_nrows(kt + 2);
        [[maybe_unused]] u32x4 pend[SPLIT ? 8 : 4];
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
                if constexpr (RQ == 0) asm volatile("" : "+v"(pfr));  // the prefetch issued in LAST retired
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (RES && KIND == W1_LAST) {
                if (j == 9) res_prefetch(has1, m1, n1);  // after this body's DMA (blocks 1-8)
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
                dma_one(isA ? rsA : rsB, isA, isA ? aslot : bd, i0, isA ? ncA : ncB);
                dma_one(isA ? rsA : rsB, isA, isA ? aslot : bd, i0 + 1, isA ? ncA : ncB);
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
        const int ncA = AKC ? 0 : a_nrows(d);
#pragma unroll
        for (int i = 0; i < 8; ++i) dma_one(rsA, true, d, i, ncA);
#pragma unroll
        for (int i = 0; i < 8; ++i) dma_one(rsB, false, d, i, ncB);
    }
    if constexpr (RES) {
        res_prefetch(true, m0, n0);  // (counted in the first EPI's wait, as LAST's is)
        vm_wait<20>();               // K-tile 0 (own DMA) landed
    } else {
        vm_wait<16>();  // K-tile 0 (own DMA) landed
    }
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
            psd = sd0;
            m0 = m1;
            n0 = n1;
            ik0 = ik1;
            sd0 = sd1;
            set_next(s + 1);
        }
        pm_live = s > 0;
        ktile(KEpi{}, 0);
        int kt1 = 1;
        if constexpr (!RES) {
            if (nk >= 3) {
                ktile(std::integral_constant<int, W1_POST>{}, 1);
                kt1 = 2;
            }
        }
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
        const u32x4 crs = st_rs(p.C, m0, n0, sd0);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
        for (int pp = 0; pp < 8; ++pp) {
            __builtin_amdgcn_sched_barrier(0);
            u32x4 o[SPLIT ? 8 : 4];
            epi_convert(pp, o, true);
            epi_store(o, pp, crs, n0);
        }
    }
    // nothing in flight at exit (the zero-record DMA / prefetch of the nonexistent next tile included)
    vm_wait<0>();
    if constexpr (RES) asm volatile("" : "+v"(pfr));
}

// host: persistent grid of min(tiles, CUs) workgroups, 160 KiB LDS each
template <int FP8, int ACT, bool ALPHA, bool BKC, int DBG = 0, bool RES = false, bool AKC = true, bool SPLIT = false>
void launch_w1_t(GemmArgs& a, hipStream_t st) {
    auto kern = gemm_w1<FP8, ACT, ALPHA, BKC, DBG, RES, AKC, SPLIT>;
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
    const int items = a.tiles_m * a.tiles_n * (SPLIT ? a.split : 1);
    const int grid = items < cu_n ? items : cu_n;
    kern<<<grid, 256, W1_LDS, st>>>(a);
}

}  // namespace rn_gemm_detail
