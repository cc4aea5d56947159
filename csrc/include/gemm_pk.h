// Persistent 256×256 bf16 GEMM with a half-tile LDS-DMA stream and staggered wave groups
// (tile config 9; the default for every plain/fused GEMM whose shape it accepts).
//
// Why a second main loop (gemm_impl.h keeps the one-tile-per-block kernels for conv and fp8):
//   * the one-tile-per-block kernel pays a prologue (first DMA round trip from HBM) and an
//     epilogue (output stores) per 256² tile with the matrix cores idle: at K = 768 that was
//     ≈35 % of the GEMM (profiles/gemm_k_sweep_r1d.txt);
//   * its 2-stage ring (128 KiB of the 160 KiB LDS) leaves one K-tile of slack for a DMA and
//     drains it with a vmcnt(0) barrier per K-tile.
//
// Structure (MI355X guide §5 "256² 8-phase template", T1–T5, rebuilt for this framework's
// three operand layouts and fused epilogues):
//   * one workgroup per CU (512 threads = 8 waves, 128 KiB LDS), the grid walks the output
//     tiles (× split-K slices) persistently; block ids are remapped per XCD so the blocks of
//     one XCD work on contiguous tiles (shared A/B panels in that XCD's L2);
//   * operands stream through LDS as HALF-TILES of 16 KiB — A rows 0-127 ("At"), B columns
//     0-127 ("Bl"), B columns 128-255 ("Br"), A rows 128-255 ("Ab") of one 64-deep K-tile,
//     issued in that order, one half-tile per phase, 6 half-tiles ahead of the phase that
//     reads them, into an 8-slot ring.  The stream runs straight through tile boundaries, so
//     the next tile's operands are already in flight during an epilogue;
//   * a K-tile is 4 phases, one per 128×128 quadrant of the block tile (each wave owns a 64×32
//     piece of every quadrant: its 128×64 output is spread over both A halves and both B
//     halves): q0 = (At, Bl), q1 = (At, Br), q2 = (Ab, Br), q3 = (Ab, Bl).  Each phase:
//       vmcnt wait (counted: 3 half-tiles stay in flight) → issue one half-tile (2 LDS-DMA per
//       wave) → ds_read this phase's fragments → s_barrier → lgkmcnt(0) → 16 MFMAs → s_barrier;
//   * waves 4-7 run one barrier behind waves 0-3 (one extra s_barrier up front): on every SIMD
//     one wave's fragment reads and DMA issue overlap its partner's MFMAs (guide T3/T4 stagger);
//   * the DMA of a slot is issued ≥ 2 phases after its last read and read ≥ 1 phase after the
//     wait that retires it (the guide's RAW/WAR placement rules for a staggered pair);
//   * B fragments are loaded with a column permutation so that after the MFMAs each lane holds
//     8 CONTIGUOUS output columns of one row: the epilogue stores 16 B per lane straight from
//     the accumulators (no LDS staging, which would need the ring), through buffer stores whose
//     range check drops out-of-bounds lanes — every wave issues the same number of stores, so
//     the counted vmcnt waits after an epilogue stay exact;
//   * bias comes through the scalar cache (s_load, lgkmcnt) so a bias epilogue does not drain
//     the in-flight operand DMA; epilogues that read a full tile (residual, saved
//     pre-activation, accumulate target) do wait for it.
//
// Epilogue operand reads (residual, saved activation): the full-tile read at the end of an item
// waits behind a vmcnt(0) that also drains the next item's in-flight operand DMA (≈ 15-20 % of a
// K = 768 tile, profiles/gemm_epilogue_aux_r3k.txt).  An L2 prefetch of that tile during the
// item's last K-tiles (extra LDS-DMA into scratch LDS) changed nothing, holding the tile in
// registers ahead of time does not fit the 256-VGPR budget (it spills), and streaming it through
// the operand ring as two extra K-tiles (round 4) was slower on every such shape (fc2 + residual
// 269 → 312 us, fc1 act-backward dgrad 403 → 412 us: profiles/gemm_staged_ab_r4f.txt,
// gemm_staged_pmc_r4g.txt) and was removed.  Staggering the blocks' start so their epilogues do
// not coincide (all 256 CUs read / store their tiles in lock step) was no better either
// (profiles/gemm_stagger_ab_r4i.txt).
//
// Tile schedule (DYN instantiations; chosen per launch while the queue is enabled — by the data-
// parallel reducer whenever collectives can run beside the backward, rn_gemm_set_sched): the grid
// does not walk a
// static list (bid + s·grid) but DEQUEUES its work, so a workgroup that starts late — because an
// RCCL kernel on the comm stream held its CU when the GEMM launched — simply takes fewer tiles
// instead of delaying the whole GEMM by the collective's duration.
//   * the unit of work is one item (tile × split-K slice) of ≥ 5 K-tiles (shorter items — K per
//     slice < 320 — keep the static walk), so one dequeue (+ one retry) has 3.5 K-tiles to come
//     back before the DMA cursor needs the next item, and the cursor is never more than one item
//     ahead of the compute side;
//   * one queue per dispatch group (blockIdx & 7: the blocks that share an XCD and its L2) over
//     exactly the units the static walk would give that group in all but its last round, plus
//     one shared tail queue over the rest: the same L2 locality as the static walk, balanced at
//     the end;
//   * wave 0 issues ONE returning buffer atomic per K-tile, at q0 right after q0's wait and BEFORE
//     q0's DMA: lane 0 is in range only when a dequeue is wanted (at an item's first K-tile, or to
//     retry on the shared tail), otherwise every lane is out of range and the atomic is a no-op.
//     It is older than q0's DMA, so the next K-tile's q0 wait retires it (vmcnt is in order) and
//     in between (q1-q3) wave 0's waits allow exactly one more op than the other waves'.  The
//     value is consumed at the next q0, right before the next atomic redefines the register: it
//     is never live across a second definition, so the register allocator has no reason to copy
//     a register the hardware has not written yet.  The unit id goes to a 4-slot LDS ring past
//     the operand ring, read by every wave ≥ 1 phase later (the DMA placement rule);
//   * the counters (home 0-7, tail, exit; one 128-B line each) reset themselves: the last block
//     to finish zeroes them, so a slot is reusable by the next launch on the stream and graph
//     replays need no memset node.
// Outputs are bitwise identical to the static walk's (same per-tile K order and epilogue).
//
// LDS images (all written lane-linearly by the DMA, the XOR swizzle applied to the per-lane
// SOURCE address and again on the read, guide rule 21):
//   K-contiguous operand, A side: [128 rows][64 k] 128-B rows, chunk c of row r at c ^ swz_kc(r);
//   K-contiguous operand, B side: same image, swizzle swz_kcp (rows are read in the permuted
//     order; the swizzle keeps every ds_read_b128 lane group on 16 distinct 16-B slots);
//   MN-contiguous operand: two [64 k][64 mn] sub-images, read with ds_read_b64_tr_b16; the B
//     side uses swz_mnp, which is conflict-free for the permuted column blocks.
#pragma once
#include <type_traits>

#include "gemm_impl.h"

namespace rn_gemm_detail {

constexpr int PK_HALF = 16384;  // bytes per half-tile slot
constexpr int PK_RING = 8 * PK_HALF;   // operand ring
constexpr int PK_LDS = PK_RING + 64;   // + the dynamic schedule's unit-id ring (4 ints)
constexpr int PK_CTR_STRIDE = 32;      // ints between schedule counters (one 128-B line each)
constexpr int PK_SCHED_INTS = 10 * PK_CTR_STRIDE;

RN_DEV int swz_kcp(int r) { return (((r >> 3) & 3) << 1) | ((r >> 1) & 1); }
RN_DEV int swz_mnp(int k) { return ((k >> 1) & 1) | (((k >> 3) & 1) << 2); }

// One 16 KiB half-tile (128 mn × 64 k) into `lds`, 2 LDS-DMA instructions per wave.
// PERM: the B-side swizzles.  `live` false: out-of-range source for every lane (the DMA
// writes zeros and reads nothing) — keeps the per-wave instruction count uniform.
template <bool KC, bool PERM>
RN_DEV void pk_stage(const u32x4& rs, long ld, int mn_lim, int k_lim, char* lds, int wave, int lane, bool live) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ins = wave * 2 + i;
        uint32_t voff;
        if constexpr (KC) {
            const int r = ins * 8 + (lane >> 3);
            const int cg = (lane & 7) ^ (PERM ? swz_kcp(r) : swz_kc(r));
            const int k = cg * 8;
            const bool ok = live && (r < mn_lim) && (k < k_lim);
            voff = ok ? (uint32_t)(((long)r * ld + k) * 2) : 0xFFFFFFF0u;
        } else {
            const int sub = ins >> 3, within = ins & 7;
            const int r = within * 8 + (lane >> 3);
            const int cg = (lane & 7) ^ (PERM ? swz_mnp(r) : swz_mn(r));
            const int mn = sub * 64 + cg * 8;
            const bool ok = live && (r < k_lim) && (mn < mn_lim);
            voff = ok ? (uint32_t)(((long)r * ld + mn) * 2) : 0xFFFFFFF0u;
        }
        dma16(rs, voff, lds + ins * 1024);
    }
}

// fp8 MN-contiguous half-tile image (FP8 with !AK / !BKC: the weight gradient dW = dYᵀ·X reads both
// operands as stored, [k = token][mn]): [128 k rows][128 mn bytes], 16-B chunk c of row r at
// c ^ swz_f8(r).  Read with ds_read_b64_tr_b8 (gfx950 transposing LDS read: per 16-lane group, lane
// 2q+p supplies 8 bytes of row q, columns 8p..8p+7, and lane i receives column i of the 8 rows), so a
// lane gets 8 consecutive k of one mn column.  swz_f8 puts the same-parity rows a 32-lane half reads
// (rows 16g + 8t + q of groups g, g+1) on 8 distinct chunks: conflict-free.
RN_DEV int swz_f8(int r) { return ((r >> 1) & 3) | (((r >> 4) & 1) << 2); }

// fp8 MN fragment (k-step s ∈ {0, 1}: k = 64·s + 16·(lane>>4) + 0..15) of the 16 mn columns
// col0 .. col0 + 15 (col0 % 16 == 0), column col0 + (lane & 15) per lane: the same byte → k map as the
// K-contiguous fp8 fragment (chunks g and g + 4 of a 128-byte k row), so either layout pairs with
// either in one scaled MFMA.
RN_DEV s16x8 pk_frag8_mn(const char* lds, int col0, int s, int lane) {
    typedef int i32x2v __attribute__((ext_vector_type(2)));
    const int g = lane >> 4, ii = lane & 15, q = ii >> 1, pp = ii & 1;
    const int cb = col0 + 8 * pp;
    i32x2v v[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int row = s * 64 + 16 * g + 8 * t + q;
        const char* a = lds + row * 128 + (((cb >> 4) ^ swz_f8(row)) << 4) + (cb & 15);
        v[t] = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2v*)a);
    }
    const i32x4 w = {v[0][0], v[0][1], v[1][0], v[1][1]};
    return __builtin_bit_cast(s16x8, w);
}

// A fragment (k-step s) of rows mnbase + (lane & 15) of a half-tile image.
template <bool KC>
RN_DEV s16x8 pk_frag_a(const char* lds, int mnbase, int s, int lane) {
    return frag<KC>(lds, mnbase, s, lane);
}

// B fragment j (0/1) of the wave's 32 columns starting at colbase (multiple of 32) of a
// half-tile image, permuted: MFMA operand row i = lane & 15 holds column
//   colbase + 8·(i>>2) + 4·(j ^ a(i>>2)) + (i&3),   a(g) = 0 (KC image) or g & 1 (MN image),
// so output group G = lane>>4 ends up with columns colbase + 8G .. 8G+7 over j = 0, 1.
template <bool KC>
RN_DEV s16x8 pk_frag_b(const char* lds, int colbase, int j, int s, int lane) {
    if constexpr (KC) {
        const int i = lane & 15;
        const int row = colbase + 8 * (i >> 2) + 4 * j + (i & 3);
        const int chunk = s * 4 + (lane >> 4);
        return *reinterpret_cast<const s16x8*>(lds + row * 128 + ((chunk ^ swz_kcp(row)) << 4));
    } else {
        const char* sub = lds + (colbase >> 6) * 8192;
        const int cl = colbase & 63;
        const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
        const int c = (cl >> 3) + p;
        const int half = j ^ (p & 1);
        const int k0 = s * 32 + 8 * g + q;
        const int k1 = k0 + 4;
        const char* a0 = sub + k0 * 128 + ((c ^ swz_mnp(k0)) << 4) + half * 8;
        const char* a1 = sub + k1 * 128 + ((c ^ swz_mnp(k1)) << 4) + half * 8;
        s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
        s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
        s16x8 r;
        r[0] = v0[0]; r[1] = v0[1]; r[2] = v0[2]; r[3] = v0[3];
        r[4] = v1[0]; r[5] = v1[1]; r[6] = v1[2]; r[7] = v1[3];
        return r;
    }
}

RN_DEV __amdgpu_buffer_rsrc_t pk_rsrc(const void* base, uint32_t bytes) {
    const uint64_t bp = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}

RN_DEV u32x4 pk_rsrc_u(const void* base, uint32_t bytes) {
    const uint64_t bp = (uint64_t)base;
    u32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    r[2] = bytes;
    r[3] = 0x00020000u;
    return r;
}

// 16-B buffer store the compiler does not see: it then inserts no vmcnt waits of its own for
// the epilogue stores (its counts would ignore the in-flight operand DMA, and a WAR wait on the
// store data registers would drain it); s_nop 1 covers the store-data read hazard (guide §5.7).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#if defined(RN_PK_ST_NT)  // A/B builds (REPLICANN_EXTRA_DEFS): epilogue store cache policy
#define RN_PK_ST_POLICY "nt"
#elif defined(RN_PK_ST_SC)
#define RN_PK_ST_POLICY "sc0 sc1"
#else
#define RN_PK_ST_POLICY ""
#endif
RN_DEV void pk_st16(const u32x4 v, const u32x4& rs, uint32_t voff) {
    asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen " RN_PK_ST_POLICY "\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs) : "memory");
}
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
RN_DEV void pk_st8(const u32x2v v, const u32x4& rs, uint32_t voff) {
    asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs) : "memory");
}
RN_DEV void pk_st16_nt(const u32x4 v, const u32x4& rs, uint32_t voff) {
    asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen nt\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs) : "memory");
}
#pragma clang diagnostic pop

RN_DEV uint32_t pk_pack2(float a, float b) {
    bf16x2 v = {(bf16)a, (bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}
// bf16 pairs -> f32 by shifts (exact).  NOTE: __builtin_bit_cast(bf16x2, u[d]) on an element of
// a vector reference miscompiles on ROCm 7.2 (every d reads element 0).
RN_DEV void pk_unpack8(const u32x4 u, float* f) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        f[2 * d] = __builtin_bit_cast(float, w[d] << 16);
        f[2 * d + 1] = __builtin_bit_cast(float, w[d] & 0xFFFF0000u);
    }
}

// Stores each wave issues per epilogue (all issued, out-of-range lanes dropped by the
// buffer range check), for the counted vmcnt waits of the 4 phases after it.
template <int ACT, bool SPLIT, bool F32>
constexpr int pk_epi_stores() {
    return 16 * ((SPLIT || F32) ? 2 : 1) + (act_fwd(ACT) ? 16 : 0) + (act_bwd(ACT) ? 4 : 0);
}

// DBG (timing-only ablation builds: gemm_pk_dbg.hip, cfg 90 + DBG; outputs are wrong): bit 0
// skips the main-loop operand DMA, bit 1 the counted vmcnt waits, bit 2 the epilogue body, bit 3
// issues the DMA between the two k-steps' MFMAs, bit 4 issues every main-loop DMA instruction with
// an out-of-range offset (same instructions, no memory traffic, no LDS writes), bit 5 (32) issues
// the bf16 epilogue's stores with an out-of-range offset (same instructions, no traffic), bit 6
// (64) drops them (the values stay live; the counted waits drop their allowance too).
// FP8: e4m3 operands, both K-contiguous (the forward x·Wᵀ), staged as "bf16 pairs" (K, lda, ldb
// in 2-byte units, so the DMA stream, the LDS images and the fragment reads are byte-identical to
// the bf16 kernel's); each phase's two k-step fragments of a row (16 B each) are concatenated into
// the 32-B operand of ONE v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales, the per-tensor
// scales in alpha).  A and B use the same byte→k mapping, so the permutation of k inside the
// 128-deep step cancels in the dot product.  8 scaled MFMAs (2x the cycles of a bf16 16x16x32
// each) per phase instead of 16: the same MFMA time per staged byte, i.e. twice the FLOP rate.
RN_DEV i32x8 pk_cat8(const s16x8 a, const s16x8 b) {
    const i32x4 x = __builtin_bit_cast(i32x4, a), y = __builtin_bit_cast(i32x4, b);
    return (i32x8){x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

// Returning +1 on a schedule counter by lane 0 only (a buffer atomic whose other lanes are out of
// range: no exec-mask branch), invisible to the compiler's waitcnt insertion like the DMA: the
// caller counts it in its vmcnt waits and reads the value only through pk_deq_take after the wait
// that retires it.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
RN_DEV void pk_deq_issue(uint32_t& v, const int* ctr, bool live) {
    const u32x4 rs = pk_rsrc_u(ctr, ctr ? 4u : 0u);
    const uint32_t off = live ? 0u : 0xFFFFFFF0u;
    v = 1u;
    asm volatile("buffer_atomic_add %0, %1, %2, 0 offen sc0 ; rn_deq_issue" : "+v"(v) : "v"(off), "s"(rs) : "memory");
}
RN_DEV int pk_deq_take(uint32_t v) {
    asm volatile("; rn_deq_take %0" : "+v"(v));
    return (int)__builtin_amdgcn_readfirstlane(v);
}
#pragma clang diagnostic pop

template <bool AK, bool BKC, int ACT, bool SPLIT, bool F32, int DBG = 0, int FP8 = 0, bool DYN = false>
__global__ void __launch_bounds__(512, 1) gemm_pk(GemmArgs p) {
    // FP8: 0 bf16; 1 e4m3 x e4m3; 2 A e5m2 (a gradient) x B e4m3.  Operand layouts: both K-contiguous
    // (the forward x·Wᵀ), A K- and B MN-contiguous (the data gradient dY·W), both MN-contiguous (the
    // weight gradient dYᵀ·X: fp32 split-K slabs only)
    static_assert(!FP8 || !(DBG & 8), "fp8: no DBG 8");
    static_assert(!FP8 || AK || (!BKC && SPLIT), "fp8 MN-contiguous A: weight gradient (both MN, split-K slabs) only");
    constexpr bool F8A_MN = FP8 && !AK;   // fp8 MN-contiguous images, read by transposing tr_b8 reads
    constexpr bool F8B_MN = FP8 && !BKC;
    constexpr bool F8MN = F8A_MN;  // (A MN implies B MN)
    // fp8 MN B: each lane holds two runs of 4 output columns (see the epilogue's column map), so a
    // bf16 output takes two 8-byte stores per fragment row; plain epilogue only
    static_assert(!F8B_MN || SPLIT || (ACT == ACT_NONE && !F32), "fp8 MN B, bf16 output: plain epilogue only");
    constexpr int S_EPI = (DBG & 64) ? 0 : pk_epi_stores<ACT, SPLIT, F32>() + ((F8B_MN && !SPLIT) ? 16 : 0);
    static_assert(!DYN || (!FP8 && DBG == 0), "dynamic schedule: bf16 production kernels only");
    constexpr int BM = 256, BN = 256;
    constexpr int WY = 6;  // ops younger than a phase's target half-tile: 3 half-tiles × 2 DMA
    static_assert(WY + 1 + S_EPI <= 63, "vmcnt range");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave >> 2, wc = wave & 3;  // wr: stagger group and A row block; wc: B column block
    const int G = lane >> 4;                  // output column group of this lane
    const int tiles = p.tiles_m * p.tiles_n;
    const int items = tiles * p.split;
    const int grid = gridDim.x;
    const int bid = xcd_remap(blockIdx.x, grid);
    const int nk = p.k_per_split / BK;

    // ---- tile schedule (see the header): static walk or dynamic queue over the items ----
    // DYN (a separate instantiation, so the static walk carries none of the queue's code; the
    // host takes it only for K slices of >= 5 K-tiles with a counter slot — not for fp8, whose
    // register pressure makes hipcc reuse the schedule op's register as a temporary between issue
    // and retire: tests/test_gemm_isa.py checks every instantiation)
    constexpr bool dyn = DYN;
    int* const ring = reinterpret_cast<int*>(smem + PK_RING);
    auto unit_of = [&](int s) -> int {
        if constexpr (!DYN) {
            const int u = bid + s * grid;
            return u < items ? u : -1;
        }
        return __builtin_amdgcn_readfirstlane(*(volatile int*)(ring + (s & 3)));
    };
    // the item of the v-th dequeue from queue q (0-7: dispatch group q's share of the static walk's
    // first rounds, grid a multiple of 8 with a power-of-two share; 8: the shared tail), -2 = group
    // queue drained, -1 = no work left
    auto deq_map = [&](int q, int v) -> int {
        const int per = grid >> 3;
        const bool home = (grid & 7) == 0 && (per & (per - 1)) == 0;
        const int rh = home ? max(0, items / grid - 1) : 0;
        if (q < 8) {
            const int sh = 31 - __builtin_clz(per | 1);
            return (unsigned)v < (unsigned)(rh * per) ? (v >> sh) * grid + q * per + (v & (per - 1)) : -2;
        }
        return (unsigned)v < (unsigned)(items - rh * grid) ? rh * grid + v : -1;
    };

    float alpha = 1.f;
    if (p.alpha) alpha = *p.alpha;
    asm volatile("" ::"v"(alpha));  // its load retires here, before any DMA is in flight

    // ---- DMA issue stream: half-tile σ = 4·t + h of K-tile t (stream order over the block's
    // items) goes to slot σ % 8.  Phase q of compute K-tile u issues h = (q + 2) % 4 of K-tile
    // u + 1 (q0, q1) or u + 2 (q2, q3): the half index is a compile-time constant per phase and
    // the source comes from a cursor that advances once per K-tile. ----
    auto item_coords = [&](int item, int& m0, int& n0, int& kb, int& ke, int& tm) {
        const int sid = item / tiles;
        int tn;
        group_tile(item - sid * tiles, p.tiles_m, p.tiles_n, tm, tn);
        m0 = tm * BM;
        n0 = tn * BN;
        kb = sid * p.k_per_split;
        ke = min(p.K, kb + p.k_per_split);
    };
    // per-lane (mn, k) coordinates of this wave's two DMA instructions of a half-tile, and their
    // in-tile byte offsets (kept: 4 VGPRs; the coordinates are recomputed on ragged tiles only)
    auto lane_mnk = [&](bool isA, int i, int& mn, int& k) {
        const int ins = wave * 2 + i;
        const bool kc = isA ? AK : BKC;
        if (kc) {
            mn = ins * 8 + (lane >> 3);
            k = ((lane & 7) ^ (isA ? swz_kc(mn) : swz_kcp(mn))) * 8;
        } else if (FP8) {  // k: byte row 0..127 of the fp8 MN image; mn: byte column
            k = ins * 8 + (lane >> 3);
            mn = ((lane & 7) ^ swz_f8(k)) * 16;
        } else {
            k = (ins & 7) * 8 + (lane >> 3);
            mn = (ins >> 3) * 64 + ((lane & 7) ^ (isA ? swz_mn(k) : swz_mnp(k))) * 8;
        }
    };
    uint32_t a_off[2], b_off[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int mn, k;
        lane_mnk(true, i, mn, k);
        // (fp8 MN: lda / ldb in BYTES, offsets in bytes)
        a_off[i] = (uint32_t)(F8A_MN ? (long)k * p.lda + mn : (AK ? (long)mn * p.lda + k : (long)k * p.lda + mn) * 2);
        lane_mnk(false, i, mn, k);
        b_off[i] = (uint32_t)(F8B_MN ? (long)k * p.ldb + mn : (BKC ? (long)mn * p.ldb + k : (long)k * p.ldb + mn) * 2);
    }
    const long a_step = AK ? (long)BK : (long)BK * p.lda, b_step = BKC ? (long)BK : (long)BK * p.ldb;
    // (fp8 MN: one K-tile = 128 k rows of lda bytes = 64·lda bf16 elements, the a_step formula; the
    // second half-tile starts 128 mn BYTES = 64 bf16 elements in)
    const long a_half = AK ? 128L * p.lda : (F8A_MN ? 64L : 128L), b_half = BKC ? 128L * p.ldb : (F8B_MN ? 64L : 128L);
    // cursor: the K-tile being issued (limits 0 once the block's items are exhausted: every
    // lane then reads out of range and the DMA only zero-fills its slot)
    const bf16* ca = p.A;
    const bf16* cb = p.B;
    int cml = 0, cnl = 0, ckl = 0, ckt = 0, ct = 0;
    int cu = -1, cs = 0;  // cursor: the item being issued, its sequence number (ring slot)
    // bit H: half-tile H of the K-tile being issued is interior (no per-lane range checks);
    // recomputed once per K-tile instead of in every phase's DMA issue
    uint32_t intr = 0;
    auto cur_intr = [&]() {
        const bool kf = ckl >= BK;
        intr = kf ? ((cml >= 128 ? 1u : 0u) | (cnl >= 128 ? 2u : 0u) | (cnl >= 256 ? 4u : 0u) | (cml >= 256 ? 8u : 0u))
                  : 0u;
    };
    bool in_loop = false;
    auto cur_set = [&]() {
        int m0, n0, kb, ke, tm;
        item_coords(cu, m0, n0, kb, ke, tm);
        ca = AK ? p.A + (long)m0 * p.lda + kb : p.A + (long)kb * p.lda + (F8A_MN ? m0 / 2 : m0);
        cb = BKC ? p.B + (long)n0 * p.ldb + kb : p.B + (long)kb * p.ldb + (F8B_MN ? n0 / 2 : n0);
        cml = p.M - m0;
        cnl = p.N - n0;
        ckl = ke - kb;
        cur_intr();
    };
    auto cur_adv = [&]() {
        ++ct;
        if (cu < 0) return;  // exhausted: every later DMA only zero-fills its slot
        if (++ckt < nk) {
            ca += a_step;
            cb += b_step;
            ckl -= BK;
            if (ckl < BK) intr = 0u;  // ragged last K-tile
            return;
        }
        ckt = 0;
        cu = unit_of(++cs);
        if (cu >= 0) {
            cur_set();
        } else {
            cml = cnl = ckl = 0;
            intr = 0u;
        }
    };
    const uint32_t lds0 = lds_addr(smem) + wave * 2048;  // this wave's 2 KiB of every slot
    auto issue_h = [&](auto hc) {
        constexpr int H = decltype(hc)::value;
        if constexpr (DBG & 1) {
            if (in_loop) return;
        }
        const uint32_t dst = lds0 + (uint32_t)(((ct & 1) * 4 + H) * PK_HALF);
        const bool isA = (H == 0 || H == 3);
        const bf16* base = isA ? (H == 3 ? ca + a_half : ca) : (H == 2 ? cb + b_half : cb);
        const int mnl = isA ? (H == 3 ? cml - 128 : cml) : (H == 2 ? cnl - 128 : cnl);
        const u32x4 rs = rsrc_sgpr(base);
        if constexpr (DBG & 16) {
            if (in_loop) {
#pragma unroll
                for (int i = 0; i < 2; ++i) dma16_at(rs, 0xFFFFFFF0u, dst + i * 1024);
                return;
            }
        }
        if (intr & (1u << H)) {  // interior half-tile: no per-lane checks
#pragma unroll
            for (int i = 0; i < 2; ++i) dma16_at(rs, isA ? a_off[i] : b_off[i], dst + i * 1024);
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                int mn, kk;
                lane_mnk(isA, i, mn, kk);
                const uint32_t o = isA ? a_off[i] : b_off[i];
                const bool f8mn = isA ? F8A_MN : F8B_MN;
                const bool kin = f8mn ? kk < 2 * ckl : kk < ckl;  // (fp8 MN: kk is a k byte, ckl in 2-byte units)
                dma16_at(rs, (mn < mnl && kin) ? o : 0xFFFFFFF0u, dst + i * 1024);
            }
        }
    };
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    using H2 = std::integral_constant<int, 2>;
    using H3 = std::integral_constant<int, 3>;

    f32x4 acc[2][2][4][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    s16x8 Af[4][2], Bl[2][2], Br[2][2];
    // fragment reads: bf16 / fp8 K-contiguous images as before; fp8 MN images by transposing reads,
    // the B side then in plain column order (fragment j = the wave's columns 16j .. 16j + 15, see the
    // epilogue's column map)
    auto frag_a = [&](const char* half, int mnbase, int s) -> s16x8 {
        if constexpr (F8A_MN) return pk_frag8_mn(half, mnbase, s, lane);
        else return pk_frag_a<AK>(half, mnbase, s, lane);
    };
    auto frag_b = [&](const char* half, int j, int s) -> s16x8 {
        if constexpr (F8B_MN) return pk_frag8_mn(half, wc * 32 + 16 * j, s, lane);
        else return pk_frag_b<BKC>(half, wc * 32, j, s, lane);
    };

    // ---- epilogue of one output tile, straight from the accumulators ----
    auto epilogue = [&](int m0, int n0, int tm, int sid) {
        const int mlim = p.M - m0, nlim = p.N - n0;
        // per-tile byte-range descriptors (tile-relative offsets stay far below 2^31)
        const long ldc = SPLIT ? (long)p.N : p.ldc;
        constexpr int ES = (SPLIT || F32) ? 4 : 2;
        char* cbase = SPLIT ? (char*)(p.ws + ((long)sid * p.M + m0) * p.N + n0) : (char*)p.C + ((long)m0 * ldc + n0) * ES;
        const __amdgpu_buffer_rsrc_t crs = pk_rsrc(cbase, 0x7FFFFFF0u);
        const u32x4 crs_u = pk_rsrc_u(cbase, 0x7FFFFFF0u);
        // output column of a lane's first value: 8 contiguous columns per lane group G (the permuted B
        // fragments), or for fp8 MN two runs of 4: columns 4G.. (fragment 0) and 16 + 4G.. (fragment 1)
        auto off = [&](int mh, int i, int nh, int es, int dc = 0) -> uint32_t {
            const int r = mh * 128 + wr * 64 + i * 16 + (lane & 15);
            const int c = nh * 128 + wc * 32 + (F8B_MN ? 4 : 8) * G + dc;
            return (r < mlim && c < nlim) ? (uint32_t)(((long)r * ldc + c) * es) : 0xFFFFFFF0u;
        };
        // bias: the wave's 2 × 32 columns through the scalar cache, then each lane picks its 8
        float bias[2][8];
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
            for (int t = 0; t < 8; ++t) bias[nh][t] = 0.f;
        if (!SPLIT && !act_bwd(ACT) && p.bias) {  // (activation-backward epilogues never take a bias)
#pragma unroll
            for (int nh = 0; nh < 2; ++nh) {
                const int cb = n0 + nh * 128 + wc * 32;
                if (cb + 32 <= p.N) {
                    const __attribute__((address_space(4))) u32x4* bp =
                        (const __attribute__((address_space(4))) u32x4*)(p.bias + cb);
                    u32x4 b0 = bp[0], b1 = bp[1], b2 = bp[2], b3 = bp[3];
                    // opaque SGPR values: otherwise the select below becomes a per-lane select of
                    // ADDRESSES and the scalar loads turn into vector loads (a vmcnt(0) drain)
                    asm volatile("" : "+s"(b0), "+s"(b1), "+s"(b2), "+s"(b3));
                    const u32x4 bsel = G == 0 ? b0 : (G == 1 ? b1 : (G == 2 ? b2 : b3));
                    pk_unpack8(bsel, bias[nh]);
                } else if (cb + 8 * G < p.N) {  // ragged last column block (N % 32 != 0)
                    const u32x4 u = *reinterpret_cast<const u32x4*>(p.bias + cb + 8 * G);
                    pk_unpack8(u, bias[nh]);
                }
            }
        }
        // full-tile operand read by the epilogue: saved pre-activation (act backward), residual,
        // or the accumulate target (bf16 out)
        const bf16* auxp = SPLIT ? nullptr
                                 : (act_bwd(ACT) ? p.pre : (p.res ? p.res : ((p.accumulate && !F32) ? (const bf16*)p.C : nullptr)));
        // (loaded one 128-row half at a time: 32 VGPRs, all 8 loads of a half in flight together;
        // both halves at once spill: the kernel is at the 256-VGPR limit)
        // activation-backward epilogues (no bias, no pre-activation store) load BOTH halves up front:
        // one exposed load round trip per tile instead of two
        constexpr bool AUX2 = act_bwd(ACT) && !SPLIT && !F32;
        u32x4 aux[AUX2 ? 2 : 1][4][2];
        const __amdgpu_buffer_rsrc_t ars = pk_rsrc(auxp ? auxp + (long)m0 * p.ldc + n0 : nullptr, 0x7FFFFFF0u);
        const u32x4 prs = pk_rsrc_u(act_fwd(ACT) && p.pre ? (void*)(p.pre + (long)m0 * p.ldc + n0) : nullptr,
                                    act_fwd(ACT) && p.pre ? 0x7FFFFFF0u : 0u);
        float csum[2][8];
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
            for (int t = 0; t < 8; ++t) csum[nh][t] = 0.f;
#pragma unroll
        for (int mh = 0; mh < 2; ++mh) {
            if (auxp && (!AUX2 || mh == 0)) {
#pragma unroll
                for (int ah = 0; ah < (AUX2 ? 2 : 1); ++ah)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int nh = 0; nh < 2; ++nh) {
#ifdef RN_PK_NO_AUX  // A/B only: no aux traffic and no wait (wrong outputs)
                        aux[ah][i][nh] = (u32x4){0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
#else
                        aux[ah][i][nh] = __builtin_amdgcn_raw_buffer_load_b128(ars, off(AUX2 ? ah : mh, i, nh, 2), 0, 0);
#endif
                    }
                // retire them HERE, in the branch that issued them (vmcnt(0); this epilogue drains the
                // operand DMA anyway): with the wait left to the separately-branched consumers below,
                // the compiler's wait insertion assumed the loads could still be pending at the main
                // loop's head and put vmcnt(2) + vmcnt(0) into every K-tile's first phase
#ifndef RN_PK_NO_AUX
                __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int nh = 0; nh < 2; ++nh) {
                    float v[8];
                    const bool swp = !BKC && !F8B_MN && (G & 1);  // bf16 MN image: odd lane groups hold fragment 1 first
#pragma unroll
                    for (int c = 0; c < 8; ++c) {
                        // compile-time register indices on both sides of the select (a runtime
                        // index would send the accumulators to scratch)
                        const float x0 = acc[mh][nh][i][c >> 2][c & 3], x1 = acc[mh][nh][i][(c >> 2) ^ 1][c & 3];
                        v[c] = (swp ? x1 : x0) * alpha;
                    }
                    if constexpr (SPLIT) {
                        const uint32_t o = off(mh, i, nh, 4);
                        const uint32_t o2 = F8B_MN ? off(mh, i, nh, 4, 16) : (o == 0xFFFFFFF0u ? o : o + 16);
                        pk_st16((u32x4){__builtin_bit_cast(uint32_t, v[0]), __builtin_bit_cast(uint32_t, v[1]),
                                    __builtin_bit_cast(uint32_t, v[2]), __builtin_bit_cast(uint32_t, v[3])},
                            crs_u, o);
                        pk_st16((u32x4){__builtin_bit_cast(uint32_t, v[4]), __builtin_bit_cast(uint32_t, v[5]),
                                    __builtin_bit_cast(uint32_t, v[6]), __builtin_bit_cast(uint32_t, v[7])},
                            crs_u, o2);
                        continue;
                    }
#pragma unroll
                    for (int c = 0; c < 8; ++c) v[c] += bias[nh][c];
                    if constexpr (act_fwd(ACT)) {
                        // pre-activation store (dropped when no pre buffer: zero-size descriptor);
                        // the activation is applied to the bf16-rounded value the backward sees
                        const u32x4 pu = {pk_pack2(v[0], v[1]), pk_pack2(v[2], v[3]), pk_pack2(v[4], v[5]),
                                          pk_pack2(v[6], v[7])};
                        if constexpr (ACT == ACT_GELU_D) {  // store gelu'(h) of the bf16-rounded h
                            pk_unpack8(pu, v);
                            float d[8];
#pragma unroll
                            for (int c = 0; c < 8; ++c) v[c] = gelu_and_grad_f(v[c], d[c]);
                            const u32x4 du = {pk_pack2(d[0], d[1]), pk_pack2(d[2], d[3]), pk_pack2(d[4], d[5]),
                                              pk_pack2(d[6], d[7])};
                            pk_st16(du, prs, off(mh, i, nh, 2));
                        } else {
                            pk_st16(pu, prs, off(mh, i, nh, 2));
                            if (p.pre) pk_unpack8(pu, v);
#pragma unroll
                            for (int c = 0; c < 8; ++c) v[c] = act_f<ACT>(v[c]);
                        }
                    }
                    if (auxp) {
                        float ax[8];
                        pk_unpack8(aux[AUX2 ? mh : 0][i][nh], ax);
                        if constexpr (act_bwd(ACT)) {
#pragma unroll
                            for (int c = 0; c < 8; ++c) {
                                v[c] = (float)(bf16)v[c] * act_grad_f<ACT>(ax[c]);
                                csum[nh][c] += (float)(bf16)v[c];
                            }
                        } else {
#pragma unroll
                            for (int c = 0; c < 8; ++c) v[c] += ax[c];
                        }
                    }
                    const uint32_t o = off(mh, i, nh, ES);
                    if constexpr (F32) {
                        float c8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                        if (p.accumulate) {
                            const u32x4 c0 = __builtin_amdgcn_raw_buffer_load_b128(crs, o, 0, 0);
                            const u32x4 c1 = __builtin_amdgcn_raw_buffer_load_b128(crs, o == 0xFFFFFFF0u ? o : o + 16, 0, 0);
                            const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
                            for (int d = 0; d < 8; ++d) c8[d] = __builtin_bit_cast(float, w[d]);
                        }
#pragma unroll
                        for (int c = 0; c < 8; ++c) v[c] += c8[c];
                        pk_st16((u32x4){__builtin_bit_cast(uint32_t, v[0]), __builtin_bit_cast(uint32_t, v[1]),
                                    __builtin_bit_cast(uint32_t, v[2]), __builtin_bit_cast(uint32_t, v[3])},
                            crs_u, o);
                        pk_st16((u32x4){__builtin_bit_cast(uint32_t, v[4]), __builtin_bit_cast(uint32_t, v[5]),
                                    __builtin_bit_cast(uint32_t, v[6]), __builtin_bit_cast(uint32_t, v[7])},
                            crs_u, o == 0xFFFFFFF0u ? o : o + 16);
                    } else {
                        if (p.res && p.accumulate) {  // both: residual above, accumulate target here
                            float c8[8];
                            pk_unpack8(__builtin_amdgcn_raw_buffer_load_b128(crs, o, 0, 0), c8);
#pragma unroll
                            for (int c = 0; c < 8; ++c) v[c] += c8[c];
                        }
                        const u32x4 ou = {pk_pack2(v[0], v[1]), pk_pack2(v[2], v[3]), pk_pack2(v[4], v[5]),
                                          pk_pack2(v[6], v[7])};
                        if constexpr (DBG & 64) asm volatile("" ::"v"(ou));         // ablation: no stores
                        else if constexpr (F8B_MN) {  // columns 4G.. and 16 + 4G..
                            pk_st8((u32x2v){ou.x, ou.y}, crs_u, o);
                            pk_st8((u32x2v){ou.z, ou.w}, crs_u, off(mh, i, nh, 2, 16));
                        } else if (p.st_nt & 1) pk_st16_nt(ou, crs_u, o);          // wave-uniform choice
                        else pk_st16(ou, crs_u, (DBG & 32) ? 0xFFFFFFF0u : o);   // ablation: no traffic
                    }
                }
        }
        if constexpr (act_bwd(ACT)) {
            // per-wave column sums of the stored dH (bias gradient of the layer it feeds):
            // reduce over the 16 rows of the lane group, one partial row per (M-tile, wr)
#pragma unroll
            for (int nh = 0; nh < 2; ++nh)
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    float s = csum[nh][c];
                    s += __shfl_xor(s, 1, 64);
                    s += __shfl_xor(s, 2, 64);
                    s += __shfl_xor(s, 4, 64);
                    s += __shfl_xor(s, 8, 64);
                    csum[nh][c] = s;
                }
            float* cpb = p.colpart ? p.colpart + ((long)tm * 2 + wr) * p.N + n0 : nullptr;
            const u32x4 cprs = pk_rsrc_u(cpb, cpb ? 0x7FFFFFF0u : 0u);
#pragma unroll
            for (int nh = 0; nh < 2; ++nh) {
                const int c = nh * 128 + wc * 32 + 8 * G;
                const uint32_t o = ((lane & 15) == 0 && c < nlim) ? (uint32_t)(c * 4) : 0xFFFFFFF0u;
                pk_st16((u32x4){__builtin_bit_cast(uint32_t, csum[nh][0]), __builtin_bit_cast(uint32_t, csum[nh][1]),
                            __builtin_bit_cast(uint32_t, csum[nh][2]), __builtin_bit_cast(uint32_t, csum[nh][3])},
                    cprs, o);
                pk_st16((u32x4){__builtin_bit_cast(uint32_t, csum[nh][4]), __builtin_bit_cast(uint32_t, csum[nh][5]),
                            __builtin_bit_cast(uint32_t, csum[nh][6]), __builtin_bit_cast(uint32_t, csum[nh][7])},
                    cprs, o == 0xFFFFFFF0u ? o : o + 16);
            }
        }
    };

    // ---- dynamic schedule: wave 0's dequeue state (see the header) ----
    // bits 0-3: queue of the next dequeue (0-7 dispatch group, 8 tail); 4: requested; 5: the
    // atomic in flight is a real dequeue; 6: no work left
    int deq = blockIdx.x & 7;
    uint32_t deq_v = 0u;

    // ---- prologue: the first item, then σ = 0..5 in flight (K-tile 0, halves 0/1 of K-tile 1) ----
    if constexpr (DYN) {
        if (wave == 0 && lane == 0) {  // nothing is in flight yet: plain atomics, compiler-managed waits
            int q = blockIdx.x & 7;
            int u = deq_map(q, __hip_atomic_fetch_add(p.sched + q * PK_CTR_STRIDE, 1, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
            if (u == -2) {  // this group's queue is empty: the shared tail
                q = 8;
                u = deq_map(8, __hip_atomic_fetch_add(p.sched + 8 * PK_CTR_STRIDE, 1, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
            }
            ring[0] = u;
            ring[1] = q | (u < 0 ? 64 : 0);
        }
        __syncthreads();  // no DMA in flight yet: a plain barrier drains nothing
        deq = __builtin_amdgcn_readfirstlane(ring[1]);
    }
    int c_s = 0;  // compute side: sequence number of its item (ring slot), and the item
    int c_u = unit_of(0);  // (dynamic: the cursor is never more than one item ahead, nk >= 5)
    cu = c_u;
    if (cu >= 0) {
        cur_set();
        issue_h(H0{});
        issue_h(H1{});
        issue_h(H2{});
        issue_h(H3{});
        cur_adv();
        issue_h(H0{});
        issue_h(H1{});
    }
    vm_wait<8>();
    asm volatile("s_barrier" ::: "memory");
    if (wr == 1) asm volatile("s_barrier" ::: "memory");  // stagger: waves 4-7 one barrier behind
    in_loop = true;
    __builtin_amdgcn_sched_barrier(0);

    int c_m0 = 0, c_n0 = 0, c_kb = 0, c_ke = 0, c_tm = 0, c_sid = 0, c_kt = 0;
    if (c_u >= 0) {
        item_coords(c_u, c_m0, c_n0, c_kb, c_ke, c_tm);
        c_sid = c_u / tiles;
    }
    int since_epi = 4;

    // phase wait: σ ≤ φ+2 must have landed (this wave's DMA); younger = the 3 half-tiles
    // issued in the previous 3 phases (6 ops) plus, within 4 phases of an epilogue, its stores,
    // plus in q1-q3 (XW) wave 0's schedule atomic of this K-tile
    auto phase_wait = [&](auto xw) {
        if constexpr (DBG & 2) return;
        constexpr bool XW = decltype(xw)::value;
        if (since_epi < 4) {
            if (DYN && XW && wave == 0) vm_wait<WY + 1 + S_EPI>();
            else vm_wait<WY + S_EPI>();
        } else {
            if (DYN && XW && wave == 0) vm_wait<WY + 1>();
            else vm_wait<WY>();
        }
        ++since_epi;
    };
    // q0, after its wait, before its DMA: wave 0 consumes the previous K-tile's atomic (retired by
    // that wait) and sends this K-tile's (a dequeue if one is wanted, else a no-op).  Real dequeues
    // are sent at an item's K-tile 0 or 1 only and consumed by K-tile 2 (nk >= 5); the no-op of an
    // item's last K-tile is retired before the epilogue (vm_wait<8> there), so no asynchronous
    // register write can land while the epilogue reuses registers
    auto deq_step = [&]() {
        if (DYN && wave == 0) {
            if (deq & 32) {
                const int u = deq_map(deq & 15, pk_deq_take(deq_v));
                if (u == -2) {
                    deq = (deq & 64) | 8 | 16;  // this group's queue is drained: the shared tail
                } else {
                    if (lane == 0) *(volatile int*)(ring + ((c_s + 1) & 3)) = u;
                    deq = (deq & ~32) | (u < 0 ? 64 : 0);
                }
            }
            // ONE asm on both paths (a branch per path made hipcc merge two registers by copies
            // issued before the hardware had written the value)
            const bool want = (deq & 16) != 0;
            pk_deq_issue(deq_v, p.sched + (deq & 15) * PK_CTR_STRIDE, lane == 0 && want);
            deq = (deq & ~48) | (want ? 32 : 0);
        }
    };
    auto sync_mma_begin = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
    };
    auto sync_mma_end = [&]() {
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
#define RN_PK_MMA(MH, NH, BF)                                                                          \
    if constexpr (FP8) {                                                                               \
        _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                             \
        _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                             \
            acc[MH][NH][i_][j_] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(                   \
                pk_cat8(BF[j_][0], BF[j_][1]), pk_cat8(Af[i_][0], Af[i_][1]), acc[MH][NH][i_][j_], 0,     \
                FP8 == 2 ? 1 : 0, 0, 127, 0, 127);                                                     \
    } else {                                                                                           \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                                 \
    _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                 \
    _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                                 \
        acc[MH][NH][i_][j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(BF[j_][s_], Af[i_][s_], acc[MH][NH][i_][j_], 0, 0, 0); \
    }

#define RN_PK_MMA_S(MH, NH, BF, S)                                                                    \
    _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                 \
    _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                                 \
        acc[MH][NH][i_][j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(BF[j_][S], Af[i_][S], acc[MH][NH][i_][j_], 0, 0, 0);
    // one phase: counted wait, this phase's fragment reads, the DMA of one half-tile (in the read
    // segment, or between the two k-steps' MFMAs with DBG bit 3), barrier, 16 MFMAs, barrier
#define RN_PK_PHASE(XW, READS, ISSUE, MH, NH, BF)                                                      \
    phase_wait(std::integral_constant<bool, XW>{});                                                    \
    READS                                                                                              \
    if constexpr (!(DBG & 8)) { ISSUE }                                                                \
    sync_mma_begin();                                                                                  \
    if constexpr (DBG & 8) {                                                                           \
        RN_PK_MMA_S(MH, NH, BF, 0)                                                                     \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        ISSUE                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        RN_PK_MMA_S(MH, NH, BF, 1)                                                                     \
    } else {                                                                                           \
        RN_PK_MMA(MH, NH, BF)                                                                          \
    }                                                                                                  \
    sync_mma_end();


    // static walk: the block's item count is known (bid + s·grid < items)
    const int n_static = DYN ? 0 : ((items - bid + grid - 1) / grid) * nk;
#pragma unroll 1
    for (int u = 0; DYN ? (c_u >= 0) : (u < n_static); ++u) {
        const char* sl = smem + (u & 1) * (4 * PK_HALF);
        // an item's first K-tile: wave 0 asks for the item after it (sent after q0's DMA)
        if (dyn && wave == 0 && c_kt == 0 && !(deq & 64)) deq |= 16;
        // q0: At + Bl  (fragment reads first: their latency runs under the DMA issue)
        RN_PK_PHASE(false,
            deq_step();
            _Pragma("unroll") for (int s = 0; s < 2; ++s) {
                _Pragma("unroll") for (int i = 0; i < 4; ++i) Af[i][s] = frag_a(sl, wr * 64 + i * 16, s);
                _Pragma("unroll") for (int j = 0; j < 2; ++j) Bl[j][s] = frag_b(sl + PK_HALF, j, s);
            },
            issue_h(H2{});, 0, 0, Bl)
        // q1: At + Br
        RN_PK_PHASE(true,
            _Pragma("unroll") for (int s = 0; s < 2; ++s)
                _Pragma("unroll") for (int j = 0; j < 2; ++j) Br[j][s] = frag_b(sl + 2 * PK_HALF, j, s);,
            issue_h(H3{});, 0, 1, Br)
        // q2: Ab + Br (the cursor moves on to K-tile u + 2)
        RN_PK_PHASE(true,
            _Pragma("unroll") for (int s = 0; s < 2; ++s)
                _Pragma("unroll") for (int i = 0; i < 4; ++i) Af[i][s] = frag_a(sl + 3 * PK_HALF, wr * 64 + i * 16, s);,
            cur_adv(); issue_h(H0{});, 1, 1, Br)
        // q3: Ab + Bl (all fragments already in registers)
        RN_PK_PHASE(true, , issue_h(H1{});, 1, 0, Bl)
        if (++c_kt == nk) {
            // retire wave 0's schedule op of this K-tile (issued before q0's DMA: 8 younger ops);
            // every other op this waits for, the next q0 wait would wait for anyway
            if constexpr (DYN) vm_wait<8>();
            if constexpr (!(DBG & 4)) {
                epilogue(c_m0, c_n0, c_tm, c_sid);
            } else {  // keep the accumulators (and the MFMAs feeding them) alive
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
#pragma unroll
                            for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[a][b][i][j]));
            }
            since_epi = 0;
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
            c_kt = 0;
            c_u = unit_of(++c_s);
            if (c_u >= 0) {
                item_coords(c_u, c_m0, c_n0, c_kb, c_ke, c_tm);
                c_sid = c_u / tiles;
            }
        }
    }
#undef RN_PK_MMA
#undef RN_PK_MMA_S
#undef RN_PK_PHASE
    if (wr == 0) asm volatile("s_barrier" ::: "memory");  // balance the stagger barrier
    if (DYN && wave == 0 && lane == 0) {  // the last block out resets the counters for the next launch
        int* const cnt = p.sched;
        if (__hip_atomic_fetch_add(cnt + 9 * PK_CTR_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == grid - 1) {
#pragma unroll
            for (int i = 0; i < 10; ++i) __hip_atomic_store(cnt + i * PK_CTR_STRIDE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    (void)c_kb;
    (void)c_ke;
}

// Launch: persistent grid of min(units, CUs − reserve) workgroups (1 per CU: 128 KiB LDS).
//   reserve (rn_gemm_set_reserve): CUs left free for a concurrently running collective, so RCCL's
//   workgroups find a CU at once instead of waiting for a GEMM to drain (set while a data-parallel
//   communicator is active); the dynamic schedule (rn_gemm_set_sched, default on) takes a counter
//   slot from the device pool, or falls back to the static walk if the pool cannot be created
//   (first use inside a stream capture).
}  // namespace rn_gemm_detail
extern "C" int* rn_gemm_sched_slot(int dev, hipStream_t st);
extern "C" int rn_gemm_get_reserve();
namespace rn_gemm_detail {
// non-temporal output stores: plain bf16 outputs over 1 GiB (a 256 MiB threshold also caught outputs
// the next kernel reads at once, +0.14-0.4 ms per GPT-2-small step, profiles/r3s_resume_xent_gelu.txt
// item 17)
// (a non-temporal store of the activation epilogue's second output, read only by the backward, was
// measured as no change and removed in round 4)
inline int rn_gemm_st_nt(const GemmArgs& a) {
    return (a.split <= 1 && (long)a.M * a.N * 2 > (1024L << 20)) ? 1 : 0;
}
}  // namespace rn_gemm_detail
namespace rn_gemm_detail {

// the host side of the schedule choice: a counter slot for a dynamic launch (needs K slices of
// >= 5 K-tiles and the queue enabled), else nullptr (static walk)
inline int* pk_sched_slot(const GemmArgs& a, hipStream_t st) {
    if (a.k_per_split / BK < 5) return nullptr;
    int dev = 0;
    (void)hipGetDevice(&dev);
    return rn_gemm_sched_slot(dev, st);
}

template <bool AK, bool BKC, int ACT, bool SPLIT, bool F32, int DBG = 0, int FP8 = 0, bool DYN = false>
void launch_pk_t(GemmArgs& a, hipStream_t st) {
    auto kern = gemm_pk<AK, BKC, ACT, SPLIT, F32, DBG, FP8, DYN>;
    static int attr_dev = -1;  // the >64 KiB LDS opt-in, per device the process launches on
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (attr_dev != dev) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, PK_LDS);
        attr_dev = dev;
    }
    const int items = a.tiles_m * a.tiles_n * a.split;
    int cus = 256;
    {
        static int cu_dev = -1, cu_n = 256;
        if (cu_dev != dev) {
            hipDeviceProp_t prop;
            if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cu_n = prop.multiProcessorCount;
            cu_dev = dev;
        }
        cus = cu_n;
    }
    a.st_nt = rn_gemm_st_nt(a);
    const int reserve = rn_gemm_get_reserve();
    if (reserve > 0 && reserve < cus) cus -= reserve;
    if (!DYN) a.sched = nullptr;
    const int grid = items < cus ? items : cus;
    kern<<<grid, 512, PK_LDS, st>>>(a);
}

}  // namespace rn_gemm_detail
