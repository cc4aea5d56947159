// Templated MFMA GEMM kernels (see csrc/kernels/gemm_bf16.hip for the design notes).
// Instantiated per tile config in gemm_cfg*.hip so the configs compile in parallel.
#pragma once
#include <algorithm>
#include "common.h"

namespace rn_gemm_detail {

constexpr int BK = 64;
constexpr int GROUP_M = 8;

typedef __attribute__((address_space(3))) void lds_void;

// u32 division by a runtime constant: q = (umulhi(n, mul) + n) >> shr, exact for n, d < 2^31
struct FastDiv {
    uint32_t d, mul, shr;
};
static inline FastDiv make_fastdiv(uint32_t d) {
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    const uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
    return FastDiv{d, (uint32_t)m, l};
}
RN_DEV uint32_t fdiv(uint32_t n, const FastDiv& f) { return (__umulhi(n, f.mul) + n) >> f.shr; }

// Implicit-GEMM convolution geometry (NHWC bf16, C % 64 == 0 for the gathered operand):
//   mode 1 (fwd):   A[m = (n,oh,ow)][k = (kh,kw,c)] = x[n][oh·S-P+kh][ow·S-P+kw][c]
//   mode 2 (dgrad, S = 1): A[m = (n,ih,iw)][k = (kh,kw,co)] = dY[n][ih+P-kh][iw+P-kw][co],
//                   B[k][c] = W[co][kh][kw][c]  (row stride bld = KH·KW·C)
//   mode 3 (wgrad): B[k = (n,oh,ow)][j = (kh,kw,c)] = x[n][oh·S-P+kh][ow·S-P+kw][c]
struct ConvGeom {
    int H, W, C;     // gathered tensor (x, or dY for dgrad)
    int RH, RW;      // decode of the pixel index: p = (n·RH + y)·RW + x
    int KH, KW, S, P;
    int KC;          // channels per tap in the K layout
    int BC;          // dgrad: channels of W's last dim (= GEMM N)
    long bld;        // dgrad: W row stride
    FastDiv fd_hw, fd_w, fd_kc, fd_kw;
};

struct GemmArgs {
    const bf16* A;
    const bf16* B;
    void* C;
    const bf16* bias;
    const bf16* res;
    bf16* pre;
    float* ws;
    const float* alpha;  // optional device scalar multiplying op(A)·op(B)
    int M, N, K;
    long lda, ldb, ldc;
    int tiles_m, tiles_n, split, k_per_split;
    int out_f32, accumulate;
    // optional [tiles_m][N] fp32: per-M-tile column sums of the output (bias gradient of
    // the layer the activation-backward epilogue feeds); only for act-backward epilogues
    // on configs with (threads % (BN/8)) == 0, see colpart_ok()
    float* colpart;
    ConvGeom cv;
    // optional e4m3 copy of an activation-forward output for the NEXT fp8 GEMM (delayed scaling:
    // q8st[0] = scale, rolled before the launch; the kernel records amax(|out|) in q8st[1]);
    // staged epilogue of the one-tile-per-block kernels only
    uint8_t* q8;
    float* q8st;
    // persistent kernel (cfg 9) only: dynamic tile queue counters (gemm_pk.h, "Tile schedule"),
    // nullptr = static walk
    int* sched;
    // persistent kernel only: store the bf16 output with the non-temporal policy (set by the host
    // for outputs larger than the 256 MiB Infinity Cache, e.g. the LM-head logits: such a stream
    // cannot stay resident and would only evict the operand panels the main loop re-reads)
    int st_nt;
    // split-K reduction only: slab s lives at ws + s·slab_step·M·N (<= 1: contiguous slabs); set when
    // a group pre-reduction (splitk_group_k) left its partial sums in every slab_step-th slab
    int slab_step;
    // one-wave-per-SIMD kernel (cfg 11, gemm_w1.h), fp8 operands: the two per-tensor scales (powers of
    // two, ops/fp8.py) ride the scaled MFMA's E8M0 block-scale operands instead of an epilogue multiply
    const float* sa;
    const float* sb;
    // cfg 11 tile walk: tile-rows per group (0: GROUP_M)
    int group_m;
    // split-K reduction only: optional device scalar multiplying the slab sum (the fp8 weight gradient of the
    // LM head: the loss gradient's g / n; the slabs themselves carry only the power-of-two tensor scales)
    const float* reduce_alpha;
};

template <int BN, int NT>
constexpr bool colpart_cfg_ok() { return (NT % (BN / 8)) == 0; }

RN_DEV int swz_kc(int r) { return (r >> 1) & 7; }
RN_DEV int swz_mn(int k) { return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1; }

RN_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
    // readfirstlane keeps the descriptor provably wave-uniform (no waterfall loops, guide T20)
    const uint64_t bp = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 0x7FFFFFF0, 0x00020000);
}

// Stage one ROWS(mn)×64(k) operand tile into LDS with NW waves.
//   KC:  global element (mn, k) at base[mn*ld + k]; image [ROWS][64 k] (128-B rows),
//        16-B chunk c of row r at c ^ swz_kc(r), read with ds_read_b128.
//   !KC: global element (mn, k) at base[k*ld + mn]; image = ROWS/64 sub-images
//        [64 k][64 mn] (128-B rows), chunk c of k-row r at c ^ swz_mn(r), read with
//        ds_read_b64_tr_b16.  swz_mn maps the 8 k-rows one 32-lane half reads
//        ({0..3, 8..11} + const) to 8 distinct (row parity, chunk pair) slots of the
//        256-B bank row: conflict-free.  Any multiple of 64 columns works (192 too).
// The XOR is applied to the per-lane GLOBAL source address (the DMA destination
// is lane-linear, guide rule 21) and again on the read address.
template <bool KC, int ROWS, int NW>
RN_DEV void stage(const bf16* base, long ld, int mn_lim, int k_lim, char* lds, int wave, int lane) {
    __amdgpu_buffer_rsrc_t rsrc = make_rsrc(base);
    constexpr int NINS = ROWS * 128 / 1024;  // 1 KiB per wave-instruction
    constexpr int PER = NINS / NW;
    static_assert(NINS % NW == 0, "tile / wave mismatch");
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int ins = wave * PER + i;
        uint32_t voff;
        if constexpr (KC) {
            const int r = ins * 8 + (lane >> 3);
            const int cg = (lane & 7) ^ swz_kc(r);
            const int k = cg * 8;
            const bool ok = (r < mn_lim) && (k < k_lim);
            voff = ok ? (uint32_t)(((long)r * ld + k) * 2) : 0xFFFFFFF0u;
        } else {
            const int sub = ins >> 3, within = ins & 7;
            const int r = within * 8 + (lane >> 3);
            const int cg = (lane & 7) ^ swz_mn(r);
            const int mn = sub * 64 + cg * 8;
            const bool ok = (r < k_lim) && (mn < mn_lim);
            voff = ok ? (uint32_t)(((long)r * ld + mn) * 2) : 0xFFFFFFF0u;
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + ins * 1024), 16, voff, 0, 0, 0);
    }
}

// fragment: 8 consecutive k (k-step s: k = s*32 + 8*(lane>>4) + 0..7) of row/col
// mnbase + (lane & 15) within the tile.
template <bool KC>
RN_DEV s16x8 frag(const char* lds, int mnbase, int s, int lane) {
    if constexpr (KC) {
        const int row = mnbase + (lane & 15);
        const int chunk = s * 4 + (lane >> 4);
        return *reinterpret_cast<const s16x8*>(lds + row * 128 + ((chunk ^ swz_kc(row)) << 4));
    } else {
        const char* sub = lds + (mnbase >> 6) * 8192;
        const int mnl = mnbase & 63;
        const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
        const int c = (mnl >> 3) + (p >> 1);
        const int k0 = s * 32 + 8 * g + q;
        const int k1 = k0 + 4;
        const char* a0 = sub + k0 * 128 + ((c ^ swz_mn(k0)) << 4) + (p & 1) * 8;
        const char* a1 = sub + k1 * 128 + ((c ^ swz_mn(k1)) << 4) + (p & 1) * 8;
        s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
        s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
        s16x8 r;
        r[0] = v0[0]; r[1] = v0[1]; r[2] = v0[2]; r[3] = v0[3];
        r[4] = v1[0]; r[5] = v1[1]; r[6] = v1[2]; r[7] = v1[3];
        return r;
    }
}

// XCD remap (bijective for any nblocks): the dispatcher deals block ids round-robin over the
// 8 XCDs, so blocks sharing bid%8 share an L2; give each such group a contiguous id range.
RN_DEV int xcd_remap(int bid, int nblocks) {
    const int xcd = bid & 7, loc = bid >> 3;
    const int q = nblocks >> 3, r = nblocks & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// grouped ordering of a linear tile id: GROUP_M tile-rows share B panels
RN_DEV void group_tile(int id, int tiles_m, int tiles_n, int& tm, int& tn) {
    const int per_group = GROUP_M * tiles_n;
    const int gid = id / per_group;
    const int first_m = gid * GROUP_M;
    const int gsz = min(tiles_m - first_m, GROUP_M);
    const int in = id % per_group;
    tm = first_m + in % gsz;
    tn = in / gsz;
}

// the same with a run-time group height
RN_DEV void group_tile_g(int id, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
    const int per_group = gm * tiles_n;
    const int gid = id / per_group;
    const int first_m = gid * gm;
    const int gsz = min(tiles_m - first_m, gm);
    const int in = id % per_group;
    tm = first_m + in % gsz;
    tn = in / gsz;
}

// XCD-banded order of the one-wave-per-SIMD kernel's static walk (cfg 11, round 6).  Unit u = bid + s·grid (bid the
// xcd_remap'ed block id: hardware blocks with blockIdx % 8 == x hold bids [x·per, (x+1)·per)) is
// mapped so that XCD x computes ALL tiles of the tile-row band [x·tm/8, (x+1)·tm/8) and nothing else:
// every A panel is fetched into exactly one XCD's L2 (the grouped walk over the whole grid split a
// group's tile-rows across two XCDs, so about a third of A was fetched twice from the fabric).  Inside
// the band the walk is the usual GROUP_M-grouped order.  A bijection on [0, tm·tn) when
// band_ok(): grid % 8 == 0, tm % 8 == 0 and tm·tn % grid == 0 (every block the same number of
// items) — true for every GPT-2 GEMM without split-K; other shapes keep the grouped walk.  The
// Measured (profiles/gemm_band_r6b.txt): fp8 c_attn / c_fc shape (65536 x 3072 x 1024) 1410 -> 1516 TF/s,
// MLP c_proj (K 4096) 1768 -> 1808.  On cfg 9 (bf16) the same order changed nothing — identical L2
// hit / miss / memory-side request counts: with 3 to 12 tile columns a 32-CU round covers a
// fractional number of tile-rows, so about a third of the A panels straddle two rounds and are
// fetched again after the round between evicted them, whichever XCD owns them (docs/DESIGN.md §3).
RN_DEV bool band_ok(int grid, int tiles_m, int tiles_n) {
    return (grid & 7) == 0 && (tiles_m & 7) == 0 && (tiles_m * tiles_n) % grid == 0;
}
RN_DEV void band_tile(int u, int grid, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
    const int per = grid >> 3;
    const int s = u / grid, r = u - s * grid;
    const int x = r / per;
    const int bx = tiles_m >> 3;
    group_tile_g(r - x * per + s * per, bx, tiles_n, gm, tm, tn);
    tm += x * bx;
}


RN_DEV void map_tile(int bid, int nblocks, int tiles_m, int tiles_n, int& tm, int& tn) {
    group_tile(xcd_remap(bid, nblocks), tiles_m, tiles_n, tm, tn);
}

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// fp8 fragment for v_mfma_scale_f32_16x16x128_f8f6f4: 32 e4m3 bytes of row mnbase + (lane&15)
// from the same K-contiguous 128-B-row LDS image the bf16 path uses: 16-B chunks g and g + 4
// (g = lane>>4), i.e. exactly the two chunks the bf16 path's k-steps 0 and 1 read, so the XOR
// swizzle keeps each ds_read_b128 lane group conflict-free (chunks 2g, 2g+1 — the round-1 mapping —
// measured 50 % LDS bank conflicts).  The MFMA's k order inside the 128-deep step is then a
// permutation of the row's bytes, the SAME one for A and B, so it cancels in the dot product.
RN_DEV i32x8 frag8(const char* lds, int mnbase, int lane) {
    const int row = mnbase + (lane & 15), g = lane >> 4;
    const char* rp = lds + row * 128;
    const i32x4 lo = *reinterpret_cast<const i32x4*>(rp + ((g ^ swz_kc(row)) << 4));
    const i32x4 hi = *reinterpret_cast<const i32x4*>(rp + (((g + 4) ^ swz_kc(row)) << 4));
    return (i32x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// ---- deep-pipeline support: compiler-invisible LDS-DMA + counted vmcnt waits ----
// With more than one tile in flight the compiler's own waits would drain every DMA
// (s_waitcnt vmcnt(0)) at each barrier and in front of LDS reads it cannot prove
// disjoint from the DMA target; issuing the DMA from inline asm hides it, and the
// kernel waits with counted vmcnt(N) itself (never 0 in steady state).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

RN_DEV u32x4 rsrc_sgpr(const void* base) {
    const uint64_t bp = (uint64_t)base;
    u32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    r[2] = 0x7FFFFFF0u;
    r[3] = 0x00020000u;
    return r;
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// LDS byte address (32-bit) of a dynamic-shared pointer, without the generic-pointer null check
RN_DEV uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(lds_void*)p; }
RN_DEV void dma16_at(const u32x4& rs, uint32_t voff, uint32_t lds_byte) {
    const uint32_t l = __builtin_amdgcn_readfirstlane(lds_byte);
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(l)
                 : "memory", "m0");
}
RN_DEV void dma16(const u32x4& rs, uint32_t voff, const char* lds) {
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)lds);
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(l)
                 : "memory", "m0");
}
#pragma clang diagnostic pop

template <int N>
RN_DEV void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// same tile/image as stage(), DMA through dma16
template <bool KC, int ROWS, int NW>
RN_DEV void stage_async(const bf16* base, long ld, int mn_lim, int k_lim, char* lds, int wave, int lane) {
    const u32x4 rs = rsrc_sgpr(base);
    constexpr int NINS = ROWS * 128 / 1024;
    constexpr int PER = NINS / NW;
    static_assert(NINS % NW == 0, "tile / wave mismatch");
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int ins = wave * PER + i;
        uint32_t voff;
        if constexpr (KC) {
            const int r = ins * 8 + (lane >> 3);
            const int cg = (lane & 7) ^ swz_kc(r);
            const int k = cg * 8;
            const bool ok = (r < mn_lim) && (k < k_lim);
            voff = ok ? (uint32_t)(((long)r * ld + k) * 2) : 0xFFFFFFF0u;
        } else {
            const int sub = ins >> 3, within = ins & 7;
            const int r = within * 8 + (lane >> 3);
            const int cg = (lane & 7) ^ swz_mn(r);
            const int mn = sub * 64 + cg * 8;
            const bool ok = (r < k_lim) && (mn < mn_lim);
            voff = ok ? (uint32_t)(((long)r * ld + mn) * 2) : 0xFFFFFFF0u;
        }
        dma16(rs, voff, lds + ins * 1024);
    }
}

// ---- implicit-GEMM convolution operand loaders (LDS images identical to stage()) ----
// A rows gathered from an NHWC tensor (modes 1, 2): K-contiguous image, one (kh, kw) tap and
// 64 channels per K-tile (C % 64 == 0), zero-fill outside the image (padding) and past M.
template <int ROWS, int NW, int MODE>
RN_DEV void stage_conv_a(const GemmArgs& p, int m0, int k0, int kend, char* lds, int wave, int lane) {
    const ConvGeom& g = p.cv;
    const u32x4 rs = rsrc_sgpr(p.A);
    constexpr int NINS = ROWS * 128 / 1024;
    constexpr int PER = NINS / NW;
    const int tap = (int)fdiv((uint32_t)k0, g.fd_kc);
    const int c0 = k0 - tap * g.KC;
    const int kh = (int)fdiv((uint32_t)tap, g.fd_kw), kw = tap - kh * g.KW;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int ins = wave * PER + i;
        const int r = ins * 8 + (lane >> 3);
        const int cg = (lane & 7) ^ swz_kc(r);
        const int m = m0 + r;
        const int n = (int)fdiv((uint32_t)m, g.fd_hw);
        const int rem = m - n * g.RH * g.RW;
        const int y = (int)fdiv((uint32_t)rem, g.fd_w), x = rem - y * g.RW;
        const int ih = MODE == 1 ? y * g.S - g.P + kh : y + g.P - kh;
        const int iw = MODE == 1 ? x * g.S - g.P + kw : x + g.P - kw;
        const bool ok = m < p.M && k0 < kend && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        const uint32_t voff = ok ? (uint32_t)(((((n * g.H + ih) * g.W + iw) * g.C) + c0 + cg * 8) * 2) : 0xFFFFFFF0u;
        dma16(rs, voff, lds + ins * 1024);
    }
}

// B gathered for the weight gradient (mode 3): N-contiguous image (64-column sub-images,
// k-rows = output pixels), one tap per sub-image.
template <int COLS, int NW>
RN_DEV void stage_conv_b(const GemmArgs& p, int n0, int k0, int kend, char* lds, int wave, int lane) {
    const ConvGeom& g = p.cv;
    const u32x4 rs = rsrc_sgpr(p.B);
    constexpr int NINS = COLS * 128 / 1024;
    constexpr int PER = NINS / NW;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int ins = wave * PER + i;
        const int sub = ins >> 3, within = ins & 7;
        const int r = within * 8 + (lane >> 3);
        const int cg = (lane & 7) ^ swz_mn(r);
        const int nn = n0 + sub * 64;
        const int tap = (int)fdiv((uint32_t)nn, g.fd_kc);
        const int cb = nn - tap * g.KC;
        const int kh = (int)fdiv((uint32_t)tap, g.fd_kw), kw = tap - kh * g.KW;
        const int pix = k0 + r;
        const int n = (int)fdiv((uint32_t)pix, g.fd_hw);
        const int rem = pix - n * g.RH * g.RW;
        const int y = (int)fdiv((uint32_t)rem, g.fd_w), x = rem - y * g.RW;
        const int ih = y * g.S - g.P + kh, iw = x * g.S - g.P + kw;
        const bool ok = pix < kend && nn + cg * 8 < p.N && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        const uint32_t voff = ok ? (uint32_t)(((((n * g.H + ih) * g.W + iw) * g.C) + cb + cg * 8) * 2) : 0xFFFFFFF0u;
        dma16(rs, voff, lds + ins * 1024);
    }
}

template <int BM, int BN, int WM, int WN, bool AK, bool BK_, int ACT, bool SPLIT, bool PIPE, bool FP8 = false,
          int NS = 2, int CONV = 0>
__global__ void __launch_bounds__(WM * WN * 64, 1) gemm_k(GemmArgs p) {
    constexpr int NW = WM * WN;
    constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
    constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / WN, wn = wave % WN;

    const int tiles = p.tiles_m * p.tiles_n;
    int split_id = 0, tm, tn;
    if constexpr (SPLIT) {
        // remap over the WHOLE grid first, then split = id / tiles: an XCD then holds a contiguous
        // run of tiles of the same K-slice, which share A and B panels in its L2 (decomposing
        // blockIdx first scattered a tile group over all XCDs whenever tiles % 8 != 0)
        const int id = xcd_remap(blockIdx.x, tiles * p.split);
        split_id = id / tiles;
        group_tile(id % tiles, p.tiles_m, p.tiles_n, tm, tn);
    } else {
        map_tile(blockIdx.x, tiles, p.tiles_m, p.tiles_n, tm, tn);
    }
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = split_id * p.k_per_split;
    const int kend = min(p.K, kbeg + p.k_per_split);
    const int nk = (kend - kbeg + BK - 1) / BK;

    auto a_base = [&](int k0) -> const bf16* {
        return AK ? p.A + (long)m0 * p.lda + k0 : p.A + (long)k0 * p.lda + m0;
    };
    auto b_base = [&](int k0) -> const bf16* {
        return BK_ ? p.B + (long)n0 * p.ldb + k0 : p.B + (long)k0 * p.ldb + n0;
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    if constexpr (PIPE && NS > 2) {
        // NS-stage ring (NS-1 tiles in flight): the same 4-phase schedule as below, but
        // the DMA of tile kt+NS is issued into tile kt's buffer right after the
        // end-of-tile barrier, and that barrier only waits for tile kt+1 (counted vmcnt),
        // so every tile has NS-1 tile-times to arrive from L2 / HBM.
        constexpr int HM = FM / 2;
        static_assert(FM % 2 == 0, "pipelined loop splits the wave's M fragments in two halves");
        constexpr int OPS = (BM * 128 / 1024) / NW + (BN * 128 / 1024) / NW;  // DMA instr / wave / tile
        static_assert((NS - 1) * OPS <= 63, "vmcnt range");
        auto wait_tiles = [&](int younger) {  // wait until at most `younger` tiles' DMA remain in flight
            if (younger <= 0) vm_wait<0>();
            else if (younger == 1) vm_wait<OPS>();
            else if (younger == 2) vm_wait<2 * OPS>();
            else vm_wait<3 * OPS>();
        };
        auto sync = [&]() {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        };
        auto issue = [&](int t, int buf) {
            const int k0 = kbeg + t * BK;
            char* nb = smem + buf * STAGE;
            if constexpr (CONV == 1 || CONV == 2) {
                stage_conv_a<BM, NW, CONV>(p, m0, k0, kend, nb, wave, lane);
            } else {
                stage_async<AK, BM, NW>(a_base(k0), p.lda, p.M - m0, kend - k0, nb, wave, lane);
            }
            if constexpr (CONV == 3) {
                stage_conv_b<BN, NW>(p, n0, k0, kend, nb + A_BYTES, wave, lane);
            } else if constexpr (CONV == 2) {  // W[co][kh][kw][c] rows of one tap
                const int tap = (int)fdiv((uint32_t)k0, p.cv.fd_kc), co0 = k0 - tap * p.cv.KC;
                stage_async<false, BN, NW>(p.B + (long)co0 * p.cv.bld + (long)tap * p.cv.BC + n0, p.cv.bld,
                                           p.N - n0, kend - k0, nb + A_BYTES, wave, lane);
            } else {
                stage_async<BK_, BN, NW>(b_base(k0), p.ldb, p.N - n0, kend - k0, nb + A_BYTES, wave, lane);
            }
        };
        s16x8 A0[HM], A1[HM], B0[FN], B1[FN];
#define RN_LDA(DST, LA, MH, S)                                                        \
        _Pragma("unroll") for (int i_ = 0; i_ < HM; ++i_)                          \
            DST[i_] = frag<AK>(LA, wm * (BM / WM) + ((MH) * HM + i_) * 16, S, lane);
#define RN_LDB(DST, LB, S)                                                            \
        _Pragma("unroll") for (int j_ = 0; j_ < FN; ++j_)                          \
            DST[j_] = frag<BK_>(LB, wn * (BN / WN) + j_ * 16, S, lane);
#define RN_MMA(A, B, MH)                                                              \
        _Pragma("unroll") for (int i_ = 0; i_ < HM; ++i_)                          \
        _Pragma("unroll") for (int j_ = 0; j_ < FN; ++j_)                          \
            acc[(MH) * HM + i_][j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B[j_], A[i_], acc[(MH) * HM + i_][j_], 0, 0, 0);
        const int npro = min(NS, nk);
        for (int t = 0; t < npro; ++t) issue(t, t);
        wait_tiles(npro - 1);
        sync();
        if (nk > 0) {
            RN_LDA(A0, smem, 0, 0)
            RN_LDB(B0, smem + A_BYTES, 0)
        }
        int cur = 0;
        for (int kt = 0; kt < nk; ++kt) {
            const char* la = smem + cur * STAGE;
            const char* lb = la + A_BYTES;
            _Pragma("unroll") for (int j_ = 0; j_ < FN; ++j_)
                acc[0][j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B0[j_], A0[0], acc[0][j_], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            RN_LDA(A1, la, 1, 0)
            __builtin_amdgcn_sched_barrier(0);
            _Pragma("unroll") for (int i_ = 1; i_ < HM; ++i_)
            _Pragma("unroll") for (int j_ = 0; j_ < FN; ++j_)
                acc[i_][j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B0[j_], A0[i_], acc[i_][j_], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            RN_LDA(A0, la, 0, 1)
            RN_LDB(B1, lb, 1)
            __builtin_amdgcn_sched_barrier(0);
            RN_MMA(A1, B0, 1)
            __builtin_amdgcn_sched_barrier(0);
            RN_LDA(A1, la, 1, 1)
            __builtin_amdgcn_sched_barrier(0);
            RN_MMA(A0, B1, 0)
            __builtin_amdgcn_sched_barrier(0);
            if (kt + 1 < nk) wait_tiles(min(NS - 2, nk - 2 - kt));  // tile kt+1 landed (this wave's DMA)
            sync();  // ... every wave's; every read of buffer `cur` retired
            if (kt + NS < nk) issue(kt + NS, cur);
            const int nxt = cur + 1 == NS ? 0 : cur + 1;
            if (kt + 1 < nk) {
                const char* na = smem + nxt * STAGE;
                RN_LDA(A0, na, 0, 0)
                RN_LDB(B0, na + A_BYTES, 0)
            }
            __builtin_amdgcn_sched_barrier(0);
            RN_MMA(A1, B1, 1)
            __builtin_amdgcn_sched_barrier(0);
            cur = nxt;
        }
#undef RN_LDA
#undef RN_LDB
#undef RN_MMA
        __syncthreads();  // epilogue reuses the LDS ring
    } else if constexpr (PIPE) {
        // Software-pipelined main loop: 4 MFMA phases per K-tile (k-step s × M-half),
        // the fragments of phase i+1 are read from LDS while phase i's MFMAs run,
        // ONE barrier per K-tile (before the last phase) that (a) retires the
        // LDS-DMA of tile kt+1 issued a whole tile earlier and (b) frees buffer
        // kt&1 for the DMA of tile kt+2, after which the first fragments of tile
        // kt+1 are read under the last phase's MFMAs: no LDS-latency bubble at the
        // tile seam.  sched_barrier pins the load-before-MFMA order per phase.
        constexpr int HM = FM / 2;
        static_assert(FM % 2 == 0, "pipelined loop splits the wave's M fragments in two halves");
        s16x8 A0[HM], A1[HM], B0[FN], B1[FN];
#define RN_LDA(DST, LA, MH, S)                                                        \
        _Pragma("unroll") for (int i_ = 0; i_ < HM; ++i_)                          \
            DST[i_] = frag<AK>(LA, wm * (BM / WM) + ((MH) * HM + i_) * 16, S, lane);
#define RN_LDB(DST, LB, S)                                                            \
        _Pragma("unroll") for (int j_ = 0; j_ < FN; ++j_)                          \
            DST[j_] = frag<BK_>(LB, wn * (BN / WN) + j_ * 16, S, lane);
#define RN_MMA(A, B, MH)                                                              \
        _Pragma("unroll") for (int i_ = 0; i_ < HM; ++i_)                          \
        _Pragma("unroll") for (int j_ = 0; j_ < FN; ++j_)                          \
            acc[(MH) * HM + i_][j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B[j_], A[i_], acc[(MH) * HM + i_][j_], 0, 0, 0);
        if (nk > 0) {
            stage<AK, BM, NW>(a_base(kbeg), p.lda, p.M - m0, kend - kbeg, smem, wave, lane);
            stage<BK_, BN, NW>(b_base(kbeg), p.ldb, p.N - n0, kend - kbeg, smem + A_BYTES, wave, lane);
        }
        __syncthreads();
        if (nk > 1) {
            const int k0 = kbeg + BK;
            stage<AK, BM, NW>(a_base(k0), p.lda, p.M - m0, kend - k0, smem + STAGE, wave, lane);
            stage<BK_, BN, NW>(b_base(k0), p.ldb, p.N - n0, kend - k0, smem + STAGE + A_BYTES, wave, lane);
        }
        if (nk > 0) {
            RN_LDA(A0, smem, 0, 0)
            RN_LDB(B0, smem + A_BYTES, 0)
        }
        for (int kt = 0; kt < nk; ++kt) {
            const char* la = smem + (kt & 1) * STAGE;
            const char* lb = la + A_BYTES;
            // phase 0: first MFMA row before issuing the next reads, so the wait the
            // compiler places at the loop head (it cannot count LDS reads across the
            // back-edge) only covers A0/B0, which landed under the previous phase 3
            _Pragma("unroll") for (int j_ = 0; j_ < FN; ++j_)
                acc[0][j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B0[j_], A0[0], acc[0][j_], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            RN_LDA(A1, la, 1, 0)
            __builtin_amdgcn_sched_barrier(0);
            _Pragma("unroll") for (int i_ = 1; i_ < HM; ++i_)
            _Pragma("unroll") for (int j_ = 0; j_ < FN; ++j_)
                acc[i_][j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B0[j_], A0[i_], acc[i_][j_], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            RN_LDA(A0, la, 0, 1)
            RN_LDB(B1, lb, 1)
            __builtin_amdgcn_sched_barrier(0);
            RN_MMA(A1, B0, 1)
            __builtin_amdgcn_sched_barrier(0);
            RN_LDA(A1, la, 1, 1)
            __builtin_amdgcn_sched_barrier(0);
            RN_MMA(A0, B1, 0)
            __builtin_amdgcn_sched_barrier(0);
            __syncthreads();  // all reads of buffer kt&1 retired; tile kt+1 landed (vmcnt(0))
            if (kt + 2 < nk) {
                const int k0 = kbeg + (kt + 2) * BK;
                char* nb = smem + (kt & 1) * STAGE;
                stage<AK, BM, NW>(a_base(k0), p.lda, p.M - m0, kend - k0, nb, wave, lane);
                stage<BK_, BN, NW>(b_base(k0), p.ldb, p.N - n0, kend - k0, nb + A_BYTES, wave, lane);
            }
            if (kt + 1 < nk) {
                const char* na = smem + ((kt + 1) & 1) * STAGE;
                RN_LDA(A0, na, 0, 0)
                RN_LDB(B0, na + A_BYTES, 0)
            }
            __builtin_amdgcn_sched_barrier(0);
            RN_MMA(A1, B1, 1)
            __builtin_amdgcn_sched_barrier(0);
        }
#undef RN_LDA
#undef RN_LDB
#undef RN_MMA
    } else {
    if (nk > 0) {
        stage<AK, BM, NW>(a_base(kbeg), p.lda, p.M - m0, kend - kbeg, smem, wave, lane);
        stage<BK_, BN, NW>(b_base(kbeg), p.ldb, p.N - n0, kend - kbeg, smem + A_BYTES, wave, lane);
    }
    for (int kt = 0; kt < nk; ++kt) {
        __syncthreads();  // vmcnt(0) + barrier: stage kt landed; stage kt-1 fully consumed
        const int cur = kt & 1;
        if (kt + 1 < nk) {
            const int k0 = kbeg + (kt + 1) * BK;
            char* nb = smem + (cur ^ 1) * STAGE;
            stage<AK, BM, NW>(a_base(k0), p.lda, p.M - m0, kend - k0, nb, wave, lane);
            stage<BK_, BN, NW>(b_base(k0), p.ldb, p.N - n0, kend - k0, nb + A_BYTES, wave, lane);
        }
        const char* la = smem + cur * STAGE;
        const char* lb = la + A_BYTES;
        if constexpr (FP8) {
            // one 16x16x128 block-scaled MFMA per fragment pair per 128-deep fp8 K-tile
            // (unit E8M0 block scales; the per-tensor scales enter through alpha)
            i32x8 af[FM], bfr[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) bfr[j] = frag8(lb, wn * (BN / WN) + j * 16, lane);
#pragma unroll
            for (int i = 0; i < FM; ++i) af[i] = frag8(la, wm * (BM / WM) + i * 16, lane);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af[i], acc[i][j], 0, 0, 0,
                                                                                 127, 0, 127);
            continue;
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            s16x8 af[FM], bfr[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) bfr[j] = frag<BK_>(lb, wn * (BN / WN) + j * 16, s, lane);
#pragma unroll
            for (int i = 0; i < FM; ++i) af[i] = frag<AK>(la, wm * (BM / WM) + i * 16, s, lane);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        }
    }
    }

    const float alpha = p.alpha ? *p.alpha : 1.f;

    // ---- LDS-staged epilogue (bf16 output, N % 8 == 0) ----
    // The accumulator layout gives each lane 4 consecutive columns of ONE row, so
    // direct stores write 16 rows × 32 B per wave-instruction.  Instead the tile is
    // staged through LDS (row stride BN*2+16 B: 2-way at worst on the b64 writes)
    // and written back as whole rows, 16 B per lane.  For short-K GEMMs (K = 768) the
    // store tail is otherwise as long as the main loop.
    //   * the one operand the store loop reads (pre-activation for an activation
    //     backward, else the residual, else the accumulate target) is fetched for ALL
    //     of a thread's chunks before the staging barrier: its HBM latency overlaps the
    //     LDS pass instead of being paid once per chunk (a dependent load per 16-B chunk
    //     serialised ITERS round trips per tile);
    //   * an activation forward that also saves the pre-activation stages the
    //     pre-activation once and writes both outputs from it (act of the bf16-rounded
    //     value, the same value the backward differentiates at): one LDS pass, not two.
    if constexpr (!SPLIT) {
        if (!p.out_f32 && (p.N % 8) == 0 && (p.ldc % 8) == 0) {
            constexpr int STRIDE = BN * 2 + 16;
            constexpr int CPR = BN / 8;  // 16-B chunks per tile row
            constexpr int NTH = NW * 64;
            static_assert((BM * CPR) % NTH == 0, "epilogue chunks must divide evenly over the threads");
            constexpr int ITERS = BM * CPR / NTH;
            const int mlim = min(BM, p.M - m0), nlim = min(BN, p.N - n0);
            const bool two_out = act_fwd(ACT) && p.pre != nullptr;
            [[maybe_unused]] float q8max = 0.f;
            [[maybe_unused]] const float q8inv = (act_fwd(ACT) && p.q8) ? 1.f / p.q8st[0] : 0.f;
            const bf16* auxp = act_bwd(ACT) ? p.pre
                               : (p.res ? p.res : (p.accumulate ? (const bf16*)p.C : (const bf16*)nullptr));
            s16x8 aux[ITERS];
            if (auxp) {
#pragma unroll
                for (int it = 0; it < ITERS; ++it) {  // clamped addresses: no per-load branch
                    const int q = threadIdx.x + it * NTH;
                    const int r = min(q / CPR, mlim - 1), cc = min(q % CPR, nlim / 8 - 1);
                    aux[it] = *reinterpret_cast<const s16x8*>(auxp + (long)(m0 + r) * p.ldc + n0 + cc * 8);
                }
            }
            __syncthreads();  // main-loop LDS reads retired
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int ml = wm * (BM / WM) + i * 16 + (lane & 15);
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int nl = wn * (BN / WN) + j * 16 + 4 * (lane >> 4);
                    float v[4] = {acc[i][j][0] * alpha, acc[i][j][1] * alpha, acc[i][j][2] * alpha,
                                  acc[i][j][3] * alpha};
                    if (p.bias && n0 + nl < p.N) {
                        bf16x4 b = *reinterpret_cast<const bf16x4*>(p.bias + n0 + nl);
#pragma unroll
                        for (int t = 0; t < 4; ++t) v[t] += (float)b[t];
                    }
                    if constexpr (act_fwd(ACT)) {
                        if (!two_out) {
#pragma unroll
                            for (int t = 0; t < 4; ++t) v[t] = act_f<ACT>(v[t]);
                        }
                    }
                    bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
                    *reinterpret_cast<bf16x4*>(smem + ml * STRIDE + nl * 2) = o;
                }
            }
            __syncthreads();
            bf16* dst = (bf16*)p.C;
            // column partial sums (act-backward: Σ of the output = a bias gradient; implicit-conv
            // forward: Σ and Σ² of the output = the following BatchNorm's batch statistics): with
            // NT % CPR == 0 every thread always visits the same 8-column chunk, so it sums its rows
            // in registers
            constexpr bool BNSTAT = CONV == 1;
            constexpr bool CSUM_OK = (act_bwd(ACT) || BNSTAT) && colpart_cfg_ok<BN, NTH>();
            float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            [[maybe_unused]] float csq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int it = 0; it < ITERS; ++it) {
                const int q = threadIdx.x + it * NTH;
                const int r = q / CPR, cc = q % CPR;
                if (r >= mlim || cc * 8 >= nlim) continue;
                s16x8 v = *reinterpret_cast<const s16x8*>(smem + r * STRIDE + cc * 16);
                const long goff = (long)(m0 + r) * p.ldc + n0 + cc * 8;
                float f[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) f[t] = (float)__builtin_bit_cast(bf16, (short)v[t]);
                bool changed = false;
                if constexpr (act_fwd(ACT)) {
                    if (two_out) {
                        float pv[8];
#pragma unroll
                        for (int t = 0; t < 8; ++t) f[t] = act_fwd_pre<ACT>(f[t], pv[t]);
                        if constexpr (ACT == ACT_GELU_D) store8(p.pre + goff, pv);
                        else *reinterpret_cast<s16x8*>(p.pre + goff) = v;
                        changed = true;
                        if (p.q8) {  // e4m3 of the stored bf16 values (same bytes as a separate pass)
                            float e[8];
#pragma unroll
                            for (int t = 0; t < 8; ++t) {
                                const float yb = (float)(bf16)f[t];
                                q8max = fmaxf(q8max, fabsf(yb));
                                e[t] = fminf(fmaxf(yb * q8inv, -448.f), 448.f);
                            }
                            int w0 = 0, w1 = 0;
                            w0 = __builtin_amdgcn_cvt_pk_fp8_f32(e[0], e[1], w0, false);
                            w0 = __builtin_amdgcn_cvt_pk_fp8_f32(e[2], e[3], w0, true);
                            w1 = __builtin_amdgcn_cvt_pk_fp8_f32(e[4], e[5], w1, false);
                            w1 = __builtin_amdgcn_cvt_pk_fp8_f32(e[6], e[7], w1, true);
                            *reinterpret_cast<int2*>(p.q8 + goff) = make_int2(w0, w1);
                        }
                    }
                }
                if (!auxp) {  // no residual / accumulate / activation-backward operand
                    if constexpr (BNSTAT && CSUM_OK) {  // statistics of the stored (bf16) values
                        if (!changed) {
#pragma unroll
                            for (int t = 0; t < 8; ++t) {
                                csum[t] += f[t];
                                csq[t] = __builtin_fmaf(f[t], f[t], csq[t]);
                            }
                        }
                    }
                    if (changed) store8(dst + goff, f);
                    else *reinterpret_cast<s16x8*>(dst + goff) = v;
                    continue;
                }
                float ax[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) ax[t] = (float)__builtin_bit_cast(bf16, (short)aux[it][t]);
                if constexpr (act_bwd(ACT)) {  // dH = (dY·W) ⊙ act'(pre)
#pragma unroll
                    for (int t = 0; t < 8; ++t) f[t] = (float)(bf16)f[t] * act_grad_f<ACT>(ax[t]);
                    if constexpr (CSUM_OK) {
#pragma unroll
                        for (int t = 0; t < 8; ++t) csum[t] += (float)(bf16)f[t];  // Σ of stored values
                    }
                } else {
                    // ax holds the residual if there is one, else the accumulate target
#pragma unroll
                    for (int t = 0; t < 8; ++t) f[t] += ax[t];
                    if (p.res && p.accumulate) {
                        float cc8[8];
                        load8(dst + goff, cc8);
#pragma unroll
                        for (int t = 0; t < 8; ++t) f[t] += cc8[t];
                    }
                }
                store8(dst + goff, f);
            }
            if constexpr (act_fwd(ACT)) {
                if (p.q8) {  // block amax -> one atomic (non-negative floats order as ints)
                    float* red = reinterpret_cast<float*>(smem);
                    q8max = wave_max(q8max);
                    __syncthreads();  // staged tile fully read
                    if (lane == 0) red[threadIdx.x >> 6] = q8max;
                    __syncthreads();
                    if (threadIdx.x == 0) {
                        float t = 0.f;
                        for (int w = 0; w < NW; ++w) t = fmaxf(t, red[w]);
                        atomicMax(reinterpret_cast<int*>(p.q8st + 1), __float_as_int(t));
                    }
                }
            }
            if constexpr (CSUM_OK) {
                if (p.colpart) {  // fold the NT/CPR row-groups of each chunk (fixed order)
                    constexpr int RG = NTH / CPR;
                    float* red = reinterpret_cast<float*>(smem);  // [RG][BN]
                    __syncthreads();  // staged tile fully read
                    const int cc = threadIdx.x % CPR, rg = threadIdx.x / CPR;
#pragma unroll
                    for (int t = 0; t < 8; ++t) red[rg * BN + cc * 8 + t] = csum[t];
                    __syncthreads();
                    // act-backward: colpart [tiles_m][N]; conv forward: [tiles_m][2N] = Σ | Σ²
                    const long prow = BNSTAT ? 2L * p.N : (long)p.N;
                    for (int col = threadIdx.x; col < BN; col += NTH) {
                        float tot = 0.f;
                        for (int g2 = 0; g2 < RG; ++g2) tot += red[g2 * BN + col];
                        if (n0 + col < p.N) p.colpart[(long)tm * prow + n0 + col] = tot;
                    }
                    if constexpr (BNSTAT) {
                        __syncthreads();  // first pass of `red` read
#pragma unroll
                        for (int t = 0; t < 8; ++t) red[rg * BN + cc * 8 + t] = csq[t];
                        __syncthreads();
                        for (int col = threadIdx.x; col < BN; col += NTH) {
                            float tot = 0.f;
                            for (int g2 = 0; g2 < RG; ++g2) tot += red[g2 * BN + col];
                            if (n0 + col < p.N) p.colpart[(long)tm * prow + p.N + n0 + col] = tot;
                        }
                    }
                }
            }
            return;
        }
    }

    // ---- direct epilogue: lane owns C[m][n..n+3] for each (i, j) ----
#pragma unroll
    for (int i = 0; i < FM; ++i) {
        const int m = m0 + wm * (BM / WM) + i * 16 + (lane & 15);
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int n = n0 + wn * (BN / WN) + j * 16 + 4 * (lane >> 4);
            if (n >= p.N) continue;
            float v[4] = {acc[i][j][0] * alpha, acc[i][j][1] * alpha, acc[i][j][2] * alpha, acc[i][j][3] * alpha};
            if constexpr (SPLIT) {
                float* w = p.ws + ((long)split_id * p.M + m) * p.N + n;
                if (n + 3 < p.N) *reinterpret_cast<float4*>(w) = make_float4(v[0], v[1], v[2], v[3]);
                else for (int t = 0; t < 4 && n + t < p.N; ++t) w[t] = v[t];
                continue;
            } else {
                const bool full = (n + 3 < p.N);
                if (p.bias) {
                    if (full) {
                        bf16x4 b = *reinterpret_cast<const bf16x4*>(p.bias + n);
#pragma unroll
                        for (int t = 0; t < 4; ++t) v[t] += (float)b[t];
                    } else for (int t = 0; t < 4 && n + t < p.N; ++t) v[t] += (float)p.bias[n + t];
                }
                if constexpr (act_bwd(ACT)) {
                    const bf16* pp = p.pre + (long)m * p.ldc + n;
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        if (n + t < p.N) v[t] = (float)(bf16)v[t] * act_grad_f<ACT>((float)pp[t]);
                }
                if constexpr (act_fwd(ACT)) {
                    float pv[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) v[t] = act_fwd_pre<ACT>(v[t], pv[t]);
                    if (p.pre) {
                        bf16* pp = p.pre + (long)m * p.ldc + n;
                        if (full) {
                            bf16x4 o = {(bf16)pv[0], (bf16)pv[1], (bf16)pv[2], (bf16)pv[3]};
                            *reinterpret_cast<bf16x4*>(pp) = o;
                        } else for (int t = 0; t < 4 && n + t < p.N; ++t) pp[t] = (bf16)pv[t];
                    }
                }
                if (p.res) {
                    const bf16* rp = p.res + (long)m * p.ldc + n;
                    if (full) {
                        bf16x4 r = *reinterpret_cast<const bf16x4*>(rp);
#pragma unroll
                        for (int t = 0; t < 4; ++t) v[t] += (float)r[t];
                    } else for (int t = 0; t < 4 && n + t < p.N; ++t) v[t] += (float)rp[t];
                }
                if (p.out_f32) {
                    float* cp = (float*)p.C + (long)m * p.ldc + n;
                    if (full) {
                        float4 o = make_float4(v[0], v[1], v[2], v[3]);
                        if (p.accumulate) { float4 c = *reinterpret_cast<float4*>(cp); o.x += c.x; o.y += c.y; o.z += c.z; o.w += c.w; }
                        *reinterpret_cast<float4*>(cp) = o;
                    } else for (int t = 0; t < 4 && n + t < p.N; ++t) cp[t] = v[t] + (p.accumulate ? cp[t] : 0.f);
                } else {
                    bf16* cp = (bf16*)p.C + (long)m * p.ldc + n;
                    if (full) {
                        if (p.accumulate) {
                            bf16x4 c = *reinterpret_cast<const bf16x4*>(cp);
#pragma unroll
                            for (int t = 0; t < 4; ++t) v[t] += (float)c[t];
                        }
                        bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
                        *reinterpret_cast<bf16x4*>(cp) = o;
                    } else for (int t = 0; t < 4 && n + t < p.N; ++t) cp[t] = (bf16)(v[t] + (p.accumulate ? (float)cp[t] : 0.f));
                }
            }
        }
    }
}

// Group pre-reduction for a tall slab stack over a small output (e.g. an implicit-conv weight gradient:
// 64 x 576 outputs over up to 256 pixel slabs): the one-pass reduction below would run a few dozen blocks,
// each thread walking every slab in sequence.  Here block (x, g) sums slabs [g·per, min((g+1)·per, S)) of
// its 256 four-column groups in order and writes the sum over slab g·per (read by nobody else); the final
// pass then adds the G group sums in order.  Fixed order throughout: deterministic.
template <int V = 4>  // (a template: this header is compiled into many translation units)
__global__ void __launch_bounds__(256) splitk_group_k(float* __restrict__ ws, long MN, int S, int per) {
    const long q = blockIdx.x * 256L + threadIdx.x;
    const long total4 = MN / 4;
    if (q >= total4) return;
    const int s0 = blockIdx.y * per, s1 = min(S, s0 + per);
    float4 acc = reinterpret_cast<const float4*>(ws + (long)s0 * MN)[q];
    for (int s = s0 + 1; s < s1; ++s) {
        const float4 t = reinterpret_cast<const float4*>(ws + (long)s * MN)[q];
        acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
    }
    reinterpret_cast<float4*>(ws + (long)s0 * MN)[q] = acc;
}

// Sum split-K slabs (fixed order) + epilogue.  4 consecutive columns per thread.
// BATCH: the slab loads are issued 4 at a time before their (in-order) adds, so a thread has 4
// loads in flight instead of one dependent load per slab — same summation order, same bits
template <int ACT>
__global__ void __launch_bounds__(256) splitk_reduce_k(GemmArgs p) {
    const long total4 = ((long)p.M * p.N + 3) / 4;
    const float ra = p.reduce_alpha ? *p.reduce_alpha : 1.f;
    for (long q = blockIdx.x * 256L + threadIdx.x; q < total4; q += (long)gridDim.x * 256) {
        const long e0 = q * 4;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        const long MN = (long)p.M * p.N;
        const bool vec = (p.N % 4 == 0);
        const long step = p.slab_step > 1 ? (long)p.slab_step * MN : MN;
        int s0 = 0;
        if (vec) {
            for (; s0 + 4 <= p.split; s0 += 4) {
                float4 t[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) t[u] = *reinterpret_cast<const float4*>(p.ws + (s0 + u) * step + e0);
#pragma unroll
                for (int u = 0; u < 4; ++u) { v[0] += t[u].x; v[1] += t[u].y; v[2] += t[u].z; v[3] += t[u].w; }
            }
        }
        for (int s = s0; s < p.split; ++s) {
            const float* w = p.ws + s * step + e0;
            if (vec) { float4 t = *reinterpret_cast<const float4*>(w); v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w; }
            else for (int t = 0; t < 4 && e0 + t < MN; ++t) v[t] += w[t];
        }
        for (int t = 0; t < 4; ++t) {
            const long e = e0 + t;
            if (e >= MN) break;
            const int m = e / p.N, n = e % p.N;
            float x = v[t];
            if (p.reduce_alpha) x *= ra;
            if (p.bias) x += (float)p.bias[n];
            if constexpr (act_fwd(ACT)) {
                float pv;
                x = act_fwd_pre<ACT>(x, pv);
                if (p.pre) p.pre[(long)m * p.ldc + n] = (bf16)pv;
            }
            if constexpr (act_bwd(ACT)) x = (float)(bf16)x * act_grad_f<ACT>((float)p.pre[(long)m * p.ldc + n]);
            if (p.res) x += (float)p.res[(long)m * p.ldc + n];
            if (p.out_f32) {
                float* cp = (float*)p.C + (long)m * p.ldc + n;
                *cp = x + (p.accumulate ? *cp : 0.f);
            } else {
                bf16* cp = (bf16*)p.C + (long)m * p.ldc + n;
                *cp = (bf16)(x + (p.accumulate ? (float)*cp : 0.f));
            }
        }
    }
}

// true the first time `mask`'s owner launches on the current device (the >64 KiB LDS opt-in
// attribute is per device; a process may drive several GPUs)
inline bool first_on_device(uint64_t& mask) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    const uint64_t bit = 1ull << (dev & 63);
    if (mask & bit) return false;
    mask |= bit;
    return true;
}

template <int BM, int BN, int WM, int WN, bool PIPE, bool AK, bool BK_, int ACT, int NS = 2, int CONV = 0>
void launch_t(GemmArgs& a, hipStream_t st) {
    constexpr int NT = WM * WN * 64;
    const size_t lds = std::max<size_t>((size_t)NS * (BM + BN) * BK * 2, (size_t)BM * (BN * 2 + 16));
    static_assert((size_t)NS * (BM + BN) * BK * 2 <= 163840, "LDS ring exceeds 160 KiB");
    static_assert(CONV == 0 || (PIPE && NS > 2), "implicit-GEMM conv loaders live in the NS-stage path");
    auto kmain = gemm_k<BM, BN, WM, WN, AK, BK_, ACT, false, PIPE, false, NS, CONV>;
    auto ksplit = gemm_k<BM, BN, WM, WN, AK, BK_, ACT_NONE, true, PIPE, false, NS, CONV>;
    static uint64_t attr_devs = 0;  // devices this instantiation opted in on
    if (first_on_device(attr_devs)) {  // >64 KiB of dynamic LDS must be opted into, per instantiation and device
        (void)hipFuncSetAttribute((const void*)kmain, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void*)ksplit, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    const int tiles = a.tiles_m * a.tiles_n;
    if (a.split > 1) {
        ksplit<<<tiles * a.split, NT, lds, st>>>(a);
        long total4 = ((long)a.M * a.N + 3) / 4;
        int g = (int)std::min<long>((total4 + 255) / 256, 4096);
        const long MN = (long)a.M * a.N;
        if (a.split >= 16 && g < 256 && MN % 4 == 0) {  // tall stack, small output: pre-reduce in groups
            const int G = 16, per = (a.split + G - 1) / G;
            splitk_group_k<><<<dim3(g, (a.split + per - 1) / per), 256, 0, st>>>(a.ws, MN, a.split, per);
            GemmArgs r = a;
            r.split = (a.split + per - 1) / per;
            r.slab_step = per;
            splitk_reduce_k<ACT><<<g, 256, 0, st>>>(r);
        } else {
            splitk_reduce_k<ACT><<<g, 256, 0, st>>>(a);
        }
    } else {
        kmain<<<tiles, NT, lds, st>>>(a);
    }
}

template <int BM, int BN, int WM, int WN, bool PIPE, int NS = 2>
void launch_cfg(GemmArgs& a, bool ak, bool bk, int act, hipStream_t st) {
    a.tiles_m = (a.M + BM - 1) / BM;
    a.tiles_n = (a.N + BN - 1) / BN;
#define RN_L(AKv, BKv)                                                                             \
    if (act == ACT_GELU) launch_t<BM, BN, WM, WN, PIPE, AKv, BKv, ACT_GELU, NS>(a, st);           \
    else if (act == ACT_RELU) launch_t<BM, BN, WM, WN, PIPE, AKv, BKv, ACT_RELU, NS>(a, st);      \
    else launch_t<BM, BN, WM, WN, PIPE, AKv, BKv, ACT_NONE, NS>(a, st);
    if (ak && bk) {
        if (act == ACT_GELU_D) launch_t<BM, BN, WM, WN, PIPE, true, true, ACT_GELU_D, NS>(a, st);
        else { RN_L(true, true) }
    }
    else if (ak && !bk) {  // dgrad layout: also the fused activation-backward epilogues
        if (act == ACT_GELU_BWD) launch_t<BM, BN, WM, WN, PIPE, true, false, ACT_GELU_BWD, NS>(a, st);
        else if (act == ACT_MUL_BWD) launch_t<BM, BN, WM, WN, PIPE, true, false, ACT_MUL_BWD, NS>(a, st);
        else if (act == ACT_RELU_BWD) launch_t<BM, BN, WM, WN, PIPE, true, false, ACT_RELU_BWD, NS>(a, st);
        else { RN_L(true, false) }
    }
    else if (!ak && bk) { RN_L(false, true) }
    else { RN_L(false, false) }
#undef RN_L
}

// fp8 e4m3 NT GEMM (both operands K-contiguous): staged as "bf16 pairs", so the
// caller passes K, lda, ldb in units of 2 bytes.
template <int BM, int BN, int WM, int WN, int ACT>
void launch_fp8_t(GemmArgs& a, hipStream_t st) {
    constexpr int NT = WM * WN * 64;
    const size_t lds = std::max<size_t>(2 * (BM + BN) * BK * 2, (size_t)BM * (BN * 2 + 16));
    auto kmain = gemm_k<BM, BN, WM, WN, true, true, ACT, false, false, true>;
    static uint64_t attr_devs = 0;
    if (first_on_device(attr_devs))
        (void)hipFuncSetAttribute((const void*)kmain, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    a.tiles_m = (a.M + BM - 1) / BM;
    a.tiles_n = (a.N + BN - 1) / BN;
    kmain<<<a.tiles_m * a.tiles_n, NT, lds, st>>>(a);
}

}  // namespace rn_gemm_detail
