// bf16 GEMM on CDNA4 MFMA (N2):  C = act(op(A)·op(B) + bias) + residual
//
// Block tile 128×128×64, 256 threads = 4 waves (2×2), each wave 64×64 =
// 4×4 tiles of v_mfma_f32_16x16x32_bf16 (fp32 accumulators).
//
// Operand staging: buffer_load_dwordx4 … lds (LDS-DMA, 1 KiB per
// wave-instruction, no VGPR round trip) into a double-buffered LDS image; the
// buffer descriptor's range check zero-fills out-of-range rows/columns, so
// M/N/K tails need no separate code path (K must be a multiple of 8).
//
// Two LDS images, chosen per operand at compile time:
//   K-contiguous operand ([mn][k] in HBM): image [128 mn][64 k] (128-B rows),
//     16-B chunk c of row r stored at chunk c ^ ((r>>1)&7); fragments read with
//     ds_read_b128 (conflict-light).
//   MN-contiguous operand ([k][mn] in HBM, i.e. a transposed use): image
//     [64 k][128 mn] (256-B rows), chunk c of row k stored at c ^ f(k),
//     f(k) = ((k&3) | ((k>>3)&1)<<2) << 1, and fragments read with the
//     ds_read_b64_tr_b16 hardware transpose: each 32-lane half touches 8 rows
//     with 8 distinct even XORs → all 64 banks, conflict-free.
// The XOR is applied on the per-lane GLOBAL source address (the DMA
// destination is lane-linear) and again on the read address.
// So forward (x·Wᵀ: both K-contiguous), dgrad (dY·W: B MN-contiguous) and wgrad
// (dYᵀ·X: both MN-contiguous) run on one kernel with no HBM transposes.
//
// Output orientation is swapped (mfma(Bfrag, Afrag)): each lane owns 4
// consecutive N-columns of one M-row, so the epilogue stores 8-byte bf16x4
// vectors and reads bias/residual likewise.  Epilogue fuses bias, ReLU/GELU
// (optionally saving the pre-activation), residual add, fp32 or bf16 output,
// and accumulate-into-output.
//
// Split-K (for wgrad with few output tiles): each split writes an fp32 slab,
// a reduce kernel sums the slabs in fixed order and applies the epilogue
// (deterministic, no atomics).
//
// Block→tile mapping is XCD-aware: the round-robin dispatcher puts blocks b
// and b+8 on one XCD, so block ids are remapped (bijectively) to give each
// XCD a contiguous run of tiles, walked in GROUP_M-row groups for L2 reuse.
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand per stage
constexpr int GROUP_M = 8;

typedef __attribute__((address_space(3))) void lds_void;

struct GemmArgs {
    const bf16* A;
    const bf16* B;
    void* C;
    const bf16* bias;
    const bf16* res;
    bf16* pre;
    float* ws;
    int M, N, K;
    long lda, ldb, ldc;
    int tiles_m, tiles_n, split, k_per_split;
    int out_f32, accumulate;
};

RN_DEV int swz_kc(int r) { return (r >> 1) & 7; }
RN_DEV int swz_mn(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

// Stage one 128(mn)×64(k) operand tile into LDS.
//   KC:  global element (mn, k) at base[mn*ld + k]
//   !KC: global element (mn, k) at base[k*ld + mn]
template <bool KC>
RN_DEV void stage(const bf16* base, long ld, int mn_lim, int k_lim, char* lds, int wave, int lane) {
    // readfirstlane keeps the descriptor provably wave-uniform (no waterfall loops)
    const uint64_t bp = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32));
    void* ub = (void*)(((uint64_t)hi << 32) | lo);
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(ub, 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int ins = wave * 4 + i;
        uint32_t voff;
        if constexpr (KC) {
            const int r = ins * 8 + (lane >> 3);
            const int cg = (lane & 7) ^ swz_kc(r);
            const int k = cg * 8;
            const bool ok = (r < mn_lim) && (k < k_lim);
            voff = ok ? (uint32_t)(((long)r * ld + k) * 2) : 0xFFFFFFF0u;
        } else {
            const int r = ins * 4 + (lane >> 4);
            const int cg = (lane & 15) ^ swz_mn(r);
            const int mn = cg * 8;
            const bool ok = (r < k_lim) && (mn < mn_lim);
            voff = ok ? (uint32_t)(((long)r * ld + mn) * 2) : 0xFFFFFFF0u;
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + ins * 1024), 16, voff, 0, 0, 0);
    }
}

// fragment: 8 consecutive k (k-step s: k = s*32 + 8*(lane>>4) + 0..7) of row/col
// `mn` (0..127 within the tile) for lane's (lane & 15).
template <bool KC>
RN_DEV s16x8 frag(const char* lds, int mnbase, int s, int lane) {
    if constexpr (KC) {
        const int row = mnbase + (lane & 15);
        const int chunk = s * 4 + (lane >> 4);
        return *reinterpret_cast<const s16x8*>(lds + row * 128 + ((chunk ^ swz_kc(row)) << 4));
    } else {
        const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
        const int c = (mnbase >> 3) + (p >> 1);
        const int k0 = s * 32 + 8 * g + q;
        const int k1 = k0 + 4;
        const char* a0 = lds + k0 * 256 + ((c ^ swz_mn(k0)) << 4) + (p & 1) * 8;
        const char* a1 = lds + k1 * 256 + ((c ^ swz_mn(k1)) << 4) + (p & 1) * 8;
        s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
        s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
        s16x8 r;
        r[0] = v0[0]; r[1] = v0[1]; r[2] = v0[2]; r[3] = v0[3];
        r[4] = v1[0]; r[5] = v1[1]; r[6] = v1[2]; r[7] = v1[3];
        return r;
    }
}

RN_DEV void map_tile(int bid, int nblocks, int tiles_m, int tiles_n, int& tm, int& tn) {
    // XCD remap (bijective for any nblocks): blocks sharing bid%8 get a contiguous id range
    const int xcd = bid & 7, loc = bid >> 3;
    const int q = nblocks >> 3, r = nblocks & 7;
    const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    // grouped ordering: GROUP_M tile-rows share B panels
    const int per_group = GROUP_M * tiles_n;
    const int gid = id / per_group;
    const int first_m = gid * GROUP_M;
    const int gsz = min(tiles_m - first_m, GROUP_M);
    const int in = id % per_group;
    tm = first_m + in % gsz;
    tn = in / gsz;
}

template <bool AK, bool BK_, int ACT, bool SPLIT>
__global__ void __launch_bounds__(NT, 2) gemm_k(GemmArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;

    const int tiles = p.tiles_m * p.tiles_n;
    const int split_id = SPLIT ? blockIdx.x / tiles : 0;
    const int tb = SPLIT ? blockIdx.x % tiles : blockIdx.x;
    int tm, tn;
    map_tile(tb, tiles, p.tiles_m, p.tiles_n, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = split_id * p.k_per_split;
    const int kend = min(p.K, kbeg + p.k_per_split);
    const int nk = (kend - kbeg + BK - 1) / BK;

#define bufA(i) (smem + (i) * 2 * TILE_BYTES)
#define bufB(i) (smem + TILE_BYTES + (i) * 2 * TILE_BYTES)

    auto a_base = [&](int k0) -> const bf16* {
        return AK ? p.A + (long)m0 * p.lda + k0 : p.A + (long)k0 * p.lda + m0;
    };
    auto b_base = [&](int k0) -> const bf16* {
        return BK_ ? p.B + (long)n0 * p.ldb + k0 : p.B + (long)k0 * p.ldb + n0;
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    if (nk > 0) {
        stage<AK>(a_base(kbeg), p.lda, p.M - m0, kend - kbeg, bufA(0), wave, lane);
        stage<BK_>(b_base(kbeg), p.ldb, p.N - n0, kend - kbeg, bufB(0), wave, lane);
    }
    for (int kt = 0; kt < nk; ++kt) {
        __syncthreads();  // vmcnt(0) + barrier: stage kt landed; stage kt-1 fully consumed
        const int cur = kt & 1;
        if (kt + 1 < nk) {
            const int k0 = kbeg + (kt + 1) * BK;
            stage<AK>(a_base(k0), p.lda, p.M - m0, kend - k0, bufA(cur ^ 1), wave, lane);
            stage<BK_>(b_base(k0), p.ldb, p.N - n0, kend - k0, bufB(cur ^ 1), wave, lane);
        }
        const char* la = bufA(cur);
        const char* lb = bufB(cur);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            s16x8 af[4], bfr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = frag<AK>(la, wm * 64 + i * 16, s, lane);
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[j] = frag<BK_>(lb, wn * 64 + j * 16, s, lane);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        }
    }

    // ---- epilogue: lane owns C[m][n..n+3] for each (i, j) ----
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 64 + i * 16 + (lane & 15);
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
            if (n >= p.N) continue;
            float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
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
                if constexpr (ACT != ACT_NONE) {
                    if (p.pre) {
                        bf16* pp = p.pre + (long)m * p.ldc + n;
                        if (full) {
                            bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
                            *reinterpret_cast<bf16x4*>(pp) = o;
                        } else for (int t = 0; t < 4 && n + t < p.N; ++t) pp[t] = (bf16)v[t];
                    }
#pragma unroll
                    for (int t = 0; t < 4; ++t) v[t] = act_f<ACT>(v[t]);
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

// Sum split-K slabs (fixed order) + epilogue.  4 consecutive columns per thread.
template <int ACT>
__global__ void __launch_bounds__(256) splitk_reduce_k(GemmArgs p) {
    const long total4 = ((long)p.M * p.N + 3) / 4;
    for (long q = blockIdx.x * 256L + threadIdx.x; q < total4; q += (long)gridDim.x * 256) {
        const long e0 = q * 4;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        const long MN = (long)p.M * p.N;
        const bool vec = (p.N % 4 == 0);
        for (int s = 0; s < p.split; ++s) {
            const float* w = p.ws + s * MN + e0;
            if (vec) { float4 t = *reinterpret_cast<const float4*>(w); v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w; }
            else for (int t = 0; t < 4 && e0 + t < MN; ++t) v[t] += w[t];
        }
        for (int t = 0; t < 4; ++t) {
            const long e = e0 + t;
            if (e >= MN) break;
            const int m = e / p.N, n = e % p.N;
            float x = v[t];
            if (p.bias) x += (float)p.bias[n];
            if constexpr (ACT != ACT_NONE) {
                if (p.pre) p.pre[(long)m * p.ldc + n] = (bf16)x;
                x = act_f<ACT>(x);
            }
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

template <bool AK, bool BK_, int ACT>
void launch_t(GemmArgs& a, hipStream_t st) {
    const int tiles = a.tiles_m * a.tiles_n;
    const size_t lds = 4 * TILE_BYTES;
    if (a.split > 1) {
        gemm_k<AK, BK_, ACT_NONE, true><<<tiles * a.split, NT, lds, st>>>(a);
        long total4 = ((long)a.M * a.N + 3) / 4;
        int g = (int)std::min<long>((total4 + 255) / 256, 4096);
        splitk_reduce_k<ACT><<<g, 256, 0, st>>>(a);
    } else {
        gemm_k<AK, BK_, ACT, false><<<tiles, NT, lds, st>>>(a);
    }
}

template <bool AK, bool BK_>
void launch_l(GemmArgs& a, int act, hipStream_t st) {
    if (act == ACT_GELU) launch_t<AK, BK_, ACT_GELU>(a, st);
    else if (act == ACT_RELU) launch_t<AK, BK_, ACT_RELU>(a, st);
    else launch_t<AK, BK_, ACT_NONE>(a, st);
}

}  // namespace

extern "C" {

// Workspace floats needed for a split-K launch.
long rn_gemm_ws_floats(int M, int N, int split) { return split > 1 ? (long)split * M * N : 0; }

// C[M,N] = act(op(A)[M,K] · op(B)[K,N] + bias) + res.
//   trans_a = 0: A stored [M][lda] (K contiguous);   1: A stored [K][lda] (M contiguous)
//   trans_b = 0: B stored [K][ldb] (N contiguous);   1: B stored [N][ldb] (K contiguous)
// Returns 0, or -1 if the shape violates the kernel's alignment rules.
int rn_gemm(const void* A, const void* B, void* C, const void* bias, const void* res, void* pre, float* ws, int M,
            int N, int K, long lda, long ldb, long ldc, int trans_a, int trans_b, int act, int split, int out_f32,
            int accumulate, hipStream_t st) {
    if (K % 8 != 0) return -1;
    if (trans_a && (M % 8 != 0 || lda % 8 != 0)) return -1;
    if (!trans_a && lda % 8 != 0) return -1;
    if (!trans_b && (N % 8 != 0 || ldb % 8 != 0)) return -1;
    if (trans_b && ldb % 8 != 0) return -1;
    static bool attr_done = false;
    if (!attr_done) {
        attr_done = true;  // 64 KiB dynamic LDS is below the default limit on gfx950; nothing to raise
    }
    GemmArgs a;
    a.A = (const bf16*)A; a.B = (const bf16*)B; a.C = C; a.bias = (const bf16*)bias; a.res = (const bf16*)res;
    a.pre = (bf16*)pre; a.ws = ws; a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
    a.tiles_m = (M + BM - 1) / BM; a.tiles_n = (N + BN - 1) / BN;
    a.split = split < 1 ? 1 : split;
    int kps = (K + a.split - 1) / a.split;
    kps = (kps + BK - 1) / BK * BK;
    a.k_per_split = kps;
    a.split = (K + kps - 1) / kps;
    a.out_f32 = out_f32; a.accumulate = accumulate;
    const bool ak = !trans_a, bk = trans_b;
    if (ak && bk) launch_l<true, true>(a, act, st);
    else if (ak && !bk) launch_l<true, false>(a, act, st);
    else if (!ak && bk) launch_l<false, true>(a, act, st);
    else launch_l<false, false>(a, act, st);
    return 0;
}

}  // extern "C"
