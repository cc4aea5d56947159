// bf16 GEMM on CDNA4 MFMA (N2):  C = act(op(A)·op(B) + bias) + residual
//
// Block tiles (chosen per shape on the host): 256×256×64 with 8 waves (2×4,
// each wave 128×64 = 8×4 v_mfma_f32_16x16x32_bf16 tiles, 1 block/CU, 128 KiB
// LDS), 256×128 / 128×256 with 8 waves (4×2 / 2×4, 64×64 per wave) and
// 128×128 with 4 waves (2 blocks/CU).  Bigger tiles halve the L2→LDS bytes per
// FLOP: a 128² tile at BK=64 needs ~64 B/clk/CU at the MFMA rate (≈ the whole
// L2 bandwidth), a 256² tile ~32 B/clk/CU.
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
#include <atomic>
#include <cstdlib>
#include <cstdio>
#include <mutex>

#include "common.h"

#include "gemm_pk.h"

using rn_gemm_detail::GemmArgs;
using rn_gemm_detail::BK;

void rn_gemm_launch_cfg0(GemmArgs&, bool, bool, int, hipStream_t);
int rn_gemm_launch_w1(GemmArgs& a, int fp8, int act, hipStream_t st, bool bmn);  // gemm_w1.hip (cfg 11)
void rn_gemm_launch_cfg1(GemmArgs&, bool, bool, int, hipStream_t);
void rn_gemm_launch_cfg2(GemmArgs&, bool, bool, int, hipStream_t);
void rn_gemm_launch_cfg3(GemmArgs&, bool, bool, int, hipStream_t);
void rn_gemm_launch_cfg4(GemmArgs&, bool, bool, int, hipStream_t);
void rn_gemm_launch_cfg5(GemmArgs&, bool, bool, int, hipStream_t);
void rn_gemm_launch_cfg6(GemmArgs&, bool, bool, int, hipStream_t);
void rn_gemm_launch_cfg8(GemmArgs&, bool, bool, int, hipStream_t);
void rn_gemm_launch_pk_tt(GemmArgs&, int, hipStream_t);
void rn_gemm_launch_pk_tf(GemmArgs&, int, hipStream_t);
void rn_gemm_launch_pk_ff(GemmArgs&, int, hipStream_t);
void rn_gemm_launch_pk_ft(GemmArgs&, int, hipStream_t);
#ifdef REPLICANN_DEV
int rn_gemm_launch_pk_dbg(GemmArgs&, bool, bool, int, hipStream_t);
#endif

namespace {

inline long ntiles(int M, int N, int bm, int bn) { return (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn); }

// Tile-config / split-K chooser: a wave-quantisation cost model calibrated on
// MI355X measurements of this kernel (scripts/microbench.py).  A 128² block runs
// 2 per CU, a 256² block 1 per CU and ~13 % faster per FLOP (half the L2→LDS
// bytes per FLOP); a launch takes ceil(tiles / resident slots) rounds.
struct Choice { int cfg, split; };

inline bool pk_ok(int N, long ldc, int out_f32, int act) {
    return N % 8 == 0 && ldc % 8 == 0 && !(out_f32 && act != ACT_NONE);
}

inline Choice pick(int M, int N, int K, int split_req) {
    const double flop_s_cu = 2.9e12;  // effective per-CU bf16 rate of the 128² config
    // candidates: cfg id, BM, BN, resident blocks (slots), relative per-CU rate
    const int cid[4] = {0, 1, 6, 2};
    const int bm[4] = {128, 256, 256, 256}, bn[4] = {128, 256, 192, 128}, slots[4] = {512, 256, 256, 256};
    const double rate[4] = {1.0, 1.16, 1.0, 0.9};
    Choice best = {0, 1};
    double best_t = 1e30;
    for (int c = 0; c < 4; ++c) {
        for (int sp = 1; sp <= 32; sp *= 2) {
            if (split_req > 0 && sp != split_req) continue;
            if (split_req <= 0 && sp > 1 && K / sp < 512) break;
            // split-K only when the unsplit grid cannot fill the resident slots
            if (split_req <= 0 && sp > 1 && ntiles(M, N, bm[c], bn[c]) >= slots[c]) break;
            const int kps = ((K + sp - 1) / sp + 63) / 64 * 64;
            const long tiles = ntiles(M, N, bm[c], bn[c]) * sp;
            const long rounds = (tiles + slots[c] - 1) / slots[c];
            const double per_block = 2.0 * bm[c] * bn[c] * kps / (flop_s_cu * rate[c]) * (c == 0 ? 2.0 : 1.0);
            double t = rounds * per_block + 2.5e-6;  // + prologue/epilogue per launch
            if (sp > 1) t += ((double)M * N * (4.0 * sp + 2.0)) / 4.0e12 + 3e-6;
            if (t < best_t * 0.98) { best_t = t; best = {cid[c], sp}; }
        }
    }
    return best;
}
}  // namespace

extern "C" {

// ---- persistent-GEMM schedule knobs (gemm_pk.h) ----
// sched: 1 = dynamic tile queue, 0 = static walk (default: the queue costs 3-12 % per GEMM on an
// otherwise idle GPU, profiles/gemm_sched_proxy_r3f.txt; REPLICANN_GEMM_SCHED=dynamic turns it on
// for the process, =overlap lets the data-parallel reducer turn it on while collectives are in
// flight).  reserve: CUs a cfg-9 launch leaves free for a concurrent collective.  Host-side
// state read at launch (captured graphs keep the values of their capture).
static std::atomic<int> g_sched{-1};
static std::atomic<int> g_reserve{0};
void rn_gemm_set_sched(int m) { g_sched = m ? 1 : 0; }
int rn_gemm_get_sched() {
    int v = g_sched.load();
    if (v < 0) {  // REPLICANN_GEMM_SCHED=dynamic|static: the process-wide initial setting
        const char* e = std::getenv("REPLICANN_GEMM_SCHED");
        v = (e && e[0] == 'd') ? 1 : 0;
        g_sched = v;
    }
    return v;
}
void rn_gemm_set_reserve(int r) { g_reserve = r < 0 ? 0 : (r > 128 ? 128 : r & ~7); }
int rn_gemm_get_reserve() { return g_reserve.load(); }

// Counter slots of the dynamic schedule: a per-device pool of self-resetting counter blocks
// (PK_SCHED_INTS ints each).  A slot must never be used by two launches that can run at the same
// time, so slots are keyed by stream:
//   * eager launches: each stream gets its own block of kSlotsPerStream slots, used round robin
//     (launches on one stream are ordered, and a launch leaves its slot zeroed); at most
//     kEagerStreams streams per device, further streams take the static walk;
//   * launches recorded into a graph (stream capture): a slot of their own, never handed out again
//     (a replay can run beside eager work or another graph); once that part of the pool is used
//     up, captured launches take the static walk.
constexpr int kSchedSlots = 256;
constexpr int kSlotsPerStream = 16;
constexpr int kEagerStreams = 8;  // slots [0, 128): eager; [128, 256): captured launches
static std::mutex g_pool_mu;
static int* g_pool[64] = {};
struct SlotState {
    hipStream_t streams[kEagerStreams] = {};
    unsigned next[kEagerStreams] = {};
    int n_streams = 0;
    int next_captured = kSlotsPerStream * kEagerStreams;
    bool warned = false;
};
static SlotState g_slots[64];
int rn_gemm_sched_init(int dev) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (dev < 0 || dev >= 64) return -1;
    if (g_pool[dev]) return 0;
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (cur != dev) (void)hipSetDevice(dev);
    int* p = nullptr;
    const size_t bytes = (size_t)kSchedSlots * rn_gemm_detail::PK_SCHED_INTS * sizeof(int);
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) e = hipMemset(p, 0, bytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (cur != dev) (void)hipSetDevice(cur);
    if (e != hipSuccess) return -1;
    g_pool[dev] = p;
    return 0;
}
int* rn_gemm_sched_slot(int dev, hipStream_t st) {
    if (rn_gemm_get_sched() == 0 || dev < 0 || dev >= 64) return nullptr;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cap);
    const bool capturing = cap != hipStreamCaptureStatusNone;
    if (!g_pool[dev] && (capturing || rn_gemm_sched_init(dev) != 0)) return nullptr;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    SlotState& ss = g_slots[dev];
    int s = -1;
    if (capturing) {
        if (ss.next_captured < kSchedSlots) {
            s = ss.next_captured++;
        } else if (!ss.warned) {  // captured slots are never handed back (a replay may run any time)
            ss.warned = true;
            std::fprintf(stderr, "[replicann] gemm: the captured dynamic-schedule slots of device %d are used up; "
                                 "further captured GEMMs take the static tile walk\n", dev);
        }
    } else {
        int k = 0;
        while (k < ss.n_streams && ss.streams[k] != st) ++k;
        if (k == ss.n_streams && ss.n_streams < kEagerStreams) ss.streams[ss.n_streams++] = st;
        if (k < ss.n_streams) s = k * kSlotsPerStream + (int)(ss.next[k]++ % kSlotsPerStream);
    }
    return s < 0 ? nullptr : g_pool[dev] + (size_t)s * rn_gemm_detail::PK_SCHED_INTS;
}

// Workspace floats needed for a split-K launch.
long rn_gemm_ws_floats(int M, int N, int split) { return split > 1 ? (long)split * M * N : 0; }

// C[M,N] = act(alpha · op(A)[M,K] · op(B)[K,N] + bias) + res.
//   trans_a = 0: A stored [M][lda] (K contiguous);   1: A stored [K][lda] (M contiguous)
//   trans_b = 0: B stored [K][ldb] (N contiguous);   1: B stored [N][ldb] (K contiguous)
//   cfg: -1 auto, 0 = 128x128, 1 = 256x256 pipelined, 2 = 256x128 pipelined, 3 = 128x256,
//        4 = 256x256 simple, 5 = 128x128 pipelined, 6 = 256x192 pipelined, 8 = 256x128 3-stage ring,
//        9 = persistent 256x256 half-tile stream (gemm_pk.h; needs N % 8 == 0, ldc % 8 == 0)
//        10 = skinny-M forward GEMM for decoding (gemm_skinny.hip; M <= 64, x·Wᵀ layout, split = K ranges),
//        (7 is the vendor-library candidate handled in the bindings, off by default);
//        split: -1 auto, 0/1 none
// Returns 0, or -1 if the shape violates the kernel's alignment rules.
// colpart (optional, act-backward only): [ceil(M / BM)][N] fp32 per-M-tile column sums of C
// (BM of the config actually used: rn_gemm_cfg_bm).  Returns -3 if the requested config /
// split cannot produce them (the caller then reduces C itself).
int rn_gemm_cfg_bm(int cfg) { return (cfg == 0 || cfg == 3 || cfg == 5 || cfg == 9) ? 128 : 256; }
// rows of the column-partial matrix a config writes (cfg 9: one row per (256-row tile, wave row))
long rn_gemm_colpart_rows(int cfg, int M) {
    return (cfg == 9) ? 2L * ((M + 255) / 256) : (long)((M + rn_gemm_cfg_bm(cfg) - 1) / rn_gemm_cfg_bm(cfg));
}

int rn_gemm_skinny(const void* A, const void* W, void* C, const void* bias, const void* res, void* pre, float* ws,
                   const float* alpha, int M, int N, int K, long lda, long ldw, long ldc, int trans_a, int trans_b,
                   int act, int split, int out_f32, int accumulate, const float* colpart, hipStream_t st);

int rn_gemm(const void* A, const void* B, void* C, const void* bias, const void* res, void* pre, float* ws,
            const float* alpha, int M, int N, int K, long lda, long ldb, long ldc, int trans_a, int trans_b, int act,
            int split, int out_f32, int accumulate, int cfg, hipStream_t st, float* colpart) {
    if (K % 8 != 0) return -1;
    if (cfg == 10)  // skinny-M decode GEMM (gemm_skinny.hip): its own N x K decomposition
        return rn_gemm_skinny(A, B, C, bias, res, pre, ws, alpha, M, N, K, lda, ldb, ldc, trans_a, trans_b, act,
                              split, out_f32, accumulate, colpart, st);
    if (act_bwd(act) && (trans_a || trans_b || !pre)) return -1;  // fused act-backward: dgrad layout only
    if (trans_a && (M % 8 != 0 || lda % 8 != 0)) return -1;
    if (!trans_a && lda % 8 != 0) return -1;
    if (!trans_b && (N % 8 != 0 || ldb % 8 != 0)) return -1;
    if (trans_b && ldb % 8 != 0) return -1;
    if (cfg == 11) {  // one-wave-per-SIMD persistent kernel (gemm_w1.h): x·Wᵀ, plain / bias epilogue
        if (!trans_a && act == ACT_NONE && !accumulate && !out_f32 && split <= 1 && !colpart) {
            GemmArgs w = {};
            w.A = (const bf16*)A; w.B = (const bf16*)B; w.C = C; w.bias = (const bf16*)bias; w.alpha = alpha;
            w.res = (const bf16*)res;
            w.M = M; w.N = N; w.K = K * 2; w.lda = lda * 2; w.ldb = ldb * 2; w.ldc = ldc;
            if (rn_gemm_launch_w1(w, 0, act, st, !trans_b) == 0) return 0;
        }
        cfg = 9;
    }
    GemmArgs a = {};
    a.A = (const bf16*)A; a.B = (const bf16*)B; a.C = C; a.bias = (const bf16*)bias; a.res = (const bf16*)res;
    a.pre = (bf16*)pre; a.ws = ws; a.alpha = alpha; a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
    if (cfg < 0 || split < 0) {
        Choice ch = pick(M, N, K, split);
        if (cfg < 0) cfg = pk_ok(N, ldc, out_f32, act) ? 9 : ch.cfg;
        if (split < 0) split = ch.split;
    }
    if (cfg == 9 && !pk_ok(N, ldc, out_f32, act)) cfg = 1;  // shapes the persistent kernel does not take
    if (cfg >= 90 && cfg < 90 + 256) {  // timing-only ablation builds of cfg 9 (wrong outputs)
#ifndef REPLICANN_DEV
        return -1;  // not in a production library (REPLICANN_DEV=1 builds them)
#else
        GemmArgs d = {};
        d.A = (const bf16*)A; d.B = (const bf16*)B; d.C = C; d.M = M; d.N = N; d.K = K;
        d.lda = lda; d.ldb = ldb; d.ldc = ldc; d.split = 1; d.k_per_split = (K + BK - 1) / BK * BK;
        d.tiles_m = (M + 255) / 256; d.tiles_n = (N + 255) / 256;
        return rn_gemm_launch_pk_dbg(d, !trans_a, trans_b, cfg - 90, st) == 0 ? 0 : -1;
#endif
    }
    a.split = split < 1 ? 1 : split;
    int kps = (K + a.split - 1) / a.split;
    kps = (kps + BK - 1) / BK * BK;
    a.k_per_split = kps;
    a.split = (K + kps - 1) / kps;
    a.out_f32 = out_f32; a.accumulate = accumulate;
    a.colpart = colpart;

    if (colpart && (!act_bwd(act) || a.split > 1 || out_f32 || N % 8 != 0 || ldc % 8 != 0 || cfg == 6 || cfg == 4 ||
                    cfg == 3))
        return -3;  // 256x192 (CPR 24) and the simple 256-wide configs are not wired for it
    const bool ak = !trans_a, bk = trans_b;
    switch (cfg) {
        case 1: rn_gemm_launch_cfg1(a, ak, bk, act, st); break;
        case 2: rn_gemm_launch_cfg2(a, ak, bk, act, st); break;
        case 3: rn_gemm_launch_cfg3(a, ak, bk, act, st); break;
        case 4: rn_gemm_launch_cfg4(a, ak, bk, act, st); break;
        case 5: rn_gemm_launch_cfg5(a, ak, bk, act, st); break;
        case 6: rn_gemm_launch_cfg6(a, ak, bk, act, st); break;
        case 8: rn_gemm_launch_cfg8(a, ak, bk, act, st); break;
        case 9:
            a.tiles_m = (M + 255) / 256;
            a.tiles_n = (N + 255) / 256;
            if (ak && bk) rn_gemm_launch_pk_tt(a, act, st);
            else if (ak) rn_gemm_launch_pk_tf(a, act, st);
            else if (bk) rn_gemm_launch_pk_ft(a, act, st);
            else rn_gemm_launch_pk_ff(a, act, st);
            break;
        default: rn_gemm_launch_cfg0(a, ak, bk, act, st); break;
    }
    return 0;
}

}  // extern "C"
