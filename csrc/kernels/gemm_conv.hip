// Implicit-GEMM convolution (NHWC bf16): the im2col matrix is never materialised — the
// GEMM's LDS-DMA loaders gather each K-tile (one filter tap × 64 channels) straight from
// the activation tensor, zero-filling the padding through the buffer range check.
//   mode 1  fwd    y[pix][oc]    = Σ_k x̂[pix][k] · w[oc][k]          (A gathered)
//   mode 2  dgrad  dx[pix][c]    = Σ_k dŷ[pix][k] · w[co][kh][kw][c]  (A gathered, stride 1)
//   mode 3  wgrad  dw[oc][k]     = Σ_pix dy[pix][oc] · x̂[pix][k]      (B gathered, split-K over pixels)
// All on the NS = 3 stage ring of gemm_impl.h.
#include "gemm_impl.h"

using namespace rn_gemm_detail;

namespace {

template <int BM, int BN, int WM, int WN, int MODE, bool AK, bool BK_>
void conv_launch(GemmArgs& a, hipStream_t st) {
    a.tiles_m = (a.M + BM - 1) / BM;
    a.tiles_n = (a.N + BN - 1) / BN;
    launch_t<BM, BN, WM, WN, true, AK, BK_, ACT_NONE, 3, MODE>(a, st);
}

}  // namespace

extern "C" {

// Weight-gradient tile (mode 3; M = output channels, N = taps × channels):
//   0: 128×128, 4 waves   1: 64×192, 4 waves (M = 64: no half-empty tile)
//   2: 128×192, 8 waves   3: 256×128, 8 waves   4: 64×192, 8 waves (32×48 per wave; M = 64)
// REPLICANN_CONVW=<v> forces one (A/B timing); otherwise the measured choice per shape.
int rn_conv_wgrad_variant(int M, int N) {
    static int forced = [] {
        const char* e = getenv("REPLICANN_CONVW");
        return e ? atoi(e) : -1;
    }();
    // measured (scripts/conv_ab.py, ResNet-18 B=256): 128×192 / 8 waves is fastest on every 3×3
    // layer shape (layer1 0.368 → 0.246 ms, layers 2-4 0.18-0.19 → 0.11-0.135 ms vs 128×128)
    // 64-output-channel layers (ResNet layer 1): 64×192 / 8 waves, no half-empty 128-row tile — 0.192-0.197 →
    // 0.166-0.169 ms (profiles/conv_wgrad_r5u.txt)
    int v = forced >= 0 ? forced : (M == 64 && N % 192 == 0 ? 4 : 2);
    if ((v == 1 || v == 2 || v == 4) && N % 192 != 0) v = 0;
    if ((v == 1 || v == 4) && M != 64) v = 0;
    if (v == 3 && M < 256) v = 0;
    return v;
}
void rn_conv_wgrad_tile(int M, int N, int* bm, int* bn) {
    static const int BMS[5] = {128, 64, 128, 256, 64}, BNS[5] = {128, 192, 192, 128, 192};
    const int v = rn_conv_wgrad_variant(M, N);
    *bm = BMS[v];
    *bn = BNS[v];
}

// Returns 0, or -1 if the geometry is outside the implicit path (caller falls back to im2col).
int rn_conv_gemm(int mode, const void* A, const void* B, void* C, const void* bias, float* ws, int M, int N, int K,
                 long lda, long ldb, long ldc, int H, int W, int Cg, int RH, int RW, int KH, int KW, int S, int P,
                 int KC, int BC, long bld, int split, int out_f32, int accumulate, float* colpart,
                 hipStream_t st) {
    // the gathered operand's dimension must be whole 64-channel taps: GEMM K for fwd/dgrad,
    // GEMM N for wgrad (whose K = output pixels has an arbitrary tail, zero-filled by the loaders)
    if (KC % 64 != 0 || (mode != 3 && K % 64 != 0)) return -1;
    const long pixels = mode == 3 ? K : M;  // the gathered tensor holds pixels / (RH·RW) images
    if ((long)H * W * Cg * (pixels / ((long)RH * RW) + 1) * 2 >= (1L << 31)) return -1;  // 32-bit offsets
    GemmArgs a = {};
    a.A = (const bf16*)A; a.B = (const bf16*)B; a.C = C; a.bias = (const bf16*)bias; a.ws = ws;
    a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.out_f32 = out_f32; a.accumulate = accumulate;
    // mode 1 only: [ceil(M / 256)][2N] fp32 per-M-tile Σ | Σ² of the bf16 output (BatchNorm stats);
    // both mode-1 tiles are 256 rows and NT % (BN / 8) == 0
    a.colpart = mode == 1 ? colpart : nullptr;
    ConvGeom& g = a.cv;
    g.H = H; g.W = W; g.C = Cg; g.RH = RH; g.RW = RW; g.KH = KH; g.KW = KW; g.S = S; g.P = P;
    g.KC = KC; g.BC = BC; g.bld = bld;
    g.fd_hw = make_fastdiv((uint32_t)(RH * RW));
    g.fd_w = make_fastdiv((uint32_t)RW);
    g.fd_kc = make_fastdiv((uint32_t)KC);
    g.fd_kw = make_fastdiv((uint32_t)KW);
    a.split = split < 1 ? 1 : split;
    int kps = (K + a.split - 1) / a.split;
    kps = (kps + BK - 1) / BK * BK;
    a.k_per_split = kps;
    a.split = (K + kps - 1) / kps;
    if (mode == 1) {
        if (N % 64 != 0) return -1;
        if (N == 64) conv_launch<256, 64, 8, 1, 1, true, true>(a, st);
        else conv_launch<256, 128, 4, 2, 1, true, true>(a, st);
        return 0;
    }
    if (mode == 2) {
        if (N % 64 != 0 || S != 1) return -1;
        if (N == 64) conv_launch<256, 64, 8, 1, 2, true, false>(a, st);
        else conv_launch<256, 128, 4, 2, 2, true, false>(a, st);
        return 0;
    }
    if (mode == 3) {
        if (N % 64 != 0 || M % 8 != 0 || lda % 8 != 0) return -1;
        switch (rn_conv_wgrad_variant(M, N)) {
            case 1: conv_launch<64, 192, 1, 4, 3, false, false>(a, st); break;
            case 2: conv_launch<128, 192, 2, 4, 3, false, false>(a, st); break;
            case 3: conv_launch<256, 128, 4, 2, 3, false, false>(a, st); break;
            case 4: conv_launch<64, 192, 2, 4, 3, false, false>(a, st); break;
            default: conv_launch<128, 128, 2, 2, 3, false, false>(a, st); break;
        }
        return 0;
    }
    return -1;
}

}  // extern "C"
