// 3×3 / stride 1 / pad 1 convolution with 64 input and 64 output channels (NHWC bf16) on a halo tile in LDS:
// ResNet-18's layer-1 forward convolutions and their data gradients.
//
// Why its own kernel: on the implicit-GEMM path (gemm_conv.hip) every K-tile is one filter tap gathered from
// the activation, so each activation element crosses the L2 → LDS path 9 times (925 MB per layer-1 conv at
// B = 256) and the 256×64 tile runs at ≈370 TF/s, bound by that traffic (profiles/resnet_vit_r5r.txt).
// Here a workgroup owns TR whole image rows (TR·W output pixels; W = 56 → 4 rows = 224 pixels = 14 MFMA
// row fragments), loads the (TR + 2) × (W + 2) × 64 input halo ONCE into LDS (zeros outside the image), and
// takes all 9 taps from it: tap (kh, kw) of output pixel (r, c) is halo pixel (r + kh, c + kw).  The 64 × 576
// weight matrix stays in LDS for the workgroup's whole life (persistent grid, one workgroup per CU), and the
// next tile's halo is loaded into registers while the current one computes.
//
//   out[p][n] = Σ_{tap, ci} halo[p ⊕ tap][ci] · B[n][tap·64 + ci]
//   forward:       B[n = oc][k]          = w[oc][kh][kw][ci]             (w as stored: [n][k] rows)
//   data gradient: B[n = c][tap·64 + oc] = w[oc][2 − kh][2 − kw][c]      (dx = dy ∗ flipped, transposed w)
//
// MFMA v_mfma_f32_16x16x32_bf16 with the weights as the first operand, so a lane's accumulator holds 4
// consecutive output channels of one pixel (one 8-byte store).  Both operands are K-contiguous rows in LDS
// (weight rows of 576 k, halo pixels of 64 channels): one ds_read_b128 per fragment, 8 consecutive k per lane.
// Rows are XOR-swizzled by 16-byte chunk with (row >> 1) & 7: rows are 1152 / 128 bytes apart, two rows share
// a 256-byte bank window, so the 16 rows of a fragment read land in 16 distinct 16-byte bank slots.
// FM = 4 pixel fragments per wave (64 pixels) where the tile allows it: each weight fragment read then feeds
// 4 MFMAs (LDS bytes per MFMA 0.5 KB instead of 0.75 KB at FM = 2).
// Forward epilogue: optional per-tile Σ | Σ² of the bf16 outputs per channel ([tiles][128] fp32, the following
// BatchNorm's statistics; fixed-order, no atomics).  Data-gradient epilogue: optional accumulate into `out`
// (the second gradient of a residual-block input).
#include <cstdlib>

#include "common.h"

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8v __attribute__((ext_vector_type(8)));

constexpr int C3 = 64;             // channels in and out
constexpr int KTOT = 9 * C3;       // 576
constexpr int BROW = KTOT * 2;     // bytes per weight row in LDS
constexpr int B_BYTES = C3 * BROW; // 73,728

struct Conv3Args {
    const bf16* in;   // [N][H][W][64]
    const bf16* w;    // [64][3][3][64]
    bf16* out;        // [N][H][W][64]
    float* part;      // forward statistics [tiles][128] or null
    int N, H, W, TR, waves, tiles, accumulate, dgrad;
};

__device__ inline uint32_t halo_off(int q, int chunk) { return (uint32_t)(q * 128 + ((chunk ^ ((q >> 1) & 7)) << 4)); }
__device__ inline uint32_t brow_off(int n, int chunk) { return (uint32_t)(n * BROW + ((chunk ^ ((n >> 1) & 7)) << 4)); }

constexpr int MAXLD = 12;  // halo chunks per thread (host-checked)

template <int FM>
__global__ void __launch_bounds__(512, 1) conv3x3_k(Conv3Args a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* bl = smem;                      // weights [64][576] bf16, swizzled rows
    char* hl = smem + B_BYTES;            // halo [(TR + 2) · (W + 2)][64] bf16, swizzled pixels
    const int HW2 = (a.TR + 2) * (a.W + 2);
    float* red = reinterpret_cast<float*>(hl + HW2 * 128);  // [waves][128] statistics partials
    const int tid = threadIdx.x, nth = blockDim.x;
    const int lane = tid & 63, wave = tid >> 6, g = lane >> 4, c = lane & 15;

    // ---- weights, once per workgroup ----
    if (!a.dgrad) {
        for (int e = tid; e < C3 * (KTOT / 8); e += nth) {
            const int n = e / (KTOT / 8), kc = e % (KTOT / 8);
            const uint4 v = *reinterpret_cast<const uint4*>(a.w + (long)n * KTOT + kc * 8);
            *reinterpret_cast<uint4*>(bl + brow_off(n, kc)) = v;
        }
    } else {
        // w row (oc, tap_w) holds 64 consecutive c: chunk cc scatters into rows n = 8cc .. 8cc + 7 at
        // k = (8 − tap_w)·64 + oc
        for (int e = tid; e < C3 * 9 * 8; e += nth) {
            const int oc = e / 72, rem = e % 72, tw = rem / 8, cc = rem % 8;
            const s16x8v v = *reinterpret_cast<const s16x8v*>(a.w + ((long)oc * 9 + tw) * C3 + cc * 8);
            const int k = (8 - tw) * C3 + oc;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int n = cc * 8 + j;
                *reinterpret_cast<short*>(bl + brow_off(n, k >> 3) + (k & 7) * 2) = v[j];
            }
        }
    }

    // ---- per-lane fragment geometry: wave owns pixel fragments FM·wave .. FM·wave + FM − 1 of the tile ----
    const int W2 = a.W + 2;
    int qb[FM];
#pragma unroll
    for (int f = 0; f < FM; ++f) {
        const int p = 16 * (FM * wave + f) + c;
        qb[f] = (p / a.W) * W2 + (p % a.W);  // halo pixel of tap (0, 0)
    }
    const int rows_per_img = a.H / a.TR;
    const int nchunks = HW2 * 8;
    const int nld = (nchunks + nth - 1) / nth;  // <= MAXLD (host)

    uint4 pre[MAXLD];
    auto load_halo = [&](int tile) {
        const int n = tile / rows_per_img, h0 = (tile % rows_per_img) * a.TR;
#pragma unroll
        for (int i = 0; i < MAXLD; ++i) {
            pre[i] = make_uint4(0, 0, 0, 0);
            const int u = tid + i * nth;
            if (i < nld && u < nchunks) {
                const int q = u >> 3, ch = u & 7;
                const int h = h0 - 1 + q / W2, w = q % W2 - 1;
                if (h >= 0 && h < a.H && w >= 0 && w < a.W)
                    pre[i] = *reinterpret_cast<const uint4*>(a.in + (((long)n * a.H + h) * a.W + w) * C3 + ch * 8);
            }
        }
    };
    auto store_halo = [&]() {
#pragma unroll
        for (int i = 0; i < MAXLD; ++i) {
            const int u = tid + i * nth;
            if (i < nld && u < nchunks) *reinterpret_cast<uint4*>(hl + halo_off(u >> 3, u & 7)) = pre[i];
        }
    };

    int tile = blockIdx.x;
    if (tile < a.tiles) load_halo(tile);
    for (; tile < a.tiles; tile += gridDim.x) {
        __syncthreads();  // the previous tile's halo / statistics reads are done (and the weights are in)
        store_halo();
        __syncthreads();
        if (tile + (int)gridDim.x < a.tiles) load_halo(tile + gridDim.x);  // in flight during the MFMAs

        f32x4 acc[FM][4];
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[f][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        const bool live = 16 * FM * wave < a.TR * a.W;  // (host: TR·W = 16·FM·waves, every wave live)
        if (live) {
            // (taps not unrolled: the full 18-step unroll hoisted every fragment load and spilled at 2 waves / SIMD)
#pragma unroll 1
            for (int tap = 0; tap < 9; ++tap) {
                const int toff = (tap / 3) * W2 + (tap % 3);
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int ch = 4 * s + g;  // 16-byte chunk: channels / k 32s + 8g .. +7 of this tap
                    s16x8v bf[4], af[FM];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        bf[j] = *reinterpret_cast<const s16x8v*>(bl + brow_off(16 * j + c, tap * 8 + ch));
#pragma unroll
                    for (int f = 0; f < FM; ++f)
                        af[f] = *reinterpret_cast<const s16x8v*>(hl + halo_off(qb[f] + toff, ch));
#pragma unroll
                    for (int f = 0; f < FM; ++f)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[f], acc[f][j], 0, 0, 0);
                }
            }
        }
        // ---- epilogue: lane holds out[pixel 16(2·wave + f) + c][channels 16j + 4g .. +3] ----
        const long pix0 = (long)tile * a.TR * a.W;
        float s1[4][4], s2[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
        if (live) {
#pragma unroll
            for (int f = 0; f < FM; ++f) {
                bf16* op = a.out + (pix0 + 16 * (FM * wave + f) + c) * C3;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float v[4] = {acc[f][j][0], acc[f][j][1], acc[f][j][2], acc[f][j][3]};
                    bf16* dst = op + 16 * j + 4 * g;
                    if (a.accumulate) {
                        const bf16x4 old = *reinterpret_cast<const bf16x4*>(dst);
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] += (float)old[r];
                    }
                    const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
                    *reinterpret_cast<bf16x4*>(dst) = o;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float y = (float)o[r];
                        s1[j][r] += y;
                        s2[j][r] += y * y;
                    }
                }
            }
        }
        if (a.part) {  // Σ | Σ² over the tile's pixels: 16 lanes (pixels c), then the waves in order
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) {
                        s1[j][r] += __shfl_xor(s1[j][r], o, 64);
                        s2[j][r] += __shfl_xor(s2[j][r], o, 64);
                    }
            if (c == 0) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        red[wave * 128 + 16 * j + 4 * g + r] = s1[j][r];
                        red[wave * 128 + 64 + 16 * j + 4 * g + r] = s2[j][r];
                    }
            }
            __syncthreads();
            if (tid < 128) {
                float t = 0.f;
                for (int w2 = 0; w2 < a.waves; ++w2) t += red[w2 * 128 + tid];
                a.part[(long)tile * 128 + tid] = t;
            }
        }
    }
}

size_t conv3x3_lds(int tr, int W, int fm) {
    return (size_t)B_BYTES + (size_t)(tr + 2) * (W + 2) * 128 + (size_t)(tr * W / (16 * fm)) * 128 * 4;
}
// rows per tile and pixel fragments per wave (FM 4 preferred: 64 pixels per wave); 0 = shape not taken
int conv3x3_rows(int H, int W, int* fm) {
    for (int f : {4, 2})
        for (int tr : {8, 4, 2, 1}) {
            const int px = tr * W;
            if (H % tr || px % (16 * f) || px / (16 * f) > 8) continue;
            const int nth = px / (16 * f) * 64;
            if ((tr + 2) * (W + 2) * 8 > MAXLD * nth || conv3x3_lds(tr, W, f) > 160 * 1024) continue;
            *fm = f;
            return tr;
        }
    return 0;
}

bool conv3x3_on() {
    static const bool on = [] { const char* e = std::getenv("REPLICANN_CONV3X3"); return !(e && e[0] == '0'); }();
    return on;
}

}  // namespace

extern "C" {

// tiles (rows of the statistics partials) of the halo-tile conv for this shape; 0 = not taken (the implicit
// GEMM runs instead)
int rn_conv3x3_tiles(int N, int H, int W) {
    if (!conv3x3_on()) return 0;
    int fm = 0;
    const int tr = conv3x3_rows(H, W, &fm);
    return tr == 0 ? 0 : N * (H / tr);
}

// in / out NHWC [N][H][W][64], w [64][3][3][64]; dgrad: out = dx from in = dy (w flipped / transposed);
// part: forward statistics [tiles][128] (or null); accumulate: out += result.  Returns -1 if not taken.
int rn_conv3x3(const void* in, const void* w, void* out, float* part, int N, int H, int W, int dgrad, int accumulate,
               hipStream_t st) {
    const int tiles = rn_conv3x3_tiles(N, H, W);
    if (tiles == 0) return -1;
    Conv3Args a = {};
    a.in = (const bf16*)in; a.w = (const bf16*)w; a.out = (bf16*)out; a.part = part;
    int fm = 0;
    a.N = N; a.H = H; a.W = W; a.TR = conv3x3_rows(H, W, &fm); a.waves = a.TR * W / (16 * fm); a.tiles = tiles;
    a.accumulate = accumulate; a.dgrad = dgrad;
    const size_t lds = conv3x3_lds(a.TR, W, fm);
    // the >64 KiB dynamic-LDS opt-in is per device (a process may drive several GPUs): once per device
    static uint64_t attr_devs = 0;
    static int cu_count[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    const uint64_t bit = 1ull << (dev & 63);
    if (!(attr_devs & bit)) {
        (void)hipFuncSetAttribute((const void*)conv3x3_k<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)conv3x3_k<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        cu_count[dev & 63] = cus > 0 ? cus : 256;
        attr_devs |= bit;
    }
    const int cus = cu_count[dev & 63];
    const int grid = tiles < cus ? tiles : cus;
    if (fm == 4) conv3x3_k<4><<<grid, a.waves * 64, lds, st>>>(a);
    else conv3x3_k<2><<<grid, a.waves * 64, lds, st>>>(a);
    return 0;
}

}  // extern "C"
