// PyTorch dispatcher registration for the replicann gfx950 kernels.
//
// Host-only translation unit: validates shapes/dtypes, allocates outputs with
// the caching allocator, picks the current HIP stream and calls the extern "C"
// launchers compiled from csrc/kernels/*.hip.  Ops are registered under
// torch.ops.replicann.* for the CUDA (= HIP on ROCm) dispatch key only: there is
// no CPU kernel here — CPU tensors never reach these ops (ATen path in Python).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <optional>
#include <sstream>
#include <tuple>
#include <vector>

using at::Tensor;
using c10::optional;

extern "C" {
void rn_act_fwd(const void*, void*, long, int, hipStream_t);
void rn_act_bwd(const void*, const void*, void*, long, int, hipStream_t);
void rn_dropout(const void*, void*, long, float, uint64_t, const uint64_t*, hipStream_t);
void rn_rng_next(void*, void*, hipStream_t);
void rn_add(const void*, const void*, void*, long, int, hipStream_t);
void rn_bias_act_grad(const void*, const void*, void*, float*, void*, float*, int, int, int, int, int, hipStream_t);
int rn_bias_act_grad_splits(int, int);
int rn_ln_fwd(const void*, const void*, const void*, const void*, void*, void*, float*, float*, int, int, float,
              hipStream_t, void*, float*);
void rn_fp8_roll(float*, hipStream_t);
void rn_fp8_quant_many(const void*, const long*, int, long, void*, int, hipStream_t);
int rn_ln_bwd_waves(int);
long rn_ln_bwd_ws(int, int);
int rn_ln_bwd(const void*, const void*, const void*, const void*, const float*, const float*, void*, float*, float*,
              void*, void*, void*, float*, int, int, int, hipStream_t, void*, float*);
void rn_softmax_fwd(const void*, void*, int, int, float, hipStream_t);
void rn_softmax_bwd(const void*, const void*, void*, int, int, float, hipStream_t);
void rn_xent_fwd(void*, const int64_t*, float*, float*, int, int, int, long, int, hipStream_t);
int rn_xent_fwd_q8(void*, const int64_t*, float*, float*, int, int, int, long, void*, hipStream_t);
void rn_xent_bwd(const void*, const int64_t*, const float*, const float*, void*, int, int, int, long, hipStream_t);
void rn_emb_fwd(const int64_t*, const void*, const void*, void*, int, int, int, int, hipStream_t);
void rn_vit_join_fwd(const void*, const void*, const void*, void*, int, int, int, hipStream_t);
void rn_vit_join_bwd(const void*, void*, void*, void*, int, int, int, hipStream_t);
void rn_emb_bwd_acc(const int64_t*, const void*, float*, unsigned*, void*, void*, int, int, int, int, hipStream_t);
void rn_emb_bwd_acc_det(const int64_t*, const void*, void*, unsigned*, void*, void*, int, int, int, int, hipStream_t);
void rn_emb_bwd(const int64_t*, const void*, float*, void*, void*, int, int, int, int, int, hipStream_t);
int rn_norm_ws_floats();
void rn_sumsq(const void*, long, int, float*, float*, hipStream_t);
void rn_opt_prep(float*, float, float, float, float, int, float, float, float, hipStream_t);
int rn_adamw(void*, float*, const void*, int, float*, float*, const uint8_t*, float*, long, float, float, float, float,
             float, float, int, hipStream_t);
void rn_sgd(void*, float*, const void*, int, float*, const uint8_t*, float*, long, float, float, int, float, float,
            hipStream_t);
long rn_gemm_ws_floats(int, int, int);
void rn_gemm_set_sched(int);
int rn_gemm_get_sched();
void rn_gemm_set_reserve(int);
int rn_gemm_get_reserve();
int rn_gemm_sched_init(int);
int rn_gemm(const void*, const void*, void*, const void*, const void*, void*, float*, const float*, int, int, int,
            long, long, long, int, int, int, int, int, int, int, hipStream_t, float*);
int rn_gemm_cfg_bm(int);
long rn_gemm_colpart_rows(int, int);
int rn_attn_decode(const void*, const void*, const void*, const float*, void*, int, int, int, int, const long*, float,
                   hipStream_t);
int rn_gemm_skinny_kv(const void*, const void*, const void*, void*, int, int, int, long, long, long, void*,
                      const int64_t*, long, long, int, hipStream_t);
int rn_attn_fwd(const void*, const void*, const void*, void*, float*, const float*, int, const long*, int, int, int,
                int, int, float, int, float, uint64_t, const uint64_t*, hipStream_t);
int rn_attn_bwd(const void*, const void*, const void*, const void*, const void*, const float*, const float*, int,
                void*, void*, void*, float*, float*, float*, const long*, int, int, int, int, int, float, int, float,
                uint64_t, const uint64_t*, float*, void*, float*, int, float*, hipStream_t);
long rn_attn_q8_part_floats(int, int, int, int);
void rn_colsum_f32(const float*, int, int, float*, void*, int, hipStream_t);
int rn_colsum_ws(int);
int rn_attn_is_fast(int);
void rn_conv_wgrad_tile(int, int, int*, int*);
int rn_conv3x3_tiles(int, int, int);
int rn_conv3x3(const void*, const void*, void*, float*, int, int, int, int, int, hipStream_t);
int rn_conv_gemm(int, const void*, const void*, void*, const void*, float*, int, int, int, long, long, long, int, int,
                 int, int, int, int, int, int, int, int, int, long, int, int, int, float*, hipStream_t);
void rn_im2col(const void*, void*, int, int, int, int, int, int, int, int, int, int, int, hipStream_t);
void rn_col2im(const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int, hipStream_t);
void rn_maxpool_fwd(const void*, void*, void*, int, int, int, int, int, int, int, int, int, hipStream_t);
void rn_maxpool_bwd(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, hipStream_t);
void rn_avgpool_fwd(const void*, void*, int, int, int, hipStream_t);
void rn_avgpool_bwd(const void*, void*, int, int, int, hipStream_t);
void rn_fp8_quantize(const void*, long, void*, float*, hipStream_t);
void rn_fp8_dequantize(const void*, long, const float*, void*, hipStream_t);
void rn_fp8_quantize_delayed(const void*, long, void*, float*, hipStream_t);
void rn_bf8_quantize(const void*, long, void*, float*, int, hipStream_t);
int rn_act_mul_bf8_groups(long, int);
void rn_act_mul_bf8(const void*, const void*, long, int, void*, float*, int, float*, int, hipStream_t);
void rn_gelu_q8(const void*, long, void*, float*, hipStream_t);
void rn_bf8_dequantize(const void*, long, const float*, void*, hipStream_t);
long rn_gemm_fp8_wgrad_ws(int, int, int);
int rn_gemm_fp8_wgrad(const void*, const void*, void*, const float*, const float*, float*, float*, int, int, int, long,
                      long, long, int, int, int, hipStream_t, const float*);
int rn_gemm_fp8_dgrad(const void*, const void*, void*, const float*, const float*, float*, int, int, int, long, long,
                      long, int, hipStream_t, const float*);
int rn_gemm_fp8(const void*, const void*, void*, const void*, const void*, void*, const float*, const float*, float*,
                int, int, int, long, long, long, int, hipStream_t, void*, float*);
long rn_bn_ws_floats(int, int);
int rn_bn_supported(int);
void rn_bn_fwd(const void*, const void*, const void*, float*, float*, void*, float*, float*, float*, int, int, float,
               float, int, const void*, const float*, int, void*, hipStream_t);
void rn_bn_eval(const void*, const void*, const void*, const float*, const float*, void*, int, int, float, int,
                const void*, hipStream_t);
void rn_bn_bwd(const void*, const void*, const void*, const void*, const float*, const float*, void*, void*, void*,
               float*, int, int, int, void*, int, hipStream_t);
}

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16, got ", (t).scalar_type())
#define CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define GUARD(t) c10::hip::HIPGuardMasqueradingAsCUDA _guard((t).device())

const void* optr(const optional<Tensor>& t) { return (t && t->defined()) ? t->data_ptr() : nullptr; }

// ------------------------------------------------------------------ GEMM
// Measured tile-config / split-K selection.  The first eager call of every GEMM
// shape times the candidate configs on the current stream (into a scratch output;
// the real call then runs once with the winner) and caches the choice.  Calls made
// while the stream is being captured into a hipGraph never tune: they use the
// cache, or the native cost model.  REPLICANN_GEMM_AUTOTUNE=0 disables tuning.
struct TuneKey {
    int64_t M, N, K;
    int ta, tb, act, f32, autosplit, epi;  // epi: bias | residual<<1 | alpha<<2 | accumulate<<3
    bool operator<(const TuneKey& o) const {
        return std::tie(M, N, K, ta, tb, act, f32, autosplit, epi) <
               std::tie(o.M, o.N, o.K, o.ta, o.tb, o.act, o.f32, o.autosplit, o.epi);
    }
};
static std::map<TuneKey, std::pair<int, int>> g_tune;
static std::mutex g_tune_mu;

static bool autotune_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* e = std::getenv("REPLICANN_GEMM_AUTOTUNE");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    return v == 1;
}

std::string gemm_tuning_table() {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    std::ostringstream os;
    os << "[";
    bool first = true;
    for (auto& kv : g_tune) {
        const TuneKey& k = kv.first;
        os << (first ? "" : ",") << "{\"M\":" << k.M << ",\"N\":" << k.N << ",\"K\":" << k.K << ",\"ta\":" << k.ta
           << ",\"tb\":" << k.tb << ",\"act\":" << k.act << ",\"f32\":" << k.f32 << ",\"as\":" << k.autosplit
           << ",\"epi\":" << k.epi << ",\"cfg\":" << kv.second.first << ",\"split\":" << kv.second.second << "}";
        first = false;
    }
    os << "]";
    return os.str();
}

// Replace/insert tuning entries from a gemm_tuning_table() string (data-parallel ranks adopt rank 0's
// measured picks, so every rank runs the same kernels).  Returns the number of entries loaded.
int64_t gemm_tuning_load(const std::string& js) {
    int64_t n = 0;
    size_t pos = 0;
    std::lock_guard<std::mutex> lk(g_tune_mu);
    while ((pos = js.find('{', pos)) != std::string::npos) {
        const size_t end = js.find('}', pos);
        if (end == std::string::npos) break;
        const std::string obj = js.substr(pos, end - pos + 1);
        long M, N, K;
        int ta, tb, act, f32, as, epi, cfg, split;
        if (std::sscanf(obj.c_str(),
                        "{\"M\":%ld,\"N\":%ld,\"K\":%ld,\"ta\":%d,\"tb\":%d,\"act\":%d,\"f32\":%d,\"as\":%d,"
                        "\"epi\":%d,\"cfg\":%d,\"split\":%d}",
                        &M, &N, &K, &ta, &tb, &act, &f32, &as, &epi, &cfg, &split) == 11) {
            g_tune[TuneKey{M, N, K, ta, tb, act, f32, as, epi}] = {cfg, split};
            ++n;
        }
        pos = end + 1;
    }
    return n;
}

// "cfg 7": the vendor library (hipBLASLt through at::mm) for PLAIN GEMMs only — no
// epilogue (bias / activation / residual / accumulate / alpha), bf16 out.  Reachable only
// by an explicit cfg=7 or, for A/B measurements, REPLICANN_GEMM_LIB=1 (then one more
// autotuner candidate); never a fallback.  Every default-path GEMM runs on the MFMA kernels.
constexpr int kLibCfg = 7;
// The library is NOT among the autotuner's candidates unless REPLICANN_GEMM_LIB=1 (A/B runs only).
static bool lib_candidate() {
    static int v = -1;
    if (v < 0) {
        const char* e = std::getenv("REPLICANN_GEMM_LIB");
        v = (e && e[0] == '1') ? 1 : 0;
    }
    return v == 1;
}
static void lib_gemm(const Tensor& A, const Tensor& B, bool ta, bool tb, Tensor& c) {
    at::mm_out(c, ta ? A.t() : A, tb ? B.t() : B);
}

Tensor gemm(const Tensor& a, const Tensor& b, bool ta, bool tb, const optional<Tensor>& bias,
            const optional<Tensor>& residual, int64_t act, const optional<Tensor>& preact, const optional<Tensor>& out,
            bool accumulate, int64_t split_k, bool out_fp32, const optional<Tensor>& alpha, int64_t cfg,
            const optional<Tensor>& bias_grad) {
    CHECK_CUDA(a); CHECK_BF16(a); CHECK_BF16(b);
    GUARD(a);
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2, "gemm expects 2-D operands");
    TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1, "gemm operands need unit inner stride");
    const int64_t M = ta ? a.size(1) : a.size(0);
    const int64_t K = ta ? a.size(0) : a.size(1);
    const int64_t Kb = tb ? b.size(1) : b.size(0);
    const int64_t N = tb ? b.size(0) : b.size(1);
    TORCH_CHECK(K == Kb, "gemm inner dims differ: ", K, " vs ", Kb);
    Tensor c;
    if (out && out->defined()) {
        c = *out;
        TORCH_CHECK(c.size(0) == M && c.size(1) == N && c.stride(1) == 1, "gemm out shape mismatch");
        out_fp32 = c.scalar_type() == at::kFloat;
    } else {
        c = at::empty({M, N}, a.options().dtype(out_fp32 ? at::kFloat : at::kBFloat16));
    }
    if (bias && bias->defined()) { CHECK_BF16(*bias); TORCH_CHECK(bias->numel() == N && bias->is_contiguous()); }
    if (residual && residual->defined()) {
        CHECK_BF16(*residual);
        TORCH_CHECK(residual->size(0) == M && residual->size(1) == N && residual->stride(0) == c.stride(0) &&
                    residual->stride(1) == 1, "residual must match the output layout");
    }
    if (preact && preact->defined()) {
        CHECK_BF16(*preact);
        TORCH_CHECK(preact->size(0) == M && preact->size(1) == N && preact->stride(0) == c.stride(0));
    }
    // fused activation backward: out = (A·B) ⊙ act'(preact); 6: out = (A·B) ⊙ preact (preact holds gelu'(h),
    // written by the act-5 forward)
    const bool act_bwd = act == 3 || act == 4 || act == 6;
    // bias_grad (act-backward only): Σ_rows of the output accumulated into it — from per-M-tile
    // column partials the epilogue writes (configs that support it), else one reduction pass
    const bool want_bg = bias_grad && bias_grad->defined();
    if (want_bg) {
        TORCH_CHECK(act_bwd, "gemm bias_grad needs an activation-backward epilogue");
        CHECK_BF16(*bias_grad);
        TORCH_CHECK(bias_grad->numel() == N && bias_grad->is_contiguous());
    }
    // rows: enough for every config (128-row tiles: ceil(M/128); cfg 9: 2 per 256-row tile)
    Tensor colpart = want_bg ? at::empty({2 * ((M + 255) / 256), N}, a.options().dtype(at::kFloat)) : Tensor();
    float* cp = want_bg ? colpart.data_ptr<float>() : nullptr;
    if (act_bwd)
        TORCH_CHECK(!ta && !tb && N % 8 == 0 && preact && preact->defined() && !accumulate && !(bias && bias->defined()),
                    "activation-backward epilogue: dgrad layout (A·B, B [K][N]), N % 8 == 0, preact required");
    if (M == 0 || N == 0) return c;
    int split = split_k < 0 ? -1 : (int)std::max<int64_t>(1, split_k);
    Tensor ws;  // split-K slabs: allocated once the split is known (tuned / cached / explicit)
    // K must be a multiple of 8 (16-B rows); pad both operands with zeros otherwise
    Tensor A = a, B = b;
    int64_t Kp = K;
    if (K % 8 != 0) {
        Kp = (K + 7) / 8 * 8;
        A = ta ? at::constant_pad_nd(a, {0, 0, 0, Kp - K}) : at::constant_pad_nd(a, {0, Kp - K});
        B = tb ? at::constant_pad_nd(b, {0, Kp - K}) : at::constant_pad_nd(b, {0, 0, 0, Kp - K});
    }
    if (ta && (M % 8 != 0 || A.stride(0) % 8 != 0)) {  // M-contiguous A needs 16-B aligned rows
        A = A.t().contiguous();
        ta = false;
    }
    if (!tb && (N % 8 != 0 || B.stride(0) % 8 != 0)) {
        B = B.t().contiguous();
        tb = true;
    }
    if (!ta && A.stride(0) % 8 != 0) A = A.contiguous();
    if (tb && B.stride(0) % 8 != 0) B = B.contiguous();
    if (c.stride(0) % 4 != 0 && (bias || residual)) { /* epilogue handles unaligned via scalar path */ }
    if (alpha && alpha->defined()) TORCH_CHECK(alpha->scalar_type() == at::kFloat && alpha->is_cuda());
    if (cfg < 0 && split_k <= 0) {
        const int epi = (bias && bias->defined() ? 1 : 0) | (residual && residual->defined() ? 2 : 0) |
                        (alpha && alpha->defined() ? 4 : 0) | (accumulate ? 8 : 0) | (want_bg ? 16 : 0);
        const TuneKey key{M, N, Kp, (int)ta, (int)tb, (int)act, (int)out_fp32, split_k < 0 ? 1 : 0, epi};
        bool hit = false;
        {
            std::lock_guard<std::mutex> lk(g_tune_mu);
            auto it = g_tune.find(key);
            if (it != g_tune.end()) { cfg = it->second.first; split = it->second.second; hit = true; }
        }
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        (void)hipStreamIsCapturing(cur_stream(), &cap);
        if (!hit && autotune_enabled() && cap == hipStreamCaptureStatusNone) {
            Tensor scratch = at::empty({M, N}, a.options().dtype(out_fp32 ? at::kFloat : at::kBFloat16));
            // forward activations time WITH their pre-activation / derivative store (a scratch copy): the
            // second output is a large part of the epilogue, and configs differ most in the epilogue
            const bool act_fwd_pre = !act_bwd && act != 0 && preact && preact->defined();
            Tensor scratch_pre = act_fwd_pre ? at::empty({M, N}, a.options()) : Tensor();
            const bool plain = !(bias && bias->defined()) && !(residual && residual->defined()) && act == 0 &&
                               !(alpha && alpha->defined()) && !out_fp32 && !accumulate && c.is_contiguous();
            // decode-size GEMMs (M <= 64 rows, x·Wᵀ): the skinny config 10 joins the candidates
            const bool skinny = M <= 64 && !ta && tb && !act_bwd && !accumulate && !want_bg;
            int cfgs[9] = {9, 1, 6, 0, 2, 8, 0, 0, 0};
            int ncfg = 6;
            // the one-wave-per-SIMD persistent kernel (gemm_w1.h): A K-contiguous, plain / bias / alpha epilogue
            const bool w1_ok = !ta && act == 0 && !(residual && residual->defined()) && !accumulate && !out_fp32 &&
                               !want_bg && Kp % 64 == 0 && Kp >= 128 && N % 8 == 0 && c.stride(0) % 8 == 0 &&
                               !((bias && bias->defined()) && (alpha && alpha->defined()));
            if (w1_ok) cfgs[ncfg++] = 11;
            if (plain && lib_candidate()) cfgs[ncfg++] = kLibCfg;
            if (skinny) cfgs[ncfg++] = 10;
            // non-powers of two too: the split that makes tiles × split just fill the 256 CUs
            // (e.g. 48 tiles × 5 = 240) beats the next power of two by up to 25 %
            // up to 128 slabs for tiny outputs over a huge K (e.g. a conv-stem weight gradient: 64×147
            // outputs, 3 M pixels), where even 16 splits leave most CUs idle
            // (7 and 14: 36 output tiles of 256² — GPT-2's 3072×768 weight gradients — × 7 = 252 WGs)
            const int splits[16] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 24, 32, 64, 128};
            const long out_tiles = ((M + 255) / 256) * ((N + 255) / 256);
            const int nsplit = split_k < 0 ? (out_tiles * 16 < 256 ? 16 : 12) : 1;
            Tensor tws = at::empty({rn_gemm_ws_floats(M, N, splits[nsplit - 1])}, a.options().dtype(at::kFloat));
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            float best_ms = 1e30f;
            int best_cfg = 0, best_split = 1;
            // two interleaved rounds over all candidates, best-of per candidate: one round's
            // clock / cache transients otherwise flip close calls (e.g. library vs MFMA kernel)
            for (int round = 0; round < 2; ++round)
            for (int ci = 0; ci < ncfg; ++ci) {
                for (int si = 0; si < nsplit; ++si) {
                    const int sp = splits[si];
                    if (sp > 1 && Kp / sp < 256) break;
                    if (cfgs[ci] == kLibCfg && sp > 1) break;
                    if (cfgs[ci] == 11 && sp > 1) break;  // (no split-K form)
                    auto run = [&]() {
                        if (cfgs[ci] == kLibCfg) { lib_gemm(A, B, ta, tb, scratch); return 0; }
                        return rn_gemm(A.data_ptr(), B.data_ptr(), scratch.data_ptr(), optr(bias), optr(residual),
                                       act_bwd ? preact->data_ptr() : (act_fwd_pre ? scratch_pre.data_ptr() : nullptr),
                                       tws.data_ptr<float>(), alpha && alpha->defined() ? alpha->data_ptr<float>() : nullptr,
                                       (int)M, (int)N, (int)Kp, A.stride(0), B.stride(0), scratch.stride(0), ta, tb, (int)act,
                                       sp, out_fp32, 0, cfgs[ci], cur_stream(), cp);
                    };
                    if (run() != 0) continue;
                    (void)hipEventRecord(e0, cur_stream());
                    for (int r = 0; r < 5; ++r) run();
                    (void)hipEventRecord(e1, cur_stream());
                    (void)hipEventSynchronize(e1);
                    float ms = 0.f;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    if (ms < best_ms) { best_ms = ms; best_cfg = cfgs[ci]; best_split = sp; }
                }
            }
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            {
                std::lock_guard<std::mutex> lk(g_tune_mu);
                g_tune[key] = {best_cfg, best_split};
            }
            if (std::getenv("REPLICANN_GEMM_VERBOSE"))
                std::fprintf(stderr, "[replicann gemm tune] M=%ld N=%ld K=%ld ta=%d tb=%d act=%ld -> cfg %d split %d (%.3f ms)\n",
                             (long)M, (long)N, (long)Kp, (int)ta, (int)tb, (long)act, best_cfg, best_split, best_ms / 5);
            cfg = best_cfg;
            split = best_split;
        }
    }
    if (cfg == kLibCfg) {
        TORCH_CHECK(!(bias && bias->defined()) && !(residual && residual->defined()) && act == 0 &&
                        !(alpha && alpha->defined()) && !out_fp32 && !accumulate,
                    "gemm cfg 7 (library) is for plain GEMMs only");
        lib_gemm(A, B, ta, tb, c);
        return c;
    }
    // split < 0: the native cost model picks (at most 32 slabs, K/split >= 512): size for its worst case
    const int ws_split = split > 1 ? split : (split < 0 ? (int)std::min<int64_t>(32, std::max<int64_t>(1, Kp / 512)) : 1);
    if (ws_split > 1) ws = at::empty({rn_gemm_ws_floats(M, N, ws_split)}, a.options().dtype(at::kFloat));
    auto launch = [&](float* colp) {
        return rn_gemm(A.data_ptr(), B.data_ptr(), c.data_ptr(), optr(bias), optr(residual),
                       preact && preact->defined() ? preact->data_ptr() : nullptr,
                       ws.defined() ? ws.data_ptr<float>() : nullptr,
                       alpha && alpha->defined() ? alpha->data_ptr<float>() : nullptr, (int)M, (int)N, (int)Kp,
                       A.stride(0), B.stride(0), c.stride(0), ta, tb, (int)act, split, out_fp32, accumulate, (int)cfg,
                       cur_stream(), colp);
    };
    int rc = launch(cp);
    if (rc == -3) {  // this config cannot emit column partials: plain GEMM + one reduction pass over C
        rc = launch(nullptr);
        TORCH_CHECK(rc == 0, "rn_gemm rejected shape M=", M, " N=", N, " K=", Kp);
        Tensor part = at::empty({(int64_t)(rn_bias_act_grad_splits((int)M, (int)N) + 32) * N}, a.options().dtype(at::kFloat));
        rn_bias_act_grad(c.data_ptr(), nullptr, c.data_ptr(), nullptr, bias_grad->data_ptr(), part.data_ptr<float>(),
                         (int)M, (int)N, 0, 1, 1, cur_stream());
        return c;
    }
    TORCH_CHECK(rc == 0, "rn_gemm rejected shape M=", M, " N=", N, " K=", Kp);
    if (want_bg) {
        Tensor tmp = at::empty({rn_colsum_ws((int)N)}, a.options().dtype(at::kFloat));
        rn_colsum_f32(colpart.data_ptr<float>(), (int)rn_gemm_colpart_rows((int)cfg, (int)M), (int)N, tmp.data_ptr<float>(),
                      bias_grad->data_ptr(), 1, cur_stream());
    }
    return c;
}

// returns (dH, db) with db in bf16 (the parameter dtype)
std::tuple<Tensor, Tensor> bias_act_grad(const Tensor& dy, const optional<Tensor>& h, int64_t act, bool want_bias,
                                         const optional<Tensor>& db_accum) {
    CHECK_CUDA(dy); CHECK_BF16(dy); CHECK_CONTIG(dy);
    GUARD(dy);
    const int M = dy.size(0), N = dy.size(1);
    Tensor dh = act != 0 ? at::empty_like(dy) : dy;
    const bool accum = db_accum && db_accum->defined();
    if (accum) { CHECK_BF16(*db_accum); TORCH_CHECK(db_accum->numel() == N && db_accum->is_contiguous()); }
    Tensor db = accum ? *db_accum : at::empty({want_bias ? N : 0}, dy.options());
    Tensor part = at::empty({want_bias ? (int64_t)(rn_bias_act_grad_splits(M, N) + 32) * N : 1},
                            dy.options().dtype(at::kFloat));
    if (act != 0) { TORCH_CHECK(h && h->defined(), "activation grad needs the pre-activation"); CHECK_CONTIG(*h); }
    if (M > 0)
        rn_bias_act_grad(dy.data_ptr(), optr(h), dh.data_ptr(), nullptr, want_bias ? db.data_ptr() : nullptr,
                         part.data_ptr<float>(), M, N, (int)act, want_bias, accum, cur_stream());
    else if (want_bias && !accum) db.zero_();
    return {dh, db};
}

// ------------------------------------------------------------------ elementwise
Tensor act_fwd(const Tensor& x, int64_t kind) {
    CHECK_BF16(x); CHECK_CONTIG(x); GUARD(x);
    Tensor y = at::empty_like(x);
    rn_act_fwd(x.data_ptr(), y.data_ptr(), x.numel(), (int)kind, cur_stream());
    return y;
}
Tensor act_bwd(const Tensor& dy, const Tensor& x, int64_t kind) {
    CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_CONTIG(x); GUARD(dy);
    Tensor dx = at::empty_like(dy);
    rn_act_bwd(dy.data_ptr(), x.data_ptr(), dx.data_ptr(), dy.numel(), (int)kind, cur_stream());
    return dx;
}
// seed_buf: optional 1-element int64 DEVICE tensor (from rng_next) — the kernel reads its seed there,
// so a captured hipGraph replays with a fresh draw each step
const uint64_t* seed_ptr(const optional<Tensor>& sb) {
    if (!(sb && sb->defined())) return nullptr;
    TORCH_CHECK(sb->scalar_type() == at::kLong && sb->numel() >= 1 && sb->is_cuda(), "seed_buf: 1-element int64 GPU tensor");
    return (const uint64_t*)sb->data_ptr();
}
Tensor dropout_fwd(const Tensor& x, double p, int64_t seed, const optional<Tensor>& seed_buf) {
    CHECK_BF16(x); CHECK_CONTIG(x); GUARD(x);
    Tensor y = at::empty_like(x);
    rn_dropout(x.data_ptr(), y.data_ptr(), x.numel(), (float)p, (uint64_t)seed, seed_ptr(seed_buf), cur_stream());
    return y;
}
void rng_next(const Tensor& state, const Tensor& out) {
    TORCH_CHECK(state.scalar_type() == at::kLong && out.scalar_type() == at::kLong && state.is_cuda() && out.is_cuda());
    GUARD(state);
    rn_rng_next(state.data_ptr(), out.data_ptr(), cur_stream());
}
Tensor add_act(const Tensor& a, const Tensor& b, bool relu) {
    CHECK_BF16(a); CHECK_CONTIG(a); CHECK_CONTIG(b); GUARD(a);
    TORCH_CHECK(a.sizes() == b.sizes());
    Tensor y = at::empty_like(a);
    rn_add(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), relu, cur_stream());
    return y;
}

// ------------------------------------------------------------------ softmax / xent
Tensor softmax_fwd(const Tensor& x, double scale) {
    CHECK_BF16(x); CHECK_CONTIG(x); GUARD(x);
    Tensor y = at::empty_like(x);
    if (x.numel()) rn_softmax_fwd(x.data_ptr(), y.data_ptr(), x.size(0), x.size(1), (float)scale, cur_stream());
    return y;
}
Tensor softmax_bwd(const Tensor& dy, const Tensor& y, double scale) {
    CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_CONTIG(y); GUARD(dy);
    Tensor dx = at::empty_like(dy);
    if (dy.numel()) rn_softmax_bwd(dy.data_ptr(), y.data_ptr(), dx.data_ptr(), y.size(0), y.size(1), (float)scale, cur_stream());
    return dx;
}
std::tuple<Tensor, Tensor> xent_fwd(const Tensor& logits, const Tensor& target, int64_t nvalid, int64_t ignore,
                                    bool write_grad) {
    CHECK_BF16(logits); CHECK_CONTIG(logits); GUARD(logits);
    TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous());
    const int M = logits.size(0), V = logits.size(1);
    Tensor loss = at::empty({M}, logits.options().dtype(at::kFloat));
    Tensor lse = at::empty({M}, logits.options().dtype(at::kFloat));
    if (M) rn_xent_fwd(logits.data_ptr(), target.data_ptr<int64_t>(), loss.data_ptr<float>(), lse.data_ptr<float>(), M, V,
                       (int)nvalid, (long)ignore, write_grad, cur_stream());
    return {loss, lse};
}
// the fp8 LM head's loss: as xent_fwd(write_grad) but the gradient goes to q8 (uint8 [M][V]) as e5m2 of
// (softmax - onehot) · 2^15; the logits are left unchanged
std::tuple<Tensor, Tensor> xent_fwd_q8(const Tensor& logits, const Tensor& target, int64_t nvalid, int64_t ignore,
                                       const Tensor& q8) {
    CHECK_BF16(logits); CHECK_CONTIG(logits); GUARD(logits);
    TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous());
    TORCH_CHECK(q8.scalar_type() == at::kByte && q8.is_contiguous() && q8.sizes() == logits.sizes());
    const int M = logits.size(0), V = logits.size(1);
    Tensor loss = at::empty({M}, logits.options().dtype(at::kFloat));
    Tensor lse = at::empty({M}, logits.options().dtype(at::kFloat));
    if (M) {
        int rc = rn_xent_fwd_q8(logits.data_ptr(), target.data_ptr<int64_t>(), loss.data_ptr<float>(),
                                lse.data_ptr<float>(), M, V, (int)nvalid, (long)ignore, q8.data_ptr(), cur_stream());
        TORCH_CHECK(rc == 0, "xent_fwd_q8: V must be a multiple of 8 and <= 65536, got ", V);
    }
    return {loss, lse};
}
void xent_bwd(const Tensor& logits, const Tensor& target, const Tensor& lse, const Tensor& gscale, const Tensor& grad,
              int64_t nvalid, int64_t ignore) {
    CHECK_BF16(logits); GUARD(logits);
    TORCH_CHECK(gscale.scalar_type() == at::kFloat && gscale.is_cuda());
    const int M = logits.size(0), V = logits.size(1);
    if (M) rn_xent_bwd(logits.data_ptr(), target.data_ptr<int64_t>(), lse.data_ptr<float>(), gscale.data_ptr<float>(),
                       grad.data_ptr(), M, V, (int)nvalid, (long)ignore, cur_stream());
}

// ------------------------------------------------------------------ layernorm
std::tuple<Tensor, Tensor, Tensor, Tensor> layernorm_fwd(const Tensor& x, const optional<Tensor>& r, const Tensor& w,
                                                         const optional<Tensor>& b, double eps) {
    CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); GUARD(x);
    const int M = x.size(0), E = x.size(1);
    Tensor y = at::empty_like(x);
    Tensor h = (r && r->defined()) ? at::empty_like(x) : x;
    Tensor mean = at::empty({M}, x.options().dtype(at::kFloat));
    Tensor rstd = at::empty({M}, x.options().dtype(at::kFloat));
    if (M) {
        int rc = rn_ln_fwd(x.data_ptr(), optr(r), w.data_ptr(), optr(b), y.data_ptr(), h.data_ptr(), mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), M, E, (float)eps, cur_stream(), nullptr, nullptr);
        TORCH_CHECK(rc == 0, "layernorm: E must be a multiple of 8 and <= 8192, got ", E);
    }
    return {y, h, mean, rstd};
}
// LayerNorm whose output also comes out as e4m3 for the consumer's fp8 GEMM: `state` is that
// GEMM's activation Fp8State slot (delayed scaling: rolled here, amax recorded by the kernel)
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> layernorm_fwd_q8(const Tensor& x, const optional<Tensor>& r,
                                                                    const Tensor& w, const optional<Tensor>& b,
                                                                    double eps, const Tensor& state) {
    CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); GUARD(x);
    TORCH_CHECK(state.scalar_type() == at::kFloat && state.numel() >= 4 && state.is_cuda() && state.is_contiguous());
    const int M = x.size(0), E = x.size(1);
    Tensor y = at::empty_like(x);
    Tensor h = (r && r->defined()) ? at::empty_like(x) : x;
    Tensor mean = at::empty({M}, x.options().dtype(at::kFloat));
    Tensor rstd = at::empty({M}, x.options().dtype(at::kFloat));
    Tensor q = at::empty(x.sizes(), x.options().dtype(at::kByte));
    rn_fp8_roll(state.data_ptr<float>(), cur_stream());
    if (M) {
        int rc = rn_ln_fwd(x.data_ptr(), optr(r), w.data_ptr(), optr(b), y.data_ptr(), h.data_ptr(), mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), M, E, (float)eps, cur_stream(), q.data_ptr(), state.data_ptr<float>());
        TORCH_CHECK(rc == 0, "layernorm: E must be a multiple of 8 and <= 8192, got ", E);
    }
    return {y, h, mean, rstd, q};
}
std::tuple<Tensor, Tensor, Tensor> layernorm_bwd(const Tensor& dy, const optional<Tensor>& gh, const Tensor& h,
                                                 const Tensor& w, const Tensor& mean, const Tensor& rstd,
                                                 const optional<Tensor>& dw_accum, const optional<Tensor>& db_accum,
                                                 const optional<Tensor>& dxs_accum, const optional<Tensor>& q8,
                                                 const optional<Tensor>& q8_state) {
    CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_CONTIG(h); GUARD(dy);
    if (dxs_accum && dxs_accum->defined()) {
        CHECK_BF16(*dxs_accum);
        TORCH_CHECK(dxs_accum->numel() == dy.size(1) && dxs_accum->is_contiguous());
    }
    const int M = dy.size(0), E = dy.size(1);
    Tensor dx = at::empty_like(dy);
    const bool accum = dw_accum && dw_accum->defined() && db_accum && db_accum->defined();
    Tensor dw = accum ? *dw_accum : at::empty({E}, w.options());  // parameter dtype (bf16)
    Tensor db = accum ? *db_accum : at::empty({E}, w.options());
    Tensor part = at::empty({rn_ln_bwd_ws(M, E)}, dy.options().dtype(at::kFloat));
    // q8 + q8_state: dx also in e5m2 for the fp8 linear that produced the LayerNorm input (its gradient slot)
    void* q8_ptr = nullptr;
    float* q8_st = nullptr;
    if (q8 && q8->defined()) {
        TORCH_CHECK(q8->scalar_type() == at::kByte && q8->is_contiguous() && q8->numel() == dy.numel() &&
                    q8->device() == dy.device(), "layernorm_bwd: q8 must be a contiguous uint8 twin of dy");
        TORCH_CHECK(q8_state && q8_state->defined() && q8_state->scalar_type() == at::kFloat && q8_state->numel() >= 4 &&
                    q8_state->device() == dy.device(), "layernorm_bwd: q8 needs a 4-float fp32 scale slot");
        q8_ptr = q8->data_ptr();
        q8_st = q8_state->data_ptr<float>();
    }
    if (M) {
        int rc = rn_ln_bwd(dy.data_ptr(), optr(gh), h.data_ptr(), w.data_ptr(), mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), dx.data_ptr(), nullptr, nullptr, dw.data_ptr(), db.data_ptr(),
                           (dxs_accum && dxs_accum->defined()) ? dxs_accum->data_ptr() : nullptr,
                           part.data_ptr<float>(), M, E, accum, cur_stream(), q8_ptr, q8_st);
        TORCH_CHECK(rc == 0, "layernorm_bwd: unsupported E=", E);
    } else if (!accum) { dw.zero_(); db.zero_(); }
    return {dx, dw, db};
}

// ------------------------------------------------------------------ embedding
// ViT token join: x[b] = concat(cls, patch[b]) + pos — patch (B, P, E), cls (E), pos (P + 1, E), all bf16
Tensor vit_join_fwd(const Tensor& patch, const Tensor& cls, const Tensor& pos) {
    CHECK_BF16(patch); CHECK_CONTIG(patch); CHECK_BF16(cls); CHECK_CONTIG(cls); CHECK_BF16(pos); CHECK_CONTIG(pos);
    GUARD(patch);
    TORCH_CHECK(patch.dim() == 3, "vit_join_fwd: patch must be (B, P, E)");
    const int B = patch.size(0), P = patch.size(1), E = patch.size(2);
    TORCH_CHECK(E % 8 == 0 && cls.numel() == E && pos.numel() == (long)(P + 1) * E, "vit_join_fwd: shapes");
    Tensor out = at::empty({B, P + 1, E}, patch.options());
    if (B) rn_vit_join_fwd(patch.data_ptr(), cls.data_ptr(), pos.data_ptr(), out.data_ptr(), B, P, E, cur_stream());
    return out;
}
// backward: returns dpatch (B, P, E); gcls (E) and gpos (P + 1, E) are ACCUMULATED into (bf16)
Tensor vit_join_bwd(const Tensor& dx, const Tensor& gcls, const Tensor& gpos) {
    CHECK_BF16(dx); CHECK_CONTIG(dx); CHECK_BF16(gcls); CHECK_CONTIG(gcls); CHECK_BF16(gpos); CHECK_CONTIG(gpos);
    GUARD(dx);
    TORCH_CHECK(dx.dim() == 3, "vit_join_bwd: dx must be (B, P + 1, E)");
    const int B = dx.size(0), P = dx.size(1) - 1, E = dx.size(2);
    TORCH_CHECK(P >= 0 && E % 8 == 0 && gcls.numel() == E && gpos.numel() == (long)(P + 1) * E, "vit_join_bwd: shapes");
    Tensor dpatch = at::empty({B, P, E}, dx.options());
    if (B) rn_vit_join_bwd(dx.data_ptr(), dpatch.data_ptr(), gcls.data_ptr(), gpos.data_ptr(), B, P, E, cur_stream());
    return dpatch;
}

Tensor embedding_fwd(const Tensor& ids, const Tensor& wte, const optional<Tensor>& wpe) {
    CHECK_BF16(wte); CHECK_CONTIG(wte); GUARD(wte);
    TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous());
    const int E = wte.size(1);
    TORCH_CHECK(E % 8 == 0, "embedding width must be a multiple of 8");
    const int T = ids.dim() >= 2 ? ids.size(-1) : ids.numel();
    const int rows = ids.numel();
    if (wpe && wpe->defined()) TORCH_CHECK(wpe->size(0) >= T, "sequence longer than the position table");
    auto shape = ids.sizes().vec();
    shape.push_back(E);
    Tensor x = at::empty(shape, wte.options());
    if (rows)
        rn_emb_fwd(ids.data_ptr<int64_t>(), wte.data_ptr(), optr(wpe), x.data_ptr(), rows, T, E, (int)wte.size(0),
                   cur_stream());
    return x;
}
std::tuple<Tensor, Tensor> embedding_bwd(const Tensor& dx, const Tensor& ids, int64_t V, int64_t Tp) {
    CHECK_BF16(dx); CHECK_CONTIG(dx); GUARD(dx);
    const int E = dx.size(-1);
    const int T = ids.dim() >= 2 ? ids.size(-1) : ids.numel();
    const int B = ids.numel() / std::max(T, 1);
    Tensor d32 = at::empty({V * E}, dx.options().dtype(at::kFloat));
    Tensor dwte = at::empty({V, E}, dx.options());
    Tensor dwpe = at::empty({Tp, E}, dx.options());
    rn_emb_bwd(ids.data_ptr<int64_t>(), dx.data_ptr(), d32.data_ptr<float>(), dwte.data_ptr(), Tp ? dwpe.data_ptr() : nullptr,
               B, T, (int)Tp, (int)V, E, cur_stream());
    return {dwte, dwpe};
}

// Direct-accumulate embedding backward: gwte/gwpe (flat gradient views) += scatter.
// The fp32 scratch and owner table are persistent per (device, V, E) and are left
// in their initial state by every call, so the op is hipGraph-capturable.
void embedding_bwd_acc(const Tensor& dx, const Tensor& ids, const Tensor& gwte, const optional<Tensor>& gwpe) {
    CHECK_BF16(dx); CHECK_CONTIG(dx); CHECK_BF16(gwte); CHECK_CONTIG(gwte); GUARD(dx);
    TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous());
    const int64_t V = gwte.size(0), E = gwte.size(1);
    TORCH_CHECK(dx.size(-1) == E && E % 4 == 0, "embedding_bwd_acc: width mismatch / E % 4");
    const int T = ids.dim() >= 2 ? ids.size(-1) : ids.numel();
    const int B = ids.numel() / std::max(T, 1);
    if (gwpe && gwpe->defined()) {
        CHECK_BF16(*gwpe); CHECK_CONTIG(*gwpe);
        TORCH_CHECK(gwpe->size(0) >= T && gwpe->size(1) == E);
    }
    // REPLICANN_DETERMINISTIC=1: 64-bit fixed-point scratch, order-independent integer atomics
    const char* de = std::getenv("REPLICANN_DETERMINISTIC");
    const bool det = de && de[0] == '1';
    static std::map<std::tuple<int, int64_t, int64_t, int>, std::pair<Tensor, Tensor>> scratch;
    static std::mutex mu;
    std::pair<Tensor, Tensor> buf;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto key = std::make_tuple((int)dx.get_device(), V, E, (int)det);
        auto it = scratch.find(key);
        if (it == scratch.end()) {
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            (void)hipStreamIsCapturing(cur_stream(), &cs);
            TORCH_CHECK(cs == hipStreamCaptureStatusNone,
                        "embedding_bwd_acc: first call must be eager (scratch allocation)");
            Tensor d32 = at::zeros({V * E * (det ? 2 : 1)}, dx.options().dtype(at::kFloat));
            Tensor own = at::full({V}, -1, dx.options().dtype(at::kInt));
            it = scratch.emplace(key, std::make_pair(d32, own)).first;
        }
        buf = it->second;
    }
    if (ids.numel() && det)
        rn_emb_bwd_acc_det(ids.data_ptr<int64_t>(), dx.data_ptr(), buf.first.data_ptr(),
                           reinterpret_cast<unsigned*>(buf.second.data_ptr<int>()), gwte.data_ptr(),
                           (gwpe && gwpe->defined()) ? gwpe->data_ptr() : nullptr, B, T, (int)E, (int)V, cur_stream());
    else if (ids.numel())
        rn_emb_bwd_acc(ids.data_ptr<int64_t>(), dx.data_ptr(), buf.first.data_ptr<float>(),
                       reinterpret_cast<unsigned*>(buf.second.data_ptr<int>()), gwte.data_ptr(),
                       (gwpe && gwpe->defined()) ? gwpe->data_ptr() : nullptr, B, T, (int)E, (int)V, cur_stream());
}

// ------------------------------------------------------------------ optimizers
void sumsq(const Tensor& g, const Tensor& normbuf) {
    CHECK_CONTIG(g); GUARD(g);
    TORCH_CHECK(normbuf.scalar_type() == at::kFloat && normbuf.numel() >= 2);
    Tensor part = at::empty({rn_norm_ws_floats()}, g.options().dtype(at::kFloat));
    rn_sumsq(g.data_ptr(), g.numel(), g.scalar_type() == at::kBFloat16, part.data_ptr<float>(), normbuf.data_ptr<float>(),
             cur_stream());
}
void opt_prep(const Tensor& state, double base_lr, double warmup, double total, double min_ratio, bool cosine,
              double lr_override, double b1, double b2) {
    GUARD(state);
    TORCH_CHECK(state.scalar_type() == at::kFloat && state.numel() >= 8);
    rn_opt_prep(state.data_ptr<float>(), (float)base_lr, (float)warmup, (float)total, (float)min_ratio, cosine,
                (float)lr_override, (float)b1, (float)b2, cur_stream());
}
void adamw_step(const Tensor& p, const Tensor& master, const Tensor& g, const Tensor& m, const Tensor& v,
                const Tensor& wdm, const Tensor& state, double b1, double b2, double eps, double wd, double gscale,
                double clip, bool stochastic_round) {
    CHECK_BF16(p); GUARD(p);
    TORCH_CHECK(master.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat);
    TORCH_CHECK(p.numel() == master.numel() && p.numel() == g.numel() && wdm.numel() * 64 >= p.numel());
    int rc = rn_adamw(p.data_ptr(), master.data_ptr<float>(), g.data_ptr(), g.scalar_type() == at::kBFloat16,
                      m.data_ptr<float>(), v.data_ptr<float>(), wdm.data_ptr<uint8_t>(), state.data_ptr<float>(),
                      p.numel(), (float)b1, (float)b2, (float)eps, (float)wd, (float)gscale, (float)clip,
                      stochastic_round ? 1 : 0, cur_stream());
    TORCH_CHECK(rc == 0, "adamw: flat buffer length must be a multiple of 8");
}
void sgd_step(const Tensor& p, const Tensor& master, const Tensor& g, const Tensor& buf, const Tensor& wdm,
              const Tensor& state, double mom, double wd, bool nesterov, double gscale, double clip) {
    CHECK_BF16(p); GUARD(p);
    rn_sgd(p.data_ptr(), master.data_ptr<float>(), g.data_ptr(), g.scalar_type() == at::kBFloat16, buf.data_ptr<float>(),
           wdm.data_ptr<uint8_t>(), state.data_ptr<float>(), p.numel(), (float)mom, (float)wd, nesterov, (float)gscale,
           (float)clip, cur_stream());
}

// ------------------------------------------------------------------ attention
void strides_bth(const Tensor& t, std::vector<long>& s) {
    TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, "attention tensors must be (B, T, H, D) with unit D stride");
    s.push_back(t.stride(0)); s.push_back(t.stride(1)); s.push_back(t.stride(2));
}
// decode-step QKV projection with the K|V cache append fused into the epilogue (gemm_skinny.hip):
// x (M, K), w (N, K), kv (M, L, 2, H, D) contiguous cache, pos: 1 int64 device row index
Tensor linear_kv(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, const Tensor& kv, const Tensor& pos) {
    CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(kv); GUARD(x);
    TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && w.dim() == 2 && w.stride(1) == 1, "linear_kv: 2-D row-major operands");
    const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
    TORCH_CHECK(w.size(1) == K, "linear_kv: inner dims differ");
    TORCH_CHECK(kv.dim() == 5 && kv.is_contiguous() && kv.size(0) == M && kv.size(2) == 2, "linear_kv: kv must be (M, L, 2, H, D)");
    const int64_t kvw = kv.size(2) * kv.size(3) * kv.size(4);
    TORCH_CHECK(kvw <= N, "linear_kv: cache row wider than the projection");
    TORCH_CHECK(pos.scalar_type() == at::kLong && pos.numel() == 1 && pos.is_cuda(), "linear_kv: pos must be 1 int64 on the device");
    TORCH_CHECK(w.device() == x.device() && kv.device() == x.device() && pos.device() == x.device() &&
                    (!bias || !bias->defined() || bias->device() == x.device()),
                "linear_kv: x, w, bias, kv and pos must be on one device");
    if (bias && bias->defined()) { CHECK_BF16(*bias); TORCH_CHECK(bias->numel() == N && bias->is_contiguous()); }
    Tensor c = at::empty({M, N}, x.options());
    const int rc = rn_gemm_skinny_kv(x.data_ptr(), w.data_ptr(), optr(bias), c.data_ptr(), (int)M, (int)N, (int)K,
                                     x.stride(0), w.stride(0), c.stride(0), kv.data_ptr(), pos.data_ptr<int64_t>(),
                                     kv.stride(0), kv.stride(1), (int)(N - kvw), cur_stream());
    TORCH_CHECK(rc == 0, "linear_kv: unsupported shape M=", M, " K=", K, " (M <= 64, K % 8 == 0)");
    return c;
}

// one-query attention over a KV cache (decode step, attention_decode.hip): q (B, 1, H, 64), k / v
// (B, Tk, H, 64) strided views, mask: Tk fp32 additive shared by the batch (or none)
Tensor attn_decode(const Tensor& q, const Tensor& k, const Tensor& v, const optional<Tensor>& mask, double scale) {
    CHECK_BF16(q); CHECK_BF16(k); CHECK_BF16(v); GUARD(q);
    TORCH_CHECK(q.dim() == 4 && q.size(1) == 1, "attn_decode: one query per (batch, head)");
    const int B = q.size(0), H = q.size(2), D = q.size(3), Tk = k.size(1);
    TORCH_CHECK(k.dim() == 4 && v.dim() == 4, "attn_decode: k / v must be (B, Tk, H, D)");
    TORCH_CHECK(k.size(0) == B && v.size(0) == B && k.size(2) == H && v.size(2) == H && v.size(1) == Tk &&
                    k.size(3) == D && v.size(3) == D,
                "attn_decode: shape mismatch (q ", q.sizes(), ", k ", k.sizes(), ", v ", v.sizes(), ")");
    TORCH_CHECK(k.device() == q.device() && v.device() == q.device(), "attn_decode: q, k, v on different devices");
    // the kernel reads 16-B vectors: base pointers and every non-unit stride 16-B aligned
    for (const Tensor* t : {&q, &k, &v})
        TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0 && t->stride(3) == 1,
                    "attn_decode: q / k / v need a 16-byte aligned base and a contiguous head dimension");
    if (mask && mask->defined())
        TORCH_CHECK(mask->scalar_type() == at::kFloat && mask->is_contiguous() && mask->numel() == Tk &&
                        mask->device() == q.device(),
                    "attn_decode: mask must be Tk contiguous fp32 values on q's device");
    Tensor o = at::empty({B, 1, H, D}, q.options());
    std::vector<long> s;
    std::vector<long> t;
    strides_bth(q, t); s.push_back(t[0]); s.push_back(t[2]); t.clear();
    strides_bth(k, t); s.insert(s.end(), t.begin(), t.end()); t.clear();
    strides_bth(v, t); s.insert(s.end(), t.begin(), t.end()); t.clear();
    strides_bth(o, t); s.push_back(t[0]); s.push_back(t[2]);
    const int rc = rn_attn_decode(q.data_ptr(), k.data_ptr(), v.data_ptr(),
                                  mask && mask->defined() ? mask->data_ptr<float>() : nullptr, o.data_ptr(), B, H, Tk, D,
                                  s.data(), (float)scale, cur_stream());
    TORCH_CHECK(rc == 0, "attn_decode: unsupported shape D=", D, " Tk=", Tk, " (D == 64, Tk <= 1024)");
    return o;
}

std::tuple<Tensor, Tensor> attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, const optional<Tensor>& bias,
                                    double scale, bool causal, double p, int64_t seed,
                                    const optional<Tensor>& seed_buf) {
    CHECK_BF16(q); CHECK_BF16(k); CHECK_BF16(v); GUARD(q);
    const int B = q.size(0), Tq = q.size(1), H = q.size(2), D = q.size(3), Tk = k.size(1);
    Tensor o = at::empty({B, Tq, H, D}, q.options());
    Tensor lse = at::empty({B, H, Tq}, q.options().dtype(at::kFloat));
    std::vector<long> s;
    strides_bth(q, s); strides_bth(k, s); strides_bth(v, s); strides_bth(o, s);
    int bias_b = 1;
    if (bias && bias->defined()) {
        TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->dim() == 3 && bias->is_contiguous());
        bias_b = bias->size(0);
    }
    if (B * H * Tq == 0) return {o, lse};
    int rc = rn_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(),
                         bias && bias->defined() ? bias->data_ptr<float>() : nullptr, bias_b, s.data(), B, H, Tq, Tk, D,
                         (float)scale, causal, (float)p, (uint64_t)seed, seed_ptr(seed_buf), cur_stream());
    TORCH_CHECK(rc == 0, "attention: unsupported shape D=", D, " Tk=", Tk);
    return {o, lse};
}
// q8 / q8st / q8_only: see AttnArgs (attention.hip); returns false (nothing launched) when the kernels
// cannot emit e5m2 for this shape
bool attn_bwd_impl(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                   const Tensor& lse, const optional<Tensor>& bias, double scale, bool causal, double p, int64_t seed,
                   const Tensor& dq, const Tensor& dk, const Tensor& dv, const optional<Tensor>& qkv_bias_grad = {},
                   const optional<Tensor>& seed_buf = {}, void* q8 = nullptr, float* q8st = nullptr, bool q8_only = false) {
    GUARD(q);
    const int B = q.size(0), Tq = q.size(1), H = q.size(2), D = q.size(3), Tk = k.size(1);
    std::vector<long> s;
    for (const Tensor* t : {&q, &k, &v, &o, &dout, &dq, &dk, &dv}) strides_bth(*t, s);
    Tensor delta = at::empty({B, H, Tq}, q.options().dtype(at::kFloat));
    Tensor dk32, dv32;  // (no scratch: the generic path's dK/dV kernel writes dk / dv directly)
    int bias_b = bias && bias->defined() ? bias->size(0) : 1;
    if (B * H * Tq == 0) return true;
    // packed-QKV bias gradient: per-64-row-block column partials from the kernels, then one reduction
    Tensor bsum;
    const bool want_bg = qkv_bias_grad && qkv_bias_grad->defined();
    const int nblk = (Tq + 63) / 64;
    if (want_bg) {
        CHECK_BF16(*qkv_bias_grad);
        TORCH_CHECK(qkv_bias_grad->numel() == 3L * H * D && qkv_bias_grad->is_contiguous() && rn_attn_is_fast(D) &&
                    Tq == Tk, "qkv bias gradient: packed self-attention with head_dim 32, 64 or 128 only");
        bsum = at::empty({(int64_t)B * nblk, 3L * H * D}, q.options().dtype(at::kFloat));
    }
    Tensor q8part = q8 ? at::empty({rn_attn_q8_part_floats(B, H, Tq, Tk)}, q.options().dtype(at::kFloat)) : Tensor();
    int rc = rn_attn_bwd(dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(),
                         bias && bias->defined() ? bias->data_ptr<float>() : nullptr, bias_b, dq.data_ptr(), dk.data_ptr(),
                         dv.data_ptr(), delta.data_ptr<float>(), dk32.defined() ? dk32.data_ptr<float>() : nullptr,
                         dv32.defined() ? dv32.data_ptr<float>() : nullptr, s.data(), B, H, Tq, Tk, D, (float)scale,
                         causal, (float)p, (uint64_t)seed, seed_ptr(seed_buf), want_bg ? bsum.data_ptr<float>() : nullptr,
                         q8, q8st, q8_only ? 1 : 0, q8 ? q8part.data_ptr<float>() : nullptr, cur_stream());
    if (rc == -3 && q8) return false;
    TORCH_CHECK(rc == 0, "attention backward: unsupported shape D=", D);
    if (want_bg) {
        const int C = 3 * H * D;
        Tensor tmp = at::empty({rn_colsum_ws(C)}, q.options().dtype(at::kFloat));
        rn_colsum_f32(bsum.data_ptr<float>(), B * nblk, C, tmp.data_ptr<float>(), qkv_bias_grad->data_ptr(), 1,
                      cur_stream());
    }
    return true;
}
std::tuple<Tensor, Tensor, Tensor> attn_bwd(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v,
                                            const Tensor& o, const Tensor& lse, const optional<Tensor>& bias,
                                            double scale, bool causal, double p, int64_t seed,
                                            const optional<Tensor>& seed_buf) {
    Tensor dq = at::empty(q.sizes(), q.options());
    Tensor dk = at::empty(k.sizes(), k.options());
    Tensor dv = at::empty(v.sizes(), v.options());
    attn_bwd_impl(dout, q, k, v, o, lse, bias, scale, causal, p, seed, dq, dk, dv, {}, seed_buf);
    return {dq, dk, dv};
}
void attn_bwd_out(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                  const Tensor& lse, const optional<Tensor>& bias, double scale, bool causal, double p, int64_t seed,
                  const Tensor& dq, const Tensor& dk, const Tensor& dv, const optional<Tensor>& qkv_bias_grad,
                  const optional<Tensor>& seed_buf) {
    attn_bwd_impl(dout, q, k, v, o, lse, bias, scale, causal, p, seed, dq, dk, dv, qkv_bias_grad, seed_buf);
}
// the same with the packed dQKV also (q8_only: only) written as e5m2 into q8 (uint8, dQKV's shape) with the
// delayed-scaling slot q8_state (rolled here); false = this shape cannot (nothing launched)
bool attn_bwd_out_q8(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                     const Tensor& lse, const optional<Tensor>& bias, double scale, bool causal, double p, int64_t seed,
                     const Tensor& dq, const Tensor& dk, const Tensor& dv, const optional<Tensor>& qkv_bias_grad,
                     const optional<Tensor>& seed_buf, const Tensor& q8, const Tensor& q8_state, bool q8_only) {
    TORCH_CHECK(q8.scalar_type() == at::kByte && q8.is_cuda() && q8.device() == q.device(), "attn q8: uint8 on the device");
    TORCH_CHECK(q8_state.scalar_type() == at::kFloat && q8_state.numel() >= 4 && q8_state.device() == q.device());
    // the e5m2 image uses element offsets from dq: q8 is the byte twin of the packed dQKV dq / dk / dv view
    TORCH_CHECK(q8.numel() == 3 * dq.numel() && dq.data_ptr() < dk.data_ptr() && dk.data_ptr() < dv.data_ptr(),
                "attn q8: the e5m2 twin of a packed (B, T, 3, H, D) dQKV");
    return attn_bwd_impl(dout, q, k, v, o, lse, bias, scale, causal, p, seed, dq, dk, dv, qkv_bias_grad, seed_buf,
                         q8.data_ptr(), q8_state.data_ptr<float>(), q8_only);
}

// ------------------------------------------------------------------ implicit-GEMM conv
// x / dy NHWC bf16 contiguous, w (OC, KH, KW, C) contiguous; the gathered tensor's channel count
// must be a multiple of 64 (callers check conv_implicit_ok first).
// stats: also return [ceil(M/256)][2·OC] fp32 per-256-row Σ | Σ² of y (the following BatchNorm's batch
// statistics, reduced in batchnorm_fwd instead of re-reading y)
static std::tuple<Tensor, Tensor> conv_fwd_implicit_impl(const Tensor& x, const Tensor& w,
                                                         const optional<Tensor>& bias, int64_t S, int64_t P,
                                                         bool stats) {
    CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); CHECK_CONTIG(w); GUARD(x);
    const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
    const int OC = w.size(0), KH = w.size(1), KW = w.size(2);
    TORCH_CHECK(w.size(3) == C, "conv: channel mismatch");
    const int OH = (H + 2 * P - KH) / S + 1, OW = (W + 2 * P - KW) / S + 1;
    Tensor y = at::empty({N, OH, OW, OC}, x.options());
    const int M = N * OH * OW, K = KH * KW * C;
    // 3×3 / stride 1 / pad 1, 64 → 64 channels (ResNet layer 1): the halo-tile kernel (conv3x3.hip); its
    // statistics partials are per tile of whole image rows instead of per 256 pixels
    const bool has_bias = bias && bias->defined();
    if (KH == 3 && KW == 3 && S == 1 && P == 1 && C == 64 && OC == 64 && !has_bias && M > 0) {
        const int tiles = rn_conv3x3_tiles(N, H, W);
        if (tiles > 0) {
            Tensor part3 = stats ? at::empty({tiles, 2L * OC}, x.options().dtype(at::kFloat))
                                 : at::empty({0}, x.options().dtype(at::kFloat));
            if (rn_conv3x3(x.data_ptr(), w.data_ptr(), y.data_ptr(), stats ? part3.data_ptr<float>() : nullptr, N, H,
                           W, 0, 0, cur_stream()) == 0)
                return {y, part3};
        }
    }
    Tensor part = stats ? at::empty({(M + 255) / 256, 2L * OC}, x.options().dtype(at::kFloat))
                        : at::empty({0}, x.options().dtype(at::kFloat));
    if (M == 0) return {y, part};
    float* cp = stats ? part.data_ptr<float>() : nullptr;
    if (bias && bias->defined()) { CHECK_BF16(*bias); TORCH_CHECK(bias->numel() == OC); }
    const int rc = rn_conv_gemm(1, x.data_ptr(), w.data_ptr(), y.data_ptr(), optr(bias), nullptr, M, OC, K, 0, K, OC, H,
                                W, C, OH, OW, KH, KW, (int)S, (int)P, C, 0, 0, 1, 0, 0, cp, cur_stream());
    TORCH_CHECK(rc == 0, "implicit conv fwd: unsupported geometry");
    return {y, part};
}
Tensor conv_fwd_implicit(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, int64_t S, int64_t P) {
    return std::get<0>(conv_fwd_implicit_impl(x, w, bias, S, P, false));
}
std::tuple<Tensor, Tensor> conv_fwd_implicit_stats(const Tensor& x, const Tensor& w, const optional<Tensor>& bias,
                                                   int64_t S, int64_t P) {
    return conv_fwd_implicit_impl(x, w, bias, S, P, true);
}
// out + accumulate: dx is added into `out` in the GEMM epilogue (a second gradient of the same input)
static Tensor grad_out(const optional<Tensor>& out, bool accumulate, at::IntArrayRef shape, const Tensor& like,
                       const char* what) {
    if (out && out->defined()) {
        CHECK_BF16(*out); CHECK_CONTIG(*out);
        TORCH_CHECK(out->sizes() == shape && out->device() == like.device(), what, ": out shape");
        return *out;
    }
    TORCH_CHECK(!accumulate, what, ": accumulate needs out");
    return at::empty(shape, like.options());
}
Tensor conv_dgrad_implicit(const Tensor& dy, const Tensor& w, int64_t H, int64_t W, int64_t P, const optional<Tensor>& out,
                           bool accumulate) {  // stride 1
    CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_BF16(w); CHECK_CONTIG(w); GUARD(dy);
    const int N = dy.size(0), OH = dy.size(1), OW = dy.size(2), OC = dy.size(3);
    const int KH = w.size(1), KW = w.size(2), C = w.size(3);
    TORCH_CHECK(w.size(0) == OC && OH == H + 2 * P - KH + 1 && OW == W + 2 * P - KW + 1, "conv dgrad geometry");
    Tensor dx = grad_out(out, accumulate, {N, H, W, C}, dy, "conv dgrad");
    const int M = N * (int)H * (int)W, K = KH * KW * OC;
    if (M == 0) return dx;
    if (KH == 3 && KW == 3 && P == 1 && C == 64 && OC == 64 &&
        rn_conv3x3(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), nullptr, N, (int)H, (int)W, 1, accumulate ? 1 : 0,
                   cur_stream()) == 0)
        return dx;  // the halo-tile kernel (conv3x3.hip), flipped / transposed weights
    const int rc = rn_conv_gemm(2, dy.data_ptr(), w.data_ptr(), dx.data_ptr(), nullptr, nullptr, M, C, K, 0, 0, C, OH,
                                OW, OC, (int)H, (int)W, KH, KW, 1, (int)P, OC, C, (long)KH * KW * C, 1, 0,
                                accumulate ? 1 : 0, nullptr, cur_stream());
    TORCH_CHECK(rc == 0, "implicit conv dgrad: unsupported geometry");
    return dx;
}
Tensor conv_wgrad_implicit(const Tensor& dy2, const Tensor& x, int64_t KH, int64_t KW, int64_t S, int64_t P,
                           const optional<Tensor>& out, bool accumulate) {
    CHECK_BF16(dy2); CHECK_CONTIG(dy2); CHECK_BF16(x); CHECK_CONTIG(x); GUARD(x);
    const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
    const int OH = (H + 2 * P - KH) / S + 1, OW = (W + 2 * P - KW) / S + 1;
    const int OC = dy2.size(1), PIX = N * OH * OW, K = KH * KW * C;
    TORCH_CHECK(dy2.size(0) == PIX, "conv wgrad: dy rows != output pixels");
    Tensor dw;
    if (out && out->defined()) {  // e.g. the flat gradient view of the weight (accumulate: direct grad)
        CHECK_BF16(*out); CHECK_CONTIG(*out);
        TORCH_CHECK(out->numel() == (long)OC * K && out->device() == x.device(), "conv wgrad: out shape");
        dw = *out;
    } else {
        TORCH_CHECK(!accumulate, "conv wgrad: accumulate needs out");
        dw = at::empty({OC, K}, x.options());
    }
    // split-K over the pixels so the (OC/128)×(K/128) tile grid fills the chip
    int bm, bn;
    rn_conv_wgrad_tile(OC, K, &bm, &bn);
    const long tiles = (long)((OC + bm - 1) / bm) * ((K + bn - 1) / bn);
    int split = 1;
    static const long target = [] {  // workgroups to aim for (REPLICANN_CONVW_TARGET: A/B only)
        const char* e = getenv("REPLICANN_CONVW_TARGET");
        return e ? atol(e) : 512L;
    }();
    while (tiles * split < target && PIX / (split * 2) >= 1024) split *= 2;
    Tensor ws = split > 1 ? at::empty({(long)split * OC * K}, x.options().dtype(at::kFloat)) : Tensor();
    const int rc = rn_conv_gemm(3, dy2.data_ptr(), x.data_ptr(), dw.data_ptr(), nullptr,
                                ws.defined() ? ws.data_ptr<float>() : nullptr, OC, K, PIX, OC, 0, K, H, W, C, OH, OW,
                                (int)KH, (int)KW, (int)S, (int)P, C, 0, 0, split, 0, accumulate ? 1 : 0,
                                nullptr, cur_stream());
    TORCH_CHECK(rc == 0, "implicit conv wgrad: unsupported geometry");
    return dw;
}

// ------------------------------------------------------------------ conv / pool / bn
Tensor im2col(const Tensor& x, int64_t KH, int64_t KW, int64_t S, int64_t P, int64_t Kp) {
    CHECK_BF16(x); CHECK_CONTIG(x); GUARD(x);
    const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
    const int OH = (H + 2 * P - KH) / S + 1, OW = (W + 2 * P - KW) / S + 1;
    Tensor cols = at::empty({(int64_t)N * OH * OW, Kp}, x.options());
    rn_im2col(x.data_ptr(), cols.data_ptr(), N, H, W, C, KH, KW, S, P, OH, OW, Kp, cur_stream());
    return cols;
}
Tensor col2im(const Tensor& dcols, int64_t N, int64_t H, int64_t W, int64_t C, int64_t KH, int64_t KW, int64_t S,
              int64_t P, int64_t Kp, const optional<Tensor>& out, bool accumulate) {
    CHECK_BF16(dcols); CHECK_CONTIG(dcols); GUARD(dcols);
    const int OH = (H + 2 * P - KH) / S + 1, OW = (W + 2 * P - KW) / S + 1;
    Tensor dx = grad_out(out, accumulate, {N, H, W, C}, dcols, "col2im");
    rn_col2im(dcols.data_ptr(), dx.data_ptr(), N, H, W, C, KH, KW, S, P, OH, OW, Kp, accumulate ? 1 : 0, cur_stream());
    return dx;
}
std::tuple<Tensor, Tensor> maxpool_fwd(const Tensor& x, int64_t K, int64_t S, int64_t P) {
    CHECK_BF16(x); CHECK_CONTIG(x); GUARD(x);
    TORCH_CHECK(K * K <= 256, "maxpool: window too large for byte indices");
    const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
    const int OH = (H + 2 * P - K) / S + 1, OW = (W + 2 * P - K) / S + 1;
    Tensor y = at::empty({N, OH, OW, C}, x.options());
    Tensor idx = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
    rn_maxpool_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C, K, S, P, OH, OW, cur_stream());
    return {y, idx};
}
// gy (N, OH, OW, C) + the forward's window indices → dx (N, H, W, C)
Tensor maxpool_bwd(const Tensor& gy, const Tensor& idx, int64_t H, int64_t W, int64_t K, int64_t S, int64_t P) {
    CHECK_BF16(gy); CHECK_CONTIG(gy); GUARD(gy);
    TORCH_CHECK(idx.scalar_type() == at::kByte && idx.sizes() == gy.sizes() && idx.is_contiguous());
    const int N = gy.size(0), OH = gy.size(1), OW = gy.size(2), C = gy.size(3);
    Tensor dx = at::empty({N, H, W, C}, gy.options());
    rn_maxpool_bwd(gy.data_ptr(), idx.data_ptr(), dx.data_ptr(), N, (int)H, (int)W, C, K, S, P, OH, OW, cur_stream());
    return dx;
}
Tensor avgpool_fwd(const Tensor& x) {
    CHECK_BF16(x); CHECK_CONTIG(x); GUARD(x);
    const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
    Tensor y = at::empty({N, C}, x.options());
    rn_avgpool_fwd(x.data_ptr(), y.data_ptr(), N, HW, C, cur_stream());
    return y;
}
Tensor avgpool_bwd(const Tensor& gy, int64_t H, int64_t W) {
    CHECK_BF16(gy); GUARD(gy);
    const int N = gy.size(0), C = gy.size(1);
    Tensor dx = at::empty({N, H, W, C}, gy.options());
    rn_avgpool_bwd(gy.contiguous().data_ptr(), dx.data_ptr(), N, H * W, C, cur_stream());
    return dx;
}
// NHWC BatchNorm over [M][C] rows (C % 8 == 0, C <= 2048); res (optional, same shape): y = relu(BN(x) + res)
static void check_bn(const Tensor& x, const optional<Tensor>& res) {
    CHECK_BF16(x); CHECK_CONTIG(x);
    TORCH_CHECK(rn_bn_supported((int)x.size(1)), "batchnorm: channels must be a multiple of 8 and <= 2048");
    if (res && res->defined()) {
        CHECK_BF16(*res); CHECK_CONTIG(*res);
        TORCH_CHECK(res->sizes() == x.sizes(), "batchnorm residual shape");
    }
}
// returns (y, mean, rstd, mask): mask = relu'(y) bits, [M·C/8] bytes (empty without relu)
std::tuple<Tensor, Tensor, Tensor, Tensor> batchnorm_fwd(const Tensor& x, const Tensor& w, const Tensor& b,
                                                 const Tensor& rmean, const Tensor& rvar, double mom, double eps,
                                                 bool relu, const optional<Tensor>& res,
                                                 const optional<Tensor>& partials) {
    check_bn(x, res); GUARD(x);
    TORCH_CHECK(rmean.scalar_type() == at::kFloat && rvar.scalar_type() == at::kFloat, "BN running stats must be fp32");
    const int M = x.size(0), C = x.size(1);
    // partials: [R][2C] fp32 Σ | Σ² row-block partials of x from its producer (conv_fwd_implicit_stats)
    const bool hp = partials && partials->defined();
    if (hp)
        TORCH_CHECK(partials->scalar_type() == at::kFloat && partials->dim() == 2 && partials->size(1) == 2L * C &&
                        partials->is_contiguous() && partials->device() == x.device(),
                    "batchnorm_fwd: partials must be fp32 [R][2C]");
    Tensor y = at::empty_like(x);
    Tensor mean = at::empty({C}, x.options().dtype(at::kFloat));
    Tensor rstd = at::empty({C}, x.options().dtype(at::kFloat));
    Tensor ws = at::empty({rn_bn_ws_floats(M, C)}, x.options().dtype(at::kFloat));
    Tensor mask = at::empty({relu ? (int64_t)M * C / 8 : 0}, x.options().dtype(at::kByte));
    rn_bn_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), rmean.data_ptr<float>(), rvar.data_ptr<float>(), y.data_ptr(),
              mean.data_ptr<float>(), rstd.data_ptr<float>(), ws.data_ptr<float>(), M, C, (float)mom, (float)eps, relu,
              optr(res), hp ? partials->data_ptr<float>() : nullptr, hp ? (int)partials->size(0) : 0,
              relu ? mask.data_ptr() : nullptr, cur_stream());
    return {y, mean, rstd, mask};
}
Tensor batchnorm_eval(const Tensor& x, const Tensor& w, const Tensor& b, const Tensor& rmean, const Tensor& rvar,
                      double eps, bool relu, const optional<Tensor>& res) {
    check_bn(x, res); GUARD(x);
    Tensor y = at::empty_like(x);
    rn_bn_eval(x.data_ptr(), w.data_ptr(), b.data_ptr(), rmean.data_ptr<float>(), rvar.data_ptr<float>(), y.data_ptr(),
               x.size(0), x.size(1), (float)eps, relu, optr(res), cur_stream());
    return y;
}
// returns (dx, dw, db, g') with g' = dy ⊙ relu'(y) (the fused residual's gradient) when want_gres;
// mask: batchnorm_fwd's relu'(y) bits (read only with relu)
std::tuple<Tensor, Tensor, Tensor, Tensor> batchnorm_bwd(const Tensor& gy, const Tensor& x, const Tensor& mask,
                                                         const Tensor& w, const Tensor& mean, const Tensor& rstd,
                                                         bool relu, bool want_gres, const optional<Tensor>& dw_acc,
                                                         const optional<Tensor>& db_acc) {
    check_bn(gy, c10::nullopt); GUARD(gy);
    const int M = x.size(0), C = x.size(1);
    if (relu)
        TORCH_CHECK(mask.scalar_type() == at::kByte && mask.numel() == (int64_t)M * C / 8 && mask.is_contiguous(),
                    "batchnorm_bwd: relu needs the forward's [M*C/8] uint8 mask");
    Tensor dx = at::empty_like(x);
    // dw_acc / db_acc: gradient views to ADD into (direct accumulation), both or neither
    const bool acc = dw_acc && dw_acc->defined();
    TORCH_CHECK(acc == (db_acc && db_acc->defined()), "batchnorm_bwd: dw_acc and db_acc go together");
    if (acc) {
        for (const Tensor* t : {&*dw_acc, &*db_acc}) {
            CHECK_BF16(*t); CHECK_CONTIG(*t);
            TORCH_CHECK(t->numel() == C && t->device() == x.device(), "batchnorm_bwd: accumulation target shape");
        }
    }
    Tensor dw = acc ? *dw_acc : at::empty({C}, x.options());  // bf16, the parameter dtype
    Tensor db = acc ? *db_acc : at::empty({C}, x.options());
    Tensor gres = want_gres ? at::empty_like(x) : at::empty({0}, x.options());
    Tensor ws = at::empty({rn_bn_ws_floats(M, C)}, x.options().dtype(at::kFloat));
    rn_bn_bwd(gy.data_ptr(), x.data_ptr(), relu ? mask.data_ptr() : nullptr, w.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
              dx.data_ptr(), dw.data_ptr(), db.data_ptr(), ws.data_ptr<float>(), M, C, relu,
              want_gres ? gres.data_ptr() : nullptr, acc ? 1 : 0, cur_stream());
    return {dx, dw, db, gres};
}

// ------------------------------------------------------------------ fp8
std::tuple<Tensor, Tensor> fp8_quantize(const Tensor& x) {
    CHECK_BF16(x); CHECK_CONTIG(x); GUARD(x);
    Tensor q = at::empty(x.sizes(), x.options().dtype(at::kByte));
    Tensor state = at::empty({4}, x.options().dtype(at::kFloat));
    rn_fp8_quantize(x.data_ptr(), x.numel(), q.data_ptr(), state.data_ptr<float>(), cur_stream());
    return {q, state};
}
// delayed scaling: `state` (fp32 [4], persistent per tensor) carries the amax of the previous
// quantisation; one pass over x (the two-pass fp8_quantize initialises it)
Tensor fp8_quantize_delayed(const Tensor& x, const Tensor& state) {
    CHECK_BF16(x); CHECK_CONTIG(x); GUARD(x);
    TORCH_CHECK(state.scalar_type() == at::kFloat && state.numel() >= 4 && state.is_cuda());
    Tensor q = at::empty(x.sizes(), x.options().dtype(at::kByte));
    rn_fp8_quantize_delayed(x.data_ptr(), x.numel(), q.data_ptr(), state.data_ptr<float>(), cur_stream());
    return q;
}
// e5m2 ("bf8") quantisation of a gradient operand: delayed scaling (roll + one pass) or, for a slot
// without a scale yet, current scaling; state: [scale, amax, amax the scale came from, -]
// dH = dU ⊙ d (the MLP's GELU backward against the saved gelu'(h)) written only as e5m2 with the gradient
// slot ``state`` (delayed / current scaling as bf8_quantize); with ``bias_grad`` (bf16 [N]) Σ_rows dH is
// added into it
Tensor act_mul_bf8(const Tensor& du, const Tensor& d, const Tensor& state, bool delayed, const optional<Tensor>& bias_grad,
                   bool from_h) {
    CHECK_BF16(du); CHECK_BF16(d); CHECK_CONTIG(du); CHECK_CONTIG(d); GUARD(du);
    TORCH_CHECK(du.dim() == 2 && du.sizes() == d.sizes() && du.size(1) % 8 == 0, "act_mul_bf8: matching [M][N] inputs, N % 8");
    TORCH_CHECK(state.scalar_type() == at::kFloat && state.numel() >= 4 && state.is_cuda() && state.device() == du.device());
    const long M = du.size(0);
    const int N = (int)du.size(1);
    Tensor q = at::empty(du.sizes(), du.options().dtype(at::kByte));
    if (M == 0) return q;
    const bool bg = bias_grad && bias_grad->defined();
    if (bg)
        TORCH_CHECK(bias_grad->scalar_type() == at::kBFloat16 && bias_grad->numel() == N && bias_grad->is_contiguous() &&
                        bias_grad->device() == du.device(),
                    "act_mul_bf8: bias_grad must be a contiguous bf16 [N] tensor on the same device");
    const int G = rn_act_mul_bf8_groups(M, N);
    Tensor part = bg ? at::empty({(int64_t)G * N}, du.options().dtype(at::kFloat)) : Tensor();
    rn_act_mul_bf8(du.data_ptr(), d.data_ptr(), M, N, q.data_ptr(), state.data_ptr<float>(), delayed ? 1 : 0,
                   bg ? part.data_ptr<float>() : nullptr, from_h ? 1 : 0, cur_stream());
    if (bg) {
        Tensor tmp = at::empty({rn_colsum_ws(N)}, du.options().dtype(at::kFloat));
        rn_colsum_f32(part.data_ptr<float>(), G, N, tmp.data_ptr<float>(), bias_grad->data_ptr(), 1, cur_stream());
    }
    return q;
}

// e4m3(gelu(h)) with the delayed-scaling slot ``state`` (rolled here, amax recorded): see rn_gelu_q8
Tensor gelu_q8(const Tensor& h, const Tensor& state) {
    CHECK_BF16(h); CHECK_CONTIG(h); GUARD(h);
    TORCH_CHECK(state.scalar_type() == at::kFloat && state.numel() >= 4 && state.is_cuda() && state.device() == h.device());
    TORCH_CHECK(h.numel() % 8 == 0, "gelu_q8: numel % 8");
    Tensor q = at::empty(h.sizes(), h.options().dtype(at::kByte));
    if (h.numel()) rn_gelu_q8(h.data_ptr(), h.numel(), q.data_ptr(), state.data_ptr<float>(), cur_stream());
    return q;
}

Tensor bf8_quantize(const Tensor& x, const Tensor& state, bool delayed) {
    CHECK_BF16(x); CHECK_CONTIG(x); GUARD(x);
    TORCH_CHECK(state.scalar_type() == at::kFloat && state.numel() >= 4 && state.is_cuda());
    Tensor q = at::empty(x.sizes(), x.options().dtype(at::kByte));
    rn_bf8_quantize(x.data_ptr(), x.numel(), q.data_ptr(), state.data_ptr<float>(), delayed ? 1 : 0, cur_stream());
    return q;
}
Tensor bf8_dequantize(const Tensor& q, const Tensor& state) {
    GUARD(q);
    Tensor y = at::empty(q.sizes(), q.options().dtype(at::kBFloat16));
    rn_bf8_dequantize(q.data_ptr(), q.numel(), state.data_ptr<float>(), y.data_ptr(), cur_stream());
    return y;
}
// fp8 weight gradient: out[M,N] (+)= sa·sb · a8ᵀ · b8 with a8 [K][M] (e5m2 if a_bf8, else e4m3) and
// b8 [K][N] e4m3, K = tokens (csrc/include/gemm_pk.h, fp8 MN-contiguous operands)
void gemm_fp8_wgrad(const Tensor& a8, const Tensor& b8, const Tensor& sa, const Tensor& sb, const Tensor& out,
                    bool accumulate, bool a_bf8, const optional<Tensor>& post) {
    GUARD(a8);
    TORCH_CHECK(a8.scalar_type() == at::kByte && b8.scalar_type() == at::kByte, "fp8 operands are uint8 storage");
    TORCH_CHECK(a8.dim() == 2 && b8.dim() == 2 && a8.size(0) == b8.size(0) && a8.stride(1) == 1 && b8.stride(1) == 1);
    const int K = a8.size(0), M = a8.size(1), N = b8.size(1);
    TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == N && out.stride(1) == 1);
    TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat);
    Tensor ws = at::empty({rn_gemm_fp8_wgrad_ws(M, N, K)}, a8.options().dtype(at::kFloat));
    Tensor alpha = at::empty({1}, a8.options().dtype(at::kFloat));
    int rc = rn_gemm_fp8_wgrad(a8.data_ptr(), b8.data_ptr(), out.data_ptr(), sa.data_ptr<float>(), sb.data_ptr<float>(),
                               alpha.data_ptr<float>(), ws.data_ptr<float>(), M, N, K, a8.stride(0), b8.stride(0),
                               out.stride(0), accumulate ? 1 : 0, out.scalar_type() == at::kFloat ? 1 : 0, a_bf8 ? 1 : 0,
                               cur_stream(), post ? post->data_ptr<float>() : nullptr);
    TORCH_CHECK(rc == 0, "gemm_fp8_wgrad: M, N and row strides must be multiples of 16 and K of 128, got M=", M,
                " N=", N, " K=", K);
}
// fp8 data gradient: dY8 [M][K] (e5m2 if a_bf8) · W8 [K][N] (the e4m3 weight as stored) -> bf16 [M][N]
Tensor gemm_fp8_dgrad(const Tensor& a8, const Tensor& b8, const Tensor& sa, const Tensor& sb, bool a_bf8,
                      const optional<Tensor>& post) {
    GUARD(a8);
    TORCH_CHECK(a8.scalar_type() == at::kByte && b8.scalar_type() == at::kByte, "fp8 operands are uint8 storage");
    TORCH_CHECK(a8.dim() == 2 && b8.dim() == 2 && a8.size(1) == b8.size(0) && a8.stride(1) == 1 && b8.stride(1) == 1);
    const int M = a8.size(0), K = a8.size(1), N = b8.size(1);
    Tensor c = at::empty({M, N}, a8.options().dtype(at::kBFloat16));
    Tensor alpha = at::empty({1}, a8.options().dtype(at::kFloat));
    if (M == 0) return c;
    int rc = rn_gemm_fp8_dgrad(a8.data_ptr(), b8.data_ptr(), c.data_ptr(), sa.data_ptr<float>(), sb.data_ptr<float>(),
                               alpha.data_ptr<float>(), M, N, K, a8.stride(0), b8.stride(0), c.stride(0), a_bf8 ? 1 : 0,
                               cur_stream(), post ? post->data_ptr<float>() : nullptr);
    TORCH_CHECK(rc == 0, "gemm_fp8_dgrad: K, N and row strides must be multiples of 16, got K=", K, " N=", N);
    return c;
}
Tensor fp8_dequantize(const Tensor& q, const Tensor& state) {
    GUARD(q);
    Tensor y = at::empty(q.sizes(), q.options().dtype(at::kBFloat16));
    rn_fp8_dequantize(q.data_ptr(), q.numel(), state.data_ptr<float>(), y.data_ptr(), cur_stream());
    return y;
}
Tensor gemm_fp8(const Tensor& a8, const Tensor& b8, const Tensor& sa, const Tensor& sb, const optional<Tensor>& bias,
                const optional<Tensor>& residual, int64_t act, const optional<Tensor>& preact) {
    GUARD(a8);
    TORCH_CHECK(a8.scalar_type() == at::kByte && b8.scalar_type() == at::kByte, "fp8 operands are uint8 storage");
    TORCH_CHECK(a8.dim() == 2 && b8.dim() == 2 && a8.size(1) == b8.size(1) && a8.is_contiguous() && b8.is_contiguous());
    const int M = a8.size(0), N = b8.size(0), K = a8.size(1);
    Tensor c = at::empty({M, N}, a8.options().dtype(at::kBFloat16));
    Tensor alpha = at::empty({1}, a8.options().dtype(at::kFloat));
    if (residual && residual->defined()) { CHECK_BF16(*residual); TORCH_CHECK(residual->is_contiguous()); }
    int rc = rn_gemm_fp8(a8.data_ptr(), b8.data_ptr(), c.data_ptr(), optr(bias), optr(residual),
                         preact && preact->defined() ? preact->data_ptr() : nullptr, sa.data_ptr<float>(),
                         sb.data_ptr<float>(), alpha.data_ptr<float>(), M, N, K, a8.stride(0), b8.stride(0), c.stride(0),
                         (int)act, cur_stream(), nullptr, nullptr);
    TORCH_CHECK(rc == 0, "gemm_fp8: K and row strides must be multiples of 16, got K=", K);
    return c;
}
// gemm_fp8 whose activation output also comes out in e4m3 for the next fp8 GEMM (`q8_state`: that
// GEMM's activation Fp8State slot; delayed scaling, rolled here, amax recorded by the epilogue)
std::tuple<Tensor, Tensor> gemm_fp8_q8(const Tensor& a8, const Tensor& b8, const Tensor& sa, const Tensor& sb,
                                       const optional<Tensor>& bias, int64_t act, const Tensor& preact,
                                       const Tensor& q8_state) {
    GUARD(a8);
    TORCH_CHECK(a8.scalar_type() == at::kByte && b8.scalar_type() == at::kByte, "fp8 operands are uint8 storage");
    TORCH_CHECK(a8.dim() == 2 && b8.dim() == 2 && a8.size(1) == b8.size(1) && a8.is_contiguous() && b8.is_contiguous());
    TORCH_CHECK(q8_state.scalar_type() == at::kFloat && q8_state.numel() >= 4 && q8_state.is_cuda());
    const int M = a8.size(0), N = b8.size(0), K = a8.size(1);
    TORCH_CHECK(preact.size(0) == M && preact.size(1) == N && preact.is_contiguous());
    Tensor c = at::empty({M, N}, a8.options().dtype(at::kBFloat16));
    Tensor q = at::empty({M, N}, a8.options().dtype(at::kByte));
    Tensor alpha = at::empty({1}, a8.options().dtype(at::kFloat));
    int rc = rn_gemm_fp8(a8.data_ptr(), b8.data_ptr(), c.data_ptr(), optr(bias), nullptr, preact.data_ptr(),
                         sa.data_ptr<float>(), sb.data_ptr<float>(), alpha.data_ptr<float>(), M, N, K, a8.stride(0),
                         b8.stride(0), c.stride(0), (int)act, cur_stream(), q.data_ptr(), q8_state.data_ptr<float>());
    TORCH_CHECK(rc == 0, "gemm_fp8_q8: unsupported shape / activation (rc ", rc, ")");
    return {c, q};
}

// e4m3 copies of many weights of one flat bf16 parameter buffer, two launches (see fp8.hip)
void fp8_quant_many(const Tensor& flat, const Tensor& segs, int64_t max_n, const Tensor& qbuf, bool roll) {
    CHECK_BF16(flat); GUARD(flat);
    TORCH_CHECK(segs.scalar_type() == at::kLong && segs.is_cuda() && segs.dim() == 2 && segs.size(1) == 4 &&
                segs.is_contiguous());
    TORCH_CHECK(qbuf.scalar_type() == at::kByte && qbuf.is_cuda());
    rn_fp8_quant_many(flat.data_ptr(), segs.data_ptr<int64_t>(), (int)segs.size(0), (long)max_n, qbuf.data_ptr(),
                      roll ? 1 : 0, cur_stream());
}

int64_t native_version() { return 1; }

}  // namespace

TORCH_LIBRARY(replicann, m) {
    m.def("gemm(Tensor a, Tensor b, bool ta, bool tb, Tensor? bias, Tensor? residual, int act, Tensor? preact, "
          "Tensor? out, bool accumulate, int split_k, bool out_fp32, Tensor? alpha=None, int cfg=-1, "
          "Tensor(a!)? bias_grad=None) -> Tensor");
    m.def("attn_decode(Tensor q, Tensor k, Tensor v, Tensor? mask, float scale) -> Tensor");
    m.def("linear_kv(Tensor x, Tensor w, Tensor? bias, Tensor(a!) kv, Tensor pos) -> Tensor");
    m.def("bias_act_grad(Tensor dy, Tensor? h, int act, bool want_bias, Tensor(a!)? db_accum=None) -> (Tensor, Tensor)");
    m.def("act_fwd(Tensor x, int kind) -> Tensor");
    m.def("act_bwd(Tensor dy, Tensor x, int kind) -> Tensor");
    m.def("dropout_fwd(Tensor x, float p, int seed, Tensor? seed_buf=None) -> Tensor");
    m.def("rng_next(Tensor(a!) state, Tensor(b!) out) -> ()");
    m.def("add_act(Tensor a, Tensor b, bool relu) -> Tensor");
    m.def("softmax_fwd(Tensor x, float scale) -> Tensor");
    m.def("softmax_bwd(Tensor dy, Tensor y, float scale) -> Tensor");
    m.def("xent_fwd(Tensor(a!) logits, Tensor target, int nvalid, int ignore, bool write_grad=False) -> (Tensor, Tensor)");
    m.def("xent_fwd_q8(Tensor logits, Tensor target, int nvalid, int ignore, Tensor(a!) q8) -> (Tensor, Tensor)");
    m.def("xent_bwd(Tensor logits, Tensor target, Tensor lse, Tensor gscale, Tensor(a!) grad, int nvalid, int ignore) -> ()");
    m.def("layernorm_fwd(Tensor x, Tensor? r, Tensor w, Tensor? b, float eps) -> (Tensor, Tensor, Tensor, Tensor)");
    m.def("layernorm_fwd_q8(Tensor x, Tensor? r, Tensor w, Tensor? b, float eps, Tensor(a!) state) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
    m.def("layernorm_bwd(Tensor dy, Tensor? gh, Tensor h, Tensor w, Tensor mean, Tensor rstd, "
          "Tensor(a!)? dw_accum=None, Tensor(b!)? db_accum=None, Tensor(c!)? dxs_accum=None, Tensor(d!)? q8=None, "
          "Tensor(e!)? q8_state=None) -> (Tensor, Tensor, Tensor)");
    m.def("embedding_fwd(Tensor ids, Tensor wte, Tensor? wpe) -> Tensor");
    m.def("vit_join_fwd(Tensor patch, Tensor cls, Tensor pos) -> Tensor");
    m.def("vit_join_bwd(Tensor dx, Tensor(a!) gcls, Tensor(b!) gpos) -> Tensor");
    m.def("embedding_bwd(Tensor dx, Tensor ids, int V, int Tp) -> (Tensor, Tensor)");
    m.def("embedding_bwd_acc(Tensor dx, Tensor ids, Tensor(a!) gwte, Tensor(b!)? gwpe) -> ()");
    m.def("sumsq(Tensor g, Tensor(a!) normbuf) -> ()");
    m.def("opt_prep(Tensor(a!) state, float base_lr, float warmup, float total, float min_ratio, bool cosine, "
          "float lr_override, float b1, float b2) -> ()");
    m.def("adamw_step(Tensor(a!) p, Tensor(b!) master, Tensor g, Tensor(c!) m, Tensor(d!) v, Tensor wdm, Tensor(e!) state, "
          "float b1, float b2, float eps, float wd, float gscale, float clip, bool stochastic_round=False) -> ()");
    m.def("sgd_step(Tensor(a!) p, Tensor(b!) master, Tensor g, Tensor(c!) buf, Tensor wdm, Tensor(e!) state, "
          "float mom, float wd, bool nesterov, float gscale, float clip) -> ()");
    m.def("attn_fwd(Tensor q, Tensor k, Tensor v, Tensor? bias, float scale, bool causal, float p, int seed, "
          "Tensor? seed_buf=None) -> (Tensor, Tensor)");
    m.def("attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor? bias, float scale, "
          "bool causal, float p, int seed, Tensor? seed_buf=None) -> (Tensor, Tensor, Tensor)");
    m.def("attn_bwd_out(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor? bias, float scale, "
          "bool causal, float p, int seed, Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, "
          "Tensor(d!)? qkv_bias_grad=None, Tensor? seed_buf=None) -> ()");
    m.def("attn_bwd_out_q8(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor? bias, float scale, "
          "bool causal, float p, int seed, Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, "
          "Tensor(d!)? qkv_bias_grad, Tensor? seed_buf, Tensor(e!) q8, Tensor(f!) q8_state, bool q8_only) -> bool");
    m.def("im2col(Tensor x, int KH, int KW, int S, int P, int Kp) -> Tensor");
    m.def("conv_fwd_implicit(Tensor x, Tensor w, Tensor? bias, int S, int P) -> Tensor");
    m.def("conv_fwd_implicit_stats(Tensor x, Tensor w, Tensor? bias, int S, int P) -> (Tensor, Tensor)");
    m.def("conv_dgrad_implicit(Tensor dy, Tensor w, int H, int W, int P, Tensor(a!)? out=None, bool accumulate=False) -> Tensor");
    m.def("conv_wgrad_implicit(Tensor dy2, Tensor x, int KH, int KW, int S, int P, Tensor(a!)? out=None, "
          "bool accumulate=False) -> Tensor");
    m.def("col2im(Tensor dcols, int N, int H, int W, int C, int KH, int KW, int S, int P, int Kp, Tensor(a!)? out=None, "
          "bool accumulate=False) -> Tensor");
    m.def("maxpool_fwd(Tensor x, int K, int S, int P) -> (Tensor, Tensor)");
    m.def("maxpool_bwd(Tensor gy, Tensor idx, int H, int W, int K, int S, int P) -> Tensor");
    m.def("avgpool_fwd(Tensor x) -> Tensor");
    m.def("avgpool_bwd(Tensor gy, int H, int W) -> Tensor");
    m.def("batchnorm_fwd(Tensor x, Tensor w, Tensor b, Tensor(a!) rmean, Tensor(b!) rvar, float mom, float eps, bool relu, "
          "Tensor? res=None, Tensor? partials=None) -> (Tensor, Tensor, Tensor, Tensor)");
    m.def("batchnorm_eval(Tensor x, Tensor w, Tensor b, Tensor rmean, Tensor rvar, float eps, bool relu, "
          "Tensor? res=None) -> Tensor");
    m.def("batchnorm_bwd(Tensor gy, Tensor x, Tensor mask, Tensor w, Tensor mean, Tensor rstd, bool relu, "
          "bool want_gres=False, Tensor(c!)? dw_acc=None, Tensor(d!)? db_acc=None) -> (Tensor, Tensor, Tensor, Tensor)");
    m.def("fp8_quantize(Tensor x) -> (Tensor, Tensor)");
    m.def("fp8_dequantize(Tensor q, Tensor state) -> Tensor");
    m.def("fp8_quantize_delayed(Tensor x, Tensor state) -> Tensor");
    m.def("bf8_quantize(Tensor x, Tensor(a!) state, bool delayed) -> Tensor");
    m.def("act_mul_bf8(Tensor du, Tensor d, Tensor(a!) state, bool delayed, Tensor(b!)? bias_grad=None, bool from_h=False) -> Tensor");
    m.def("gelu_q8(Tensor h, Tensor(a!) state) -> Tensor");
    m.def("bf8_dequantize(Tensor q, Tensor state) -> Tensor");
    m.def("gemm_fp8_wgrad(Tensor a8, Tensor b8, Tensor sa, Tensor sb, Tensor(a!) out, bool accumulate, bool a_bf8, "
          "Tensor? post=None) -> ()");
    m.def("gemm_fp8_dgrad(Tensor a8, Tensor b8, Tensor sa, Tensor sb, bool a_bf8, Tensor? post=None) -> Tensor");
    m.def("gemm_fp8(Tensor a8, Tensor b8, Tensor sa, Tensor sb, Tensor? bias, Tensor? residual, int act, Tensor? preact) -> Tensor");
    m.def("gemm_fp8_q8(Tensor a8, Tensor b8, Tensor sa, Tensor sb, Tensor? bias, int act, Tensor(a!) preact, Tensor(b!) q8_state) -> (Tensor, Tensor)");
    m.def("fp8_quant_many(Tensor flat, Tensor segs, int max_n, Tensor(a!) qbuf, bool roll=True) -> ()");
    m.def("native_version() -> int");
    m.def("gemm_tuning_table() -> str");
    m.def("gemm_tuning_load(str table) -> int");
    m.def("gemm_set_sched(int mode) -> ()");
    m.def("gemm_get_sched() -> int");
    m.def("gemm_set_reserve(int cus) -> ()");
    m.def("gemm_get_reserve() -> int");
    m.def("gemm_sched_init(int device) -> int");
}

TORCH_LIBRARY_IMPL(replicann, CUDA, m) {
    m.impl("gemm", &gemm);
    m.impl("attn_decode", &attn_decode);
    m.impl("linear_kv", &linear_kv);
    m.impl("bias_act_grad", &bias_act_grad);
    m.impl("act_fwd", &act_fwd);
    m.impl("act_bwd", &act_bwd);
    m.impl("dropout_fwd", &dropout_fwd);
    m.impl("rng_next", &rng_next);
    m.impl("add_act", &add_act);
    m.impl("softmax_fwd", &softmax_fwd);
    m.impl("softmax_bwd", &softmax_bwd);
    m.impl("xent_fwd", &xent_fwd);
    m.impl("xent_fwd_q8", &xent_fwd_q8);
    m.impl("xent_bwd", &xent_bwd);
    m.impl("layernorm_fwd", &layernorm_fwd);
    m.impl("layernorm_fwd_q8", &layernorm_fwd_q8);
    m.impl("layernorm_bwd", &layernorm_bwd);
    m.impl("embedding_fwd", &embedding_fwd);
    m.impl("vit_join_fwd", &vit_join_fwd);
    m.impl("vit_join_bwd", &vit_join_bwd);
    m.impl("embedding_bwd", &embedding_bwd);
    m.impl("embedding_bwd_acc", &embedding_bwd_acc);
    m.impl("sumsq", &sumsq);
    m.impl("opt_prep", &opt_prep);
    m.impl("adamw_step", &adamw_step);
    m.impl("sgd_step", &sgd_step);
    m.impl("attn_fwd", &attn_fwd);
    m.impl("attn_bwd", &attn_bwd);
    m.impl("attn_bwd_out", &attn_bwd_out);
    m.impl("attn_bwd_out_q8", &attn_bwd_out_q8);
    m.impl("im2col", &im2col);
    m.impl("conv_fwd_implicit", &conv_fwd_implicit);
    m.impl("conv_fwd_implicit_stats", &conv_fwd_implicit_stats);
    m.impl("conv_dgrad_implicit", &conv_dgrad_implicit);
    m.impl("conv_wgrad_implicit", &conv_wgrad_implicit);
    m.impl("col2im", &col2im);
    m.impl("maxpool_fwd", &maxpool_fwd);
    m.impl("maxpool_bwd", &maxpool_bwd);
    m.impl("avgpool_fwd", &avgpool_fwd);
    m.impl("avgpool_bwd", &avgpool_bwd);
    m.impl("batchnorm_fwd", &batchnorm_fwd);
    m.impl("batchnorm_eval", &batchnorm_eval);
    m.impl("batchnorm_bwd", &batchnorm_bwd);
    m.impl("fp8_quantize", &fp8_quantize);
    m.impl("fp8_dequantize", &fp8_dequantize);
    m.impl("fp8_quantize_delayed", &fp8_quantize_delayed);
    m.impl("bf8_quantize", &bf8_quantize);
    m.impl("act_mul_bf8", &act_mul_bf8);
    m.impl("gelu_q8", &gelu_q8);
    m.impl("bf8_dequantize", &bf8_dequantize);
    m.impl("gemm_fp8_wgrad", &gemm_fp8_wgrad);
    m.impl("gemm_fp8_dgrad", &gemm_fp8_dgrad);
    m.impl("gemm_fp8", &gemm_fp8);
    m.impl("gemm_fp8_q8", &gemm_fp8_q8);
    m.impl("fp8_quant_many", &fp8_quant_many);
}

// persistent-GEMM schedule knobs (csrc/include/gemm_pk.h: dynamic tile queue, CU reservation)
void gemm_set_sched(int64_t m) { rn_gemm_set_sched((int)m); }
int64_t gemm_get_sched() { return rn_gemm_get_sched(); }
void gemm_set_reserve(int64_t r) { rn_gemm_set_reserve((int)r); }
int64_t gemm_get_reserve() { return rn_gemm_get_reserve(); }
int64_t gemm_sched_init(int64_t dev) { return rn_gemm_sched_init((int)dev); }

TORCH_LIBRARY_IMPL(replicann, CompositeExplicitAutograd, m) {
    m.impl("native_version", &native_version);
    m.impl("gemm_set_sched", &gemm_set_sched);
    m.impl("gemm_get_sched", &gemm_get_sched);
    m.impl("gemm_set_reserve", &gemm_set_reserve);
    m.impl("gemm_get_reserve", &gemm_get_reserve);
    m.impl("gemm_sched_init", &gemm_sched_init);
    m.impl("gemm_tuning_table", &gemm_tuning_table);
    m.impl("gemm_tuning_load", &gemm_tuning_load);
}
