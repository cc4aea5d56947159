// Embedding gather / scatter-add (N14) and fused optimizer steps (N12/N13).
#include "common.h"

namespace {

// x[row] = wte[ids[row]] + wpe[row % T]   — one row per wave, 16-B vectors
template <bool POS>
__global__ void __launch_bounds__(256) emb_fwd_k(const int64_t* __restrict__ ids, const bf16* __restrict__ wte,
                                                 const bf16* __restrict__ wpe, bf16* __restrict__ x, int rows,
                                                 int T, int E, int V) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const long id = ids[row];
    RN_CHECK(id >= 0 && id < V);
    const int t = row % T;
    for (int c = lane; c < E / 8; c += 64) {
        float a[8];
        load8(wte + id * E + c * 8, a);
        if constexpr (POS) {
            float p[8];
            load8(wpe + (long)t * E + c * 8, p);
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] += p[j];
        }
        store8(x + (long)row * E + c * 8, a);
    }
}

// dwte (fp32, pre-zeroed) += dx rows at ids.  Each wave-instruction adds 64
// consecutive floats = 256 contiguous bytes (full-rate atomic shape).
__global__ void __launch_bounds__(256) emb_bwd_scatter_k(const int64_t* __restrict__ ids, const bf16* __restrict__ dx,
                                                         float* __restrict__ dwte, int rows, int E) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const long id = ids[row];
    for (int c = lane; c < E; c += 64) atomicAdd(dwte + id * E + c, bf2f(dx[(long)row * E + c]));
}

// ---- direct-accumulate variant (graph-safe, no full-table memset / convert) ----
// d32 is a PERSISTENT fp32 V×E scratch kept all-zero between calls and owner a
// persistent V-entry table kept at 0xFFFFFFFF.  Scatter: fp32 atomics into d32
// plus atomicMin(owner[id], position).  Finish: the owning position of each
// touched row adds the fp32 row into the bf16 gradient once, re-zeroes the
// scratch row and re-arms owner — only touched rows are visited.
__global__ void __launch_bounds__(256) emb_scatter_own_k(const int64_t* __restrict__ ids,
                                                         const bf16* __restrict__ dx, float* __restrict__ d32,
                                                         unsigned* __restrict__ owner, int rows, int E, int V) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const long id = ids[row];
    RN_CHECK(id >= 0 && id < V);
    if (lane == 0) atomicMin(owner + id, (unsigned)row);
    for (int c = lane; c < E; c += 64) atomicAdd(d32 + id * E + c, bf2f(dx[(long)row * E + c]));
}

__global__ void __launch_bounds__(256) emb_finish_k(const int64_t* __restrict__ ids, float* __restrict__ d32,
                                                    unsigned* __restrict__ owner, bf16* __restrict__ g, int rows,
                                                    int E) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const long id = ids[row];
    if (owner[id] != (unsigned)row) return;
    for (int c = lane * 4; c < E; c += 256) {
        float4 v = *reinterpret_cast<float4*>(d32 + id * E + c);
        *reinterpret_cast<float4*>(d32 + id * E + c) = make_float4(0.f, 0.f, 0.f, 0.f);
        bf16* q = g + id * E + c;
        q[0] = (bf16)((float)q[0] + v.x);
        q[1] = (bf16)((float)q[1] + v.y);
        q[2] = (bf16)((float)q[2] + v.z);
        q[3] = (bf16)((float)q[3] + v.w);
    }
    if (lane == 0) owner[id] = 0xFFFFFFFFu;
}

// Deterministic variant (REPLICANN_DETERMINISTIC=1): the same owner scheme, but the scratch
// accumulates 64-bit FIXED-POINT values (round(x · 2^40)) with integer atomics, whose sum does not
// depend on the order the rows arrive in — unlike fp32 atomics.  Each contribution is rounded to the
// nearest 2^-40 ≈ 9.1e-13 (a bf16 input is NOT represented exactly: values below 2^-41 in magnitude
// vanish), so a per-token gradient of 1e-8 (e.g. a 1/(B·T·grad_accum) loss scale) keeps ≈ 1e-4
// relative precision; the per-element range is |Σ| < 2^23 (int64 / 2^40), far above any embedding
// gradient.  Twice the scratch bytes and atomic traffic of the fp32 path
// (tests/test_determinism_gpu.py::test_embedding_scatter_deterministic_tiny_gradients).
constexpr float FX_SCALE = 1099511627776.f;  // 2^40

__global__ void __launch_bounds__(256) emb_scatter_own_fx_k(const int64_t* __restrict__ ids,
                                                            const bf16* __restrict__ dx,
                                                            unsigned long long* __restrict__ d64,
                                                            unsigned* __restrict__ owner, int rows, int E, int V) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const long id = ids[row];
    RN_CHECK(id >= 0 && id < V);
    if (lane == 0) atomicMin(owner + id, (unsigned)row);
    for (int c = lane; c < E; c += 64) {
        const long long fx = __float2ll_rn(bf2f(dx[(long)row * E + c]) * FX_SCALE);
        atomicAdd(d64 + id * E + c, (unsigned long long)fx);  // two's complement: signed sum
    }
}

__global__ void __launch_bounds__(256) emb_finish_fx_k(const int64_t* __restrict__ ids,
                                                       unsigned long long* __restrict__ d64,
                                                       unsigned* __restrict__ owner, bf16* __restrict__ g, int rows,
                                                       int E) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const long id = ids[row];
    if (owner[id] != (unsigned)row) return;
    for (int c = lane; c < E; c += 64) {
        const long long v = (long long)d64[id * E + c];
        d64[id * E + c] = 0ull;
        bf16* q = g + id * E + c;
        q[0] = (bf16)((float)q[0] + (float)((double)v * (1.0 / 1099511627776.0)));
    }
    if (lane == 0) owner[id] = 0xFFFFFFFFu;
}

// dwpe[t] += sum_b dx[b, t]
__global__ void emb_pos_acc_k(const bf16* __restrict__ dx, bf16* __restrict__ dwpe, int B, int T, int E) {
    const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (i >= (long)T * E) return;
    const int t = i / E, c = i % E;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += bf2f(dx[((long)b * T + t) * E + c]);
    dwpe[i] = f2bf(bf2f(dwpe[i]) + s);
}

// dwpe[t] = sum_b dx[b, t]   (thread per column, loops over the batch)
__global__ void emb_bwd_pos_k(const bf16* __restrict__ dx, bf16* __restrict__ dwpe, int B, int T, int Tp, int E) {
    const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (i >= (long)Tp * E) return;
    const int t = i / E, c = i % E;
    float s = 0.f;
    if (t < T)
        for (int b = 0; b < B; ++b) s += bf2f(dx[((long)b * T + t) * E + c]);
    dwpe[i] = f2bf(s);
}

__global__ void f32_to_bf16_k(const float* __restrict__ a, bf16* __restrict__ b, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n / 4; i += (long)gridDim.x * blockDim.x) {
        float4 v = reinterpret_cast<const float4*>(a)[i];
        bf16x4 o = {(bf16)v.x, (bf16)v.y, (bf16)v.z, (bf16)v.w};
        reinterpret_cast<bf16x4*>(b)[i] = o;
    }
    for (long i = (n / 4) * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        b[i] = (bf16)a[i];
}

// ---- global squared norm: fixed-order two-stage reduction (deterministic) ----
constexpr int NORM_BLOCKS = 1024;

template <typename T>
__global__ void __launch_bounds__(256) sumsq_part_k(const T* __restrict__ g, long n, float* __restrict__ part) {
    __shared__ float sm[16];
    float s = 0.f;
    if constexpr (sizeof(T) == 2) {
        for (long i = blockIdx.x * 256L + threadIdx.x; i < n / 8; i += (long)gridDim.x * 256) {
            float f[8];
            load8((const bf16*)g + i * 8, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) s += f[j] * f[j];
        }
        for (long i = (n / 8) * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
            float f = bf2f(((const bf16*)g)[i]);
            s += f * f;
        }
    } else {
        for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
            float f = ((const float*)g)[i];
            s += f * f;
        }
    }
    s = block_sum(s, sm);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) sumsq_final_k(const float* __restrict__ part, int np, float* __restrict__ out) {
    __shared__ float sm[16];
    float s = 0.f;
    for (int i = threadIdx.x; i < np; i += 256) s += part[i];
    s = block_sum(s, sm);
    if (threadIdx.x == 0) { out[0] = s; out[1] = 0.f; }
}

// clip coefficient from the device-resident squared norm; <0 means "skip step"
RN_DEV float clip_coef(const float* normbuf, float grad_scale, float clip) {
    float nrm = sqrtf(normbuf[0]) * grad_scale;
    if (!isfinite(nrm)) return -1.f;
    return (clip > 0.f && nrm > clip) ? clip / (nrm + 1e-6f) : 1.f;
}

// fp32 → bf16 with stochastic rounding: add 16 random low bits, truncate (unbiased: E[bf16] = w).
// The bits hash (element index, optimizer step): deterministic for a given step, fresh every step,
// and graph-capturable (the step count lives in device memory).
RN_DEV uint32_t sr_hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7FEB352Du;
    x ^= x >> 15; x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}
RN_DEV void store8_sr(bf16* dst, const float (&w)[8], long e, uint32_t step) {
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        uint32_t h[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const uint32_t bits = __float_as_uint(w[j + u]);
            const uint32_t r = sr_hash((uint32_t)(e + j + u) ^ (step * 0x9E3779B9u)) & 0xFFFFu;
            // finite values only (inf / nan keep nearest rounding's upper half unchanged)
            h[u] = ((bits & 0x7F800000u) == 0x7F800000u) ? (bits >> 16) : ((bits + r) >> 16);
        }
        o[j / 2] = h[0] | (h[1] << 16);
    }
    *reinterpret_cast<uint4*>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
}

// AdamW over the flat buffer, 8 elements per lane.  SR: stochastic rounding of the bf16 weight copy
// (the fp32 master is exact either way).
template <typename GT, bool SR>
__global__ void __launch_bounds__(256) adamw_k(bf16* __restrict__ p, float* __restrict__ master,
                                               const GT* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                                               const uint8_t* __restrict__ wdm, float* __restrict__ normbuf, long n,
                                               float b1, float b2, float eps, float wd, float grad_scale, float clip) {
    const uint32_t step = (uint32_t)normbuf[2];
    const float coef = clip_coef(normbuf, grad_scale, clip);
    const float lr = normbuf[3], bc1 = normbuf[4], bc2 = normbuf[5];
    if (coef < 0.f) {
        if (blockIdx.x == 0 && threadIdx.x == 0) normbuf[1] = 1.f;  // step skipped (non-finite grads)
        return;
    }
    const float gs = grad_scale * coef;
    const float rbc1 = 1.f / bc1, rbc2 = 1.f / bc2;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n / 8; i += (long)gridDim.x * 256) {
        const long e = i * 8;
        float gf[8];
        if constexpr (sizeof(GT) == 2) load8((const bf16*)g + e, gf);
        else {
            float4 a = reinterpret_cast<const float4*>(g + e)[0], b = reinterpret_cast<const float4*>(g + e)[1];
            gf[0] = a.x; gf[1] = a.y; gf[2] = a.z; gf[3] = a.w; gf[4] = b.x; gf[5] = b.y; gf[6] = b.z; gf[7] = b.w;
        }
        float4* mm = reinterpret_cast<float4*>(m + e);
        float4* vv = reinterpret_cast<float4*>(v + e);
        float4* ww = reinterpret_cast<float4*>(master + e);
        float4 m0 = mm[0], m1 = mm[1], v0 = vv[0], v1 = vv[1], w0 = ww[0], w1 = ww[1];
        float mf[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
        float vf[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        float wf[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float wdl = wdm[e >> 6] ? wd : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float gg = gf[j] * gs;
            mf[j] = b1 * mf[j] + (1.f - b1) * gg;
            vf[j] = b2 * vf[j] + (1.f - b2) * gg * gg;
            float upd = (mf[j] * rbc1) / (sqrtf(vf[j] * rbc2) + eps) + wdl * wf[j];
            wf[j] -= lr * upd;
        }
        mm[0] = make_float4(mf[0], mf[1], mf[2], mf[3]);
        mm[1] = make_float4(mf[4], mf[5], mf[6], mf[7]);
        vv[0] = make_float4(vf[0], vf[1], vf[2], vf[3]);
        vv[1] = make_float4(vf[4], vf[5], vf[6], vf[7]);
        ww[0] = make_float4(wf[0], wf[1], wf[2], wf[3]);
        ww[1] = make_float4(wf[4], wf[5], wf[6], wf[7]);
        if constexpr (SR) store8_sr(p + e, wf, e, step);
        else store8(p + e, wf);
    }
}

template <typename GT>
__global__ void __launch_bounds__(256) sgd_k(bf16* __restrict__ p, float* __restrict__ master, const GT* __restrict__ g,
                                             float* __restrict__ buf, const uint8_t* __restrict__ wdm,
                                             float* __restrict__ normbuf, long n, float mom, float wd,
                                             int nesterov, float grad_scale, float clip) {
    const float coef = clip_coef(normbuf, grad_scale, clip);
    const float lr = normbuf[3];
    const int first = normbuf[2] == 1.f;
    if (coef < 0.f) {
        if (blockIdx.x == 0 && threadIdx.x == 0) normbuf[1] = 1.f;
        return;
    }
    const float gs = grad_scale * coef;
    for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
        float gg = (sizeof(GT) == 2 ? bf2f(((const bf16*)g)[e]) : (float)((const float*)g)[e]) * gs;
        float w = master[e];
        gg += (wdm[e >> 6] ? wd : 0.f) * w;
        float b = first ? gg : mom * buf[e] + gg;
        buf[e] = b;
        float d = nesterov ? gg + mom * b : b;
        w -= lr * d;
        master[e] = w;
        p[e] = f2bf(w);
    }
}

// Optimizer step prologue (1 thread): step counter, LR schedule and Adam bias
// corrections live in device memory, so a captured hipGraph replays correct
// per-step hyper-parameters.  state: [sumsq, skipped, t, lr, bc1, bc2]
__global__ void opt_prep_k(float* __restrict__ st, float base_lr, float warmup, float total, float min_ratio,
                           int cosine, float lr_override, float b1, float b2) {
    const float t = st[2] + 1.f;
    st[2] = t;
    float lr = base_lr;
    if (lr_override >= 0.f) lr = lr_override;
    else if (cosine) {
        const float i = t - 1.f;
        if (i < warmup) lr = base_lr * (i + 1.f) / warmup;
        else {
            float x = fminf(1.f, (i - warmup) / fmaxf(1.f, total - warmup));
            lr = base_lr * (min_ratio + (1.f - min_ratio) * 0.5f * (1.f + cosf(3.14159265358979f * x)));
        }
    }
    st[3] = lr;
    st[4] = 1.f - powf(b1, t);
    st[5] = 1.f - powf(b2, t);
}

inline int grid_for(long work) {
    // grid cap of the optimizer / embedding streaming kernels (grid-stride loops past it)
    constexpr long cap = 4096L;
    long g = (work + 255) / 256;
    return (int)(g < cap ? (g > 0 ? g : 1) : cap);
}

}  // namespace

extern "C" {

void rn_emb_fwd(const int64_t* ids, const void* wte, const void* wpe, void* x, int rows, int T, int E, int V,
                hipStream_t st) {
    dim3 g((rows + 3) / 4);
    if (wpe) emb_fwd_k<true><<<g, 256, 0, st>>>(ids, (const bf16*)wte, (const bf16*)wpe, (bf16*)x, rows, T, E, V);
    else emb_fwd_k<false><<<g, 256, 0, st>>>(ids, (const bf16*)wte, nullptr, (bf16*)x, rows, T, E, V);
}

// dwte32: V*E fp32 scratch (zeroed here); dwte: bf16 out; dwpe: bf16 (Tp*E) or null
void rn_emb_bwd(const int64_t* ids, const void* dx, float* dwte32, void* dwte, void* dwpe, int B, int T, int Tp,
                int V, int E, hipStream_t st) {
    int rows = B * T;
    (void)hipMemsetAsync(dwte32, 0, (size_t)V * E * 4, st);
    emb_bwd_scatter_k<<<(rows + 3) / 4, 256, 0, st>>>(ids, (const bf16*)dx, dwte32, rows, E);
    long n = (long)V * E;
    f32_to_bf16_k<<<grid_for(n / 4), 256, 0, st>>>(dwte32, (bf16*)dwte, n);
    if (dwpe) emb_bwd_pos_k<<<rn_cdiv((long)Tp * E, 256), 256, 0, st>>>((const bf16*)dx, (bf16*)dwpe, B, T, Tp, E);
}

// E % 4 == 0.  gwte (bf16 V×E) and gwpe (bf16 ≥T×E, may be null) are accumulated into.
void rn_emb_bwd_acc(const int64_t* ids, const void* dx, float* d32, unsigned* owner, void* gwte, void* gwpe, int B,
                    int T, int E, int V, hipStream_t st) {
    const int rows = B * T;
    emb_scatter_own_k<<<(rows + 3) / 4, 256, 0, st>>>(ids, (const bf16*)dx, d32, owner, rows, E, V);
    emb_finish_k<<<(rows + 3) / 4, 256, 0, st>>>(ids, d32, owner, (bf16*)gwte, rows, E);
    if (gwpe) emb_pos_acc_k<<<rn_cdiv((long)T * E, 256), 256, 0, st>>>((const bf16*)dx, (bf16*)gwpe, B, T, E);
}

// ---- ViT token join: x[b, 0] = cls + pos[0], x[b, 1 + p] = patch[b, p] + pos[1 + p] ----
// (replaces torch.cat + broadcast add in the forward and the slice copy + two batch reductions of
// their backward: one pass each way)
__global__ void __launch_bounds__(256) vit_join_fwd_k(const bf16* __restrict__ patch, const bf16* __restrict__ cls,
                                                      const bf16* __restrict__ pos, bf16* __restrict__ out, int B, int P,
                                                      int E) {
    const long i = blockIdx.x * 256L + threadIdx.x;  // one 8-element chunk
    const int e8 = E / 8;
    if (i >= (long)B * (P + 1) * e8) return;
    const int c = (int)(i % e8);
    const long bt = i / e8;
    const int t = (int)(bt % (P + 1));
    const long b = bt / (P + 1);
    float x[8], q[8];
    load8((t == 0 ? cls : patch + (b * P + t - 1) * E) + c * 8, x);
    load8(pos + (long)t * E + c * 8, q);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] += q[j];
    store8(out + bt * E + c * 8, x);
}

// backward: dpatch[b, p] = dx[b, 1 + p]; gpos[t] += Σ_b dx[b, t]; gcls += Σ_b dx[b, 0].
// grid (P + 1, ceil(E / 256)); 256 threads = 32 column chunks of 8 × 8 batch lanes, one LDS merge
// of the 8 lane partials (fixed order: deterministic).
__global__ void __launch_bounds__(256) vit_join_bwd_k(const bf16* __restrict__ dx, bf16* __restrict__ dpatch,
                                                      bf16* __restrict__ gcls, bf16* __restrict__ gpos, int B, int P,
                                                      int E) {
    __shared__ float part[8][32 * 8];
    const int t = blockIdx.x, cg = threadIdx.x & 31, bl = threadIdx.x >> 5;
    const int col = (blockIdx.y * 32 + cg) * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (col < E) {
        for (int b = bl; b < B; b += 8) {
            float v[8];
            load8(dx + ((long)b * (P + 1) + t) * E + col, v);
            if (t > 0) store8(dpatch + ((long)b * P + t - 1) * E + col, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] += v[j];
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) part[bl][cg * 8 + j] = acc[j];
    __syncthreads();
    if (bl == 0 && col < E) {
        float s[8], g[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            s[j] = 0.f;
#pragma unroll
            for (int l = 0; l < 8; ++l) s[j] += part[l][cg * 8 + j];
        }
        load8(gpos + (long)t * E + col, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] += s[j];
        store8(gpos + (long)t * E + col, g);
        if (t == 0) {
            load8(gcls + col, g);
#pragma unroll
            for (int j = 0; j < 8; ++j) g[j] += s[j];
            store8(gcls + col, g);
        }
    }
}

// deterministic variant: d64 = persistent zeroed V×E 64-bit scratch
void rn_emb_bwd_acc_det(const int64_t* ids, const void* dx, void* d64, unsigned* owner, void* gwte, void* gwpe, int B,
                        int T, int E, int V, hipStream_t st) {
    const int rows = B * T;
    emb_scatter_own_fx_k<<<(rows + 3) / 4, 256, 0, st>>>(ids, (const bf16*)dx, (unsigned long long*)d64, owner, rows,
                                                        E, V);
    emb_finish_fx_k<<<(rows + 3) / 4, 256, 0, st>>>(ids, (unsigned long long*)d64, owner, (bf16*)gwte, rows, E);
    if (gwpe) emb_pos_acc_k<<<rn_cdiv((long)T * E, 256), 256, 0, st>>>((const bf16*)dx, (bf16*)gwpe, B, T, E);
}

void rn_vit_join_fwd(const void* patch, const void* cls, const void* pos, void* out, int B, int P, int E, hipStream_t st) {
    const long n = (long)B * (P + 1) * (E / 8);
    vit_join_fwd_k<<<rn_cdiv(n, 256), 256, 0, st>>>((const bf16*)patch, (const bf16*)cls, (const bf16*)pos, (bf16*)out, B,
                                                    P, E);
}
void rn_vit_join_bwd(const void* dx, void* dpatch, void* gcls, void* gpos, int B, int P, int E, hipStream_t st) {
    dim3 grid(P + 1, (E + 255) / 256);
    vit_join_bwd_k<<<grid, 256, 0, st>>>((const bf16*)dx, (bf16*)dpatch, (bf16*)gcls, (bf16*)gpos, B, P, E);
}

int rn_norm_ws_floats() { return NORM_BLOCKS; }

// normbuf[0] = sum(g^2), normbuf[1] = 0 (skip flag); part: NORM_BLOCKS floats
void rn_sumsq(const void* g, long n, int is_bf16, float* part, float* normbuf, hipStream_t st) {
    int gb = grid_for(n / 8);
    if (gb > NORM_BLOCKS) gb = NORM_BLOCKS;
    if (is_bf16) sumsq_part_k<bf16><<<gb, 256, 0, st>>>((const bf16*)g, n, part);
    else sumsq_part_k<float><<<gb, 256, 0, st>>>((const float*)g, n, part);
    sumsq_final_k<<<1, 256, 0, st>>>(part, gb, normbuf);
}

void rn_opt_prep(float* state, float base_lr, float warmup, float total, float min_ratio, int cosine,
                 float lr_override, float b1, float b2, hipStream_t st) {
    opt_prep_k<<<1, 1, 0, st>>>(state, base_lr, warmup, total, min_ratio, cosine, lr_override, b1, b2);
}

int rn_adamw(void* p, float* master, const void* g, int g_bf16, float* m, float* v, const uint8_t* wdm,
             float* state, long n, float b1, float b2, float eps, float wd, float grad_scale, float clip, int sr,
             hipStream_t st) {
    if (n % 8) return -1;
    int gb = grid_for(n / 8);
#define RN_ADAMW(GT, SRV) \
    adamw_k<GT, SRV><<<gb, 256, 0, st>>>((bf16*)p, master, (const GT*)g, m, v, wdm, state, n, b1, b2, eps, wd, grad_scale, clip)
    if (g_bf16) { if (sr) RN_ADAMW(bf16, true); else RN_ADAMW(bf16, false); }
    else { if (sr) RN_ADAMW(float, true); else RN_ADAMW(float, false); }
#undef RN_ADAMW
    return 0;
}

void rn_sgd(void* p, float* master, const void* g, int g_bf16, float* buf, const uint8_t* wdm, float* state, long n,
            float mom, float wd, int nesterov, float grad_scale, float clip, hipStream_t st) {
    int gb = grid_for(n);
    if (g_bf16)
        sgd_k<bf16><<<gb, 256, 0, st>>>((bf16*)p, master, (const bf16*)g, buf, wdm, state, n, mom, wd, nesterov,
                                        grad_scale, clip);
    else
        sgd_k<float><<<gb, 256, 0, st>>>((bf16*)p, master, (const float*)g, buf, wdm, state, n, mom, wd, nesterov,
                                         grad_scale, clip);
}

}  // extern "C"
