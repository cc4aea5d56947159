// Comm proxy: a one-GPU stand-in for an 8-GPU RCCL collective's footprint on the local device
// (parallel/comm.py, REPLICANN_COMM=proxy).  On a single MI355X a world-1 all-reduce is a
// ~12 µs no-op, so the interaction that matters at N = 8 — RCCL workgroups occupying CUs and
// HBM bandwidth while the backward's GEMMs run — cannot be observed.  This kernel reproduces it:
//   * K workgroups of 256 threads on the comm stream (RCCL's channel blocks; K = REPLICANN_PROXY_WGS),
//   * each moving its share of the collective's per-GPU volume (ring all-reduce: 2·(W−1)/W·S bytes)
//     through HBM as 16-B reads + writes of the bucket itself (values unchanged: read, write back),
//   * paced to the per-GPU bus bandwidth of the emulated xGMI ring (REPLICANN_PROXY_GBPS), so the
//     workgroups hold their CUs for as long as the real collective would.
// Pacing uses the 100 MHz constant clock (s_memrealtime) with s_sleep between chunks.
#include "common.h"

namespace {

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) comm_proxy_k(v4u* __restrict__ buf, long n16, long per_wg16, double ns_per16) {
    const long base = (long)blockIdx.x * per_wg16;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    constexpr long CHUNK = 256 * 16;  // 16-B elements per chunk (64 KiB)
    for (long c = 0; c < per_wg16; c += CHUNK) {
        const long end = c + CHUNK < per_wg16 ? c + CHUNK : per_wg16;
#pragma unroll 4
        for (long i = c + threadIdx.x; i < end; i += 256) {
            const long j = (base + i) % n16;  // the volume wraps over the bucket
            v4u v = __builtin_nontemporal_load(buf + j);
            asm volatile("" : "+v"(v));
            buf[j] = v;
        }
        // pace: chunk c's bytes may not complete before (c + CHUNK)·ns_per16 after the start
        const double due_ns = (double)end * ns_per16;
        for (;;) {
            const double now_ns = (double)(__builtin_amdgcn_s_memrealtime() - t0) * 10.0;
            if (now_ns >= due_ns) break;
            __builtin_amdgcn_s_sleep(8);
        }
    }
}

}  // namespace

extern "C" void rn_comm_proxy(void* buf, long bytes, double volume_bytes, int wgs, double gbps, hipStream_t st) {
    const long n16 = bytes / 16;
    if (n16 <= 0 || wgs <= 0) return;
    const long total16 = (long)(volume_bytes / 16.0);
    const long per_wg16 = (total16 + wgs - 1) / wgs;
    // each workgroup moves per_wg16·16 bytes at (gbps / wgs) GB/s  ->  ns per 16-B element
    const double ns_per16 = 16.0 * wgs / gbps;
    comm_proxy_k<<<wgs, 256, 0, st>>>(reinterpret_cast<v4u*>(buf), n16, per_wg16, ns_per16);
}
