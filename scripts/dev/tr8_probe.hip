#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x2 __attribute__((ext_vector_type(2)));
__global__ void probe(int* out, int mode) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[64 * 64];
    const int l = threadIdx.x;
    for (int i = l; i < 64 * 64; i += 64) lds[i] = (unsigned char)(((i / 64) & 15) * 16 + (i % 64 & 15));
    __syncthreads();
    const int g = l >> 4, i = l & 15;
    int row, col;
    if (mode == 0) { row = i >> 1; col = (i & 1) * 8; }        // hypothesis: lane 2q+p -> row q, cols 8p..
    else { row = i & 7; col = (i >> 3) * 8; }                  // alternative: lane q+8p
    row += g * 8;
    const char* a = (const char*)lds + row * 64 + col;
    i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)a);
    out[l * 2] = v[0];
    out[l * 2 + 1] = v[1];
}
int main() {
    int* d; hipMalloc(&d, 128 * 4);
    int h[128];
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(probe, 1, 64, 0, 0, d, mode);
        hipMemcpy(h, d, 128 * 4, hipMemcpyDeviceToHost);
        printf("mode %d\n", mode);
        for (int l = 0; l < 64; ++l) {
            const unsigned char* b = (const unsigned char*)&h[l * 2];
            printf("lane %2d:", l);
            for (int k = 0; k < 8; ++k) printf(" r%02d c%02d", b[k] >> 4, b[k] & 15);
            printf("\n");
        }
    }
    return 0;
}
