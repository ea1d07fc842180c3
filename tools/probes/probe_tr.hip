// Probe: semantics of ds_read_b64_tr_b16 and the 16x16x32 bf16 MFMA fed by it (prints per-lane data).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__global__ void k(short *out, int viaint) {
    __shared__ __attribute__((aligned(16))) short lds[64 * 32];
    for (int i = threadIdx.x; i < 64 * 32; i += 64) lds[i] = short(i);  // row r (32 cols): value r*32+c
    __syncthreads();
    const int lane = threadIdx.x, grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const short *addr = lds + (8 * grp + q) * 32 + 4 * p;  // group g: rows 8g+q, cols 4p..4p+3
    s16x4 v;
    if (viaint) v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(uintptr_t)addr);
    else v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)addr);
    for (int j = 0; j < 4; ++j) out[lane * 4 + j] = v[j];
}

int main() {
    short *d;
    hipMalloc(&d, 64 * 4 * 2);
    short h[256];
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("mode %s\n", mode ? "via uintptr" : "addrspace cast");
        for (int l = 0; l < 64; l += 5) {
            printf("lane %2d:", l);
            for (int j = 0; j < 4; ++j) printf(" (r%d c%d)", h[l * 4 + j] / 32, h[l * 4 + j] % 32);
            printf("\n");
        }
    }
    return 0;
}
