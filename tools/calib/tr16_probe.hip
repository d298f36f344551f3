// Probe of ds_read_b64_tr_b16's lane mapping (the layout bg_ppo_fused.hip assumes):
// LDS holds a [64][64] u16 tile with value = row * 256 + col; every lane of group g
// supplies the address of row q = (l & 15) >> 2, columns 4p..4p+3 (p = l & 3) of
// block (rows 4g.., cols 0..15); prints what each lane receives.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short s16x4 __attribute__((__vector_size__(4 * sizeof(short))));
__global__ void k(short* out) {
    __shared__ __attribute__((aligned(16))) short s[64 * 64];
    for (int i = threadIdx.x; i < 64 * 64; i += 64) s[i] = (short)(((i / 64) << 8) | (i % 64));
    __syncthreads();
    const int l = threadIdx.x, g = l >> 4, q = (l & 15) >> 2, p = l & 3;
    const short* a = s + (4 * g + q) * 64 + 4 * p;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) void*)a);
    for (int j = 0; j < 4; ++j) out[4 * l + j] = v[j];
}
int main() {
    short* d; hipMalloc(&d, 512); hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    short h[256]; hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) {
        printf("lane %2d:", l);
        for (int j = 0; j < 4; ++j) printf(" (r%d,c%d)", (h[4 * l + j] >> 8) & 255, h[4 * l + j] & 255);
        printf("\n");
    }
    return 0;
}
