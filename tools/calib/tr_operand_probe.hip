// Checks bg_ppo_fused.hip's tr_operand on a swizzled [32][128] u16 image (value =
// row << 8 | col): element j of lane l must be row 16s + 8(j>>2) + 4(l>>5) + (j&3),
// column 32u + (l & 31).  Prints the mismatch count and the first few.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define BGX_PPO_GW2_TASK_TILES 32
namespace probe {
typedef short s16x4 __attribute__((__vector_size__(4 * sizeof(short))));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint32_t swz(int row, int ch) {
    return 256u * (uint32_t)row + 16u * (uint32_t)(ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}
__device__ __forceinline__ s16x4 tr16(const uint8_t* lds) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) void*)lds);
}
__device__ __forceinline__ void tr_operand(const uint8_t* img, int row0, int s, int u, int l, short* o) {
    const int g = l >> 4, q = (l & 15) >> 2, p = l & 3;
    const int r = row0 + 16 * s + 4 * (g >> 1) + q;
    const int ch = 4 * u + 2 * (g & 1) + (p >> 1);
    const s16x4 a = tr16(img + swz(r, ch) + 8 * (p & 1));
    const s16x4 b = tr16(img + swz(r + 8, ch) + 8 * (p & 1));
    for (int j = 0; j < 4; ++j) { o[j] = a[j]; o[4 + j] = b[j]; }
}
__global__ void k(short* out) {
    __shared__ __attribute__((aligned(16))) uint8_t img[32 * 256];
    const int l = threadIdx.x;
    for (int i = l; i < 32 * 128; i += 64) {
        const int row = i / 128, col = i % 128;
        *(short*)(img + swz(row, col / 8) + 2 * (col % 8)) = (short)((row << 8) | col);
    }
    __syncthreads();
    for (int s = 0; s < 2; ++s)
        for (int u = 0; u < 4; ++u) tr_operand(img, 0, s, u, l, out + ((s * 4 + u) * 64 + l) * 8);
}
}
int main() {
    short* d; hipMalloc(&d, 2 * 4 * 64 * 8 * 2);
    hipLaunchKernelGGL(probe::k, dim3(1), dim3(64), 0, 0, d);
    static short h[2 * 4 * 64 * 8]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int s = 0; s < 2; ++s) for (int u = 0; u < 4; ++u) for (int l = 0; l < 64; ++l) for (int j = 0; j < 8; ++j) {
        const short v = h[((s * 4 + u) * 64 + l) * 8 + j];
        const int er = 16 * s + 8 * (j >> 2) + 4 * (l >> 5) + (j & 3), ec = 32 * u + (l & 31);
        if (((v >> 8) & 255) != er || (v & 255) != ec) {
            if (bad < 12) printf("s%d u%d lane %d j%d: got (r%d,c%d) want (r%d,c%d)\n", s, u, l, j, (v >> 8) & 255, v & 255, er, ec);
            ++bad;
        }
    }
    printf("mismatches %d of %d\n", bad, 2 * 4 * 64 * 8);
    return 0;
}
