// Does v_pk_fma_f32 with op_sel:[0,1,0] give wrong results on gfx950 when two waves
// share a SIMD?  (round 4's 2-ply evaluator fault.)
//
// The 2-ply evaluator's wide value-head epilogue in isolation (bg_search.hip
// eval_leaves_fact, kWide): two 32-leaf tiles x 4 unit tiles of MFMA accumulators
// (6 k-blocks of v_mfma_f32_32x32x16_f16), then a[n] += relu(x[n][t][r]) * w over
// 128 units with the head weights read from LDS as float4.  Three forms of the
// epilogue, which must agree bit for bit (an FMA is rounded per element either way):
//   MODE 0  scalar v_fma_f32 (the reference)
//   MODE 1  the two tiles packed into v_pk_fma_f32, the odd weights broadcast with
//           op_sel:[0,1,0] -- the instruction sequence of the failing round-4 build
//   MODE 2  the same packing, the odd weights first copied (v_mov) and broadcast with
//           op_sel_hi:[1,0,1] (the form the product library may contain)
// The packed forms are inline asm, each followed by the one wait state LLVM puts
// after a packed-FP32 result (its hazard recognizer cannot see into asm).
// The host runs MODE 0 once as the reference, then each mode several times at
// 2 waves/SIMD (512-thread workgroups, one per CU by LDS) and 1 wave/SIMD (256
// threads), and counts mismatches by leaf tile and lane group of 16.
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form
//        tools/calib/pk_opsel_probe.hip -o tools/calib/pk_opsel_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float relu_raw(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// features: small exact f16 values (0, 0.5, 1, 1.5) from a hash
__device__ __forceinline__ f16x8 feat(uint32_t s) {
    f16x8 f;
    #pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = (_Float16)(0.5f * (float)((s >> (2 * i)) & 3u));
    return f;
}

// acc += x * (w.lo, w.lo)
__device__ __forceinline__ void pk_lo(f32x2& acc, f32x2 x, f32x2 w) {
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]\n\ts_nop 0" : "+v"(acc) : "v"(x), "v"(w));
}
// acc += x * (w.hi, w.hi) by op_sel (the low element reads the high dword)
__device__ __forceinline__ void pk_hi_opsel(f32x2& acc, f32x2 x, f32x2 w) {
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0]\n\ts_nop 0" : "+v"(acc) : "v"(x), "v"(w));
}
// acc += x * (w.hi, w.hi) by a copy to the low position first
__device__ __forceinline__ void pk_hi_mov(f32x2& acc, f32x2 x, f32x2 w) {
    f32x2 t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t.x) : "v"(w.y));
    t.y = 0.0f;
    pk_lo(acc, x, t);
}

template <int MODE>
__global__ void __launch_bounds__(512) k_epilogue(const f16x8* __restrict__ wq, const float4* __restrict__ wv,
                                                  float* __restrict__ out, int iters, int z) {
    extern __shared__ float4 wvs[];            // 16 x 64 float4 used; the launch asks for more (occupancy)
    const int l = threadIdx.x & 63, h = l >> 5;
    for (int i = threadIdx.x; i < 16 * 64; i += blockDim.x) wvs[i] = wv[i];
    __syncthreads();
    const uint32_t gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    for (int it = 0; it < iters; ++it) {
        f32x16 x[2][4];
        #pragma unroll
        for (int kb = 0; kb < 6; ++kb) {
            f16x8 f[2];
            #pragma unroll
            for (int n = 0; n < 2; ++n) f[n] = feat(mix((gw * 64 + it) * 32 + kb * 4 + n * 2 + h) ^ mix(l + 77));
            #pragma unroll
            for (int t = 0; t < 4; ++t) {
                const f16x8 a = wq[(kb * 4 + t) * 64 + l + z];
                #pragma unroll
                for (int n = 0; n < 2; ++n)
                    x[n][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, f[n], kb == 0 ? (f32x16){} : x[n][t], 0, 0, 0);
            }
        }
        float a0 = 0.0f, a1 = 0.0f;
        f32x2 acc = {0.0f, 0.0f};
        #pragma unroll
        for (int t = 0; t < 4; ++t)
            #pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const float4 w = wvs[(t * 4 + r4) * 64 + l + z];
                if constexpr (MODE == 0) {
                    #pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float wj = j == 0 ? w.x : j == 1 ? w.y : j == 2 ? w.z : w.w;
                        a0 = fmaf(relu_raw(x[0][t][4 * r4 + j]), wj, a0);
                        a1 = fmaf(relu_raw(x[1][t][4 * r4 + j]), wj, a1);
                    }
                } else {
                    const f32x2 wxy = {w.x, w.y}, wzw = {w.z, w.w};
                    f32x2 p[4];
                    #pragma unroll
                    for (int j = 0; j < 4; ++j) p[j] = (f32x2){relu_raw(x[0][t][4 * r4 + j]), relu_raw(x[1][t][4 * r4 + j])};
                    pk_lo(acc, p[0], wxy);
                    if constexpr (MODE == 1) pk_hi_opsel(acc, p[1], wxy); else pk_hi_mov(acc, p[1], wxy);
                    pk_lo(acc, p[2], wzw);
                    if constexpr (MODE == 1) pk_hi_opsel(acc, p[3], wzw); else pk_hi_mov(acc, p[3], wzw);
                }
            }
        if constexpr (MODE != 0) { a0 = acc.x; a1 = acc.y; }
        out[((size_t)gw * iters + it) * 128 + l] = a0;
        out[((size_t)gw * iters + it) * 128 + 64 + l] = a1;
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

template <int MODE>
void launch(int blocks, int threads, size_t lds, const f16x8* wq, const float4* wv, float* out, int iters) {
    hipLaunchKernelGGL(k_epilogue<MODE>, dim3(blocks), dim3(threads), lds, 0, wq, wv, out, iters, 0);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 1024, iters = argc > 2 ? atoi(argv[2]) : 16,
              trials = argc > 3 ? atoi(argv[3]) : 4;
    const size_t lds = 100 * 1024;          // one workgroup per CU (160 KiB of LDS per CU)
    srand(1234);
    std::vector<_Float16> hq(24 * 64 * 8);
    for (auto& v : hq) v = (_Float16)((float)(rand() % 2001 - 1000) / 1000.0f);
    std::vector<float> hw(16 * 64 * 4);
    for (auto& v : hw) v = (float)(rand() % 2001 - 1000) / 997.0f;
    f16x8* wq; float4* wv; float *ref, *out;
    CK(hipMalloc(&wq, hq.size() * 2)); CK(hipMalloc(&wv, hw.size() * 4));
    CK(hipMemcpy(wq, hq.data(), hq.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(wv, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute((const void*)k_epilogue<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)k_epilogue<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)k_epilogue<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const size_t n_max = (size_t)blocks * 8 * iters * 128;
    CK(hipMalloc(&ref, n_max * 4)); CK(hipMalloc(&out, n_max * 4));
    std::vector<uint32_t> hr(n_max), ho(n_max);
    long bad_total[3] = {};
    for (int threads : {512, 256}) {
        const size_t n = (size_t)blocks * (threads / 64) * iters * 128;
        launch<0>(blocks, threads, lds, wq, wv, ref, iters);
        CK(hipGetLastError()); CK(hipDeviceSynchronize());
        CK(hipMemcpy(hr.data(), ref, n * 4, hipMemcpyDeviceToHost));
        for (int mode = 0; mode < 3; ++mode)
            for (int tr = 0; tr < trials; ++tr) {
                CK(hipMemset(out, 0xff, n * 4));
                hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
                CK(hipEventRecord(e0));
                if (mode == 0) launch<0>(blocks, threads, lds, wq, wv, out, iters);
                else if (mode == 1) launch<1>(blocks, threads, lds, wq, wv, out, iters);
                else launch<2>(blocks, threads, lds, wq, wv, out, iters);
                CK(hipGetLastError()); CK(hipEventRecord(e1)); CK(hipDeviceSynchronize());
                float ms = 0; CK(hipEventElapsedTime(&ms, e0, e1));
                CK(hipMemcpy(ho.data(), out, n * 4, hipMemcpyDeviceToHost));
                long bad = 0, by[2][4] = {};
                for (size_t i = 0; i < n; ++i)
                    if (hr[i] != ho[i]) { ++bad; by[(i / 64) & 1][(i & 63) / 16]++; }
                bad_total[mode] += bad;
                printf("{\"waves_per_simd\": %d, \"mode\": %d, \"trial\": %d, \"ms\": %.3f, \"values\": %zu, \"mismatches\": %ld, "
                       "\"tile0_by_lane16\": [%ld, %ld, %ld, %ld], \"tile1_by_lane16\": [%ld, %ld, %ld, %ld]}\n",
                       threads / 256, mode, tr, ms, n, bad, by[0][0], by[0][1], by[0][2], by[0][3],
                       by[1][0], by[1][1], by[1][2], by[1][3]);
                fflush(stdout);
            }
    }
    printf("{\"mismatches_by_mode\": [%ld, %ld, %ld]}\n", bad_total[0], bad_total[1], bad_total[2]);
    return 0;
}
