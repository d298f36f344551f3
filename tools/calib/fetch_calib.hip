// FETCH_SIZE / WRITE_SIZE calibration for the env step's narrow access shapes
// (MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated: calibrate on
// a known byte count in your own access pattern").  Each kernel touches a known
// number of distinct bytes in distinct lines, from buffers far larger than the
// L2s and the 256 MiB Infinity Cache is flushed by a 512 MiB sweep in between.
//   k_rec64   one wave per 64-B record, 1 B per lane (load_rec), stride 4 KiB: 64 B/wave
//   k_u64     one wave per lane-slot, lane 0 loads 8 B at stride 4 KiB:        8 B/wave
//   k_u32     same, 4 B                                                          4 B/wave
//   k_wide    16 B/lane coalesced stream (the guide's calibrated case)
//   k_st64 / k_st8 / k_st4   the same shapes as stores
// Prints nothing; run under rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t kStride = 4096;
constexpr int kWaves = 32768;

__global__ __launch_bounds__(64) void k_rec64(const uint8_t* p, int* sink) {
    const int v = p[(size_t)blockIdx.x * kStride + threadIdx.x];
    if (v == 0xAB) sink[0] = v;
}
// the lane-record array itself: 64-B records back to back (two per 128-B line)
__global__ __launch_bounds__(64) void k_rec64_dense(const uint8_t* p, int* sink) {
    const int v = p[(size_t)blockIdx.x * 64 + threadIdx.x];
    if (v == 0xAB) sink[0] = v;
}
__global__ __launch_bounds__(64) void k_u64(const uint64_t* p, int* sink) {
    if (threadIdx.x == 0) { const uint64_t v = p[(size_t)blockIdx.x * (kStride / 8)]; if (v == 0x7fffffffull) sink[0] = 1; }
}
__global__ __launch_bounds__(64) void k_u32(const uint32_t* p, int* sink) {
    if (threadIdx.x == 0) { const uint32_t v = p[(size_t)blockIdx.x * (kStride / 4)]; if (v == 0x7fffffffu) sink[0] = 1; }
}
__global__ __launch_bounds__(256) void k_wide(const uint4* p, int* sink, size_t n) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) { const uint4 v = p[i]; acc ^= v.x ^ v.w; }
    if (acc == 0x7fffffffu) sink[0] = 1;
}
__global__ __launch_bounds__(64) void k_st64(uint8_t* p) { p[(size_t)blockIdx.x * kStride + threadIdx.x] = 1; }
__global__ __launch_bounds__(64) void k_st8(uint64_t* p) { if (threadIdx.x == 0) p[(size_t)blockIdx.x * (kStride / 8)] = 1; }
__global__ __launch_bounds__(64) void k_st4(uint32_t* p) { if (threadIdx.x == 0) p[(size_t)blockIdx.x * (kStride / 4)] = 1; }
__global__ __launch_bounds__(256) void k_flush(uint4* p, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = make_uint4(i, 0, 0, 0);
}

int main() {
    const size_t big = (size_t)kWaves * kStride;          // 128 MiB
    const size_t flush = (size_t)512 << 20;
    uint8_t *a, *f; int* sink;
    if (hipMalloc(&a, big) || hipMalloc(&f, flush) || hipMalloc(&sink, 64)) return 1;
    if (hipMemset(a, 0, big)) return 1;
    auto fl = [&] { hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, (uint4*)f, flush / 16); };
    for (int rep = 0; rep < 3; ++rep) {
        fl(); hipLaunchKernelGGL(k_rec64, dim3(kWaves), dim3(64), 0, 0, a, sink);
        fl(); hipLaunchKernelGGL(k_rec64_dense, dim3(kWaves), dim3(64), 0, 0, a, sink);
        fl(); hipLaunchKernelGGL(k_u64, dim3(kWaves), dim3(64), 0, 0, (const uint64_t*)a, sink);
        fl(); hipLaunchKernelGGL(k_u32, dim3(kWaves), dim3(64), 0, 0, (const uint32_t*)a, sink);
        fl(); hipLaunchKernelGGL(k_wide, dim3(4096), dim3(256), 0, 0, (const uint4*)a, sink, big / 16);
        fl(); hipLaunchKernelGGL(k_st64, dim3(kWaves), dim3(64), 0, 0, a);
        fl(); hipLaunchKernelGGL(k_st8, dim3(kWaves), dim3(64), 0, 0, (uint64_t*)a);
        fl(); hipLaunchKernelGGL(k_st4, dim3(kWaves), dim3(64), 0, 0, (uint32_t*)a);
    }
    if (hipDeviceSynchronize()) return 2;
    printf("known bytes per launch: rec64 %d, u64 %d, u32 %d, wide %zu\n", kWaves * 64, kWaves * 8, kWaves * 4, big);
    return 0;
}
