#include <hip/hip_runtime.h>
// What wait states does LLVM insert on gfx950 (compile only; read the .s):
//   hipcc --offload-arch=gfx950 -O3 -c tools/calib/llvm_hazard_probe.hip --save-temps
// valu_to_mfma: VALU write -> MFMA read (2 wait states), MFMA -> VALU read (s_nop 11);
// chain_*: dependent packed-FP32 ops get one s_nop 0 between them; op_sel gets nothing more.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));
extern "C" __global__ void valu_to_mfma(const h8* a, const unsigned* b, f16v* c, float* o) {
  int l = threadIdx.x;
  unsigned x = b[l];
  h8 bb; 
  for (int i = 0; i < 8; ++i) bb[i] = (_Float16)(float)((x >> i) & 3);
  f16v acc = c[l];
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[l], bb, acc, 0, 0, 0);
  // MFMA -> VALU read
  float s = acc[0] * 3.0f + acc[5];
  o[l] = s;
}
extern "C" __global__ void pk(const f2* a, const f2* w, f2* o) {
  int l = threadIdx.x;
  f2 x = a[l], ww = w[l];
  f2 r = x * (f2){ww.y, ww.y} + ww;
  o[l] = r;
}
extern "C" __global__ void chain_hi(const f2* a, const f2* w, f2* o) {
  int l = threadIdx.x; f2 x = a[l], acc = {0,0};
  #pragma unroll
  for (int i = 0; i < 6; ++i) { f2 ww = w[i]; acc = x * (f2){ww.x, ww.x} + acc; }
  o[l] = acc;
}
extern "C" __global__ void chain_sel(const f2* a, const f2* w, f2* o) {
  int l = threadIdx.x; f2 x = a[l], acc = {0,0};
  #pragma unroll
  for (int i = 0; i < 6; ++i) { f2 ww = w[i]; acc = x * (f2){ww.y, ww.y} + acc; }
  o[l] = acc;
}
extern "C" __global__ void chain_add(const f2* a, const f2* w, f2* o) {
  int l = threadIdx.x; f2 x = a[l], acc = {0,0};
  #pragma unroll
  for (int i = 0; i < 6; ++i) { f2 ww = w[i]; acc = acc + x + ww; }
  float s = acc.x + 1.0f;
  o[l] = acc + s;
}
