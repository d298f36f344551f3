// bg_ppo.hip — the PPO loss head of the update (ppo_agent.py:268-305) fused into
// one pass over the logits: masked log-softmax (mask = log(1e-45) for illegal
// actions, ppo_agent.py:166), the clipped surrogate, the value MSE and the
// entropy bonus, and their gradients with respect to the logits and the value,
// exactly as torch autograd forms them (min(): ties split the gradient in half;
// clamp(): inclusive bounds pass it).  Replaces ~20 elementwise / softmax passes
// over the [n, A] logits (forward and backward) with one read and one write.
//
// One wave per row (A <= 512: 8 columns per lane), rows grid-strided; the loss
// sums go to three double accumulators (one atomic per wave).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/bgx.h"

namespace {

constexpr float kMaskLog = -103.27892990343185f;   // log(1e-45) in fp32 (policy.py MASK_LOG)

template <typename T> __device__ __forceinline__ float ld(const T* p) { return (float)*p; }
template <typename T> __device__ __forceinline__ T cvt(float x) { return (T)x; }

__device__ __forceinline__ float wave_max(float v) {
    #pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
    #pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <typename T>
__global__ __launch_bounds__(256) void k_ppo_head(const T* __restrict__ logits, int64_t ld_logits,
                                                  const T* __restrict__ values, const uint8_t* __restrict__ records,
                                                  const int32_t* __restrict__ actions,
                                                  const float* __restrict__ old_logp,
                                                  const float* __restrict__ returns, const float* __restrict__ adv,
                                                  int n, int A, float eps_clip, float c_value, float c_entropy,
                                                  float gscale, T* __restrict__ dlogits, int64_t ld_dlogits,
                                                  T* __restrict__ dvalues, double* __restrict__ sums) {
    const int l = threadIdx.x & 63;
    const int nw = gridDim.x * (blockDim.x >> 6);
    double s_pol = 0.0, s_val = 0.0, s_ent = 0.0;
    for (int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); row < n; row += nw) {
        const T* lg = logits + (int64_t)row * ld_logits;
        const uint8_t* rec = records + (int64_t)row * 64;
        const int cnt = (int)rec[60] | ((int)rec[61] << 8);
        float z[8];
        #pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = l + 64 * k;
            z[k] = j < A ? ld(lg + j) + (j < cnt ? 0.0f : kMaskLog) : -INFINITY;
        }
        float m = z[0];
        #pragma unroll
        for (int k = 1; k < 8; ++k) m = fmaxf(m, z[k]);
        m = wave_max(m);
        float se = 0.0f;
        #pragma unroll
        for (int k = 0; k < 8; ++k) se += z[k] == -INFINITY ? 0.0f : expf(z[k] - m);
        const float lse = m + logf(wave_sum(se));
        float lp[8], p[8], ent = 0.0f;
        #pragma unroll
        for (int k = 0; k < 8; ++k) {
            lp[k] = z[k] - lse;
            p[k] = z[k] == -INFINITY ? 0.0f : expf(lp[k]);
            ent -= z[k] == -INFINITY ? 0.0f : p[k] * lp[k];
        }
        ent = wave_sum(ent);
        const int act = actions[row];
        const float nl = __shfl(lp[(act >> 6) & 7], act & 63);          // log pi(act)
        const float a = adv[row];
        const float r = expf(nl - old_logp[row]);
        const float s1 = r * a;
        const float rc = fminf(fmaxf(r, 1.0f - eps_clip), 1.0f + eps_clip);
        const float s2 = rc * a;
        const float pol = -fminf(s1, s2);
        // d(-min(s1, s2))/d logp: torch min() splits ties, clamp() passes inside [lo, hi]
        const float w1 = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const float w2 = (1.0f - w1) * ((r >= 1.0f - eps_clip && r <= 1.0f + eps_clip) ? 1.0f : 0.0f);
        const float g_lp = -a * r * (w1 + w2);
        const float v = ld(values + row), R = returns[row];
        const float dv = v - R;
        #pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = l + 64 * k;
            if (j < A) {
                const float g = g_lp * ((j == act ? 1.0f : 0.0f) - p[k]) + c_entropy * p[k] * (lp[k] + ent);
                dlogits[(int64_t)row * ld_dlogits + j] = cvt<T>(gscale * g);
            }
        }
        if (l == 0) {
            dvalues[row] = cvt<T>(gscale * c_value * 2.0f * dv);
            s_pol += pol;
            s_val += (double)dv * dv;
            s_ent += ent;
        }
    }
    if (l == 0) {
        atomicAdd(sums + 0, s_pol);
        atomicAdd(sums + 1, s_val);
        atomicAdd(sums + 2, s_ent);
    }
}

}  // namespace

extern int bgx_internal_fail(hipError_t e);

extern "C" int bgx_ppo_head(const void* logits, int32_t dtype, int64_t ld_logits, const void* values,
                            const uint8_t* records, const int32_t* actions, const float* old_logp,
                            const float* returns, const float* adv, int32_t n, int32_t n_actions, float eps_clip,
                            float c_value, float c_entropy, float grad_scale, void* dlogits, int64_t ld_dlogits,
                            void* dvalues, double* sums, void* stream) {
    if (n < 0 || n_actions <= 0 || n_actions > 512 || (dtype != 0 && dtype != 1)) return BGX_EINVAL;
    if (n > 0 && (!logits || !values || !records || !actions || !old_logp || !returns || !adv || !dlogits ||
                  !dvalues || !sums))
        return BGX_EINVAL;
    if (n == 0) return BGX_OK;
    const int blocks = (n + 3) / 4 < 16384 ? (n + 3) / 4 : 16384;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == 0)
        hipLaunchKernelGGL(k_ppo_head<float>, dim3(blocks), dim3(256), 0, s, (const float*)logits, ld_logits,
                           (const float*)values, records, actions, old_logp, returns, adv, n, n_actions, eps_clip,
                           c_value, c_entropy, grad_scale, (float*)dlogits, ld_dlogits, (float*)dvalues, sums);
    else
        hipLaunchKernelGGL(k_ppo_head<_Float16>, dim3(blocks), dim3(256), 0, s, (const _Float16*)logits, ld_logits,
                           (const _Float16*)values, records, actions, old_logp, returns, adv, n, n_actions,
                           eps_clip, c_value, c_entropy, grad_scale, (_Float16*)dlogits, ld_dlogits,
                           (_Float16*)dvalues, sums);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}
