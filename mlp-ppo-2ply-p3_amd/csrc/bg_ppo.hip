// bg_ppo.hip — the PPO loss head of the update (ppo_agent.py:268-305) fused into
// one pass over the logits: masked log-softmax (mask = log(1e-45) for illegal
// actions, ppo_agent.py:166), the clipped surrogate, the value MSE and the
// entropy bonus, and their gradients with respect to the logits and the value,
// exactly as torch autograd forms them (min(): ties split the gradient in half;
// clamp(): inclusive bounds pass it).  Replaces ~20 elementwise / softmax passes
// over the [n, A] logits (forward and backward) with one read and one write.
//
// One wave per row (A <= 512: 8 consecutive columns per lane, two 8-byte fp16 /
// 16-byte fp32 accesses when the rows are aligned), rows grid-strided; the loss
// sums go to three double accumulators (one atomic each per workgroup).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/bgx.h"

namespace {

constexpr float kMaskLog = -103.27892990343185f;   // log(1e-45) in fp32 (policy.py MASK_LOG)
constexpr int kPpoColBlocks = BGX_PPO_COLSUM_BLOCKS;
// fp32 log(eps) and log(1 - eps), eps = FLT_EPSILON (torch clamp_probs bounds)
constexpr float kLogEps = -15.942384719848633f;
constexpr float kLog1mEps = -1.1920930376163597e-07f;


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

// 8 consecutive columns per lane as one 16-byte (fp16) / two 16-byte (fp32) access
template <typename T> struct Vec8;
template <> struct Vec8<_Float16> {          // two 8-byte halves (a 500-wide fp16 row is 8-byte aligned)
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    static constexpr int kAlign = 8;
    static __device__ __forceinline__ void load(const _Float16* p, float* z) {
        const h4 a = ((const h4*)p)[0], b = ((const h4*)p)[1];
        #pragma unroll
        for (int i = 0; i < 4; ++i) { z[i] = (float)a[i]; z[4 + i] = (float)b[i]; }
    }
    static __device__ __forceinline__ void store(_Float16* p, const float* g) {
        h4 a, b;
        #pragma unroll
        for (int i = 0; i < 4; ++i) { a[i] = (_Float16)g[i]; b[i] = (_Float16)g[4 + i]; }
        ((h4*)p)[0] = a;
        ((h4*)p)[1] = b;
    }
};
template <> struct Vec8<float> {
    static constexpr int kAlign = 16;
    static __device__ __forceinline__ void load(const float* p, float* z) {
        const float4 a = ((const float4*)p)[0], b = ((const float4*)p)[1];
        z[0] = a.x; z[1] = a.y; z[2] = a.z; z[3] = a.w; z[4] = b.x; z[5] = b.y; z[6] = b.z; z[7] = b.w;
    }
    static __device__ __forceinline__ void store(float* p, const float* g) {
        ((float4*)p)[0] = make_float4(g[0], g[1], g[2], g[3]);
        ((float4*)p)[1] = make_float4(g[4], g[5], g[6], g[7]);
    }
};

template <typename T>
__global__ __launch_bounds__(256) void k_ppo_head(const T* __restrict__ logits, int64_t ld_logits,
                                                  const T* __restrict__ values, const uint8_t* __restrict__ records,
                                                  const int32_t* __restrict__ actions,
                                                  const float* __restrict__ old_logp,
                                                  const float* __restrict__ returns, const float* __restrict__ adv,
                                                  int n, int A, float eps_clip, float c_value, float c_entropy,
                                                  float gscale, T* __restrict__ dlogits, int64_t ld_dlogits,
                                                  T* __restrict__ dvalues, double* __restrict__ sums, int vec,
                                                  int pad, float* __restrict__ colsum) {
    const int l = threadIdx.x & 63;
    const int nw = gridDim.x * (blockDim.x >> 6);
    const int j0 = 8 * l;                      // this lane's columns j0 .. j0+7
    double s_pol = 0.0, s_val = 0.0, s_ent = 0.0;
    float cs[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};   // column sums of the stored gradient
    for (int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); row < n; row += nw) {
        const T* lg = logits + (int64_t)row * ld_logits;
        const uint8_t* rec = records + (int64_t)row * 64;
        const int cnt = (int)rec[60] | ((int)rec[61] << 8);
        float z[8];
        if (vec && j0 + 8 <= A) {
            Vec8<T>::load(lg + j0, z);
        } else {
            #pragma unroll
            for (int i = 0; i < 8; ++i) z[i] = j0 + i < A ? (float)lg[j0 + i] : 0.0f;
        }
        float m = -INFINITY;
        #pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int j = j0 + i;
            z[i] = j < A ? z[i] + (j < cnt ? 0.0f : kMaskLog) : -INFINITY;
            m = fmaxf(m, z[i]);
        }
        m = wave_max(m);
        float e[8], se = 0.0f;
        #pragma unroll
        for (int i = 0; i < 8; ++i) { e[i] = z[i] == -INFINITY ? 0.0f : __expf(z[i] - m); se += e[i]; }
        se = wave_sum(se);
        const float lse = m + __logf(se), inv = 1.0f / se;
        // torch.distributions.Categorical(probs) semantics (ppo_agent.py:273-291):
        // log_prob and entropy use L = log(clamp(p, eps, 1 - eps)) (clamp_probs),
        // whose gradient is zero outside [eps, 1 - eps]
        float lp[8], inb[8], ent = 0.0f, s_in = 0.0f;
        #pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float u = z[i] - lse;
            inb[i] = (u >= kLogEps && u <= kLog1mEps) ? 1.0f : 0.0f;
            lp[i] = fminf(fmaxf(u, kLogEps), kLog1mEps);
            e[i] *= inv;                           // p
            ent -= z[i] == -INFINITY ? 0.0f : e[i] * lp[i];
            s_in += e[i] * inb[i];
        }
        ent = wave_sum(ent);
        s_in = wave_sum(s_in);
        const int act = actions[row];
        float la = 0.0f, ina = 0.0f;
        #pragma unroll
        for (int i = 0; i < 8; ++i) {
            la = (act & 7) == i ? lp[i] : la;
            ina = (act & 7) == i ? inb[i] : ina;
        }
        const float nl = __shfl(la, (act >> 3) & 63);          // log pi(act), clamped
        const float in_a = __shfl(ina, (act >> 3) & 63);
        const float a = adv[row];
        const float r = __expf(nl - old_logp[row]);
        const float s1 = r * a;
        const float rc = fminf(fmaxf(r, 1.0f - eps_clip), 1.0f + eps_clip);
        const float s2 = rc * a;
        const float pol = -fminf(s1, s2);
        // d(-min(s1, s2))/d logp: torch min() splits ties, clamp() passes inside [lo, hi]
        const float w1 = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const float w2 = (1.0f - w1) * ((r >= 1.0f - eps_clip && r <= 1.0f + eps_clip) ? 1.0f : 0.0f);
        const float g_lp = -a * r * (w1 + w2) * in_a;
        // d/dz_k of  -min(.) - c_e * H  with H = -sum L_j p_j:
        //   g_lp (d_ka - p_k) + c_e p_k (L_k + in_k + H - sum_j p_j in_j)
        const float ent_c = ent - s_in;
        float g[8];
        #pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float pi = e[i];
            g[i] = gscale * (g_lp * ((j0 + i == act ? 1.0f : 0.0f) - pi) + c_entropy * pi * (lp[i] + inb[i] + ent_c));
        }
        const float v = (float)values[row], dv = v - returns[row];
        const float gv = gscale * c_value * 2.0f * dv;
        T* dl = dlogits + (int64_t)row * ld_dlogits;
        if (vec && j0 + 8 <= A) {
            Vec8<T>::store(dl + j0, g);
            #pragma unroll
            for (int i = 0; i < 8; ++i) cs[i] += (float)(T)g[i];
        } else {
            // the row's tail; with `pad` also column A = the value gradient and
            // zeros up to ld_dlogits (the layout of a [logits | value | 0] GEMM)
            #pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int j = j0 + i;
                const T t = j < A ? (T)g[i] : (j == A ? (T)gv : (T)0.0f);
                if (j < A || (pad && j < ld_dlogits)) {
                    dl[j] = t;
                    cs[i] += (float)t;
                }
            }
        }
        if (l == 0) {
            dvalues[row] = (T)gv;
            s_pol += pol;
            s_val += (double)dv * dv;
            s_ent += ent;
        }
    }
    // one set of double atomics per workgroup (per-wave atomics on three addresses
    // serialised: measured 2.5 ms per 1M rows)
    __shared__ double red[4][3];
    const int w = threadIdx.x >> 6;
    if (l == 0) { red[w][0] = s_pol; red[w][1] = s_val; red[w][2] = s_ent; }
    __syncthreads();
    if (threadIdx.x < 3) {
        double t = 0.0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i][threadIdx.x];
        atomicAdd(sums + threadIdx.x, t);
    }
    if (colsum) {                              // this workgroup's column sums -> colsum[block][512]
        __shared__ float cred[4][512];
        #pragma unroll
        for (int i = 0; i < 8; ++i) cred[w][j0 + i] = cs[i];
        __syncthreads();
        for (int c = threadIdx.x; c < 512; c += blockDim.x) {
            float t = 0.0f;
            for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += cred[i][c];
            colsum[(int64_t)blockIdx.x * 512 + c] = t;
        }
    }
}

}  // namespace

extern int bgx_internal_fail(hipError_t e);

extern "C" int bgx_ppo_head_ex(const void* logits, int32_t dtype, int64_t ld_logits, const void* values,
                               const uint8_t* records, const int32_t* actions, const float* old_logp,
                               const float* returns, const float* adv, int32_t n, int32_t n_actions, float eps_clip,
                               float c_value, float c_entropy, float grad_scale, void* dlogits, int64_t ld_dlogits,
                               void* dvalues, double* sums, int32_t pad_value_col, float* colsum, void* stream) {
    if (n < 0 || n_actions <= 0 || n_actions > 512 || (dtype != 0 && dtype != 1)) return BGX_EINVAL;
    if (pad_value_col && (ld_dlogits <= n_actions || ld_dlogits > 512)) return BGX_EINVAL;
    if (n > 0 && (!logits || !values || !records || !actions || !old_logp || !returns || !adv || !dlogits ||
                  !dvalues || !sums))
        return BGX_EINVAL;
    if (n == 0 && !colsum) return BGX_OK;
    // with column sums the grid is fixed (colsum is [kPpoColBlocks][512], every block writes its row)
    const int blocks = colsum ? kPpoColBlocks : ((n + 3) / 4 < 2048 ? (n + 3) / 4 : 2048);
    hipStream_t s = (hipStream_t)stream;
    const int esz = dtype == 0 ? 4 : 2;
    const int al = dtype == 0 ? 16 : 8;
    const int vec = ((uintptr_t)logits % al == 0 && (uintptr_t)dlogits % al == 0 && (ld_logits * esz) % al == 0 &&
                     (ld_dlogits * esz) % al == 0) ? 1 : 0;
    const int pad = pad_value_col ? 1 : 0;
    if (dtype == 0)
        hipLaunchKernelGGL(k_ppo_head<float>, dim3(blocks), dim3(256), 0, s, (const float*)logits, ld_logits,
                           (const float*)values, records, actions, old_logp, returns, adv, n, n_actions, eps_clip,
                           c_value, c_entropy, grad_scale, (float*)dlogits, ld_dlogits, (float*)dvalues, sums, vec,
                           pad, colsum);
    else
        hipLaunchKernelGGL(k_ppo_head<_Float16>, dim3(blocks), dim3(256), 0, s, (const _Float16*)logits, ld_logits,
                           (const _Float16*)values, records, actions, old_logp, returns, adv, n, n_actions,
                           eps_clip, c_value, c_entropy, grad_scale, (_Float16*)dlogits, ld_dlogits,
                           (_Float16*)dvalues, sums, vec, pad, colsum);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}

extern "C" int bgx_ppo_head(const void* logits, int32_t dtype, int64_t ld_logits, const void* values,
                            const uint8_t* records, const int32_t* actions, const float* old_logp,
                            const float* returns, const float* adv, int32_t n, int32_t n_actions, float eps_clip,
                            float c_value, float c_entropy, float grad_scale, void* dlogits, int64_t ld_dlogits,
                            void* dvalues, double* sums, void* stream) {
    return bgx_ppo_head_ex(logits, dtype, ld_logits, values, records, actions, old_logp, returns, adv, n, n_actions,
                           eps_clip, c_value, c_entropy, grad_scale, dlogits, ld_dlogits, dvalues, sums, 0, nullptr,
                           stream);
}
