// bg_ppo.hip — the PPO loss head of the update (ppo_agent.py:268-305) fused into
// one pass over the logits: masked log-softmax (mask = log(1e-45) for illegal
// actions, ppo_agent.py:166), the clipped surrogate, the value MSE and the
// entropy bonus, and their gradients with respect to the logits and the value,
// exactly as torch autograd forms them (min(): ties split the gradient in half;
// clamp(): inclusive bounds pass it).  Replaces ~20 elementwise / softmax passes
// over the [n, A] logits (forward and backward) with one read and one write.
//
// Two rows per wave (A <= 512: 16 consecutive columns per lane of a 32-lane half,
// four 8-byte fp16 / 16-byte fp32 accesses when the rows are aligned), rows
// grid-strided; the loss sums go to three double accumulators (one atomic each per
// workgroup).
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
constexpr float kL2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;


// Reductions over a 32-lane half-wave: DPP row_ror 8/4/2/1 inside each 16-lane row,
// then ds_swizzle xor 16 (32-lane bitmask mode) across the two rows; every lane of
// the half gets the result.
template <int CTRL>
__device__ __forceinline__ float dpp_ror(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float swz_x16(float v) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));   // and 0x1f, xor 0x10
}
#define BGX_HALF_REDUCE(OP, v)                \
    do {                                     \
        v = OP(v, dpp_ror<0x128>(v));        \
        v = OP(v, dpp_ror<0x124>(v));        \
        v = OP(v, dpp_ror<0x122>(v));        \
        v = OP(v, dpp_ror<0x121>(v));        \
        v = OP(v, swz_x16(v));               \
    } while (0)
__device__ __forceinline__ float fadd(float a, float b) { return a + b; }

// 16 consecutive columns per lane: 8-byte (fp16: 4 columns) / 16-byte (fp32: 4) accesses
template <typename T> struct Vec16;
template <> struct Vec16<_Float16> {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ void load(const _Float16* p, float* z) {
        h4 a[4];
        #pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = ((const h4*)p)[k];
        #pragma unroll
        for (int k = 0; k < 4; ++k)
            #pragma unroll
            for (int i = 0; i < 4; ++i) z[4 * k + i] = (float)a[k][i];
    }
    static __device__ __forceinline__ void store(_Float16* p, const float* g) {
        #pragma unroll
        for (int k = 0; k < 4; ++k) {
            h4 a;
            #pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = (_Float16)g[4 * k + i];
            ((h4*)p)[k] = a;
        }
    }
};
template <> struct Vec16<float> {
    static __device__ __forceinline__ void load(const float* p, float* z) {
        float4 a[4];
        #pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = ((const float4*)p)[k];
        #pragma unroll
        for (int k = 0; k < 4; ++k) { z[4 * k] = a[k].x; z[4 * k + 1] = a[k].y; z[4 * k + 2] = a[k].z; z[4 * k + 3] = a[k].w; }
    }
    static __device__ __forceinline__ void store(float* p, const float* g) {
        #pragma unroll
        for (int k = 0; k < 4; ++k) ((float4*)p)[k] = make_float4(g[4 * k], g[4 * k + 1], g[4 * k + 2], g[4 * k + 3]);
    }
};

// Two rows per wave, one per 32-lane half (lane l: row half l >> 5, columns
// 16 (l & 31) .. +15): the row reductions are DPP rotations + one swizzle (no
// LDS memory round trips), 16 columns per lane keep the registers at 4 waves
// per SIMD, and the chosen action's logit is read directly (its log-prob needs
// no per-column select).  Rows grid-strided over the halves.
template <typename T>
__global__ __launch_bounds__(256, 4) void k_ppo_head(const T* __restrict__ logits, int64_t ld_logits,
                                                  const T* __restrict__ values, const uint8_t* __restrict__ records,
                                                  const int32_t* __restrict__ actions,
                                                  const float* __restrict__ old_logp,
                                                  const float* __restrict__ returns, const float* __restrict__ adv,
                                                  int n, int A, float eps_clip, float c_value, float c_entropy,
                                                  float gscale, T* __restrict__ dlogits, int64_t ld_dlogits,
                                                  T* __restrict__ dvalues, double* __restrict__ sums, int vec,
                                                  int pad, float* __restrict__ colsum) {
    constexpr int C = 16;
    const int l = threadIdx.x & 63;
    const int c32 = l & 31;
    const int nh = gridDim.x * (blockDim.x >> 5);          // 32-lane halves in the grid
    const int j0 = C * c32;                                 // this lane's columns j0 .. j0+15
    const bool vload = vec && j0 + C <= ld_logits;
    const bool vstore = vec && j0 + C <= ld_dlogits && (pad || j0 + C <= A);
    // per-half loss partials in fp64: a call may give one half thousands of rows
    double s_pol = 0.0, s_val = 0.0, s_ent = 0.0;
    float cs[C];
    #pragma unroll
    for (int i = 0; i < C; ++i) cs[i] = 0.0f;
    for (int row = blockIdx.x * (blockDim.x >> 5) + (threadIdx.x >> 5); row < n; row += nh) {
        const T* lg = logits + (int64_t)row * ld_logits;
        const uint8_t* rec = records + (int64_t)row * 64;
        const int cnt = (int)rec[60] | ((int)rec[61] << 8);
        const int act = actions[row];
        const float a = adv[row], olp = old_logp[row], ret = returns[row];
        const float v = (float)values[row];
        const float za = (float)lg[act] + (act < cnt ? 0.0f : kMaskLog);
        // base-2 domain: z2 = (z + mask) log2(e) for the legal / masked columns,
        // -inf past A (those columns do not exist in the reference's softmax)
        float z[C];
        if (vload) {
            Vec16<T>::load(lg + j0, z);
        } else {
            #pragma unroll
            for (int i = 0; i < C; ++i) z[i] = j0 + i < A ? (float)lg[j0 + i] : 0.0f;
        }
        float m = -INFINITY;
        #pragma unroll
        for (int i = 0; i < C; ++i) {
            const int j = j0 + i;
            const float t = fmaf(z[i], kL2e, j < cnt ? 0.0f : kMaskLog * kL2e);
            z[i] = j < A ? t : -INFINITY;
            m = fmaxf(m, z[i]);
        }
        BGX_HALF_REDUCE(fmaxf, m);
        float se = 0.0f;
        #pragma unroll
        for (int i = 0; i < C; ++i) se += __builtin_amdgcn_exp2f(z[i] - m);     // exp2(-inf) = 0
        BGX_HALF_REDUCE(fadd, se);
        const float lse2 = m + __log2f(se), nlse = -lse2 * kLn2;
        // torch.distributions.Categorical(probs) semantics (ppo_agent.py:273-291):
        // log_prob and entropy use L = log(clamp(p, eps, 1 - eps)) (clamp_probs),
        // whose gradient is zero outside [eps, 1 - eps].  z[i] <- p, q[i] <- L + in
        float q[C], ent = 0.0f, entq = 0.0f;
        #pragma unroll
        for (int i = 0; i < C; ++i) {
            const float u = fmaf(z[i], kLn2, nlse);            // natural log-prob
            const float lp = fminf(fmaxf(u, kLogEps), kLog1mEps);
            const float pi = __builtin_amdgcn_exp2f(z[i] - lse2);
            z[i] = pi;
            q[i] = lp + (lp == u ? 1.0f : 0.0f);
            ent = fmaf(-pi, lp, ent);                           // p = 0 past A
            entq = fmaf(-pi, q[i], entq);
        }
        BGX_HALF_REDUCE(fadd, ent);
        BGX_HALF_REDUCE(fadd, entq);
        const float ua = za - lse2 * kLn2;
        const float la = fminf(fmaxf(ua, kLogEps), kLog1mEps);          // log pi(act), clamped
        const float ina = la == ua ? 1.0f : 0.0f;
        const float r = __expf(la - olp);
        const float s1 = r * a;
        const float rc = fminf(fmaxf(r, 1.0f - eps_clip), 1.0f + eps_clip);
        const float s2 = rc * a;
        const float pol = -fminf(s1, s2);
        // d(-min(s1, s2))/d logp: torch min() splits ties, clamp() passes inside [lo, hi]
        const float w1 = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const float w2 = (1.0f - w1) * ((r >= 1.0f - eps_clip && r <= 1.0f + eps_clip) ? 1.0f : 0.0f);
        const float g_lp = -a * r * (w1 + w2) * ina;
        // d/dz_k of  -min(.) - c_e * H  with H = -sum L_j p_j:
        //   g_lp (d_ka - p_k) + c_e p_k (L_k + in_k + H - sum_j p_j in_j)
        //   = p_k (K1 q_k + K2) + [k == a] gscale g_lp,  K1 = gscale c_e,
        //   K2 = K1 (H - sum p in) - gscale g_lp,  H - sum p in = -sum p q
        const float k1 = gscale * c_entropy, gla = gscale * g_lp, k2 = fmaf(k1, entq, -gla);
        const float dv = v - ret;
        const float gv = gscale * c_value * 2.0f * dv;
        // past A, p = 0 and g = 0: with `pad` the stored layout [logits | value | 0]
        // gets the value gradient in column A, written by the lane that owns that
        // column in the same store as its other columns (one writer per address)
        T* dl = dlogits + (int64_t)row * ld_dlogits;
        if (vstore) {
            #pragma unroll
            for (int k = 0; k < C / 4; ++k) {
                typedef T t4 __attribute__((ext_vector_type(4)));
                t4 w;
                #pragma unroll
                for (int i = 4 * k; i < 4 * k + 4; ++i) {
                    const float g = pad && j0 + i == A ? gv : fmaf(z[i], fmaf(k1, q[i], k2), j0 + i == act ? gla : 0.0f);
                    const T t = (T)g;
                    w[i - 4 * k] = t;
                    cs[i] += (float)t;
                }
                ((t4*)(dl + j0))[k] = w;
            }
        } else {
            #pragma unroll
            for (int i = 0; i < C; ++i) {
                const int j = j0 + i;
                if (j < A || (pad && j < ld_dlogits)) {
                    const float g = j == A ? gv : fmaf(z[i], fmaf(k1, q[i], k2), j == act ? gla : 0.0f);
                    const T t = (T)g;
                    dl[j] = t;
                    cs[i] += (float)t;
                }
            }
        }
        if (c32 == 0) {
            dvalues[row] = (T)gv;
            s_pol += (double)pol;
            s_val += (double)dv * (double)dv;
            s_ent += (double)ent;
        }
    }
    // one set of double atomics per workgroup (per-wave atomics on three addresses
    // serialised: measured 2.5 ms per 1M rows)
    __shared__ double red[8][3];
    const int half = threadIdx.x >> 5;
    if (c32 == 0) { red[half][0] = s_pol; red[half][1] = s_val; red[half][2] = s_ent; }
    __syncthreads();
    if (threadIdx.x < 3) {
        double t = 0.0;
        for (int i = 0; i < (int)(blockDim.x >> 5); ++i) t += red[i][threadIdx.x];
        atomicAdd(sums + threadIdx.x, t);
    }
    if (colsum) {                              // this workgroup's column sums -> colsum[block][512]
        __shared__ float cred[8][512];
        #pragma unroll
        for (int i = 0; i < C; ++i) cred[half][j0 + i] = cs[i];
        __syncthreads();
        for (int c = threadIdx.x; c < 512; c += blockDim.x) {
            float t = 0.0f;
            for (int i = 0; i < (int)(blockDim.x >> 5); ++i) t += cred[i][c];
            colsum[(int64_t)blockIdx.x * 512 + c] = t;
        }
    }
}

// ReLU backward of fc1 in place (torch.relu's gradient: passed where the output is
// > 0, policy_network.py:70) fused with the bias gradient's column sums: dh, h fp16
// [n][H] (H % 8 == 0, H <= 256), each thread 8 columns (one 16-byte access) of
// a row; per-block column sums of the masked dh -> colsum[block][H] (fp32).
__global__ __launch_bounds__(256) void k_relu_bwd(_Float16* __restrict__ dh, const _Float16* __restrict__ h, int n,
                                                  int H, float* __restrict__ colsum) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const int tpr = H / 8;                          // threads per row
    const int rows_per_it = blockDim.x / tpr;
    const int t = threadIdx.x;
    const int slot = t / tpr, c0 = 8 * (t - slot * tpr);
    float cs[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if (slot < rows_per_it) {
        for (int row = blockIdx.x * rows_per_it + slot; row < n; row += gridDim.x * rows_per_it) {
            h8* pd = (h8*)(dh + (int64_t)row * H + c0);
            h8 d = *pd;
            const h8 a = *(const h8*)(h + (int64_t)row * H + c0);
            #pragma unroll
            for (int i = 0; i < 8; ++i) {
                d[i] = a[i] > (_Float16)0.0f ? d[i] : (_Float16)0.0f;
                cs[i] += (float)d[i];
            }
            *pd = d;
        }
    }
    __shared__ float red[256][9];
    #pragma unroll
    for (int i = 0; i < 8; ++i) red[t][i] = cs[i];
    __syncthreads();
    for (int c = t; c < H; c += blockDim.x) {
        const int tc = c / 8, i = c - 8 * tc;
        float acc = 0.0f;
        for (int r = 0; r < rows_per_it; ++r) acc += red[r * tpr + tc][i];
        colsum[(int64_t)blockIdx.x * H + c] = acc;
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
    const int blocks = colsum ? kPpoColBlocks : ((n + 7) / 8 < 2048 ? (n + 7) / 8 : 2048);
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

extern "C" int bgx_relu_backward(void* dh, const void* h, int32_t n, int32_t hidden, float* colsum, int32_t blocks,
                                 void* stream) {
    if (n < 0 || hidden <= 0 || hidden % 8 || hidden > 256 || blocks <= 0 || !colsum ||
        (n > 0 && (!dh || !h)))
        return BGX_EINVAL;
    if (((uintptr_t)dh | (uintptr_t)h) % 16) return BGX_EINVAL;
    hipLaunchKernelGGL(k_relu_bwd, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (_Float16*)dh,
                       (const _Float16*)h, n, hidden, colsum);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}
