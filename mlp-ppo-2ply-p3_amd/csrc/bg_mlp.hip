// bg_mlp.hip — BackgammonPolicyNetwork (agent/policy_network.py:44-75) on MFMA,
// fused with the feature encoder and select_action's masked sampling
// (agent/ppo_agent.py:164-187).
//
// One wave = 32 game rows.  GEMM1 computes X1 = W1 . F^T (hidden x rows) with
// v_mfma_f32_32x32x2_f32, the B operand (features) generated on the fly from the
// rows' int8 lane records staged in LDS.  The accumulator layout of X1 (column =
// row on the lane, hidden units in registers) is used UNMOVED as the B operand of
// GEMM2 (Y = W2 . X1, W2 = [action_head; value_head]): the host packs W2's
// columns in the k order the accumulator registers deliver.  Each lane then
// owns 16 outputs of one row per 32-row output tile, so masked log-sum-exp and
// Gumbel-max sampling run in registers with one cross-half shuffle per row.
//
// f32-input MFMA is an exact f32 FMA chain (cdna_hip_programming.md §3), so the
// logits/values match torch fp32 to ~1e-6 (tests/test_gpu_policy.py).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/bgx.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kIn = 198;
constexpr int kK1 = kIn / 2;          // 99 k-steps of 32x32x2
constexpr float kMaskLog = -103.27892990343185f;  // log(fp32(1e-45)) (ppo_agent.py:166)

__constant__ float kOff15m[16] = {
    0.0f / 15.0f, 1.0f / 15.0f, 2.0f / 15.0f, 3.0f / 15.0f, 4.0f / 15.0f, 5.0f / 15.0f,
    6.0f / 15.0f, 7.0f / 15.0f, 8.0f / 15.0f, 9.0f / 15.0f, 10.0f / 15.0f, 11.0f / 15.0f,
    12.0f / 15.0f, 13.0f / 15.0f, 14.0f / 15.0f, 15.0f / 15.0f};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// feature k (0..197) of the row whose 64-byte record starts at rec (LDS)
__device__ __forceinline__ float feat(const uint8_t* rec, int k) {
    if (k >= 196) return (k == 196) == (rec[52] == 0) ? 1.0f : 0.0f;
    const int p = k >= 98 ? 1 : 0;
    const int g = k - 98 * p;
    if (g < 96) {
        const int n = rec[p * 24 + (g >> 2)];
        const int u = g & 3;
        if (u < 3) return n > u ? 1.0f : 0.0f;
        return n >= 3 ? (float)(n - 3) * 0.5f : 0.0f;
    }
    if (g == 96) return (float)rec[48 + p] * 0.5f;
    return kOff15m[rec[50 + p] & 15];
}

__device__ __forceinline__ uint32_t mulhi(uint32_t a, uint32_t b) { return __umulhi(a, b); }

// Philox4x32-10 -> 4 uniforms strictly inside (0,1)
__device__ __forceinline__ void philox4(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                        uint32_t k1, float u[4]) {
    #pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t h0 = mulhi(0xD2511F53u, c0), l0 = 0xD2511F53u * c0;
        const uint32_t h1 = mulhi(0xCD9E8D57u, c2), l1 = 0xCD9E8D57u * c2;
        c0 = h1 ^ c1 ^ k0; c1 = l1; c2 = h0 ^ c3 ^ k1; c3 = l0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    const uint32_t w[4] = {c0, c1, c2, c3};
    #pragma unroll
    // 23 bits + 1/2: exactly representable, u in [2^-24, 1 - 2^-24] (never 0 or 1)
    for (int i = 0; i < 4; ++i) u[i] = ((float)(w[i] >> 9) + 0.5f) * (1.0f / 8388608.0f);
}

// Packed weights (bgx_policy_pack):
//   w1p [99][T][64]       w1p[kk][t][l] = W1[32t + (l&31)][2kk + (l>>5)]
//   b1p [T][16][64]       b1p[t][r][l]  = b1[32t + hid(r, l>>5)]
//   w2p [OT][16T][64]     w2p[o][kk][l] = W2[32o + (l&31)][32(kk/16) + hid(kk%16, l>>5)]
//   b2p [OT][16][64]      b2p[o][r][l]  = b2[32o + hid(r, l>>5)]
// with hid(r, h) = (r&3) + 8(r>>2) + 4h (the 32x32 accumulator row map) and
// W2 = [action_head.weight; value_head.weight; 0], b2 likewise (OT*32 rows).
__device__ __forceinline__ int hid(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <int T>
__global__ __launch_bounds__(64) void k_policy_act(const uint8_t* __restrict__ recs, int n, const float* __restrict__ w1p,
                                                   const float* __restrict__ b1p, const float* __restrict__ w2p,
                                                   const float* __restrict__ b2p, int n_actions, int n_otiles,
                                                   uint32_t seed_lo, uint32_t seed_hi, uint32_t step, int greedy,
                                                   int32_t* act_out, float* logp_out, float* value_out,
                                                   float* logits_out) {
    __shared__ uint8_t srec[32 * 64];
    const int l = lane_id();
    const int row0 = blockIdx.x * 32;
    // stage 32 records (2 KiB): lane l copies 32 bytes
    {
        const int r = l >> 1, off = (l & 1) * 32;
        const int gr = row0 + r < n ? row0 + r : n - 1;
        const uint4* src = (const uint4*)(recs + (size_t)gr * 64 + off);
        uint4* dst = (uint4*)(srec + r * 64 + off);
        dst[0] = src[0];
        dst[1] = src[1];
    }
    __syncthreads();
    const int j = l & 31, h = l >> 5;
    const uint8_t* myrec = srec + j * 64;
    const int count = (int)myrec[60] | ((int)myrec[61] << 8);

    // ---- GEMM1: X1[t] = W1[32t..32t+31, :] . F^T  (+ b1, ReLU)
    f32x16 x1[T];
    #pragma unroll
    for (int t = 0; t < T; ++t)
        #pragma unroll
        for (int r = 0; r < 16; ++r) x1[t][r] = b1p[(t * 16 + r) * 64 + l];
    for (int kk = 0; kk < kK1; ++kk) {
        const float b = feat(myrec, 2 * kk + h);
        #pragma unroll
        for (int t = 0; t < T; ++t) {
            const float a = w1p[(kk * T + t) * 64 + l];
            x1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, x1[t], 0, 0, 0);
        }
    }
    #pragma unroll
    for (int t = 0; t < T; ++t)
        #pragma unroll
        for (int r = 0; r < 16; ++r) x1[t][r] = fmaxf(x1[t][r], 0.0f);

    // ---- GEMM2 per 32-output tile + online masked log-sum-exp + Gumbel-max
    float m = -INFINITY, s = 0.0f, best = -INFINITY, bestz = 0.0f, value = 0.0f;
    int besta = 0;
    const int grow = row0 + j;
    for (int o = 0; o < n_otiles; ++o) {
        f32x16 y;
        #pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = b2p[(o * 16 + r) * 64 + l];
        const float* wo = w2p + (size_t)o * (16 * T) * 64 + l;
        #pragma unroll
        for (int t = 0; t < T; ++t) {
            #pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float a = wo[(t * 16 + r) * 64];
                y = __builtin_amdgcn_mfma_f32_32x32x2f32(a, x1[t][r], y, 0, 0, 0);
            }
        }
        // lane l holds outputs a = 32o + hid(r, h), r = 0..15, of row j
        float u[16];
        if (!greedy) {
            #pragma unroll
            for (int g = 0; g < 4; ++g)
                philox4((uint32_t)grow, step, (uint32_t)(o * 8 + g * 2 + h), 0x504F4C59u, seed_lo, seed_hi, u + 4 * g);
        }
        #pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int a = 32 * o + hid(r, h);
            const float z0 = y[r];
            if (logits_out && grow < n && a <= n_actions) logits_out[(size_t)grow * (32 * n_otiles) + a] = z0;
            if (a == n_actions) value = z0;
            if (a < n_actions) {
                const float z = a < count ? z0 : z0 + kMaskLog;
                const float mn = fmaxf(m, z);
                s = s * __expf(m - mn) + __expf(z - mn);
                m = mn;
                // Gumbel(0,1) noise; accurate logf near u = 1
                const float key = greedy ? z : z - logf(-logf(u[r]));
                if (key > best) { best = key; besta = a; bestz = z; }
            }
        }
    }
    // combine the two lane halves of each row (lanes j and j+32)
    const float m2 = __shfl_xor(m, 32), s2 = __shfl_xor(s, 32);
    const float best2 = __shfl_xor(best, 32), bestz2 = __shfl_xor(bestz, 32);
    const int besta2 = __shfl_xor(besta, 32);
    const float value2 = __shfl_xor(value, 32);
    const float mm = fmaxf(m, m2);
    const float ss = s * __expf(m - mm) + s2 * __expf(m2 - mm);
    const bool take2 = best2 > best || (best2 == best && besta2 < besta);
    const int a_fin = take2 ? besta2 : besta;
    const float z_fin = take2 ? bestz2 : bestz;
    const float v_fin = h == 0 ? value + value2 : 0.0f;   // the value row sits in exactly one half
    if (h == 0 && grow < n) {
        act_out[grow] = a_fin;
        if (logp_out) logp_out[grow] = z_fin - (mm + __logf(ss));
        if (value_out) value_out[grow] = v_fin;
    }
}

// Pack torch-layout weights into the MFMA operand layouts above.
__global__ void k_policy_pack(const float* W1, const float* b1, const float* Wa, const float* ba, const float* wv,
                              const float* bv, int H, int A, int T, int OT, float* w1p, float* b1p, float* w2p,
                              float* b2p) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int n1 = kK1 * T * 64, nb1 = T * 16 * 64, n2 = OT * 16 * T * 64, nb2 = OT * 16 * 64;
    auto W2 = [&](int o, int k) -> float {
        if (k >= H) return 0.0f;
        if (o < A) return Wa[(size_t)o * H + k];
        if (o == A) return wv[k];
        return 0.0f;
    };
    auto B2 = [&](int o) -> float { return o < A ? ba[o] : (o == A ? bv[0] : 0.0f); };
    if (tid < n1) {
        const int l = tid % 64, t = (tid / 64) % T, kk = tid / (64 * T);
        const int hrow = 32 * t + (l & 31), k = 2 * kk + (l >> 5);
        w1p[tid] = hrow < H ? W1[(size_t)hrow * kIn + k] : 0.0f;
    } else if (tid < n1 + nb1) {
        const int i = tid - n1;
        const int l = i % 64, r = (i / 64) % 16, t = i / (64 * 16);
        const int hrow = 32 * t + hid(r, l >> 5);
        b1p[i] = hrow < H ? b1[hrow] : 0.0f;
    } else if (tid < n1 + nb1 + n2) {
        const int i = tid - n1 - nb1;
        const int l = i % 64, kk = (i / 64) % (16 * T), o = i / (64 * 16 * T);
        const int k = 32 * (kk / 16) + hid(kk % 16, l >> 5);
        w2p[i] = W2(32 * o + (l & 31), k);
    } else if (tid < n1 + nb1 + n2 + nb2) {
        const int i = tid - n1 - nb1 - n2;
        const int l = i % 64, r = (i / 64) % 16, o = i / (64 * 16);
        b2p[i] = B2(32 * o + hid(r, l >> 5));
    }
}

}  // namespace

extern "C" {

int bgx_policy_packed_size(int32_t hidden, int32_t n_actions) {
    if (hidden <= 0 || hidden > 128 || n_actions <= 0) return BGX_EINVAL;
    const int T = (hidden + 31) / 32, OT = (n_actions + 1 + 31) / 32;
    return kK1 * T * 64 + T * 16 * 64 + OT * 16 * T * 64 + OT * 16 * 64;
}

int bgx_policy_pack(const float* W1, const float* b1, const float* Wa, const float* ba, const float* wv, const float* bv,
                    int32_t hidden, int32_t n_actions, float* packed, void* stream) {
    const int total = bgx_policy_packed_size(hidden, n_actions);
    if (total < 0 || !W1 || !b1 || !Wa || !ba || !wv || !bv || !packed) return BGX_EINVAL;
    const int T = (hidden + 31) / 32, OT = (n_actions + 1 + 31) / 32;
    float* w1p = packed;
    float* b1p = w1p + kK1 * T * 64;
    float* w2p = b1p + T * 16 * 64;
    float* b2p = w2p + OT * 16 * T * 64;
    hipLaunchKernelGGL(k_policy_pack, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, W1, b1, Wa, ba, wv,
                       bv, hidden, n_actions, T, OT, w1p, b1p, w2p, b2p);
    return hipGetLastError() == hipSuccess ? BGX_OK : BGX_EDEVICE;
}

int bgx_policy_act(const uint8_t* records_dev, int32_t n, const float* packed, int32_t hidden, int32_t n_actions,
                   uint64_t seed, uint32_t step, int32_t greedy, int32_t* act_out, float* logp_out, float* value_out,
                   float* logits_out, void* stream) {
    if (bgx_policy_packed_size(hidden, n_actions) < 0 || n < 0 || (n > 0 && (!records_dev || !packed || !act_out)))
        return BGX_EINVAL;
    if (n == 0) return BGX_OK;
    const int T = (hidden + 31) / 32, OT = (n_actions + 1 + 31) / 32;
    const float* w1p = packed;
    const float* b1p = w1p + kK1 * T * 64;
    const float* w2p = b1p + T * 16 * 64;
    const float* b2p = w2p + OT * 16 * T * 64;
    const dim3 grid((n + 31) / 32), blk(64);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
    switch (T) {
        case 1: hipLaunchKernelGGL(k_policy_act<1>, grid, blk, 0, s, records_dev, n, w1p, b1p, w2p, b2p, n_actions, OT, lo, hi, step, greedy, act_out, logp_out, value_out, logits_out); break;
        case 2: hipLaunchKernelGGL(k_policy_act<2>, grid, blk, 0, s, records_dev, n, w1p, b1p, w2p, b2p, n_actions, OT, lo, hi, step, greedy, act_out, logp_out, value_out, logits_out); break;
        case 3: hipLaunchKernelGGL(k_policy_act<3>, grid, blk, 0, s, records_dev, n, w1p, b1p, w2p, b2p, n_actions, OT, lo, hi, step, greedy, act_out, logp_out, value_out, logits_out); break;
        default: hipLaunchKernelGGL(k_policy_act<4>, grid, blk, 0, s, records_dev, n, w1p, b1p, w2p, b2p, n_actions, OT, lo, hi, step, greedy, act_out, logp_out, value_out, logits_out); break;
    }
    return hipGetLastError() == hipSuccess ? BGX_OK : BGX_EDEVICE;
}

}  // extern "C"
