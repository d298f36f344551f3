// bg_ppo_fused.hip — the fp16 (autocast) PPO epoch's output layer and loss head
// (ppo_agent.py:268-305 under autocast, policy_network.py:71-75) without the
// [n, 512] logits or their gradient ever reaching HBM.
//
// The round-2 epoch ran, per 2^20-row chunk, a hipBLASLt GEMM writing the fp16
// logits y = h W2h^T + b2h ([action_head; value_head; 0], 512 columns), the loss
// head reading them and writing dy (2 GiB of HBM traffic), dh = dy W2h, the ReLU
// backward and gW2 = dy^T h.  Here:
//
//  * k_ppo_rows — one wave per 32 rows, W2h (128 KiB) in LDS for the workgroup's
//    life.  Z^T = W2h h^T on v_mfma_f32_32x32x16_f16 (lane = row, 16 logits per
//    lane and 32-action tile), rounded to fp16 and kept packed in registers; the
//    masked log-softmax, the clipped surrogate, the value error and the entropy
//    run in registers (one cross-half shuffle per row reduction); the gradient
//    dz = dL/dy (fp16, exactly as the loss-head kernel bgx_ppo_head_ex forms it)
//    is consumed UNMOVED as the B operand of dh^T = W2h^T dz^T (W2h^T read from
//    the same LDS image with ds_read_b64_tr_b16), the ReLU mask applied, and dh
//    stored.  Per row it writes 20 bytes of statistics for the second kernel.
//  * k_ppo_gw2 — gW2 = dz^T h needs dz with the ROW on the reduction axis, i.e.
//    the other orientation: Z = h W2h^T for one 32-action tile per wave (lane =
//    action), dz recomputed from the row statistics (bit-identical formulas),
//    and dz^T h accumulated over the wave's rows (h^T from a per-wave LDS tile
//    via ds_read_b64_tr_b16); the bias gradient gb2 is the row sum of dz in the
//    lane.  Per-task partials are summed by k_ppo_gw2_sum1/2 (fixed order).
//
// Sparsity (exact): a row with cnt >= 1 legal actions has masked logits at
// z + log(1e-45) (ppo_agent.py:166), i.e. probabilities below 1e-44 relative:
// their fp16 gradients are exactly 0 (fp16's smallest subnormal is 6e-8) and their
// entropy / log-sum-exp terms lie 40 orders of magnitude below fp32 resolution.
// So a row needs only the action tiles holding its legal columns, plus the tile
// holding the value column; a row with no legal action (all 500 masked by the same
// constant: softmax is shift-invariant) needs all 16.  Rows are sorted by that
// tile count (host side, once per update), so a wave's 32 rows need the same tiles
// and k_ppo_gw2 visits, for action tile a, only the rows that reach it.  Mean
// legal count in self-play is ~19, so most rows need 2 of the 16 tiles.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/bgx.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((__vector_size__(4 * sizeof(short))));

constexpr int kA = 500;                 // action_size (agent/config.py; max_legal_moves)
constexpr int kAp = 512;                // [action_head; value_head; zero rows]
constexpr int kH = 128;                 // hidden_size (agent/config.py:8)
constexpr int kNT = kAp / 32;           // 16 action tiles
constexpr int kVT = kA / 32;            // 15: the tile holding the value column kA
constexpr int kVr = kA - 32 * kVT;      // its row in the tile (20)
constexpr int kVi = (kVr & 3) + 4 * (kVr >> 3);   // accumulator register holding it (8)
constexpr int kVh = (kVr >> 2) & 1;               // on lane half kVh (1)
constexpr int kTS = BGX_PPO_GW2_TASK_TILES;       // row tiles per k_ppo_gw2 task
constexpr int kPart = 32 * kH + 32;               // floats per task partial (gW2 tile + gb2 tile)

constexpr float kL2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
// fp32 log(eps) and log(1 - eps), eps = FLT_EPSILON (torch clamp_probs bounds)
constexpr float kLogEps = -15.942384719848633f;
constexpr float kLog1mEps = -1.1920930376163597e-07f;

__device__ __forceinline__ f16x8 as_h8(uint4 v) { return __builtin_bit_cast(f16x8, v); }

// byte offset of 16-byte chunk ch (0..15) of row `row` in an LDS image of 256-byte
// rows, XOR-swizzled so that both the row reads (ds_read_b128) and the transposed
// reads (ds_read_b64_tr_b16) of the 32x32x16 operands are bank-conflict free
// (cdna_hip_programming.md T10, layout (b))
__device__ __forceinline__ uint32_t swz(int row, int ch) {
    return 256u * (uint32_t)row + 16u * (uint32_t)(ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ s16x4 tr16(const uint8_t* lds) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) void*)lds);
}

// The 32x32x16 operand whose lane is column n = l & 31 of a [k][n] tile held
// row-major in a swizzled LDS image of 256-byte rows: element j of lane half hh is
// row 16s + 8(j >> 2) + 4hh + (j & 3) -- the k order in which an accumulator's
// registers 8s..8s+7 deliver their rows -- at column 32u + n.  Two transposed reads
// (rows +0..3 and +8..11 of the half's block).  Image rows start at `row0`.
// `l` is the lane id, passed laundered by callers inside unrolled loops so that LLVM
// recomputes these few address instructions per use instead of hoisting every
// (tile, s, u) combination into registers of its own.
__device__ __forceinline__ int laundered_lane() {
    int l = (int)(threadIdx.x & 63);
    __asm__ volatile("" : "+v"(l));
    return l;
}
__device__ __forceinline__ f16x8 tr_operand(const uint8_t* img, int row0, int s, int u, int l) {
    const int g = l >> 4, q = (l & 15) >> 2, p = l & 3;
    const int r = row0 + 16 * s + 4 * (g >> 1) + q;
    const int ch = 4 * u + 2 * (g & 1) + (p >> 1);
    // whole-register casts: element-wise short -> _Float16 inserts were lowered to
    // v_perm sequences that dropped the upper dword of each read
    const uint2 a = __builtin_bit_cast(uint2, tr16(img + swz(r, ch) + 8 * (p & 1)));
    const uint2 b = __builtin_bit_cast(uint2, tr16(img + swz(r + 8, ch) + 8 * (p & 1)));
    return __builtin_bit_cast(f16x8, make_uint4(a.x, a.y, b.x, b.y));
}

__device__ __forceinline__ float hsum(float v) { return v + __shfl_xor(v, 32); }

// the loss head's per-element quantities (bgx_ppo_head_ex's formulas): tz = the
// logit in log2 units or -inf when out of play; u = natural log-prob; lp = its
// clamp to [log eps, log(1 - eps)] (torch clamp_probs); p; q = lp + [not clamped]
struct Elem {
    float u, lp, p, q;
};
__device__ __forceinline__ Elem elem(float tz, float lse2, float nlse) {
    Elem e;
    e.u = fmaf(tz, kLn2, nlse);
    e.lp = fminf(fmaxf(e.u, kLogEps), kLog1mEps);
    e.p = __builtin_amdgcn_exp2f(tz - lse2);
    e.q = e.lp + (e.lp == e.u ? 1.0f : 0.0f);
    return e;
}

struct RowsArgs {
    const _Float16* h;          // [m][128] fc1 output (fp16, after ReLU), original row order
    const int32_t* perm;        // sorted position -> original row
    const uint8_t* recs;        // [m][64] lane records (legal count at bytes 60-61)
    const int32_t* act;
    const float* old_logp;
    const float* ret;
    const float* adv;
    const _Float16* w2h;        // [512][128] fp16 [action_head; value_head; 0]
    const _Float16* b2h;        // [512]
    int m;
    float eps_clip, c_value, c_entropy, gscale;
    _Float16* dh;               // [m][128] dL/dh after the ReLU mask, original row order
    float4* stats;              // [m] sorted order: lse2, k2, gla, gv
    int32_t* info;              // [m] sorted order: act | lim << 16
    double* sums;               // policy loss, value error^2, entropy sums
    _Float16* dy;               // optional [m][512] dL/dy (tests), original row order
    _Float16* z;                // optional [m][512] fp16 logits of the tiles computed (tests), original row order
};

// One variant per bound TM on the leading action tiles a row tile needs (TM = 1, 2, 4,
// 16): the used W2h tiles sit in LDS (tile t < TM at image tile t, the value tile at
// image tile TM), the packed logits take 8 registers per used tile, and the small
// variants keep 4 waves per workgroup with the next row tile's inputs loaded behind the
// current one's work.  Each variant walks the row tiles [range[0], range[1]) of the
// sorted order.
template <int TM>
struct RowsCfg {
    static constexpr int kImg = TM < kNT ? TM + 1 : kNT;        // W2h tiles in LDS
    static constexpr int kWaves = TM < kNT ? 4 : 8;              // waves per workgroup
    static constexpr bool kPrefetch = false;
};

struct RowIn {
    int row, cnt, act;
    float adv, olp, ret;
    uint4 hf[8];                                                 // B operand: h[row][16s + 8hh + j]
};

__device__ __forceinline__ void load_row(const RowsArgs& a, int tile, RowIn& in) {
    const int l = threadIdx.x & 63;
    const int pos = tile * 32 + (l & 31);
    const int p = pos < a.m ? pos : a.m - 1;
    in.row = a.perm ? a.perm[p] : p;
    const uint8_t* rec = a.recs + (size_t)in.row * 64;
    in.cnt = (int)rec[60] | ((int)rec[61] << 8);
    in.act = a.act[in.row];
    in.adv = a.adv[in.row];
    in.olp = a.old_logp[in.row];
    in.ret = a.ret[in.row];
    const uint4* hp = (const uint4*)(a.h + (size_t)in.row * kH);
    #pragma unroll
    for (int s = 0; s < 8; ++s) in.hf[s] = hp[2 * s + (l >> 5)];
}

template <int TM>
__global__ __launch_bounds__(TM < kNT ? 256 : 512) __attribute__((amdgpu_waves_per_eu(TM == 1 ? 2 : (TM == 2 ? 2 : 2))))
void k_ppo_rows(RowsArgs a, const int32_t* __restrict__ range) {
    using C = RowsCfg<TM>;
    constexpr int kW = C::kWaves;
    __shared__ __attribute__((aligned(16))) uint8_t sw[C::kImg * 32 * 256];
    __shared__ __attribute__((aligned(16))) float sb[C::kImg * 32];
    __shared__ double red[kW][3];
    const int lo = range[0], hi = range[1];
    if (lo + (int)blockIdx.x * kW >= hi) return;                  // whole workgroups only
    for (int i = threadIdx.x; i < C::kImg * 32 * 16; i += blockDim.x) {
        const int irow = i >> 4, it = irow >> 5;
        const int srow = 32 * (it < TM ? it : kVT) + (irow & 31);
        *(uint4*)(sw + swz(irow, i & 15)) = ((const uint4*)a.w2h)[srow * 16 + (i & 15)];
    }
    for (int i = threadIdx.x; i < C::kImg * 32; i += blockDim.x)
        sb[i] = (float)a.b2h[32 * ((i >> 5) < TM ? (i >> 5) : kVT) + (i & 31)];
    __syncthreads();

    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r = l & 31, hh = l >> 5;
    const float k1 = a.gscale * a.c_entropy;
    float s_pol = 0.0f, s_val = 0.0f, s_ent = 0.0f;
    const int stride = gridDim.x * kW;
    int tile = lo + blockIdx.x * kW + wv;
    RowIn cur;
    if (C::kPrefetch && tile < hi) load_row(a, tile, cur);
    for (; tile < hi; tile += stride) {
        RowIn nxt;
        if (C::kPrefetch) {
            if (tile + stride < hi) load_row(a, tile + stride, nxt);
        } else {
            load_row(a, tile, cur);
        }
        const int pos = tile * 32 + r;
        const bool valid = pos < a.m;
        const int row = cur.row, act = cur.act;
        const int lim = cur.cnt == 0 ? kA : (cur.cnt < kA ? cur.cnt : kA);   // columns [0, lim) in play
        // leading action tiles this row needs; T = the wave's largest (1..16), by a binary
        // search over ballots (no lane shuffles to keep addresses for)
        const int tr = (lim + 31) >> 5;
        int T = 0;
        #pragma unroll
        for (int b = 16; b >= 1; b >>= 1) T += __ballot(tr >= T + b) ? b : 0;

        uint32_t hm[4];                                           // bit k: h[row][32u + k] > 0
        #pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint32_t own = 0;
            #pragma unroll
            for (int half = 0; half < 2; ++half) {
                const uint4 w = cur.hf[2 * u + half];
                const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
                #pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const short b = (short)(ws[j >> 1] >> (16 * (j & 1)));
                    own |= (b > 0 ? 1u : 0u) << (16 * half + 8 * hh + j);
                }
            }
            hm[u] = own | (uint32_t)__shfl_xor((int)own, 32);
        }

        // Z^T tiles (lane = row; register i = action 32t + (i&3) + 8(i>>2) + 4hh); image
        // tile k holds action tile t = k < TM ? k : kVT.  The logits are fp16 (autocast's
        // GEMM output).  Small variants keep tz = z log2(e) (or -inf out of play) in fp32
        // registers; the 16-tile one keeps the packed fp16 logits and re-derives tz per pass.
        constexpr bool kKeep = TM < kNT;
        f16x2 Z[kKeep ? 1 : C::kImg][8];
        float TZ[kKeep ? C::kImg : 1][16];
        float v_own = 0.0f;
#define BGX_TILE_ON(k) (((k) < TM && (k) != kVT) ? (k) < T : true)
#define BGX_TILE_T(k) ((k) < TM ? (k) : kVT)
        constexpr int kVk = C::kImg - 1;                          // image tile of the value column
        #pragma unroll
        for (int k = 0; k < C::kImg; ++k) {
            if (BGX_TILE_ON(k)) {
                f32x16 acc;
                #pragma unroll
                for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
                const int ll = laundered_lane();
                #pragma unroll
                for (int s = 0; s < 8; ++s)
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                        as_h8(*(const uint4*)(sw + swz(32 * k + (ll & 31), 2 * s + (ll >> 5)))), as_h8(cur.hf[s]), acc,
                        0, 0, 0);
                const int lt = lim - 32 * BGX_TILE_T(k) - 4 * hh;
                #pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 bb = *(const float4*)(sb + 32 * k + 8 * q + 4 * hh);
                    const float bq[4] = {bb.x, bb.y, bb.z, bb.w};
                    #pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int i = 4 * q + e;
                        const _Float16 zh = (_Float16)(acc[i] + bq[e]);
                        if (k == kVk && i == kVi) v_own = (float)zh;
                        if (a.z && valid)
                            a.z[(size_t)row * kAp + 32 * BGX_TILE_T(k) + (i & 3) + 8 * (i >> 2) + 4 * hh] = zh;
                        if (kKeep) {
                            const int ko = (i & 3) + 8 * (i >> 2);
                            TZ[kKeep ? k : 0][i] = ko < lt ? (float)zh * kL2e : -INFINITY;
                        } else {
                            Z[kKeep ? 0 : k][i >> 1][i & 1] = zh;
                        }
                    }
                }
                __asm__ volatile("" ::: "memory");       // one tile's LDS reads in flight at a time
            }
        }
        const float v = __shfl(v_own, r + 32 * kVh);

// Each pass of the 16-tile variant re-reads the packed fp16 logits: laundering them
// first keeps LLVM from keeping the fp32 conversions alive across passes.
#define BGX_LAUNDER_Z()                                                           \
        _Pragma("unroll") for (int k = 0; k < C::kImg; ++k) {                     \
            if (!kKeep && BGX_TILE_ON(k)) {                                       \
                _Pragma("unroll") for (int q = 0; q < 8; ++q) {                   \
                    uint32_t w_ = __builtin_bit_cast(uint32_t, Z[kKeep ? 0 : k][q]); \
                    __asm__ volatile("" : "+v"(w_));                              \
                    Z[kKeep ? 0 : k][q] = __builtin_bit_cast(f16x2, w_);          \
                }                                                                 \
            }                                                                     \
        }
// The small variants' rows have lim <= 32 TM <= 128, so the value tile's action columns
// (480-499) are never in play: tz = -inf there, p = 0, and every pass below would add exact
// zeros (round 6: the passes skip it; its dz is gv at the value column, zero elsewhere).
#define BGX_TILE_SM(k) (BGX_TILE_ON(k) && !(kKeep && (k) == kVk))
#define BGX_FOR_ELEM(BODY)                                                        \
        BGX_LAUNDER_Z()                                                           \
        _Pragma("unroll") for (int k = 0; k < C::kImg; ++k) {                     \
            if (BGX_TILE_SM(k)) {                                                 \
                const int lt = lim - 32 * BGX_TILE_T(k) - 4 * hh;                 \
                const int at = act - 32 * BGX_TILE_T(k) - 4 * hh;                 \
                (void)at;                                                         \
                _Pragma("unroll") for (int i = 0; i < 16; ++i) {                  \
                    const int ko = (i & 3) + 8 * (i >> 2);                        \
                    const float tz = kKeep ? TZ[kKeep ? k : 0][i]                 \
                        : (ko < lt ? (float)Z[kKeep ? 0 : k][i >> 1][i & 1] * kL2e : -INFINITY); \
                    BODY                                                          \
                }                                                                 \
            }                                                                     \
        }

        float mx = -INFINITY;
        BGX_FOR_ELEM(mx = fmaxf(mx, tz);)
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        float se = 0.0f;
        BGX_FOR_ELEM(se += __builtin_amdgcn_exp2f(tz - mx);)
        se = hsum(se);
        const float lse2 = mx + __log2f(se), nlse = -lse2 * kLn2;
        float ent = 0.0f, entq = 0.0f, ua = -INFINITY;
        BGX_FOR_ELEM(const Elem e = elem(tz, lse2, nlse); ent = fmaf(-e.p, e.lp, ent); entq = fmaf(-e.p, e.q, entq);
                     ua = ko == at ? e.u : ua;)
        ent = hsum(ent);
        entq = hsum(entq);
        ua = fmaxf(ua, __shfl_xor(ua, 32));                           // -inf: act out of play
        // per row (bgx_ppo_head_ex): ratio, clipped surrogate and their gradient
        const float adv = cur.adv, olp = cur.olp, ret = cur.ret;
        const float la = fminf(fmaxf(ua, kLogEps), kLog1mEps);
        const float ina = la == ua ? 1.0f : 0.0f;
        const float rt = __expf(la - olp);
        const float s1 = rt * adv;
        const float rc = fminf(fmaxf(rt, 1.0f - a.eps_clip), 1.0f + a.eps_clip);
        const float s2 = rc * adv;
        const float pol = -fminf(s1, s2);
        const float w1 = s1 < s2 ? 1.0f : (s1 == s2 ? 0.5f : 0.0f);
        const float w2 = (1.0f - w1) * ((rt >= 1.0f - a.eps_clip && rt <= 1.0f + a.eps_clip) ? 1.0f : 0.0f);
        const float g_lp = -adv * rt * (w1 + w2) * ina;
        const float gla = a.gscale * g_lp, k2 = fmaf(k1, entq, -gla);
        const float dv = v - ret;
        const float gv = a.gscale * a.c_value * 2.0f * dv;
        if (valid && hh == 0) {
            s_pol += pol;
            s_val += dv * dv;
            s_ent += ent;
            a.stats[pos] = make_float4(lse2, k2, gla, gv);
            a.info[pos] = (act & 0xFFFF) | (lim << 16);
        }

        // dz (fp16, [dlogits | dvalue | 0]); the 16-tile variant writes it over its logits
        f16x2 Dz[kKeep ? C::kImg : 1][8];
#define BGX_DZ(k) (kKeep ? Dz[kKeep ? (k) : 0] : Z[kKeep ? 0 : (k)])
        BGX_LAUNDER_Z()
        #pragma unroll
        for (int k = 0; k < C::kImg; ++k) {
            if (BGX_TILE_ON(k)) {
                const int t = BGX_TILE_T(k);
                const int lt = lim - 32 * t - 4 * hh;
                const int at = act - 32 * t - 4 * hh;
                #pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    float d2[2];
                    #pragma unroll
                    for (int e2 = 0; e2 < 2; ++e2) {
                        const int ii = i + e2;
                        const int ko = (ii & 3) + 8 * (ii >> 2);
                        float d;
                        if (kKeep && k == kVk) {      // out of play: p = 0 (an out-of-play act keeps gla = 0)
                            d = ko == at ? gla : 0.0f;
                        } else {
                            const float tz = kKeep ? TZ[kKeep ? k : 0][ii]
                                : (ko < lt ? (float)Z[kKeep ? 0 : k][ii >> 1][ii & 1] * kL2e : -INFINITY);
                            const Elem e = elem(tz, lse2, nlse);
                            d = fmaf(e.p, fmaf(k1, e.q, k2), ko == at ? gla : 0.0f);
                        }
                        if (k == kVk && ii == kVi) d = hh == kVh ? gv : d;
                        d2[e2] = d;
                    }
                    BGX_DZ(k)[i >> 1] = f16x2{(_Float16)d2[0], (_Float16)d2[1]};
                }
                if (a.dy && valid) {
                    _Float16* dyr = a.dy + (size_t)row * kAp + 32 * t + 4 * hh;
                    #pragma unroll
                    for (int q = 0; q < 4; ++q)
                        *(uint2*)(dyr + 8 * q) = make_uint2(__builtin_bit_cast(uint32_t, BGX_DZ(k)[2 * q]),
                                                            __builtin_bit_cast(uint32_t, BGX_DZ(k)[2 * q + 1]));
                }
            }
        }
        if (a.dy && valid) {                         // the action tiles skipped hold zeros
            const int t0 = T < TM ? T : TM;
            _Float16* dyr = a.dy + (size_t)row * kAp;
            for (int c = 32 * t0 + 8 * hh; c < 32 * kVT; c += 16) *(uint4*)(dyr + c) = make_uint4(0, 0, 0, 0);
        }
        // dh^T = W2h^T dz^T per 32-unit hidden tile u: dz consumed unmoved as the B
        // operand (registers 8s..8s+7 of a tile = its k-step s), W2h^T from the LDS
        // image by transposed reads; then fp16 rounding and ReLU's mask (h > 0).
        // Register i = hidden 32u + (i&3) + 8(i>>2) + 4hh: 4 units per 8-byte store.
        #pragma unroll
        for (int u = 0; u < 4; ++u) {
            f32x16 dacc;
            #pragma unroll
            for (int i = 0; i < 16; ++i) dacc[i] = 0.0f;
            #pragma unroll
            for (int k = 0; k < C::kImg; ++k) {
                if (BGX_TILE_ON(k)) {
                    const int ll = laundered_lane();
                    #pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const f16x8 bfr = __builtin_bit_cast(
                            f16x8, make_uint4(__builtin_bit_cast(uint32_t, BGX_DZ(k)[4 * s]),
                                              __builtin_bit_cast(uint32_t, BGX_DZ(k)[4 * s + 1]),
                                              __builtin_bit_cast(uint32_t, BGX_DZ(k)[4 * s + 2]),
                                              __builtin_bit_cast(uint32_t, BGX_DZ(k)[4 * s + 3])));
                        dacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(tr_operand(sw, 32 * k, s, u, ll), bfr, dacc,
                                                                      0, 0, 0);
                    }
                    __asm__ volatile("" ::: "memory");
                }
            }
            {
                // units 32u + 8q + 4hh + 0..3 on lane half hh: one v_permlane32_swap per dword
                // pairs the halves, so that lane hh stores the 16 contiguous bytes of units
                // 32u + 8(2p + hh) + 0..7 (half the store instructions of 8-byte stores)
                _Float16* dhr = a.dh + (size_t)row * kH + 32 * u;
                #pragma unroll
                for (int p = 0; p < 2; ++p) {
                    f16x4 o[2];
                    #pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const int q = 2 * p + c;
                        #pragma unroll
                        for (int e = 0; e < 4; ++e)
                            o[c][e] = (hm[u] >> (8 * q + 4 * hh + e)) & 1u ? (_Float16)dacc[4 * q + e] : (_Float16)0.0f;
                    }
                    const uint2 x = __builtin_bit_cast(uint2, o[0]), y = __builtin_bit_cast(uint2, o[1]);
                    const auto s0 = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
                    const auto s1 = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
                    if (valid) *(uint4*)(dhr + 8 * (2 * p + hh)) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
                }
            }
        }
        if (C::kPrefetch) cur = nxt;
    }
#undef BGX_FOR_ELEM
#undef BGX_LAUNDER_Z
#undef BGX_TILE_SM
#undef BGX_TILE_ON
#undef BGX_TILE_T
#undef BGX_DZ
    // each lane of half 0 holds the fp32 sums of its own rows (a few dozen per lane);
    // the wave and the workgroup add them in fp64
    double dp = (double)s_pol, dvv = (double)s_val, de = (double)s_ent;
    #pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        dp += __shfl_xor(dp, o);
        dvv += __shfl_xor(dvv, o);
        de += __shfl_xor(de, o);
    }
    if (l == 0) { red[wv][0] = dp; red[wv][1] = dvv; red[wv][2] = de; }
    __syncthreads();
    if (threadIdx.x < 3) {
        double t = 0.0;
        for (int i = 0; i < kW; ++i) t += red[i][threadIdx.x];
        atomicAdd(a.sums + threadIdx.x, t);
    }
}

struct Gw2Args {
    const _Float16* h;
    const int32_t* perm;
    const float4* stats;
    const int32_t* info;
    const _Float16* w2h;
    const _Float16* b2h;
    int m;
    float k1;
    const int32_t* plan;        // [0..16] task prefix per action tile, [17..32] first row tile per action tile
    float* part;                // [task][kPart]
};

__global__ __launch_bounds__(256) void k_ppo_gw2(Gw2Args a) {
    __shared__ __attribute__((aligned(16))) uint8_t sh[4][32 * 256];       // per-wave h tile, 8 KiB
    __shared__ __attribute__((aligned(16))) float4 sst[4][32];
    __shared__ int32_t sinf[4][32];
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r = l & 31, hh = l >> 5;
    const int t = blockIdx.x * 4 + wv;                                      // launch order
    if (t >= a.plan[kNT]) return;                                           // whole waves only
    // Launch order = row group major: the tasks of one group of kTS row tiles (one per
    // action tile its rows reach) are consecutive, so the waves reading the same h rows
    // run together on one CU and all but the first read them from the L2 (action-tile
    // major, each h row came from HBM once per action tile: ~2.5x).  Group g reaches
    // action tile o iff f_o = start(o) / kTS <= g; P(g) = tasks of the groups before g
    // = sum_o max(0, g - f_o).  A task's partial keeps its action-tile-major slot
    // plan[o] + (g - f_o), so the fixed-order sums see the same layout.
    const int ntiles = (a.m + 31) >> 5;
    const int ngroups = (ntiles + kTS - 1) / kTS;
    int f[kNT];
    #pragma unroll
    for (int o = 0; o < kNT; ++o) f[o] = a.plan[17 + o] / kTS;
    auto prefix = [&](int g) {
        int p = 0;
        #pragma unroll
        for (int o = 0; o < kNT; ++o) p += max(0, g - f[o]);
        return p;
    };
    int lo = 0, hi = ngroups;                                               // largest g with P(g) <= t
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (prefix(mid) <= t) lo = mid; else hi = mid;
    }
    const int g = lo;
    int j = t - prefix(g), at = 0;
    #pragma unroll
    for (int o = kNT - 1; o >= 0; --o) {                                     // the j-th o with f_o <= g
        if (f[o] <= g) {
            int before = 0;
            #pragma unroll
            for (int q = 0; q < kNT; ++q) before += (q < o && f[q] <= g) ? 1 : 0;
            if (before == j) at = o;
        }
    }
    const int task = a.plan[at] + (g - f[at]);                              // the partial's slot
    const int tile0 = max(g * kTS, a.plan[17 + at]);
    const int tile1 = min((g + 1) * kTS, ntiles);
    uint4 bw[8];                                                            // B operand: W2h[32at + r][16s + 8hh + j]
    const uint4* wp = (const uint4*)(a.w2h + (size_t)(32 * at + r) * kH);
    #pragma unroll
    for (int s = 0; s < 8; ++s) bw[s] = wp[2 * s + hh];
    const float bias = (float)a.b2h[32 * at + r];
    const int k = 32 * at + r;                                              // this lane's action column
    f32x16 acc[4];
    #pragma unroll
    for (int u = 0; u < 4; ++u)
        #pragma unroll
        for (int i = 0; i < 16; ++i) acc[u][i] = 0.0f;
    float gb = 0.0f;
    uint8_t* img = sh[wv];
    // software pipeline: the row index two tiles ahead, the h row and statistics one
    // tile ahead (the loop is otherwise bound by the latency of its dependent loads)
    auto row_of = [&](int tile) {
        const int pos = tile * 32 + r, p = pos < a.m ? pos : a.m - 1;
        return a.perm ? a.perm[p] : p;
    };
    uint4 ha[8];                                                            // A operand: h[row][16s + 8hh + j]
    float4 stc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    int infc = 0, row_nn = 0;
    if (tile0 < tile1) {
        const uint4* hp = (const uint4*)(a.h + (size_t)row_of(tile0) * kH);
        #pragma unroll
        for (int s = 0; s < 8; ++s) ha[s] = hp[2 * s + hh];
        const int pos = tile0 * 32 + r;
        if (pos < a.m) { stc = a.stats[pos]; infc = a.info[pos]; }          // else lim 0: nothing in play
        if (tile0 + 1 < tile1) row_nn = row_of(tile0 + 1);
    }
    for (int tile = tile0; tile < tile1; ++tile) {
        uint4 hn[8];
        float4 stn = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        int infn = 0, row_n3 = 0;
        if (tile + 1 < tile1) {
            const uint4* hp = (const uint4*)(a.h + (size_t)row_nn * kH);
            #pragma unroll
            for (int s = 0; s < 8; ++s) hn[s] = hp[2 * s + hh];
            const int pos = (tile + 1) * 32 + r;
            if (pos < a.m) { stn = a.stats[pos]; infn = a.info[pos]; }
            if (tile + 2 < tile1) row_n3 = row_of(tile + 2);
        }
        #pragma unroll
        for (int s = 0; s < 8; ++s) *(uint4*)(img + swz(r, 2 * s + hh)) = ha[s];
        if (hh == 0) {
            sst[wv][r] = stc;
            sinf[wv][r] = infc;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        // the value tile of row tiles whose rows have no action column there in play (every
        // class but the 16-tile one, lim <= 480): p = 0 on its action columns, so dz is the
        // value gradient at column kA and zero elsewhere -- no logits needed (round 6)
        const bool vfast = at == kVT && __ballot((infc >> 16) > 32 * kVT) == 0ull;
        uint32_t D[8];
        if (vfast) {
            #pragma unroll
            for (int i = 0; i < 16; i += 2) {
                float d2[2];
                #pragma unroll
                for (int e2 = 0; e2 < 2; ++e2) {
                    const int ri = ((i + e2) & 3) + 8 * ((i + e2) >> 2) + 4 * hh;
                    const float4 st = sst[wv][ri];
                    const int act = sinf[wv][ri] & 0xFFFF;
                    const float d = k == kA ? st.w : (k == act ? st.z : 0.0f);
                    const _Float16 dh16 = (_Float16)d;
                    gb += (float)dh16;
                    d2[e2] = (float)dh16;
                }
                D[i >> 1] = __builtin_bit_cast(uint32_t, f16x2{(_Float16)d2[0], (_Float16)d2[1]});
            }
        } else {
        f32x16 z;
        #pragma unroll
        for (int i = 0; i < 16; ++i) z[i] = 0.0f;
        #pragma unroll
        for (int s = 0; s < 8; ++s) z = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_h8(ha[s]), as_h8(bw[s]), z, 0, 0, 0);
        #pragma unroll
        for (int i = 0; i < 16; i += 2) {
            float d2[2];
            #pragma unroll
            for (int e2 = 0; e2 < 2; ++e2) {
                const int ii = i + e2;
                const int ri = (ii & 3) + 8 * (ii >> 2) + 4 * hh;           // the register's row
                const float4 st = sst[wv][ri];
                const int inf = sinf[wv][ri];
                const int lim = inf >> 16, act = inf & 0xFFFF;
                const float zz = (float)(_Float16)(z[ii] + bias);
                const float tz = k < lim ? zz * kL2e : -INFINITY;
                const float nlse = -st.x * kLn2;
                const Elem e = elem(tz, st.x, nlse);
                float d = fmaf(e.p, fmaf(a.k1, e.q, st.y), k == act ? st.z : 0.0f);
                if (k == kA) d = st.w;
                const _Float16 dh16 = (_Float16)d;
                gb += (float)dh16;
                d2[e2] = (float)dh16;
            }
            D[i >> 1] = __builtin_bit_cast(uint32_t, f16x2{(_Float16)d2[0], (_Float16)d2[1]});
        }
        }
        #pragma unroll
        for (int s = 0; s < 2; ++s) {
            const f16x8 afr = __builtin_bit_cast(f16x8, make_uint4(D[4 * s], D[4 * s + 1], D[4 * s + 2], D[4 * s + 3]));
            #pragma unroll
            for (int u = 0; u < 4; ++u)
                acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(afr, tr_operand(img, 0, s, u, l), acc[u], 0, 0, 0);
        }
        __builtin_amdgcn_wave_barrier();                                    // tile reads done before the next stores
        #pragma unroll
        for (int s = 0; s < 8; ++s) ha[s] = hn[s];
        stc = stn;
        infc = infn;
        row_nn = row_n3;
    }
    gb = hsum(gb);
    // C = gW2 tile: lane = hidden 32u + r, register i = action row (i&3) + 8(i>>2) + 4hh
    float* out = a.part + (size_t)task * kPart;
    #pragma unroll
    for (int u = 0; u < 4; ++u)
        #pragma unroll
        for (int i = 0; i < 16; ++i) out[((i & 3) + 8 * (i >> 2) + 4 * hh) * kH + 32 * u + r] = acc[u][i];
    if (hh == 0) out[32 * kH + r] = gb;
}

// gW2[32at + i][c] += sum over the action tile's tasks of their partials, in a fixed
// order: k_ppo_gw2_sum1 sums the tasks of residue g mod kRed (8-way unrolled
// independent loads), k_ppo_gw2_sum2 the kRed group sums.
constexpr int kRed = 32;
__global__ __launch_bounds__(256) void k_ppo_gw2_sum1(const float* __restrict__ part, const int32_t* __restrict__ plan,
                                                      float* __restrict__ part2) {
    const int at = blockIdx.y, g = blockIdx.z;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kPart) return;
    const int t0 = plan[at] + g, t1 = plan[at + 1];
    float acc[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    int t = t0;
    for (; t + 7 * kRed < t1; t += 8 * kRed) {
        #pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += part[(size_t)(t + k * kRed) * kPart + e];
    }
    for (int k = 0; t < t1; t += kRed, ++k) acc[k] += part[(size_t)t * kPart + e];
    part2[((size_t)at * kRed + g) * kPart + e] =
        ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}
__global__ __launch_bounds__(256) void k_ppo_gw2_sum2(const float* __restrict__ part2, float* __restrict__ gw2,
                                                      float* __restrict__ gb2) {
    const int at = blockIdx.y;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kPart) return;
    float s = 0.0f;
    #pragma unroll 8
    for (int g = 0; g < kRed; ++g) s += part2[((size_t)at * kRed + g) * kPart + e];
    if (e < 32 * kH) gw2[(size_t)(32 * at) * kH + e] += s;
    else gb2[32 * at + (e - 32 * kH)] += s;
}


// ---- gW1 / gb1 of the fp16 epoch straight from the records (fc1 of
// policy_network.py:69-70 under autocast; ppo_agent.py:268-305's backward):
// gw1[u][f] = sum over rows of dh[row][u] * x[row][f], x = [the 198 features (fp16,
// as autocast casts them) | 1 (column 198: gb1) | 0], fp32 accumulation.  The
// round-3 epoch read 208-wide fp16 feature rows materialised once per update
// (0.8 GB) through a split-K hipBLASLt GEMM; here the features are generated on
// chip from the 64-byte records.  The reduction axis is the row, so both MFMA
// operands need 8 consecutive rows per lane: dh [32 rows][128] is staged in a
// swizzled LDS image and read transposed (tr_operand), the records are staged
// TRANSPOSED ([byte][row]) so that one 32-bit LDS read yields a byte for 4
// consecutive rows.  A workgroup = 7 waves, wave fb owning features 32fb..32fb+31
// (224 >= 199) as the A operand (lane = feature) and all 4 unit blocks as B: 4
// accumulators, 8 MFMAs per 32-row tile.  Every feature is one byte value v (a
// point count, bar, off, or the mover) through clamp(v * a + b, 0, c):
// n >= k: (1, -(k - 1), 1); (n - 3) / 2 for n >= 3: (1/2, -3/2, 64); bar / 2:
// (1/2, 0, 64); off / 15: (1/15, 0, 1) (fp16(v * fp32(1/15)) == fp16(fp32(v / 15))
// for v = 0..15); mover one-hot: (-1, 1, 1) / (1, 0, 1); ones column (0, 1, 1).
constexpr int kFB = 7;                      // feature blocks of 32
constexpr int kW1 = 208;                    // gw1 row width (198 features, ones column, zeros)
constexpr int kGw1Part = kFB * 32 * kH;     // floats per workgroup partial, [224][128]
constexpr int kGw1Grid = 512;               // workgroups (2 per CU)
constexpr int kGw1Rows = 64;                // rows per LDS stage: two 32-row MFMA tiles per barrier
                                            // (32 rows: the same time; 128: registers spill, 2x slower)
constexpr int kGw1Dh = kGw1Rows * 16 / 512; // 16-byte dh chunks per thread and stage
constexpr int kGw1RecThreads = kGw1Rows / 4 * 14;     // record loaders: 4 rows x one dword each

// Every feature but off / 15 is exact in f16 arithmetic on t = 1024 + v (f16 has unit
// spacing at 1024): u = min(max(t A + B, 0), C) with n >= k: (1, -1024 - k, 1);
// (n - 3) / 2: (1/2, -513.5, 64); bar / 2: (1/2, -512, 64); mover one-hot f196:
// (-1, 1025, 1), f197: (1, -1024, 1); the ones column: (0, 1, 1); padding: 0.
// off / 15 (fp16(v * fp32(1/15)), as autocast casts fp32 v / 15) stays on the fp32 path.
__device__ __forceinline__ void gw1_param(int f, int& byte, float& fa, float& fbias, float& fc, bool& off) {
    byte = 0; fa = 0.0f; fbias = 0.0f; fc = 0.0f; off = false;
    if (f < 196) {
        const int p = f >= 98 ? 1 : 0, q = f - 98 * p;
        if (q < 96) {
            const int k = q & 3;
            byte = 24 * p + (q >> 2);
            if (k < 3) { fa = 1.0f; fbias = -1024.0f - (float)k; fc = 1.0f; }
            else { fa = 0.5f; fbias = -513.5f; fc = 64.0f; }
        } else if (q == 96) { byte = 48 + p; fa = 0.5f; fbias = -512.0f; fc = 64.0f; }
        else { byte = 50 + p; off = true; }
    } else if (f < 198) { byte = 52; fa = f == 196 ? -1.0f : 1.0f; fbias = f == 196 ? 1025.0f : -1024.0f; fc = 1.0f; }
    else if (f == 198) { fbias = 1.0f; fc = 1.0f; }
}

// the A operand (8 rows of this lane's feature) from two dwords of 4 row bytes each
__device__ __forceinline__ f16x8 gw1_feats(uint32_t w0, uint32_t w1, f16x2 fa, f16x2 fb, f16x2 fc, bool off) {
    uint4 r;
    uint32_t* rp = &r.x;
    #pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t w = j < 2 ? w0 : w1;
        // (0x64 | byte 2j', 0x64 | byte 2j'+1) of w -> the f16 pair (1024 + v0, 1024 + v1)
        const uint32_t tb = __builtin_amdgcn_perm(0x64646464u, w, (j & 1) ? 0x04030402u : 0x04010400u);
        f16x2 u = __builtin_elementwise_fma(__builtin_bit_cast(f16x2, tb), fa, fb);
        u = __builtin_elementwise_min(__builtin_elementwise_max(u, (f16x2){(_Float16)0.0f, (_Float16)0.0f}), fc);
        rp[j] = __builtin_bit_cast(uint32_t, u);
    }
    if (off) {                                     // lane-divergent: the 2 off features of 224
        #pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t w = j < 2 ? w0 : w1;
            const int b0 = 16 * (j & 1);
            const _Float16 x0 = (_Float16)((float)((w >> b0) & 255u) * (1.0f / 15.0f));
            const _Float16 x1 = (_Float16)((float)((w >> (b0 + 8)) & 255u) * (1.0f / 15.0f));
            rp[j] = __builtin_bit_cast(uint32_t, (f16x2){x0, x1});
        }
    }
    return __builtin_bit_cast(f16x8, r);
}

struct Gw1Args {
    const _Float16* dh;         // [m][128]
    const uint8_t* rec;         // [m][64], the same row order
    int m, stages_per_wg;
    float* part;                // [grid][224][128]
};

// The transposed records [byte][row]: byte b of row r at b * kGw1Rows + ((r + 4 (b >> 2)) mod
// kGw1Rows), a rotation by the byte's dword so that the 14 lanes storing one row group's 14
// dwords hit 14 banks; 4 consecutive rows r = 0 mod 4 stay one aligned dword, stored whole.
// (Round 4 stored single bytes, all 56 lanes of a row-major mapping on one bank: 90 of the
// kernel's 342 us per 2^21 rows.)
__device__ __forceinline__ int srt_at(int b, int r) { return b * kGw1Rows + ((r + 4 * (b >> 2)) & (kGw1Rows - 1)); }

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_ppo_gw1(Gw1Args a) {
    __shared__ __attribute__((aligned(16))) uint8_t sdh[2][kGw1Rows * 256];
    __shared__ __attribute__((aligned(16))) uint8_t srt[2][56 * kGw1Rows];
    const int tid = threadIdx.x, fb = tid >> 6, hh = (tid >> 5) & 1;
    const int nst = (a.m + kGw1Rows - 1) / kGw1Rows;
    const int t0 = blockIdx.x * a.stages_per_wg, t1 = min(t0 + a.stages_per_wg, nst);
    int byte;
    float pa, pb, pc;
    bool off;
    gw1_param(32 * fb + (tid & 31), byte, pa, pb, pc, off);
    const f16x2 fa = {(_Float16)pa, (_Float16)pa}, fbv = {(_Float16)pb, (_Float16)pb}, fc = {(_Float16)pc, (_Float16)pc};
    f32x16 acc[4];
    #pragma unroll
    for (int u = 0; u < 4; ++u)
        #pragma unroll
        for (int i = 0; i < 16; ++i) acc[u][i] = 0.0f;
    // 8 waves: waves 0-6 own the feature blocks, wave 7 only loads.  Loaders per stage: dh =
    // 64 rows x 16 chunks of 16 B (chunks tid, tid + 512); records = 64 rows x 14 dwords
    // (bytes 0..55): dwords tid and, for tid < 384, tid + 512.  Two stages in flight: the
    // loads of stage t + 2 are issued while stage t is computed.
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    // records: thread t < kGw1RecThreads loads dword dw = t % 14 of rows 4g..4g+3, g = t / 14
    // (lanes of one row group read one row's 56 bytes contiguously per load) and stores the
    // four transposed dwords (byte 4dw + q of the 4 rows) whole
    struct Ld { uint4 d[kGw1Dh]; uint32_t rw[4]; };
    const int rg = tid / 14, rdw = tid - 14 * rg;
    auto load = [&](int st) {
        Ld x;
        #pragma unroll
        for (int k = 0; k < kGw1Dh; ++k) x.d[k] = z4;
        #pragma unroll
        for (int j = 0; j < 4; ++j) x.rw[j] = 0u;
        if (st >= t1) return x;
        const int row0 = st * kGw1Rows;
        #pragma unroll
        for (int k = 0; k < kGw1Dh; ++k) {
            const int c = tid + 512 * k;
            x.d[k] = row0 + (c >> 4) < a.m ? ((const uint4*)(a.dh + (size_t)(row0 + (c >> 4)) * kH))[c & 15] : z4;
        }
        if (tid < kGw1RecThreads)
            #pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = row0 + 4 * rg + j, gr = r < a.m ? r : a.m - 1;
                x.rw[j] = ((const uint32_t*)(a.rec + (size_t)gr * 64))[rdw];
            }
        return x;
    };
    Ld q0 = load(t0), q1 = load(t0 + 1);
    int buf = 0;
    for (int st = t0; st < t1; ++st, buf ^= 1) {
        #pragma unroll
        for (int k = 0; k < kGw1Dh; ++k) {
            const int c = tid + 512 * k;
            *(uint4*)(sdh[buf] + swz(c >> 4, c & 15)) = q0.d[k];
        }
        if (tid < kGw1RecThreads)
            #pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t v = ((q0.rw[0] >> (8 * q)) & 255u) | (((q0.rw[1] >> (8 * q)) & 255u) << 8) |
                                   (((q0.rw[2] >> (8 * q)) & 255u) << 16) | (((q0.rw[3] >> (8 * q)) & 255u) << 24);
                *(uint32_t*)(srt[buf] + srt_at(4 * rdw + q, 4 * rg)) = v;
            }
        __syncthreads();
        q0 = q1;
        q1 = load(st + 2);                                  // behind this stage's MFMAs
        if (fb == kFB) continue;                            // the loader wave (wave-uniform)
        #pragma unroll
        for (int sub = 0; sub < kGw1Rows / 32; ++sub)
            #pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                int rr = 4 * (byte >> 2) + 4 * hh;          // laundered: recomputed per use, not
                __asm__ volatile("" : "+v"(rr));            // hoisted into 8 registers
                const uint8_t* bp = srt[buf] + byte * kGw1Rows;
                const f16x8 A = gw1_feats(*(const uint32_t*)(bp + ((rr + 32 * sub + 16 * s2) & (kGw1Rows - 1))),
                                          *(const uint32_t*)(bp + ((rr + 32 * sub + 16 * s2 + 8) & (kGw1Rows - 1))),
                                          fa, fbv, fc, off);
                #pragma unroll
                for (int u = 0; u < 4; ++u)
                    acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                        A, tr_operand(sdh[buf], 32 * sub, s2, u, laundered_lane()), acc[u], 0, 0, 0);
            }
    }
    // C = [32 features][32 units] per u: lane = unit 32u + (l & 31), register i = feature (i&3) + 8(i>>2) + 4hh
    if (fb == kFB) return;
    float* out = a.part + (size_t)blockIdx.x * kGw1Part;
    #pragma unroll
    for (int u = 0; u < 4; ++u)
        #pragma unroll
        for (int i = 0; i < 16; ++i)
            out[(32 * fb + (i & 3) + 8 * (i >> 2) + 4 * hh) * kH + 32 * u + (tid & 31)] = acc[u][i];
}

// gw1[u][f] += the workgroups' partials [f][u], summed in a fixed order (group g sums
// workgroups g, g + kRed, ...; then the kRed group sums), f < 208
__global__ __launch_bounds__(256) void k_ppo_gw1_sum1(const float* __restrict__ part, int nwg, float* __restrict__ part2) {
    const int g = blockIdx.y;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kGw1Part) return;
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    int w = g, k = 0;
    for (; w < nwg; w += kRed, k = (k + 1) & 3) acc[k] += part[(size_t)w * kGw1Part + e];
    part2[(size_t)g * kGw1Part + e] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
}
__global__ __launch_bounds__(256) void k_ppo_gw1_sum2(const float* __restrict__ part2, float* __restrict__ gw1) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kW1 * kH) return;
    float s = 0.0f;
    #pragma unroll 8
    for (int g = 0; g < kRed; ++g) s += part2[(size_t)g * kGw1Part + e];
    const int f = e / kH, u = e - kH * f;
    gw1[u * kW1 + f] += s;
}


// ---- discounted returns per game lane (bgx.train.lane_returns; ppo_agent.py:206-216
// restated per lane): R_t = r_t + gamma R_{t+1}, R reset at done -- one thread per lane
// walking its T steps backwards, the same two fp32 roundings as the torch ops (no fma)
__global__ __launch_bounds__(256) void k_lane_returns(const float* __restrict__ r, const uint8_t* __restrict__ d,
                                                      int T, int B, float gamma, float* __restrict__ out) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    float R = 0.0f;
    for (int t = T - 1; t >= 0; --t) {
        const size_t i = (size_t)t * B + b;
        if (d[i]) R = 0.0f;
        R = __fadd_rn(r[i], __fmul_rn(gamma, R));
        out[i] = R;
    }
}

// ---- the rollout's episode accounting per game lane (bgx_episode_stats;
// bgx.train.episode_stats restated, train.py:55-99): one thread per lane walks its T
// steps, accumulating the unfinished episode's reward from the carry, closing it at each
// done; per-block sums of the six statistics (fp64: the rewards are multiples of 1/2, so
// every sum is exact in any order), then one block adds the block sums in order.  The
// mover byte (record byte 52) is read only at winning steps.
constexpr int kEpStats = 6;
__global__ __launch_bounds__(256) void k_episode_partials(const float* __restrict__ r, const uint8_t* __restrict__ d,
                                                          const uint8_t* __restrict__ rec, double* __restrict__ carry,
                                                          int T, int B, double* __restrict__ part) {
    __shared__ double red[4][kEpStats];
    const int b = blockIdx.x * 256 + threadIdx.x;
    double v[kEpStats] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (b < B) {
        double acc = carry[b];
        for (int t = 0; t < T; ++t) {
            const size_t i = (size_t)t * B + b;
            const double rw = (double)r[i];
            acc += rw;
            if (d[i]) {
                v[0] += 1.0;                               // finished episodes
                v[1] += acc;                               // their rewards (carry included)
                acc = 0.0;
                if (rw > 0.0) {
                    v[2] += 1.0;                           // wins (the mover of a winning step)
                    v[3] += rec[i * 64 + 52] == 0 ? 1.0 : 0.0;     // by PLAYER1
                }
                v[4] += rw == 1.5 ? 1.0 : 0.0;             // gammon wins
                v[5] += rw == 2.0 ? 1.0 : 0.0;             // backgammon wins
            }
        }
        carry[b] = acc;
    }
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    #pragma unroll
    for (int k = 0; k < kEpStats; ++k) {
        double x = v[k];
        #pragma unroll
        for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
        if (l == 0) red[w][k] = x;
    }
    __syncthreads();
    if (threadIdx.x < kEpStats)
        part[(size_t)blockIdx.x * kEpStats + threadIdx.x] =
            red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}
__global__ __launch_bounds__(64) void k_episode_sum(const double* __restrict__ part, int nb, double* __restrict__ out) {
    if (threadIdx.x >= kEpStats) return;
    double s = 0.0;
    for (int k = 0; k < nb; ++k) s += part[(size_t)k * kEpStats + threadIdx.x];
    out[threadIdx.x] = s;
}

// ---- the update's rollout rows in plan order (bgx_gather_rollout): 4 threads per row,
// each copying 16 bytes of the record; thread 0..3 of a row also copies one of the four
// per-row fields
__global__ __launch_bounds__(256) void k_gather_rollout(const int32_t* __restrict__ perm, int n,
                                                        const uint4* __restrict__ rec, const int32_t* __restrict__ act,
                                                        const float* __restrict__ old, const float* __restrict__ ret,
                                                        const float* __restrict__ adv, uint4* __restrict__ rec_o,
                                                        int32_t* __restrict__ act_o, float* __restrict__ old_o,
                                                        float* __restrict__ ret_o, float* __restrict__ adv_o) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t i = t >> 2;
    const int q = (int)(t & 3);
    if (i >= n) return;
    const int64_t src = perm[i];
    rec_o[i * 4 + q] = rec[src * 4 + q];
    if (q == 0) act_o[i] = act[src];
    else if (q == 1) old_o[i] = old[src];
    else if (q == 2) ret_o[i] = ret[src];
    else adv_o[i] = adv[src];
}

// ---- the fused head's row plan on the device (bgx_ppo_plan; round 5).  A row's class
// is the number of 32-action tiles it needs: ceil(lim / 32), lim = n_actions for a row
// with no legal move, else min(count, n_actions) (the count from record bytes 60-61).
// The rows are ordered by class, stably (a counting sort: per-block class counts, one
// block scanning them per class, then each row's rank from ballots), and the plan of
// k_ppo_gw2 / the bgx_ppo_rows variants follows from the 17 class totals.  Replaces
// torch's argsort + bincount (a host sync: bincount sizes its output from the data) +
// cumsum and a dozen small launches of round 4's ppo_row_plan.
constexpr int kPlanCls = 17;                 // classes 0..16 (0 never occurs)
constexpr int kPlanRows = 1024;              // rows per counting block

__device__ __forceinline__ int plan_class(const uint8_t* rec, int64_t i, int n_actions) {
    const int cnt = (int)rec[i * 64 + 60] | ((int)rec[i * 64 + 61] << 8);
    const int lim = cnt == 0 ? n_actions : (cnt < n_actions ? cnt : n_actions);
    return (lim + 31) >> 5;
}

// per-wave class counts of this block's rows (LDS wc[16][17]) for the row's class c (0
// past the end); returns its rank among the wave's rows of that class
__device__ __forceinline__ int plan_wave_counts(int c, int (*wc)[kPlanCls]) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint64_t below = (1ull << l) - 1ull;
    int rank = 0;
    #pragma unroll
    for (int k = 1; k < kPlanCls; ++k) {
        const uint64_t b = __ballot(c == k);
        if (c == k) rank = __popcll(b & below);
        if (l == 0) wc[w][k] = __popcll(b);
    }
    if (l == 0) wc[w][0] = 0;
    __syncthreads();
    return rank;
}

// bcnt class-major: bcnt[k][b] = block b's class-k rows
__global__ __launch_bounds__(kPlanRows) void k_plan_count(const uint8_t* __restrict__ rec, int m, int n_actions,
                                                          int32_t* __restrict__ bcnt) {
    __shared__ int wc[kPlanRows / 64][kPlanCls];
    const int64_t i = (int64_t)blockIdx.x * kPlanRows + threadIdx.x;
    (void)plan_wave_counts(i < m ? plan_class(rec, i, n_actions) : 0, wc);
    if (threadIdx.x < kPlanCls) {
        int t = 0;
        #pragma unroll
        for (int w = 0; w < kPlanRows / 64; ++w) t += wc[w][threadIdx.x];
        bcnt[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = t;
    }
}

// one workgroup, wave k - 1 scanning class k over the blocks: boff[k][b] = the position of
// block b's first class-k row among the class-k rows, base[k] = the class's first sorted
// position; then the plan from the class totals.  Round 6: the counts class-major, each
// lane's 32 loads in flight before the scans (was one strided load per 64 blocks in a
// dependent chain: 52 us per 2^21 rows)
constexpr int kPlanScanRegs = 32;
__global__ __launch_bounds__(1024) void k_plan_scan(const int32_t* __restrict__ bcnt, int nb, int m,
                                                    int32_t* __restrict__ boff, int32_t* __restrict__ gbase,
                                                    int32_t* __restrict__ plan, int32_t* __restrict__ row_plan) {
    __shared__ int tot[kPlanCls];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, k = w + 1;
    const int32_t* src = bcnt + (size_t)k * nb;
    int32_t* dst = boff + (size_t)k * nb;
    int run = 0;
    for (int b0 = 0; b0 < nb; b0 += 64 * kPlanScanRegs) {
        int v[kPlanScanRegs];
        #pragma unroll
        for (int j = 0; j < kPlanScanRegs; ++j) {
            const int b = b0 + 64 * j + l;
            v[j] = b < nb ? src[b] : 0;
        }
        #pragma unroll
        for (int j = 0; j < kPlanScanRegs; ++j) {
            const int b = b0 + 64 * j + l;
            int x = v[j];                                // inclusive scan over the 64 lanes
            #pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o);
                if (l >= o) x += y;
            }
            if (b < nb) dst[b] = run + x - v[j];
            run += __shfl(x, 63);
        }
    }
    if (l == 0) tot[k] = run;
    if (threadIdx.x == 0) tot[0] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        int cum[kPlanCls];
        for (int c = 0; c < kPlanCls; ++c) { gbase[c] = acc; acc += tot[c]; cum[c] = acc; }
        // ppo_row_plan (bgx/train.py): start[o] = first row tile reaching action tile o
        // (the value column's tile 15: every row); tasks of kTS row tiles per action tile
        const int ntiles = (m + 31) / 32;
        int pre = 0;
        for (int o = 0; o < 16; ++o) {
            const int st = o == 15 ? 0 : cum[o] / 32;
            plan[17 + o] = st;
            plan[o] = pre;
            pre += (ntiles + kTS - 1) / kTS - st / kTS;          // kTS-aligned row groups from st
        }
        plan[16] = pre;
        int e[3];
        const int ks[3] = {1, 2, 4};
        for (int j = 0; j < 3; ++j) e[j] = cum[ks[j]] >= m ? ntiles : cum[ks[j]] / 32;
        row_plan[0] = 0; row_plan[1] = e[0]; row_plan[2] = e[0]; row_plan[3] = e[1];
        row_plan[4] = e[1]; row_plan[5] = e[2]; row_plan[6] = e[2]; row_plan[7] = ntiles;
    }
}

// each row's sorted position; writes perm (may be null) and, when rows.rec_o is set, the
// row itself there (round 6: the gather of the update's rows folded into the scatter --
// the record read once, coalesced, instead of a perm pass and a random-read gather)
struct PlanRows {
    const int32_t* act;
    const float *old, *ret, *adv;
    uint4* rec_o;
    int32_t* act_o;
    float *old_o, *ret_o, *adv_o;
};
__global__ __launch_bounds__(kPlanRows) void k_plan_scatter(const uint8_t* __restrict__ rec, int m, int n_actions,
                                                            const int32_t* __restrict__ boff,
                                                            const int32_t* __restrict__ gbase,
                                                            int32_t* __restrict__ perm, PlanRows rows) {
    __shared__ int wc[kPlanRows / 64][kPlanCls];
    const int64_t i = (int64_t)blockIdx.x * kPlanRows + threadIdx.x;
    const int c = i < m ? plan_class(rec, i, n_actions) : 0;
    const int rank = plan_wave_counts(c, wc);
    int off = 0;
    if (i < m) {
        off = gbase[c] + boff[(size_t)c * gridDim.x + blockIdx.x] + rank;
        for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) off += wc[w][c];
        if (perm) perm[off] = (int32_t)i;
    }
    if (rows.rec_o) {
        // the wave's 64 records, 4 lanes per record (16 bytes each), 16 records per pass: each
        // store instruction writes whole 64-byte records (a thread per record wrote 16-byte
        // pieces of 64 different records per instruction: 111 us per 2^21 rows)
        const int l = threadIdx.x & 63;
        const int64_t wbase = i - l;
        #pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int rr = 16 * it + (l >> 2);
            const int dst = __shfl(off, rr);
            if (wbase + rr < m) rows.rec_o[(int64_t)dst * 4 + (l & 3)] = ((const uint4*)rec)[(wbase + rr) * 4 + (l & 3)];
        }
        if (i < m) {
            rows.act_o[off] = rows.act[i];
            rows.old_o[off] = rows.old[i];
            rows.ret_o[off] = rows.ret[i];
            rows.adv_o[off] = rows.adv[i];
        }
    }
}

// ---- the optimizer step (bgx_adam_step): torch.optim.Adam(fused=True) driven by
// GradScaler.step + update, as three launches over the flat element range of every
// tensor instead of torch's per-tensor multi-tensor chunks (a 90 k-parameter net ran
// as ~4 workgroups each walking 65,536 elements: 69 us for the Adam kernel alone, plus
// the inf check, the step increments and the scale update as separate launches)
constexpr int kAdamMax = 8;
struct AdamArgs {
    float* p[kAdamMax];
    float* g[kAdamMax];
    float* m[kAdamMax];
    float* v[kAdamMax];
    float* step[kAdamMax];
    int64_t end[kAdamMax];            // exclusive prefix sums of the element counts
    int n;
    int64_t total;
    double lr, beta1, beta2, eps;     // torch passes them as doubles
    const float* scale;               // GradScaler scale (null: no scaler)
    int32_t* found;                   // non-finite flag (0 between calls)
};

__device__ __forceinline__ int adam_tensor(const AdamArgs& a, int64_t i) {
    int t = 0;
    #pragma unroll
    for (int k = 0; k < kAdamMax - 1; ++k)
        t += (k < a.n - 1 && i >= a.end[k]) ? 1 : 0;
    return t;
}

// GradScaler._check_inf_per_device: any non-finite scaled gradient
__global__ __launch_bounds__(256) void k_adam_check(AdamArgs a) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool bad = false;
    if (i < a.total) {
        const int t = adam_tensor(a, i);
        const float g = a.g[t][i - (t ? a.end[t - 1] : 0)];
        bad = !isfinite(g);
    }
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(a.found, 1);
}

// _fused_adam_ (ADAM_MODE::ORIGINAL, no weight decay / amsgrad / maximize): the
// gradient unscaled by the GradScaler scale (and stored back, as torch does), then the
// moments and the parameter at step s + 1; nothing when the check found a non-finite.
// The mixed fp32 / fp64 arithmetic follows torch's adam_math (fp32 state, double
// hyper-parameters: the moment updates and the unscale round from fp64, the bias
// corrections are fp64 rounded to fp32, the parameter update is fp32)
__global__ __launch_bounds__(256) void k_adam_apply(AdamArgs a) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.total || (a.scale && *a.found)) return;
    const int t = adam_tensor(a, i);
    const int64_t j = i - (t ? a.end[t - 1] : 0);
    float g = a.g[t][j];
    if (a.scale) {
        g = (float)((double)g / (double)*a.scale);
        a.g[t][j] = g;
    }
    const double s = (double)(*a.step[t] + 1.0f);
    float m = a.m[t][j], v = a.v[t][j];
    m = (float)(a.beta1 * (double)m + (1.0 - a.beta1) * (double)g);
    v = (float)(a.beta2 * (double)v + (1.0 - a.beta2) * (double)g * (double)g);
    const float bc1 = (float)(1.0 - pow(a.beta1, s));
    const float bc2s = (float)sqrt(1.0 - pow(a.beta2, s));
    const float step_size = (float)(a.lr / (double)bc1);
    const float denom = (float)((double)(sqrtf(v) / bc2s) + a.eps);
    a.p[t][j] -= step_size * m / denom;
    a.m[t][j] = m;
    a.v[t][j] = v;
}

// the step counters (+1 unless skipped) and _amp_update_scale_; the flag back to 0
__global__ void k_adam_finish(AdamArgs a, float* scale, int32_t* tracker, float growth, float backoff, int interval) {
    const int l = threadIdx.x;
    const int found = (a.scale && *a.found) ? 1 : 0;
    if (l < a.n && !found) *a.step[l] += 1.0f;
    if (l == 0 && scale) {
        if (found) {
            *scale = (float)((double)*scale * (double)backoff);
            *tracker = 0;
        } else {
            const int succ = *tracker + 1;
            if (succ == interval) {
                const float ns = (float)((double)*scale * (double)growth);
                if (isfinite(ns)) *scale = ns;
                *tracker = 0;
            } else {
                *tracker = succ;
            }
        }
        *a.found = 0;
    }
}

}  // namespace

extern int bgx_internal_fail(hipError_t e);

extern "C" int bgx_adam_step(int32_t n, float* const* params, float* const* grads, float* const* exp_avg,
                             float* const* exp_avg_sq, float* const* steps, const int64_t* numels, double lr,
                             double beta1, double beta2, double eps, float* scale, int32_t* growth_tracker,
                             float growth_factor, float backoff_factor, int32_t growth_interval, int32_t* found,
                             void* stream) {
    if (n <= 0 || n > kAdamMax || !params || !grads || !exp_avg || !exp_avg_sq || !steps || !numels || !found)
        return BGX_EINVAL;
    if (scale && !growth_tracker) return BGX_EINVAL;
    AdamArgs a{};
    int64_t tot = 0;
    for (int t = 0; t < n; ++t) {
        if (!params[t] || !grads[t] || !exp_avg[t] || !exp_avg_sq[t] || !steps[t] || numels[t] < 0) return BGX_EINVAL;
        a.p[t] = params[t]; a.g[t] = grads[t]; a.m[t] = exp_avg[t]; a.v[t] = exp_avg_sq[t]; a.step[t] = steps[t];
        tot += numels[t];
        a.end[t] = tot;
    }
    for (int t = n; t < kAdamMax; ++t) a.end[t] = tot;
    a.n = n; a.total = tot;
    a.lr = lr; a.beta1 = beta1; a.beta2 = beta2; a.eps = eps;
    a.scale = scale; a.found = found;
    hipStream_t s = (hipStream_t)stream;
    const unsigned blocks = (unsigned)((tot + 255) / 256);
    if (tot > 0) {
        if (scale) hipLaunchKernelGGL(k_adam_check, dim3(blocks), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_adam_apply, dim3(blocks), dim3(256), 0, s, a);
    }
    hipLaunchKernelGGL(k_adam_finish, dim3(1), dim3(64), 0, s, a, scale, growth_tracker, growth_factor, backoff_factor,
                       growth_interval);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}

extern "C" int bgx_ppo_rows(const void* h, const int32_t* perm, const uint8_t* records, const int32_t* actions,
                            const float* old_logp, const float* returns, const float* adv, int32_t m, int32_t hidden,
                            int32_t n_actions, const void* w2h, const void* b2h, float eps_clip, float c_value,
                            float c_entropy, float grad_scale, void* dh, void* stats, int32_t* info, double* sums,
                            void* dy, void* z, const int32_t* row_plan, int32_t grid, void* stream) {
    if (hidden != kH || n_actions != kA || m < 0) return BGX_EINVAL;
    if (m == 0) return BGX_OK;
    if (!h || !records || !actions || !old_logp || !returns || !adv || !w2h || !b2h || !dh || !stats ||
        !info || !sums || !row_plan)
        return BGX_EINVAL;
    if (((uintptr_t)h | (uintptr_t)w2h | (uintptr_t)stats | (uintptr_t)dy) % 16 || ((uintptr_t)dh | (uintptr_t)b2h) % 8 ||
        (uintptr_t)z % 2)
        return BGX_EINVAL;
    RowsArgs a{(const _Float16*)h, perm, records, actions, old_logp, returns, adv, (const _Float16*)w2h,
               (const _Float16*)b2h, m, eps_clip, c_value, c_entropy, grad_scale, (_Float16*)dh, (float4*)stats,
               info, sums, (_Float16*)dy, (_Float16*)z};
    hipStream_t s = (hipStream_t)stream;
    const int ntiles = (m + 31) / 32;
    // persistent grids: at most enough workgroups for every row tile, else `grid` (<= 0:
    // 4 per CU for the small variants, 1 per CU for the 16-tile one)
    auto wgs = [&](int waves, int dflt) {
        const int need = (ntiles + waves - 1) / waves, g = grid > 0 ? grid : dflt;
        return dim3(need < g ? need : g);
    };
    // (the 16-tile variant on a side stream beside the small ones, launched first, was
    // measured slower: k_ppo_rows<1> 255 -> 392 us with a quarter of its LDS slots,
    // update 7.27 -> 7.6 ms; profiles/r5/rejected/rows_fork)
    hipLaunchKernelGGL(k_ppo_rows<1>, wgs(4, 1024), dim3(256), 0, s, a, row_plan + 0);
    hipLaunchKernelGGL(k_ppo_rows<2>, wgs(4, 1024), dim3(256), 0, s, a, row_plan + 2);
    hipLaunchKernelGGL(k_ppo_rows<4>, wgs(4, 1024), dim3(256), 0, s, a, row_plan + 4);
    hipLaunchKernelGGL(k_ppo_rows<kNT>, wgs(8, 256), dim3(512), 0, s, a, row_plan + 6);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}

extern "C" int64_t bgx_ppo_gw2_workspace(int32_t m) {
    if (m < 0) return BGX_EINVAL;
    const int64_t ntiles = (m + 31) / 32;
    // task partials, then kRed group sums per action tile
    return ((int64_t)kNT * ((ntiles + kTS - 1) / kTS) + (int64_t)kNT * kRed) * kPart * (int64_t)sizeof(float);
}

extern "C" int bgx_ppo_gw2(const void* h, const int32_t* perm, const void* stats, const int32_t* info, int32_t m,
                           int32_t hidden, int32_t n_actions, const void* w2h, const void* b2h, float k1,
                           const int32_t* plan, float* workspace, float* gw2, float* gb2, void* stream) {
    if (hidden != kH || n_actions != kA || m < 0) return BGX_EINVAL;
    if (m == 0) return BGX_OK;
    if (!h || !stats || !info || !w2h || !b2h || !plan || !workspace || !gw2 || !gb2) return BGX_EINVAL;
    if (((uintptr_t)h | (uintptr_t)w2h | (uintptr_t)stats) % 16) return BGX_EINVAL;
    const int ntiles = (m + 31) / 32;
    const int max_tasks = kNT * ((ntiles + kTS - 1) / kTS);
    Gw2Args a{(const _Float16*)h, perm, (const float4*)stats, info, (const _Float16*)w2h, (const _Float16*)b2h, m, k1,
              plan, workspace};
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_ppo_gw2, dim3((max_tasks + 3) / 4), dim3(256), 0, s, a);
    float* part2 = workspace + (size_t)max_tasks * kPart;
    hipLaunchKernelGGL(k_ppo_gw2_sum1, dim3((kPart + 255) / 256, kNT, kRed), dim3(256), 0, s, workspace, plan, part2);
    hipLaunchKernelGGL(k_ppo_gw2_sum2, dim3((kPart + 255) / 256, kNT), dim3(256), 0, s, part2, gw2, gb2);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}


extern "C" int64_t bgx_ppo_gw1_workspace(int32_t m) {
    if (m < 0) return BGX_EINVAL;
    const int64_t nst = (m + kGw1Rows - 1) / kGw1Rows;
    const int64_t wgs = nst < kGw1Grid ? (nst > 0 ? nst : 1) : kGw1Grid;
    return (wgs + kRed) * kGw1Part * (int64_t)sizeof(float);
}

extern "C" int bgx_ppo_gw1(const void* dh, const uint8_t* records, int32_t m, int32_t hidden, float* workspace,
                           float* gw1, void* stream) {
    if (hidden != kH || m < 0) return BGX_EINVAL;
    if (m == 0) return BGX_OK;
    if (!dh || !records || !workspace || !gw1) return BGX_EINVAL;
    if (((uintptr_t)dh | (uintptr_t)records) % 16 || (uintptr_t)workspace % 16) return BGX_EINVAL;
    const int nst = (m + kGw1Rows - 1) / kGw1Rows;
    const int wgs = nst < kGw1Grid ? nst : kGw1Grid;
    const int per = (nst + wgs - 1) / wgs;
    Gw1Args a{(const _Float16*)dh, records, m, per, workspace};
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_ppo_gw1, dim3(wgs), dim3(512), 0, s, a);
    float* part2 = workspace + (size_t)wgs * kGw1Part;
    hipLaunchKernelGGL(k_ppo_gw1_sum1, dim3((kGw1Part + 255) / 256, kRed), dim3(256), 0, s, workspace, wgs, part2);
    hipLaunchKernelGGL(k_ppo_gw1_sum2, dim3((kW1 * kH + 255) / 256), dim3(256), 0, s, part2, gw1);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}

extern "C" int bgx_gather_rollout(const int32_t* perm, int32_t n, const uint8_t* records, const int32_t* actions,
                                  const float* old_logp, const float* returns, const float* adv, uint8_t* records_out,
                                  int32_t* actions_out, float* old_logp_out, float* returns_out, float* adv_out,
                                  void* stream) {
    if (n < 0) return BGX_EINVAL;
    if (n == 0) return BGX_OK;
    if (!perm || !records || !actions || !old_logp || !returns || !adv || !records_out || !actions_out ||
        !old_logp_out || !returns_out || !adv_out)
        return BGX_EINVAL;
    if (((uintptr_t)records | (uintptr_t)records_out) % 16) return BGX_EINVAL;
    const int64_t threads = (int64_t)n * 4;
    hipLaunchKernelGGL(k_gather_rollout, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       perm, n, (const uint4*)records, actions, old_logp, returns, adv, (uint4*)records_out,
                       actions_out, old_logp_out, returns_out, adv_out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}

extern "C" int64_t bgx_ppo_plan_workspace(int32_t m) {
    if (m < 0) return BGX_EINVAL;
    const int64_t nb = ((int64_t)m + kPlanRows - 1) / kPlanRows;
    return (2 * nb * kPlanCls + kPlanCls) * 4;
}

static int ppo_plan(const uint8_t* records, int32_t m, int32_t n_actions, int32_t* workspace, int32_t* perm,
                    const PlanRows& rows, int32_t* plan, int32_t* row_plan, void* stream) {
    const int nb = (m + kPlanRows - 1) / kPlanRows;
    hipStream_t s = (hipStream_t)stream;
    int32_t* bcnt = workspace;
    int32_t* boff = workspace + (size_t)nb * kPlanCls;
    int32_t* gbase = boff + (size_t)nb * kPlanCls;
    if (nb > 0) hipLaunchKernelGGL(k_plan_count, dim3(nb), dim3(kPlanRows), 0, s, records, m, n_actions, bcnt);
    hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(1024), 0, s, bcnt, nb, m, boff, gbase, plan, row_plan);
    if (nb > 0)
        hipLaunchKernelGGL(k_plan_scatter, dim3(nb), dim3(kPlanRows), 0, s, records, m, n_actions, boff, gbase, perm,
                           rows);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}

extern "C" int bgx_ppo_plan(const uint8_t* records, int32_t m, int32_t n_actions, int32_t* workspace, int32_t* perm,
                            int32_t* plan, int32_t* row_plan, void* stream) {
    if (m < 0 || n_actions <= 0 || n_actions > kNT * 32 - 1 || (m > 0 && (!records || !workspace || !perm)) ||
        !plan || !row_plan)
        return BGX_EINVAL;
    return ppo_plan(records, m, n_actions, workspace, perm, PlanRows{}, plan, row_plan, stream);
}

extern "C" int bgx_ppo_plan_rows(const uint8_t* records, int32_t m, int32_t n_actions, int32_t* workspace,
                                 const int32_t* actions, const float* old_logp, const float* returns, const float* adv,
                                 uint8_t* records_out, int32_t* actions_out, float* old_logp_out, float* returns_out,
                                 float* adv_out, int32_t* perm_or_null, int32_t* plan, int32_t* row_plan,
                                 void* stream) {
    if (m < 0 || n_actions <= 0 || n_actions > kNT * 32 - 1 || !plan || !row_plan ||
        (m > 0 && (!records || !workspace || !actions || !old_logp || !returns || !adv || !records_out ||
                   !actions_out || !old_logp_out || !returns_out || !adv_out)))
        return BGX_EINVAL;
    if (((uintptr_t)records | (uintptr_t)records_out) % 16) return BGX_EINVAL;
    const PlanRows rows{actions, old_logp, returns, adv, (uint4*)records_out, actions_out, old_logp_out, returns_out,
                        adv_out};
    return ppo_plan(records, m, n_actions, workspace, perm_or_null, rows, plan, row_plan, stream);
}

// The fused epoch's gradients into the parameters' .grad tensors, scaled by `post` in
// fp32 (as Tensor.mul_ of the accumulators), in one launch (bgx_ppo_epoch_grads; replaces
// three multiplies and six slice copies per epoch); block 0 also evaluates the masked-
// action shortcut's bound: guard |= 2 (max_a |W2h[a]| sqrt(hmax2) + max_a |b2h[a]|) > limit
// over the action rows a < A (the same quantities as the torch form, fp32; the per-row
// norms come from bgx_ppo_epoch_prep, one wave per row).
struct EpochGrads {
    const float *gw1, *gw2, *gb2;
    int hidden, n_actions;
    float post;
    float *w1g, *b1g, *wag, *bag, *wvg, *bvg;
    const float* hmax2;
    float limit;
    uint8_t* guard;
    const float* bound;         // [2][512] from bgx_ppo_epoch_prep
    const double* sums;         // the epoch's loss sums (may be NULL: no parts)
    double n_total, c_value, c_entropy;
    double* parts;              // [4] += (policy, value, entropy, total) of this epoch
};
__global__ __launch_bounds__(256) void k_ppo_epoch_grads(EpochGrads a) {
    const int H = a.hidden, A = a.n_actions;
    if (a.parts && blockIdx.x == gridDim.x - 1) {
        // the epoch's loss parts as the torch form computes them (fp64, no contraction):
        // m = sums / n; total = m0 + c_v m1 - c_e m2; parts += (m0, m1, m2, total)
        if (threadIdx.x == 0) {
            const double m0 = __ddiv_rn(a.sums[0], a.n_total), m1 = __ddiv_rn(a.sums[1], a.n_total),
                         m2 = __ddiv_rn(a.sums[2], a.n_total);
            const double tot = __dsub_rn(__dadd_rn(m0, __dmul_rn(a.c_value, m1)), __dmul_rn(a.c_entropy, m2));
            a.parts[0] = __dadd_rn(a.parts[0], m0);
            a.parts[1] = __dadd_rn(a.parts[1], m1);
            a.parts[2] = __dadd_rn(a.parts[2], m2);
            a.parts[3] = __dadd_rn(a.parts[3], tot);
        }
        return;
    }
    if (blockIdx.x == 0 && a.guard) {
        __shared__ float mn[256], mb[256];
        float n2 = 0.0f, b = 0.0f;
        for (int r = threadIdx.x; r < A; r += 256) {       // the row bounds bgx_ppo_epoch_prep wrote
            n2 = fmaxf(n2, a.bound[r]);
            b = fmaxf(b, a.bound[512 + r]);
        }
        mn[threadIdx.x] = n2;
        mb[threadIdx.x] = b;
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if (threadIdx.x < o) {
                mn[threadIdx.x] = fmaxf(mn[threadIdx.x], mn[threadIdx.x + o]);
                mb[threadIdx.x] = fmaxf(mb[threadIdx.x], mb[threadIdx.x + o]);
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            const float U = mn[0] * sqrtf(a.hmax2[0]) + mb[0];
            if (2.0f * U > a.limit) a.guard[0] = 1;
        }
        return;
    }
    const long long n0 = (long long)H * 198, n1 = n0 + H, n2 = n1 + (long long)A * H, n3 = n2 + A, n4 = n3 + H,
                    n5 = n4 + 1;
    const int nb = (int)gridDim.x - (a.guard ? 1 : 0) - (a.parts ? 1 : 0), b0 = a.guard ? blockIdx.x - 1 : blockIdx.x;
    for (long long g = (long long)b0 * 256 + threadIdx.x; g < n5; g += (long long)nb * 256) {
        if (g < n0) {
            const int u = (int)(g / 198), f = (int)(g % 198);
            a.w1g[g] = a.gw1[(size_t)u * 208 + f] * a.post;
        } else if (g < n1) {
            const int u = (int)(g - n0);
            a.b1g[u] = a.gw1[(size_t)u * 208 + 198] * a.post;
        } else if (g < n2) {
            a.wag[g - n1] = a.gw2[g - n1] * a.post;
        } else if (g < n3) {
            a.bag[g - n2] = a.gb2[g - n2] * a.post;
        } else if (g < n4) {
            a.wvg[g - n3] = a.gw2[(size_t)A * H + (g - n3)] * a.post;
        } else {
            a.bvg[0] = a.gb2[A] * a.post;
        }
    }
}

extern "C" int bgx_ppo_epoch_grads(const float* gw1_dev, const float* gw2_dev, const float* gb2_dev, int32_t hidden,
                                   int32_t n_actions, float post, float* w1_grad, float* b1_grad, float* wa_grad,
                                   float* ba_grad, float* wv_grad, float* bv_grad, const float* bound_dev,
                                   const float* hmax2_dev, float limit, uint8_t* guard_dev_or_null,
                                   const double* sums_dev, double n_total, double c_value, double c_entropy,
                                   double* parts_dev_or_null, void* stream) {
    if (hidden <= 0 || hidden > 128 || n_actions <= 0 || n_actions >= 512) return BGX_EINVAL;
    if (!gw1_dev || !gw2_dev || !gb2_dev || !w1_grad || !b1_grad || !wa_grad || !ba_grad || !wv_grad || !bv_grad)
        return BGX_EINVAL;
    if (guard_dev_or_null && (!bound_dev || !hmax2_dev)) return BGX_EINVAL;
    if (parts_dev_or_null && (!sums_dev || !(n_total > 0.0))) return BGX_EINVAL;
    EpochGrads a{gw1_dev, gw2_dev, gb2_dev, hidden, n_actions, post, w1_grad, b1_grad, wa_grad, ba_grad, wv_grad,
                 bv_grad, hmax2_dev, limit, guard_dev_or_null, bound_dev, sums_dev, n_total, c_value, c_entropy,
                 parts_dev_or_null};
    hipLaunchKernelGGL(k_ppo_epoch_grads, dim3(256 + (guard_dev_or_null ? 1 : 0) + (parts_dev_or_null ? 1 : 0)),
                       dim3(256), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}

extern "C" int64_t bgx_episode_stats_workspace(int32_t B) {
    if (B < 0) return BGX_EINVAL;
    return (int64_t)((B + 255) / 256) * kEpStats * (int64_t)sizeof(double);
}

extern "C" int bgx_episode_stats(const float* rewards, const uint8_t* dones, const uint8_t* records, double* carry,
                                 int32_t T, int32_t B, double* workspace, double* out, void* stream) {
    if (T < 0 || B < 0 || !out || (B > 0 && (!carry || !workspace)) ||
        (T > 0 && B > 0 && (!rewards || !dones || !records)))
        return BGX_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int nb = (B + 255) / 256;
    if (nb > 0)
        hipLaunchKernelGGL(k_episode_partials, dim3(nb), dim3(256), 0, s, rewards, dones, records, carry, T, B,
                           workspace);
    hipLaunchKernelGGL(k_episode_sum, dim3(1), dim3(64), 0, s, workspace, nb, out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}

extern "C" int bgx_lane_returns(const float* rewards, const uint8_t* dones, int32_t T, int32_t B, float gamma,
                                float* out, void* stream) {
    if (T < 0 || B < 0 || (T > 0 && B > 0 && (!rewards || !dones || !out))) return BGX_EINVAL;
    if (T == 0 || B == 0) return BGX_OK;
    hipLaunchKernelGGL(k_lane_returns, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, rewards, dones, T, B,
                       gamma, out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BGX_OK : bgx_internal_fail(e);
}
