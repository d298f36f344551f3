// bg_mlp.hip — BackgammonPolicyNetwork (agent/policy_network.py:44-75) on MFMA,
// fused with the feature encoder and select_action's masked sampling
// (agent/ppo_agent.py:164-187).
//
// One wave = 32 game rows.  GEMM1 computes X1 = W1 . F^T (hidden x rows), the B
// operand (features) generated on the fly from the rows' int8 lane records
// staged in LDS.  The accumulator layout of X1 (column = row on the lane, hidden
// units in registers) is used UNMOVED as the B operand of GEMM2
// (Y = W2 . X1, W2 = [action_head; value_head]): the host packs W2's columns in
// the k order the accumulator registers deliver.  Each lane then owns 16
// outputs of one row per 32-row output tile, so the masked log-sum-exp and the
// Gumbel-max draw run in registers with one cross-half shuffle per row.
//
// Precision: fp32 semantics from f16 MFMA (v_mfma_f32_32x32x16_f16, 16x the
// f32-MFMA rate).  Every operand x is split x = hi + lo (hi = f16(x),
// lo = f16(x - hi)) and a product is hi*hi + hi*lo + lo*hi: 22 significant bits
// per operand, products exact in the f32 accumulator, the dropped lo*lo term
// below 2^-22 relative.  GEMM1's features are exact f16 values (K order
// permuted, kperm_src), so only W1 is split: 2 MFMAs per k-block and tile.  Power-of-two scales keep the parts in f16's normal
// range: per weight matrix (pack time, max |w| -> [2^13, 2^14)) and per wave for
// the hidden layer; they are undone exactly.  Logits/values match torch fp32 to
// ~1e-6 (tests/test_gpu_policy.py asserts 1e-5).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "../../include/bgx.h"
#include "bg_debug.h"


namespace {

constexpr int kW1Ahead = 2;      // k-blocks of W1 fragments in flight in the policy kernel's GEMM1

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int kIn = 198;
constexpr int kKB1 = (kIn + 15) / 16;     // 13 k-blocks of 16 (features padded to 208)
constexpr float kMaskLog = -103.27892990343185f;  // log(fp32(1e-45)) (ppo_agent.py:166)
constexpr int kHdr = 16;                  // header floats: [0] = e1, [1] = e2 (int bits)

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// GEMM1's K order is permuted so that every feature is an exact f16 value
// generated without branches (bgx_policy_pack packs W1's columns to match):
// k-blocks 0-5 = P1 points 0..23, 6-11 = P2 points, 4 features per point
// [n>=1, n>=2, n>=3, (n-3)/2] — lane half h of k-block kb holds points
// 4(kb mod 6) + 2h + {0, 1}; k-block 12 (h = 0) = P1 bar/2, P1 off, P2 bar/2,
// P2 off, one-hot[2], then zeros.  The off features are the counts themselves:
// their W1 columns are pre-divided by 15 (the reference's off/15).
// Returns the reference feature index (immutable_board.py:171-212) or -1.
__host__ __device__ inline int kperm_src(int kb, int h, int i) {
    if (kb < 12) {
        const int p = kb >= 6 ? 1 : 0;
        const int pt = 4 * (kb - 6 * p) + 2 * h + (i >> 2);
        return 98 * p + 4 * pt + (i & 3);
    }
    if (kb > 12 || h != 0 || i >= 6) return -1;
    return i < 2 ? 96 + i : 192 + i;             // 96, 97, 194, 195, 196, 197
}

// the 8 f16 features of lane half h in k-block kb (K order above) of the row
// whose 64-byte record starts at rec (LDS)
__device__ __forceinline__ f16x8 feats8(const uint8_t* rec, int kb, int h) {
    f16x8 f;
    if (kb < 12) {
        const int base = (kb >= 6 ? 24 + 4 * (kb - 6) : 4 * kb) + 2 * h;
        #pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int n = rec[base + q];
            f[4 * q + 0] = n >= 1 ? (_Float16)1.0f : (_Float16)0.0f;
            f[4 * q + 1] = n >= 2 ? (_Float16)1.0f : (_Float16)0.0f;
            f[4 * q + 2] = n >= 3 ? (_Float16)1.0f : (_Float16)0.0f;
            f[4 * q + 3] = (_Float16)(n >= 3 ? (float)(n - 3) * 0.5f : 0.0f);
        }
    } else {
        const bool on = h == 0;
        f[0] = on ? (_Float16)((float)rec[48] * 0.5f) : (_Float16)0.0f;
        f[1] = on ? (_Float16)(float)rec[50] : (_Float16)0.0f;
        f[2] = on ? (_Float16)((float)rec[49] * 0.5f) : (_Float16)0.0f;
        f[3] = on ? (_Float16)(float)rec[51] : (_Float16)0.0f;
        f[4] = on && rec[52] == 0 ? (_Float16)1.0f : (_Float16)0.0f;
        f[5] = on && rec[52] != 0 ? (_Float16)1.0f : (_Float16)0.0f;
        f[6] = (_Float16)0.0f;
        f[7] = (_Float16)0.0f;
    }
    return f;
}

__device__ __forceinline__ void split(float x, _Float16& hi, _Float16& lo) {
    hi = (_Float16)x;
    lo = (_Float16)(x - (float)hi);
}

__device__ __forceinline__ f16x8 as_h8(uint4 v) { return __builtin_bit_cast(f16x8, v); }

// exponent e with max_abs * 2^e in [2^13, 2^14) (0 for 0 / non-finite)
__device__ __forceinline__ int scale_exp(float max_abs) {
    if (!(max_abs > 0.0f) || !(max_abs < INFINITY)) return 0;
    int q;
    (void)frexpf(max_abs, &q);
    const int e = 14 - q;
    return e < -100 ? -100 : (e > 100 ? 100 : e);
}

// 32-bit mixer (lowbias32): a bijection with good avalanche; noise for the
// Gumbel-max draw keyed by (seed, step, row, action)
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    return x;
}

// v_log_f32 / v_exp_f32 directly (base 2): every argument below is a normal float
__device__ __forceinline__ float fast_ln(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

// gumbel() below is at most -log(2^-24) = 16.64 (u <= 1 - 2^-24)
constexpr float kGumbelMax = 17.0f;

// Gumbel(0,1) = -log(E), E = -log(u) ~ Exp(1), u = ((w >> 9) + 1/2) 2^-23 in (0,1).
// For u close to 1, -log(u) = v + v^2/2 + v^3/3 with v = 1 - u (exact), so E keeps
// full relative precision where the hardware log would lose it.
__device__ __forceinline__ float gumbel(uint32_t w) {
    const float u = ((float)(w >> 9) + 0.5f) * (1.0f / 8388608.0f);
    const float v = 1.0f - u;
    const float series = v * (1.0f + v * (0.5f + v * (1.0f / 3.0f)));
    const float e = v < (1.0f / 64.0f) ? series : -fast_ln(u);
    return -fast_ln(e);
}

// Packed layout (bgx_policy_pack), in floats:
//   hdr  [16]                       e1, e2 (int bits)
//   w1q  [13][T][2][64] x uint4     lane l: W1s[32t + (l&31)][kperm_src(kb, l>>5, i)], i = 0..7, part 0 = hi,
//                                   1 = lo (off columns / 15; 0 where kperm_src < 0)
//   b1p  [T][16][64] f32            b1[32t + hid(r, l>>5)] * 2^e1
//   w2q  [OT][T][2][2][64] x uint4  lane l, sub-block m: W2s[32o + (l&31)][32t + hid(8m + i, l>>5)]
//   b2p  [OT][16][64] f32           b2[32o + hid(r, l>>5)]  (unscaled)
// with W1s = W1 * 2^e1, W2s = W2 * 2^e2, hid(r, h) = (r&3) + 8(r>>2) + 4h (the
// 32x32 accumulator row map), W2 = [action_head.weight; value_head.weight; 0].
__device__ __forceinline__ int hid(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

struct PackView {
    const int* hdr;
    const uint4* w1q;
    const float* b1p;
    const uint4* w2q;
    const float* b2p;
};

__host__ __device__ inline int sz_w1q(int T) { return kKB1 * T * 2 * 64 * 4; }
__host__ __device__ inline int sz_b1p(int T) { return T * 16 * 64; }
__host__ __device__ inline int sz_w2q(int T, int OT) { return OT * T * 2 * 2 * 64 * 4; }
__host__ __device__ inline int sz_b2p(int OT) { return OT * 16 * 64; }

template <typename P>
__host__ __device__ inline void views(P base, int T, int OT, P& hdr, P& w1q, P& b1p, P& w2q, P& b2p) {
    hdr = base;
    w1q = hdr + kHdr;
    b1p = w1q + sz_w1q(T);
    w2q = b1p + sz_b1p(T);
    b2p = w2q + sz_w2q(T, OT);
}

// MODE 0: sampling without the logits output (the rollout: no per-output
// branches in the tile loop); MODE -1: greedy / logits_out as passed.
//
// MODE 0 with skip_arg != 0 (round 3): masked-action tile skip.  A 32-row wave whose
// rows have at most c legal actions needs output tiles 0 .. ceil(c/32)-1 and the
// value tile only: every other output a < n_actions of those rows is masked,
// z = z0 + kMaskLog with z0 <= ub = max ba + max_a |Wa[a]|_2 |h|_2 (Cauchy-Schwarz;
// header floats 2-3).  When, for every row, ub + kMaskLog lies kSkipMargin below the
// row's running max (its log-sum-exp terms are then below half an ulp of the sum,
// which is >= 1) and ub + kMaskLog + kGumbelMax below the row's best Gumbel key (no
// key of the tile can win), those tiles cannot change any output: the wave jumps to
// the value tile.  A row with no legal move (count 0) samples from all n_actions
// outputs, so the main waves leave such rows to 2 extra workgroups per kZWin rows
// in the same launch (the grid's first blocks), each gathering up to 32 of the
// window's count-0 rows; its 4 waves split the output tiles (a quarter each) and
// wave 0 merges their partial log-sum-exp / Gumbel-max states through LDS, so the
// extra workgroups last about as long as the skipping main waves.  A window with
// more than kZCap count-0 rows (never at self-play's ~5 %) keeps them on its main
// waves, unskipped.  Outputs equal the unskipped kernel's up to the log-sum-exp's
// summation order (the noise is keyed by (row, action)); BGX_POLICY_SKIP=0 turns
// the skip off.  MODE 0 workgroups are 4 waves: 4 x 32 rows, or one gathered set.
// Round 5: the extra workgroups also take the rows with more than skip_arg (64) legal
// actions (BGX_POLICY_HEAVY), so no main wave walks more than 2 action tiles plus the
// value tile: per-wave stamps (tools/policy_stamps.py) showed the main waves of a
// 16,384-row launch at 12.6 us of output tiles on average but 36 us for the slowest --
// a 32-row group holding a doubles row with hundreds of legal moves walks all 16 tiles
// alone -- and that wave set the launch at 45.7 us; now 20.3 us (C3 380 -> 412 M env
// steps/s; 32 is worse: the 64-row windows of the extra workgroups overflow).
constexpr int kZWin = 256, kZCap = 64;
constexpr int kHeavyDefault = 64;

#ifdef BGX_POLICY_STAMPS
// experiment: per-wave s_memrealtime stamps of the rollout policy kernel (tools/policy_stamps.py)
// [wave][6]: start, after the count-0 scan + staging, after GEMM1, end, flags (extra | main), tiles
constexpr int kStampWaves = 8192;
__device__ unsigned long long g_pstamp[kStampWaves][6];
#define PSTAMP(k) do { if (MODE == 0 && sw < kStampWaves && lane_id() == 0) g_pstamp[sw][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define PSTAMP(k) do { } while (0)
#endif
constexpr float kSkipMargin = 30.0f;

template <int T, int MODE>
__global__ __launch_bounds__(MODE == 0 ? 256 : 64) __attribute__((amdgpu_waves_per_eu(2))) void k_policy_act(const uint8_t* __restrict__ recs, int n,
                                                   const float* __restrict__ packed, int n_actions, int n_otiles,
                                                   uint32_t seed_lo, uint32_t seed_hi, uint32_t step_arg,
                                                   const uint32_t* __restrict__ step_ctr, int greedy_arg,
                                                   int32_t* act_out, float* logp_out, float* value_out,
                                                   float* logits_arg, uint8_t* records_out, int skip_arg) {
    // the noise's step: the argument, plus a device counter when given (a replayed graph)
#ifdef BGX_POLICY_STAMPS
    const int sw = (int)(blockIdx.x * (MODE == 0 ? 4 : 1) + (threadIdx.x >> 6));
#endif
    PSTAMP(0);
    const uint32_t step = step_arg + (step_ctr ? *step_ctr : 0u);
    constexpr int kW = MODE == 0 ? 4 : 1;              // waves per workgroup
    const bool greedy = MODE < 0 ? greedy_arg != 0 : false;
    float* const logits_out = MODE < 0 ? logits_arg : nullptr;
    const bool skip_on = MODE == 0 && skip_arg != 0;
    __shared__ uint8_t srec_[kW][32 * 64];
    __shared__ int zl[MODE == 0 ? kZCap : 1];
    const float *hdrf, *w1f, *b1p, *w2f, *b2p;
    views(packed, T, n_otiles, hdrf, w1f, b1p, w2f, b2p);
    const uint4* w1q = (const uint4*)w1f;
    const uint4* w2q = (const uint4*)w2f;
    const int e1 = __builtin_bit_cast(int, hdrf[0]), e2 = __builtin_bit_cast(int, hdrf[1]);
    const int l = lane_id();
    const int j = l & 31, h = l >> 5;
    const int wv = kW > 1 ? (int)(threadIdx.x >> 6) : 0;
    uint8_t* const srec = srec_[wv];
    // the extra workgroups come first in the grid: they start first
    const int n_extra = skip_on ? 2 * ((n + kZWin - 1) / kZWin) : 0;
    const bool extra = (int)blockIdx.x < n_extra;
    const int row0 = (((int)blockIdx.x - n_extra) * kW + wv) * 32;
    if (!extra && row0 >= n) return;                   // main waves: no barrier below
    // count-0 rows of the kZWin-row window (the first kZCap of them in zl, extra waves)
    int nzw = 0;
    if (skip_on) {
        const int base = (extra ? (int)blockIdx.x >> 1 : row0 / kZWin) * kZWin;
        uint16_t cw[kZWin / 64];                       // all loads in flight before the first ballot
        #pragma unroll
        for (int k = 0; k < kZWin / 64; ++k)
            cw[k] = *(const uint16_t*)(recs + (size_t)min(base + 64 * k + l, n - 1) * 64 + 60);
        #pragma unroll
        for (int k = 0; k < kZWin / 64; ++k) {
            const int r = base + 64 * k + l;
            const bool z = r < n && (cw[k] == 0 || (int)cw[k] > skip_arg);
            const uint64_t m = __ballot(z);
            const int pos = nzw + __popcll(m & ((1ull << l) - 1ull));
            if (extra && wv == 0 && z && pos < kZCap) zl[pos] = r;
            nzw += __popcll(m);
        }
    }
    const int kx = extra ? ((int)blockIdx.x & 1) : 0;
    const int nz = extra ? min(nzw - 32 * kx, 32) : 32;       // rows of this wave (extra: gathered)
    if (extra && (nzw > kZCap || nz <= 0)) return;             // uniform in the workgroup
    const bool self_zero = skip_on && !extra && nzw > kZCap;   // gathered rows stay on the main wave
    const int vt = n_actions >> 5;                     // the tile holding the value output
    if (extra) __syncthreads();                        // zl
    // stage 32 records (2 KiB, this wave's own copy): lane l copies 32 bytes
    {
        const int r = l >> 1, off = (l & 1) * 32;
        const int gr = extra ? zl[32 * kx + (r < nz ? r : 0)] : (row0 + r < n ? row0 + r : n - 1);
        const uint4* src = (const uint4*)(recs + (size_t)gr * 64 + off);
        uint4* dst = (uint4*)(srec + r * 64 + off);
        const uint4 v0 = src[0], v1 = src[1];
        dst[0] = v0;
        dst[1] = v1;
        if (!extra && records_out && row0 + r < n) {   // the rollout row's copy of the record
            uint4* o = (uint4*)(records_out + (size_t)(row0 + r) * 64 + off);
            o[0] = v0;
            o[1] = v1;
        }
    }
    if (kW > 1) __builtin_amdgcn_wave_barrier(); else __syncthreads();
    const uint8_t* myrec = srec + j * 64;
    const int count = (int)myrec[60] | ((int)myrec[61] << 8);
    // this row is an extra workgroup's (count 0, or more than skip_arg legal actions)
    const bool gathered = skip_on && !extra && !self_zero && (count == 0 || count > skip_arg);
    const bool row_ok = extra ? j < nz : row0 + j < n;
    const int grow = extra ? zl[32 * kx + (j < nz ? j : 0)] : row0 + j;
    // output tiles of this wave: all (main), a quarter (extra)
    const int per = extra ? (n_otiles + kW - 1) / kW : n_otiles;
    const int o_beg = extra ? min(wv * per, n_otiles) : 0, o_end = extra ? min(o_beg + per, n_otiles) : n_otiles;

    PSTAMP(1);
    // ---- GEMM1: X1s[t] = W1s[32t.., :] . F^T + b1 * 2^e1  (= 2^e1 X1)
    f32x16 x1[T];
    #pragma unroll
    for (int t = 0; t < T; ++t)
        #pragma unroll
        for (int r = 0; r < 16; ++r) x1[t][r] = b1p[(t * 16 + r) * 64 + l];
    // W1's fragments stream from L2 kPD k-blocks ahead of their MFMAs (a ring of
    // registers): at one or two waves per SIMD nothing else hides the L2 latency
    constexpr int kPD = kW1Ahead;
    uint4 wf[kPD + 1][2 * T];
    #pragma unroll
    for (int p = 0; p < kPD; ++p)
        #pragma unroll
        for (int f = 0; f < 2 * T; ++f) wf[p][f] = w1q[(p * 2 * T + f) * 64 + l];
    #pragma unroll
    for (int kb = 0; kb < kKB1; ++kb) {
        if (kb + kPD < kKB1) {
            #pragma unroll
            for (int f = 0; f < 2 * T; ++f) wf[(kb + kPD) % (kPD + 1)][f] = w1q[((kb + kPD) * 2 * T + f) * 64 + l];
        }
        __builtin_amdgcn_sched_barrier(0);
        const f16x8 bf = feats8(myrec, kb, h);         // exact in f16: no lo part
        #pragma unroll
        for (int t = 0; t < T; ++t) {
            const f16x8 ah = as_h8(wf[kb % (kPD + 1)][2 * t + 0]);
            const f16x8 al = as_h8(wf[kb % (kPD + 1)][2 * t + 1]);
            x1[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bf, x1[t], 0, 0, 0);
            x1[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bf, x1[t], 0, 0, 0);
        }
    }
    // ReLU, then a per-wave scale 2^ex for the split of the hidden layer
    float mx = 0.0f, hn2 = 0.0f;
    #pragma unroll
    for (int t = 0; t < T; ++t)
        #pragma unroll
        for (int r = 0; r < 16; ++r) {
            x1[t][r] = fmaxf(x1[t][r], 0.0f);
            mx = fmaxf(mx, x1[t][r]);
            if (skip_on) hn2 = fmaf(x1[t][r], x1[t][r], hn2);
        }
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) mx = fmaxf(mx, __shfl_xor(mx, d));
    // the skip's first skippable tile o_s (none: n_otiles) and the rows' logit bound
    int o_s = n_otiles;
    float ub = INFINITY;
    if (skip_on && !extra) {
        int cm = gathered ? 0 : count;
        #pragma unroll
        for (int d = 1; d < 32; d <<= 1) cm = max(cm, __shfl_xor(cm, d));
        o_s = max((cm + 31) >> 5, 1);
        hn2 += __shfl_xor(hn2, 32);                    // the row's two lane halves
        const float u0 = hdrf[2] + hdrf[3] * ldexpf(sqrtf(hn2), -e1);
        ub = u0 + 1e-3f * fabsf(u0) + 1e-3f;           // rounding slack (the margin is 30)
    }
    const int ex = scale_exp(mx);
    f16x8 xh[T][2], xl[T][2];
    #pragma unroll
    for (int t = 0; t < T; ++t)
        #pragma unroll
        for (int m = 0; m < 2; ++m)
            #pragma unroll
            for (int i = 0; i < 8; ++i) {
                _Float16 a, b;
                split(ldexpf(x1[t][8 * m + i], ex), a, b);
                xh[t][m][i] = a; xl[t][m][i] = b;
            }
    // Y' = W2s . (2^(e1+ex) X1) + b2 2^E = 2^E Y,  E = e2 + e1 + ex
    const int E = e2 + e1 + ex;
    const float up = ldexpf(1.0f, E), down = ldexpf(1.0f, -E);

    PSTAMP(2);
    // ---- GEMM2 per 32-output tile + online masked log-sum-exp + Gumbel-max
    // (branch-free: outputs that are not actions of this lane enter as -inf)
    float m = -INFINITY, s = 0.0f, best = -INFINITY, bestz = 0.0f, value = 0.0f;
    int besta = 0;
    const uint32_t rowkey = mix32(mix32(seed_lo ^ mix32(seed_hi + 0x9E3779B9u)) ^ step) ^ (uint32_t)grow * 0x85EBCA6Bu;
    constexpr int NF = T * 2 * 2;                      // weight fragments per output tile
    uint4 w[NF];
    #pragma unroll
    for (int f = 0; f < NF; ++f) w[f] = o_beg < o_end ? w2q[((size_t)o_beg * NF + f) * 64 + l] : make_uint4(0, 0, 0, 0);
    for (int o = o_beg; o < o_end;) {
        f32x16 y;
        #pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = b2p[(o * 16 + r) * 64 + l] * up;
        #pragma unroll
        for (int t = 0; t < T; ++t)
            #pragma unroll
            for (int mm = 0; mm < 2; ++mm) {
                const f16x8 ah = as_h8(w[(t * 2 + mm) * 2 + 0]);
                const f16x8 al = as_h8(w[(t * 2 + mm) * 2 + 1]);
                y = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, xh[t][mm], y, 0, 0, 0);
                y = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xl[t][mm], y, 0, 0, 0);
                y = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xh[t][mm], y, 0, 0, 0);
            }
        // the next tile's fragments go into the same registers once this tile's
        // MFMAs have issued; the loads overlap the sampling math below.  At the
        // skippable range the value tile's are fetched (the skip usually holds).
        const bool at_s = o + 1 == o_s && o_s < vt;
        const int nx = at_s ? vt : o + 1;
        __asm__ volatile("" ::: "memory");
        if (nx < o_end) {
            #pragma unroll
            for (int f = 0; f < NF; ++f) w[f] = w2q[((size_t)nx * NF + f) * 64 + l];
        }
        // lane l holds outputs a = 32o + hid(r, h), r = 0..15, of row j
        float z[16];
        float tm = -INFINITY;
        #pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int a = 32 * o + hid(r, h);
            const float z0 = y[r] * down;
            if (logits_out && row_ok && a <= n_actions) logits_out[(size_t)grow * (32 * n_otiles) + a] = z0;
            value = a == n_actions ? z0 : value;
            z[r] = a < n_actions ? (a < count ? z0 : z0 + kMaskLog) : -INFINITY;
            tm = fmaxf(tm, z[r]);
        }
        const float mn = fmaxf(m, tm);
        if (mn != -INFINITY) {                         // else nothing of this lane's row so far
            float acc = 0.0f;
            #pragma unroll
            for (int r = 0; r < 16; ++r) acc += fast_exp(z[r] - mn);
            s = s * fast_exp(m - mn) + acc;
            m = mn;
        }
        // A key is z + g with g <= kGumbelMax, so when tm + kGumbelMax < best no
        // output of this tile can replace the lane's current best: the noise is
        // skipped (exact — the same keys are never larger).  Past the legal
        // actions' tile(s) this holds for every lane of a row with legal moves
        // (masked outputs sit 103 below).
        if (greedy ? tm > best : !(tm + kGumbelMax < best)) {
            #pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int a = 32 * o + hid(r, h);
                const float key = greedy ? z[r] : z[r] + gumbel(mix32(rowkey ^ ((uint32_t)a * 0xC2B2AE35u)));
                const bool up_ = key > best;
                best = up_ ? key : best;
                besta = up_ ? a : besta;
                bestz = up_ ? z[r] : bestz;
            }
        }
        int next = o + 1;
        if (at_s) {
            const float m_row = fmaxf(m, __shfl_xor(m, 32)), b_row = fmaxf(best, __shfl_xor(best, 32));
            const bool ok = gathered || (ub + kMaskLog < m_row - kSkipMargin && ub + kMaskLog + kGumbelMax < b_row);
            if (__ballot(!ok) == 0ull) {
                next = vt;
            } else {                                   // no skip: tile o + 1 after all
                #pragma unroll
                for (int f = 0; f < NF; ++f) w[f] = w2q[((size_t)(o + 1) * NF + f) * 64 + l];
            }
        }
        o = next;
    }
    if (kW > 1 && extra) {
        // waves 1..3 hand their per-lane states to wave 0 (same lane = same row half)
        __shared__ float pm[kW > 1 ? kW - 1 : 1][5][64];
        __shared__ int pa[kW > 1 ? kW - 1 : 1][64];
        if (wv > 0) {
            pm[wv - 1][0][l] = m; pm[wv - 1][1][l] = s; pm[wv - 1][2][l] = best; pm[wv - 1][3][l] = bestz;
            pm[wv - 1][4][l] = value; pa[wv - 1][l] = besta;
        }
        __syncthreads();
        if (wv > 0) return;
        #pragma unroll
        for (int q = 0; q < kW - 1; ++q) {
            const float mq = pm[q][0][l], sq = pm[q][1][l], bq = pm[q][2][l], zq = pm[q][3][l];
            const int aq = pa[q][l];
            const float mn = fmaxf(m, mq);
            if (mn != -INFINITY) s = s * fast_exp(m - mn) + sq * fast_exp(mq - mn);
            m = mn;
            const bool tk = bq > best || (bq == best && aq < besta);
            best = tk ? bq : best;
            besta = tk ? aq : besta;
            bestz = tk ? zq : bestz;
            value += pm[q][4][l];
        }
    }
    PSTAMP(3);
#ifdef BGX_POLICY_STAMPS
    if (MODE == 0 && sw < kStampWaves && lane_id() == 0) g_pstamp[sw][4] = extra ? 1 : 2;
#endif
    // combine the two lane halves of each row (lanes j and j+32)
    const float m2 = __shfl_xor(m, 32), s2 = __shfl_xor(s, 32);
    const float best2 = __shfl_xor(best, 32), bestz2 = __shfl_xor(bestz, 32);
    const int besta2 = __shfl_xor(besta, 32);
    const float value2 = __shfl_xor(value, 32);
    const float mm = fmaxf(m, m2);
    const float ss = s * fast_exp(m - mm) + s2 * fast_exp(m2 - mm);
    const bool take2 = best2 > best || (best2 == best && besta2 < besta);
    const int a_fin = take2 ? besta2 : besta;
    const float z_fin = take2 ? bestz2 : bestz;
    const float v_fin = h == 0 ? value + value2 : 0.0f;   // the value row sits in exactly one half
    // count-0 rows of the main waves belong to the extra waves
    if (h == 0 && row_ok && !gathered) {
        act_out[grow] = a_fin;
        // Categorical.log_prob = log(clamp(p, eps, 1 - eps)) (torch clamp_probs), in the log domain
        if (logp_out) logp_out[grow] = fminf(fmaxf(z_fin - (mm + logf(ss)), -15.942384719848633f),
                                             -1.1920930376163597e-07f);
        if (value_out) value_out[grow] = v_fin;
    }
}

// max |w| of W1 and of W2 = [Wa; wv] -> header exponents; max ba and max_a |Wa[a]|_2
// -> the tile skip's logit bound (one workgroup)
__global__ __launch_bounds__(1024) void k_policy_scale(const float* W1, const float* Wa, const float* ba,
                                                       const float* wv, int H, int A, float* hdr) {
    __shared__ float r1[16], r2[16], r3[16], r4[16];
    const int t = threadIdx.x;
    float m1 = 0.0f, m2 = 0.0f, bmax = -INFINITY, nmax = 0.0f;
    for (int i = t; i < H * kIn; i += 1024) m1 = fmaxf(m1, fabsf(W1[i]));
    for (int i = t; i < A * H; i += 1024) m2 = fmaxf(m2, fabsf(Wa[i]));
    for (int i = t; i < H; i += 1024) m2 = fmaxf(m2, fabsf(wv[i]));
    for (int a = t; a < A; a += 1024) {
        double q = 0.0;
        for (int k = 0; k < H; ++k) q += (double)Wa[(size_t)a * H + k] * (double)Wa[(size_t)a * H + k];
        nmax = fmaxf(nmax, (float)sqrt(q));
        bmax = fmaxf(bmax, ba[a]);
    }
    #pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        m1 = fmaxf(m1, __shfl_xor(m1, d)); m2 = fmaxf(m2, __shfl_xor(m2, d));
        bmax = fmaxf(bmax, __shfl_xor(bmax, d)); nmax = fmaxf(nmax, __shfl_xor(nmax, d));
    }
    if ((t & 63) == 0) { r1[t >> 6] = m1; r2[t >> 6] = m2; r3[t >> 6] = bmax; r4[t >> 6] = nmax; }
    __syncthreads();
    if (t == 0) {
        for (int w = 1; w < 16; ++w) {
            m1 = fmaxf(m1, r1[w]); m2 = fmaxf(m2, r2[w]); bmax = fmaxf(bmax, r3[w]); nmax = fmaxf(nmax, r4[w]);
        }
        hdr[0] = __builtin_bit_cast(float, scale_exp(m1));
        hdr[1] = __builtin_bit_cast(float, scale_exp(m2));
        hdr[2] = bmax;                                 // -inf / nan: no skip (ub is not finite)
        hdr[3] = nmax * (1.0f + 1.0f / 1024.0f);
        for (int i = 4; i < kHdr; ++i) hdr[i] = 0.0f;
    }
}

// Pack torch-layout weights into the MFMA operand layouts above.
__global__ void k_policy_pack(const float* W1, const float* b1, const float* Wa, const float* ba, const float* wv,
                              const float* bv, int H, int A, int T, int OT, float* packed) {
    float *hdr, *w1f, *b1p, *w2f, *b2p;
    views(packed, T, OT, hdr, w1f, b1p, w2f, b2p);
    const int e1 = __builtin_bit_cast(int, hdr[0]), e2 = __builtin_bit_cast(int, hdr[1]);
    _Float16* w1h = (_Float16*)w1f;
    _Float16* w2h = (_Float16*)w2f;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    // one thread per (fragment, lane, element i) for the f16 parts; hi and lo written together
    const int n1 = kKB1 * T * 64 * 8, nb1 = T * 16 * 64, n2 = OT * T * 2 * 64 * 8, nb2 = OT * 16 * 64;
    auto W2 = [&](int o, int k) -> float {
        if (k >= H) return 0.0f;
        if (o < A) return Wa[(size_t)o * H + k];
        if (o == A) return wv[k];
        return 0.0f;
    };
    auto B2 = [&](int o) -> float { return o < A ? ba[o] : (o == A ? bv[0] : 0.0f); };
    if (tid < n1) {
        const int i = tid % 8, l = (tid / 8) % 64, t = (tid / 512) % T, kb = tid / (512 * T);
        const int hrow = 32 * t + (l & 31), k = kperm_src(kb, l >> 5, i);
        const float wk = hrow < H && k >= 0 ? W1[(size_t)hrow * kIn + k] : 0.0f;
        const float w = ldexpf(k == 97 || k == 195 ? wk / 15.0f : wk, e1);   // off columns: W / 15
        _Float16 a, b;
        split(w, a, b);
        w1h[(((kb * T + t) * 2 + 0) * 64 + l) * 8 + i] = a;
        w1h[(((kb * T + t) * 2 + 1) * 64 + l) * 8 + i] = b;
    } else if (tid < n1 + nb1) {
        const int q = tid - n1;
        const int l = q % 64, r = (q / 64) % 16, t = q / (64 * 16);
        const int hrow = 32 * t + hid(r, l >> 5);
        b1p[q] = hrow < H ? ldexpf(b1[hrow], e1) : 0.0f;
    } else if (tid < n1 + nb1 + n2) {
        const int q = tid - n1 - nb1;
        const int i = q % 8, l = (q / 8) % 64, mm = (q / 512) % 2, t = (q / 1024) % T, o = q / (1024 * T);
        const int k = 32 * t + hid(8 * mm + i, l >> 5);
        _Float16 a, b;
        split(ldexpf(W2(32 * o + (l & 31), k), e2), a, b);
        const size_t f = (((size_t)(o * T + t) * 2 + mm) * 2) * 64 + l;
        w2h[f * 8 + i] = a;
        w2h[(f + 64) * 8 + i] = b;
    } else if (tid < n1 + nb1 + n2 + nb2) {
        const int q = tid - n1 - nb1 - n2;
        const int l = q % 64, r = (q / 64) % 16, o = q / (64 * 16);
        b2p[q] = B2(32 * o + hid(r, l >> 5));
    }
}


// ---- the PPO update's fc1 forward under fp16 autocast, straight from the records
// (ppo_agent.py:274 autocast + policy_network.py:69-70): h = fp16(relu(W1h . fp16(x)
// + b1h)) with fp32 accumulation, as the autocast addmm; x = get_board_features of
// each stored 64-byte record, generated in registers in kperm_src's K order (every
// feature is the fp16 cast of the fp32 feature: off / 15 rounded as autocast rounds
// it).  Replaces the [n, 208] fp16 feature read + hipBLASLt GEMM (~270 us per 2^20
// rows) by a 64-byte record read.  One wave = 32 rows per pass, 4 waves per
// workgroup sharing the W1 fragments (13 k-blocks x T tiles x 1 KiB) in LDS.
__constant__ static const float kOffDiv15[16] = {
    0.0f / 15.0f, 1.0f / 15.0f, 2.0f / 15.0f, 3.0f / 15.0f, 4.0f / 15.0f, 5.0f / 15.0f,
    6.0f / 15.0f, 7.0f / 15.0f, 8.0f / 15.0f, 9.0f / 15.0f, 10.0f / 15.0f, 11.0f / 15.0f,
    12.0f / 15.0f, 13.0f / 15.0f, 14.0f / 15.0f, 15.0f / 15.0f};

// w1h [hidden][198] fp16 -> fragments [13][T][64] x uint4: lane l of (kb, t) holds
// W1h[32t + (l & 31)][kperm_src(kb, l >> 5, i)], i = 0..7 (0 where the unit or the
// feature does not exist)
__global__ void k_fc1_pack(const _Float16* __restrict__ w1h, int hidden, int T, uint4* __restrict__ out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= kKB1 * T * 64) return;
    const int l = g & 63, t = (g >> 6) % T, kb = (g >> 6) / T;
    const int u = 32 * t + (l & 31);
    f16x8 v;
    #pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int src = kperm_src(kb, l >> 5, i);
        v[i] = (u < hidden && src >= 0) ? w1h[(size_t)u * kIn + src] : (_Float16)0.0f;
    }
    out[g] = __builtin_bit_cast(uint4, v);
}

template <int T>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_fc1_rec(const uint8_t* __restrict__ recs, int n,
                                                  const uint4* __restrict__ w1f, const _Float16* __restrict__ b1h,
                                                  int hidden, _Float16* __restrict__ hout, float* __restrict__ hmax2) {
    // the W1 fragments live in LDS for the workgroup's lifetime (T = 4: 52 KiB, shared by
    // 8 waves; the bias is added in the epilogue from LDS, as the GEMM epilogue adds it, so
    // the kernel fits 128 VGPRs: 4 waves/SIMD); each wave walks 32-row tiles grid-strided, the next tile's records loaded behind the
    // current tile's MFMAs (read per wave from L2 they were 52 KiB per 32 rows: the
    // kernel ran at the L2's rate, 195 us per 2^20 rows)
    __shared__ uint4 sw[kKB1 * T * 64];
    __shared__ __attribute__((aligned(16))) uint8_t srec[8][32 * 64];
    __shared__ float sb[32 * T];
    for (int i = threadIdx.x; i < kKB1 * T * 64; i += blockDim.x) sw[i] = w1f[i];
    for (int i = threadIdx.x; i < 32 * T; i += blockDim.x) sb[i] = i < hidden ? (float)b1h[i] : 0.0f;
    __syncthreads();
    const int l = lane_id(), wv = threadIdx.x >> 6;
    const int j = l & 31, h = l >> 5;
    const int ntiles = (n + 31) / 32, stride = gridDim.x * 8;
    int tile = blockIdx.x * 8 + wv;
    __shared__ float swm[8];
    float hm = 0.0f;
    const int r = l >> 1, off = (l & 1) * 32;
    uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0;
    if (tile < ntiles) {
        const int gr = tile * 32 + r < n ? tile * 32 + r : n - 1;
        const uint4* src = (const uint4*)(recs + (size_t)gr * 64 + off);
        v0 = src[0];
        v1 = src[1];
    }
    for (; tile < ntiles; tile += stride) {
        const int row0 = tile * 32;
        uint4* dst = (uint4*)(srec[wv] + r * 64 + off);
        dst[0] = v0;
        dst[1] = v1;
        __builtin_amdgcn_wave_barrier();
        if (tile + stride < ntiles) {                   // next tile's records in flight
            const int nr = (tile + stride) * 32 + r;
            const uint4* src = (const uint4*)(recs + (size_t)(nr < n ? nr : n - 1) * 64 + off);
            v0 = src[0];
            v1 = src[1];
        }
        const uint8_t* myrec = srec[wv] + j * 64;
        f32x16 acc[T];
        #pragma unroll
        for (int t = 0; t < T; ++t)
            #pragma unroll
            for (int q = 0; q < 16; ++q) acc[t][q] = 0.0f;
        #pragma unroll
        for (int kb = 0; kb < kKB1; ++kb) {
            f16x8 bf = feats8(myrec, kb, h);
            if (kb == 12) {                             // off counts -> fp16(off / 15), as autocast casts x
                bf[1] = h == 0 ? (_Float16)kOffDiv15[myrec[50] & 15] : (_Float16)0.0f;
                bf[3] = h == 0 ? (_Float16)kOffDiv15[myrec[51] & 15] : (_Float16)0.0f;
            }
            #pragma unroll
            for (int t = 0; t < T; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_h8(sw[(kb * T + t) * 64 + l]), bf, acc[t], 0, 0, 0);
        }
        __builtin_amdgcn_wave_barrier();                // srec reads done before the next tile's stores
        float ss = 0.0f;                                // this lane's part of the row's |h|^2
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        if (hidden % 8 == 0) {
            // the two lane halves of a row hold units 8q + 0..3 (h = 0) and 8q + 4..7 (h = 1):
            // one v_permlane32_swap per dword pairs them, so that lane h writes the 16
            // contiguous bytes of units 8(2p + h) + 0..7 (half the store instructions and
            // request fragments of 8-byte stores)
            _Float16* orow = hout + (size_t)(row0 + j) * hidden;
            #pragma unroll
            for (int t = 0; t < T; ++t)
                #pragma unroll
                for (int p = 0; p < 2; ++p) {
                    h4 v[2];
                    #pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int q = 2 * p + e, u = 32 * t + 8 * q + 4 * h;
                        #pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            v[e][i] = (_Float16)fmaxf(acc[t][4 * q + i] + sb[u + i], 0.0f);
                            if (u < hidden) ss = fmaf((float)v[e][i], (float)v[e][i], ss);
                        }
                    }
                    const uint2 a = __builtin_bit_cast(uint2, v[0]), b = __builtin_bit_cast(uint2, v[1]);
                    const auto s0 = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
                    const auto s1 = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
                    // lane h = 0: (units 8q0 + 0..3, 8q0 + 4..7); h = 1: (8q1 + 0..3, 8q1 + 4..7)
                    const int u8 = 32 * t + 8 * (2 * p + h);
                    if (row0 + j < n && u8 < hidden)
                        *(uint4*)(orow + u8) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
                }
        } else if (row0 + j < n) {
            _Float16* orow = hout + (size_t)(row0 + j) * hidden;
            #pragma unroll
            for (int t = 0; t < T; ++t)
                #pragma unroll
                for (int q = 0; q < 4; ++q) {           // units 32t + 8q + 4h + 0..3: one 8-byte store
                    const int u = 32 * t + 8 * q + 4 * h;
                    if (u < hidden) {
                        h4 v;
                        #pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            v[i] = (_Float16)fmaxf(acc[t][4 * q + i] + sb[u + i], 0.0f);
                            ss = fmaf((float)v[i], (float)v[i], ss);
                        }
                        *(h4*)(orow + u) = v;
                    }
                }
        }
        if (row0 + j >= n) ss = 0.0f;
        hm = fmaxf(hm, ss + __shfl_xor(ss, 32));        // this lane's row: both halves' parts
    }
    if (hmax2) {                                        // max |h_row|^2 of the workgroup, one atomic
        #pragma unroll
        for (int o = 16; o > 0; o >>= 1) hm = fmaxf(hm, __shfl_xor(hm, o));
        if (l == 0) swm[wv] = hm;
        __syncthreads();
        if (threadIdx.x == 0) {
            float m = swm[0];
            for (int w = 1; w < 8; ++w) m = fmaxf(m, swm[w]);
            atomicMax((int*)hmax2, __float_as_int(m));      // non-negative: int order = float order
        }
    }
}

// The fused fp16 PPO epoch's operands from the fp32 weights, and its zeroed gradient
// accumulators, in one launch (bgx_ppo_epoch_prep; replaces a dozen torch casts, fills
// and slice copies per epoch): the packed W1 fragments of fp16(W1) (k_fc1_pack's layout),
// fp16(b1), W2h = fp16([action_head; value_head; 0]) [512][H], b2h, and zeros in gW1
// [H][208], gW2 [512][H], gb2 [512] and hmax2.  fp16 conversions round to nearest, as
// Tensor.half() does.
struct EpochPrep {
    const float *w1, *b1, *wa, *ba, *wv, *bv;
    int hidden, n_actions, T;
    uint4* w1pack;
    _Float16 *b1h, *w2h, *b2h;
    float *gw1, *gw2, *gb2, *hmax2;
    float* bound;        // [2][512]: |fp16(action row a)| and |fp16(action bias a)| (may be NULL)
    double* sums;        // the epoch's 3 fp64 loss sums, zeroed (may be NULL)
};
__global__ __launch_bounds__(256) void k_ppo_epoch_prep(EpochPrep a) {
    const int H = a.hidden, A = a.n_actions;
    if (a.bound) {                          // one wave per action row, lanes over its columns
        const int r = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
        if (r < A) {
            float s = 0.0f;
            for (int c = l; c < H; c += 64) {
                const float v = (float)(_Float16)a.wa[(size_t)r * H + c];
                s = fmaf(v, v, s);
            }
            #pragma unroll
            for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
            if (l == 0) {
                a.bound[r] = sqrtf(s);
                a.bound[512 + r] = fabsf((float)(_Float16)a.ba[r]);
            }
        }
    }
    const long long n0 = (long long)kKB1 * a.T * 64, n1 = n0 + H, n2 = n1 + 512LL * H, n3 = n2 + 512,
                    n4 = n3 + (long long)H * 208, n5 = n4 + 512LL * H, n6 = n5 + 512, n7 = n6 + 1;
    for (long long g = (long long)blockIdx.x * 256 + threadIdx.x; g < n7; g += (long long)gridDim.x * 256) {
        if (g < n0) {
            const int l = (int)(g & 63), t = (int)((g >> 6) % a.T), kb = (int)((g >> 6) / a.T);
            const int u = 32 * t + (l & 31);
            f16x8 v;
            #pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int src = kperm_src(kb, l >> 5, i);
                v[i] = (u < H && src >= 0) ? (_Float16)a.w1[(size_t)u * kIn + src] : (_Float16)0.0f;
            }
            a.w1pack[g] = __builtin_bit_cast(uint4, v);
        } else if (g < n1) {
            const int u = (int)(g - n0);
            a.b1h[u] = (_Float16)a.b1[u];
        } else if (g < n2) {
            const long long e = g - n1;
            const int r = (int)(e / H), c = (int)(e % H);
            a.w2h[e] = r < A ? (_Float16)a.wa[(size_t)r * H + c] : (r == A ? (_Float16)a.wv[c] : (_Float16)0.0f);
        } else if (g < n3) {
            const int r = (int)(g - n2);
            a.b2h[r] = r < A ? (_Float16)a.ba[r] : (r == A ? (_Float16)a.bv[0] : (_Float16)0.0f);
        } else if (g < n4) {
            a.gw1[g - n3] = 0.0f;
        } else if (g < n5) {
            a.gw2[g - n4] = 0.0f;
        } else if (g < n6) {
            a.gb2[g - n5] = 0.0f;
        } else if (a.hmax2) {
            a.hmax2[0] = 0.0f;
        }
    }
    if (a.sums && blockIdx.x == 0 && threadIdx.x < 3) a.sums[threadIdx.x] = 0.0;
}

__global__ void k_counter_add(uint32_t* ctr, uint32_t v) {
    if (threadIdx.x == 0) *ctr += v;
}

}  // namespace

extern "C" {

int bgx_policy_packed_size(int32_t hidden, int32_t n_actions) {
    if (hidden <= 0 || hidden > 128 || n_actions <= 0) return BGX_EINVAL;
    const int T = (hidden + 31) / 32, OT = (n_actions + 1 + 31) / 32;
    return kHdr + sz_w1q(T) + sz_b1p(T) + sz_w2q(T, OT) + sz_b2p(OT);
}

int bgx_policy_pack(const float* W1, const float* b1, const float* Wa, const float* ba, const float* wv, const float* bv,
                    int32_t hidden, int32_t n_actions, float* packed, void* stream) {
    const int total = bgx_policy_packed_size(hidden, n_actions);
    if (total < 0 || !W1 || !b1 || !Wa || !ba || !wv || !bv || !packed) return BGX_EINVAL;
    const int T = (hidden + 31) / 32, OT = (n_actions + 1 + 31) / 32;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_policy_scale, dim3(1), dim3(1024), 0, s, W1, Wa, ba, wv, hidden, n_actions, packed);
    const int work = kKB1 * T * 64 * 8 + T * 16 * 64 + OT * T * 2 * 64 * 8 + OT * 16 * 64;
    hipLaunchKernelGGL(k_policy_pack, dim3((work + 255) / 256), dim3(256), 0, s, W1, b1, Wa, ba, wv, bv, hidden,
                       n_actions, T, OT, packed);
    return hipGetLastError() == hipSuccess ? BGX_OK : BGX_EDEVICE;
}

#ifdef BGX_POLICY_STAMPS
extern "C" int bgx_debug_policy_stamps(unsigned long long* out, int32_t waves) {
    if (hipDeviceSynchronize() != hipSuccess) return BGX_EDEVICE;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pstamp), (size_t)(waves < kStampWaves ? waves : kStampWaves) * 48) != hipSuccess)
        return BGX_EDEVICE;
    static unsigned long long z[kStampWaves][6];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_pstamp), z, sizeof z) == hipSuccess ? BGX_OK : BGX_EDEVICE;
}
#endif

int bgx_policy_act_ctr(const uint8_t* records_dev, int32_t n, const float* packed, int32_t hidden, int32_t n_actions,
                       uint64_t seed, uint32_t step, const uint32_t* step_ctr, int32_t greedy, int32_t* act_out,
                       float* logp_out, float* value_out, float* logits_out, uint8_t* records_out, void* stream) {
    if (bgx_policy_packed_size(hidden, n_actions) < 0 || n < 0 || (n > 0 && (!records_dev || !packed || !act_out)))
        return BGX_EINVAL;
    if (n == 0) return BGX_OK;
    const int T = (hidden + 31) / 32, OT = (n_actions + 1 + 31) / 32;
    const int n_main = (n + 31) / 32;
    const dim3 grid(n_main), blk(64);
    const int n_wg = (n + 127) / 128;                  // MODE 0: 4-wave workgroups
    hipStream_t s = (hipStream_t)stream;
    const uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
    const bool plain = !greedy && !logits_out;
    // the masked-action tile skip (k_policy_act, MODE 0): 2 extra waves per kZWin rows for count-0 rows
    // (tests compare both paths in one process through bgx_debug_option)
    const bool skip = bgx_dbg_int("BGX_POLICY_SKIP", 1) != 0;
    // rows with more legal actions than this go to the extra workgroups too (their tiles split
    // four ways), so no main wave walks more than ceil(heavy / 32) action tiles (round 5)
    const int heavy = (int)bgx_dbg_int("BGX_POLICY_HEAVY", kHeavyDefault);
    const dim3 grid0(skip ? n_wg + 2 * ((n + kZWin - 1) / kZWin) : n_wg);
#define BGX_ACT(TT)                                                                                           \
    do {                                                                                                      \
        if (plain)                                                                                            \
            hipLaunchKernelGGL((k_policy_act<TT, 0>), grid0, dim3(256), 0, s, records_dev, n, packed, n_actions, OT, \
                               lo, hi, step, step_ctr, greedy, act_out, logp_out, value_out, logits_out,     \
                               records_out, skip ? (heavy > 0 ? heavy : 1) : 0);                             \
        else                                                                                                  \
            hipLaunchKernelGGL((k_policy_act<TT, -1>), grid, blk, 0, s, records_dev, n, packed, n_actions, OT,   \
                               lo, hi, step, step_ctr, greedy, act_out, logp_out, value_out, logits_out,     \
                               records_out, 0);                                                               \
    } while (0)
    switch (T) {
        case 1: BGX_ACT(1); break;
        case 2: BGX_ACT(2); break;
        case 3: BGX_ACT(3); break;
        default: BGX_ACT(4); break;
    }
#undef BGX_ACT
    return hipGetLastError() == hipSuccess ? BGX_OK : BGX_EDEVICE;
}

int bgx_policy_act_rec(const uint8_t* records_dev, int32_t n, const float* packed, int32_t hidden, int32_t n_actions,
                       uint64_t seed, uint32_t step, int32_t greedy, int32_t* act_out, float* logp_out,
                       float* value_out, float* logits_out, uint8_t* records_out, void* stream) {
    return bgx_policy_act_ctr(records_dev, n, packed, hidden, n_actions, seed, step, nullptr, greedy, act_out, logp_out,
                              value_out, logits_out, records_out, stream);
}

int bgx_counter_add(uint32_t* ctr_dev, uint32_t v, void* stream) {
    if (!ctr_dev) return BGX_EINVAL;
    hipLaunchKernelGGL(k_counter_add, dim3(1), dim3(64), 0, (hipStream_t)stream, ctr_dev, v);
    return hipGetLastError() == hipSuccess ? BGX_OK : BGX_EDEVICE;
}

int bgx_policy_act(const uint8_t* records_dev, int32_t n, const float* packed, int32_t hidden, int32_t n_actions,
                   uint64_t seed, uint32_t step, int32_t greedy, int32_t* act_out, float* logp_out, float* value_out,
                   float* logits_out, void* stream) {
    return bgx_policy_act_rec(records_dev, n, packed, hidden, n_actions, seed, step, greedy, act_out, logp_out,
                              value_out, logits_out, nullptr, stream);
}

int bgx_fc1_packed_size(int32_t hidden) {
    if (hidden <= 0 || hidden > 128 || hidden % 4) return BGX_EINVAL;
    return kKB1 * ((hidden + 31) / 32) * 64 * 16;
}

int bgx_fc1_pack(const void* w1h_dev, int32_t hidden, void* packed_dev, void* stream) {
    if (bgx_fc1_packed_size(hidden) < 0 || !w1h_dev || !packed_dev) return BGX_EINVAL;
    if ((uintptr_t)packed_dev % 16) return BGX_EINVAL;
    const int T = (hidden + 31) / 32, work = kKB1 * T * 64;
    hipLaunchKernelGGL(k_fc1_pack, dim3((work + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const _Float16*)w1h_dev, hidden, T, (uint4*)packed_dev);
    return hipGetLastError() == hipSuccess ? BGX_OK : BGX_EDEVICE;
}

int bgx_ppo_epoch_prep(const float* w1_dev, const float* b1_dev, const float* wa_dev, const float* ba_dev,
                       const float* wv_dev, const float* bv_dev, int32_t hidden, int32_t n_actions, void* w1pack_dev,
                       void* b1h_dev, void* w2h_dev, void* b2h_dev, float* gw1_dev, float* gw2_dev, float* gb2_dev,
                       float* hmax2_dev_or_null, float* bound_dev_or_null, double* sums_dev_or_null, void* stream) {
    if (bgx_fc1_packed_size(hidden) < 0 || n_actions <= 0 || n_actions >= 512) return BGX_EINVAL;
    if (!w1_dev || !b1_dev || !wa_dev || !ba_dev || !wv_dev || !bv_dev || !w1pack_dev || !b1h_dev || !w2h_dev ||
        !b2h_dev || !gw1_dev || !gw2_dev || !gb2_dev || (uintptr_t)w1pack_dev % 16)
        return BGX_EINVAL;
    EpochPrep a{w1_dev, b1_dev, wa_dev, ba_dev, wv_dev, bv_dev, hidden, n_actions, (hidden + 31) / 32,
                (uint4*)w1pack_dev, (_Float16*)b1h_dev, (_Float16*)w2h_dev, (_Float16*)b2h_dev, gw1_dev, gw2_dev,
                gb2_dev, hmax2_dev_or_null, bound_dev_or_null, sums_dev_or_null};
    hipLaunchKernelGGL(k_ppo_epoch_prep, dim3(512), dim3(256), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? BGX_OK : BGX_EDEVICE;
}

int bgx_fc1_records(const uint8_t* records_dev, int32_t n, const void* packed_dev, const void* b1h_dev,
                    int32_t hidden, void* h_dev, void* stream) {
    return bgx_fc1_records_ex(records_dev, n, packed_dev, b1h_dev, hidden, h_dev, nullptr, stream);
}

int bgx_fc1_records_ex(const uint8_t* records_dev, int32_t n, const void* packed_dev, const void* b1h_dev,
                       int32_t hidden, void* h_dev, float* hmax2_dev, void* stream) {
    if (bgx_fc1_packed_size(hidden) < 0 || n < 0 || (n > 0 && (!records_dev || !packed_dev || !b1h_dev || !h_dev)))
        return BGX_EINVAL;
    if (((uintptr_t)records_dev | (uintptr_t)packed_dev) % 16 || (uintptr_t)h_dev % 8) return BGX_EINVAL;
    if (n == 0) return BGX_OK;
    const int T = (hidden + 31) / 32;
    const int tiles8 = (n + 255) / 256;                 // 8 waves x 32 rows per workgroup and pass
    const dim3 grid(tiles8 < 512 ? tiles8 : 512), blk(512);
    hipStream_t s = (hipStream_t)stream;
    const uint4* w = (const uint4*)packed_dev;
    const _Float16* b = (const _Float16*)b1h_dev;
    _Float16* o = (_Float16*)h_dev;
    switch (T) {
        case 1: hipLaunchKernelGGL((k_fc1_rec<1>), grid, blk, 0, s, records_dev, n, w, b, hidden, o, hmax2_dev); break;
        case 2: hipLaunchKernelGGL((k_fc1_rec<2>), grid, blk, 0, s, records_dev, n, w, b, hidden, o, hmax2_dev); break;
        case 3: hipLaunchKernelGGL((k_fc1_rec<3>), grid, blk, 0, s, records_dev, n, w, b, hidden, o, hmax2_dev); break;
        default: hipLaunchKernelGGL((k_fc1_rec<4>), grid, blk, 0, s, records_dev, n, w, b, hidden, o, hmax2_dev); break;
    }
    return hipGetLastError() == hipSuccess ? BGX_OK : BGX_EDEVICE;
}

}  // extern "C"
