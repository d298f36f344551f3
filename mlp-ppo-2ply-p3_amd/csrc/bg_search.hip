// bg_search.hip — 1-ply greedy and 2-ply expectimax over the 21 dice rolls
//  with the MLP value head (policy_network.py:54-56,72-75) on MFMA.
//
// 2-ply, per root lane (board, mover, roll) with legal afterstates a_0..a_{n-1}:
//   Q(a) = sum_r p_r * min_{b in replies(a, r)} V(enc(b, opponent))       (leaf = a if no reply)
//   best = first argmax_a Q(a)
// Work item ("job") = (afterstate row, roll r): one wave enumerates the
// opponent's replies with the exact reference move generator (bg_core.h, LDS
// dedup + revisit memo), keeps the surviving afterstate KEYS in an LDS list,
// and evaluates them 32 at a time: features are generated on the fly from
// (afterstate bytes, key) and fed as the B operand of v_mfma_f32_32x32x2_f32
// (W1 . F^T), the value is a dot with the value head in registers, and the wave
// keeps the running minimum.  Leaves never touch HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "bg_engine.h"

using namespace bg;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kK1 = 99;            // 198 / 2 k-steps of 32x32x2
constexpr int kKeyCap = 512;       // LDS reply-key list per wave (8 KiB), flushed when full
constexpr int kSearchLog = 10;     // LDS dedup table (16 KiB)
constexpr int kSlowQueue = 1 << 20;

__constant__ float kOff15s[16] = {
    0.0f / 15.0f, 1.0f / 15.0f, 2.0f / 15.0f, 3.0f / 15.0f, 4.0f / 15.0f, 5.0f / 15.0f,
    6.0f / 15.0f, 7.0f / 15.0f, 8.0f / 15.0f, 9.0f / 15.0f, 10.0f / 15.0f, 11.0f / 15.0f,
    12.0f / 15.0f, 13.0f / 15.0f, 14.0f / 15.0f, 15.0f / 15.0f};
// get_all_dice_rolls_tensor (get_all_dice_rolls.py:5-34): (1,1),(1,2),...,(6,6)
__constant__ uint8_t kRoll0[21] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6};
__constant__ uint8_t kRoll1[21] = {1, 2, 3, 4, 5, 6, 2, 3, 4, 5, 6, 3, 4, 5, 6, 4, 5, 6, 5, 6, 6};

__device__ __forceinline__ int hid(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Value net packed for MFMA (bgx_value_pack): w1p [99][T][64], b1p [T][16][64],
// wvp [T][16][64] (= value_head.weight[32t + hid(r, l>>5)]), then bv.
struct VNet { const float* w1p; const float* b1p; const float* wvp; float bv; };

// Feature k of the board (root bytes `ab` in LDS) after player q moved to the
// afterstate with key (klo, khi, k3): q's counts come from the key nibbles, the
// other side's from ab minus the hit blots; one-hot = `cur`.
__device__ __forceinline__ float feat_key(const uint8_t* ab, uint64_t klo, uint32_t khi, uint32_t k3, int q, int cur,
                                          int k) {
    if (k >= 196) return (k == 196) == (cur == 0) ? 1.0f : 0.0f;
    const int P = k >= 98 ? 1 : 0;
    const int g = k - 98 * P;
    const uint32_t hits = k3 >> 8;
    if (g < 96) {
        const int pt = g >> 2, u = g & 3;
        int n;
        if (P == q) {
            const uint64_t w = pt < 16 ? klo : (uint64_t)khi;
            n = (int)((w >> (4 * (pt & 15))) & 15u);
        } else {
            n = (int)ab[P * 24 + pt] - (int)((hits >> pt) & 1u);
        }
        if (u < 3) return n > u ? 1.0f : 0.0f;
        return n >= 3 ? (float)(n - 3) * 0.5f : 0.0f;
    }
    if (g == 96) {
        const int bar = P == q ? (int)(k3 & 15u) : (int)ab[48 + P] + __builtin_popcount(hits);
        return (float)bar * 0.5f;
    }
    const int off = P == q ? (int)((k3 >> 4) & 15u) : (int)ab[50 + P];
    return kOff15s[off & 15];
}

// V for the 32 rows held by lanes (row j = lane & 31; both lane halves return it).
template <int T>
__device__ __forceinline__ float eval_rows(const VNet& vn, const uint8_t* ab, uint64_t klo, uint32_t khi, uint32_t k3,
                                           int q, int cur) {
    const int l = threadIdx.x & 63, h = l >> 5;
    f32x16 x1[T];
    #pragma unroll
    for (int t = 0; t < T; ++t)
        #pragma unroll
        for (int r = 0; r < 16; ++r) x1[t][r] = vn.b1p[(t * 16 + r) * 64 + l];
    for (int kk = 0; kk < kK1; ++kk) {
        const float b = feat_key(ab, klo, khi, k3, q, cur, 2 * kk + h);
        #pragma unroll
        for (int t = 0; t < T; ++t)
            x1[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(vn.w1p[(kk * T + t) * 64 + l], b, x1[t], 0, 0, 0);
    }
    float v = 0.0f;
    #pragma unroll
    for (int t = 0; t < T; ++t)
        #pragma unroll
        for (int r = 0; r < 16; ++r) v = fmaf(fmaxf(x1[t][r], 0.0f), vn.wvp[(t * 16 + r) * 64 + l], v);
    v += __shfl_xor(v, 32);
    return v + vn.bv;
}

__device__ __forceinline__ float wave_min(float v) {
    #pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}

// Sink for the reply enumeration: afterstate keys -> LDS list -> batched V -> min.
template <int T>
struct MinSink {
    uint4* klist;
    const uint8_t* ab;
    VNet vn;
    int q;
    float best;
    int evaluated;

    __device__ __forceinline__ void reset() { best = INFINITY; }

    __device__ __attribute__((noinline)) void flush(int n) {
        const int l = threadIdx.x & 63, j = l & 31;
        for (int base = 0; base < n; base += 32) {
            const uint4 k = klist[base + (j < n - base ? j : 0)];
            const float v = eval_rows<T>(vn, ab, (uint64_t)k.x | ((uint64_t)k.y << 32), k.z, k.w, q, q);
            best = fminf(best, wave_min(j < n - base ? v : INFINITY));
        }
        evaluated += n;
    }

    __device__ __forceinline__ void push(const Node& s, uint64_t, int idx) {
        const int slot = idx % kKeyCap;
        if ((threadIdx.x & 63) == 0) klist[slot] = make_uint4((uint32_t)s.lo, (uint32_t)(s.lo >> 32), s.hi, s.k3);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (slot == kKeyCap - 1) flush(kKeyCap);
    }

    // keys of the lanes in m (<= 64 of them < kKeyCap), list positions idx0, idx0+1, ...
    __device__ __forceinline__ void push_lanes(uint64_t m, const Node& t, uint64_t, int idx0) {
        const int pos = idx0 % kKeyCap, n = __popcll(m);
        const int r = lane_rank(m);
        const bool on = (m >> (threadIdx.x & 63)) & 1ull;
        const uint4 key = make_uint4((uint32_t)t.lo, (uint32_t)(t.lo >> 32), t.hi, t.k3);
        if (on && pos + r < kKeyCap) klist[pos + r] = key;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (pos + n >= kKeyCap) {
            flush(kKeyCap);
            if (on && pos + r >= kKeyCap) klist[pos + r - kKeyCap] = key;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }
    }
};

__device__ __forceinline__ uint64_t uload64(const uint64_t* p) {
    const uint64_t v = *p;
    // cast through uint32_t: the builtin returns int, and sign extension would
    // smear bit 31 (sub-move 2's valid bit) over sub-moves 3-4
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}

__device__ __forceinline__ Node apply_move(Node s, uint64_t m, int pl) {
    for (int i = 0; i < 4; ++i) {
        const uint32_t e = (uint32_t)(m >> (16 * i)) & 0xFFFFu;
        if (!(e & 0x8000u)) break;
        Sub sm; sm.src = (int)(e & 31u); sm.dst = (int)((e >> 5) & 31u); sm.hit = (int)((e >> 10) & 1u); sm.enc = e;
        s = apply(s, sm, pl);
    }
    return s;
}

struct SearchArgs {
    const int32_t* row_lane;     // [rows] root lane of each afterstate row
    const int32_t* lane_off;     // [B] first row of each lane
    const int64_t* rows_total;   // device scalar
    float* minv;                 // [rows][21]
    unsigned long long* leaves;  // device counter
    int32_t* slow_count;         // overflow queue
    int32_t* slow_queue;
};

// One (row, roll) job: opponent reply enumeration + leaf minimum.
template <int LOG, typename SlotPtr, int T>
__device__ __forceinline__ bool two_ply_job(const Args& A, const SearchArgs& S, const VNet& vn, int64_t job,
                                            SlotPtr tab, int cap_unique, uint4* memo, uint4* klist, uint8_t* ab) {
    const int64_t row = job / 21;
    const int r = (int)(job - row * 21);
    const int lane_g = S.row_lane[row];
    const int a = (int)(row - S.lane_off[lane_g]);
    const int l = threadIdx.x & 63;
    int bv = load_rec(A, lane_g);
    const int mover = rd(bv, R_CUR);
    const uint64_t m = uload64(A.moves + (size_t)lane_g * A.max_moves + a);
    uint32_t blocked;
    Node s = node_from_bytes(bv, mover, blocked);
    s = apply_move(s, m, mover);
    const int bva = bytes_from_node(bv, s, mover);      // the afterstate a, one byte per lane
    if (l < 64) ab[l] = (uint8_t)bva;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int q = 1 - mover;
    // clear tables
    for (int i = l; i < (1 << LOG); i += 64) tab[i] = make_uint4(0u, 0u, 0u, 0u);
    const int r0 = kRoll0[r], r1 = kRoll1[r];
    if (r0 == r1)
        for (int i = l; i < kMemoSlots; i += 64) memo[i] = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    Gen<LOG, SlotPtr, MinSink<T>> g;
    g.tab = tab; g.pl = q; g.cap_unique = cap_unique;
    g.memo2 = r0 == r1 ? memo : nullptr;
    g.memo3 = r0 == r1 ? memo + (1 << kLogMemo2) : nullptr;
    g.sink.klist = klist; g.sink.ab = ab; g.sink.vn = vn; g.sink.q = q; g.sink.best = INFINITY;
    g.sink.evaluated = 0;
    uint32_t blk;
    const Node sq = node_from_bytes(bva, q, blk);
    g.blocked = blk;
    g.run(sq, r0, r1);
    if (g.ovf) return false;
    const int rem = g.count % kKeyCap;
    if (g.count == 0) {                 // no reply: the opponent passes, the leaf is a itself
        if (l == 0) klist[0] = make_uint4((uint32_t)sq.lo, (uint32_t)(sq.lo >> 32), sq.hi, sq.k3);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        g.sink.flush(1);
    } else if (rem) {
        g.sink.flush(rem);
    }
    if (l == 0) {
        S.minv[row * 21 + r] = g.sink.best;
        atomicAdd(S.leaves, (unsigned long long)(g.count ? g.count : 1));
    }
    return true;
}

template <int T>
__global__ __launch_bounds__(64) void k_two_ply(Args A, SearchArgs S, VNet vn) {
    __shared__ uint4 tab[1 << kSearchLog];
    __shared__ uint4 memo[kMemoSlots];
    __shared__ uint4 klist[kKeyCap];
    __shared__ uint8_t ab[64];
    const int64_t njobs = (int64_t)(*S.rows_total) * 21;
    for (int64_t job = blockIdx.x; job < njobs; job += gridDim.x) {
        if (!two_ply_job<kSearchLog, uint4*, T>(A, S, vn, job, tab, cap_fast<kSearchLog>(), memo, klist, ab)) {
            if ((threadIdx.x & 63) == 0) {
                const int qi = atomicAdd(S.slow_count, 1);
                if (qi < kSlowQueue) S.slow_queue[qi] = (int32_t)job;
                else atomicOr(A.err, 2);
            }
        }
    }
}

template <int T>
__global__ __launch_bounds__(64) void k_two_ply_slow(Args A, SearchArgs S, VNet vn, uint4* tables) {
    __shared__ uint4 memo[kMemoSlots];
    __shared__ uint4 klist[kKeyCap];
    __shared__ uint8_t ab[64];
    uint4* tab = tables + ((size_t)blockIdx.x << kLogSlotsSlow);
    const int n = min(*S.slow_count, kSlowQueue);
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t job = S.slow_queue[i];
        if (!two_ply_job<kLogSlotsSlow, uint4*, T>(A, S, vn, job, tab, kCapSlow, memo, klist, ab))
            if ((threadIdx.x & 63) == 0) atomicOr(A.err, 1);
    }
}

// Exclusive scan of the lanes' legal-move counts (one workgroup).
__global__ __launch_bounds__(1024) void k_scan(Args A, int32_t* lane_off, int64_t* total) {
    __shared__ int64_t part[1024];
    const int t = threadIdx.x;
    const int per = (A.B + 1023) / 1024;
    const int lo = t * per, hi = min(A.B, lo + per);
    int64_t sum = 0;
    for (int i = lo; i < hi; ++i) {
        const uint8_t* rr = A.lanes + (size_t)i * 64;
        sum += (int)rr[R_NM0] | ((int)rr[R_NM1] << 8);
    }
    part[t] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int64_t v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int64_t run = part[t] - sum;
    for (int i = lo; i < hi; ++i) {
        lane_off[i] = (int32_t)run;
        const uint8_t* rr = A.lanes + (size_t)i * 64;
        run += (int)rr[R_NM0] | ((int)rr[R_NM1] << 8);
    }
    if (t == 1023) *total = part[1023];
}

__global__ void k_expand(Args A, const int32_t* lane_off, int32_t* row_lane) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.B) return;
    const uint8_t* rr = A.lanes + (size_t)i * 64;
    const int n = (int)rr[R_NM0] | ((int)rr[R_NM1] << 8);
    for (int a = 0; a < n; ++a) row_lane[lane_off[i] + a] = i;
}

// Q(a) = sum_r p_r minv[a][r] (fp32, r in roll order), first argmax.
__global__ void k_two_ply_reduce(Args A, const int32_t* lane_off, const float* minv, int32_t* best, float* bestq,
                                 float* qout) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.B) return;
    const uint8_t* rr = A.lanes + (size_t)i * 64;
    const int n = (int)rr[R_NM0] | ((int)rr[R_NM1] << 8);
    float bq = -INFINITY;
    int ba = 0;
    for (int a = 0; a < n; ++a) {
        const float* mv = minv + ((size_t)lane_off[i] + a) * 21;
        float q = 0.0f;
        for (int r = 0; r < 21; ++r) q = fmaf(kRoll0[r] == kRoll1[r] ? 1.0f / 36.0f : 2.0f / 36.0f, mv[r], q);
        if (qout) qout[(size_t)i * A.max_moves + a] = q;
        if (q > bq) { bq = q; ba = a; }
    }
    best[i] = ba;
    if (bestq) bestq[i] = n ? bq : 0.0f;
}

// 1-ply: every lane's afterstates a (mover's one-hot), first argmax V(a).
template <int T>
__global__ __launch_bounds__(64) void k_one_ply(Args A, VNet vn, int32_t* best, float* bestv, float* vout) {
    __shared__ uint8_t ab[64];
    const int gi = blockIdx.x;
    const int l = threadIdx.x & 63, j = l & 31;
    const int bv = load_rec(A, gi);
    const int mover = rd(bv, R_CUR);
    const int n = rd(bv, R_NM0) | (rd(bv, R_NM1) << 8);
    ab[l] = (uint8_t)bv;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    uint32_t blocked;
    const Node s0 = node_from_bytes(bv, mover, blocked);
    float bvv = -INFINITY;
    int ba = 0;
    for (int base = 0; base < n; base += 32) {
        const int a = base + (j < n - base ? j : 0);
        const Node s = apply_move(s0, A.moves[(size_t)gi * A.max_moves + a], mover);   // per-lane move
        const float v = eval_rows<T>(vn, ab, s.lo, s.hi, s.k3, mover, mover);
        if (vout && l < 32 && base + j < n) vout[(size_t)gi * A.max_moves + base + j] = v;
        float key = j < n - base ? v : -INFINITY;
        int idx = base + j;
        #pragma unroll
        for (int o = 16; o >= 1; o >>= 1) {     // first argmax over the 32 rows (lanes 0..31 == 32..63)
            const float k2 = __shfl_xor(key, o);
            const int i2 = __shfl_xor(idx, o);
            if (k2 > key || (k2 == key && i2 < idx)) { key = k2; idx = i2; }
        }
        if (key > bvv) { bvv = key; ba = idx; }
    }
    if (l == 0) { best[gi] = ba; if (bestv) bestv[gi] = n ? bvv : 0.0f; }
}

__global__ void k_value_pack(const float* W1, const float* b1, const float* wv, const float* bv, int H, int T,
                             float* w1p, float* b1p, float* wvp, float* bvp) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int n1 = kK1 * T * 64, nb = T * 16 * 64;
    if (tid < n1) {
        const int l = tid % 64, t = (tid / 64) % T, kk = tid / (64 * T);
        const int hrow = 32 * t + (l & 31);
        w1p[tid] = hrow < H ? W1[(size_t)hrow * 198 + 2 * kk + (l >> 5)] : 0.0f;
    } else if (tid < n1 + 2 * nb) {
        const int i = (tid - n1) % nb;
        const bool isb = tid < n1 + nb;
        const int l = i % 64, r = (i / 64) % 16, t = i / (64 * 16);
        const int hrow = 32 * t + hid(r, l >> 5);
        if (isb) b1p[i] = hrow < H ? b1[hrow] : 0.0f;
        else wvp[i] = hrow < H ? wv[hrow] : 0.0f;
    } else if (tid == n1 + 2 * nb) {
        bvp[0] = bv[0];
    }
}

}  // namespace

extern int bgx_internal_fail(hipError_t e);
#define SCK(x) do { hipError_t _e = (x); if (_e != hipSuccess) return bgx_internal_fail(_e); } while (0)

static int value_tiles(int H) { return H <= 32 ? 1 : 2; }

extern "C" {

int bgx_value_packed_size(int32_t hidden) {
    if (hidden <= 0 || hidden > 64) return BGX_EINVAL;
    const int T = value_tiles(hidden);
    return kK1 * T * 64 + 2 * T * 16 * 64 + 4;
}

int bgx_value_pack(const float* W1, const float* b1, const float* wv, const float* bv, int32_t hidden, float* packed,
                   void* stream) {
    const int total = bgx_value_packed_size(hidden);
    if (total < 0 || !W1 || !b1 || !wv || !bv || !packed) return BGX_EINVAL;
    const int T = value_tiles(hidden);
    float* w1p = packed;
    float* b1p = w1p + kK1 * T * 64;
    float* wvp = b1p + T * 16 * 64;
    float* bvp = wvp + T * 16 * 64;
    hipLaunchKernelGGL(k_value_pack, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, W1, b1, wv, bv, hidden,
                       T, w1p, b1p, wvp, bvp);
    SCK(hipGetLastError());
    return BGX_OK;
}

static VNet make_vnet(const float* packed, int hidden, float bv_host) {
    const int T = value_tiles(hidden);
    VNet v;
    v.w1p = packed;
    v.b1p = v.w1p + kK1 * T * 64;
    v.wvp = v.b1p + T * 16 * 64;
    v.bv = bv_host;
    return v;
}

int bgx_one_ply(bgx_engine* e, const float* vpacked, int32_t hidden, float value_bias, int32_t* best_out,
                float* bestv_out, float* values_out, void* stream) {
    if (!e || !vpacked || !best_out || bgx_value_packed_size(hidden) < 0) return BGX_EINVAL;
    SCK(hipSetDevice(e->device));
    const VNet vn = make_vnet(vpacked, hidden, value_bias);
    hipStream_t s = (hipStream_t)stream;
    if (value_tiles(hidden) == 1)
        hipLaunchKernelGGL(k_one_ply<1>, dim3(e->a.B), dim3(64), 0, s, e->a, vn, best_out, bestv_out, values_out);
    else
        hipLaunchKernelGGL(k_one_ply<2>, dim3(e->a.B), dim3(64), 0, s, e->a, vn, best_out, bestv_out, values_out);
    SCK(hipGetLastError());
    return BGX_OK;
}

int bgx_two_ply(bgx_engine* e, const float* vpacked, int32_t hidden, float value_bias, int32_t* best_out,
                float* bestq_out, float* q_out, uint64_t* stats_host, void* stream) {
    if (!e || !vpacked || !best_out || bgx_value_packed_size(hidden) < 0) return BGX_EINVAL;
    SCK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    Args& A = e->a;
    const size_t B = (size_t)A.B;
    // workspace: [lane_off B i32][rows_total i64][leaves u64][slow_count i32 x4][slow_queue][row_lane][minv]
    const size_t head = B * 4 + 64 + (size_t)kSlowQueue * 4;
    if (e->search_ws_bytes < head) {
        if (e->search_ws) SCK(hipFree(e->search_ws));
        e->search_ws = nullptr; e->search_ws_bytes = 0;
        SCK(hipMalloc(&e->search_ws, head));
        e->search_ws_bytes = head;
    }
    char* ws = (char*)e->search_ws;
    int32_t* lane_off = (int32_t*)ws;
    int64_t* rows_total = (int64_t*)(ws + B * 4);
    unsigned long long* leaves = (unsigned long long*)(ws + B * 4 + 8);
    int32_t* slow_count = (int32_t*)(ws + B * 4 + 16);
    SCK(hipMemsetAsync(ws + B * 4, 0, 64, s));
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, A, lane_off, rows_total);
    SCK(hipGetLastError());
    int64_t rows = 0;
    SCK(hipMemcpyAsync(&rows, rows_total, 8, hipMemcpyDeviceToHost, s));
    SCK(hipStreamSynchronize(s));
    const size_t need = head + (size_t)rows * 4 + (size_t)rows * 21 * 4 + 256;
    if (e->search_ws_bytes < need) {
        // grow (keeps nothing: everything below is recomputed)
        void* nw = nullptr;
        SCK(hipMalloc(&nw, need + need / 4));
        SCK(hipMemcpyAsync(nw, e->search_ws, head, hipMemcpyDeviceToDevice, s));
        SCK(hipStreamSynchronize(s));
        SCK(hipFree(e->search_ws));
        e->search_ws = nw;
        e->search_ws_bytes = need + need / 4;
        ws = (char*)nw;
        lane_off = (int32_t*)ws;
        rows_total = (int64_t*)(ws + B * 4);
        leaves = (unsigned long long*)(ws + B * 4 + 8);
        slow_count = (int32_t*)(ws + B * 4 + 16);
    }
    int32_t* slow_queue = (int32_t*)(ws + B * 4 + 64);
    int32_t* row_lane = (int32_t*)(ws + head);
    float* minv = (float*)(ws + head + (((size_t)rows * 4 + 255) & ~(size_t)255));
    hipLaunchKernelGGL(k_expand, dim3((A.B + 255) / 256), dim3(256), 0, s, A, lane_off, row_lane);
    SearchArgs S{row_lane, lane_off, rows_total, minv, leaves, slow_count, slow_queue};
    const VNet vn = make_vnet(vpacked, hidden, value_bias);
    const int64_t njobs = rows * 21;
    const int grid = (int)(njobs < 8192 ? (njobs > 0 ? njobs : 1) : 8192);
    if (value_tiles(hidden) == 1) {
        hipLaunchKernelGGL(k_two_ply<1>, dim3(grid), dim3(64), 0, s, A, S, vn);
        hipLaunchKernelGGL(k_two_ply_slow<1>, dim3(e->slow_waves), dim3(64), 0, s, A, S, vn, e->slow_tables);
    } else {
        hipLaunchKernelGGL(k_two_ply<2>, dim3(grid), dim3(64), 0, s, A, S, vn);
        hipLaunchKernelGGL(k_two_ply_slow<2>, dim3(e->slow_waves), dim3(64), 0, s, A, S, vn, e->slow_tables);
    }
    SCK(hipGetLastError());
    hipLaunchKernelGGL(k_two_ply_reduce, dim3((A.B + 255) / 256), dim3(256), 0, s, A, lane_off, minv, best_out,
                       bestq_out, q_out);
    SCK(hipGetLastError());
    if (stats_host) {
        unsigned long long lv = 0;
        SCK(hipMemcpyAsync(&lv, leaves, 8, hipMemcpyDeviceToHost, s));
        SCK(hipStreamSynchronize(s));
        stats_host[0] = lv;
        stats_host[1] = (uint64_t)njobs;
        stats_host[2] = (uint64_t)rows;
    }
    return BGX_OK;
}

}  // extern "C"
