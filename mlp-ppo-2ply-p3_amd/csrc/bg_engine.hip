// bg_engine.hip — MI355X (gfx950) self-play engine: lane records in HBM, one
// wavefront per game, move enumeration + board apply + dice + encoder as HIP
// kernels, exported through the C ABI declared in include/bgx.h.
//
// Data layout in HBM (per engine, batch B, max_moves M):
//   lanes   [B][64]  u8   board52 | cur | roll[2] | game_over | match_over |
//                         score[2] | need | n_moves(i16) | flags | pad
//   moves   [B][M]   u64  current legal-move list (first M of the filtered list)
//   n_total [B]      i32  untruncated count
//   mt      [B][640] u32  per-lane numpy-legacy MT19937 state (+ index at [624])
//   ctr     [B]      u64  per-lane Philox draw counters
// Kernels are launched one 64-thread workgroup (= one wave) per game.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <algorithm>
#include <cmath>
#include <mutex>
#include <string>
#include <vector>

#include "bg_engine.h"
#include "bg_debug.h"
#include <map>

using namespace bg;

namespace {

constexpr int kMaxRegions = BGX_MAX_COPY_REGIONS;
using namespace bg;

// -------------------------------------------------------------- kernels --
// PHASE 0: apply + advance fused (per-lane dice); 1: apply only; 2: advance only.
// One lane's step: apply (PHASE 0/1), roll + movegen (PHASE 0/2), record, next
// dispatch class.
template <int PHASE, int LOG, int MEMO, bool NO_DOUBLES = false>
__device__ __forceinline__ void step_lane(const Args& A, int gi, uint4* tab, uint4* memo, const int32_t* actions,
                                          float* obs, float* reward, uint8_t* done, int32_t* info) {
    const uint64_t t0 = A.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    // issue the independent loads together (record, action, dice counter)
    int bv = load_rec(A, gi);
    const int act = PHASE != 2 ? (int)ufl((uint32_t)actions[gi]) : 0;
    uint64_t ctr = A.dice_mode == BGX_DICE_PHILOX ? A.ctr[gi] : 0;
    if (PHASE != 2) bv = apply_lane(bv, gi, act, A, reward, done, info);
    if (PHASE != 1) {
        bv = advance_lane<LOG, MEMO == 2 ? 2 : 0, NO_DOUBLES>(bv, gi, A, tab, memo, &ctr);
        if (obs) write_obs(bv, obs + (size_t)gi * 198);
    }
    store_rec(A, gi, bv);
    if (PHASE == 0 && A.cls) {
        uint32_t cache;
        const int c = predict_class(bv, ctr, A, gi, cache);
        if (lane_id() == 0) {
            A.cls[gi] = (uint8_t)c;
            if (cache) A.ctr[gi] = (ctr & kCtrMask) | ((uint64_t)cache << 48);
        }
    }
    if (A.stamps && lane_id() == 0) {
        A.stamps[2 * gi] = t0;
        A.stamps[2 * gi + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// `base` offsets blockIdx into the dispatch order.  MEMO: 0 = no revisit memo,
// 1 = separate memo tables (10 KB of LDS), 2 = memo inside the dedup table.
// NO_DOUBLES: doubles rolls are deferred to the overflow tiers (light launch).
template <int PHASE, int LOG, int MEMO = 1, bool NO_DOUBLES = false, int WPE = 1>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_step(Args A, const int32_t* actions, float* obs, float* reward, uint8_t* done,
                                             int32_t* info, int base) {
    __shared__ uint4 tab[1 << LOG];
    __shared__ uint4 memo_[MEMO == 1 ? kMemoSlots : 1];
    uint4* memo = MEMO == 1 ? memo_ : MEMO == 2 ? tab : nullptr;
    const int bi = (int)blockIdx.x + base;
    const int gi = A.perm ? (int)ufl((uint32_t)A.perm[bi]) : lane_of_block(A, bi);
    step_lane<PHASE, LOG, MEMO, NO_DOUBLES>(A, gi, tab, memo, actions, obs, reward, done, info);
}

template <int LOG>
__global__ __launch_bounds__(64) void k_reset(Args A, const uint8_t* lane_mask, float* obs, int mark_only) {
    __shared__ uint4 tab[1 << LOG];
    __shared__ uint4 memo[kMemoSlots];
    const int gi = blockIdx.x;
    int bv = load_rec(A, gi);
    uint64_t ctr = A.dice_mode == BGX_DICE_PHILOX ? A.ctr[gi] : 0;
    const bool sel = lane_mask == nullptr || ufl(lane_mask[gi]) != 0u;
    if (sel) bv = wr(bv, R_NEED, NEED_RESET);
    if (!mark_only) {
        bv = advance_lane<LOG>(bv, gi, A, tab, memo, &ctr);
        if (obs) write_obs(bv, obs + (size_t)gi * 198);
        if (A.cls) {
            uint32_t cache;
            const int c = predict_class(bv, ctr, A, gi, cache);
            if (lane_id() == 0) {
                A.cls[gi] = (uint8_t)c;
                if (cache) A.ctr[gi] = (ctr & kCtrMask) | ((uint64_t)cache << 48);
            }
        }
    }
    store_rec(A, gi, bv);
}

// Next dispatch order = lanes grouped by predicted class (class 0 first), in
// lane order within a class: a two-pass counting sort over blocks of 1024
// lanes.  perm is a full permutation of 0..B-1 whatever cls holds.
//
// XCD-aware form (B % 128 == 0): the lanes are split into 8 sub-lists by
// x = (lane >> 4) & 7 (runs of 16 lanes), each sub-list is class-sorted on its
// own, and position 8k + x holds the k-th lane of sub-list x.  Blocks b and
// b + 8 of a launch run on one XCD (round-robin placement; the launch bases are
// multiples of 8), so every 16-lane run -- one 64-B line of the reward / action
// / n_total arrays, one 128-B line of the Philox counters, 8 lane records -- is
// stepped by ONE XCD per launch and its partial-line loads and stores meet in
// that XCD's L2 instead of crossing all eight.  The 8 sub-lists have nearly the
// same class mix, so the interleave keeps the heaviest-first order.
constexpr int kXcd = 8, kRun = 16;
__device__ __forceinline__ int order_class(const uint8_t* cls, int i, int B) {
    return i < B ? min((int)cls[i], kClasses - 1) : kClasses;     // kClasses = padding, never written
}

// pass 1: cnt[b][x][c] = lanes of class c in sub-list x of block b (x = 0 when !xcd)
__global__ __launch_bounds__(1024) void k_order_count(const uint8_t* cls, int32_t* cnt, int B, int32_t* zero_next,
                                                      int xcd) {
    __shared__ int sc[kXcd][kClasses];
    const int t = threadIdx.x, i = blockIdx.x * 1024 + t, w = t >> 6;
    if (blockIdx.x == 0 && t < 4) zero_next[t] = 0;     // the next step's overflow counters
    if (t < kXcd * kClasses) sc[t / kClasses][t % kClasses] = 0;
    __syncthreads();
    const int c = order_class(cls, i, B);
    #pragma unroll
    for (int k = 0; k < kClasses; ++k) {
        const uint64_t m = __ballot(c == k);
        if (xcd) {
            // the wave's four 16-lane runs belong to sub-lists (4w + s) & 7
            if ((t & 63) < 4) {
                const int s = t & 3;
                const int n = __popcll(m & (0xFFFFull << (16 * s)));
                if (n) atomicAdd(&sc[(4 * w + s) & 7][k], n);
            }
        } else if ((t & 63) == 0 && m) {
            atomicAdd(&sc[0][k], __popcll(m));
        }
    }
    __syncthreads();
    if (t < kXcd * kClasses) cnt[blockIdx.x * kXcd * kClasses + t] = sc[t / kClasses][t % kClasses];
}

// pass 2: position (within the lane's sub-list) = (lanes of lower classes) +
// (class-c lanes of earlier blocks) + (class-c lanes earlier in this block)
__global__ __launch_bounds__(1024) void k_order_scatter(const uint8_t* cls, const int32_t* cnt, int32_t* perm, int B,
                                                        int nblk, int xcd) {
    constexpr int NC = kXcd * kClasses;
    __shared__ int tot[NC], pre[NC], wsum[16][4][kClasses];
    const int t = threadIdx.x, b = blockIdx.x, w = t >> 6, l = t & 63;
    if (t < NC) { tot[t] = 0; pre[t] = 0; }
    __syncthreads();
    // thread t < NC sums counter t over the blocks (40 counters, <= B/1024 blocks)
    if (t < NC) {
        int a_tot = 0, a_pre = 0;
        for (int j = 0; j < nblk; ++j) {
            const int v = cnt[j * NC + t];
            a_tot += v;
            a_pre += j < b ? v : 0;
        }
        tot[t] = a_tot;
        pre[t] = a_pre;
    }
    const int i = b * 1024 + t;
    const int c = order_class(cls, i, B);
    const int s = xcd ? (l >> 4) : 0;                 // the lane's 16-lane run within the wave
    const uint64_t seg = xcd ? (0xFFFFull << (16 * s)) : ~0ull;
    int rank = 0;
    #pragma unroll
    for (int k = 0; k < kClasses; ++k) {
        const uint64_t m = __ballot(c == k);
        if (c == k) rank = __popcll(m & seg & ((1ull << l) - 1ull));
        if (l < 4) wsum[w][l][k] = __popcll(m & (xcd ? (0xFFFFull << (16 * l)) : (l == 0 ? ~0ull : 0ull)));
    }
    __syncthreads();
    if (c < kClasses) {
        const int x = xcd ? ((4 * w + s) & 7) : 0;
        int pos = pre[x * kClasses + c] + rank;
        for (int k = 0; k < c; ++k) pos += tot[x * kClasses + k];
        // earlier waves of this block holding runs of the same sub-list: w' = w (mod 2)
        for (int v = xcd ? (w & 1) : 0; v < w; v += xcd ? 2 : 1) pos += wsum[v][s][c];
        perm[xcd ? pos * kXcd + x : pos] = i;
    }
}

// SHARED dice: one wave draws every lane's dice from ONE MT stream in lane order
// (VectorizedBackgammonEnv: all envs call np.random.randint on the global state).
__global__ __launch_bounds__(64) void k_shared_dice(Args A) {
    __shared__ uint32_t sh[640];
    Rng rng;
    rng.init_mt(A.mt, sh);
    for (int base = 0; base < A.B; base += 64) {
        const int j = base + lane_id();
        const int needv = j < A.B ? (int)A.lanes[(size_t)j * 64 + R_NEED] : 0;
        const int cnt = A.B - base < 64 ? A.B - base : 64;
        for (int t = 0; t < cnt; ++t) {
            const int need = __builtin_amdgcn_readlane(needv, t);
            if (need == NEED_NONE) continue;
            int r0, r1, starter = 0;
            if (need == NEED_RESET) {
                int a, b;
                do { a = rng.die(); b = rng.die(); } while (a == b);
                starter = a < b ? 1 : 0;
                do { r0 = rng.die(); r1 = rng.die(); } while (r0 == r1);
            } else {
                r0 = rng.die(); r1 = rng.die();
            }
            if (lane_id() == 0) {
                uint8_t* sr = A.shared_rolls + (size_t)(base + t) * 4;
                sr[0] = (uint8_t)r0; sr[1] = (uint8_t)r1; sr[2] = (uint8_t)starter;
            }
        }
    }
    rng.finish(nullptr);
}

// Standalone get_all_possible_moves on arbitrary boards.
template <int LOG>
__global__ __launch_bounds__(64) void k_movegen(const int8_t* boards, const uint8_t* players, const uint8_t* dice,
                                                int n, int cap, int16_t* nmoves, int32_t* ntotal, uint64_t* moves,
                                                int32_t* ovf_count, int32_t* ovf_queue, int cap_unique) {
    __shared__ uint4 tab[1 << LOG];
    __shared__ uint4 memo[kMemoSlots];
    const int gi = blockIdx.x;
    const int l = lane_id();
    const int bv = l < 52 ? (int)boards[(size_t)gi * 52 + l] : 0;
    const int pl = (int)ufl(players[gi]);
    const int r0 = (int)ufl(dice[2 * gi]), r1 = (int)ufl(dice[2 * gi + 1]);
    int total;
    bool ovf;
    int nm = run_movegen<LOG>(bv, pl, r0, r1, moves + (size_t)gi * cap, cap, tab, cap_unique, &total, &ovf, memo);
    if (ovf) {
        if (l == 0) { const int q = atomicAdd(ovf_count, 1); ovf_queue[q] = gi; }
        nm = 0; total = 0;
    }
    if (l == 0) { nmoves[gi] = (int16_t)nm; if (ntotal) ntotal[gi] = total; }
}

// Overflow tiers for positions whose dedup set outgrew the main LDS table
// (cap 7/8 of 2^LOG slots), fed by the overflow queue.  Tier 1: the same code with a
// 4,096-slot (64 KiB) LDS table; a position with more distinct afterstates (> 3,584)
// runs again in the same wave on tier 2, a 131,072-slot table in HBM that is the
// workgroup's own (grid = kSlowWaves tables).  Every position stays exact.  Round 6:
// one launch of kSlowWaves workgroups for both tiers (was 256 tier-1 workgroups, then a
// tier-2 launch fed by a second queue): the queue is empty or short on almost every
// step, so the launch is mostly its own cost.  SRC 0 = engine lanes, 1 = standalone arrays.
constexpr int kLogMid = 12;

template <int SRC>
__global__ __launch_bounds__(64) void k_movegen_over(Args A, const int8_t* boards, const uint8_t* players,
                                                     const uint8_t* dice, int cap, int16_t* nmoves, int32_t* ntotal,
                                                     uint64_t* moves, uint4* tables) {
    __shared__ uint4 memo[kMemoSlots];
    __shared__ uint4 lds_tab[1 << kLogMid];
    uint4* slow = tables + ((size_t)blockIdx.x << kLogSlotsSlow);
    const int count = (int)ufl((uint32_t)A.ovf_count[0]);
    for (int q = blockIdx.x; q < count; q += gridDim.x) {
        const int gi = (int)ufl((uint32_t)A.ovf_queue[q]);
        const int l = lane_id();
        int bv, pl, r0, r1;
        if (SRC == 0) {
            bv = load_rec(A, gi); pl = rd(bv, R_CUR); r0 = rd(bv, R_ROLL0); r1 = rd(bv, R_ROLL1);
        } else {
            bv = l < 52 ? (int)boards[(size_t)gi * 52 + l] : 0;
            pl = (int)ufl(players[gi]); r0 = (int)ufl(dice[2 * gi]); r1 = (int)ufl(dice[2 * gi + 1]);
        }
        uint64_t* out = SRC == 0 ? A.moves + (size_t)gi * A.max_moves : moves + (size_t)gi * cap;
        const int c = SRC == 0 ? A.max_moves : cap;
        int total;
        bool ovf;
        int nm = run_movegen<kLogMid>(bv, pl, r0, r1, out, c, lds_tab, A.cap_mid, &total, &ovf, memo);
        if (ovf) nm = run_movegen<kLogSlotsSlow>(bv, pl, r0, r1, out, c, slow, kCapSlow, &total, &ovf, memo);
        if (ovf) {
            if (l == 0) atomicOr(A.err, 1);
            nm = 0; total = 0;
        }
        if (SRC == 0) {
            bv = wr(bv, R_NM0, nm & 0xFF);
            bv = wr(bv, R_NM1, (nm >> 8) & 0xFF);
            bv = wr(bv, R_FLAGS, rd(bv, R_FLAGS) & ~1);
            store_rec(A, gi, bv);
            if (l == 0) A.n_total[gi] = total;
        } else if (l == 0) {
            nmoves[gi] = (int16_t)nm;
            if (ntotal) ntotal[gi] = total;
        }
    }
}

__global__ __launch_bounds__(64) void k_encode(const int8_t* boards, const uint8_t* players, int n, float* out) {
    const int gi = blockIdx.x;
    const int l = lane_id();
    const int bv = l < 52 ? (int)boards[(size_t)gi * 52 + l] : 0;
    const int cur = (int)ufl(players[gi]);
    float* row = out + (size_t)gi * 198;
    #pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int f = l + 64 * t;
        const float v = feature_at(bv, f < 198 ? f : 197, cur);
        if (f < 198) row[f] = v;
    }
}

// The 198 features of n 64-byte lane records (the rollout's stored records), as
// T = float or _Float16 (fp16: the rounding of the fp32 features that autocast's
// cast applies, ppo_agent.py:274), feature_at's encoding (immutable_board.py:171-212).
// A 256-thread block encodes 64 consecutive records into an LDS image of their
// contiguous output (64 x 198 T): one wave per record, lane l < 48 holding byte
// l = the count of point l % 24 of player l / 24 (its 4 units at 98 (l / 24) +
// 4 (l % 24)), lanes 48 / 49 (bar, off) of P1 / P2, lane 50 the one-hot; then the
// block copies the image out with 16-byte stores (coalesced, whole lines).
template <typename T>
__device__ __forceinline__ void lds_pair(T* o, float a, float b) {
    if (sizeof(T) == 2) {
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        h2 v; v[0] = (_Float16)a; v[1] = (_Float16)b;
        *(h2*)o = v;
    } else {
        *(float2*)o = make_float2(a, b);
    }
}

template <typename T, int W>
__global__ __launch_bounds__(256) void k_encode_rec(const uint8_t* __restrict__ records, int n, T* __restrict__ out) {
    static_assert(W >= 198 && W % 2 == 0 && (W - 198) / 2 <= 13, "row width: 198 features + up to 26 zero columns");
    constexpr int kRows = 64, kImg = kRows * W * (int)sizeof(T);          // bytes
    __shared__ __attribute__((aligned(16))) uint8_t img[kImg];
    T* im = (T*)img;
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int l2 = l == 48 ? 50 : (l == 49 ? 51 : 52);      // off1 / off2 / mover byte
    for (int r0 = blockIdx.x * kRows; r0 < n; r0 += gridDim.x * kRows) {
        const int nr = min(kRows, n - r0);
        int b[16], b2[16];
        #pragma unroll
        for (int k = 0; k < 16; ++k) {                      // this wave's 16 records, loads in flight
            const int r = r0 + w + 4 * k;
            b[k] = r < n ? records[(size_t)r * 64 + l] : 0;
            b2[k] = r < n ? records[(size_t)r * 64 + l2] : 0;
        }
        __syncthreads();                                    // the previous image is copied out
        #pragma unroll
        for (int k = 0; k < 16; ++k) {
            T* o = im + (w + 4 * k) * W;
            const int v = b[k], v2 = b2[k];
            if (l < 48) {
                const int P = l >= 24 ? 1 : 0, f = 98 * P + 4 * (l - 24 * P);
                lds_pair(o + f, v >= 1 ? 1.0f : 0.0f, v >= 2 ? 1.0f : 0.0f);
                lds_pair(o + f + 2, v >= 3 ? 1.0f : 0.0f, v >= 3 ? (float)(v - 3) * 0.5f : 0.0f);
            } else if (l < 50) {
                lds_pair(o + (l == 48 ? 96 : 194), (float)v * 0.5f, kOff15[v2 & 15]);
            } else if (l == 50) {
                lds_pair(o + 196, v2 == 0 ? 1.0f : 0.0f, v2 == 0 ? 0.0f : 1.0f);
            } else if (l < 51 + (W - 198) / 2) {            // zero padding columns (GEMM-aligned rows)
                lds_pair(o + 198 + 2 * (l - 51), 0.0f, 0.0f);
            }
        }
        __syncthreads();
        const int nbytes = nr * W * (int)sizeof(T);
        uint8_t* dst = (uint8_t*)(out + (size_t)r0 * W);
        if (((uintptr_t)dst & 15) == 0) {
            for (int q = threadIdx.x; q < nbytes / 16; q += blockDim.x) ((uint4*)dst)[q] = ((const uint4*)img)[q];
            for (int q = (nbytes & ~15) + threadIdx.x; q < nbytes; q += blockDim.x) dst[q] = img[q];
        } else {                                            // rows not 16-byte aligned: 4-byte copies
            for (int q = threadIdx.x; q < nbytes / 4; q += blockDim.x) ((uint32_t*)dst)[q] = ((const uint32_t*)img)[q];
        }
    }
}

// Afterstates / afterstate features of every legal move of a lane.
// MODE 0: int8 boards [M][52]; MODE 1: float features [M][198] (mover one-hot).
template <int MODE>
__global__ __launch_bounds__(64) void k_legal(Args A, int lane0, void* out) {
    const int gi = lane0 + blockIdx.x;
    const int l = lane_id();
    const int bv = load_rec(A, gi);
    const int cur = rd(bv, R_CUR);
    const int n = rd(bv, R_NM0) | (rd(bv, R_NM1) << 8);
    uint32_t blocked;
    const Node s0 = node_from_bytes(bv, cur, blocked);
    for (int m = 0; m < A.max_moves; ++m) {
        int nb = 0;
        if (m < n) {
            const uint64_t mv = A.moves[(size_t)gi * A.max_moves + m];
            const uint32_t mlo = ufl((uint32_t)mv), mhi = ufl((uint32_t)(mv >> 32));
            const uint64_t mm = (uint64_t)mlo | ((uint64_t)mhi << 32);
            Node s = s0;
            for (int i = 0; i < 4; ++i) {
                const uint32_t e = (uint32_t)(mm >> (16 * i)) & 0xFFFFu;
                if (!(e & 0x8000u)) break;
                Sub sm; sm.src = (int)(e & 31u); sm.dst = (int)((e >> 5) & 31u); sm.hit = (int)((e >> 10) & 1u);
                sm.enc = e;
                s = apply(s, sm, cur);
            }
            nb = bytes_from_node(bv, s, cur);
        }
        const size_t row = (size_t)blockIdx.x * A.max_moves + m;
        if (MODE == 0) {
            if (l < 52) ((int8_t*)out)[row * 52 + l] = (int8_t)(m < n ? nb : 0);
        } else {
            float* o = (float*)out + row * 198;
            #pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int f = l + 64 * t;
                const float v = m < n ? feature_at(nb, f < 198 ? f : 197, cur) : 0.0f;
                if (f < 198) o[f] = v;
            }
        }
    }
}

__global__ void k_action_masks(Args A, int16_t* counts, float* masks) {
    const int gi = blockIdx.x;
    const uint8_t* r = A.lanes + (size_t)gi * 64;
    const int n = (int)r[R_NM0] | ((int)r[R_NM1] << 8);
    if (counts && threadIdx.x == 0) counts[gi] = (int16_t)n;
    if (masks)
        for (int m = threadIdx.x; m < A.max_moves; m += blockDim.x) masks[(size_t)gi * A.max_moves + m] = m < n ? 1.0f : 0.0f;
}

// Re-enumerate the legal moves of caller-posed lanes (bgx_set_lanes).
template <int LOG>
__global__ __launch_bounds__(64) void k_regen(Args A, int lane0) {
    __shared__ uint4 tab[1 << LOG];
    __shared__ uint4 memo[kMemoSlots];
    const int gi = lane0 + blockIdx.x;
    int bv = load_rec(A, gi);
    const int cur = rd(bv, R_CUR), r0 = rd(bv, R_ROLL0), r1 = rd(bv, R_ROLL1);
    int total;
    bool ovf;
    int n = run_movegen<LOG>(bv, cur, r0, r1, A.moves + (size_t)gi * A.max_moves, A.max_moves, tab, cap_fast<LOG>(),
                             &total, &ovf, memo);
    int flags = rd(bv, R_FLAGS) & ~1;
    if (ovf) {
        if (lane_id() == 0) { const int q = atomicAdd(A.ovf_count, 1); A.ovf_queue[q] = gi; }
        n = 0; total = 0; flags |= 1;
    }
    if (lane_id() == 0) A.n_total[gi] = total;
    bv = wr(bv, R_NM0, n & 0xFF);
    bv = wr(bv, R_NM1, (n >> 8) & 0xFF);
    bv = wr(bv, R_FLAGS, flags);
    bv = wr(bv, R_NEED, NEED_NONE);
    store_rec(A, gi, bv);
}

// numpy legacy seeding (_legacy_seeding -> init_genrand): mt[0]=s,
// mt[i] = 1812433253*(mt[i-1]^(mt[i-1]>>30)) + i; index = 624.
__global__ void k_mt_seed(uint32_t* mt, const uint32_t* seeds, int B) {
    const int gi = blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= B) return;
    uint32_t* s = mt + (size_t)gi * kMtWords;
    uint32_t x = seeds[gi];
    s[0] = x;
    for (int i = 1; i < 624; ++i) { x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i; s[i] = x; }
    s[624] = 624u;
}


// ---- rollout rows to pinned host memory (bgx_copy_regions): up to 8 strided 2-D
// copies in one launch, 16 bytes per thread-step, non-temporal stores (the
// destination is host memory across PCIe; nothing on the device reads it back).
struct CopyRegions {
    const uint8_t* src[kMaxRegions];
    uint8_t* dst[kMaxRegions];
    int64_t wchunks[kMaxRegions], spitch[kMaxRegions], dpitch[kMaxRegions];
    int64_t pre[kMaxRegions + 1];               // chunk prefix over the regions
    int n;
};

__global__ __launch_bounds__(256) void k_copy_regions(CopyRegions R) {
    const int64_t total = R.pre[R.n];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        int r = 0;
        #pragma unroll
        for (int k = 1; k < kMaxRegions; ++k) r += (k < R.n && i >= R.pre[k]) ? 1 : 0;
        const int64_t j = i - R.pre[r], row = j / R.wchunks[r], col = j - row * R.wchunks[r];
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = *(const u32x4*)(R.src[r] + row * R.spitch[r] + 16 * col);
        __builtin_nontemporal_store(v, (u32x4*)(R.dst[r] + row * R.dpitch[r] + 16 * col));
    }
}

thread_local std::string g_err;

int fail(hipError_t e, int code = BGX_EDEVICE) {
    g_err = hipGetErrorString(e);
    return code;
}

}  // namespace


// error hooks for the other translation units (bg_search.hip, bg_ppo*.hip)
int bgx_internal_fail(hipError_t e) { return fail(e); }
void bgx_set_error(const char* msg) { g_err = msg; }
// the explicit debug options (bg_debug.h, bgx_debug_option)
static std::mutex g_dbg_mu;
static std::map<std::string, std::string> g_dbg;
std::string bgx_dbg(const char* name) {
    std::lock_guard<std::mutex> g(g_dbg_mu);
    const auto it = g_dbg.find(name);
    return it == g_dbg.end() ? std::string() : it->second;
}
long long bgx_dbg_int(const char* name, long long dflt) {
    const std::string v = bgx_dbg(name);
    return v.empty() ? dflt : strtoll(v.c_str(), nullptr, 10);
}

#define CK(x) do { hipError_t _e = (x); if (_e != hipSuccess) return fail(_e); } while (0)
// the per-position kernels (reset, standalone movegen, regeneration) with the
// 512-slot dedup table
#define LAUNCH_LOG(e, K, grid, s, ...) hipLaunchKernelGGL(K<9>, grid, dim3(64), 0, s, __VA_ARGS__)
#define CKL() do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return fail(_e); } while (0)

static void launch_order(bgx_engine* e, hipStream_t s) {
    const int nblk = (e->a.B + 1023) / 1024;
    hipLaunchKernelGGL(k_order_count, dim3(nblk), dim3(1024), 0, s, e->a.cls, e->order_cnt, e->a.B,
                       e->ovf_base + 4 * (e->ovf_parity ^ 1), e->a.xcd);
    e->ovf_next_zeroed = true;
    hipLaunchKernelGGL(k_order_scatter, dim3(nblk), dim3(1024), 0, s, e->a.cls, e->order_cnt, e->perm, e->a.B, nblk,
                       e->a.xcd);
    e->perm_valid = true;
}

static void launch_step(hipStream_t s, const Args& a, int grid, const int32_t* actions, float* obs, float* reward,
                        uint8_t* done, int32_t* info, int base = 0) {
    if (grid <= 0) return;
    // the split's doubles prefix: a 512-slot table and no revisit memo (8 KB of LDS):
    // the doubles walks that cannot bear off use no table at all, so occupancy
    // (VGPR-bound, 4 waves/SIMD) beats a bigger table (C3: 1,024 slots + memo 242 M/s,
    // 512 slots + memo inside 284 M/s, no memo 288 M/s; measured round 2)
    hipLaunchKernelGGL((k_step<0, 9, 0>), dim3(grid), dim3(64), 0, s, a, actions, obs, reward, done, info, base);
}

// Doubles share of the dispatch order (Philox mode): the expected doubles
// fraction 1/6 plus 4 sigma.  Lanes past it run in the light launch whatever
// their class (exact either way; an unpredicted doubles lane is only slower).
// With the XCD-aware order the count is a multiple of 8, so the light launch's
// blocks keep the order's position -> XCD residue.
static int heavy_grid(int B, bool xcd) {
    const double g = B / 6.0 + 4.0 * std::sqrt(B * 5.0 / 36.0) + 32.0;
    int h = g >= B ? B : (int)g;
    if (xcd) h = (h + 7) & ~7;
    return h > B ? B : h;
}

static int slow_path(bgx_engine* e, hipStream_t s, int src, const int8_t* boards, const uint8_t* players,
                     const uint8_t* dice, int cap, int16_t* nm, int32_t* nt, uint64_t* moves) {
    if (src == 0)
        hipLaunchKernelGGL(k_movegen_over<0>, dim3(e->slow_waves), dim3(64), 0, s, e->a, boards, players, dice, cap,
                           nm, nt, moves, e->slow_tables);
    else
        hipLaunchKernelGGL(k_movegen_over<1>, dim3(e->slow_waves), dim3(64), 0, s, e->a, boards, players, dice, cap,
                           nm, nt, moves, e->slow_tables);
    CKL();
    return BGX_OK;
}

extern "C" {

int bgx_engine_create(int device, int32_t batch, int32_t max_moves, uint64_t seed, int32_t dice_mode,
                      int32_t auto_reset, int32_t match_length, bgx_engine** out) {
    if (!out || batch <= 0 || max_moves <= 0 || max_moves > 32767 || dice_mode < 0 || dice_mode > 2)
        return BGX_EINVAL;
    CK(hipSetDevice(device));
    bgx_engine* e = new bgx_engine();
    memset(&e->a, 0, sizeof e->a);
    e->device = device;
    e->seed = seed;
    e->order_pending = false;
    e->step_fork = true;
    Args& A = e->a;
    A.B = batch; A.max_moves = max_moves; A.dice_mode = dice_mode; A.auto_reset = auto_reset ? 1 : 0;
    A.match_length = match_length;
    A.key0 = (uint32_t)seed; A.key1 = (uint32_t)(seed >> 32);
    A.xcd = batch % 128 == 0 && bgx_dbg_int("BGX_XCD", 1) != 0 ? 1 : 0;
    e->step_debug = !bgx_dbg("BGX_STEP_DEBUG").empty();
    // the overflow tiers' caps (tests force positions through tier 1 and tier 2 with small ones)
    A.cap_mid = (int)std::min<long long>(std::max<long long>(bgx_dbg_int("BGX_TIER1_CAP", cap_fast<kLogMid>()), 1),
                                         cap_fast<kLogMid>());
    A.cap_main = (int)std::min<long long>(std::max<long long>(bgx_dbg_int("BGX_MOVEGEN_CAP", cap_fast<9>()), 1),
                                          cap_fast<9>());
    e->slow_waves = kSlowWaves;
    const size_t B = (size_t)batch;
    hipError_t err = hipSuccess;
    auto alloc = [&](void** p, size_t bytes) { if (err == hipSuccess) err = hipMalloc(p, bytes); };
    alloc((void**)&A.lanes, B * 64);
    alloc((void**)&A.moves, B * (size_t)max_moves * 8);
    alloc((void**)&A.n_total, B * 4);
    alloc((void**)&A.mt, (dice_mode == BGX_DICE_MT_SHARED ? 1 : (dice_mode == BGX_DICE_MT_LANE ? B : 1)) * kMtWords * 4);
    alloc((void**)&A.ctr, B * 8);
    alloc((void**)&A.shared_rolls, B * 4);
    alloc((void**)&e->ovf_base, 32);
    A.ovf_count = e->ovf_base;
    alloc((void**)&A.ovf_queue, B * 4);
    alloc((void**)&A.err, 16);
    alloc((void**)&e->slow_tables, (size_t)kSlowWaves * ((size_t)16 << kLogSlotsSlow));
    if (!bgx_dbg("BGX_STAMPS").empty()) alloc((void**)&A.stamps, B * 16);
    if (dice_mode == BGX_DICE_PHILOX && bgx_dbg_int("BGX_ORDER", 1) != 0) {
        alloc((void**)&e->perm, B * 4);
        alloc((void**)&A.cls, B);
        alloc((void**)&e->order_cnt, (B / 1024 + 1) * kXcd * kClasses * 4);
    }
    if (err != hipSuccess) { bgx_engine_destroy(e); return fail(err, BGX_ENOMEM); }
    if (hipMemset(A.lanes, 0, B * 64) != hipSuccess || hipMemset(A.ctr, 0, B * 8) != hipSuccess ||
        hipMemset(e->ovf_base, 0, 32) != hipSuccess || hipMemset(A.err, 0, 16) != hipSuccess ||
        hipMemset(A.n_total, 0, B * 4) != hipSuccess || (A.cls && hipMemset(A.cls, 0, B) != hipSuccess)) {
        bgx_engine_destroy(e);
        return fail(hipGetLastError());
    }
    // default seeds: lane i -> seed + i
    std::vector<uint32_t> seeds(B);
    for (size_t i = 0; i < B; ++i) seeds[i] = (uint32_t)(seed + i);
    int rc = bgx_engine_seed(e, seeds.data(), seed);
    if (rc != BGX_OK) { bgx_engine_destroy(e); return rc; }
    *out = e;
    return BGX_OK;
}

int bgx_engine_join(bgx_engine* e, void* stream) {
    if (!e) return BGX_EINVAL;
    CK(hipSetDevice(e->device));
    EngineUse use(e, (hipStream_t)stream);
    CK(use.err);
    if (e->order_pending) {                  // the next step's dispatch order, on the side stream
        CK(hipStreamWaitEvent((hipStream_t)stream, e->step_ev[3], 0));
        e->order_pending = false;
    }
    return BGX_OK;
}

int bgx_engine_set_fork(bgx_engine* e, int32_t fork, void* stream) {
    if (!e) return BGX_EINVAL;
    CK(hipSetDevice(e->device));
    EngineUse use(e, (hipStream_t)stream);
    CK(use.err);
    if (!fork && e->order_pending) {         // a pending dispatch order joins `stream` first
        CK(hipStreamWaitEvent((hipStream_t)stream, e->step_ev[3], 0));
        e->order_pending = false;
    }
    e->step_fork = fork != 0;
    return BGX_OK;
}

int bgx_engine_destroy(bgx_engine* e) {
    if (!e) return BGX_EINVAL;
    (void)hipSetDevice(e->device);
    if (e->use_valid) (void)hipEventSynchronize(e->use_ev);   // the last call's work is done
    if (e->use_ev) (void)hipEventDestroy(e->use_ev);
    Args& A = e->a;
    void* ptrs[] = {A.lanes, A.moves, A.n_total, A.mt, A.ctr, A.shared_rolls, e->ovf_base, A.ovf_queue, A.err,
                    e->slow_tables, e->search_ws, e->search_pool, e->oneply_ws, A.stamps, e->perm, A.cls, e->order_cnt};
    for (void* p : ptrs) if (p) (void)hipFree(p);
    for (hipEvent_t ev : e->search_ev) if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : e->step_ev) if (ev) (void)hipEventDestroy(ev);
    if (e->step_side) (void)hipStreamDestroy(e->step_side);
    if (e->search_side) (void)hipStreamDestroy(e->search_side);
    delete e;
    return BGX_OK;
}

int bgx_engine_seed(bgx_engine* e, const uint32_t* seeds_host, uint64_t philox_seed) {
    if (!e || !seeds_host) return BGX_EINVAL;
    CK(hipSetDevice(e->device));
    Args& A = e->a;
    // device-wide order (bgx.h "Stream ordering"): every earlier call on any stream has
    // finished before the dice state changes, and the new state is in place on return
    CK(hipDeviceSynchronize());
    A.key0 = (uint32_t)philox_seed; A.key1 = (uint32_t)(philox_seed >> 32);
    CK(hipMemset(A.ctr, 0, (size_t)A.B * 8));
    if (A.dice_mode == BGX_DICE_PHILOX) {
        CK(hipDeviceSynchronize());
        return BGX_OK;
    }
    const int n = A.dice_mode == BGX_DICE_MT_LANE ? A.B : 1;
    uint32_t* dseeds = nullptr;
    CK(hipMalloc(&dseeds, (size_t)n * 4));
    hipError_t err = hipMemcpy(dseeds, seeds_host, (size_t)n * 4, hipMemcpyHostToDevice);
    if (err == hipSuccess) {
        hipLaunchKernelGGL(k_mt_seed, dim3((n + 255) / 256), dim3(256), 0, 0, A.mt, dseeds, n);
        err = hipGetLastError();
    }
    if (err == hipSuccess) err = hipDeviceSynchronize();
    (void)hipFree(dseeds);
    if (err != hipSuccess) return fail(err);
    return BGX_OK;
}

int bgx_engine_mt_state(bgx_engine* e, int32_t lane, uint32_t* state_host, int32_t set) {
    if (!e || !state_host) return BGX_EINVAL;
    Args& A = e->a;
    if (A.dice_mode == BGX_DICE_PHILOX) return BGX_EINVAL;
    if (A.dice_mode == BGX_DICE_MT_SHARED) lane = 0;
    if (lane < 0 || lane >= A.B) return BGX_EINVAL;
    CK(hipSetDevice(e->device));
    CK(hipDeviceSynchronize());
    uint32_t* dev = A.mt + (size_t)lane * kMtWords;
    if (set) CK(hipMemcpy(dev, state_host, 625 * 4, hipMemcpyHostToDevice));
    else CK(hipMemcpy(state_host, dev, 625 * 4, hipMemcpyDeviceToHost));
    return BGX_OK;
}

#ifdef BGX_COUNTERS
extern "C" int bgx_debug_counters(unsigned long long* out16) {
    CK(hipDeviceSynchronize());
    constexpr size_t n = 16 * (size_t)bg::kCntSlots;
    std::vector<unsigned long long> h(n), z(n, 0ull);
    CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(bg::g_cnt), n * 8));
    for (int i = 0; i < 16; ++i) {
        out16[i] = 0;
        for (int k = 0; k < bg::kCntSlots; ++k) out16[i] += h[(size_t)i * bg::kCntSlots + k];
    }
    CK(hipMemcpyToSymbol(HIP_SYMBOL(bg::g_cnt), z.data(), n * 8));
    return BGX_OK;
}
#endif

// diagnostics: copy the per-lane [start, end] s_memrealtime stamps of the last step
extern "C" int bgx_debug_stamps(bgx_engine* e, uint64_t* host_out) {
    if (!e || !host_out || !e->a.stamps) return BGX_EINVAL;
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(host_out, e->a.stamps, (size_t)e->a.B * 16, hipMemcpyDeviceToHost));
    return BGX_OK;
}

int bgx_engine_buffers(bgx_engine* e, bgx_buffers* out) {
    if (!e || !out) return BGX_EINVAL;
    out->lanes = e->a.lanes; out->moves = e->a.moves; out->n_total = e->a.n_total;
    out->batch = e->a.B; out->max_moves = e->a.max_moves;
    return BGX_OK;
}

int bgx_reset(bgx_engine* e, const uint8_t* lane_mask_dev, float* obs_dev, void* stream) {
    if (!e) return BGX_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    Args& A = e->a;
    CK(hipSetDevice(e->device));
    EngineUse use(e, s);
    CK(use.err);
    if (e->order_pending) {                  // a step's dispatch order still on the side stream
        CK(hipStreamWaitEvent(s, e->step_ev[3], 0));
        e->order_pending = false;
    }
    if (e->ovf_next_zeroed) {             // the previous step's k_order_count zeroed the other set
        e->ovf_parity ^= 1;
        A.ovf_count = e->ovf_base + 4 * e->ovf_parity;
        e->ovf_next_zeroed = false;
    } else {
        CK(hipMemsetAsync(A.ovf_count, 0, 16, s));
    }
    if (A.dice_mode == BGX_DICE_MT_SHARED) {
        LAUNCH_LOG(e, k_reset, dim3(A.B), s, A, lane_mask_dev, obs_dev, 1);
        hipLaunchKernelGGL(k_shared_dice, dim3(1), dim3(64), 0, s, A);
        LAUNCH_LOG(e, k_reset, dim3(A.B), s, A, nullptr, obs_dev, 0);
    } else {
        LAUNCH_LOG(e, k_reset, dim3(A.B), s, A, lane_mask_dev, obs_dev, 0);
    }
    CKL();
    if (A.cls) {
        launch_order(e, s);
    }
    return slow_path(e, s, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr);
}

int bgx_step(bgx_engine* e, const int32_t* actions_dev, float* obs_dev, float* reward_dev, uint8_t* done_dev,
             int32_t* info_dev, void* stream) {
    if (!e || !actions_dev || !reward_dev || !done_dev) return BGX_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    Args& A = e->a;
    CK(hipSetDevice(e->device));
    EngineUse use(e, s);
    CK(use.err);
    if (e->ovf_next_zeroed) {             // the previous step's k_order_count zeroed the other set
        e->ovf_parity ^= 1;
        A.ovf_count = e->ovf_base + 4 * e->ovf_parity;
        e->ovf_next_zeroed = false;
    } else {
        CK(hipMemsetAsync(A.ovf_count, 0, 16, s));
    }
    if (A.dice_mode == BGX_DICE_MT_SHARED) {
        hipLaunchKernelGGL((k_step<1, 9>), dim3(A.B), dim3(64), 0, s, A, actions_dev, obs_dev, reward_dev, done_dev,
                           info_dev, 0);
        hipLaunchKernelGGL(k_shared_dice, dim3(1), dim3(64), 0, s, A);
        hipLaunchKernelGGL((k_step<2, 9>), dim3(A.B), dim3(64), 0, s, A, actions_dev, obs_dev, reward_dev, done_dev,
                           info_dev, 0);
    } else {
        if (e->order_pending) {              // the previous step's dispatch order (side stream)
            CK(hipStreamWaitEvent(s, e->step_ev[3], 0));
            e->order_pending = false;
        }
        Args a = A;
        a.perm = e->perm_valid ? e->perm : nullptr;
        const int heavy = a.perm ? heavy_grid(A.B, A.xcd != 0) : A.B;
        // Split dispatch (Philox mode): the predicted-doubles prefix of the order
        // with the big dedup table + revisit memo (26 KB of LDS per wave), then the
        // rest with a 256-slot table, no memo, no doubles code (4 KB, 49 VGPRs: the
        // hardware wave limit, ~5x the resident waves; doubles go to the overflow tiers).
        // Plain stream order -- no cross-stream wait that a serializing tool
        // (profiler) or a shared hardware queue could deadlock.
        if (heavy < A.B && e->step_fork) {
            // fork-join on events: the light launch runs on a side stream beside
            // the heavy one (filling the CUs its tail leaves idle)
            if (!e->step_side) {
                CK(hipStreamCreateWithFlags(&e->step_side, hipStreamNonBlocking));
                for (hipEvent_t& ev : e->step_ev) CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            }
            CK(hipEventRecord(e->step_ev[0], s));
            CK(hipStreamWaitEvent(e->step_side, e->step_ev[0], 0));
            auto light = [&] {
                hipLaunchKernelGGL((k_step<0, 8, 0, true>), dim3(A.B - heavy), dim3(64), 0, e->step_side, a,
                                   actions_dev, obs_dev, reward_dev, done_dev, info_dev, heavy);
            };
            launch_step(s, a, heavy, actions_dev, obs_dev, reward_dev, done_dev, info_dev);
            light();
            CK(hipEventRecord(e->step_ev[1], e->step_side));
            if (A.cls) {
                // the next dispatch order on the side stream once both launches have
                // written their classes: it runs beside this stream's overflow tiers
                // and the caller's next policy kernel instead of before them; the
                // next bgx_step waits for it (step_ev[3]) before its own launches
                CK(hipEventRecord(e->step_ev[2], s));
                CK(hipStreamWaitEvent(e->step_side, e->step_ev[2], 0));
                launch_order(e, e->step_side);
                CK(hipEventRecord(e->step_ev[3], e->step_side));
                e->order_pending = true;
            }
            CK(hipStreamWaitEvent(s, e->step_ev[1], 0));
        } else {
            launch_step(s, a, heavy, actions_dev, obs_dev, reward_dev, done_dev, info_dev);
            if (heavy < A.B)
                hipLaunchKernelGGL((k_step<0, 8, 0, true>), dim3(A.B - heavy), dim3(64), 0, s, a, actions_dev,
                                   obs_dev, reward_dev, done_dev, info_dev, heavy);
        }
        if (A.cls && !e->order_pending) launch_order(e, s);
    }
    CKL();
    const int rc = slow_path(e, s, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr);
    if (e->step_debug) {                     // overflow-tier queue sizes of this step
        int32_t q[2] = {0, 0};
        CK(hipMemcpyAsync(q, A.ovf_count, 8, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        fprintf(stderr, "[bgx step] overflow queue %d of %d lanes\n", q[0], A.B);
        for (int i = 0; i < q[0] && i < 4; ++i) {
            int32_t gi = 0;
            uint8_t rec[64];
            CK(hipMemcpy(&gi, A.ovf_queue + i, 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(rec, A.lanes + (size_t)gi * 64, 64, hipMemcpyDeviceToHost));
            int own = 0, outside = 0;
            const int pl = rec[52];
            for (int p = 0; p < 24; ++p) {
                own += rec[pl * 24 + p] > 0;
                if (!(pl == 0 ? p >= 18 : p < 6)) outside += rec[pl * 24 + p];
            }
            fprintf(stderr, "   lane %d pl %d roll %d-%d points %d outside %d bar %d off %d n %d\n", gi, pl, rec[53],
                    rec[54], own, outside, rec[48 + pl], rec[50 + pl], rec[60] | (rec[61] << 8));
        }
    }
    return rc;
}

int bgx_movegen(bgx_engine* e, const int8_t* boards52_dev, const uint8_t* players_dev, const uint8_t* dice_dev,
                int32_t n, int32_t max_moves, int16_t* n_moves_dev, int32_t* n_total_dev, uint64_t* moves_dev,
                void* stream) {
    if (!e || n < 0 || max_moves <= 0 || !boards52_dev || !players_dev || !dice_dev || !n_moves_dev || !moves_dev)
        return BGX_EINVAL;
    if (n > e->a.B) return BGX_EINVAL;   // overflow queue is sized by the engine batch
    if (n == 0) return BGX_OK;
    hipStream_t s = (hipStream_t)stream;
    CK(hipSetDevice(e->device));
    EngineUse use(e, s);
    CK(use.err);
    CK(hipMemsetAsync(e->a.ovf_count, 0, 16, s));
    LAUNCH_LOG(e, k_movegen, dim3(n), s, boards52_dev, players_dev, dice_dev, n, max_moves, n_moves_dev, n_total_dev,
               moves_dev, e->a.ovf_count, e->a.ovf_queue, e->a.cap_main);
    CKL();
    return slow_path(e, s, 1, boards52_dev, players_dev, dice_dev, max_moves, n_moves_dev, n_total_dev, moves_dev);
}

int bgx_encode(const int8_t* boards52_dev, const uint8_t* players_dev, int32_t n, float* out_dev, void* stream) {
    if (n < 0 || (n > 0 && (!boards52_dev || !players_dev || !out_dev))) return BGX_EINVAL;
    if (n == 0) return BGX_OK;
    hipLaunchKernelGGL(k_encode, dim3(n), dim3(64), 0, (hipStream_t)stream, boards52_dev, players_dev, n, out_dev);
    CKL();
    return BGX_OK;
}

int bgx_encode_records_ex(const uint8_t* records_dev, int32_t n, int32_t dtype, int32_t width, void* out_dev,
                          void* stream) {
    if (n < 0 || (dtype != 0 && dtype != 1) || (width != 198 && width != 208) || (n > 0 && (!records_dev || !out_dev)))
        return BGX_EINVAL;
    if (n == 0) return BGX_OK;
    const int blocks = (n + 63) / 64 < 4096 ? (n + 63) / 64 : 4096;
    const hipStream_t s = (hipStream_t)stream;
    if (dtype == 0 && width == 198)
        hipLaunchKernelGGL((k_encode_rec<float, 198>), dim3(blocks), dim3(256), 0, s, records_dev, n, (float*)out_dev);
    else if (dtype == 0)
        hipLaunchKernelGGL((k_encode_rec<float, 208>), dim3(blocks), dim3(256), 0, s, records_dev, n, (float*)out_dev);
    else if (width == 198)
        hipLaunchKernelGGL((k_encode_rec<_Float16, 198>), dim3(blocks), dim3(256), 0, s, records_dev, n,
                           (_Float16*)out_dev);
    else
        hipLaunchKernelGGL((k_encode_rec<_Float16, 208>), dim3(blocks), dim3(256), 0, s, records_dev, n,
                           (_Float16*)out_dev);
    CKL();
    return BGX_OK;
}

int bgx_encode_records(const uint8_t* records_dev, int32_t n, int32_t dtype, void* out_dev, void* stream) {
    return bgx_encode_records_ex(records_dev, n, dtype, 198, out_dev, stream);
}

int bgx_afterstates(bgx_engine* e, int32_t lane0, int32_t nlanes, int8_t* boards52_dev, void* stream) {
    if (!e || !boards52_dev || lane0 < 0 || nlanes < 0 || lane0 + nlanes > e->a.B) return BGX_EINVAL;
    if (nlanes == 0) return BGX_OK;
    CK(hipSetDevice(e->device));
    EngineUse use(e, (hipStream_t)stream);
    CK(use.err);
    hipLaunchKernelGGL(k_legal<0>, dim3(nlanes), dim3(64), 0, (hipStream_t)stream, e->a, lane0, (void*)boards52_dev);
    CKL();
    return BGX_OK;
}

int bgx_legal_features(bgx_engine* e, int32_t lane0, int32_t nlanes, float* out_dev, void* stream) {
    if (!e || !out_dev || lane0 < 0 || nlanes < 0 || lane0 + nlanes > e->a.B) return BGX_EINVAL;
    if (nlanes == 0) return BGX_OK;
    CK(hipSetDevice(e->device));
    EngineUse use(e, (hipStream_t)stream);
    CK(use.err);
    hipLaunchKernelGGL(k_legal<1>, dim3(nlanes), dim3(64), 0, (hipStream_t)stream, e->a, lane0, (void*)out_dev);
    CKL();
    return BGX_OK;
}

int bgx_action_masks(bgx_engine* e, int16_t* counts_dev, float* masks_dev, void* stream) {
    if (!e) return BGX_EINVAL;
    if (!counts_dev && !masks_dev) return BGX_OK;
    CK(hipSetDevice(e->device));
    EngineUse use(e, (hipStream_t)stream);
    CK(use.err);
    hipLaunchKernelGGL(k_action_masks, dim3(e->a.B), dim3(masks_dev ? 256 : 64), 0, (hipStream_t)stream, e->a,
                       counts_dev, masks_dev);
    CKL();
    return BGX_OK;
}

int bgx_copy_lanes(bgx_engine* e, int32_t lane0, int32_t n, uint8_t* lanes_dst, uint64_t* moves_dst,
                   int32_t* n_total_dst, void* stream) {
    if (!e || lane0 < 0 || n < 0 || lane0 + n > e->a.B) return BGX_EINVAL;
    if (n == 0) return BGX_OK;
    hipStream_t s = (hipStream_t)stream;
    const Args& A = e->a;
    CK(hipSetDevice(e->device));
    EngineUse use(e, s);
    CK(use.err);
    if (lanes_dst) CK(hipMemcpyAsync(lanes_dst, A.lanes + (size_t)lane0 * 64, (size_t)n * 64, hipMemcpyDeviceToDevice, s));
    if (moves_dst)
        CK(hipMemcpyAsync(moves_dst, A.moves + (size_t)lane0 * A.max_moves, (size_t)n * A.max_moves * 8,
                          hipMemcpyDeviceToDevice, s));
    if (n_total_dst) CK(hipMemcpyAsync(n_total_dst, A.n_total + lane0, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    return BGX_OK;
}

int bgx_set_lanes(bgx_engine* e, int32_t lane0, int32_t n, const uint8_t* lanes_src, void* stream) {
    return bgx_set_lanes_ex(e, lane0, n, lanes_src, 1, stream);
}

int bgx_set_lanes_ex(bgx_engine* e, int32_t lane0, int32_t n, const uint8_t* lanes_src, int32_t regen, void* stream) {
    if (!e || !lanes_src || lane0 < 0 || n < 0 || lane0 + n > e->a.B) return BGX_EINVAL;
    if (n == 0) return BGX_OK;
    hipStream_t s = (hipStream_t)stream;
    Args& A = e->a;
    CK(hipSetDevice(e->device));
    EngineUse use(e, s);
    CK(use.err);
    CK(hipMemcpyAsync(A.lanes + (size_t)lane0 * 64, lanes_src, (size_t)n * 64, hipMemcpyDeviceToDevice, s));
    if (!regen) return BGX_OK;
    CK(hipMemsetAsync(A.ovf_count, 0, 16, s));
    LAUNCH_LOG(e, k_regen, dim3(n), s, A, lane0);
    CKL();
    return slow_path(e, s, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr);
}

int bgx_engine_error(bgx_engine* e, int32_t* err_out) {
    if (!e || !err_out) return BGX_EINVAL;
    CK(hipSetDevice(e->device));
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(err_out, e->a.err, 4, hipMemcpyDeviceToHost));
    return BGX_OK;
}

int bgx_host_device_ptr(void* host_ptr, void** dev_ptr_out) {
    if (!host_ptr || !dev_ptr_out) return BGX_EINVAL;
    CK(hipHostGetDevicePointer(dev_ptr_out, host_ptr, 0));
    return BGX_OK;
}

int bgx_copy_regions(const bgx_region* regions, int32_t n, int32_t workgroups, void* stream) {
    if (!regions || n < 0 || n > kMaxRegions) return BGX_EINVAL;
    CopyRegions R;
    memset(&R, 0, sizeof R);
    R.n = n;
    int64_t acc = 0;
    for (int i = 0; i < n; ++i) {
        const bgx_region& g = regions[i];
        if (!g.src || !g.dst || g.width < 0 || g.rows < 0 || g.width % 16 || g.spitch % 16 || g.dpitch % 16 ||
            (uintptr_t)g.src % 16 || (uintptr_t)g.dst % 16 || (g.rows > 1 && (g.spitch < g.width || g.dpitch < g.width)))
            return BGX_EINVAL;
        R.src[i] = (const uint8_t*)g.src; R.dst[i] = (uint8_t*)g.dst;
        R.wchunks[i] = g.width / 16 > 0 ? g.width / 16 : 1;
        R.spitch[i] = g.spitch; R.dpitch[i] = g.dpitch;
        R.pre[i] = acc;
        acc += g.width / 16 * g.rows;
    }
    for (int i = n; i <= kMaxRegions; ++i) R.pre[i] = acc;
    if (acc == 0) return BGX_OK;
    const int64_t need = (acc + 255) / 256;
    const int wg = (int)(workgroups > 0 && workgroups < need ? workgroups : (need < 64 ? need : 64));
    hipLaunchKernelGGL(k_copy_regions, dim3(wg), dim3(256), 0, (hipStream_t)stream, R);
    CKL();
    return BGX_OK;
}

const char* bgx_last_error(void) { return g_err.c_str(); }

int bgx_debug_option(const char* name, const char* value) {
    if (!name || !name[0]) return BGX_EINVAL;
    std::lock_guard<std::mutex> g(g_dbg_mu);
    if (value) g_dbg[name] = value; else g_dbg.erase(name);
    return BGX_OK;
}

#ifndef BGX_BUILD_ID
#define BGX_BUILD_ID "unknown"
#endif
// the tag lets build() read the id from the file without loading it
__attribute__((used)) static const char kBuildId[] = "bgx-build-id:" BGX_BUILD_ID;
const char* bgx_build_id(void) { return kBuildId + 13; }

}  // extern "C"
