// bg_engine.h — engine internals shared by bg_engine.hip and bg_search.hip:
// lane-record layout, dice streams (numpy-legacy MT19937 / Philox), and the
// per-wave move-generation driver over an LDS dedup table.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string>

#include "bg_core.h"
#include "../../include/bgx.h"

namespace bg {

// LDS dedup table: 2^LOG slots x 16 B (LOG 9 = 8 KiB, 10 = 16 KiB); chosen at
// engine creation (env BGX_LDS_LOG), capacity 7/8 of the slots.
template <int LOG> constexpr int cap_fast() { return (7 << LOG) / 8; }
constexpr int kLogSlotsSlow = 17;             // 131072-slot global table (2 MiB) per slow wave
constexpr int kCapSlow = (7 << kLogSlotsSlow) / 8;
constexpr int kSlowWaves = 32;
constexpr int kMtWords = 640;

// lane record byte offsets
constexpr int R_CUR = 52, R_ROLL0 = 53, R_ROLL1 = 54, R_OVER = 55, R_MATCH = 56, R_S0 = 57, R_S1 = 58,
              R_NEED = 59, R_NM0 = 60, R_NM1 = 61, R_FLAGS = 62;
constexpr int NEED_NONE = 0, NEED_ROLL = 1, NEED_RESET = 2;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int rd(int bv, int i) { return __builtin_amdgcn_readlane(bv, i); }
__device__ __forceinline__ int wr(int bv, int i, int v) { return lane_id() == i ? v : bv; }
__device__ __forceinline__ uint32_t ufl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// immutable_board.py:25-40 in the 52-byte layout
__device__ __forceinline__ int initial_byte(int l) {
    switch (l) {
        case 0: return 2;  case 11: return 5; case 16: return 3; case 18: return 5;
        case 24 + 23: return 2; case 24 + 12: return 5; case 24 + 7: return 3; case 24 + 5: return 5;
        default: return 0;
    }
}

// ------------------------------------------------------------------- dice --
// backgammon_env.py:245-246: np.random.randint(1,7) on numpy's legacy MT19937:
// x = next_u32 & 7, rejected while x > 5, die = x + 1.
struct Rng {
    int mode;                 // BGX_DICE_*
    // MT19937 (per lane, or the shared stream for SHARED mode's serial kernel)
    uint32_t* mt;             // 640 words in HBM
    uint32_t* sh;             // 624 words of LDS scratch (twist)
    int idx, wbase;
    uint32_t win;
    bool wvalid, twisted, used;
    // Philox4x32-10
    uint64_t ctr, blkid;
    uint32_t k0, k1, lane;
    uint32_t blk0, blk1, blk2, blk3;

    __device__ void init_mt(uint32_t* state, uint32_t* lds) {
        mode = BGX_DICE_MT_LANE; mt = state; sh = lds;
        idx = (int)ufl(state[624]); wvalid = false; twisted = false; used = false;
    }
    __device__ void init_philox(uint64_t c, uint32_t key0, uint32_t key1, uint32_t lane_no) {
        mode = BGX_DICE_PHILOX; ctr = c; blkid = ~0ull; k0 = key0; k1 = key1; lane = lane_no; used = false;
    }

    __device__ void twist() {
        const int l = lane_id();
        constexpr uint32_t UP = 0x80000000u, LO = 0x7fffffffu, MAG = 0x9908b0dfu;
        if (!twisted) {
            for (int j = l; j < 624; j += 64) sh[j] = mt[j];
        }
        __syncthreads();
        // new[kk] = sh[kk+off] ^ f(old[kk], old[kk+1]); chunks ascend, reads before writes
        for (int pass = 0; pass < 2; ++pass) {
            const int lo = pass == 0 ? 0 : 227, hi = pass == 0 ? 227 : 623, off = pass == 0 ? 397 : -227;
            for (int base = lo; base < hi; base += 64) {
                const int kk = base + l;
                uint32_t v = 0;
                if (kk < hi) {
                    const uint32_t y = (sh[kk] & UP) | (sh[kk + 1] & LO);
                    v = sh[kk + off] ^ (y >> 1) ^ ((y & 1u) ? MAG : 0u);
                }
                __syncthreads();
                if (kk < hi) sh[kk] = v;
                __syncthreads();
            }
        }
        if (l == 0) {
            const uint32_t y = (sh[623] & UP) | (sh[0] & LO);
            sh[623] = sh[396] ^ (y >> 1) ^ ((y & 1u) ? MAG : 0u);
        }
        __syncthreads();
        twisted = true;
        idx = 0;
        wvalid = false;
    }

    __device__ uint32_t next_mt() {
        if (idx >= 624) twist();
        if (!wvalid || idx >= wbase + 64) {
            const int j = idx + lane_id();
            win = j < 624 ? (twisted ? sh[j] : mt[j]) : 0u;
            wbase = idx;
            wvalid = true;
        }
        uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)win, idx - wbase);
        ++idx;
        y ^= y >> 11; y ^= (y << 7) & 0x9d2c5680u; y ^= (y << 15) & 0xefc60000u; y ^= y >> 18;
        return y;
    }

    __device__ uint32_t next_philox() {
        const uint64_t b = ctr >> 2;
        if (b != blkid) {
            uint32_t c0 = (uint32_t)b, c1 = (uint32_t)(b >> 32), c2 = lane, c3 = 0x42474D4Eu;
            uint32_t a0 = k0, a1 = k1;
            #pragma unroll
            for (int r = 0; r < 10; ++r) {
                const uint32_t h0 = __umulhi(0xD2511F53u, c0), l0 = 0xD2511F53u * c0;
                const uint32_t h1 = __umulhi(0xCD9E8D57u, c2), l1 = 0xCD9E8D57u * c2;
                c0 = h1 ^ c1 ^ a0; c1 = l1; c2 = h0 ^ c3 ^ a1; c3 = l0;
                a0 += 0x9E3779B9u; a1 += 0xBB67AE85u;
            }
            blk0 = c0; blk1 = c1; blk2 = c2; blk3 = c3; blkid = b;
        }
        const uint32_t w = (uint32_t)(ctr & 3u);
        ++ctr;
        return w == 0 ? blk0 : w == 1 ? blk1 : w == 2 ? blk2 : blk3;
    }

    __device__ int die() {
        used = true;
        for (;;) {
            const uint32_t x = (mode == BGX_DICE_PHILOX ? next_philox() : next_mt()) & 7u;
            if (x <= 5u) return (int)x + 1;
        }
    }

    // write the per-lane state back
    __device__ void finish(uint64_t* ctr_out) {
        if (!used) return;
        if (mode == BGX_DICE_PHILOX) {
            if (lane_id() == 0) *ctr_out = ctr;
            return;
        }
        if (twisted) {
            for (int j = lane_id(); j < 624; j += 64) mt[j] = sh[j];
        }
        if (lane_id() == 0) mt[624] = (uint32_t)idx;
    }
};

// ---------------------------------------------------------------- engine --
struct Args {
    uint8_t* lanes;
    uint64_t* moves;
    int32_t* n_total;
    uint32_t* mt;
    uint64_t* ctr;
    uint8_t* shared_rolls;    // [B][4] r0, r1, starter (SHARED mode)
    int32_t* ovf_count;
    int32_t* ovf_queue;
    int32_t* err;
    int B, max_moves, dice_mode, auto_reset, match_length;
    uint32_t key0, key1;
    uint64_t* stamps;         // diagnostics only (debug option BGX_STAMPS): [B][2] start/end s_memrealtime
    int cap_mid;              // tier 1's unique-afterstate cap (cap_fast<kLogMid>; tests: BGX_TIER1_CAP)
    int cap_main;             // bgx_movegen's main-table cap (cap_fast<9>; tests: BGX_MOVEGEN_CAP)
    // dispatch order (Philox mode): each step predicts its lane's next-turn cost class
    // into cls; k_order turns the classes into perm (heaviest first) for the next launch.
    int32_t* perm;            // blockIdx -> lane, or null (identity)
    uint8_t* cls;             // [B] predicted cost class, or null
    int xcd;                  // B % 128 == 0: XCD-aware dispatch (16-lane runs per XCD, bg_engine.hip k_order_*)
};

// blockIdx -> lane when there is no dispatch order: blocks b, b + 8, ... (one XCD
// under round-robin placement) take the 16 consecutive lanes of one run, so a
// run's partial-line loads and stores stay in one XCD's L2.  Identity otherwise.
__device__ __forceinline__ int lane_of_block(const Args& A, int bi) {
    if (!A.xcd) return bi;
    const int r = bi & 127;
    return (bi & ~127) | ((r & 7) << 4) | (r >> 3);
}

constexpr int kClasses = 5;

// Philox counters (the low 48 bits) carry in bits 48-63 the lane's next roll as
// the previous step predicted it (predict_class): valid << 15 | r0 | r1 << 3 |
// draws << 6.  The next normal roll takes it instead of running the same Philox
// block again and advances the counter by the draws; a reset ignores it (it
// draws from the counter as if nothing had been predicted), so the dice stream
// is exactly the one without the cache.
constexpr uint64_t kCtrMask = (1ull << 48) - 1ull;

// Cost class of the lane's NEXT movegen (0 = heaviest).  Philox dice are a pure
// function of (key, lane, counter), so the next roll is known now; the mover
// after the next apply is 1 - cur.  Doubles dominate (a 4-deep DFS) and grow
// with the number of points the mover occupies.  Only a scheduling hint.
__device__ __forceinline__ int predict_class(int bv, uint64_t ctr, const Args& A, int gi, uint32_t& cache) {
    cache = 0u;
    if (rd(bv, R_OVER)) return kClasses - 1;              // next: reset -> opening roll (never doubles)
    Rng r;
    const uint64_t c0 = ctr & kCtrMask;
    r.init_philox(c0, A.key0, A.key1, (uint32_t)gi);
    const int a = r.die(), b = r.die();
    const uint64_t draws = r.ctr - c0;
    if (draws < 32) cache = 0x8000u | (uint32_t)a | ((uint32_t)b << 3) | ((uint32_t)draws << 6);
    if (a != b) return kClasses - 1;
    const int nxt = 1 - rd(bv, R_CUR);
    const int l = lane_id();
    const int off = nxt * 24;
    const bool mine = l >= off && l < off + 24 && bv > 0;
    const int pts = __popcll(__ballot(mine)) + (rd(bv, 48 + nxt) > 0 ? 2 : 0);
    // tail risk of a doubles movegen grows with the points the mover occupies and
    // falls with the die (tools/stamps.py table: p99 150-270 us at >= 9 points
    // for 1-1 .. 4-4, ~60 us at 5 points): longest-first order
    if (pts >= 10 && a <= 4) return 0;
    if ((pts >= 8 && a <= 5) || pts >= 10) return 1;
    return pts >= 5 ? 2 : 3;
}

// Enumerate the legal moves of (board in bv, player pl, roll) into `out`.
// Returns n_moves (truncated); *total = untruncated count; *ovf on overflow.
template <int LOG, typename SlotPtr, int MEMO_KIND = 0, bool NO_DOUBLES = false>
__device__ __forceinline__ int run_movegen(int bv, int pl, int r0, int r1, uint64_t* out, int cap, SlotPtr tab,
                                           int cap_unique, int* total, bool* ovf, uint4* memo) {
    const bool dbl = r0 == r1;
    Gen<LOG, SlotPtr, MoveSink, MEMO_KIND> g;       // clears its table (and memo) when needed
    g.tab = tab; g.sink.out = out; g.sink.cap = cap; g.pl = pl; g.cap_unique = cap_unique;
    g.memo2 = memo && dbl ? memo : nullptr;
    g.memo3 = memo && dbl ? (MEMO_KIND != 0 ? memo : memo + (1 << kLogMemo2)) : nullptr;
    uint32_t blocked;
    const Node s0 = node_from_bytes(bv, pl, blocked);
    g.blocked = blocked;
    if (NO_DOUBLES) g.run_nd(s0, r0, r1);
    else g.run(s0, r0, r1);
    *ovf = g.ovf;
    *total = g.count;
    return g.count < cap ? g.count : cap;
}

// Reset / dice part of advance_lane (reset: backgammon_env.py:78-113; pass/turn:
// :183-188 roll_dice).  Returns false when the lane needs nothing this step.
// mt_scratch: 624 words of LDS for the MT19937 twist (MT_LANE mode only).
__device__ __forceinline__ bool roll_lane(int& bv, int gi, const Args& A, uint32_t* mt_scratch, uint64_t* ctr_io,
                                          int& r0, int& r1) {
    const int need = rd(bv, R_NEED);
    if (need == NEED_NONE) return false;
    Rng rng;
    bool cached = false;
    if (A.dice_mode == BGX_DICE_PHILOX) {
        const uint32_t cache = (uint32_t)(*ctr_io >> 48);
        const uint64_t c = *ctr_io & kCtrMask;
        cached = need != NEED_RESET && (cache & 0x8000u) != 0u;     // the roll predicted last step
        rng.init_philox(cached ? c + ((cache >> 6) & 31u) : c, A.key0, A.key1, (uint32_t)gi);
        if (cached) {
            r0 = (int)(cache & 7u);
            r1 = (int)((cache >> 3) & 7u);
            if (lane_id() == 0) A.ctr[gi] = rng.ctr;
        }
    }
    else if (A.dice_mode == BGX_DICE_MT_LANE) rng.init_mt(A.mt + (size_t)gi * kMtWords, mt_scratch);
    if (cached) {
    } else if (need == NEED_RESET) {
        if (rd(bv, R_MATCH)) { bv = wr(bv, R_S0, 0); bv = wr(bv, R_S1, 0); bv = wr(bv, R_MATCH, 0); }
        if (lane_id() < 52) bv = initial_byte(lane_id());
        bv = wr(bv, R_OVER, 0);
        int starter;
        if (A.dice_mode == BGX_DICE_MT_SHARED) {
            const uint8_t* sr = A.shared_rolls + (size_t)gi * 4;
            r0 = (int)ufl(sr[0]); r1 = (int)ufl(sr[1]); starter = (int)ufl(sr[2]);
        } else {
            int a, b;
            do { a = rng.die(); b = rng.die(); } while (a == b);
            starter = a < b ? 1 : 0;
            do { r0 = rng.die(); r1 = rng.die(); } while (r0 == r1);
        }
        bv = wr(bv, R_CUR, starter);
    } else {
        if (A.dice_mode == BGX_DICE_MT_SHARED) {
            const uint8_t* sr = A.shared_rolls + (size_t)gi * 4;
            r0 = (int)ufl(sr[0]); r1 = (int)ufl(sr[1]);
        } else {
            r0 = rng.die(); r1 = rng.die();
        }
    }
    rng.finish(A.ctr + gi);
    if (A.dice_mode == BGX_DICE_PHILOX) *ctr_io = rng.ctr;
    bv = wr(bv, R_ROLL0, r0);
    bv = wr(bv, R_ROLL1, r1);
    return true;
}

// update_legal_moves (backgammon_env.py:193-231) for the rolled dice: move list,
// counts and flags into the record / HBM; overflowed lanes are queued for the
// bigger tables.
template <int LOG, int MEMO_KIND, bool NO_DOUBLES = false>
__device__ __forceinline__ int movegen_lane(int bv, int gi, const Args& A, int r0, int r1, uint4* lds_tab,
                                            uint4* lds_memo) {
    const int cur = rd(bv, R_CUR);
    int total;
    bool ovf;
    int n = run_movegen<LOG, uint4*, MEMO_KIND, NO_DOUBLES>(bv, cur, r0, r1, A.moves + (size_t)gi * A.max_moves,
                                                             A.max_moves, lds_tab, cap_fast<LOG>(), &total, &ovf,
                                                             lds_memo);
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
    return bv;
}

// Hand the lane to the overflow tiers (k_movegen_over) instead of enumerating here.
__device__ __forceinline__ int defer_lane(int bv, int gi, const Args& A) {
    if (lane_id() == 0) { const int q = atomicAdd(A.ovf_count, 1); A.ovf_queue[q] = gi; A.n_total[gi] = 0; }
    bv = wr(bv, R_NM0, 0);
    bv = wr(bv, R_NM1, 0);
    bv = wr(bv, R_FLAGS, rd(bv, R_FLAGS) | 1);
    return wr(bv, R_NEED, NEED_NONE);
}

// Roll + movegen for one lane according to its `need` byte.  NO_DOUBLES (the
// light launch of the split dispatch): a doubles roll goes to the overflow tiers,
// so this instantiation carries only the non-doubles enumeration (registers).
template <int LOG, int MEMO_KIND = 0, bool NO_DOUBLES = false>
__device__ __forceinline__ int advance_lane(int bv, int gi, const Args& A, uint4* lds_tab, uint4* lds_memo,
                                            uint64_t* ctr_io) {
    int r0, r1;
    if (!roll_lane(bv, gi, A, (uint32_t*)lds_tab, ctr_io, r0, r1)) return bv;
    if (NO_DOUBLES && r0 == r1) return defer_lane(bv, gi, A);
    return movegen_lane<LOG, MEMO_KIND, NO_DOUBLES>(bv, gi, A, r0, r1, lds_tab, lds_memo);
}

__device__ __forceinline__ void write_obs(int bv, float* obs_row) {
    const int cur = rd(bv, R_CUR);
    #pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int f = lane_id() + 64 * t;
        const float v = feature_at(bv, f < 198 ? f : 197, cur);
        if (f < 198) obs_row[f] = v;
    }
}

// backgammon_env.py:115-191 up to (not including) roll/update_legal_moves.
__device__ __forceinline__ int apply_lane(int bv, int gi, int action, const Args& A, float* reward, uint8_t* done,
                                          int32_t* info) {
    const int mover = rd(bv, R_CUR);
    int winner = -1, score = 0, kind = 0, dn = 0;
    float rew = 0.0f;
    if (rd(bv, R_OVER)) {                               // :119-121
        bv = wr(bv, R_NEED, NEED_RESET);
        dn = 1; kind = 3;
    } else {
        const int n = rd(bv, R_NM0) | (rd(bv, R_NM1) << 8);
        if (n == 0) {                                     // :124-140 pass
            bv = wr(bv, R_CUR, 1 - mover);
            bv = wr(bv, R_NEED, NEED_ROLL);
            kind = 1;
        } else {
            const int a = action < 0 ? action + A.max_moves : action;
            if (a < 0 || a >= n) {                        // :143-149 invalid action
                rew = -1.0f; kind = 2;
            } else {                                      // :152-188
                const uint64_t mv = A.moves[(size_t)gi * A.max_moves + a];
                const uint32_t mlo = ufl((uint32_t)mv), mhi = ufl((uint32_t)(mv >> 32));
                const uint64_t m = (uint64_t)mlo | ((uint64_t)mhi << 32);
                uint32_t blocked;
                Node s = node_from_bytes(bv, mover, blocked);
                for (int i = 0; i < 4; ++i) {
                    const uint32_t e = (uint32_t)(m >> (16 * i)) & 0xFFFFu;
                    if (!(e & 0x8000u)) break;
                    Sub sm; sm.src = (int)(e & 31u); sm.dst = (int)((e >> 5) & 31u); sm.hit = (int)((e >> 10) & 1u);
                    sm.enc = e;
                    s = apply(s, sm, mover);
                }
                bv = bytes_from_node(bv, s, mover);
                if (rd(bv, 50 + mover) == 15) {            // win (:156-182)
                    const int opp = 1 - mover;
                    const bool opp_off0 = rd(bv, 50 + opp) == 0;
                    const int l = lane_id();
                    const int hl = mover == 0 ? 18 : 0;     // mover's home board (:388-391)
                    const bool in_home = l >= opp * 24 + hl && l < opp * 24 + hl + 6 && bv > 0;
                    const bool bg = opp_off0 && (__ballot(in_home) != 0ull || rd(bv, 48 + opp) > 0);
                    score = bg ? 3 : (opp_off0 ? 2 : 1);
                    rew = bg ? 2.0f : (opp_off0 ? 1.5f : 1.0f);
                    winner = mover; dn = 1;
                    const int ns = rd(bv, R_S0 + mover) + score;
                    bv = wr(bv, R_S0 + mover, ns > 255 ? 255 : ns);
                    bv = wr(bv, R_OVER, 1);
                    if (ns >= A.match_length) bv = wr(bv, R_MATCH, 1);
                    if (A.auto_reset) bv = wr(bv, R_NEED, NEED_RESET);   // vec_bg_env.py:35-36
                } else {
                    bv = wr(bv, R_CUR, 1 - mover);
                    bv = wr(bv, R_NEED, NEED_ROLL);
                }
            }
        }
    }
    if (lane_id() == 0) {
        reward[gi] = rew;
        done[gi] = (uint8_t)dn;
        if (info) info[gi] = mover | ((winner + 1) << 8) | (score << 16) | (kind << 24);
    }
    return bv;
}

__device__ __forceinline__ int load_rec(const Args& A, int gi) { return (int)A.lanes[(size_t)gi * 64 + lane_id()]; }
__device__ __forceinline__ void store_rec(const Args& A, int gi, int bv) { A.lanes[(size_t)gi * 64 + lane_id()] = (uint8_t)bv; }


}  // namespace bg

// Engine object behind the C ABI's opaque bgx_engine*.
struct bgx_engine {
    bool step_debug = false;        // BGX_STEP_DEBUG (bgx_debug_option) at creation: per-step tier sizes
    int device;
    bg::Args a;
    uint4* slow_tables;
    int slow_waves;
    int32_t* perm;        // dispatch order for k_step (Philox mode), built by k_order
    bool perm_valid;
    int32_t* order_cnt;   // k_order_count -> k_order_scatter, [B/1024+1][kClasses]
    // overflow counters, two 16-byte sets: a Philox step uses set `ovf_parity`
    // (Args::ovf_count) and its k_order_count zeroes the other set for the next
    // step, so the step needs no separate memset launch
    hipStream_t step_side;      // the light launch beside the heavy one, and the next dispatch order
    hipEvent_t step_ev[4];      // fork, light done, heavy done, dispatch order done
    bool order_pending;         // the next step's launches wait for step_ev[3]
    bool step_fork;             // bgx_engine_set_fork: light launch + dispatch order on step_side
    int32_t* ovf_base;
    int ovf_parity;
    bool ovf_next_zeroed;
    uint64_t seed;
    // bg_search.hip workspace (grown on demand)
    void* search_ws;
    size_t search_ws_bytes;
    void* search_pool;        // 2-ply leaf pool: keys [cap] x 16 B, then tags [cap] x 4 B
    size_t search_pool_cap;
    hipStream_t search_side;  // 2-ply: second stream for the concurrent enumerator (created on demand)
    hipEvent_t search_ev[5];  // 2-ply phase marks: start, enumerated, evaluated, fork, join
    float search_ms[2];       // last bgx_two_ply call, round 0: enumeration ms, evaluation ms
    void* oneply_ws;          // bgx_one_ply workspace (rows sized for B x max_moves)
    size_t oneply_ws_bytes;
    // Cross-stream ordering of the engine's own calls (bgx.h "Stream ordering"): the end of
    // the last eager call that touched the engine's device state (lanes, moves, overflow
    // queues and tables, search workspace) and the stream it ran on.  A call on another
    // stream waits for it first.
    hipEvent_t use_ev;
    hipStream_t use_stream;
    bool use_valid;           // use_ev marks the last call (false: none yet, or it was captured)
};

// RAII guard of one engine call on stream s: the constructor makes s wait for the engine's
// previous call when that ran on another stream; the destructor marks this call's end.  A
// call made while s is being captured into a HIP graph neither waits nor marks (its work
// runs when the graph is launched; the launch stream orders it): the guard then forgets the
// last mark, so the next eager call on any stream does not wait on a stale event.
struct EngineUse {
    bgx_engine* e;
    hipStream_t s;
    bool captured;
    hipError_t err;
    EngineUse(bgx_engine* e_, hipStream_t s_) : e(e_), s(s_), captured(false), err(hipSuccess) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) captured = true;
        if (!captured && e->use_valid && e->use_stream != s) err = hipStreamWaitEvent(s, e->use_ev, 0);
    }
    ~EngineUse() {
        if (captured) { e->use_valid = false; return; }
        if (!e->use_ev && hipEventCreateWithFlags(&e->use_ev, hipEventDisableTiming) != hipSuccess) {
            e->use_ev = nullptr;
            e->use_valid = false;
            return;
        }
        e->use_valid = hipEventRecord(e->use_ev, s) == hipSuccess;
        e->use_stream = s;
    }
};
