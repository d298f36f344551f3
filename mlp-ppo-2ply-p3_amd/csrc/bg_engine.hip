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
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <mutex>
#include <string>
#include <vector>

#include "bg_core.h"
#include "../../include/bgx.h"

using namespace bg;

namespace {

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
};

// Enumerate the legal moves of (board in bv, player pl, roll) into `out`.
// Returns n_moves (truncated); *total = untruncated count; *ovf on overflow.
template <int LOG, typename SlotPtr>
__device__ __forceinline__ int run_movegen(int bv, int pl, int r0, int r1, uint64_t* out, int cap, SlotPtr tab,
                                           int cap_unique, int* total, bool* ovf, uint4* memo) {
    constexpr int slots = 1 << LOG;
    for (int i = lane_id(); i < slots; i += 64) tab[i] = make_uint4(0u, 0u, 0u, 0u);
    const bool dbl = r0 == r1;
    if (memo && dbl)
        for (int i = lane_id(); i < (2 << kLogMemo); i += 64) memo[i] = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    Gen<LOG, SlotPtr> g;
    g.tab = tab; g.out = out; g.cap = cap; g.pl = pl; g.cap_unique = cap_unique;
    g.memo2 = memo && dbl ? memo : nullptr;
    g.memo3 = memo && dbl ? memo + (1 << kLogMemo) : nullptr;
    uint32_t blocked;
    const Node s0 = node_from_bytes(bv, pl, blocked);
    g.blocked = blocked;
    g.run(s0, r0, r1);
    *ovf = g.ovf;
    *total = g.count;
    return g.count < cap ? g.count : cap;
}

// Roll + movegen + obs for one lane according to its `need` byte
// (reset: backgammon_env.py:78-113; pass/turn: :183-188 roll_dice + update_legal_moves).
template <int LOG>
__device__ __forceinline__ int advance_lane(int bv, int gi, const Args& A, uint4* lds_tab, uint4* lds_memo) {
    const int need = rd(bv, R_NEED);
    if (need == NEED_NONE) return bv;
    Rng rng;
    if (A.dice_mode == BGX_DICE_PHILOX) rng.init_philox(A.ctr[gi], A.key0, A.key1, (uint32_t)gi);
    else if (A.dice_mode == BGX_DICE_MT_LANE) rng.init_mt(A.mt + (size_t)gi * kMtWords, (uint32_t*)lds_tab);
    int r0, r1;
    if (need == NEED_RESET) {
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
    bv = wr(bv, R_ROLL0, r0);
    bv = wr(bv, R_ROLL1, r1);
    const int cur = rd(bv, R_CUR);
    int total;
    bool ovf;
    int n = run_movegen<LOG>(bv, cur, r0, r1, A.moves + (size_t)gi * A.max_moves, A.max_moves, lds_tab,
                             cap_fast<LOG>(), &total, &ovf, lds_memo);
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

// -------------------------------------------------------------- kernels --
// PHASE 0: apply + advance fused (per-lane dice); 1: apply only; 2: advance only.
template <int PHASE, int LOG>
__global__ __launch_bounds__(64) void k_step(Args A, const int32_t* actions, float* obs, float* reward, uint8_t* done,
                                             int32_t* info) {
    __shared__ uint4 tab[1 << LOG];
    __shared__ uint4 memo[2 << kLogMemo];
    const int gi = blockIdx.x;
    int bv = load_rec(A, gi);
    if (PHASE != 2) bv = apply_lane(bv, gi, (int)ufl((uint32_t)actions[gi]), A, reward, done, info);
    if (PHASE != 1) {
        bv = advance_lane<LOG>(bv, gi, A, tab, memo);
        if (obs) write_obs(bv, obs + (size_t)gi * 198);
    }
    store_rec(A, gi, bv);
}

template <int LOG>
__global__ __launch_bounds__(64) void k_reset(Args A, const uint8_t* lane_mask, float* obs, int mark_only) {
    __shared__ uint4 tab[1 << LOG];
    __shared__ uint4 memo[2 << kLogMemo];
    const int gi = blockIdx.x;
    int bv = load_rec(A, gi);
    const bool sel = lane_mask == nullptr || ufl(lane_mask[gi]) != 0u;
    if (sel) bv = wr(bv, R_NEED, NEED_RESET);
    if (!mark_only) {
        bv = advance_lane<LOG>(bv, gi, A, tab, memo);
        if (obs) write_obs(bv, obs + (size_t)gi * 198);
    }
    store_rec(A, gi, bv);
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
                                                int32_t* ovf_count, int32_t* ovf_queue) {
    __shared__ uint4 tab[1 << LOG];
    __shared__ uint4 memo[2 << kLogMemo];
    const int gi = blockIdx.x;
    const int l = lane_id();
    const int bv = l < 52 ? (int)boards[(size_t)gi * 52 + l] : 0;
    const int pl = (int)ufl(players[gi]);
    const int r0 = (int)ufl(dice[2 * gi]), r1 = (int)ufl(dice[2 * gi + 1]);
    int total;
    bool ovf;
    int nm = run_movegen<LOG>(bv, pl, r0, r1, moves + (size_t)gi * cap, cap, tab, cap_fast<LOG>(), &total, &ovf, memo);
    if (ovf) {
        if (l == 0) { const int q = atomicAdd(ovf_count, 1); ovf_queue[q] = gi; }
        nm = 0; total = 0;
    }
    if (l == 0) { nmoves[gi] = (int16_t)nm; if (ntotal) ntotal[gi] = total; }
}

// Slow path for positions whose dedup set outgrew the LDS table: same code,
// 2 MiB table in HBM per wave.  SRC 0 = engine lanes, 1 = standalone arrays.
template <int SRC>
__global__ __launch_bounds__(64) void k_movegen_slow(Args A, const int8_t* boards, const uint8_t* players,
                                                     const uint8_t* dice, int cap, int16_t* nmoves, int32_t* ntotal,
                                                     uint64_t* moves, uint4* tables) {
    __shared__ uint4 memo[2 << kLogMemo];
    uint4* tab = tables + ((size_t)blockIdx.x << kLogSlotsSlow);
    const int count = (int)ufl((uint32_t)*A.ovf_count);
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
        int nm = run_movegen<kLogSlotsSlow>(bv, pl, r0, r1, out, c, tab, kCapSlow, &total, &ovf, memo);
        if (ovf) { if (l == 0) atomicOr(A.err, 1); nm = 0; total = 0; }
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
    __shared__ uint4 memo[2 << kLogMemo];
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

thread_local std::string g_err;

int fail(hipError_t e, int code = BGX_EDEVICE) {
    g_err = hipGetErrorString(e);
    return code;
}

}  // namespace

struct bgx_engine {
    int device;
    int lds_log;      // 9 or 10
    Args a;
    uint4* slow_tables;
    int slow_waves;
    uint64_t seed;
};

#define CK(x) do { hipError_t _e = (x); if (_e != hipSuccess) return fail(_e); } while (0)
#define LAUNCH_LOG(e, K, grid, s, ...)                                                            \
    do {                                                                                          \
        if ((e)->lds_log == 9) hipLaunchKernelGGL(K<9>, grid, dim3(64), 0, s, __VA_ARGS__);       \
        else hipLaunchKernelGGL(K<10>, grid, dim3(64), 0, s, __VA_ARGS__);                        \
    } while (0)
#define CKL() do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return fail(_e); } while (0)

static int slow_path(bgx_engine* e, hipStream_t s, int src, const int8_t* boards, const uint8_t* players,
                     const uint8_t* dice, int cap, int16_t* nm, int32_t* nt, uint64_t* moves) {
    if (src == 0)
        hipLaunchKernelGGL(k_movegen_slow<0>, dim3(e->slow_waves), dim3(64), 0, s, e->a, boards, players, dice, cap,
                           nm, nt, moves, e->slow_tables);
    else
        hipLaunchKernelGGL(k_movegen_slow<1>, dim3(e->slow_waves), dim3(64), 0, s, e->a, boards, players, dice, cap,
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
    const char* ll = getenv("BGX_LDS_LOG");
    e->lds_log = (ll && atoi(ll) == 9) ? 9 : 10;
    Args& A = e->a;
    A.B = batch; A.max_moves = max_moves; A.dice_mode = dice_mode; A.auto_reset = auto_reset ? 1 : 0;
    A.match_length = match_length;
    A.key0 = (uint32_t)seed; A.key1 = (uint32_t)(seed >> 32);
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
    alloc((void**)&A.ovf_count, 16);
    alloc((void**)&A.ovf_queue, B * 4);
    alloc((void**)&A.err, 16);
    alloc((void**)&e->slow_tables, (size_t)kSlowWaves * ((size_t)16 << kLogSlotsSlow));
    if (err != hipSuccess) { bgx_engine_destroy(e); return fail(err, BGX_ENOMEM); }
    if (hipMemset(A.lanes, 0, B * 64) != hipSuccess || hipMemset(A.ctr, 0, B * 8) != hipSuccess ||
        hipMemset(A.ovf_count, 0, 16) != hipSuccess || hipMemset(A.err, 0, 16) != hipSuccess ||
        hipMemset(A.n_total, 0, B * 4) != hipSuccess) {
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

int bgx_engine_destroy(bgx_engine* e) {
    if (!e) return BGX_EINVAL;
    (void)hipSetDevice(e->device);
    Args& A = e->a;
    void* ptrs[] = {A.lanes, A.moves, A.n_total, A.mt, A.ctr, A.shared_rolls, A.ovf_count, A.ovf_queue, A.err,
                    e->slow_tables};
    for (void* p : ptrs) if (p) (void)hipFree(p);
    delete e;
    return BGX_OK;
}

int bgx_engine_seed(bgx_engine* e, const uint32_t* seeds_host, uint64_t philox_seed) {
    if (!e || !seeds_host) return BGX_EINVAL;
    CK(hipSetDevice(e->device));
    Args& A = e->a;
    A.key0 = (uint32_t)philox_seed; A.key1 = (uint32_t)(philox_seed >> 32);
    CK(hipMemset(A.ctr, 0, (size_t)A.B * 8));
    if (A.dice_mode == BGX_DICE_PHILOX) return BGX_OK;
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
    CK(hipMemsetAsync(A.ovf_count, 0, 16, s));
    if (A.dice_mode == BGX_DICE_MT_SHARED) {
        LAUNCH_LOG(e, k_reset, dim3(A.B), s, A, lane_mask_dev, obs_dev, 1);
        hipLaunchKernelGGL(k_shared_dice, dim3(1), dim3(64), 0, s, A);
        LAUNCH_LOG(e, k_reset, dim3(A.B), s, A, nullptr, obs_dev, 0);
    } else {
        LAUNCH_LOG(e, k_reset, dim3(A.B), s, A, lane_mask_dev, obs_dev, 0);
    }
    CKL();
    return slow_path(e, s, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr);
}

int bgx_step(bgx_engine* e, const int32_t* actions_dev, float* obs_dev, float* reward_dev, uint8_t* done_dev,
             int32_t* info_dev, void* stream) {
    if (!e || !actions_dev || !reward_dev || !done_dev) return BGX_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    Args& A = e->a;
    CK(hipSetDevice(e->device));
    CK(hipMemsetAsync(A.ovf_count, 0, 16, s));
    if (A.dice_mode == BGX_DICE_MT_SHARED) {
        hipLaunchKernelGGL((k_step<1, 9>), dim3(A.B), dim3(64), 0, s, A, actions_dev, obs_dev, reward_dev, done_dev,
                           info_dev);
        hipLaunchKernelGGL(k_shared_dice, dim3(1), dim3(64), 0, s, A);
        if (e->lds_log == 9)
            hipLaunchKernelGGL((k_step<2, 9>), dim3(A.B), dim3(64), 0, s, A, actions_dev, obs_dev, reward_dev, done_dev,
                               info_dev);
        else
            hipLaunchKernelGGL((k_step<2, 10>), dim3(A.B), dim3(64), 0, s, A, actions_dev, obs_dev, reward_dev,
                               done_dev, info_dev);
    } else {
        if (e->lds_log == 9)
            hipLaunchKernelGGL((k_step<0, 9>), dim3(A.B), dim3(64), 0, s, A, actions_dev, obs_dev, reward_dev, done_dev,
                               info_dev);
        else
            hipLaunchKernelGGL((k_step<0, 10>), dim3(A.B), dim3(64), 0, s, A, actions_dev, obs_dev, reward_dev,
                               done_dev, info_dev);
    }
    CKL();
    return slow_path(e, s, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr);
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
    CK(hipMemsetAsync(e->a.ovf_count, 0, 16, s));
    LAUNCH_LOG(e, k_movegen, dim3(n), s, boards52_dev, players_dev, dice_dev, n, max_moves, n_moves_dev, n_total_dev,
               moves_dev, e->a.ovf_count, e->a.ovf_queue);
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

int bgx_afterstates(bgx_engine* e, int32_t lane0, int32_t nlanes, int8_t* boards52_dev, void* stream) {
    if (!e || !boards52_dev || lane0 < 0 || nlanes < 0 || lane0 + nlanes > e->a.B) return BGX_EINVAL;
    if (nlanes == 0) return BGX_OK;
    CK(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_legal<0>, dim3(nlanes), dim3(64), 0, (hipStream_t)stream, e->a, lane0, (void*)boards52_dev);
    CKL();
    return BGX_OK;
}

int bgx_legal_features(bgx_engine* e, int32_t lane0, int32_t nlanes, float* out_dev, void* stream) {
    if (!e || !out_dev || lane0 < 0 || nlanes < 0 || lane0 + nlanes > e->a.B) return BGX_EINVAL;
    if (nlanes == 0) return BGX_OK;
    CK(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_legal<1>, dim3(nlanes), dim3(64), 0, (hipStream_t)stream, e->a, lane0, (void*)out_dev);
    CKL();
    return BGX_OK;
}

int bgx_action_masks(bgx_engine* e, int16_t* counts_dev, float* masks_dev, void* stream) {
    if (!e) return BGX_EINVAL;
    if (!counts_dev && !masks_dev) return BGX_OK;
    CK(hipSetDevice(e->device));
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
    if (lanes_dst) CK(hipMemcpyAsync(lanes_dst, A.lanes + (size_t)lane0 * 64, (size_t)n * 64, hipMemcpyDeviceToDevice, s));
    if (moves_dst)
        CK(hipMemcpyAsync(moves_dst, A.moves + (size_t)lane0 * A.max_moves, (size_t)n * A.max_moves * 8,
                          hipMemcpyDeviceToDevice, s));
    if (n_total_dst) CK(hipMemcpyAsync(n_total_dst, A.n_total + lane0, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    return BGX_OK;
}

int bgx_set_lanes(bgx_engine* e, int32_t lane0, int32_t n, const uint8_t* lanes_src, void* stream) {
    if (!e || !lanes_src || lane0 < 0 || n < 0 || lane0 + n > e->a.B) return BGX_EINVAL;
    if (n == 0) return BGX_OK;
    hipStream_t s = (hipStream_t)stream;
    Args& A = e->a;
    CK(hipSetDevice(e->device));
    CK(hipMemcpyAsync(A.lanes + (size_t)lane0 * 64, lanes_src, (size_t)n * 64, hipMemcpyDeviceToDevice, s));
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

const char* bgx_last_error(void) { return g_err.c_str(); }

}  // extern "C"
