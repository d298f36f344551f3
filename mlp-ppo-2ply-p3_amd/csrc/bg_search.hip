// bg_search.hip — 1-ply greedy and 2-ply expectimax over the 21 dice rolls
//  with the MLP value head (policy_network.py:54-56,72-75) on MFMA.
//
// 2-ply, per root lane (board, mover m, roll) with legal afterstates a_0..a_{n-1}:
//   Q(a) = sum_r p_r * min_{b in replies(a, r)} V(enc(b, m))       (leaf = a if no reply)
//   best = first argmax_a Q(a)
// Leaves are encoded with the ROOT mover's one-hot, as the reference's
// expectiminimax evaluates every node for the root player (expect_minmax.py:57-58,
// 100-143) and as the critic is trained (observation one-hot = player to move,
// backgammon_env.py:193-196: after the reply, m is to move); the opponent picks
// the reply that minimises m's value.
// 1-ply: V(enc(a, m)) for every afterstate (legal_board_features' one-hot), first
// argmax -- the same evaluator on the "no reply" leaf of each row.
// Work item ("job") = (afterstate row, roll r).  The pipeline is decoupled:
//   k_rows    one wave per row: the afterstate a as a 64-byte record + the
//             mover's side of a (16 B) for the evaluator;
//   k_enum    one wave per job (persistent, grid-stride): the opponent's replies
//             with the exact reference move generator (bg_core.h, LDS dedup +
//             revisit memo), each surviving-candidate afterstate KEY (16 B) and a
//             tag (job, sub-move count) streamed to an HBM leaf pool in 256-slot
//             blocks; three variants: non-doubles rolls (4 KiB of LDS, no doubles
//             code), doubles rolls (dedup table + memo), and an explicit job list;
//   k_enum_tier  jobs whose dedup set outgrew their table: 1,024- then 4,096-slot LDS tables;
//   k_enum_slow  jobs that outgrew that too, on 131,072-slot HBM tables;
//   k_eval    dense pass over the pool: features from (row side, key) as exact
//             f16 values, W1 split hi+lo on v_mfma_f32_32x32x16_f16, value head
//             in registers, segmented min per job + atomicMin into minv[job];
//   k_two_ply_reduce  Q(a) and the first argmax.
// 1-ply: k_scan, k_expand, k_rows (row keys), k_eval_rows (V per row), k_one_ply_reduce.
// The reference's filter_full_moves_by_max_submoves (get_all_moves.py:73-94) is
// applied by the evaluator: a leaf counts iff its sub-move count equals the
// job's final maximum (written at job end), which is exactly "first insertion
// of an afterstate had the maximal length" -- the surviving set.  A job whose
// pool allocation failed is re-run in a later round (a min over a subset of
// leaves plus the min over all of them is the min over all of them).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "bg_engine.h"
#include "bg_debug.h"

using namespace bg;

namespace {

// Work counters of the 2-ply enumerators (experiments, -DBGX_COUNTERS; tools/enum_counters.py):
// this file's own set, apart from bg_core.h's move-generator counters
#ifdef BGX_COUNTERS
__device__ unsigned long long g_scnt[16 * bg::kCntSlots];     // spread by workgroup (bg_core.h)
#define SC_CNT(i, v) do { if ((threadIdx.x & 63) == 0) \
    atomicAdd(&g_scnt[(i) * bg::kCntSlots + (blockIdx.x & (bg::kCntSlots - 1))], (unsigned long long)(v)); } while (0)
#define SC_T0(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#define SC_T1(i, t) SC_CNT(i, __builtin_amdgcn_s_memtime() - t)
#else
#define SC_CNT(i, v) do { } while (0)
#define SC_T0(t) do { } while (0)
#define SC_T1(i, t) do { } while (0)
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int kEvalWideWaves = 8, kEvalNarrowWaves = 4;   // waves per LDS-weight evaluator workgroup
constexpr int kKB = 13;            // 208 / 16 k-steps of v_mfma_f32_32x32x16_f16
constexpr int kSlowQueue = 1 << 20;
// Leaf-pool allocation block (slots): a wave claims kBlk slots with one atomic on the
// pool's single cursor.  That cursor is one address hit from all eight XCDs: at 256 slots
// (1.9 M claims per 65,536-root batch) the claims serialised the enumerators (23.7 ms
// per batch; 1,024: 19.0 ms; 4,096: 19.1 ms with 0.4 ms more evaluation of the wasted
// tails; profiles/r5/pool_block/)
#ifndef BGX_POOL_BLK
#define BGX_POOL_BLK 1024
#endif
constexpr int kBlk = BGX_POOL_BLK;
constexpr uint32_t kTagNone = 0xFFFFFFFFu;
constexpr int kLogLight = 8;       // non-doubles reply enumeration: 256-slot table (4 KiB)
constexpr int kMaxRounds = 256;

// get_all_dice_rolls_tensor (get_all_dice_rolls.py:5-34): (1,1),(1,2),...,(6,6)
__constant__ uint8_t kRoll0[21] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6};
__constant__ uint8_t kRoll1[21] = {1, 2, 3, 4, 5, 6, 2, 3, 4, 5, 6, 3, 4, 5, 6, 4, 5, 6, 5, 6, 6};
// The same in arithmetic (the enumerators' per-job path: a table read there is a
// dependent global load per job): roll r starts its first die's run at
// 7(r0-1) - (r0-1)r0/2; the 15 non-doubles in order as nibbles.
__host__ __device__ constexpr int roll_start(int r0) { return 7 * (r0 - 1) - (r0 - 1) * r0 / 2; }
__device__ __forceinline__ void roll_dice(int r, int& r0, int& r1) {
    r0 = 1 + (r >= 6) + (r >= 11) + (r >= 15) + (r >= 18) + (r >= 20);
    r1 = r - roll_start(r0) + r0;
}
constexpr uint64_t kNdR0 = 0x544333222211111ull, kNdR1 = 0x665654654365432ull;
__device__ __forceinline__ int nd_roll(int k) {     // k-th non-doubles roll index
    const int a = (int)((kNdR0 >> (4 * k)) & 15u), b = (int)((kNdR1 >> (4 * k)) & 15u);
    return roll_start(a) + b - a;
}

// Value net packed for MFMA (bgx_value_pack), in floats (H <= 128):
//                         hdr [4] (e1 as int bits), then NT = ceil(H/16) 16-unit
//                         slices.  Narrow form (NT <= 4): NT tiles of 16 hidden units
//                         with their hi AND lo parts in one 32-row MFMA tile (row m:
//                         unit 16t + (m&7) + 8(m>>4), part (m>>3)&1):
//     w1q [13][NT][64] x uint4   lane l: the 8 f16 of row l&31 at k = kperm(kb, l>>5, i),
//                                i = 0..7, of W1s = [W1 | b1] * 2^e1 (the two `off`
//                                columns divided by 15; b1 rides a constant-1 feature)
//     wvq [NT][8][64] f32        value_head.weight[unit(t, j, l)] * 2^-e1 for the
//                                accumulator pair (r, r+4), r = j < 4 ? j : j + 4
//                         Wide form (NT > 4): NW = ceil(NT/2) tiles of 32 units, the
//                         hi and lo parts as two k-blocks of the same accumulator:
//     w1q [13][NW][2][64] x uint4  lane l: row unit 32T + (l&31), part 0 = hi, 1 = lo
//     wvq [NW][4][64][4] f32     value_head.weight[32T + 8(r>>2) + 4(l>>5) + (r&3)] * 2^-e1
//                                for accumulator register r of lane l (at [T][r>>2][l][r&3])
// The features are then exact small integers / halves in f16, so one hi and one
// lo MFMA product give fp32-grade accuracy: narrow, hi + lo of a unit are summed
// from two accumulator registers of the same lane; wide, the accumulator sums them.
__host__ __device__ constexpr bool wide_tiles(int NT) { return NT > 4; }
__host__ __device__ constexpr int slices(int NT) { return wide_tiles(NT) ? (NT + 1) & ~1 : NT; }
__host__ __device__ inline int sz_f16(int NT) { return 4 + kKB * slices(NT) * 64 * 4 + slices(NT) * 8 * 64; }

constexpr int kFeatBias = -2;
// Permuted K order of the f16 section: k-blocks 0-5 = P1 points, 6-11 = P2 points;
// lane half h of block kb holds points 2pp, 2pp+1 with pp = 2(kb%6) + h, as
// [u0(a), u0(b), u1(a), u1(b), u2(a), u2(b), u3(a), u3(b)] (point pairs packed for
// u16x2 arithmetic); block 12 = [bar1, off1, bar2, off2, onehot0, onehot1, 1 (bias), 0]
// on h = 0.  Returns the reference feature index (immutable_board.py:171-212),
// kFeatBias or -1 (pad).
__host__ __device__ inline int kperm(int kb, int h, int i) {
    if (kb < 12) {
        const int P = kb / 6, pp = 2 * (kb % 6) + h, point = 2 * pp + (i & 1);
        return 98 * P + 4 * point + (i >> 1);
    }
    if (h) return -1;
    const int ex[8] = {96, 97, 194, 195, 196, 197, kFeatBias, -1};
    return ex[i];
}

__device__ __forceinline__ float wave_min(float v) {
    #pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}

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

// ------------------------------------------------------------------ 2-ply --
struct S2 {
    const uint8_t* rowrec;            // [rows][64]: afterstate bytes 0..51, byte 52 = replier q
    int32_t row0, row1;               // rows of this launch (implicit-job variants)
    uint4* keys;                      // leaf pool [cap]
    uint32_t* tags;                   // [cap] job | len << 29, kTagNone = unused slot
    unsigned long long* cursor;       // next free pool slot (kBlk granularity; may run past cap)
    unsigned long long cap;
    uint8_t* maxlen;                  // [jobs] final max sub-move count (0xFF = not finished)
    unsigned long long* leaves;       // surviving-leaf counter (stats)
    int32_t* qcount;                  // [kTiers] overflow queues: 0 -> 1,024-slot LDS tier,
    int32_t* queues;                  // [kTiers][kSlowQueue]   1 -> 4,096-slot LDS tier, 2 -> HBM tier
    int32_t* retry_count;
    int32_t* retry_list;              // [jobs]
    const int32_t* list;              // explicit job list (variant 2)
    const int32_t* list_count;
    int32_t* err;
    int cap_light, cap_heavy, cap_mid;   // unique-entry capacity of the LDS tables (tests shrink them)
    int memo_mask, memo_share;           // revisit memo at depth 2 (bit 0) / 3 (bit 1); in-table share /8
    int bar_rows;                        // nd_row_bar on (tests turn it off: BGX_2PLY_BARROW=0)
};

__device__ __forceinline__ unsigned long long bcast64(unsigned long long v) {
    return (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
           ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}

// Gen sink of the reply enumeration: every entry of the current maximal length
// goes to the leaf pool as (key, job | len << 29); the wave owns a kBlk-slot
// block at a time (one atomic per block).  On pool exhaustion the job is `lost`
// (re-run next round); its leaves already written stay valid candidates.
struct KeySink {
    static constexpr bool kEnc = false;    // keys only: the move encodings are dead
    static constexpr bool kSet = true;     // the SET of afterstates (min over replies): order is free
    uint4* keys;
    uint32_t* tags;
    unsigned long long* cursor;
    unsigned long long cap;
    unsigned long long blk;
    int fill;
    uint32_t job;
    bool lost;

    __device__ __forceinline__ void reset() {}

    __device__ __forceinline__ void push_lanes(uint64_t m, const Node& t, uint64_t, int, int len) {
        if (lost) return;
        const int n = __popcll(m);
        const int l = threadIdx.x & 63;
        const bool on = (m >> l) & 1ull;
        int p = fill + lane_rank(m);
        unsigned long long b = blk;
        if (fill + n > kBlk) {
            unsigned long long nb = 0;
            if (l == 0) nb = atomicAdd(cursor, (unsigned long long)kBlk);
            nb = bcast64(nb);
            if (nb + kBlk > cap) { lost = true; return; }
            if (p >= kBlk) { b = nb; p -= kBlk; }
            blk = nb;
            fill = fill + n - kBlk;
        } else {
            fill += n;
        }
        if (on) {
            keys[b + p] = make_uint4((uint32_t)t.lo, (uint32_t)(t.lo >> 32), t.hi, t.k3);
            tags[b + p] = job | ((uint32_t)len << 29);
        }
    }
    __device__ __forceinline__ void push(const Node& s, uint64_t enc, int idx, int len) {
        push_lanes(1ull, s, enc, idx, len);
    }
    // push_lanes with the job given per lane (the row-level walk, nd_row)
    __device__ __forceinline__ void push_lanes_job(uint64_t m, const Node& t, uint32_t job_lane, int len) {
        if (lost) return;
        const int n = __popcll(m);
        const int l = threadIdx.x & 63;
        const bool on = (m >> l) & 1ull;
        int p = fill + lane_rank(m);
        unsigned long long b = blk;
        if (fill + n > kBlk) {
            unsigned long long nb = 0;
            if (l == 0) nb = atomicAdd(cursor, (unsigned long long)kBlk);
            nb = bcast64(nb);
            if (nb + kBlk > cap) { lost = true; return; }
            if (p >= kBlk) { b = nb; p -= kBlk; }
            blk = nb;
            fill = fill + n - kBlk;
        } else {
            fill += n;
        }
        if (on) {
            keys[b + p] = make_uint4((uint32_t)t.lo, (uint32_t)(t.lo >> 32), t.hi, t.k3);
            tags[b + p] = job_lane | ((uint32_t)len << 29);
        }
    }
    // mark the unused tail of the wave's current block
    __device__ __forceinline__ void finish() {
        for (int i = fill + (threadIdx.x & 63); i < kBlk; i += 64) tags[blk + i] = kTagNone;
    }
};

// One (row, roll) job.  KIND 0: non-doubles roll, 1: doubles roll, 2: either.
// Returns 0 done, 1 LDS/HBM table overflow, 2 pool exhausted.
// MK: revisit memo kind (-1 none, 0 separate depth-2/3 tables, 1 one combined table,
// 2 tagged entries inside the dedup table itself).
template <int LOG, typename SlotPtr, int MK, int KIND>
__device__ __forceinline__ int enum_job(const S2& S, int job, int r, int q, const Node& sq, uint32_t blocked,
                                        SlotPtr tab, int cap_unique, uint4* memo, KeySink& sink,
                                        unsigned long long& leaves) {
    int r0, r1;
    roll_dice(r, r0, r1);
    const int l = lane_id();
    const bool dbl = KIND == 1 || (KIND == 2 && r0 == r1);
    Gen<LOG, SlotPtr, KeySink, MK < 0 ? 0 : MK> g;     // clears its table (and memo) when needed
    g.tab = tab; g.pl = q; g.cap_unique = cap_unique; g.blocked = blocked;
    if (MK == 2) memo = (uint4*)tab;    // non-null: pruning on (entries live in tab)
    g.memo2 = MK >= 0 && dbl && (S.memo_mask & 1) ? memo : nullptr;
    g.memo3 = MK >= 0 && dbl && (S.memo_mask & 2) ? (MK == 1 ? memo : memo + (1 << kLogMemo2)) : nullptr;
    g.memo_share = S.memo_share;
    g.sink = sink;
    g.sink.job = (uint32_t)job;
    g.sink.lost = false;
    if (KIND == 0) g.run_nd(sq, r0, r1);
    else if (KIND == 1) {
        SC_T0(tdd);
        g.run_d(sq, r0);
        if ((sq.k3 & 15u) != 0u) { SC_CNT(7, 1); SC_T1(15, tdd); }
        else if (g.pure_walk) { SC_CNT(2, 1); SC_T1(14, tdd); }
        else SC_T1(0, tdd);
    }
    else g.run(sq, r0, r1);
    if (!g.ovf && g.count == 0) g.sink.push(sq, 0ull, 0, 0);     // no reply: the leaf is a itself
    sink = g.sink;
    if (g.ovf) return 1;
    if (sink.lost) return 2;
    if (l == 0) S.maxlen[job] = (uint8_t)g.cur_max;
    leaves += (unsigned long long)(g.count ? g.count : 1);
    return 0;
}

// All 15 non-doubles rolls of a row whose replier has checkers on the bar (round 5; the
// counters put 44 % of C4's rows here, and the light enumerator spent most of its wave time
// in their 15 per-job walks, each clearing and probing a dedup table).  The first sub-move
// of either die order is the bar entry, and no bear-off can follow (an entered checker
// stands outside its home), so nd_both's paths (handle_non_doubles + the skip rule,
// get_all_moves.py:33-53) reduce to closed cases, table-free:
// * two or more on the bar: both entries open -> one leaf (both orders give the same
//   afterstate), length 2; only one open -> that entry, length 1 (pass 1's single ends the
//   walk, or pass 1 is empty and pass 2 has it); none -> no reply (the leaf is a itself);
// * one on the bar, e(d) the entry point of die d: with e(hi) open and a lo-move after
//   it, family A = enter hi then any lo-move (the entered checker included) and family B =
//   enter lo then any hi-move, length 2.  Within a family the sources differ, so the
//   states do; across them the count changes {+e(hi), -c, +(c+lo)} and {+e(lo), -c',
//   +(c'+hi)} agree only for the chain through the entry points (c = e(hi), c' = e(lo):
//   both end at e(hi) + lo = e(lo) + hi), and then the states are equal iff neither entry
//   point held a blot (the hit sets differ otherwise): the set is A plus B without that
//   chain when it repeats A's.  e(hi) open but no lo-move after it: pass 1's single entry
//   ends the walk (the skip rule), length 1.  e(hi) blocked: family B (length 2), or the
//   lo entry alone (length 1), or no reply.
// Lane l < 24: A's child from point l; lane 32 + l: B's.
__device__ __forceinline__ uint32_t nd_row_bar(const S2& S, int row, const Node& s0, int q, uint32_t blocked,
                                               KeySink& sink, unsigned long long& leaves) {
    const int l = lane_id();
    const int bar = (int)(s0.k3 & 15u);
    const uint32_t job0 = (uint32_t)row * 21u;
    uint32_t open = 0u;                              // dice whose entry point is open
    #pragma unroll
    for (int d = 1; d <= 6; ++d) open |= ((blocked >> entry_point(q, d)) & 1u) ? 0u : 1u << d;
    const Kids kbar{1u << 31, kBar};
    unsigned long long emitted = 0;
    if (bar >= 2) {
        // lane k < 15: the k-th non-doubles roll; one leaf per roll
        int lo = 1, hi = 2;
        const int r = l < 15 ? nd_roll(l) : 0;
        if (l < 15) roll_dice(r, lo, hi);
        const bool oh = (open >> hi) & 1u, ol = (open >> lo) & 1u;
        Node leaf = s0;
        if (oh) leaf = apply(leaf, child(leaf, kbar, 31, hi, q), q);
        if (ol) leaf = apply(leaf, child(leaf, kbar, 31, lo, q), q);
        const int len = (int)oh + (int)ol;
        const bool on = l < 15;
        #pragma unroll
        for (int n = 0; n <= 2; ++n) {              // the pool tag carries the length
            const uint64_t em = __ballot(on && len == n);
            if (em) sink.push_lanes_job(em, leaf, job0 + (uint32_t)r, n);
        }
        if (on && !sink.lost) S.maxlen[job0 + (uint32_t)r] = (uint8_t)len;
        emitted = 15;
    } else {
        const int half = l >> 5, b = l & 31;
        #pragma unroll 1
        for (int k = 0; k < 15; ++k) {
            const int r = nd_roll(k);
            int lo, hi;
            roll_dice(r, lo, hi);
            const bool oh = (open >> hi) & 1u, ol = (open >> lo) & 1u;
            Node th = s0, tl = s0;
            uint32_t qa = 0u, qb = 0u;
            if (oh) { th = apply(s0, child(s0, kbar, 31, hi, q), q); qa = gen(th, lo, q, blocked).bits; }
            if (ol) { tl = apply(s0, child(s0, kbar, 31, lo, q), q); qb = gen(tl, hi, q, blocked).bits; }
            int len;
            if (oh && !qa) {                         // pass 1's single entry, the skip rule
                len = 1;
                if (!sink.lost) sink.push_lanes_job(1ull, th, job0 + (uint32_t)r, 1);
                emitted += 1;
            } else if (!oh && !qb) {                 // pass 2's single entry, or no reply
                len = ol ? 1 : 0;
                if (!sink.lost) sink.push_lanes_job(1ull, ol ? tl : s0, job0 + (uint32_t)r, len);
                emitted += 1;
            } else {
                len = 2;
                if (!oh) qa = 0u;
                const int eh = entry_point(q, hi), el = entry_point(q, lo);
                if (((qa >> eh) & 1u) && ((qb >> el) & 1u) && !((s0.blot >> eh) & 1u) && !((s0.blot >> el) & 1u))
                    qb &= ~(1u << el);                                   // B's chain repeats A's
                const uint32_t mk = half ? qb : qa;
                const bool act = b < 24 && ((mk >> b) & 1u);
                Node leaf = s0;
                if (act) {
                    const Node& par = half ? tl : th;
                    leaf = apply(par, child(par, Kids{mk, -1}, b, half ? hi : lo, q), q);
                }
                const uint64_t em = __ballot(act);
                sink.push_lanes_job(em, leaf, job0 + (uint32_t)r, 2);
                emitted += (unsigned long long)__popcll(em);
            }
            if (l == 0 && !sink.lost) S.maxlen[job0 + (uint32_t)r] = (uint8_t)len;
        }
    }
    SC_CNT(6, 1);
    if (!sink.lost) leaves += emitted;
    return 0u;
}

// All 15 non-doubles rolls of one row in one pass (the 2-ply's set semantics):
// the first sub-moves of all six dice on the lanes (die d_l, source a_l), each
// lane's second-level child lists for the five other dice, then the two-steps of
// every roll as flat 64-lane chunks, one per second die -- instead of 15 jobs that
// each rebuild two first levels and run their own chunks.  Only for rows without
// bar entries or bear-offs (no bar, >= 2 checkers off the home board), where
// Gen::nd_both decides every two-step without a table (pure, or the first of a
// chain / reverse / pass-2 family: nd_first_of); a roll whose pass 1 has no
// two-step (the sequential singles semantics), and every roll of any other row,
// is left to the per-job walk.  Returns the mask of roll indices (0..20) left.
__device__ __forceinline__ uint32_t nd_row(const S2& S, int row, const Node& s0, int q, uint32_t blocked,
                                           KeySink& sink, unsigned long long& leaves) {
    constexpr uint32_t kAllNd = 0x000B77BEu;        // the 15 non-doubles roll indices
    const int off = (int)((s0.k3 >> 4) & 15u);
    SC_CNT(1, 1);
    if ((s0.k3 & 15u) != 0u && S.bar_rows) return nd_row_bar(S, row, s0, q, blocked, sink, leaves);
    if ((s0.k3 & 15u) != 0u || 15 - s0.n_home - off < 2) { SC_CNT(3, 1); return kAllNd; }
    const int l = lane_id();
    uint32_t K[7];
    int st[8];
    st[1] = 0;
    #pragma unroll
    for (int d = 1; d <= 6; ++d) {
        K[d] = gen(s0, d, q, blocked).bits;
        st[d + 1] = st[d] + __popc(K[d]);
    }
    const int n1 = st[7];
    if (n1 > 64) { SC_CNT(3, 1); return kAllNd; }
    // lane l: first sub-move (die dl, source al)
    const bool act = l < n1;
    int dl = 1;
    #pragma unroll
    for (int d = 2; d <= 6; ++d) dl = l >= st[d] ? d : dl;
    uint32_t kd = K[1];
    #pragma unroll
    for (int d = 2; d <= 6; ++d) kd = dl == d ? K[d] : kd;
    int kst = 0;
    #pragma unroll
    for (int d = 1; d <= 6; ++d) kst = dl == d ? st[d] : kst;
    const int al = act ? select_bit(kd, l - kst) : 0;
    Node t1 = s0;
    uint32_t Q[7];
    Q[0] = 0u;
    if (act) {
        const Kids k{kd, -1};
        t1 = apply(s0, child(s0, k, al, dl, q), q);
    }
    #pragma unroll
    for (int e = 1; e <= 6; ++e) Q[e] = act && e != dl ? gen(t1, e, q, blocked).bits : 0u;
    // roll (hi, lo) is fast iff its pass 1 (hi first) has a two-step
    uint64_t M[7], N[7];
    #pragma unroll
    for (int d = 1; d <= 6; ++d) { M[d] = __ballot(act && dl == d); N[d] = __ballot(Q[d] != 0u); }
    uint32_t slow = 0u;
    #pragma unroll
    for (int hi = 2; hi <= 6; ++hi)
        #pragma unroll
        for (int lo = 1; lo < hi; ++lo)
            if (!(M[hi] & N[lo])) slow |= 1u << (roll_start(lo) + hi - lo);
    const int sg = q == 0 ? 1 : -1;
    const uint32_t root_occ = s0.occ, root_blot = s0.blot;
    const uint32_t job0 = (uint32_t)row * 21u;
    unsigned long long emitted = 0;
    #pragma unroll 1
    for (int e = 1; e <= 6; ++e) {
        // this lane's two-steps with second die e: pass 1 of roll (dl, e) if dl > e,
        // pass 2 of roll (e, dl) if dl < e (only its chain child)
        const int hi = dl > e ? dl : e, lo = dl > e ? e : dl;
        const int r = roll_start(lo) + hi - lo;
        uint32_t c = Q[e];
        if (dl < e) c &= 1u << (al + sg * dl);
        if (!act || dl == e || ((slow >> r) & 1u)) c = 0u;
        const uint32_t cnt = (uint32_t)__popc(c);
        uint32_t pre = 0, total = 0;
        const uint64_t below = (1ull << l) - 1ull;
        #pragma unroll
        for (int b = 0; b < 5; ++b) {
            const uint64_t m = __ballot((cnt >> b) & 1u);
            pre += (uint32_t)__popcll(m & below) << b;
            total += (uint32_t)__popcll(m) << b;
        }
        const int meta = al | (dl << 5) | (r << 8);
        SC_CNT(5, (total + 63) / 64);
        for (uint32_t ch = 0; ch < total; ch += 64) {
            const uint32_t pp = ch + (uint32_t)l;
            const bool valid = pp < total;
            const int src = parent_of(pp, pre + cnt);
            const uint32_t qb = (uint32_t)__shfl((int)c, src);
            const int j = (int)(pp - (uint32_t)__shfl((int)pre, src));
            const Node s1 = shfl_node(t1, src);
            const int mt = __shfl(meta, src);
            const int pa = mt & 31, pd = (mt >> 5) & 7, pr = mt >> 8;
            Node leaf = s1;
            bool emit = false;
            if (valid) {
                const int cb = select_bit(qb, j);
                const Kids k{qb, -1};
                const Sub m = child(s1, k, cb, e, q);
                leaf = apply(s1, m, q);
                if (pd > e) {               // pass 1: (pa, hi = pd) then (cb, lo = e)
                    const int dst_a = pa + sg * pd;
                    const bool chain = cb == dst_a, rev = m.dst == pa;
                    emit = (!chain && !rev) ||
                           nd_first_of(chain ? pa : cb, chain ? 1 : 2, e, pd, q, root_occ, root_blot, blocked);
                } else {                    // pass 2: (pa, lo = pd) then its chain (cb, hi = e)
                    emit = nd_first_of(pa, 3, pd, e, q, root_occ, root_blot, blocked);
                }
            }
            const uint64_t em = __ballot(valid && emit);
            sink.push_lanes_job(em, leaf, job0 + (uint32_t)pr, 2);
            emitted += (unsigned long long)__popcll(em);
        }
    }
    // every fast roll has a first pass-1 two-step (emitted): max length 2
    const uint32_t fast = kAllNd & ~slow;
    SC_CNT(4, __popc(slow));
    SC_CNT(13, emitted);
    if (l < 21 && ((fast >> l) & 1u) && !sink.lost) S.maxlen[job0 + (uint32_t)l] = 2;
    if (!sink.lost) leaves += emitted;
    return slow;
}

// The replier's node of row `row` (its 64-byte record, one byte per lane).
__device__ __forceinline__ Node row_node(int bv, int& q, uint32_t& blocked) {
    q = rd(bv, 52);
    return node_from_bytes(bv, q, blocked);
}

// job by its id alone (explicit lists, overflow tiers)
template <int LOG, typename SlotPtr, int MK>
__device__ __forceinline__ int enum_job_id(const S2& S, int job, SlotPtr tab, int cap_unique, uint4* memo,
                                           KeySink& sink, unsigned long long& leaves) {
    const int row = job / 21;
    int q;
    uint32_t blocked;
    const Node sq = row_node((int)S.rowrec[(size_t)row * 64 + lane_id()], q, blocked);
    return enum_job<LOG, SlotPtr, MK, 2>(S, job, job - row * 21, q, sq, blocked, tab, cap_unique, memo, sink, leaves);
}

__device__ __forceinline__ void queue_job(int32_t* count, int32_t* list, int cap, int job, int32_t* overflow_count,
                                          int32_t* overflow_list) {
    if (lane_id() != 0) return;
    const int i = atomicAdd(count, 1);
    if (i < cap) { list[i] = job; return; }
    atomicSub(count, 1);
    overflow_list[atomicAdd(overflow_count, 1)] = job;
}

__device__ __forceinline__ KeySink make_sink(const S2& S) {
    KeySink k;
    k.keys = S.keys; k.tags = S.tags; k.cursor = S.cursor; k.cap = S.cap;
    k.blk = 0; k.fill = kBlk; k.job = 0; k.lost = false;
    return k;
}

// VARIANT 0: jobs (row, non-doubles roll) implicit, 1: (row, doubles roll)
// implicit, 2: the explicit list, 3: as 0 with the row-level walk (nd_row) first.
template <int LOG, int MK, int VARIANT, int WPE = 1>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_enum(S2 S) {
    __shared__ uint4 tab[1 << LOG];
    __shared__ uint4 memo_[MK == 0 ? kMemoSlots : (MK == 1 ? (1 << kLogCMemo) : 1)];
    uint4* memo = MK >= 0 ? memo_ : nullptr;
    KeySink sink = make_sink(S);
    unsigned long long leaves = 0;
    const int cap = VARIANT == 0 || VARIANT == 3 ? S.cap_light : S.cap_heavy;
    auto done = [&](int st, int job) {
        if (st == 1) {
            const int qo = LOG < 10 ? 0 : 1;
            queue_job(S.qcount + qo, S.queues + (size_t)qo * kSlowQueue, kSlowQueue, job, S.retry_count, S.retry_list);
        } else if (st == 2) {
            queue_job(S.retry_count, S.retry_list, 0x7FFFFFFF, job, S.retry_count, S.retry_list);
        }
    };
    if (VARIANT == 2) {
        const int n = *S.list_count;
        for (int i = blockIdx.x; i < n; i += gridDim.x) {
            const int job = S.list[i];
            done(enum_job_id<LOG, uint4*, MK>(S, job, tab, cap, memo, sink, leaves), job);
        }
    } else {
        // one row at a time: its 15 non-doubles (VARIANT 0) or 6 doubles rolls share
        // the replier's node; the next row's record is loaded behind this row's work
        int row = S.row0 + blockIdx.x;
        int bv = row < S.row1 ? (int)S.rowrec[(size_t)row * 64 + lane_id()] : 0;
        for (; row < S.row1; row += gridDim.x) {
            const int nrow = row + gridDim.x < S.row1 ? row + gridDim.x : row;
            const int bv_next = (int)S.rowrec[(size_t)nrow * 64 + lane_id()];
            int q;
            uint32_t blocked;
            const Node sq = row_node(bv, q, blocked);
            if (VARIANT == 3) {
                // the row-level walk; what it leaves (and a lost pool block: the
                // whole row again) runs per job
                SC_T0(t0);
                uint32_t left = nd_row(S, row, sq, q, blocked, sink, leaves);
                SC_T1(9, t0);
                if (sink.lost) left = 0x000B77BEu;
                SC_T0(t1);
                #pragma unroll 1
                for (; left; left &= left - 1u) {
                    const int r = __builtin_ctz(left);
                    const int job = row * 21 + r;
                    SC_CNT(11, 1);
                    done(enum_job<LOG, uint4*, MK, 0>(S, job, r, q, sq, blocked, tab, cap, memo, sink, leaves), job);
                }
                SC_T1(10, t1);
            } else {
                constexpr int nr = VARIANT == 0 ? 15 : 6;
                SC_T0(t2);
                #pragma unroll 1
                for (int k = 0; k < nr; ++k) {
                    const int r = VARIANT == 0 ? nd_roll(k) : roll_start(k + 1);
                    const int job = row * 21 + r;
                    done(enum_job<LOG, uint4*, MK, VARIANT>(S, job, r, q, sq, blocked, tab, cap, memo, sink, leaves),
                         job);
                }
                SC_T1(12, t2);
            }
            bv = bv_next;
        }
    }
    sink.finish();
    if (lane_id() == 0 && leaves) atomicAdd(S.leaves, leaves);
}

// Overflow tiers in LDS: queue QI (jobs whose dedup set outgrew their table) on a
// 2^LOG-slot table; what outgrows it too goes to queue QI + 1.
constexpr int kLogMid = 12;
template <int LOG, int QI>
__global__ __launch_bounds__(64) void k_enum_tier(S2 S) {
    __shared__ uint4 tab[1 << LOG];
    __shared__ uint4 memo[kMemoSlots];
    KeySink sink = make_sink(S);
    unsigned long long leaves = 0;
    const int n = min(S.qcount[QI], kSlowQueue);
    const int32_t* qin = S.queues + (size_t)QI * kSlowQueue;
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int job = qin[i];
        const int st = enum_job_id<LOG, uint4*, 0>(S, job, tab, min(S.cap_mid, cap_fast<LOG>()), memo,
                                                   sink, leaves);
        if (st == 1) queue_job(S.qcount + QI + 1, S.queues + (size_t)(QI + 1) * kSlowQueue, kSlowQueue, job,
                               S.retry_count, S.retry_list);
        else if (st == 2) queue_job(S.retry_count, S.retry_list, 0x7FFFFFFF, job, S.retry_count, S.retry_list);
    }
    sink.finish();
    if (lane_id() == 0 && leaves) atomicAdd(S.leaves, leaves);
}

// Tier 2: a 131,072-slot HBM table per wave.
__global__ __launch_bounds__(64) void k_enum_slow(S2 S, uint4* tables) {
    __shared__ uint4 memo[kMemoSlots];
    uint4* tab = tables + ((size_t)blockIdx.x << kLogSlotsSlow);
    KeySink sink = make_sink(S);
    unsigned long long leaves = 0;
    const int n = min(S.qcount[2], kSlowQueue);
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int job = S.queues[2 * (size_t)kSlowQueue + i];
        const int st = enum_job_id<kLogSlotsSlow, uint4*, 0>(S, job, tab, kCapSlow, memo, sink, leaves);
        if (st == 1 && lane_id() == 0) atomicOr(S.err, 1);
        else if (st == 2) queue_job(S.retry_count, S.retry_list, 0x7FFFFFFF, job, S.retry_count, S.retry_list);
    }
    sink.finish();
    if (lane_id() == 0 && leaves) atomicAdd(S.leaves, leaves);
}

// The afterstate of every row (root lane, legal move a): 64-byte record for the
// enumerators and the mover's side of a (nibbles, bar, off, replier q) for k_eval;
// rowkey (1-ply, may be null): the replier's side of a as a leaf key (no hits) --
// the row's "no reply" leaf.  The row count comes from *nrows (k_scan's total).
// A row whose (lane, move index) is not a legal move of the lane as it stands now -- the
// lanes changed between k_scan and this kernel, which the engine's stream ordering rules
// out (bgx.h) -- sets *bad and becomes the empty board's row instead of reading past the
// lane's move list.
__global__ __launch_bounds__(256) void k_rows(Args A, const int32_t* row_lane, const int32_t* lane_off,
                                              const int64_t* nrows, uint8_t* rowrec, uint4* rowside, uint4* rowkey,
                                              int32_t* bad) {
    const int l = lane_id();
    const int nw = gridDim.x * (blockDim.x >> 6);
    const int rows = (int)*nrows;
    for (int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); row < rows; row += nw) {
        const int lane_g = row_lane[row];
        bool ok = lane_g >= 0 && lane_g < A.B;
        const int a = ok ? row - lane_off[lane_g] : 0;
        int bv = ok ? load_rec(A, lane_g) : 0;
        if (ok) {
            const int n = rd(bv, R_NM0) | (rd(bv, R_NM1) << 8);
            ok = a >= 0 && a < n && a < A.max_moves;
        }
        if (!ok) {
            if (l == 0) atomicOr(bad, 2);
            bv = 0;
        }
        const int mover = rd(bv, R_CUR);
        const uint64_t m = ok ? uload64(A.moves + (size_t)lane_g * A.max_moves + a) : 0ull;
        uint32_t blocked;
        Node s = node_from_bytes(bv, mover, blocked);
        s = apply_move(s, m, mover);
        const int bva = bytes_from_node(bv, s, mover);
        const int q = 1 - mover;
        if (rowrec) rowrec[(size_t)row * 64 + l] = (uint8_t)(l < 52 ? bva : (l == 52 ? q : 0));
        if (rowkey) {
            uint32_t bq;
            const Node sq = node_from_bytes(bva, q, bq);
            if (l == 0) rowkey[row] = make_uint4((uint32_t)sq.lo, (uint32_t)(sq.lo >> 32), sq.hi, sq.k3 & 0xFFu);
        }
        if (l == 0)
            rowside[row] = make_uint4((uint32_t)s.lo, (uint32_t)(s.lo >> 32), s.hi,
                                      (s.k3 & 15u) | (((s.k3 >> 4) & 15u) << 4) | ((uint32_t)q << 8));
    }
}

// ---- leaf evaluation on f16 MFMA ----
// bit i of x (i < 16) -> bit 4i
__device__ __forceinline__ uint64_t spread4(uint32_t x) {
    uint64_t v = x & 0xFFFFu;
    v = (v | (v << 24)) & 0x000000FF000000FFull;
    v = (v | (v << 12)) & 0x000F000F000F000Full;
    v = (v | (v << 6)) & 0x0303030303030303ull;
    v = (v | (v << 3)) & 0x1111111111111111ull;
    return v;
}

struct Leaf {
    uint64_t lo[2];    // P1, P2 point counts 0..15 (nibbles)
    uint32_t hi[2];    // points 16..23
    uint32_t bar[2], off[2];
    int q, job;
    bool valid;
    uint32_t hits;     // the root mover's blots the reply hit (bit p = point p)
    int row;           // the leaf's row (its job's, 0 for an unused slot)
};

struct EvalArgs {
    const uint4* keys;
    const uint32_t* tags;
    const unsigned long long* lo;     // pool range [*lo, min(*hi, cap)) of this launch
    const unsigned long long* hi;
    unsigned long long cap;
    const uint4* rowside;
    const uint8_t* maxlen;
    int32_t* minv;                    // [jobs] ordered-int encoding of the min
    const uint4* w1q;
    const float* wvq;
    float bv;
    const float* rowpart;             // [rows][16 slices] the root mover's part of X1 per row (k_rowpart)
    float* vdbg;                      // test hook (BGX_2PLY_DUMP): V per pool slot, else null
};

struct LeafRaw { uint4 key; uint32_t tag; };
struct LeafRow { uint4 rs; uint32_t ml; };

__device__ __forceinline__ LeafRaw load_raw(const EvalArgs& E, unsigned long long i) {
    return LeafRaw{E.keys[i], E.tags[i]};
}
__device__ __forceinline__ LeafRow load_row(const EvalArgs& E, const LeafRaw& r) {
    const int job = r.tag != kTagNone ? (int)(r.tag & 0x1FFFFFFFu) : 0;
    return LeafRow{E.rowside[job / 21], (uint32_t)E.maxlen[job]};
}

// Both sides of the reply afterstate: the replier q's from the key, the root
// mover's = its side of a minus the blots q hit (a hit point held exactly one).
// The one-hot is the root mover's, 1 - q (feat16).
__device__ __forceinline__ Leaf make_leaf(const LeafRaw& r, const LeafRow& w) {
    const uint4 key = r.key, rs = w.rs;
    Leaf L;
    const bool used = r.tag != kTagNone;
    L.valid = used && w.ml == (r.tag >> 29);
    L.job = L.valid ? (int)(r.tag & 0x1FFFFFFFu) : -1;
    L.row = used ? (int)(r.tag & 0x1FFFFFFFu) / 21 : 0;
    const uint32_t hits = key.w >> 8;
    L.hits = L.valid ? hits : 0u;
    const uint64_t mlo = (((uint64_t)rs.y << 32) | rs.x) - spread4(hits & 0xFFFFu);
    const uint32_t mhi = rs.z - (uint32_t)spread4(hits >> 16);
    const uint32_t mbar = (rs.w & 15u) + (uint32_t)__builtin_popcount(hits), moff = (rs.w >> 4) & 15u;
    const uint64_t qlo = ((uint64_t)key.y << 32) | key.x;
    const uint32_t qhi = key.z, qbar = key.w & 15u, qoff = (key.w >> 4) & 15u;
    L.q = (int)((rs.w >> 8) & 1u);
    const bool q0 = L.q == 0;
    L.lo[0] = q0 ? qlo : mlo;  L.lo[1] = q0 ? mlo : qlo;
    L.hi[0] = q0 ? qhi : mhi;  L.hi[1] = q0 ? mhi : qhi;
    L.bar[0] = q0 ? qbar : mbar;  L.bar[1] = q0 ? mbar : qbar;
    L.off[0] = q0 ? qoff : moff;  L.off[1] = q0 ? moff : qoff;
    return L;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));

// (a, b) small non-negative integers (< 1024) -> the f16 pair (a*s0, b*s1) exactly:
// 1024 + k is an f16 with unit spacing, so (bits(k) | 0x6400) - 1024 == k.
__device__ __forceinline__ uint32_t f16_pair(uint32_t ab, float s0, float s1) {
    const h16x2 t = __builtin_bit_cast(h16x2, ab | 0x64006400u);
    const h16x2 sc = {(_Float16)s0, (_Float16)s1};
    const h16x2 r = t * sc - (h16x2){(_Float16)(1024.0f * s0), (_Float16)(1024.0f * s1)};
    return __builtin_bit_cast(uint32_t, r);
}

// the four units of two points with counts (a, b) (immutable_board.py:180-195) as
// f16 pairs [u_k(a), u_k(b)], k = 0..3: n>=1, n>=2, n>=3, (n-3)/2 if n>=3.
// t = (1024 + a, 1024 + b) in f16 (unit spacing there, so every step is exact):
// u_k = clamp01(t - 1024 - k) for k < 3, u_3 = max(t/2 - 513.5, 0).  Written with
// builtins (round 5): hipcc folds min(max(x, 0), 1) into the VOP3P clamp bit, so this is
// the same five instructions (3 v_pk_add_f16 clamp, v_pk_fma_f16, v_pk_max_f16) as the
// round-3/4 inline-asm block, and the hazard recognizer now sees every one of them (the
// asm string hid them; it was not the cause of the two-tiles-in-flight fault: see
// eval_tile_wide).
__device__ __forceinline__ h16x2 clamp01h(h16x2 x) {
    return __builtin_elementwise_min(__builtin_elementwise_max(x, (h16x2){0, 0}), (h16x2){1, 1});
}
__device__ __forceinline__ uint4 units_pair(uint32_t byte) {
    uint32_t tb = (byte & 15u) | ((byte & 0xF0u) << 12) | 0x64006400u;
    // an empty asm (no instruction, so no hazard) pins where the units are formed: without
    // it the scheduler hoists the features of later k-blocks and k_eval<3> / k_eval<8>
    // spill 22 / 14 VGPRs
    __asm__ volatile("" : "+v"(tb));
    const h16x2 t = __builtin_bit_cast(h16x2, tb);
    constexpr _Float16 k0 = -1024.0f, k1 = -1025.0f, k2 = -1026.0f, k3 = -513.5f;
    const h16x2 u0 = clamp01h(t + (h16x2){k0, k0});
    const h16x2 u1 = clamp01h(t + (h16x2){k1, k1});
    const h16x2 u2 = clamp01h(t + (h16x2){k2, k2});
    const h16x2 u3 = __builtin_elementwise_max(t * (h16x2){0.5f16, 0.5f16} + (h16x2){k3, k3}, (h16x2){0, 0});
    return make_uint4(__builtin_bit_cast(uint32_t, u0), __builtin_bit_cast(uint32_t, u1),
                      __builtin_bit_cast(uint32_t, u2), __builtin_bit_cast(uint32_t, u3));
}

// the two point counts (nibbles) k-block kb < 12 takes from this lane's half h:
// points 4 k6 + 2h, +1 = byte (2 k6 + h) of the player's 96-bit nibble vector
__device__ __forceinline__ uint32_t side_byte(uint64_t lo, uint32_t hi, int k6, int h) {
    const uint32_t dw = k6 < 2 ? (uint32_t)lo : (k6 < 4 ? (uint32_t)(lo >> 32) : hi);
    return (dw >> (16 * (k6 & 1) + 8 * h)) & 0xFFu;
}
__device__ __forceinline__ uint32_t kb_byte(const Leaf& L, int kb, int h) {
    const int P = kb / 6, k6 = kb % 6;
    return side_byte(L.lo[P], L.hi[P], k6, h);
}

// B operand of k-block kb for this lane's half h (permuted K order, kperm)
__device__ __forceinline__ f16x8 feat16(const Leaf& L, int kb, int h) {
    uint4 v;
    if (kb < 12) {
        v = units_pair(kb_byte(L, kb, h));
    } else if (h == 0) {
        v = make_uint4(f16_pair(L.bar[0] | (L.off[0] << 16), 0.5f, 1.0f),
                       f16_pair(L.bar[1] | (L.off[1] << 16), 0.5f, 1.0f),
                       L.q == 1 ? 0x3C00u : 0x3C000000u, 0x3C00u);     // one-hot of the root mover 1 - q
    } else {
        v = make_uint4(0u, 0u, 0u, 0u);
    }
    return __builtin_bit_cast(f16x8, v);
}

__device__ __forceinline__ int ord_f32(float v) {
    const int b = __float_as_int(v);
    return b >= 0 ? b : b ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float unord_f32(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

// V of 2 x 32 leaves (column c = lane & 31 of tile n; both lane halves return it):
// X1s = [W1 | b1]s . [F | 1]^T on v_mfma_f32_32x32x16_f16, one MFMA per (k-block,
// 16 hidden units, 32 leaves) -- the units' hi and lo weight parts sit in rows m
// and m+8 of the same tile (accumulator registers r and r+4 of a lane) -- then
// V = sum wv 2^-e1 relu(hi + lo) + bv.  The weight fragments come from LDS (wq,
// wvs) and are shared by the two leaf tiles.  At most 4 unit tiles (64 units) are
// accumulated per pass (2 x 4 x 16 accumulator VGPRs); H = 128 takes two passes
// over K, regenerating the features.  `z` = an opaque zero offset that keeps the
// LDS fragment reads inside the loops.
// relu as one v_max_i32 on the float's bits (a negative float is a negative int;
// fmaxf would first canonicalize the MFMA result with a second v_max_f32, and inline
// asm would hide the MFMA-result read from the hazard recognizer, which must pad it)
__device__ __forceinline__ float relu_raw(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

// Wide tiles (H > 64) in the unfactored form (no row parts), one leaf tile of 32 columns
// at a time.  The factored form (eval_leaves_fact, the C4 path) keeps two leaf tiles in
// flight.  Round 4's wrong values with two tiles in flight (columns 16-31 of one tile,
// 0.01-0.1 % of leaves, varying from run to run) came from packed-fp32 FMAs that LLVM's
// SLP vectorizer formed across the two tiles' value heads (v_pk_fma_f32 broadcasting the
// odd head weights with op_sel:[0,1,0], an instruction form no other kernel here uses);
// bg_search.hip is built without SLP vectorization (__graft_entry__.SOURCE_FLAGS) and the
// two-tile form is exact on every leaf.
template <int NT>
__device__ __forceinline__ float eval_tile_wide(const uint4* wq, const float* wvs, const Leaf& L, int z, float bias) {
    constexpr int NW = slices(NT) / 2;
    const int l = lane_id(), h = l >> 5;
    f32x16 x[NW];
    #pragma unroll
    for (int kb = 0; kb < kKB; ++kb) {
        const f16x8 f = feat16(L, kb, h);
        #pragma unroll
        for (int t = 0; t < NW; ++t) {
            const f16x8 ah = __builtin_bit_cast(f16x8, wq[((kb * NW + t) * 2 + 0) * 64 + l + z]);
            const f16x8 al = __builtin_bit_cast(f16x8, wq[((kb * NW + t) * 2 + 1) * 64 + l + z]);
            x[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, f, kb == 0 ? (f32x16){} : x[t], 0, 0, 0);
            x[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, f, x[t], 0, 0, 0);
        }
    }
    // value head: relu times the head weights, 4 registers' weights per ds_read_b128
    float a = 0.0f;
    #pragma unroll
    for (int t = 0; t < NW; ++t)
        #pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
            const float4 w = reinterpret_cast<const float4*>(wvs)[(t * 4 + r4) * 64 + l + z];
            a = fmaf(relu_raw(x[t][4 * r4 + 0]), w.x, a);
            a = fmaf(relu_raw(x[t][4 * r4 + 1]), w.y, a);
            a = fmaf(relu_raw(x[t][4 * r4 + 2]), w.z, a);
            a = fmaf(relu_raw(x[t][4 * r4 + 3]), w.w, a);
        }
    return a + __shfl_xor(a, 32) + bias;
}

template <int NT>
__device__ __forceinline__ void eval_leaves_wide(const uint4* wq, const float* wvs, const Leaf (&L)[2], int z,
                                                 float bias, float (&v)[2]) {
    v[0] = eval_tile_wide<NT>(wq, wvs, L[0], z, bias);
    __builtin_amdgcn_sched_barrier(0);              // the tiles stay apart (not interleaved)
    int z1 = z;                                     // opaque: the second tile re-reads its fragments
    __asm__ volatile("" : "+s"(z1));
    v[1] = eval_tile_wide<NT>(wq, wvs, L[1], z1, bias);
}

template <int NT>
__device__ __forceinline__ void eval_leaves(const uint4* wq, const float* wvs, const Leaf (&L)[2], int z, float bias,
                                            float (&v)[2]) {
    if constexpr (wide_tiles(NT)) {
        eval_leaves_wide<NT>(wq, wvs, L, z, bias, v);
        return;
    }
    constexpr int G = NT < 4 ? NT : 4;
    const int l = lane_id(), h = l >> 5;
    v[0] = 0.0f;
    v[1] = 0.0f;
    // passes kept apart (not unrolled): interleaved, two passes' accumulators spill
    #pragma unroll 1
    for (int g0 = 0; g0 < NT; g0 += G) {
        f32x16 x[2][G];
        #pragma unroll
        for (int kb = 0; kb < kKB; ++kb) {
            const f16x8 f0 = feat16(L[0], kb, h), f1 = feat16(L[1], kb, h);
            #pragma unroll
            for (int t = 0; t < G; ++t) {
                if (g0 + t < NT) {
                    const f16x8 a = __builtin_bit_cast(f16x8, wq[(kb * NT + g0 + t) * 64 + l + z]);
                    const f32x16 c0 = kb == 0 ? (f32x16){} : x[0][t];
                    const f32x16 c1 = kb == 0 ? (f32x16){} : x[1][t];
                    x[0][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, f0, c0, 0, 0, 0);
                    x[1][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, f1, c1, 0, 0, 0);
                }
            }
        }
        #pragma unroll
        for (int n = 0; n < 2; ++n)
            #pragma unroll
            for (int t = 0; t < G; ++t)
                if (g0 + t < NT)
                    #pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int r = j < 4 ? j : j + 4;
                        v[n] = fmaf(fmaxf(x[n][t][r] + x[n][t][r + 4], 0.0f), wvs[((g0 + t) * 8 + j) * 64 + l + z],
                                    v[n]);
                    }
    }
    #pragma unroll
    for (int n = 0; n < 2; ++n) v[n] += __shfl_xor(v[n], 32) + bias;
}

// ---- round 4: the evaluator factored by row ----
// X1 = W1s . f is linear in f, and a leaf's features are the replier's points (from
// its key), block 12 (bars, offs, one-hot, bias) and the ROOT MOVER's points -- which
// are the same for every leaf of a row (root, move a) except at the mover's blots the
// reply hit (count 1 -> 0: u0 goes from 1 to 0, the other three units stay 0).  So
// k_rowpart computes the mover's part of X1 once per row (its 6 point k-blocks, hi +
// lo, fp32 accumulation) and a leaf pair starts its accumulators from it (C = rowpart
// of each column's row), then runs the replier's 6 point k-blocks, block 12, and --
// only for the mover k-blocks that hold a hit point of some leaf of the pair -- that
// block's weights against the hit delta (-1 at u0 of each hit point): 7 + (hit
// blocks) of the 13 k-blocks.  Which blocks are the replier's depends on q, so the
// pair's valid leaves must share q (rows are laid out grouped by replier, k_scan);
// a pair that mixes them takes the full 13-block form (eval_leaves).
__device__ __forceinline__ f16x8 hit_delta(uint32_t hits, int k6, int h) {
    const uint32_t b = (hits >> (4 * k6 + 2 * h)) & 3u;      // points 4 k6 + 2h, +1: elements 0, 1 (u0)
    return __builtin_bit_cast(f16x8, make_uint4((b & 1u ? 0xBC00u : 0u) | (b & 2u ? 0xBC000000u : 0u), 0u, 0u, 0u));
}

// mask of the mover k-blocks (4 points each) that hold a hit point of any lane, wave-uniform
__device__ __forceinline__ uint32_t hit_blocks(uint32_t hits) {
    uint32_t m = 0u;
    #pragma unroll
    for (int k6 = 0; k6 < 6; ++k6) m |= __ballot((hits >> (4 * k6)) & 15u) ? 1u << k6 : 0u;
    return m;
}

// what the factored form needs of a leaf: the replier's nibbles, the block-12 operand,
// the hit mask and the row
struct FLeaf {
    uint64_t rlo;
    uint32_t rhi;
    uint32_t b12;      // bar0 | off0 << 8 | bar1 << 16 | off1 << 24 | q << 31
    uint32_t hits;
    int row;
};
__device__ __forceinline__ FLeaf fleaf(const Leaf& L) {
    FLeaf F;
    F.rlo = L.q ? L.lo[1] : L.lo[0];
    F.rhi = L.q ? L.hi[1] : L.hi[0];
    F.b12 = L.bar[0] | (L.off[0] << 8) | (L.bar[1] << 16) | (L.off[1] << 24) | ((uint32_t)L.q << 31);
    F.hits = L.hits;
    F.row = L.row;
    return F;
}
// feat16(L, 12, h) from the packed form
__device__ __forceinline__ f16x8 feat12(uint32_t b, int h) {
    const uint32_t p1 = (b & 0xFFu) | ((b & 0xFF00u) << 8), p2 = ((b >> 16) & 0xFFu) | ((b >> 8) & 0x0F0000u);
    const uint4 v = make_uint4(f16_pair(p1, 0.5f, 1.0f), f16_pair(p2, 0.5f, 1.0f), b >> 31 ? 0x3C00u : 0x3C000000u,
                               0x3C00u);
    return __builtin_bit_cast(f16x8, h ? make_uint4(0u, 0u, 0u, 0u) : v);
}

template <int NT, int NN>
__device__ __forceinline__ void eval_leaves_fact(const uint4* wq, const float* wvs, const FLeaf* L, int z,
                                                 float bias, const float* rowpart, int q, float* v) {
    constexpr bool kWide = wide_tiles(NT);
    constexpr int NA = kWide ? slices(NT) / 2 : NT;      // accumulator tiles per 32 leaves
    constexpr int HP = 16 * slices(NT);                  // rowpart row stride (floats)
    const int l = lane_id(), h = l >> 5;
    f32x16 x[NN][NA];
    // narrow: the row parts are loaded first and added after the MFMAs (their latency hidden
    // behind them; 15.9 vs 31.5 ms per C4 batch at H = 40); wide: they start the accumulators
    // (30.6 vs 31.4 ms at H = 128)
    constexpr bool kLate = !kWide;
    float4 rpv[NN][NA][kWide ? 4 : 2];
    if constexpr (kLate) {
    #pragma unroll
    for (int n = 0; n < NN; ++n) {
        const float4* rp = reinterpret_cast<const float4*>(rowpart + (size_t)L[n].row * HP + 4 * h);
        #pragma unroll
        for (int t = 0; t < NA; ++t)
            #pragma unroll
            for (int j = 0; j < (kWide ? 4 : 2); ++j) rpv[n][t][j] = rp[(kWide ? 32 * t + 8 * j : 16 * t + 8 * j) / 4];
    }
    } else {
    #pragma unroll
    for (int n = 0; n < NN; ++n) {
        const float4* rp = reinterpret_cast<const float4*>(rowpart + (size_t)L[n].row * HP + 4 * h);
        #pragma unroll
        for (int t = 0; t < NA; ++t) {
            if constexpr (kWide) {           // register 4j + i <- unit 32t + 8j + 4h + i
                #pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float4 a = rp[(32 * t + 8 * j) / 4];
                    x[n][t][4 * j + 0] = a.x; x[n][t][4 * j + 1] = a.y;
                    x[n][t][4 * j + 2] = a.z; x[n][t][4 * j + 3] = a.w;
                }
            } else {                         // hi rows: r 0-3 <- unit 16t + 4h + r, r 8-11 <- 16t + 8 + 4h + r - 8
                const float4 a = rp[(16 * t) / 4], b = rp[(16 * t + 8) / 4];
                x[n][t] = (f32x16){a.x, a.y, a.z, a.w, 0.0f, 0.0f, 0.0f, 0.0f, b.x, b.y, b.z, b.w, 0.0f, 0.0f, 0.0f, 0.0f};
            }
        }
    }
    }
    auto block = [&](int kb, const f16x8 (&f)[NN], bool first) {
        #pragma unroll
        for (int t = 0; t < NA; ++t) {
            if constexpr (kWide) {
                const f16x8 ah = __builtin_bit_cast(f16x8, wq[((kb * NA + t) * 2 + 0) * 64 + l + z]);
                const f16x8 al = __builtin_bit_cast(f16x8, wq[((kb * NA + t) * 2 + 1) * 64 + l + z]);
                #pragma unroll
                for (int n = 0; n < NN; ++n) {
                    x[n][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, f[n], first ? (f32x16){} : x[n][t], 0, 0, 0);
                    x[n][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, f[n], x[n][t], 0, 0, 0);
                }
            } else {
                const f16x8 a = __builtin_bit_cast(f16x8, wq[(kb * NT + t) * 64 + l + z]);
                #pragma unroll
                for (int n = 0; n < NN; ++n)
                    x[n][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, f[n], first ? (f32x16){} : x[n][t], 0, 0, 0);
            }
        }
    };
    // the replier's points (each column's own replier: a column of the other replier in
    // this pass is discarded by the caller), then block 12
    #pragma unroll
    for (int j = 0; j < 6; ++j) {
        f16x8 f[NN];
        #pragma unroll
        for (int n = 0; n < NN; ++n) f[n] = __builtin_bit_cast(f16x8, units_pair(side_byte(L[n].rlo, L[n].rhi, j, h)));
        block(6 * q + j, f, kLate && j == 0);
    }
    {
        f16x8 f[NN];
        #pragma unroll
        for (int n = 0; n < NN; ++n) f[n] = feat12(L[n].b12, h);
        block(12, f, false);
    }
    // the hit deltas, per mover k-block that holds a hit point of the leaves (wave-uniform test)
    const int P = 1 - q;
    uint32_t hall = 0u;
    #pragma unroll
    for (int n = 0; n < NN; ++n) hall |= L[n].hits;
    #pragma unroll 1
    for (uint32_t hb = hit_blocks(hall); hb; hb &= hb - 1u) {
        const int k6 = __builtin_ctz(hb);
        f16x8 f[NN];
        #pragma unroll
        for (int n = 0; n < NN; ++n) f[n] = hit_delta(L[n].hits, k6, h);
        block(6 * P + k6, f, false);
    }
    if constexpr (kLate)
    #pragma unroll
    for (int n = 0; n < NN; ++n)
        #pragma unroll
        for (int t = 0; t < NA; ++t)
            #pragma unroll
            for (int j = 0; j < (kWide ? 4 : 2); ++j) {
                const int r0 = kWide ? 4 * j : 8 * j;     // wide: regs 4j..; narrow: hi regs 0-3, 8-11
                x[n][t][r0 + 0] += rpv[n][t][j].x; x[n][t][r0 + 1] += rpv[n][t][j].y;
                x[n][t][r0 + 2] += rpv[n][t][j].z; x[n][t][r0 + 3] += rpv[n][t][j].w;
            }
    if constexpr (kWide) {
        float a[NN];
        #pragma unroll
        for (int n = 0; n < NN; ++n) a[n] = 0.0f;
        #pragma unroll
        for (int t = 0; t < NA; ++t)
            #pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const float4 w = reinterpret_cast<const float4*>(wvs)[(t * 4 + r4) * 64 + l + z];
                #pragma unroll
                for (int n = 0; n < NN; ++n) {
                    a[n] = fmaf(relu_raw(x[n][t][4 * r4 + 0]), w.x, a[n]);
                    a[n] = fmaf(relu_raw(x[n][t][4 * r4 + 1]), w.y, a[n]);
                    a[n] = fmaf(relu_raw(x[n][t][4 * r4 + 2]), w.z, a[n]);
                    a[n] = fmaf(relu_raw(x[n][t][4 * r4 + 3]), w.w, a[n]);
                }
            }
        #pragma unroll
        for (int n = 0; n < NN; ++n) v[n] = a[n] + __shfl_xor(a[n], 32) + bias;
    } else {
        #pragma unroll
        for (int n = 0; n < NN; ++n) v[n] = 0.0f;
        #pragma unroll
        for (int n = 0; n < NN; ++n)
            #pragma unroll
            for (int t = 0; t < NT; ++t)
                #pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int r = j < 4 ? j : j + 4;
                    v[n] = fmaf(fmaxf(x[n][t][r] + x[n][t][r + 4], 0.0f), wvs[(t * 8 + j) * 64 + l + z], v[n]);
                }
        #pragma unroll
        for (int n = 0; n < NN; ++n) v[n] += __shfl_xor(v[n], 32) + bias;
    }
}

// rowpart[row][u] = sum over the root mover's 12 x 4 point features of (W1s hi + lo)[u]
// x feature, fp32 accumulation, for every row (the mover's side of a from rowside, no
// hits; the replier's side zero, so all 12 point k-blocks can run whatever the mover).
// Units in the evaluators' accumulator order: narrow unit 16t + (r & 3) + 4h + 8(r >> 3)
// is hi register r + lo register r + 4 of tile t; wide unit 32t + 8(r >> 2) + 4h + (r & 3).
template <int NT>
__global__ __launch_bounds__(256) void k_rowpart(const uint4* rowside, const int64_t* nrows, const uint4* w1q,
                                                 float* rowpart) {
    constexpr bool kWide = wide_tiles(NT);
    constexpr int NA = kWide ? slices(NT) / 2 : NT, HP = 16 * slices(NT);
    const int l = lane_id(), h = l >> 5, c = l & 31;
    const long long rows = *nrows;
    const long long tiles = (rows + 31) / 32;
    for (long long tile = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); tile < tiles;
         tile += (long long)gridDim.x * 4) {
        const long long r = tile * 32 + c;
        const bool in = r < rows;
        const uint4 rs = in ? rowside[r] : make_uint4(0u, 0u, 0u, 0u);
        const int P = 1 - (int)((rs.w >> 8) & 1u);
        Leaf L{};
        L.lo[P] = ((uint64_t)rs.y << 32) | rs.x;
        L.hi[P] = rs.z;
        f32x16 x[NA];
        // rows are grouped by replier (k_scan by_mover): a tile of one mover runs only its
        // 6 point k-blocks (the replier's contribute exact zeros), a mixed tile all 12
        const uint64_t pm = __ballot(in && P == 1), pz = __ballot(in && P == 0);
        const int kb0 = pm == 0 ? 0 : (pz == 0 ? 6 : 0), kb1 = pz == 0 ? 12 : (pm == 0 ? 6 : 12);
        #pragma unroll 1
        for (int kb = kb0; kb < kb1; ++kb) {
            const f16x8 f = __builtin_bit_cast(f16x8, units_pair(kb_byte(L, kb, h)));
            #pragma unroll
            for (int t = 0; t < NA; ++t) {
                if constexpr (kWide) {
                    const f16x8 ah = __builtin_bit_cast(f16x8, w1q[((kb * NA + t) * 2 + 0) * 64 + l]);
                    const f16x8 al = __builtin_bit_cast(f16x8, w1q[((kb * NA + t) * 2 + 1) * 64 + l]);
                    x[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, f, kb == kb0 ? (f32x16){} : x[t], 0, 0, 0);
                    x[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, f, x[t], 0, 0, 0);
                } else {
                    const f16x8 a = __builtin_bit_cast(f16x8, w1q[(kb * NT + t) * 64 + l]);
                    x[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, f, kb == kb0 ? (f32x16){} : x[t], 0, 0, 0);
                }
            }
        }
        if (!in) continue;
        float* out = rowpart + (size_t)r * HP + 4 * h;
        #pragma unroll
        for (int t = 0; t < NA; ++t) {
            if constexpr (kWide) {
                #pragma unroll
                for (int j = 0; j < 4; ++j)
                    *reinterpret_cast<float4*>(out + 32 * t + 8 * j) =
                        make_float4(x[t][4 * j], x[t][4 * j + 1], x[t][4 * j + 2], x[t][4 * j + 3]);
            } else {
                *reinterpret_cast<float4*>(out + 16 * t) =
                    make_float4(x[t][0] + x[t][4], x[t][1] + x[t][5], x[t][2] + x[t][6], x[t][3] + x[t][7]);
                *reinterpret_cast<float4*>(out + 16 * t + 8) =
                    make_float4(x[t][8] + x[t][12], x[t][9] + x[t][13], x[t][10] + x[t][14], x[t][11] + x[t][15]);
            }
        }
    }
}

// workgroup shape of the evaluators: 4 waves (NT <= 4: <= 52 KiB of weights in LDS,
// several workgroups per CU) or 8 waves (H = 128: 120 KiB, one workgroup per CU,
// two waves per SIMD)
template <int NT> struct EvalShape {
    static constexpr int kWaves = NT <= 4 ? kEvalNarrowWaves : kEvalWideWaves;
};

template <int NT>
__device__ __forceinline__ void stage_weights(uint4* wq, float* wvs, const uint4* w1q, const float* wvq) {
    for (int i = threadIdx.x; i < kKB * slices(NT) * 64; i += blockDim.x) wq[i] = w1q[i];
    for (int i = threadIdx.x; i < slices(NT) * 8 * 64; i += blockDim.x) wvs[i] = wvq[i];
    __syncthreads();
}

// 2-ply: pool tiles of 64 leaves; per job the min over its leaves (leaves of a job
// are contiguous in the pool): segmented min over each 32-column tile, one
// atomicMin per job segment.  Workgroups share the packed weights in LDS; every
// wave walks its own tiles with the next tile's pool entries in flight during the
// current tile's MFMAs.
template <int NT>
__global__ __launch_bounds__(64 * EvalShape<NT>::kWaves) __attribute__((amdgpu_waves_per_eu(2)))
void k_eval(EvalArgs E) {
    constexpr int W = EvalShape<NT>::kWaves;
    __shared__ uint4 wq[kKB * slices(NT) * 64];
    __shared__ float wvs[slices(NT) * 8 * 64];
    const int l = lane_id(), h = l >> 5, c = l & 31;
    stage_weights<NT>(wq, wvs, E.w1q, E.wvq);
    const unsigned long long used = *E.hi < E.cap ? *E.hi : E.cap;
    const unsigned long long tiles = used / 64;
    const unsigned long long stride = (unsigned long long)gridDim.x * W;
    unsigned long long tile = *E.lo / 64 + (unsigned long long)blockIdx.x * W + (threadIdx.x >> 6);
    if (tile >= tiles) return;
    LeafRaw raw[2];
    LeafRow row[2];
    #pragma unroll
    for (int n = 0; n < 2; ++n) { raw[n] = load_raw(E, tile * 64 + 32 * n + c); row[n] = load_row(E, raw[n]); }
    // the next tile's pool entries are loaded behind the current tile's MFMAs, except at
    // H = 128 (two leaf tiles' 128 accumulators: the prefetch registers would spill)
    constexpr bool kPrefetch = !wide_tiles(NT);
    for (; tile < tiles; tile += stride) {
        Leaf L[2];
        if constexpr (!kPrefetch) {
            #pragma unroll
            for (int n = 0; n < 2; ++n) { raw[n] = load_raw(E, tile * 64 + 32 * n + c); row[n] = load_row(E, raw[n]); }
        }
        #pragma unroll
        for (int n = 0; n < 2; ++n) L[n] = make_leaf(raw[n], row[n]);
        int z = 0;
        __asm__ volatile("" : "+s"(z));
        if constexpr (kPrefetch) {
            const unsigned long long nxt = tile + stride < tiles ? tile + stride : tile;
            #pragma unroll
            for (int n = 0; n < 2; ++n) raw[n] = load_raw(E, nxt * 64 + 32 * n + c);
        }
        float v[2];
        if (E.rowpart) {
            // the factored form once per replier among the pair's valid leaves (wave-uniform;
            // rows grouped by replier make two rare), so a leaf's V never depends on its pair
            const uint64_t b1 = __ballot((L[0].valid && L[0].q) || (L[1].valid && L[1].q));
            const uint64_t b0 = __ballot((L[0].valid && !L[0].q) || (L[1].valid && !L[1].q));
            v[0] = v[1] = 0.0f;
            const FLeaf F[2] = {fleaf(L[0]), fleaf(L[1])};
            #pragma unroll 1
            for (int qq = b0 ? 0 : 1; qq <= (b1 ? 1 : 0); ++qq) {
                float w[2];
                int zq = z;                               // opaque per pass: no LDS read hoisted out
                __asm__ volatile("" : "+s"(zq));
#ifdef BGX_WIDE_SINGLE
                if constexpr (wide_tiles(NT)) {         // experiment: one leaf tile at a time
                    eval_leaves_fact<NT, 1>(wq, wvs, &F[0], zq, E.bv, E.rowpart, qq, &w[0]);
                    __builtin_amdgcn_sched_barrier(0);
                    int zr = zq;
                    __asm__ volatile("" : "+s"(zr));
                    eval_leaves_fact<NT, 1>(wq, wvs, &F[1], zr, E.bv, E.rowpart, qq, &w[1]);
                } else
#endif
                {
                    eval_leaves_fact<NT, 2>(wq, wvs, F, zq, E.bv, E.rowpart, qq, w);
                }
                #pragma unroll
                for (int n = 0; n < 2; ++n) v[n] = L[n].q == qq ? w[n] : v[n];
            }
        } else {
            eval_leaves<NT>(wq, wvs, L, z, E.bv, v);
        }
        if constexpr (kPrefetch) {
            #pragma unroll
            for (int n = 0; n < 2; ++n) row[n] = load_row(E, raw[n]);
        }
        if (E.vdbg && h == 0) {
            E.vdbg[tile * 64 + c] = v[0];
            E.vdbg[tile * 64 + 32 + c] = v[1];
        }
        #pragma unroll
        for (int n = 0; n < 2; ++n) {
            const int jb = L[n].job;
            float vv = L[n].valid ? v[n] : INFINITY;
            // segmented min over equal-job runs of the 32 columns (lanes 0..31 == 32..63)
            #pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
                const float v2 = __shfl_down(vv, o, 32);
                const int j2 = __shfl_down(jb, o, 32);
                if (c + o < 32 && j2 == jb) vv = fminf(vv, v2);
            }
            const int jp = __shfl_up(jb, 1, 32);
            if (h == 0 && jb >= 0 && (c == 0 || jp != jb)) atomicMin(E.minv + jb, ord_f32(vv));
        }
    }
}

// 1-ply: V of every row's afterstate (the row's "no reply" leaf: rowkey + rowside),
// 64 rows per tile, grid-stride over ceil(*nrows / 64) tiles.
struct EvalRowsArgs {
    const uint4* rowkey;
    const uint4* rowside;
    const int64_t* nrows;
    float* vrow;
    const uint4* w1q;
    const float* wvq;
    float bv;
};

template <int NT>
__global__ __launch_bounds__(64 * EvalShape<NT>::kWaves) void k_eval_rows(EvalRowsArgs E) {
    constexpr int W = EvalShape<NT>::kWaves;
    __shared__ uint4 wq[kKB * slices(NT) * 64];
    __shared__ float wvs[slices(NT) * 8 * 64];
    const int l = lane_id(), h = l >> 5, c = l & 31;
    stage_weights<NT>(wq, wvs, E.w1q, E.wvq);
    const long long rows = *E.nrows;
    const long long tiles = (rows + 63) / 64;
    for (long long tile = (long long)blockIdx.x * W + (threadIdx.x >> 6); tile < tiles;
         tile += (long long)gridDim.x * W) {
        Leaf L[2];
        #pragma unroll
        for (int n = 0; n < 2; ++n) {
            const long long r = tile * 64 + 32 * n + c;
            const bool in = r < rows;
            const LeafRaw raw{in ? E.rowkey[r] : make_uint4(0u, 0u, 0u, 0u), in ? 0u : kTagNone};
            const LeafRow rw{in ? E.rowside[r] : make_uint4(0u, 0u, 0u, 0u), 0u};
            L[n] = make_leaf(raw, rw);
        }
        int z = 0;
        __asm__ volatile("" : "+s"(z));
        float v[2];
        eval_leaves<NT>(wq, wvs, L, z, E.bv, v);
        #pragma unroll
        for (int n = 0; n < 2; ++n) {
            const long long r = tile * 64 + 32 * n + c;
            if (h == 0 && r < rows) E.vrow[r] = v[n];
        }
    }
}

// The first argmax of one lane's row values, one wave per lane: lane j of the wave takes
// rows j, j + 64, ... (value(a) by the caller's functor), keeps its first strict maximum,
// then a wave reduction by (larger value, then smaller index) -- the sequential scan's
// "first a with the largest value" (values that never beat -inf, NaN included, never win;
// then the choice is 0 as in the scan).  Round 3 ran one thread per lane: at C2's
// B = 4,096 that was 16 workgroups walking ~20-500 rows each (38 us of a 186 us step).
template <typename F>
__device__ __forceinline__ void wave_first_argmax(int n, F value, int& best, float& bestv) {
    float bv = -INFINITY;
    int ba = 0x7FFFFFFF;
    for (int a = lane_id(); a < n; a += 64) {
        const float x = value(a);
        if (x > bv) { bv = x; ba = a; }
    }
    #pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float v2 = __shfl_xor(bv, o);
        const int a2 = __shfl_xor(ba, o);
        if (v2 > bv || (v2 == bv && a2 < ba)) { bv = v2; ba = a2; }
    }
    best = ba == 0x7FFFFFFF ? 0 : ba;
    bestv = n ? bv : 0.0f;
}

// a lane's legal-move count, held inside the scanned row range [0, total) (equal to the
// record's count whenever the lanes did not change since k_scan: bgx.h stream ordering)
__device__ __forceinline__ int row_count(const uint8_t* rr, int32_t off, int64_t total) {
    const int n = (int)rr[R_NM0] | ((int)rr[R_NM1] << 8);
    const int64_t room = off >= 0 && off <= total ? total - off : 0;
    return n < room ? n : (int)room;
}

// 1-ply choice per lane: first argmax of V over its rows (values_out row a = V(a)); one
// wave per lane.
__global__ __launch_bounds__(256) void k_one_ply_reduce(Args A, const int32_t* lane_off, const int64_t* total,
                                                        const float* vrow, int32_t* best, float* bestv, float* vout) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= A.B) return;
    const uint8_t* rr = A.lanes + (size_t)i * 64;
    const int n = row_count(rr, lane_off[i], *total);
    const float* v = vrow + lane_off[i];
    int ba;
    float bv;
    wave_first_argmax(n, [&](int a) {
        const float x = v[a];
        if (vout) vout[(size_t)i * A.max_moves + a] = x;
        return x;
    }, ba, bv);
    if (lane_id() == 0) {
        best[i] = ba;
        if (bestv) bestv[i] = bv;
    }
}

// Q(a) = sum_r p_r minv[a][r] (fp32 FMA, r in roll order), first argmax; one wave per lane.
__global__ __launch_bounds__(256) void k_two_ply_reduce(Args A, const int32_t* lane_off, const int64_t* total,
                                                        const int32_t* minv, int32_t* best, float* bestq,
                                                        float* qout) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= A.B) return;
    const uint8_t* rr = A.lanes + (size_t)i * 64;
    const int n = row_count(rr, lane_off[i], *total);
    int ba;
    float bq;
    wave_first_argmax(n, [&](int a) {
        const int32_t* mv = minv + ((size_t)lane_off[i] + a) * 21;
        float q = 0.0f;
        for (int r = 0; r < 21; ++r)
            q = fmaf(kRoll0[r] == kRoll1[r] ? 1.0f / 36.0f : 2.0f / 36.0f, unord_f32(mv[r]), q);
        if (qout) qout[(size_t)i * A.max_moves + a] = q;
        return q;
    }, ba, bq);
    if (lane_id() == 0) {
        best[i] = ba;
        if (bestq) bestq[i] = bq;
    }
}

__device__ __forceinline__ void split16(float x, _Float16& hi, _Float16& lo) {
    hi = (_Float16)x;
    lo = (_Float16)(x - (float)hi);
}

// f16 section of the value pack (one workgroup): e1 from max |[W1s | b1]|, then
// w1q and wvq (layout above).
__global__ __launch_bounds__(1024) void k_value_pack16(const float* W1, const float* b1, const float* wv, int H,
                                                       int NT, int* hdr, _Float16* w1q, float* wvq) {
    __shared__ float red[1024];
    const int tid = threadIdx.x;
    float mx = 0.0f;
    for (int i = tid; i < H * 199; i += 1024) {
        const int u = i / 199, f = i % 199;
        const float w = f == 198 ? b1[u] : ((f == 97 || f == 195) ? W1[u * 198 + f] / 15.0f : W1[u * 198 + f]);
        mx = fmaxf(mx, fabsf(w));
    }
    red[tid] = mx;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if (tid < o) red[tid] = fmaxf(red[tid], red[tid + o]);
        __syncthreads();
    }
    int e1 = 0;
    if (red[0] > 0.0f && red[0] < INFINITY) {
        int qe;
        (void)frexpf(red[0], &qe);
        e1 = 14 - qe;
        e1 = e1 < -100 ? -100 : (e1 > 100 ? 100 : e1);
    }
    if (tid == 0) { hdr[0] = e1; hdr[1] = 0; hdr[2] = 0; hdr[3] = 0; }
    const bool wide = wide_tiles(NT);
    const int NS = slices(NT);              // 64-lane uint4 fragments per k-block
    const int n = kKB * NS * 64 * 8;
    for (int idx = tid; idx < n; idx += 1024) {
        const int i = idx & 7, l = (idx >> 3) & 63, t = (idx >> 9) % NS, kb = (idx >> 9) / NS;
        const int m = l & 31;
        const int unit = wide ? 32 * (t >> 1) + m : 16 * t + (m & 7) + 8 * (m >> 4);
        const int part = wide ? (t & 1) : (m >> 3) & 1;
        const int f = kperm(kb, l >> 5, i);
        float w = 0.0f;
        if (unit < H) {
            if (f == kFeatBias) w = b1[unit];
            else if (f >= 0) w = (f == 97 || f == 195) ? W1[(size_t)unit * 198 + f] / 15.0f : W1[(size_t)unit * 198 + f];
        }
        _Float16 hi, lo;
        split16(ldexpf(w, e1), hi, lo);
        w1q[((size_t)(kb * NS + t) * 64 + l) * 8 + i] = part ? lo : hi;
    }
    for (int idx = tid; idx < NS * 8 * 64; idx += 1024) {
        const int l = idx & 63;
        int unit;
        if (wide) {
            const int lw = (idx >> 2) & 63, r = (idx & 3) + 4 * ((idx >> 8) & 3), T = idx >> 10;
            unit = 32 * T + 8 * (r >> 2) + 4 * (lw >> 5) + (r & 3);
        } else {
            const int j = (idx >> 6) & 7, t = idx >> 9;
            unit = 16 * t + (j & 3) + 8 * (j >> 2) + 4 * (l >> 5);
        }
        wvq[idx] = unit < H ? ldexpf(wv[unit], -e1) : 0.0f;
    }
}

// Exclusive scan of the lanes' legal-move counts (one workgroup): lane i's rows start at
// lane_off[i].  by_mover (2-ply): the rows of lanes whose mover is PLAYER1 come first, then
// PLAYER2's (each group in lane order), so the enumerators' pool output -- every wave walks
// rows a grid stride apart -- holds long runs of one replier, which the factored evaluator
// needs per leaf pair (eval_leaves_fact).
__global__ __launch_bounds__(1024) void k_scan(Args A, int32_t* lane_off, int64_t* total, int by_mover) {
    __shared__ int64_t part[2][1024];
    const int t = threadIdx.x;
    const int per = (A.B + 1023) / 1024;
    const int lo = t * per, hi = min(A.B, lo + per);
    int64_t sum[2] = {0, 0};
    for (int i = lo; i < hi; ++i) {
        const uint8_t* rr = A.lanes + (size_t)i * 64;
        sum[by_mover ? rr[R_CUR] & 1 : 0] += (int)rr[R_NM0] | ((int)rr[R_NM1] << 8);
    }
    part[0][t] = sum[0];
    part[1][t] = sum[1];
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int64_t v0 = t >= o ? part[0][t - o] : 0, v1 = t >= o ? part[1][t - o] : 0;
        __syncthreads();
        part[0][t] += v0;
        part[1][t] += v1;
        __syncthreads();
    }
    int64_t run[2] = {part[0][t] - sum[0], part[0][1023] + part[1][t] - sum[1]};
    for (int i = lo; i < hi; ++i) {
        const uint8_t* rr = A.lanes + (size_t)i * 64;
        const int g = by_mover ? rr[R_CUR] & 1 : 0;
        lane_off[i] = (int32_t)run[g];
        run[g] += (int)rr[R_NM0] | ((int)rr[R_NM1] << 8);
    }
    if (t == 1023) *total = part[0][1023] + part[1][1023];
}

// row -> lane map, one wave per lane (coalesced stores; one thread per lane walked up to
// 500 rows serially)
__global__ __launch_bounds__(256) void k_expand(Args A, const int32_t* lane_off, const int64_t* total,
                                                int32_t* row_lane) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= A.B) return;
    const int o = lane_off[i];
    const int n = row_count(A.lanes + (size_t)i * 64, o, *total);
    for (int a = lane_id(); a < n; a += 64) row_lane[o + a] = i;
}

}  // namespace

extern int bgx_internal_fail(hipError_t e);
extern void bgx_set_error(const char* msg);
#define SCK(x) do { hipError_t _e = (x); if (_e != hipSuccess) return bgx_internal_fail(_e); } while (0)

static int value_tiles16(int H) { return (H + 15) / 16; }   // 16 hidden units (hi + lo rows) per MFMA tile
constexpr int kMaxHidden = 128;                              // 8 tiles: 120 KiB of weights in LDS

template <typename K>
static int persistent_grid(const bgx_engine* e, K kernel, int per_cu_cap) {
    int cus = 0, occ = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->device) != hipSuccess || cus <= 0)
        cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, 64, 0) != hipSuccess || occ <= 0) occ = 8;
    if (occ > per_cu_cap) occ = per_cu_cap;
    return cus * occ;
}

typedef void (*EvalFn)(EvalArgs);
typedef void (*EvalRowsFn)(EvalRowsArgs);
static int eval_waves(int NT) { return NT <= 4 ? kEvalNarrowWaves : kEvalWideWaves; }
// the 2-ply evaluator for NT 16-unit slices and its workgroup size; the row-part kernel
struct EvalPick { EvalFn fn; int threads; };
static EvalPick eval_kernel(int NT) {
    switch (NT) {
        case 1: return {k_eval<1>, 64 * eval_waves(1)}; case 2: return {k_eval<2>, 64 * eval_waves(2)};
        case 3: return {k_eval<3>, 64 * eval_waves(3)}; case 4: return {k_eval<4>, 64 * eval_waves(4)};
        case 5: return {k_eval<5>, 64 * eval_waves(5)}; case 6: return {k_eval<6>, 64 * eval_waves(6)};
        case 7: return {k_eval<7>, 64 * eval_waves(7)}; default: return {k_eval<8>, 64 * eval_waves(8)};
    }
}
typedef void (*RowPartFn)(const uint4*, const int64_t*, const uint4*, float*);
static RowPartFn rowpart_kernel(int NT) {
    switch (NT) {
        case 1: return k_rowpart<1>; case 2: return k_rowpart<2>; case 3: return k_rowpart<3>;
        case 4: return k_rowpart<4>; case 5: return k_rowpart<5>; case 6: return k_rowpart<6>;
        case 7: return k_rowpart<7>; default: return k_rowpart<8>;
    }
}
static EvalRowsFn eval_rows_kernel(int NT) {
    switch (NT) {
        case 1: return k_eval_rows<1>; case 2: return k_eval_rows<2>; case 3: return k_eval_rows<3>;
        case 4: return k_eval_rows<4>; case 5: return k_eval_rows<5>; case 6: return k_eval_rows<6>;
        case 7: return k_eval_rows<7>; default: return k_eval_rows<8>;
    }
}
// the launch's workgroup size must be the kernels' EvalShape<NT>::kWaves (their tile stride)

// resident workgroups of an evaluator over the whole device
template <typename K>
static int eval_grid(const bgx_engine* e, K kernel, int NT) {
    int occ = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, 64 * eval_waves(NT), 0) != hipSuccess || occ <= 0)
        occ = 1;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, e->device) != hipSuccess || ncu <= 0)
        ncu = 256;
    return occ * ncu;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

extern "C" {

int bgx_value_packed_size(int32_t hidden) {
    if (hidden <= 0 || hidden > kMaxHidden) return BGX_EINVAL;
    return sz_f16(value_tiles16(hidden));
}

int bgx_value_pack(const float* W1, const float* b1, const float* wv, const float* bv, int32_t hidden, float* packed,
                   void* stream) {
    const int total = bgx_value_packed_size(hidden);
    if (total < 0 || !W1 || !b1 || !wv || !bv || !packed) return BGX_EINVAL;
    const int NT = value_tiles16(hidden);
    hipLaunchKernelGGL(k_value_pack16, dim3(1), dim3(1024), 0, (hipStream_t)stream, W1, b1, wv, hidden, NT,
                       (int*)packed, (_Float16*)(packed + 4), packed + 4 + kKB * slices(NT) * 64 * 4);
    SCK(hipGetLastError());
    return BGX_OK;
}

int bgx_one_ply(bgx_engine* e, const float* vpacked, int32_t hidden, float value_bias, int32_t* best_out,
                float* bestv_out, float* values_out, void* stream) {
    if (!e || !vpacked || !best_out || bgx_value_packed_size(hidden) < 0) return BGX_EINVAL;
    SCK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    EngineUse use(e, s);
    SCK(use.err);
    Args& A = e->a;
    const size_t B = (size_t)A.B, R = B * (size_t)A.max_moves;
    // [lane_off B i32][row total i64][row_lane R i32][rowside R][rowkey R][vrow R f32]: sized for
    // the worst case, so the pass runs without a host sync (the row count stays on the device)
    const size_t o_tot = align256(B * 4), o_rl = o_tot + 256, o_side = align256(o_rl + R * 4),
                 o_key = align256(o_side + R * 16), o_v = align256(o_key + R * 16), need = align256(o_v + R * 4);
    if (e->oneply_ws_bytes < need) {
        SCK(hipStreamSynchronize(s));
        if (e->oneply_ws) SCK(hipFree(e->oneply_ws));
        e->oneply_ws = nullptr;
        e->oneply_ws_bytes = 0;
        SCK(hipMalloc(&e->oneply_ws, need));
        e->oneply_ws_bytes = need;
    }
    char* ws = (char*)e->oneply_ws;
    int32_t* lane_off = (int32_t*)ws;
    int64_t* total = (int64_t*)(ws + o_tot);
    int32_t* row_lane = (int32_t*)(ws + o_rl);
    uint4* rowside = (uint4*)(ws + o_side);
    uint4* rowkey = (uint4*)(ws + o_key);
    float* vrow = (float*)(ws + o_v);
    const int NT = value_tiles16(hidden);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, A, lane_off, total, 0);
    hipLaunchKernelGGL(k_expand, dim3((A.B + 3) / 4), dim3(256), 0, s, A, lane_off, total, row_lane);
    // ~20 legal moves per lane on average: one wave per ~5 rows at B = 4,096
    const size_t gr = B * 6 < 16384 ? (B * 6 > 64 ? B * 6 : 64) : 16384;
    hipLaunchKernelGGL(k_rows, dim3((unsigned)gr), dim3(256), 0, s, A, row_lane, lane_off, total, nullptr, rowside,
                       rowkey, A.err);
    const EvalRowsFn kr = eval_rows_kernel(NT);
    const EvalRowsArgs E{rowkey, rowside, total, vrow, (const uint4*)(vpacked + 4), vpacked + 4 + kKB * slices(NT) * 64 * 4,
                         value_bias};
    hipLaunchKernelGGL(kr, dim3(eval_grid(e, kr, NT)), dim3(64 * eval_waves(NT)), 0, s, E);
    hipLaunchKernelGGL(k_one_ply_reduce, dim3((A.B + 3) / 4), dim3(256), 0, s, A, lane_off, total, vrow, best_out,
                       bestv_out, values_out);
    SCK(hipGetLastError());
    return BGX_OK;
}

int bgx_two_ply(bgx_engine* e, const float* vpacked, int32_t hidden, float value_bias, int32_t* best_out,
                float* bestq_out, float* q_out, uint64_t* stats_host, void* stream) {
    if (!e || !vpacked || !best_out || bgx_value_packed_size(hidden) < 0) return BGX_EINVAL;
    SCK(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    EngineUse use(e, s);
    SCK(use.err);
    Args& A = e->a;
    const size_t B = (size_t)A.B;
    // workspace head: [lane_off B i32][counters 256 B][overflow queues]
    struct Ctr {
        int64_t rows;
        unsigned long long leaves, cursor;
        int32_t qcount[3], retry_count, list_count, bad;    // bad: k_rows found a changed lane
        unsigned long long zero;                      // start of the evaluated pool range
    };
    static_assert(sizeof(Ctr) <= 256, "counters");
    const size_t o_ctr = align256(B * 4), o_q = o_ctr + 256, head = align256(o_q + (size_t)3 * kSlowQueue * 4);
    auto grow = [&](size_t need) -> int {
        if (e->search_ws_bytes >= need) return BGX_OK;
        void* nw = nullptr;
        SCK(hipStreamSynchronize(s));
        SCK(hipMalloc(&nw, need + need / 4));
        if (e->search_ws) SCK(hipFree(e->search_ws));
        e->search_ws = nw;
        e->search_ws_bytes = need + need / 4;
        return BGX_OK;
    };
    int rc = grow(head);
    if (rc != BGX_OK) return rc;
    char* ws = (char*)e->search_ws;
    SCK(hipMemsetAsync(ws + o_ctr, 0, 256, s));
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, A, (int32_t*)ws, (int64_t*)(ws + o_ctr), 1);
    SCK(hipGetLastError());
    int64_t rows64 = 0;
    SCK(hipMemcpyAsync(&rows64, ws + o_ctr, 8, hipMemcpyDeviceToHost, s));
    SCK(hipStreamSynchronize(s));
    const int64_t jobs64 = rows64 * 21;
    if (jobs64 >= (int64_t)0x1FFFFFFF) return BGX_EINVAL;     // job ids are 29-bit pool tags
    const int rows = (int)rows64, jobs = (int)jobs64;
    // [row_lane rows][rowrec rows*64][rowside rows*16][minv jobs*4][maxlen jobs][list jobs*4][retry jobs*4]
    // [rowpart rows*16*slices f32]
    const int NT = value_tiles16(hidden);
    const size_t o_rl = head, o_rec = align256(o_rl + (size_t)rows * 4), o_side = align256(o_rec + (size_t)rows * 64),
                 o_minv = align256(o_side + (size_t)rows * 16), o_ml = align256(o_minv + (size_t)jobs * 4),
                 o_list = align256(o_ml + (size_t)jobs), o_retry = align256(o_list + (size_t)jobs * 4),
                 o_rp = align256(o_retry + (size_t)jobs * 4),
                 need = align256(o_rp + (size_t)rows * 16 * slices(NT) * 4);
    if (e->search_ws_bytes < need) {
        // keep the head (lane_off, counters) across the regrow
        void* nw = nullptr;
        SCK(hipMalloc(&nw, need + need / 4));
        SCK(hipMemcpyAsync(nw, e->search_ws, head, hipMemcpyDeviceToDevice, s));
        SCK(hipStreamSynchronize(s));
        SCK(hipFree(e->search_ws));
        e->search_ws = nw;
        e->search_ws_bytes = need + need / 4;
        ws = (char*)nw;
    }
    int32_t* lane_off = (int32_t*)ws;
    Ctr* ctr = (Ctr*)(ws + o_ctr);
    int32_t* row_lane = (int32_t*)(ws + o_rl);
    uint8_t* rowrec = (uint8_t*)(ws + o_rec);
    uint4* rowside = (uint4*)(ws + o_side);
    int32_t* minv = (int32_t*)(ws + o_minv);
    uint8_t* maxlen = (uint8_t*)(ws + o_ml);
    int32_t* list = (int32_t*)(ws + o_list);
    int32_t* retry = (int32_t*)(ws + o_retry);
    float* rowpart = (float*)(ws + o_rp);

    if (rows > 0) {
        hipLaunchKernelGGL(k_expand, dim3((A.B + 3) / 4), dim3(256), 0, s, A, lane_off, &ctr->rows, row_lane);
        SCK(hipMemsetAsync(minv, 0x7F, (size_t)jobs * 4, s));
        SCK(hipMemsetAsync(maxlen, 0xFF, (size_t)jobs, s));
        hipLaunchKernelGGL(k_rows, dim3((rows + 3) / 4 < 16384 ? (rows + 3) / 4 : 16384), dim3(256), 0, s, A, row_lane,
                           lane_off, &ctr->rows, rowrec, rowside, nullptr, &ctr->bad);
        SCK(hipGetLastError());
        const bool barrow = bgx_dbg_int("BGX_2PLY_BARROW", 1) != 0;      // tests: 0 = the bar rows per job
        S2 S{rowrec, 0, rows, nullptr, nullptr, &ctr->cursor, 0ull, maxlen, &ctr->leaves,
             ctr->qcount, (int32_t*)(ws + o_q), &ctr->retry_count,
             retry, list, &ctr->list_count, A.err, cap_fast<kLogLight>(), 0, cap_fast<kLogMid>(), 3, 3,
             barrow ? 1 : 0};
        // doubles enumerator: 512-slot dedup table with the revisit memo inside it, held to
        // 128 VGPRs (4 waves/SIMD, +1.5 %).  Tests (BGX_2PLY_HEAVY = 9:0 / 10:0) run the
        // exact alternatives without the memo (9:0) or with a 1,024-slot table (10:0): the
        // same leaves, Q and choices (tests/test_gpu_search.py)
        int hlog = 9, hmk = 2;
        if (const std::string hv = bgx_dbg("BGX_2PLY_HEAVY"); !hv.empty()) {
            hlog = atoi(hv.c_str());
            const char* c = strchr(hv.c_str(), ':');
            hmk = c ? atoi(c + 1) : 2;
        }
        void (*kheavy)(S2) = k_enum<9, 2, 1, 4>;
        void (*klist)(S2) = k_enum<9, 2, 2, 4>;
        if (hlog == 9 && hmk == 0) { kheavy = k_enum<9, 0, 1>; klist = k_enum<9, 0, 2>; }
        else if (hlog == 10 && hmk == 0) { kheavy = k_enum<10, 0, 1>; klist = k_enum<10, 0, 2>; }
        else { hlog = 9; hmk = 2; }
        S.cap_heavy = (7 << hlog) / 8;
        if (const std::string fs = bgx_dbg("BGX_2PLY_LDS_CAP"); !fs.empty()) {    // tests: force the overflow tiers ("first[:mid]")
            S.cap_light = S.cap_heavy = S.cap_mid = atoi(fs.c_str());
            if (const char* c = strchr(fs.c_str(), ':')) S.cap_mid = atoi(c + 1);
        }
        const bool dbg = !bgx_dbg("BGX_2PLY_DEBUG").empty();
        const float* f16s = vpacked;
        const uint4* w1q = (const uint4*)(f16s + 4);
        // the root mover's part of X1 per row (the factored evaluator); BGX_2PLY_UNFACTORED
        // (tests) evaluates every leaf over all 13 k-blocks instead
        const bool factored = bgx_dbg("BGX_2PLY_UNFACTORED").empty();
        if (factored)
            hipLaunchKernelGGL(rowpart_kernel(NT), dim3((rows + 127) / 128 < 8192 ? (rows + 127) / 128 : 8192), dim3(256),
                               0, s, rowside, &ctr->rows, w1q, rowpart);
        EvalArgs E{nullptr, nullptr, &ctr->zero, &ctr->cursor, 0ull, rowside, maxlen, minv,
                   w1q, f16s + 4 + kKB * slices(NT) * 64 * 4, value_bias, factored ? rowpart : nullptr, nullptr};
        // the non-doubles enumerator: the row-level walk held to 80 VGPRs (6 waves/SIMD,
        // +1.2 % over its natural 91)
        void (*klight)(S2) = k_enum<kLogLight, -1, 3, 6>;
        const int g_light = persistent_grid(e, klight, 32);
        const int g_heavy = persistent_grid(e, kheavy, 32);
        const int g_list = persistent_grid(e, klist, 32);
        const int g_t0 = persistent_grid(e, k_enum_tier<10, 0>, 32);
        const int g_mid = persistent_grid(e, k_enum_tier<kLogMid, 1>, 32);
        // leaf pool: ~32 slots per job (mean ~19 survivors at mid-game positions);
        // BGX_2PLY_POOL overrides (tests force retry rounds with a tiny pool)
        // every resident wave may hold a partly filled block in each tier
        size_t cap = (size_t)jobs * 32 + (size_t)(g_light + g_heavy + g_list + g_t0 + g_mid + e->slow_waves) * kBlk * 2;
        if (const long long ps = bgx_dbg_int("BGX_2PLY_POOL", 0); ps > 0) cap = (size_t)ps;
        cap = (cap + kBlk - 1) / kBlk * kBlk;
        if (cap < (size_t)kBlk * 4) cap = (size_t)kBlk * 4;
        if (cap > ((size_t)1 << 31)) cap = (size_t)1 << 31;
        if (e->search_pool_cap < cap) {
            SCK(hipStreamSynchronize(s));
            if (e->search_pool) SCK(hipFree(e->search_pool));
            e->search_pool = nullptr; e->search_pool_cap = 0;
            SCK(hipMalloc(&e->search_pool, cap * 20));
            e->search_pool_cap = cap;
        }
        const size_t pcap = cap;           // the pool may be larger (kept from a bigger call)
        S.keys = (uint4*)e->search_pool;
        S.tags = (uint32_t*)(S.keys + pcap);
        E.keys = S.keys;
        E.tags = S.tags;
        S.cap = E.cap = (unsigned long long)pcap;
        float* vdbg = nullptr;
        const std::string dump = bgx_dbg("BGX_2PLY_DUMP");
        if (!dump.empty()) {
            SCK(hipMalloc(&vdbg, pcap * 4));
            SCK(hipMemsetAsync(vdbg, 0, pcap * 4, s));
            E.vdbg = vdbg;
        }
        const EvalPick keval = eval_kernel(NT);
        int occ_eval = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_eval, keval.fn, keval.threads, 0) != hipSuccess ||
            occ_eval <= 0)
            occ_eval = 1;
        const int g_eval = occ_eval * persistent_grid(e, keval.fn, 1);     // resident workgroups
        if (!e->search_ev[0])
            for (hipEvent_t& ev : e->search_ev) SCK(hipEventCreate(&ev));
        if (!e->search_side) SCK(hipStreamCreateWithFlags(&e->search_side, hipStreamNonBlocking));
        SCK(hipEventRecord(e->search_ev[0], s));
        auto eval = [&](hipStream_t st) {
            hipLaunchKernelGGL(keval.fn, dim3(g_eval), dim3(keval.threads), 0, st, E);
        };
        // retry rounds run few waves: every wave holding a block wastes its unused
        // part, and a round must leave pool for its jobs to finish (progress with any pool)
        int gcap = 1 << 30;
        auto g = [&](int grid) { return grid < gcap ? grid : gcap; };
        auto tiers = [&]() {
            hipLaunchKernelGGL((k_enum_tier<10, 0>), dim3(g(g_t0)), dim3(64), 0, s, S);
            hipLaunchKernelGGL((k_enum_tier<kLogMid, 1>), dim3(g(g_mid)), dim3(64), 0, s, S);
            hipLaunchKernelGGL(k_enum_slow, dim3(g(e->slow_waves)), dim3(64), 0, s, S, e->slow_tables);
        };
        for (int round = 0;; ++round) {
            if (round == 0) {       // the non-doubles enumerator beside the doubles one
                SCK(hipEventRecord(e->search_ev[3], s));
                SCK(hipStreamWaitEvent(e->search_side, e->search_ev[3], 0));
                hipLaunchKernelGGL(kheavy, dim3(g_heavy), dim3(64), 0, s, S);
                hipLaunchKernelGGL(klight, dim3(g_light), dim3(64), 0, e->search_side, S);
                SCK(hipEventRecord(e->search_ev[4], e->search_side));
                SCK(hipStreamWaitEvent(s, e->search_ev[4], 0));
                tiers();
                SCK(hipEventRecord(e->search_ev[1], s));
                eval(s);
            } else {
                const long long blocks = (long long)(pcap / kBlk);
                gcap = (int)(blocks / 16 > 1 ? (blocks / 16 < (1 << 30) ? blocks / 16 : (1 << 30)) : 1);
                hipLaunchKernelGGL(klist, dim3(g(g_list)), dim3(64), 0, s, S);
                tiers();
                eval(s);
            }
            SCK(hipGetLastError());
            if (round == 0) SCK(hipEventRecord(e->search_ev[2], s));
            Ctr hc;
            SCK(hipMemcpyAsync(&hc, ctr, sizeof hc, hipMemcpyDeviceToHost, s));
            SCK(hipStreamSynchronize(s));
            const int32_t nretry = hc.retry_count;
            if (hc.bad) {                      // the lanes changed under the call (bgx.h stream ordering)
                bgx_set_error("bgx_two_ply: the lanes' move lists changed under the call (stream ordering)");
                return BGX_ESTATE;
            }
            if (round == 0) {
                SCK(hipEventElapsedTime(&e->search_ms[0], e->search_ev[0], e->search_ev[1]));
                SCK(hipEventElapsedTime(&e->search_ms[1], e->search_ev[1], e->search_ev[2]));
            }
            if (dbg)
                fprintf(stderr, "[bgx 2-ply] round %d: pool %llu/%zu, tier1 %d, tier2 %d, retry %d, leaves %llu\n", round,
                        hc.cursor, pcap, hc.qcount[0] + hc.qcount[1], hc.qcount[2], hc.retry_count, hc.leaves);
            if (nretry == 0) {
                // test hook (tests/test_gpu_search.py): per-job minv, row parts, the pool, V per slot
                if (!dump.empty()) {
                    const char* dp = dump.c_str();
                    int32_t* hm = (int32_t*)malloc((size_t)jobs * 4);
                    SCK(hipMemcpy(hm, minv, (size_t)jobs * 4, hipMemcpyDeviceToHost));
                    FILE* f = fopen(dp, "wb");
                    if (f) { fwrite(hm, 4, (size_t)jobs, f); fclose(f); }
                    free(hm);
                    const size_t nrp = (size_t)rows * 16 * slices(NT);
                    float* hr = (float*)malloc(nrp * 4);
                    SCK(hipMemcpy(hr, rowpart, nrp * 4, hipMemcpyDeviceToHost));
                    char nm[512];
                    snprintf(nm, sizeof nm, "%s.rp", dp);
                    f = fopen(nm, "wb");
                    if (f) { fwrite(hr, 4, nrp, f); fclose(f); }
                    free(hr);
                    const size_t used = hc.cursor < pcap ? hc.cursor : pcap;
                    auto dumpd = [&](const void* d, size_t bytes, const char* ext) {
                        void* hb = malloc(bytes);
                        if (hipMemcpy(hb, d, bytes, hipMemcpyDeviceToHost) == hipSuccess) {
                            snprintf(nm, sizeof nm, "%s.%s", dp, ext);
                            if (FILE* g = fopen(nm, "wb")) { fwrite(hb, 1, bytes, g); fclose(g); }
                        }
                        free(hb);
                    };
                    dumpd(S.keys, used * 16, "keys");
                    dumpd(S.tags, used * 4, "tags");
                    dumpd(vdbg, used * 4, "v");
                    dumpd(rowside, (size_t)rows * 16, "side");
                    dumpd(maxlen, (size_t)jobs, "ml");
                    (void)hipFree(vdbg);
                }
                break;
            }
            if (round + 1 >= kMaxRounds) return BGX_ENOMEM;
            // next round: the lost jobs become the explicit list, the pool starts over
            SCK(hipMemcpyAsync(list, retry, (size_t)nretry * 4, hipMemcpyDeviceToDevice, s));
            SCK(hipMemcpyAsync(&ctr->list_count, &ctr->retry_count, 4, hipMemcpyDeviceToDevice, s));
            SCK(hipMemsetAsync(&ctr->cursor, 0, 8, s));
            SCK(hipMemsetAsync(ctr->qcount, 0, 16, s));          // qcount[3], retry_count
        }
    }
    hipLaunchKernelGGL(k_two_ply_reduce, dim3((A.B + 3) / 4), dim3(256), 0, s, A, lane_off, &ctr->rows, minv, best_out,
                       bestq_out, q_out);
    SCK(hipGetLastError());
    if (stats_host) {
        unsigned long long lv = 0;
        SCK(hipMemcpyAsync(&lv, &ctr->leaves, 8, hipMemcpyDeviceToHost, s));
        SCK(hipStreamSynchronize(s));
        stats_host[0] = lv;
        stats_host[1] = (uint64_t)jobs64;
        stats_host[2] = (uint64_t)rows64;
    }
    return BGX_OK;
}

#ifdef BGX_COUNTERS
// this translation unit's work counters (experiments; bg_engine.hip has its own set)
int bgx_debug_search_counters(unsigned long long* out32) {
    SCK(hipDeviceSynchronize());
    constexpr size_t n = 16 * (size_t)bg::kCntSlots;
    std::vector<unsigned long long> h(n), z(n, 0ull);
    SCK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_scnt), n * 8));
    for (int i = 0; i < 16; ++i) {
        out32[i] = 0;
        for (int k = 0; k < bg::kCntSlots; ++k) out32[i] += h[(size_t)i * bg::kCntSlots + k];
    }
    SCK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(bg::g_cnt), n * 8));   // the move generator's (bg_core.h)
    for (int i = 0; i < 16; ++i) {
        out32[16 + i] = 0;
        for (int k = 0; k < bg::kCntSlots; ++k) out32[16 + i] += h[(size_t)i * bg::kCntSlots + k];
    }
    SCK(hipMemcpyToSymbol(HIP_SYMBOL(g_scnt), z.data(), n * 8));
    SCK(hipMemcpyToSymbol(HIP_SYMBOL(bg::g_cnt), z.data(), n * 8));
    return BGX_OK;
}
#endif

int bgx_two_ply_timings(bgx_engine* e, float* ms2) {
    if (!e || !ms2) return BGX_EINVAL;
    ms2[0] = e->search_ms[0];
    ms2[1] = e->search_ms[1];
    return BGX_OK;
}

}  // extern "C"
