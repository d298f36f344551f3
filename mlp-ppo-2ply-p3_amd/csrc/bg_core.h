// bg_core.h — device-side backgammon rules for gfx950 (CDNA4).
//
// One WAVEFRONT owns one game.  The move tree is walked as a wave-uniform
// (SGPR) program over bitboards: the mover's 24 point counts live in a 96-bit
// nibble vector, and the opponent is reduced to two 24-bit masks (blocked =
// opp>=2, blot = opp==1) because the opponent never moves during enumeration.
// The dedup set of afterstates ("add_unique_board", handle_moves.py:313-341) is
// an open-addressing table in LDS probed 64 slots at a time (one ds_read_b128
// per lane + two ballots).
//
// Exactness: the afterstate of any sub-move sequence from a fixed root is
// determined by (own counts, own bar, own off, set of hit blots); that 128-bit
// KEY is a bijection of the reference's full (4,24) tensor given the root (opp
// row = root opp - hits, opp bar = root bar + |hits|), so key equality ==
// tensor-byte equality, the reference's dedup semantics (immutable_board.py:236).
//
// Citations are path:line in the reference's src/.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bg {

// Work counters for experiments (built with -DBGX_COUNTERS only).
#ifdef BGX_COUNTERS
// each counter spread over kCntSlots addresses (by workgroup): one address hit by every
// wave of the chip serialises the atomics and distorts the timings being measured
constexpr int kCntSlots = 1024;
__device__ unsigned long long g_cnt[16 * kCntSlots];
#define BG_CNT(i, v) do { if ((threadIdx.x & 63) == 0) \
    atomicAdd(&bg::g_cnt[(i) * bg::kCntSlots + (blockIdx.x & (bg::kCntSlots - 1))], (unsigned long long)(v)); } while (0)
#define BG_T0(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#define BG_T1(i, t) BG_CNT(i, __builtin_amdgcn_s_memtime() - t)
#else
#define BG_CNT(i, v) do { } while (0)
#define BG_T0(t) do { } while (0)
#define BG_T1(i, t) do { } while (0)
#endif

constexpr int kBar = 24;   // moves/move_types.py:33
constexpr int kOff = 25;   // moves/move_types.py:34
constexpr uint32_t kHome[2] = {0xFC0000u, 0x3Fu};   // P1 home 18..23, P2 home 0..5 (conditions.py:122-126)

// ------------------------------------------------------------------ state --
struct Node {
    uint64_t lo;      // own counts, points 0..15, 4 bits each
    uint32_t hi;      // own counts, points 16..23
    uint32_t k3;      // own_bar | own_off << 4 | hit-mask << 8
    uint32_t occ;     // own > 0
    uint32_t blot;    // opp == 1 and not hit yet
    int n_home;       // own checkers on home points
};

// branch-free (s_cselect) nibble access: point p lives in lo for p < 16, else hi
__device__ __forceinline__ int own_at(const Node& s, int p) {
    const uint64_t w = p < 16 ? s.lo : (uint64_t)s.hi;
    return (int)((w >> (4 * (p & 15))) & 15u);
}
__device__ __forceinline__ void own_inc(Node& s, int p) {
    const uint64_t m = 1ull << (4 * (p & 15));
    s.lo += p < 16 ? m : 0ull;
    s.hi += p < 16 ? 0u : (uint32_t)m;
}
__device__ __forceinline__ void own_dec(Node& s, int p) {
    const uint64_t m = 1ull << (4 * (p & 15));
    s.lo -= p < 16 ? m : 0ull;
    s.hi -= p < 16 ? 0u : (uint32_t)m;
}

// A node's child list (get_moves_with_one_die, move_logic.py:20-44): bits 0..23
// are normal-move sources in ascending order (move_logic.py:67); bit 31 is the
// single special move (bar entry :95-137, or the one bear-off :211-253), which
// always comes last.  Proof that at most one bear-off is ever emitted and that
// it sorts after every normal move: DESIGN.md §"Move generation".
struct Kids { uint32_t bits; int extra; };

__device__ __forceinline__ int entry_point(int pl, int d) { return pl == 0 ? d - 1 : 24 - d; }

__device__ __forceinline__ Kids gen(const Node& s, int d, int pl, uint32_t blocked) {
    Kids k{0u, -1};
    const int own_bar = (int)(s.k3 & 15u), own_off = (int)((s.k3 >> 4) & 15u);
    if (own_off == 15) return k;                                   // GAME_OVER (:262-263)
    if (own_bar > 0) {                                             // ON_BAR
        const int dst = entry_point(pl, d);
        if (!((blocked >> dst) & 1u)) { k.bits = 1u << 31; k.extra = kBar; }
        return k;
    }
    const uint32_t home = kHome[pl];
    uint32_t m;
    if (pl == 0) m = s.occ & ~(blocked >> d) & ((1u << (24 - d)) - 1u);
    else m = s.occ & ~(blocked << d) & 0xFFFFFFu & ~((1u << d) - 1u);
    k.bits = m;
    // BEAR_OFF: all_checkers_home (conditions.py:111-147); bar already 0 here.
    if ((s.occ & ~home) == 0u && s.n_home + own_off == 15) {
        if (pl == 0) {
            const int far = __builtin_ctz(s.occ & home);          // :197-201
            if (far + d >= 24) { k.extra = far; }
            else { const int e = 24 - d; if (e != far && ((s.occ >> e) & 1u)) k.extra = e; }
        } else {
            const int far = 31 - __builtin_clz(s.occ & home);     // :203-208
            if (far - d < 0) { k.extra = far; }
            else { const int e = d - 1; if (e != far && ((s.occ >> e) & 1u)) k.extra = e; }
        }
        if (k.extra >= 0) k.bits |= 1u << 31;
    }
    return k;
}

struct Sub { int src, dst, hit; uint32_t enc; };

// Child b of list k: (start, end, hits_blot) as SubMove (move_types.py:38-42),
// encoded start | end<<5 | hit<<10 | valid<<15.
__device__ __forceinline__ Sub child(const Node& s, const Kids& k, int b, int d, int pl) {
    Sub m;
    if (b == 31) { m.src = k.extra; m.dst = k.extra == kBar ? entry_point(pl, d) : kOff; }
    else { m.src = b; m.dst = pl == 0 ? b + d : b - d; }
    m.hit = m.dst < 24 ? (int)((s.blot >> m.dst) & 1u) : 0;
    m.enc = (uint32_t)m.src | ((uint32_t)m.dst << 5) | ((uint32_t)m.hit << 10) | 0x8000u;
    return m;
}

// Canonical sub-move order (exact pruning of commuted duplicates, DESIGN.md
// §3.1).  Two consecutive NORMAL sub-moves A (source a, child bit a) then B
// (source b < a) with b != dst(A) commute: from the node before A, B is a child
// (its checker, its unblocked destination and the node state do not depend on
// A), A is a child after B, and both orders give the same node (same counts,
// same hit set).  The order (B, A) comes first in the DFS (bit b < bit a), so
// every leaf below (A, B) repeats one below (B, A): the walk skips it.  The
// smallest-key path to any state is never skipped (its prefixes are smallest-key
// too), so the visited set keeps every first occurrence, in DFS order, and the
// memo's revisit argument is unchanged.  Children allowed after a sub-move with
// child bit `bit` (31 = bar entry / bear-off: no restriction) and die d, t = the
// node after it: bits >= bit, plus, for PLAYER2 (moving down), the chain bit
// bit - d when the moved checker is alone there (with another checker already
// there, moving that one first is the same pair in the smaller order).
// PLAYER1 walks that cannot bear off visit every state exactly once (a state's
// sub-move multiset is recovered from its count changes, point by point from
// the far end, and the ascending order of that multiset is its only visited
// path), so they run without table or memo (Gen::pure_walk; tools/check_canon.py
// checks it on random positions).
// mirror (PLAYER2 walks that cannot bear off, set semantics only -- the 2-ply
// replies): bits <= bit, the mirror image of PLAYER1's order, again one visit per
// state; the set of afterstates is the same, their order is not.
__device__ __forceinline__ uint32_t canon_mask(int bit, int d, int pl, const Node& t, bool mirror = false) {
    if (bit >= 24) return 0xFFFFFFFFu;
    if (mirror) return (1u << 31) | ((2u << bit) - 1u);
    const uint32_t ge = ~((1u << bit) - 1u);
    if (pl == 0 || bit < d) return ge;
    const int c = bit - d;
    const uint64_t w = c < 16 ? t.lo : (uint64_t)t.hi;
    return ((w >> (4 * (c & 15))) & 15u) == 1u ? ge | (1u << c) : ge;
}

// move_checker (immutable_board.py:42-89) on the bitboard state; generated
// sub-moves never take the reference's "invalid" branches.
__device__ __forceinline__ Node apply(const Node& s, const Sub& m, int pl) {
    Node t = s;
    const uint32_t home = kHome[pl];
    if (m.src == kBar) t.k3 -= 1u;
    else {
        own_dec(t, m.src);
        if (own_at(t, m.src) == 0) t.occ &= ~(1u << m.src);
        if ((home >> m.src) & 1u) t.n_home -= 1;
    }
    if (m.hit) { t.blot &= ~(1u << m.dst); t.k3 |= 1u << (8 + m.dst); }
    if (m.dst == kOff) t.k3 += 16u;
    else {
        own_inc(t, m.dst);
        t.occ |= 1u << m.dst;
        if ((home >> m.dst) & 1u) t.n_home += 1;
    }
    return t;
}

// ----------------------------------------------------------- dedup tables --
__device__ __forceinline__ uint32_t key_hash(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    uint32_t h = a * 0x9E3779B1u ^ (b * 0x85EBCA77u) ^ (c * 0xC2B2AE3Du) ^ (d * 0x27D4EB2Fu);
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return h;
}

// Key tests as xor/or reductions ending in ONE compare.  The empty asm hides the
// reduction from LLVM, which otherwise re-forms a <4 x i32> compare and expands
// it into per-word compares, cndmasks and 16-bit mask arithmetic.
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
    __asm__("" : "+v"(x));
    return x;
}
__device__ __forceinline__ bool key_eq(const uint4& v, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return opaque((v.x ^ a) | (v.y ^ b) | (v.z ^ c) | (v.w ^ d)) == 0u;
}
__device__ __forceinline__ bool key_empty(const uint4& v) { return opaque(v.x | v.y | v.z | v.w) == 0u; }

// Open addressing, linear probing, empty == all-zero key (a real afterstate
// always has a non-zero own count/bar/off).  The whole wave probes 64
// consecutive slots per step.  Never more than 7/8 full (callers enforce).
// Every probe loop is bounded by the table size (a hang guard: a valid table
// always stops them long before).
template <int LOG_SLOTS, typename SlotPtr>
__device__ __forceinline__ bool table_insert(SlotPtr tab, uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                             bool may_insert = true) {
    constexpr uint32_t mask = (1u << LOG_SLOTS) - 1u;
    const int lane = threadIdx.x & 63;
    uint32_t base = key_hash(a, b, c, d);
    for (uint32_t it = 0; it <= (mask >> 6) + 1u; ++it) {
        const uint32_t slot = (base + (uint32_t)lane) & mask;
        const uint4 v = tab[slot];
        const bool eq = key_eq(v, a, b, c, d);
        const bool em = key_empty(v);
        const uint64_t beq = __ballot(eq), bem = __ballot(em);
        if (beq) return false;                 // no deletions: a match precedes any empty
        if (bem) {
            const int f = __ffsll((unsigned long long)bem) - 1;
            if (may_insert && lane == f) tab[slot] = make_uint4(a, b, c, d);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            return true;
        }
        base += 64u;
    }
    // exhausted (unreachable under the 7/8 cap): report "inserted" without a
    // slot, so the caller's n_unique reaches cap_unique and the walk overflows
    // to the next tier instead of dropping the entry as a duplicate
    return true;
}

// Per-lane (divergent) membership test along the same linear probe sequence.
template <int LOG_SLOTS, typename SlotPtr>
__device__ __forceinline__ bool table_contains_lane(SlotPtr tab, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    constexpr uint32_t mask = (1u << LOG_SLOTS) - 1u;
    uint32_t h = key_hash(a, b, c, d) & mask;
    for (uint32_t it = 0; it <= mask; ++it) {
        const uint4 v = tab[h];
        if (key_eq(v, a, b, c, d)) return true;
        if (key_empty(v)) return false;
        h = (h + 1u) & mask;
    }
    return false;
}

__device__ __forceinline__ uint32_t rdl(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

// Per-lane lookup that also reports where the key would go: on a miss, `slot`
// is the first empty slot of the key's probe sequence.  Four consecutive slots
// per step (independent LDS reads in flight): the chain walk of a loaded table
// costs a quarter of the dependent round trips.
template <int LOG_SLOTS, typename SlotPtr>
__device__ __forceinline__ bool probe_lane(SlotPtr tab, uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                           uint32_t& slot) {
    constexpr uint32_t mask = (1u << LOG_SLOTS) - 1u;
    uint32_t h = key_hash(a, b, c, d) & mask;
    for (uint32_t it = 0; it <= (mask >> 2); ++it) {
        uint4 v0 = tab[h], v1 = tab[(h + 1u) & mask], v2 = tab[(h + 2u) & mask], v3 = tab[(h + 3u) & mask];
        // all four reads in flight before the first use (one wait, not four)
        __asm__ volatile("" : "+v"(v0.x), "+v"(v1.x), "+v"(v2.x), "+v"(v3.x));
        const uint32_t meq = (uint32_t)key_eq(v0, a, b, c, d) | ((uint32_t)key_eq(v1, a, b, c, d) << 1) |
                             ((uint32_t)key_eq(v2, a, b, c, d) << 2) | ((uint32_t)key_eq(v3, a, b, c, d) << 3);
        const uint32_t mem = (uint32_t)key_empty(v0) | ((uint32_t)key_empty(v1) << 1) |
                             ((uint32_t)key_empty(v2) << 2) | ((uint32_t)key_empty(v3) << 3);
        const uint32_t stop = meq | mem;
        if (stop) {
            const uint32_t q = (uint32_t)__builtin_ctz(stop);
            slot = (h + q) & mask;
            return (meq >> q) & 1u;
        }
        h = (h + 4u) & mask;
    }
    // exhausted (unreachable under the 7/8 cap): "absent", so the caller's fill
    // check (commit: fill() + n >= cap_unique; memo_batch: no room) overflows the
    // walk or leaves the state unrecorded -- never a silently dropped entry
    slot = h;
    return false;
}

// Insert the keys of the lanes in `fresh`, each lane's `slot` from probe_lane
// against the current table (all absent).  Rounds: among the pending lanes the
// lowest lane targeting a slot wins it and all winners write at once; a loser
// finds its slot taken -- with DEDUP (keys may repeat: cousins from different
// parents) it drops out if the winner's key equals its own, otherwise it
// re-probes (checking equality too) to the next empty slot of its own probe
// sequence, and competes in the next round.  Returns `fresh` minus duplicates;
// the kept lane of equal keys is the lowest (equal keys share their probe
// chain, so they always meet on the same slot).  Linear probing stays valid.
// LDS tables (LOG_SLOTS <= 12) elect the winners with one ds_max_u32 of
// (64 - lane) on the target slot's last word and a read-back (3 LDS operations
// per round); the HBM tier compares slots lane by lane (v_readlane loop).
template <int LOG_SLOTS, bool DEDUP, typename SlotPtr>
__device__ __forceinline__ uint64_t place_batch(SlotPtr tab, uint64_t fresh, uint32_t a, uint32_t b, uint32_t c,
                                                uint32_t d, uint32_t slot) {
    constexpr uint32_t mask = (1u << LOG_SLOTS) - 1u;
    constexpr bool kLds = LOG_SLOTS <= 12;
    const int lane = threadIdx.x & 63;
    uint64_t pend = fresh;
    while (pend) {
        bool win = (pend >> lane) & 1ull;
        if (kLds) {
            // the claim marks are transient: every claimed slot is empty and is
            // overwritten by its winner's key before any lane reads the table again
            const uint32_t mark = 64u - (uint32_t)lane;
            uint32_t* w = (uint32_t*)&tab[slot] + 3;
            if (win) atomicMax(w, mark);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            if (win) win = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) == mark;
        } else {
            for (uint64_t m = pend; m; m &= m - 1ull) {
                const int src = __ffsll((unsigned long long)m) - 1;
                const uint32_t hs = rdl(slot, src);
                win = win && !(src < lane && slot == hs);
            }
        }
        if (win) tab[slot] = make_uint4(a, b, c, d);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        pend &= ~__ballot(win);
        if (!pend) break;
        bool drop = false;
        if ((pend >> lane) & 1ull) {
            drop = true;
            for (uint32_t it = 0; it <= mask; ++it) {
                const uint4 v = tab[slot];
                if (DEDUP && key_eq(v, a, b, c, d)) break;
                if (key_empty(v)) { drop = false; break; }
                slot = (slot + 1u) & mask;
            }
        }
        const uint64_t dups = __ballot(drop);
        pend &= ~dups;
        fresh &= ~dups;
    }
    return fresh;
}

// The lane whose run [pre, pre + cnt) holds flat position pp: the first lane with
// inclusive prefix incl = pre + cnt > pp (incl is non-decreasing over the lanes,
// so it is a lane with cnt > 0).  Binary search, 6 ds_bpermute.
__device__ __forceinline__ int parent_of(uint32_t pp, uint32_t incl) {
    int i = 0;
    #pragma unroll
    for (int st = 32; st >= 1; st >>= 1) {
        const uint32_t v = (uint32_t)__shfl((int)incl, i + st - 1);
        i = v <= pp ? i + st : i;
    }
    return i < 64 ? i : 63;
}

__device__ __forceinline__ int lane_rank(uint64_t m) {          // set bits of m below this lane
    const int lane = threadIdx.x & 63;
    return __popcll(m & ((1ull << lane) - 1ull));
}

// position of the j-th (0-based) set bit of m (j < popcount(m)), per lane
__device__ __forceinline__ int select_bit(uint32_t m, int j) {
    int pos = 0;
    #pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        const int c = __popc(m & ((1u << w) - 1u));
        const bool up = j >= c;
        j -= up ? c : 0;
        m = up ? m >> w : m;
        pos += up ? w : 0;
    }
    return pos;
}

// lane `src`'s Node (per-lane source index: ds_bpermute)
__device__ __forceinline__ Node shfl_node(const Node& t, int src) {
    Node s;
    s.lo = (uint64_t)(uint32_t)__shfl((int)(uint32_t)t.lo, src) |
           ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(t.lo >> 32), src) << 32);
    s.hi = (uint32_t)__shfl((int)t.hi, src);
    s.k3 = (uint32_t)__shfl((int)t.k3, src);
    s.occ = (uint32_t)__shfl((int)t.occ, src);
    s.blot = (uint32_t)__shfl((int)t.blot, src);
    s.n_home = __shfl(t.n_home, src);
    return s;
}

__device__ __forceinline__ Node rd_node(const Node& t, int src) {
    Node s;
    s.lo = (uint64_t)rdl((uint32_t)t.lo, src) | ((uint64_t)rdl((uint32_t)(t.lo >> 32), src) << 32);
    s.hi = rdl(t.hi, src);
    s.k3 = rdl(t.k3, src);
    s.occ = rdl(t.occ, src);
    s.blot = rdl(t.blot, src);
    s.n_home = (int)rdl((uint32_t)t.n_home, src);
    return s;
}

// ------------------------------------------------------------ enumeration --
// Filtered-list bookkeeping (filter_full_moves_by_max_submoves,
// get_all_moves.py:73-94): entries shorter than the running maximum can never
// survive the final filter, so the kernel keeps only entries of the current
// maximum length, in insertion order, and restarts the list when a longer one
// appears.  The first `cap` survivors are written (env truncation,
// backgammon_env.py:219-231); `count` keeps the untruncated total.
// Revisit pruning for doubles (exact): the insert attempts of a subtree depend
// only on its root state S and depth (plus got4, which only ever turns on).
// When S is reached again at the same depth, every attempt it would make was
// already made by the first visit (a partial prefix is attempted only while
// got4 is off, and got4 off now means it was off throughout the first visit;
// 4-long leaves are attempted unconditionally), so all of them are duplicates
// and the revisit is a no-op: skip it.  Memo tables are per depth (2 and 3),
// in LDS, 128 slots at depth 2 and 512 at depth 3 (a big doubles position has
// ~60-130 distinct depth-2 states and ~250-700 at depth 3; a nearly full table
// means long probe chains); when one fills up it stops recording (still exact).
constexpr int kLogMemo2 = 7, kLogMemo3 = 9;
constexpr int kMemoSlots = (1 << kLogMemo2) + (1 << kLogMemo3);    // memo2 = [0, 128), memo3 = [128, 640)
constexpr int kMemoCap2 = (7 << kLogMemo2) / 8, kMemoCap3 = (7 << kLogMemo3) / 8;
constexpr int kLogCMemo = 9;      // MEMO_KIND 1: depth-2 and depth-3 entries share one 512-slot table

// Where surviving entries go.  MoveSink: the env's ordered move list in HBM
// (first `cap` entries).  Other sinks (bg_search.hip) keep afterstate keys.
struct MoveSink {
    static constexpr bool kEnc = true;     // needs the move encodings
    static constexpr bool kSet = false;    // the ORDERED list (first occurrences in DFS order)
    uint64_t* out;      // this game's move list, `cap` entries
    int cap;
    __device__ __forceinline__ void reset() {}
    __device__ __forceinline__ void push(const Node&, uint64_t enc, int idx, int /*len*/) {
        if (idx < cap && (threadIdx.x & 63) == 0) out[idx] = enc;
    }
    // entries of the lanes in m (lane order) at idx0, idx0+1, ...
    __device__ __forceinline__ void push_lanes(uint64_t m, const Node&, uint64_t enc, int idx0, int /*len*/) {
        const int idx = idx0 + lane_rank(m);
        if (((m >> (threadIdx.x & 63)) & 1ull) && idx < cap) out[idx] = enc;
    }
};

// MEMO_KIND: 0 = separate depth-2 / depth-3 memo tables; 1 = one combined memo
// table; 2 = the memo lives in the dedup table itself.  Kinds 1-2 store tagged
// keys (hit-mask field complemented: >= 20 bits set, impossible for a real
// afterstate, which hits at most 4 blots; depth 3 also flips the bar nibble,
// and bar + off + sum(counts) = 15 keeps the depth-2 and depth-3 images apart).
constexpr uint32_t kTag2 = 0xFFFFFF00u, kTag3 = 0xFFFFFF0Fu;

// Gen::nd_first as a free function (also the 2-ply's row-level non-doubles walk)
__device__ __forceinline__ bool nd_first_of(int c, int kind, int lo, int hi, int pl, uint32_t root_occ,
                                            uint32_t root_blot, uint32_t blocked) {
    const int sg = pl == 0 ? 1 : -1, ph = c + sg * hi, pl_ = c + sg * lo;
    const bool rev_ok = (root_occ >> pl_) & 1u;
    const bool chain_ok = !((blocked >> ph) & 1u);
    const bool hblot = (root_blot >> ph) & 1u, lblot = (root_blot >> pl_) & 1u;
    if (kind == 1) return pl == 0 || !(rev_ok && !hblot);
    if (kind == 2) return pl == 1 || !(chain_ok && !hblot);
    return !rev_ok && !(chain_ok && !hblot && !lblot);
}

template <int LOG_SLOTS, typename SlotPtr, typename Sink = MoveSink, int MEMO_KIND = 0>
struct Gen {
    static constexpr bool TAGGED = MEMO_KIND == 2;
    SlotPtr tab;
    uint4* memo2;       // LDS memo tables (nullptr = no pruning)
    uint4* memo3;
    int memo_share = 3;  // MEMO_KIND 2: memo entries may take memo_share/8 of the table's capacity
    int n_memo2, n_memo3;
    Sink sink;
    int pl;
    uint32_t blocked;
    int cur_max, count, n_unique, cap_unique;
    bool ovf;
    bool pure_walk = false;   // this doubles walk visits every state once: no table, no memo
    bool mirror = false;      // ... in PLAYER2's mirrored order (set semantics only)
    bool forbid = false;      // ... PLAYER2, ordered: forbidden-point masks (kids())
    bool nd_free = false;     // nd_both's two-steps decided without the table (flat_leaves)
    bool clean = false;       // table (and memo) cleared for this run: callers leave it
                              // dirty and the walk clears it only if it needs it
    uint32_t root_occ = 0, root_blot = 0;

    // The children a walk visits below a sub-move with child bit `bit` that led
    // from node `from` to node `t` (q = t's child list, F = the forbidden points
    // above it).  forbid (PLAYER2 walks without bear-off, ordered semantics): the
    // walk visits the reference's smallest-key path of every state exactly once --
    // a point below an earlier sub-move's source that was occupied when that
    // sub-move was made could have moved first, in the smaller order, so it is
    // forbidden from then on (F grows by from.occ below bit; tools/check_canon.py
    // checks the lists against the oracle).  Otherwise canon_mask.
    __device__ __forceinline__ uint32_t kids(uint32_t q, int bit, int d, const Node& from, const Node& t,
                                             uint32_t& F) const {
        if (!forbid) return q & canon_mask(bit, d, pl, t, mirror);
        if (bit < 24) F |= from.occ & ((1u << bit) - 1u);
        return q & ~F;
    }

    // clear the dedup table and the separate memo tables before first use
    __device__ __forceinline__ void need_table() {
        if (clean) return;
        const int l = threadIdx.x & 63;
        for (int i = l; i < (1 << LOG_SLOTS); i += 64) tab[i] = make_uint4(0u, 0u, 0u, 0u);
        if (MEMO_KIND != 2 && memo2) {
            constexpr int n = MEMO_KIND == 1 ? (1 << kLogCMemo) : kMemoSlots;
            for (int i = l; i < n; i += 64) memo2[i] = make_uint4(0u, 0u, 0u, 0u);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        clean = true;
    }

    // table slots in use (dedup entries + tagged memo entries)
    __device__ __forceinline__ int fill() const { return n_unique + (TAGGED ? n_memo2 + n_memo3 : 0); }

    __device__ __forceinline__ void insert(const Node& s, uint64_t enc, int len) {
        const uint32_t a = (uint32_t)s.lo, b = (uint32_t)(s.lo >> 32);
        if (!pure_walk) {
            if (!table_insert<LOG_SLOTS>(tab, a, b, s.hi, s.k3)) return;
            ++n_unique;
            if (fill() >= cap_unique) { ovf = true; return; }
        }
        if (len > cur_max) { cur_max = len; count = 0; sink.reset(); }
        if (len == cur_max) {
            sink.push(s, enc, count, len);
            ++count;
        }
    }

    // Child `lane` of node s (list k, die d) on each lane whose bit is set in
    // k.bits: the expansion of one node runs one child per lane.
    __device__ __forceinline__ bool lane_child(const Node& s, const Kids& k, int d, Node& t, uint32_t& enc) const {
        const int l = threadIdx.x & 63;
        const bool act = l < 32 && ((k.bits >> l) & 1u);
        if (act) {
            const Sub m = child(s, k, l, d, pl);
            t = apply(s, m, pl);
            enc = Sink::kEnc ? m.enc : 0u;
        }
        return act;
    }

    // Add the entries of the lanes in `fresh` (length len), in lane order.
    // DEDUP: the batch may hold equal keys (cousins); first one wins.
    // pure: lanes whose entry is known to be new and never met again (nd_both's
    // pure two-steps): listed without a table slot.
    template <bool DEDUP = false>
    __device__ __forceinline__ void commit(uint64_t fresh, const Node& t, uint64_t enc, uint32_t slot, int len,
                                           uint64_t pure = 0ull) {
        int n = __popcll(fresh);
        if (!n && !pure) return;
        if (n) {
            BG_T0(tc);
            if (fill() + n >= cap_unique) { ovf = true; return; }
            fresh = place_batch<LOG_SLOTS, DEDUP>(tab, fresh, (uint32_t)t.lo, (uint32_t)(t.lo >> 32), t.hi, t.k3, slot);
            BG_T1(13, tc);
            BG_CNT(2, 1);
            if (DEDUP) n = __popcll(fresh);
            n_unique += n;
        }
        fresh |= pure;
        n = __popcll(fresh);
        BG_CNT(8, n);
        if (len > cur_max) { cur_max = len; count = 0; sink.reset(); }
        if (len == cur_max) {
            BG_T0(ts);
            sink.push_lanes(fresh, t, enc, count, len);
            BG_T1(11, ts);
            count += n;
        }
    }

    // Siblings (children of one node) are pairwise distinct afterstates
    // (different source points), so their duplicate checks against the set as
    // it stood before the batch run one per lane and only the new ones are
    // added, in child order -- the same set, list order and counts as the
    // reference's one-by-one add_unique_board calls.
    __device__ __forceinline__ void batch(bool act, const Node& t, uint64_t enc, int len) {
        uint32_t slot = 0;
        bool found = true;
        if (act) found = probe_lane<LOG_SLOTS>(tab, (uint32_t)t.lo, (uint32_t)(t.lo >> 32), t.hi, t.k3, slot);
        commit(__ballot(act && !found), t, enc, slot, len);
    }

    // All children of the parent nodes on the lanes in `parents` (lane = the
    // parent's child bit, so lane order is DFS order), flattened into 64-lane
    // chunks: leaf p of the chunk belongs to the parent whose prefix range holds
    // it and is that parent's (p - prefix)-th child.  Entries are
    // penc | enc << shift of length len.  Cousins may coincide: DEDUP commit.
    // d_up >= 0: both non-doubles passes in one batch (nd_both): parents on lanes
    // 0-31 are pass 1's first sub-moves (die d_up, child bit = lane), their
    // children use die d; parents on lanes 32-63 are pass 2's, children die d_up.
    // A pass-1 two-step (A, B) of two NORMAL sub-moves with b != dst(A) (no chain)
    // and dst(B) != a (no reverse chain) is PURE: its count change is -1 at a and
    // b, +1 at dst(A) and dst(B) with nothing cancelling, which only the same pair
    // produces within pass 1; every other walked entry either has a cancelling
    // pair (chains: one checker moved by both dice) or changes the bar / off
    // counts (bar entries, bear-offs), and pass 2 walks no other kind
    // (nd_both).  So a pure entry is new and is never met again: no table slot.
    __device__ __forceinline__ void flat_leaves(uint64_t parents, const Node& t, uint32_t q, int x, uint64_t penc,
                                                int d, int shift, int len, int d_up = -1) {
        const int l = threadIdx.x & 63;
        const bool par = (parents >> l) & 1ull;
        const uint32_t cnt = par ? (uint32_t)__popc(q) : 0u;         // <= 25
        uint32_t pre = 0, total = 0;
        const uint64_t below = (1ull << l) - 1ull;
        #pragma unroll
        for (int b = 0; b < 5; ++b) {
            const uint64_t m = __ballot((cnt >> b) & 1u);
            pre += (uint32_t)__popcll(m & below) << b;
            total += (uint32_t)__popcll(m) << b;
        }
        BG_CNT(6, 1);
        BG_CNT(7, total);
        for (uint32_t c = 0; c < total; c += 64) {
            const uint32_t pp = c + (uint32_t)l;
            const bool valid = pp < total;
            const int src = parent_of(pp, pre + cnt);
            const uint32_t qb = (uint32_t)__shfl((int)q, src);
            const int j = (int)(pp - (uint32_t)__shfl((int)pre, src));
            const Node s = shfl_node(t, src);
            const Kids k{qb, __shfl(x, src)};
            const uint64_t pe = !Sink::kEnc ? 0ull : (uint64_t)(uint32_t)__shfl((int)(uint32_t)penc, src) |
                                ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(penc >> 32), src) << 32);
            Node leaf;
            uint64_t enc = 0;
            uint32_t slot = 0;
            bool found = true, pure = false;
            if (valid) {
                const int cb = select_bit(qb, j);
                const Sub m = child(s, k, cb, d_up >= 0 && src >= 32 ? d_up : d, pl);
                leaf = apply(s, m, pl);
                enc = Sink::kEnc ? pe | ((uint64_t)m.enc << shift) : 0ull;
                if (d_up >= 0 && src < 24 && cb < 24) {
                    const int dst_a = pl == 0 ? src + d_up : src - d_up;
                    pure = cb != dst_a && m.dst != src;
                    if (nd_free && !pure) pure = nd_first(cb == dst_a ? src : cb, cb == dst_a ? 1 : 2, d, d_up);
                } else if (nd_free) {
                    pure = nd_first(src - 32, 3, d, d_up);      // pass 2: a chain (no specials here)
                }
                pure = pure || pure_walk;
                BG_T0(tp);
                if (!pure && !nd_free)
                    found = probe_lane<LOG_SLOTS>(tab, (uint32_t)leaf.lo, (uint32_t)(leaf.lo >> 32), leaf.hi, leaf.k3, slot);
                BG_T1(12, tp);
            }
            if (nd_free) { commit(0ull, leaf, enc, slot, len, __ballot(valid && pure)); continue; }
            commit<true>(__ballot(valid && !pure && !found), leaf, enc, slot, len, __ballot(valid && pure));
            if (ovf) return;
        }
    }

    // handle_non_doubles (handle_moves.py:109-200) for both dice orders of
    // get_all_possible_moves (get_all_moves.py:33-53) at once: lanes 0-31 hold the
    // first level of pass 1 (hi then lo; lane = child bit), lanes 32-63 that of
    // pass 2 (lo then hi); each pass's pre-scan (:144-155) is one ballot.
    // * Pass 1 has a two-step: its entries are two-steps (cur_max 2 from its first,
    //   never duplicate, leaf), so the skip rule (:41-53) cannot fire.  Pass 2 then
    //   adds either two-steps -- in the same flat batch, after pass 1's (lane order
    //   = insertion order; the first occurrence wins) -- or only singles, which can
    //   never survive the max-length filter: skipped.
    // * Otherwise the passes run in order (pass 1's singles, the skip rule, pass 2).
    // Pass 2's two-step (B, A) of two NORMAL sub-moves where A does not move B's
    // checker on (a != dst(B)) commutes (the argument of canon_mask with the dice
    // swapped): (A, B) is a pass-1 two-step, already inserted, so only chain moves
    // and bar entries / bear-offs are walked.
    // Without bar entries or bear-offs (nd_both: root not on the bar, >= 2
    // checkers off the home board) the only two-steps that can coincide move ONE
    // checker from c by hi + lo (s = the mover's direction):
    //   chain     (c, hi)(c+s.hi, lo), pass 1   hits: c+s.hi, c+s(hi+lo) if blots
    //   reverse   (c+s.lo, hi)(c, lo), pass 1   valid iff the root has a checker on
    //                                           c+s.lo (so no blot there); hits: c+s(hi+lo)
    //   pass-2    (c, lo)(c+s.lo, hi)           hits: c+s.lo, c+s(hi+lo)
    // (every other two-step changes the counts without cancelling: unique).  The
    // reverse one equals the pass-2 one whenever it exists, and the chain equals
    // the reverse one iff c+s.hi is no blot, the pass-2 one iff neither c+s.hi nor
    // c+s.lo is.  Walk order: PLAYER1 chain < reverse < pass-2 (first sub-move c <
    // c+lo), PLAYER2 reverse < chain < pass-2.  Returns whether the entry of kind
    // `kind` (1 chain, 2 reverse, 3 pass-2) is the first of its equals -- the one
    // the reference keeps -- with the chain's validity (c+s.hi not blocked).
    __device__ __forceinline__ bool nd_first(int c, int kind, int lo, int hi) const {
        return nd_first_of(c, kind, lo, hi, pl, root_occ, root_blot, blocked);
    }

    __device__ __forceinline__ void nd_both(const Node& s0, int hi, int lo) {
        const int l = threadIdx.x & 63;
        const bool up = l >= 32;
        const int bit = l & 31, da = up ? lo : hi, db = up ? hi : lo;
        const Kids kh = gen(s0, hi, pl, blocked), kl = gen(s0, lo, pl, blocked);
        const Kids k1{up ? kl.bits : kh.bits, up ? kl.extra : kh.extra};
        const bool a1 = (k1.bits >> bit) & 1u;
        Node t1;
        uint32_t e1 = 0, q2 = 0;
        int x2 = -1;
        if (a1) {
            const Sub m = child(s0, k1, bit, da, pl);
            t1 = apply(s0, m, pl);
            e1 = Sink::kEnc ? m.enc : 0u;
            const Kids k = gen(t1, db, pl, blocked);
            q2 = k.bits;
            x2 = k.extra;
        }
        constexpr uint64_t kLow = 0xFFFFFFFFull;
        const uint64_t two = __ballot(a1 && q2 != 0u);
        if (two & kLow) {
            if (up && a1 && bit < 24) q2 &= (1u << 31) | (1u << (pl == 0 ? bit + da : bit - da));
            uint64_t par = __ballot(a1 && q2 != 0u);
            if (!(two >> 32)) par &= kLow;
            nd_free = (s0.k3 & 15u) == 0u && 15 - s0.n_home - (int)((s0.k3 >> 4) & 15u) >= 2;
            if (nd_free) { root_occ = s0.occ; root_blot = s0.blot; }
            else need_table();
            flat_leaves(par, t1, q2, x2, (uint64_t)e1, lo, 16, 2, hi);
            nd_free = false;
            return;
        }
        need_table();
        batch(a1 && !up, t1, (uint64_t)e1, 1);                  // pass 1: singles
        if (ovf || (n_unique == 1 && cur_max == 1)) return;     // :41-53
        if (two) flat_leaves(two, t1, q2, x2, (uint64_t)e1, hi, 16, 2);
        else batch(a1 && up, t1, (uint64_t)e1, 1);
    }

    // Revisit check of a sibling batch at one depth: returns the lanes not seen
    // before and records them (while the memo has room).
    // DEDUP: the batch may hold equal states (cousins); the first in lane order is
    // the visit, later ones are revisits (pruned) -- when recorded.
    template <int LOGM, bool DEDUP = false>
    __device__ __forceinline__ uint64_t memo_batch(uint4* memo, int& nm, bool act, const Node& t, uint32_t tag) {
        if (!memo || pure_walk) return __ballot(act);
        constexpr int LOGT = MEMO_KIND == 1 ? kLogCMemo : LOGM;
        uint32_t slot = 0;
        bool found = true;
        const uint32_t k3 = MEMO_KIND != 0 ? t.k3 ^ tag : t.k3;
        if (act) {
            if (TAGGED) found = probe_lane<LOG_SLOTS>(tab, (uint32_t)t.lo, (uint32_t)(t.lo >> 32), t.hi, k3, slot);
            else found = probe_lane<LOGT>(memo, (uint32_t)t.lo, (uint32_t)(t.lo >> 32), t.hi, k3, slot);
        }
        const uint64_t fresh = __ballot(act && !found);
        uint64_t rec = fresh;
        int n = __popcll(rec);
        int room;
        if (MEMO_KIND == 0) room = ((7 << LOGM) / 8) - nm;
        else if (MEMO_KIND == 1) room = ((7 << kLogCMemo) / 8) - n_memo2 - n_memo3;
        else room = min(((7 << LOGM) / 8) - nm, cap_unique * memo_share / 8 - n_memo2 - n_memo3);
        while (n > room && rec) { rec &= ~(1ull << (63 - __clzll((long long)rec))); --n; }
        uint64_t kept = rec;
        if (rec) {
            if (TAGGED) kept = place_batch<LOG_SLOTS, DEDUP>(tab, rec, (uint32_t)t.lo, (uint32_t)(t.lo >> 32), t.hi, k3, slot);
            else kept = place_batch<LOGT, DEDUP>(memo, rec, (uint32_t)t.lo, (uint32_t)(t.lo >> 32), t.hi, k3, slot);
        }
        nm += __popcll(kept);
        return fresh & ~(rec & ~kept);
    }

    // Once got4 holds (dead ends are no-ops), the rest of a depth-1 subtree runs
    // level by level in DFS order: all depth-3 children of the depth-2 nodes on
    // the lanes in `parents` (lane order = DFS order), 64 at a time, the revisit
    // check (first in lane order wins) and each chunk's leaves as one flat batch.
    __device__ __forceinline__ void flat_depth3(uint64_t parents, const Node& t2, uint32_t q3, int x3, uint64_t penc2,
                                                int d, uint32_t F2) {
        const int l = threadIdx.x & 63;
        const bool par = (parents >> l) & 1ull;
        const uint32_t cnt = par ? (uint32_t)__popc(q3) : 0u;
        uint32_t pre = 0, total = 0;
        const uint64_t below = (1ull << l) - 1ull;
        #pragma unroll
        for (int b = 0; b < 5; ++b) {
            const uint64_t m = __ballot((cnt >> b) & 1u);
            pre += (uint32_t)__popcll(m & below) << b;
            total += (uint32_t)__popcll(m) << b;
        }
        BG_CNT(15, total);
        for (uint32_t c = 0; c < total; c += 64) {
            const uint32_t pp = c + (uint32_t)l;
            const bool valid = pp < total;
            const int src = parent_of(pp, pre + cnt);
            const uint32_t qb = (uint32_t)__shfl((int)q3, src);
            const int j = (int)(pp - (uint32_t)__shfl((int)pre, src));
            const Node s2 = shfl_node(t2, src);
            const Kids k{qb, __shfl(x3, src)};
            const uint64_t pe = !Sink::kEnc ? 0ull : (uint64_t)(uint32_t)__shfl((int)(uint32_t)penc2, src) |
                                ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(penc2 >> 32), src) << 32);
            uint32_t F3 = forbid ? (uint32_t)__shfl((int)F2, src) : 0u;
            Node t3;
            uint64_t pe3 = 0;
            int cb = 31;
            if (valid) {
                cb = select_bit(qb, j);
                const Sub m = child(s2, k, cb, d, pl);
                t3 = apply(s2, m, pl);
                pe3 = Sink::kEnc ? pe | ((uint64_t)m.enc << 32) : 0ull;
            }
            const uint64_t f3 = memo_batch<kLogMemo3, true>(memo3, n_memo3, valid, t3, kTag3);
            uint32_t q4 = 0;
            int x4 = -1;
            if ((f3 >> l) & 1ull) { const Kids kk = gen(t3, d, pl, blocked); q4 = kids(kk.bits, cb, d, s2, t3, F3); x4 = kk.extra; }
            flat_leaves(__ballot(((f3 >> l) & 1ull) && q4 != 0u), t3, q4, x4, pe3, d, 48, 4);
            if (ovf) return;
        }
    }

    // The same one level up: the depth-2 children of the depth-1 nodes on the
    // lanes in `parents`, 64 at a time, revisit check, then flat_depth3 per chunk.
    __device__ __forceinline__ void flat_depth2(uint64_t parents, const Node& t1, uint32_t q2, int x2, uint64_t penc1,
                                                int d, uint32_t F1) {
        const int l = threadIdx.x & 63;
        const bool par = (parents >> l) & 1ull;
        const uint32_t cnt = par ? (uint32_t)__popc(q2) : 0u;
        uint32_t pre = 0, total = 0;
        const uint64_t below = (1ull << l) - 1ull;
        #pragma unroll
        for (int b = 0; b < 5; ++b) {
            const uint64_t m = __ballot((cnt >> b) & 1u);
            pre += (uint32_t)__popcll(m & below) << b;
            total += (uint32_t)__popcll(m) << b;
        }
        BG_CNT(14, total);
        for (uint32_t c = 0; c < total; c += 64) {
            const uint32_t pp = c + (uint32_t)l;
            const bool valid = pp < total;
            const int src = parent_of(pp, pre + cnt);
            const uint32_t qb = (uint32_t)__shfl((int)q2, src);
            const int j = (int)(pp - (uint32_t)__shfl((int)pre, src));
            const Node s1 = shfl_node(t1, src);
            const Kids k{qb, __shfl(x2, src)};
            const uint64_t pe = !Sink::kEnc ? 0ull : (uint64_t)(uint32_t)__shfl((int)(uint32_t)penc1, src);
            uint32_t F2 = forbid ? (uint32_t)__shfl((int)F1, src) : 0u;
            Node t2;
            uint64_t pe2 = 0;
            int cb = 31;
            if (valid) {
                cb = select_bit(qb, j);
                const Sub m = child(s1, k, cb, d, pl);
                t2 = apply(s1, m, pl);
                pe2 = Sink::kEnc ? pe | ((uint64_t)m.enc << 16) : 0ull;
            }
            const uint64_t f2 = memo_batch<kLogMemo2, true>(memo2, n_memo2, valid, t2, kTag2);
            uint32_t q3 = 0;
            int x3 = -1;
            if ((f2 >> l) & 1ull) { const Kids kk = gen(t2, d, pl, blocked); q3 = kids(kk.bits, cb, d, s1, t2, F2); x3 = kk.extra; }
            flat_depth3(__ballot(((f2 >> l) & 1ull) && q3 != 0u), t2, q3, x3, pe2, d, F2);
            if (ovf) return;
        }
    }

    // handle_doubles (handle_moves.py:203-310): 4-deep pre-order DFS; partial
    // prefixes are inserted at dead ends only until the first 4-long sequence.
    // Each node's children are expanded one per lane (state, revisit check,
    // next-level child list); the walk itself stays in order.
    __device__ __forceinline__ void doubles(const Node& s0, int d) {
        BG_T0(td);
        doubles_(s0, d);
        BG_T1(1, td);
    }
    __device__ __forceinline__ void doubles_(const Node& s0, int d) {
        bool got4 = false;
        BG_CNT(0, 1);
        BG_T0(t_phase_a);
        const int l = threadIdx.x & 63;
        // no bear-off within 4 sub-moves: more than 3 checkers off the home board
        // (bar included; 15 - home - off, which only over-counts a short board)
        pure_walk = 15 - s0.n_home - (int)((s0.k3 >> 4) & 15u) > 3;
        mirror = pure_walk && pl == 1 && Sink::kSet;
        forbid = pure_walk && pl == 1 && !Sink::kSet;
        if (!pure_walk) need_table();
        // q*: a node's child list (dead-end test); c*: the children the walk
        // visits (canon_mask of the node's own child bit, which is its lane here)
        const Kids k1 = gen(s0, d, pl, blocked);
        Node t1;
        uint32_t e1 = 0;
        const bool a1 = lane_child(s0, k1, d, t1, e1);
        uint32_t q2 = 0, c2 = 0;
        int x2 = -1;
        uint32_t F1 = 0;       // forbidden points below each node (forbid mode)
        if (a1) { const Kids k = gen(t1, d, pl, blocked); q2 = k.bits; c2 = kids(q2, l, d, s0, t1, F1); x2 = k.extra; }
        if (pure_walk) {
            // Every state is visited once and no bear-off occurs, so a state's depth is
            // its length: when some 4-long sequence exists the list is exactly the
            // 4-long leaves in DFS order (the shorter dead ends are all filtered and
            // equal none of them) -- one flat pass over every depth-1 node, without
            // the in-order descent to the first 4-long leaf.  Otherwise (no 4-long
            // leaf: the dead ends are the list) the walk below runs from the start.
            flat_depth2(__ballot(a1 && c2 != 0u), t1, c2, x2, (uint64_t)e1, d, F1);
            if (ovf || cur_max == 4) return;
            count = 0;
            cur_max = 0;
            sink.reset();
        }
        for (uint32_t b1 = k1.bits; b1; b1 &= b1 - 1u) {
            if (got4) {
                flat_depth2((uint64_t)b1 & __ballot(c2 != 0u), t1, c2, x2, (uint64_t)e1, d, F1);
                return;
            }
            const int i1 = __builtin_ctz(b1);
            const Node s1 = rd_node(t1, i1);
            const Kids k2{rdl(c2, i1), (int)rdl((uint32_t)x2, i1)};
            const uint64_t m1 = rdl(e1, i1);
            if (!rdl(q2, i1)) {
                if (!got4) { insert(s1, m1, 1); if (ovf) return; }
                continue;
            }
            Node t2;
            uint32_t e2l = 0;
            const bool a2 = lane_child(s1, k2, d, t2, e2l);
            const uint64_t f2 = memo_batch<kLogMemo2>(memo2, n_memo2, a2, t2, kTag2);
            BG_CNT(3, __popcll(f2));
            uint32_t q3 = 0, c3 = 0;
            int x3 = -1;
            uint32_t F2 = forbid ? rdl(F1, i1) : 0u;
            if ((f2 >> l) & 1ull) { const Kids k = gen(t2, d, pl, blocked); q3 = k.bits; c3 = kids(q3, l, d, s1, t2, F2); x3 = k.extra; }
            for (uint64_t b2 = f2; b2; b2 &= b2 - 1ull) {
                if (got4) {
                    flat_depth3(b2 & __ballot(c3 != 0u), t2, c3, x3, m1 | ((uint64_t)e2l << 16), d, F2);
                    if (ovf) return;
                    break;
                }
                const int i2 = __ffsll((unsigned long long)b2) - 1;
                const Node s2 = rd_node(t2, i2);
                const Kids k3{rdl(c3, i2), (int)rdl((uint32_t)x3, i2)};
                const uint64_t m2 = m1 | ((uint64_t)rdl(e2l, i2) << 16);
                if (!rdl(q3, i2)) {
                    if (!got4) { insert(s2, m2, 2); if (ovf) return; }
                    continue;
                }
                Node t3;
                uint32_t e3l = 0;
                const bool a3 = lane_child(s2, k3, d, t3, e3l);
                const uint64_t f3 = memo_batch<kLogMemo3>(memo3, n_memo3, a3, t3, kTag3);
                BG_CNT(5, __popcll(f3));
                uint32_t q4 = 0, c4 = 0;
                int x4 = -1;
                uint32_t F3 = forbid ? rdl(F2, i2) : 0u;
                if ((f3 >> l) & 1ull) { const Kids k = gen(t3, d, pl, blocked); q4 = k.bits; c4 = kids(q4, l, d, s2, t3, F3); x4 = k.extra; }
                for (uint64_t b3 = f3; b3; b3 &= b3 - 1ull) {
                    const int i3 = __ffsll((unsigned long long)b3) - 1;
                    if (!rdl(q4, i3)) {
                        if (!got4) {
                            insert(rd_node(t3, i3), m2 | ((uint64_t)rdl(e3l, i3) << 32), 3);
                            if (ovf) return;
                        }
                        continue;
                    }
                    // from the first node with children on, got4 holds: dead ends are
                    // no-ops and every remaining node's leaves go out as one flat batch
                    // (that node's first visited child is the walk's first 4-long leaf:
                    // a skipped one would repeat an earlier 4-long leaf)
                    const uint64_t rest = b3 & __ballot(c4 != 0u);
                    BG_T1(9, t_phase_a); BG_CNT(10, 1);
                    flat_leaves(rest, t3, c4, x4, m2 | ((uint64_t)e3l << 32), d, 48, 4);
                    if (ovf) return;
                    got4 = true;
                    break;
                }
            }
        }
    }

    // non-doubles only (r0 != r1): the same as run() without the doubles code
    __device__ __forceinline__ void run_nd(const Node& s0, int r0, int r1) {
        cur_max = 0; count = 0; n_unique = 0; ovf = false; n_memo2 = 0; n_memo3 = 0; pure_walk = false; mirror = false; forbid = false; nd_free = false;
        const int hi = r0 > r1 ? r0 : r1, lo = r0 > r1 ? r1 : r0;
        nd_both(s0, hi, lo);
    }

    // doubles only (r0 == r1 == d)
    __device__ __forceinline__ void run_d(const Node& s0, int d) {
        cur_max = 0; count = 0; n_unique = 0; ovf = false; n_memo2 = 0; n_memo3 = 0; pure_walk = false; mirror = false; forbid = false; nd_free = false;
        doubles(s0, d);
    }

    // get_all_possible_moves (get_all_moves.py:9-70)
    __device__ __forceinline__ void run(const Node& s0, int r0, int r1) {
        cur_max = 0; count = 0; n_unique = 0; ovf = false; n_memo2 = 0; n_memo3 = 0; pure_walk = false; mirror = false; forbid = false; nd_free = false;
        if (r0 != r1) {
            const int hi = r0 > r1 ? r0 : r1, lo = r0 > r1 ? r1 : r0;
            nd_both(s0, hi, lo);
        } else {
            doubles(s0, r0);
        }
    }
};

// ------------------------------------------------------- board <-> state --
// Lane l holds byte l of a 64-byte lane record (bytes 0..51 = the board in the
// product layout p1[24] p2[24] bar[2] off[2]).  Returns the wave-uniform node
// of player `pl` plus the opponent masks.
__device__ __forceinline__ Node node_from_bytes(int bv, int pl, uint32_t& blocked) {
    const int lane = threadIdx.x & 63;
    const int p = lane < 24 ? lane : 0;
    int own = __shfl(bv, pl * 24 + p);
    int opp = __shfl(bv, (1 - pl) * 24 + p);
    if (lane >= 24) { own = 0; opp = 0; }
    Node s;
    s.occ = (uint32_t)__ballot(own > 0);
    blocked = (uint32_t)__ballot(opp >= 2);
    s.blot = (uint32_t)__ballot(opp == 1);
    uint32_t w = (uint32_t)(own & 15) << (4 * (lane & 7));
    w |= __shfl_xor(w, 1); w |= __shfl_xor(w, 2); w |= __shfl_xor(w, 4);
    s.lo = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(w, 0) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(w, 8) << 32);
    s.hi = (uint32_t)__builtin_amdgcn_readlane(w, 16);
    const uint32_t own_bar = (uint32_t)__builtin_amdgcn_readlane(bv, 48 + pl);
    const uint32_t own_off = (uint32_t)__builtin_amdgcn_readlane(bv, 50 + pl);
    s.k3 = (own_bar & 15u) | ((own_off & 15u) << 4);
    int nh = 0;
    if (pl == 0) { for (int q = 18; q < 24; ++q) nh += (int)((s.hi >> (4 * (q - 16))) & 15u); }
    else { for (int q = 0; q < 6; ++q) nh += (int)((s.lo >> (4 * q)) & 15u); }
    s.n_home = nh;
    return s;
}

// Inverse: the new byte for lane l (< 52) after the mover `pl` went from the
// root (bytes bv) to node s.  Bytes >= 52 are returned unchanged.
__device__ __forceinline__ int bytes_from_node(int bv, const Node& s, int pl) {
    const int lane = threadIdx.x & 63;
    const uint32_t hits = s.k3 >> 8;
    int v = bv;
    if (lane < 48) {
        const int row = lane / 24, p = lane - 24 * row;
        if (row == pl) v = own_at(s, p);
        else v = bv - (int)((hits >> p) & 1u);
    } else if (lane == 48 + pl) v = (int)(s.k3 & 15u);
    else if (lane == 49 - pl) v = bv + __builtin_popcount(hits);
    else if (lane == 50 + pl) v = (int)((s.k3 >> 4) & 15u);
    return v;
}

// ----------------------------------------------------------------- encoder --
// get_board_features (immutable_board.py:171-212) == get_board_features_batch_
// from_tensors (ai/batching.py:78-147): 198 f32 per board.
__constant__ static const float kOff15[16] = {
    0.0f / 15.0f, 1.0f / 15.0f, 2.0f / 15.0f, 3.0f / 15.0f, 4.0f / 15.0f, 5.0f / 15.0f,
    6.0f / 15.0f, 7.0f / 15.0f, 8.0f / 15.0f, 9.0f / 15.0f, 10.0f / 15.0f, 11.0f / 15.0f,
    12.0f / 15.0f, 13.0f / 15.0f, 14.0f / 15.0f, 15.0f / 15.0f};

// Feature f (0..197) of the board whose byte l is in lane l's `bv`.
__device__ __forceinline__ float feature_at(int bv, int f, int cur) {
    const int p = f >= 98 ? 1 : 0;
    const int g = f - 98 * p;
    int idx;
    if (f >= 196) idx = 0;
    else if (g < 96) idx = p * 24 + (g >> 2);
    else idx = (g == 96 ? 48 : 50) + p;
    const int n = __shfl(bv, idx);
    if (f >= 196) return (f == 196) == (cur == 0) ? 1.0f : 0.0f;
    if (g < 96) {
        const int u = g & 3;
        if (u < 3) return n >= u + 1 ? 1.0f : 0.0f;
        return n >= 3 ? (float)(n - 3) * 0.5f : 0.0f;
    }
    if (g == 96) return (float)n * 0.5f;
    return kOff15[n & 15];
}

}  // namespace bg
