/*
 * bgx.h — C ABI of the MI355X-native backgammon self-play engine (libbgx.so).
 *
 * Plain C: pointers and sizes only, no exceptions, no torch/HIP types.  Every
 * device pointer is a HIP device allocation on the engine's device; `stream`
 * is a hipStream_t passed as void* (NULL = the default stream).  All work is
 * enqueued on that stream; no entry point synchronises the host unless it says
 * so.  Return value: BGX_OK (0) or a negative bgx_status.
 *
 * Each entry point names the reference interface it replaces
 * (Nick-qsv/MLP-PPO-2PLY-P3, paths relative to its src/).
 *
 * Data formats
 *   board52   int8[52]  = P1 points[24], P2 points[24], bar[2] (P1,P2), off[2]
 *                         (the reference's (4,24) int8 tensor, immutable_board.py:20-24,
 *                          with its 44 always-zero bytes dropped)
 *   move      uint64    = up to 4 sub-moves, sub-move i in bits 16i..16i+15:
 *                         start(5) | end(5)<<5 | hits_blot(1)<<10 | valid(1)<<15,
 *                         start/end are Position values (0..23, BAR=24, BEAR_OFF=25)
 *                         (SubMove/FullMove, moves/move_types.py:38-48)
 *   features  float[198] per board (immutable_board.py:171-212)
 *   info      int32 per lane: mover | (winner+1)<<8 | game_score<<16 | kind<<24,
 *                         kind 0 = move, 1 = pass, 2 = invalid action, 3 = reset on game over
 */
#ifndef BGX_H
#define BGX_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bgx_engine bgx_engine;

enum bgx_status {
    BGX_OK = 0,
    BGX_EINVAL = -1,     /* bad argument */
    BGX_EDEVICE = -2,    /* HIP error (launch, memory, device selection) */
    BGX_ENOMEM = -3,     /* device allocation failed */
    BGX_EOVERFLOW = -4,  /* a position exceeded the slow-path dedup capacity */
    BGX_ESTATE = -5      /* the engine's lanes changed while a call was reading them (see below) */
};

/* Stream ordering.  Every call that takes a bgx_engine* orders itself after the
 * engine's previous call: when it comes on a different stream than that call, its
 * stream first waits (hipStreamWaitEvent) for the previous call's work, so a step on
 * one stream followed by bgx_two_ply / bgx_one_ply / bgx_copy_lanes / ... on another
 * reads the lanes the step wrote (the engine's lanes, move lists, overflow queues and
 * tables and the search workspace are one piece of device state).  Calls captured into
 * a HIP graph are ordered by the graph: its launch stream must follow whatever else
 * used the engine, and a call after a graph launch on another stream must be ordered
 * by the caller.  Kernels that take raw lane pointers (bgx_policy_act*, reading
 * bgx_buffers.lanes) run on the caller's stream as given.  The host-side state calls
 * without a stream (bgx_engine_seed, bgx_engine_mt_state, bgx_engine_error) synchronise
 * the device before and after.  bgx_two_ply returns
 * BGX_ESTATE (and bgx_one_ply sets bit 1 of the engine's error word) if it finds a
 * lane whose legal moves no longer match its row layout, instead of reading past them. */

enum bgx_dice_mode {
    BGX_DICE_MT_LANE = 0,    /* lane i == one BackgammonEnv after env.seed(seeds[i]) (numpy legacy MT19937) */
    BGX_DICE_MT_SHARED = 1,  /* one numpy stream consumed in lane order == VectorizedBackgammonEnv after np.random.seed */
    BGX_DICE_PHILOX = 2      /* Philox4x32-10 per lane (speed mode; same die distribution) */
};

/* BackgammonEnv(match_length, max_legal_moves) x batch (backgammon_env.py:38-75,
 * vec_bg_env.py:8-18).  auto_reset=1: a finished game is reset inside the same
 * step and the post-reset observation is returned (VectorizedBackgammonEnv.step,
 * vec_bg_env.py:35-36); auto_reset=0: BackgammonEnv semantics (the NEXT step
 * resets and returns done=1, backgammon_env.py:119-121). */
int bgx_engine_create(int device, int32_t batch, int32_t max_moves, uint64_t seed, int32_t dice_mode,
                      int32_t auto_reset, int32_t match_length, bgx_engine** out);
/* Order `stream` after every piece of a step still running on the engine's own
 * side streams (the next step's dispatch order): a HIP graph capture of steps
 * calls it before capturing and as its last captured call, so the graph holds no
 * work it does not join. */
int bgx_engine_join(bgx_engine* e, void* stream);
/* Where a Philox step's light launch (the non-predicted-doubles rest of the dispatch
 * order) and the next step's dispatch order run: fork = 1 (default) on the engine's
 * side stream, fork-joined on events beside the heavy launch; fork = 0 on the caller's
 * stream after it.  Same results either way.  A HIP graph of fork = 0 steps is one
 * linear chain: several such engines on their own streams then map one-to-one onto
 * the hardware queues (bench.py C3: 4 shards), where forked graphs' internal streams
 * share queues with the other shards' and serialise them.
 * Turning the fork off joins a pending dispatch order into `stream`. */
int bgx_engine_set_fork(bgx_engine* e, int32_t fork, void* stream);
int bgx_engine_destroy(bgx_engine* e);

/* BackgammonEnv.seed (backgammon_env.py:357-363): per-lane MT19937 seeds
 * (host array of `batch` uint32; mode SHARED uses seeds[0]); Philox: key = seed. */
int bgx_engine_seed(bgx_engine* e, const uint32_t* seeds_host, uint64_t philox_seed);

/* Read (set=0) or overwrite (set=1) the MT19937 state of one lane (mode
 * MT_LANE) or of the shared stream (mode MT_SHARED, lane ignored):
 * state_host uint32[625] = numpy's get_state() key[624] + pos.  Lets the
 * drop-in classes draw dice from numpy's global RandomState exactly as the
 * reference does (backgammon_env.py:245-246).  Synchronous. */
int bgx_engine_mt_state(bgx_engine* e, int32_t lane, uint32_t* state_host, int32_t set);

/* Device buffers owned by the engine (read-only for callers unless stated). */
typedef struct {
    uint8_t* lanes;      /* [batch][64] lane records: board52, cur(52), roll(53,54), game_over(55),
                            match_over(56), score P1/P2 (57,58), n_moves int16 (60,61) */
    uint64_t* moves;     /* [batch][max_moves] legal moves of the current position */
    int32_t* n_total;    /* [batch] untruncated legal-move count (len before [:max_moves]) */
    int32_t batch, max_moves;
} bgx_buffers;
int bgx_engine_buffers(bgx_engine* e, bgx_buffers* out);

/* BackgammonEnv.reset (backgammon_env.py:78-113) for lanes with lane_mask[i]!=0
 * (lane_mask NULL = all lanes).  obs_dev: float[batch][198] (all lanes written; may be NULL). */
int bgx_reset(bgx_engine* e, const uint8_t* lane_mask_dev, float* obs_dev, void* stream);

/* BackgammonEnv.step / VectorizedBackgammonEnv.step (backgammon_env.py:115-191,
 * vec_bg_env.py:28-49) on every lane.  actions_dev int32[batch]; outputs
 * obs float[batch][198], reward float[batch], done uint8[batch], info int32[batch]
 * (obs_dev and info_dev may be NULL: a rollout that stores int8 boards skips the
 * 792-byte fp32 observation). */
int bgx_step(bgx_engine* e, const int32_t* actions_dev, float* obs_dev, float* reward_dev, uint8_t* done_dev,
             int32_t* info_dev, void* stream);

/* get_all_possible_moves (moves/get_all_moves.py:9-70) + truncation to max_moves
 * (backgammon_env.py:219-231) on n arbitrary positions.  boards52_dev int8[n][52],
 * players_dev uint8[n], dice_dev uint8[n][2]; outputs n_moves int16[n] (truncated),
 * n_total int32[n] (untruncated, may be NULL), moves uint64[n][max_moves]. */
int bgx_movegen(bgx_engine* e, const int8_t* boards52_dev, const uint8_t* players_dev, const uint8_t* dice_dev,
                int32_t n, int32_t max_moves, int16_t* n_moves_dev, int32_t* n_total_dev, uint64_t* moves_dev,
                void* stream);

/* ImmutableBoard.get_board_features (immutable_board.py:171-212) /
 * get_board_features_batch_from_tensors (ai/batching.py:78-147). */
int bgx_encode(const int8_t* boards52_dev, const uint8_t* players_dev, int32_t n, float* out_dev, void* stream);

/* The same 198 features from n 64-byte lane records (records_dev: n x 64 bytes,
 * board bytes 0..51, player to move at byte 52 -- the rollout rows the PPO update
 * re-encodes, ppo_agent.py:221-229 / 274 stacks the stored observations and casts
 * them under autocast).  dtype 0: fp32 [n][198]; 1: fp16 [n][198], the round to
 * nearest of the fp32 features (autocast's cast). */
int bgx_encode_records(const uint8_t* records_dev, int32_t n, int32_t dtype, void* out_dev, void* stream);
/* The same with a row width of 198 or 208 elements: columns 198..width-1 are
 * zero (208: 16-byte aligned rows, which hipBLASLt's vector-load GEMMs need for
 * the PPO update's fc1 forward and weight gradient; the zero columns meet zero
 * weight columns, so the products are unchanged). */
int bgx_encode_records_ex(const uint8_t* records_dev, int32_t n, int32_t dtype, int32_t width, void* out_dev,
                          void* stream);

/* execute_full_move_on_board_copy (immutable_board.py:224-233) over every legal
 * move of lanes [lane0, lane0+nlanes): boards52 int8[nlanes][max_moves][52]
 * (rows past n_moves are zero). */
int bgx_afterstates(bgx_engine* e, int32_t lane0, int32_t nlanes, int8_t* boards52_dev, void* stream);

/* generate_all_board_features + zero padding (ai/batching.py:10-75,
 * backgammon_env.py:207-243) for lanes [lane0, lane0+nlanes):
 * out float[nlanes][max_moves][198], the mover's one-hot. */
int bgx_legal_features(bgx_engine* e, int32_t lane0, int32_t nlanes, float* out_dev, void* stream);

/* BackgammonEnv.action_mask / VectorizedBackgammonEnv.get_action_masks
 * (backgammon_env.py:232-236, vec_bg_env.py:51-56): counts_dev int16[batch]
 * (= number of legal actions, mask = iota < count; may be NULL) and/or
 * masks_dev float[batch][max_moves] (1.0 for the first count entries; may be NULL). */
int bgx_action_masks(bgx_engine* e, int16_t* counts_dev, float* masks_dev, void* stream);

/* Copy lane state [lane0, lane0+n) out of the engine (device-to-device, async):
 * lanes_dst uint8[n][64], moves_dst uint64[n][max_moves], n_total_dst int32[n];
 * any destination may be NULL.  (The reference exposes env.board / env.legal_moves
 * / env.current_player / env.roll_result as attributes, backgammon_env.py:51-75.) */
int bgx_copy_lanes(bgx_engine* e, int32_t lane0, int32_t n, uint8_t* lanes_dst, uint64_t* moves_dst,
                   int32_t* n_total_dst, void* stream);

/* Overwrite lane records [lane0, lane0+n) (board52 + metadata, 64 bytes each) and
 * re-enumerate their legal moves for the stored player/roll: lets a caller pose
 * arbitrary positions (tests, analysis).  lanes_src uint8[n][64] on the device. */
int bgx_set_lanes(bgx_engine* e, int32_t lane0, int32_t n, const uint8_t* lanes_src, void* stream);
/* bgx_set_lanes with regen = 0: the records are written as given and the stored
 * legal moves / counts are left as they were -- the reference's BackgammonEnv.roll_dice
 * and pass_turn change roll_result / current_player without touching legal_moves
 * until update_legal_moves() runs (backgammon_env.py:198-251); regen = 1 is
 * bgx_set_lanes (that update_legal_moves). */
int bgx_set_lanes_ex(bgx_engine* e, int32_t lane0, int32_t n, const uint8_t* lanes_src, int32_t regen, void* stream);

/* Rollout rows to pinned host memory (the reference keeps its rollout memory on
 * the host, ppo_agent.py:175-187): up to BGX_MAX_COPY_REGIONS strided 2-D copies in
 * ONE kernel launch, so a HIP graph of rollout steps can carry the copy of a slot
 * pair of every field as one node.  Region i copies `rows` rows of `width` bytes
 * from src (row pitch spitch) to dst (pitch dpitch); device pointers on both sides
 * (a pinned host buffer's device pointer from bgx_host_device_ptr); widths,
 * pitches and pointers 16-byte aligned.  workgroups <= 0: up to 64. */
#define BGX_MAX_COPY_REGIONS 8
typedef struct {
    const void* src;
    void* dst;
    int64_t width, rows, spitch, dpitch;
} bgx_region;
int bgx_copy_regions(const bgx_region* regions, int32_t n, int32_t workgroups, void* stream);
/* The device-side address of pinned (hipHostMalloc / torch pin_memory) host memory. */
int bgx_host_device_ptr(void* host_ptr, void** dev_ptr_out);

/* Sticky device error word (bit 0: a position overflowed the slow-path dedup
 * table; bit 1: bgx_one_ply found a lane changed under it, see "Stream ordering").
 * Synchronises the engine's device. */
int bgx_engine_error(bgx_engine* e, int32_t* err_out);

/* ---- policy network (agent/policy_network.py:44-75) + select_action (ppo_agent.py:138-191) ----
 * Weights are packed once per update into MFMA operand order (f16 hi/lo split
 * pairs with power-of-two scales; fp32-equivalent results, see bg_mlp.hip):
 * bgx_policy_packed_size(H, A) floats; H <= 128.  Inputs are torch nn.Linear
 * layouts: W1 [H][198], b1 [H], Wa [A][H], ba [A], wv [H], bv [1]. */
int bgx_policy_packed_size(int32_t hidden, int32_t n_actions);
int bgx_policy_pack(const float* W1, const float* b1, const float* Wa, const float* ba, const float* wv, const float* bv,
                    int32_t hidden, int32_t n_actions, float* packed_dev, void* stream);

/* One fused pass per game lane: features from the 64-byte lane record
 * (bgx_buffers.lanes layout), relu(W1 x + b1), logits = Wa h + ba, value = wv h + bv,
 * masked = logits + log(mask + 1e-45) with mask = [a < legal count], then
 * action ~ Categorical(softmax(masked)) (Gumbel-max, noise hashed from (seed, step, row, a))
 * or argmax if greedy (eval mode, ppo_agent.py:188-191).  act_out int32[n],
 * logp_out float[n] (log softmax(masked)[action]), value_out float[n];
 * logits_out float[n][32*ceil((A+1)/32)] (raw logits, value at column A) may be
 * NULL, as may logp_out/value_out. */
int bgx_policy_act(const uint8_t* records_dev, int32_t n, const float* packed_dev, int32_t hidden, int32_t n_actions,
                   uint64_t seed, uint32_t step, int32_t greedy, int32_t* act_out, float* logp_out, float* value_out,
                   float* logits_out, void* stream);

/* bgx_policy_act that also writes each row's 64-byte input record to
 * records_out uint8[n][64] (the rollout's stored observation,
 * select_action appends the state to memory, ppo_agent.py:176-185), so a rollout reads the
 * engine's lane buffer (bgx_buffers.lanes) in place with no separate copy.
 * records_out may be NULL (then identical to bgx_policy_act). */
int bgx_policy_act_rec(const uint8_t* records_dev, int32_t n, const float* packed_dev, int32_t hidden,
                       int32_t n_actions, uint64_t seed, uint32_t step, int32_t greedy, int32_t* act_out,
                       float* logp_out, float* value_out, float* logits_out, uint8_t* records_out, void* stream);

/* bgx_policy_act_rec whose noise step is step + *step_ctr, read on the device when
 * the kernel runs (step_ctr may be NULL: then exactly bgx_policy_act_rec).  A HIP
 * graph that captures rollout steps replays with fresh draws when the graph also
 * advances the counter (bgx_counter_add). */
int bgx_policy_act_ctr(const uint8_t* records_dev, int32_t n, const float* packed_dev, int32_t hidden,
                       int32_t n_actions, uint64_t seed, uint32_t step, const uint32_t* step_ctr, int32_t greedy,
                       int32_t* act_out, float* logp_out, float* value_out, float* logits_out, uint8_t* records_out,
                       void* stream);
/* *ctr_dev += v on the stream (one thread). */
int bgx_counter_add(uint32_t* ctr_dev, uint32_t v, void* stream);

/* ---- value head search: V(x) = value_head(relu(fc1 x)), H <= 128 ----
 * bgx_value_pack packs fc1.weight [H][198], fc1.bias [H], value_head.weight [H],
 * value_head.bias [1] into bgx_value_packed_size(H) floats (MFMA operand order);
 * value_bias is value_head.bias[0] passed by value. */
int bgx_value_packed_size(int32_t hidden);
int bgx_value_pack(const float* W1, const float* b1, const float* wv, const float* bv, int32_t hidden,
                   float* packed_dev, void* stream);

/* 1-ply greedy over every lane's legal afterstates (features with the mover's
 * one-hot, as legal_board_features, backgammon_env.py:207-216): best_out int32[B]
 * = first argmax V, bestv_out float[B], values_out float[B][max_moves] (may be NULL). */
int bgx_one_ply(bgx_engine* e, const float* vpacked_dev, int32_t hidden, float value_bias, int32_t* best_out,
                float* bestv_out, float* values_out, void* stream);

/* 2-ply expectimax over the 21 rolls (get_all_dice_rolls.py:5-34) for every lane:
 * Q(a) = sum_r p_r min_{opponent replies b} V(enc(b, mover)), leaf = a when the
 * opponent cannot move (every leaf carries the root mover's one-hot, the
 * reference's evaluate_board(board, current_player), expect_minmax.py:57-58,
 * 100-143); best_out = first argmax Q.  q_out float[B][max_moves] and
 * bestq_out may be NULL; stats_host (may be NULL) receives {leaves evaluated,
 * (afterstate, roll) jobs, afterstates}.  Synchronises the stream (sizes its
 * workspace from the afterstate count). */
int bgx_two_ply(bgx_engine* e, const float* vpacked_dev, int32_t hidden, float value_bias, int32_t* best_out,
                float* bestq_out, float* q_out, uint64_t* stats_host, void* stream);

/* ---- PPO update loss head (ppo_agent.py:268-305), fused ----
 * For n rows: masked log-softmax of the logits (dtype 0 = fp32, 1 = fp16, row
 * stride ld_logits; mask from the legal count in bytes 60-61 of each 64-byte
 * lane record: log(1e-45) for illegal actions), ratio = exp(logp[action] -
 * old_logp), clipped surrogate (eps_clip), value MSE, entropy.  Writes the
 * gradients of  policy + c_value * value - c_entropy * entropy  (per-row losses,
 * times grad_scale) with respect to the logits (dlogits, same dtype, row stride
 * ld_dlogits) and the values (dvalues, same dtype), as torch autograd forms them,
 * and adds the sums of the per-row policy loss, squared value error and entropy
 * to sums[0..2] (double, device). */
int bgx_ppo_head(const void* logits_dev, int32_t dtype, int64_t ld_logits, const void* values_dev,
                 const uint8_t* records_dev, const int32_t* actions_dev, const float* old_logp_dev,
                 const float* returns_dev, const float* adv_dev, int32_t n, int32_t n_actions, float eps_clip,
                 float c_value, float c_entropy, float grad_scale, void* dlogits_dev, int64_t ld_dlogits,
                 void* dvalues_dev, double* sums_dev, void* stream);

/* bgx_ppo_head for a [logits | value | 0 ...] layout (one GEMM for both heads,
 * row stride ld_dlogits <= 512): with pad_value_col != 0 the kernel also writes
 * the value gradient into column n_actions of dlogits and zeros up to
 * ld_dlogits; with colsum != NULL (float[BGX_PPO_COLSUM_BLOCKS][512]) each
 * workgroup writes the column sums of the gradient it stored (fp16-rounded
 * when dtype = 1) — the bias gradient, summed over the first dimension by the
 * caller.  dvalues_dev is written as in bgx_ppo_head. */
#define BGX_PPO_COLSUM_BLOCKS 2048
int bgx_ppo_head_ex(const void* logits_dev, int32_t dtype, int64_t ld_logits, const void* values_dev,
                    const uint8_t* records_dev, const int32_t* actions_dev, const float* old_logp_dev,
                    const float* returns_dev, const float* adv_dev, int32_t n, int32_t n_actions, float eps_clip,
                    float c_value, float c_entropy, float grad_scale, void* dlogits_dev, int64_t ld_dlogits,
                    void* dvalues_dev, double* sums_dev, int32_t pad_value_col, float* colsum_dev, void* stream);

/* The fp16 epoch's ReLU backward of fc1 (policy_network.py:70; autograd passes the
 * gradient where relu's output > 0) in place on dh [n][hidden] fp16, given the
 * stored activations h [n][hidden] fp16 (16-byte aligned, hidden % 8 == 0,
 * hidden <= 256), with the bias gradient's partial column sums of the masked dh
 * in colsum[blocks][hidden] (fp32; the caller sums the rows). */
int bgx_relu_backward(void* dh, const void* h, int32_t n, int32_t hidden, float* colsum, int32_t blocks,
                      void* stream);

/* The fp16 epoch's fc1 forward from the stored records (ppo_agent.py:274 under
 * autocast, policy_network.py:69-70): h[n][hidden] fp16 = relu(W1h . fp16(x) + b1h)
 * with fp32 accumulation, x = the 198 features of each 64-byte record (off/15
 * rounded to fp16 as autocast's cast rounds it).  W1h [hidden][198] fp16 is packed
 * once per weight update by bgx_fc1_pack into bgx_fc1_packed_size(hidden) bytes
 * (16-byte aligned); b1h [hidden] fp16.  hidden % 4 == 0, hidden <= 128; h 8-byte
 * aligned.  Replaces the materialised feature rows + GEMM for the forward; the
 * weight gradient still reads the encoded features. */
int bgx_fc1_packed_size(int32_t hidden);
int bgx_fc1_pack(const void* w1h_dev, int32_t hidden, void* packed_dev, void* stream);
int bgx_fc1_records(const uint8_t* records_dev, int32_t n, const void* packed_dev, const void* b1h_dev,
                    int32_t hidden, void* h_dev, void* stream);
/* bgx_fc1_records that also raises *hmax2_dev (fp32, device; may be NULL) to the
 * largest |h_row|^2 of its rows (the bound PPOTrainer checks for the fused head's
 * masked-action shortcut, bgx_ppo_rows). */
int bgx_fc1_records_ex(const uint8_t* records_dev, int32_t n, const void* packed_dev, const void* b1h_dev,
                       int32_t hidden, void* h_dev, float* hmax2_dev, void* stream);

/* The fp16 epoch's output layer + loss head without materialised logits
 * (csrc/bg_ppo_fused.hip; replaces, inside ppo_agent.py:268-305 under autocast,
 * the [action_head; value_head] GEMM of policy_network.py:71-75, the loss head of
 * bgx_ppo_head_ex, dh = dy W2h, the ReLU backward and gW2 / gb2 = dy^T [h | 1]).
 * hidden = 128, n_actions = 500; W2h [512][128] fp16 = [action_head.weight;
 * value_head.weight; 0] and b2h [512] fp16 likewise; h [m][128] fp16 = the fc1
 * output (bgx_fc1_records).  perm [m] lists the rows in ascending order of the
 * number of 32-action tiles they need (ceil(cnt / 32), 16 for cnt = 0; any order
 * is correct, sorted is fast); perm = NULL: the rows are already in that order
 * (PPOTrainer gathers them so once per update, and every kernel reads them
 * contiguously).
 * bgx_ppo_rows: per row the loss parts (added to sums[0..2] as bgx_ppo_head),
 * dh [m][128] fp16 = ReLU'(h) * fp16(dy W2h) (original row order), and the row
 * statistics stats [m] (16 B, 16-byte aligned) + info [m] (int32) in perm order
 * for bgx_ppo_gw2; dy_or_null [m][512] fp16 receives dy = [dlogits | dvalue | 0]
 * and z_or_null [m][512] fp16 the logits [y | value] of the 32-column tiles the row's
 * variant computed (other columns untouched) -- both for tests.  row_plan int32[8] = the row tiles (of perm order) [lo, hi) handled by
 * the variants for at most 1, 2, 4 and 16 leading action tiles (every row tile in
 * exactly one range; a tile's count is the largest of its rows').  grid <= 0:
 * persistent grids of 4 workgroups per CU (1 for the 16-tile variant).
 * bgx_ppo_gw2: gw2 [512][128] += dy^T h and gb2 [512] += column sums of dy (fp32),
 * dy recomputed from the statistics; plan int32[33] = task prefix per action tile
 * (17 entries; the tasks of action tile o are the groups of BGX_PPO_GW2_TASK_TILES
 * row tiles, aligned at multiples of it, that hold a row tile >= its start) then the
 * first row tile (of perm order) each action tile needs (16); workspace of
 * bgx_ppo_gw2_workspace(m) bytes. */
#define BGX_PPO_GW2_TASK_TILES 32
int bgx_ppo_rows(const void* h_dev, const int32_t* perm_dev, const uint8_t* records_dev, const int32_t* actions_dev,
                 const float* old_logp_dev, const float* returns_dev, const float* adv_dev, int32_t m, int32_t hidden,
                 int32_t n_actions, const void* w2h_dev, const void* b2h_dev, float eps_clip, float c_value,
                 float c_entropy, float grad_scale, void* dh_dev, void* stats_dev, int32_t* info_dev,
                 double* sums_dev, void* dy_or_null, void* z_or_null, const int32_t* row_plan_dev, int32_t grid,
                 void* stream);
int64_t bgx_ppo_gw2_workspace(int32_t m);
int bgx_ppo_gw2(const void* h_dev, const int32_t* perm_dev, const void* stats_dev, const int32_t* info_dev, int32_t m,
                int32_t hidden, int32_t n_actions, const void* w2h_dev, const void* b2h_dev, float k1,
                const int32_t* plan_dev, float* workspace_dev, float* gw2_dev, float* gb2_dev, void* stream);

/* The fp16 epoch's fc1 weight and bias gradients straight from the records
 * (replaces, inside ppo_agent.py:268-305 under autocast, the weight-gradient GEMM
 * dh^T x of policy_network.py:69-70 over materialised fp16 feature rows):
 * gw1 [128][208] fp32 += dh^T [x | 1 | 0], x = the 198 fp16 features of each
 * 64-byte record (off / 15 rounded as autocast rounds it), column 198 = gb1,
 * 199..207 += 0.  dh [m][128] fp16 (bgx_ppo_rows' output) and records [m][64] in
 * the same row order, both 16-byte aligned; hidden = 128; workspace of
 * bgx_ppo_gw1_workspace(m) bytes (16-byte aligned).  Deterministic (fixed-order
 * partial sums). */
int64_t bgx_ppo_gw1_workspace(int32_t m);
int bgx_ppo_gw1(const void* dh_dev, const uint8_t* records_dev, int32_t m, int32_t hidden, float* workspace_dev,
                float* gw1_dev, void* stream);

/* Discounted returns of a [T][B] rollout per game lane (the reference's
 * compute_returns, ppo_agent.py:206-216, restated per lane: R_t = r_t + gamma R_{t+1},
 * reset where done): out [T][B] fp32, the same fp32 roundings as r + gamma * R. */
int bgx_lane_returns(const float* rewards_dev, const uint8_t* dones_dev, int32_t T, int32_t B, float gamma,
                     float* out_dev, void* stream);

/* The fused fp16 PPO epoch's prologue and epilogue (bgx.train._ppo_epoch_amp_fused), one
 * launch each.  bgx_ppo_epoch_prep: from the fp32 parameters (fc1 weight [H][198] and bias,
 * action_head [A][H] and bias, value_head [1][H] and bias) the packed fc1 fragments of
 * fp16(W1) (bgx_fc1_pack's layout, bgx_fc1_packed_size(H) bytes), fp16(b1) [H], W2h =
 * fp16([action_head; value_head; 0]) [512][H], b2h [512], and zeros in the accumulators
 * gw1 [H][208], gw2 [512][H], gb2 [512] and hmax2 [1] (may be NULL), and in bound [2][512]
 * (may be NULL) each action row's |fp16(W)| and |fp16(b)|.  bgx_ppo_epoch_grads:
 * the parameters' gradients from the accumulators times post (fp32): fc1 weight = gw1[:,
 * :198], bias = gw1[:, 198], action_head = gw2[:A], gb2[:A], value_head = gw2[A], gb2[A];
 * with guard_dev (uint8, may be NULL) also guard |= 2 (max_a |W2h[a]| sqrt(hmax2[0]) +
 * max_a |b2h[a]|) > limit over a < A from prep's bound (the fused head's masked-action bound).
 * Loss parts (both may be NULL): prep zeroes sums_dev [3] (fp64, the epoch's loss sums that
 * bgx_ppo_rows adds to); grads adds (m0, m1, m2, m0 + c_value m1 - c_entropy m2), m = sums /
 * n_total, to parts_dev [4] in fp64 (the torch form's arithmetic, no contraction). */
int bgx_ppo_epoch_prep(const float* w1_dev, const float* b1_dev, const float* wa_dev, const float* ba_dev,
                       const float* wv_dev, const float* bv_dev, int32_t hidden, int32_t n_actions, void* w1pack_dev,
                       void* b1h_dev, void* w2h_dev, void* b2h_dev, float* gw1_dev, float* gw2_dev, float* gb2_dev,
                       float* hmax2_dev_or_null, float* bound_dev_or_null, double* sums_dev_or_null, void* stream);
int bgx_ppo_epoch_grads(const float* gw1_dev, const float* gw2_dev, const float* gb2_dev, int32_t hidden,
                        int32_t n_actions, float post, float* w1_grad, float* b1_grad, float* wa_grad, float* ba_grad,
                        float* wv_grad, float* bv_grad, const float* bound_dev, const float* hmax2_dev,
                        float limit, uint8_t* guard_dev_or_null, const double* sums_dev, double n_total,
                        double c_value, double c_entropy, double* parts_dev_or_null, void* stream);

/* The episode accounting of a [T][B] rollout (the reference driver's per-env loop,
 * train.py:55-99; bgx.train.episode_stats): records_dev uint8[T][B][64] (the mover is
 * byte 52), carry_dev fp64[B] = each lane's reward of its unfinished episode, updated in
 * place; out_dev fp64[6] = finished episodes, their summed rewards, wins, PLAYER1 wins,
 * gammon wins, backgammon wins.  workspace of bgx_episode_stats_workspace(B) bytes. */
int64_t bgx_episode_stats_workspace(int32_t B);
int bgx_episode_stats(const float* rewards_dev, const uint8_t* dones_dev, const uint8_t* records_dev,
                      double* carry_dev, int32_t T, int32_t B, double* workspace_dev, double* out_dev, void* stream);

/* The PPO update's rollout rows in a given order, once per update (the fused head's
 * row plan, bgx.train.ppo_row_plan; the reference batches memory rows in order,
 * ppo_agent.py:235-266): row i of each output = row perm[i] of its input, for the
 * 64-byte records and the four per-row fields (action, old log-prob, return,
 * advantage).  One kernel (16-byte copies of the records). */
/* The PPO optimizer step: torch.optim.Adam(fused=True) (ADAM_MODE::ORIGINAL; no weight
 * decay, amsgrad or maximize) as GradScaler.step + GradScaler.update drive it
 * (ppo_agent.py:302-305 `scaler.step(self.optimizer); scaler.update()`), for up to 8
 * fp32 tensors: params/grads/exp_avg/exp_avg_sq device pointers, steps = each tensor's
 * fp32 step counter (device scalar), numels element counts (host arrays of n).  With
 * scale (GradScaler._scale, fp32) non-null: a non-finite scaled gradient anywhere skips
 * the step (no parameter, moment or counter changes) and backs the scale off; else the
 * gradients are unscaled in place and the step is taken; growth_tracker (int32) and the
 * scale follow _amp_update_scale_.  scale = NULL: a plain Adam step.  found: an int32
 * device flag, zero before the first call (each call leaves it zero). */
int bgx_adam_step(int32_t n, float* const* params, float* const* grads, float* const* exp_avg,
                  float* const* exp_avg_sq, float* const* steps, const int64_t* numels, double lr, double beta1,
                  double beta2, double eps, float* scale, int32_t* growth_tracker, float growth_factor,
                  float backoff_factor, int32_t growth_interval, int32_t* found, void* stream);
/* The fused head's row plan for m rollout rows (replaces torch's argsort + bincount +
 * cumsum in bgx/train.py ppo_row_plan, which are its CPU / reference form): a row's class
 * is ceil(lim / 32) with lim = n_actions when its legal count (record bytes 60-61) is 0,
 * else min(count, n_actions); perm_dev int32[m] = the rows ordered by class, stably (the
 * order k_ppo_rows / k_ppo_gw2 read them in); plan_dev int32[33] = the k_ppo_gw2 task
 * prefix per action tile (17) then the first row tile reaching each action tile (16);
 * row_plan_dev int32[8] = the row-tile ranges of the bgx_ppo_rows variants.  Device
 * only, no host sync; workspace_dev: bgx_ppo_plan_workspace(m) bytes. */
int64_t bgx_ppo_plan_workspace(int32_t m);
int bgx_ppo_plan(const uint8_t* records_dev, int32_t m, int32_t n_actions, int32_t* workspace_dev, int32_t* perm_dev,
                 int32_t* plan_dev, int32_t* row_plan_dev, void* stream);
int bgx_gather_rollout(const int32_t* perm_dev, int32_t n, const uint8_t* records_dev, const int32_t* actions_dev,
                       const float* old_logp_dev, const float* returns_dev, const float* adv_dev,
                       uint8_t* records_out, int32_t* actions_out, float* old_logp_out, float* returns_out,
                       float* adv_out, void* stream);
/* bgx_ppo_plan and bgx_gather_rollout in one pass (round 6): the plan, and each row's
 * record and four fields written straight to its plan-order position (the scatter reads
 * the records once, coalesced; no perm pass, no random-read gather).  perm_or_null: the
 * permutation too (tests).  Same workspace; records and records_out 16-byte aligned. */
int bgx_ppo_plan_rows(const uint8_t* records_dev, int32_t m, int32_t n_actions, int32_t* workspace_dev,
                      const int32_t* actions_dev, const float* old_logp_dev, const float* returns_dev,
                      const float* adv_dev, uint8_t* records_out, int32_t* actions_out, float* old_logp_out,
                      float* returns_out, float* adv_out, int32_t* perm_or_null, int32_t* plan_dev,
                      int32_t* row_plan_dev, void* stream);

/* Phase times of the last bgx_two_ply call on e (first round, HIP events on the
 * caller's stream): ms2[0] = reply enumeration (all tiers), ms2[1] = leaf
 * evaluation after it (k_eval, the MFMA kernel). */
int bgx_two_ply_timings(bgx_engine* e, float* ms2);

/* Debug options (tests and diagnostics only; the product path never reads the
 * environment).  Sets option `name` to `value` (NULL: unset) for the process.  Names:
 * BGX_2PLY_HEAVY "log:memo" (9:0 / 10:0: the doubles enumerator without the memo / with
 * a 1,024-slot table), BGX_2PLY_LDS_CAP "first[:mid]" (forced overflow tiers),
 * BGX_2PLY_POOL n (leaf-pool slots: retry rounds), BGX_2PLY_UNFACTORED (the 13-k-block
 * evaluator), BGX_2PLY_BARROW 0 (bar rows per job), BGX_2PLY_DUMP path (pool, row sides,
 * V per slot), BGX_2PLY_DEBUG (round sizes on stderr), BGX_POLICY_SKIP 0 (no tile skip),
 * BGX_POLICY_HEAVY n (the policy's heavy-row bound); read at engine creation: BGX_XCD 0,
 * BGX_ORDER 0 (lane-order dispatch), BGX_STAMPS, BGX_STEP_DEBUG.  Every alternative is
 * exact: results are identical, only the schedule or the diagnostics change. */
int bgx_debug_option(const char* name, const char* value_or_null);

/* Last HIP error string of this thread (diagnostics). */
const char* bgx_last_error(void);

/* Build provenance: sha256 (hex) of the sources and compile flags this library
 * was built from (bgx._lib.source_hash); smoke() and the tests compare it with
 * the tree they run from. */
const char* bgx_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* BGX_H */
