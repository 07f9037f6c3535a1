/* mzgo.h -- C ABI of the MI355X-native MuZero-Go self-play engine (libmzgo.so).
 *
 * The reference (Sir-Teo/MuZero-Go) is pure Python with no FFI; its hot path
 * is reached through duck-typed protocols.  Each entry point below replaces
 * one of them (citations are into the reference snapshot):
 *
 *   mzgo_initial_inference    MuZeroNet.initial_inference      self_play.py:121-124
 *   mzgo_recurrent_inference  MuZeroNet.recurrent_inference    self_play.py:125-128
 *   mzgo_set_weights          MuZeroNet.load_state_dict /       self_play.py:404-412
 *                             MuZeroAgent.load_weights
 *   mzgo_search               MCTS.run                         self_play.py:148-237
 *   mzgo_board_reset          GoEnv.reset (GymGo)              self_play.py:455
 *   mzgo_board_step           GoEnv.step  (GymGo)              self_play.py:479
 *   mzgo_board_planes         the observation array GoEnv returns
 *   mzgo_selfplay_move        one iteration of run_self_play_game's loop,
 *                             for every game slot              self_play.py:465-507
 *   mzgo_records_export       GameHistory / the pickle writer  self_play.py:415-450, :561-583
 *
 * Conventions
 *   - All tensor arguments are DEVICE pointers (hipMalloc / torch CUDA tensors)
 *     unless the name ends in _host.  Shapes are C-contiguous.
 *   - ``stream`` is a hipStream_t (NULL = the null stream).  Calls enqueue work
 *     and return; nothing synchronises unless documented.
 *   - Return value: 0 on success, a negative MZGO_E* code on failure;
 *     mzgo_last_error() then describes it (thread-local).
 *   - An engine is not thread-safe.
 *   - Actions are row-major cells a = r*N + c, pass = N*N (GymGo's flattening).
 *   - Observation planes are [6][N][N]: BLACK, WHITE, TURN, INVD, PASS, DONE.
 */
#ifndef MZGO_H
#define MZGO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  MZGO_OK = 0,
  MZGO_EINVAL = -1,      /* bad argument / unsupported configuration */
  MZGO_EHIP = -2,        /* HIP runtime error */
  MZGO_ENOWEIGHTS = -3,  /* network weights incomplete */
  MZGO_EASSERT = -4      /* GymGo assertion (invalid move, step after done) */
};

typedef struct mzgo_config {
  int board_size;           /* N: 5, 6, 9 or 19 (self_play.py:20) */
  int latent_dim;           /* C: 96 (self_play.py:21); 0 = board-only engine */
  int num_games;            /* G: game slots held on the device */
  int num_simulations;      /* S: MCTS simulations per move (self_play.py:23) */
  int max_moves;            /* move cap, N*N in the reference (self_play.py:461); 0 = N*N */
  int compat;               /* 0 = reference (zero visit counts, §0.6), 1 = fixed */
  int temperature_moves;    /* 15 (self_play.py:29) */
  int search_variant;       /* 0 = self_play.py's MCTS (:142-343), 1 = main.py's MCTS
                               (main.py:246-368: trainer self-play and arena rules) */
  double c_puct;            /* 2.5 (self_play.py:143); main.py's variant uses 2 */
  double discount;          /* 0.99 */
  double dirichlet_alpha;   /* 0.15 */
  double dirichlet_epsilon; /* 0.02 */
  double pass_epsilon;      /* 0.01 */
  double temperature;       /* 1.0 */
  double komi;              /* 0 (self_play.py:544) */
  uint64_t seed;            /* counter-RNG seed */
  int game_base;            /* global id of slot 0 (multi-GPU game sharding) */
  int device;               /* HIP device ordinal */
  int direct_dynamics;      /* 0 = factored expansion (default): a search convolves each
                               parent once and expands children as relu(Y + E[a]), exact
                               up to fp32 rounding (see muzero-go_amd/csrc/mzgo_expand.hpp);
                               1 = one dynamics conv per simulation, as the reference does */
  int tower;                /* 0 = the reference network (self_play.py:63-128); 1 = the
                               residual-tower network of BASELINE config 5 (mzgo/resnet.py:
                               conv_in + res_blocks residual blocks in the representation and
                               the dynamics, the reference's heads), bf16 MFMA with fp32
                               accumulation, latent_dim a multiple of 64, N in {5, 9, 19} */
  int res_blocks;           /* residual blocks per tower network (tower = 1) */
} mzgo_config;

typedef struct mzgo_engine mzgo_engine;

/* Fill *cfg with the reference defaults (self_play.py:19-33) for board size N. */
void mzgo_default_config(mzgo_config* cfg, int board_size);

int mzgo_engine_create(const mzgo_config* cfg, mzgo_engine** out);
void mzgo_engine_destroy(mzgo_engine* eng);
const char* mzgo_last_error(void);
/* Bytes of device memory the engine owns. */
int64_t mzgo_engine_device_bytes(const mzgo_engine* eng);

/* Load one state_dict tensor (host float32, reference key and shape, e.g.
 * "dynamics.conv.weight" (C,C,3,3)); packed into MFMA fragment order on upload.
 * mzgo_weights_ready() returns 1 once all 22 keys are loaded. */
int mzgo_set_weights(mzgo_engine* eng, const char* key, const float* data_host,
                     const int64_t* shape, int ndim);
int mzgo_weights_ready(const mzgo_engine* eng);

/* MuZeroNet protocol, batch B (any B >= 1):
 *   obs f32 [B][6][N][N] -> latent f32 [B][C][N][N], value f32 [B][1], logits f32 [B][N*N+1]  */
int mzgo_initial_inference(mzgo_engine* eng, const float* obs, int B, float* latent,
                           float* value, float* logits, void* stream);
/*   latent f32 [B][C][N][N], action i64 [B] -> next_latent, reward [B][1], value [B][1], logits */
int mzgo_recurrent_inference(mzgo_engine* eng, const float* latent, const int64_t* action, int B,
                             float* next_latent, float* reward, float* value, float* logits,
                             void* stream);
/* Synchronises ``stream`` and reports (then clears) an out-of-range action seen
 * by mzgo_recurrent_inference (nn.Embedding's IndexError). */
int mzgo_check_inference_errors(mzgo_engine* eng, void* stream);

/* MCTS.run for the first G slots: root_obs f32 [G][6][N][N]; noise f64 [G][A]
 * injected Dirichlet samples or NULL (sampled from the counter RNG keyed by
 * (seed, game_base + g, move_index)).  Outputs: root_child_visits i32 [G][A]
 * (the true child visit counts) and root_value f64 [G] (may be NULL).  The
 * tree stays on the device for mzgo_tree_export. */
int mzgo_search(mzgo_engine* eng, const float* root_obs, const double* noise, int G, int move_index,
                int32_t* root_child_visits, double* root_value, void* stream);
/* Copy slot g's last search tree to host buffers (synchronises ``stream``):
 * n_nodes; child i32 [n][A]; visits i32 [n]; value_sum f64 [n]; prior f32 [n][A]
 * (row 0 unused); root_prior f64 [A].  Buffers must hold S+1 nodes; NULL skips.
 * After mzgo_search every row is final.  After mzgo_selfplay_move on the
 * reference network (tower = 0), a node that no select reached has NO formed
 * rows: a batched child's policy head is lazy (never computed), so its prior
 * row holds whatever an earlier search left there and its child row either
 * the same stale ids (boards whose tree lives in LDS, 5x5-9x9: the node is
 * marked in the kernel's LDS bitmask) or the sentinel -3 in entry 0 (HBM
 * trees, 19x19); the rows are formed when a select first reaches the node
 * (it has no children before), and the move never reads the others.  Tower
 * engines settle such rows here first (the search API's settle kernel), so
 * their exports are complete. */
int mzgo_tree_export(mzgo_engine* eng, int g, int32_t* n_nodes_host, int32_t* child_host,
                     int32_t* visits_host, double* value_sum_host, float* prior_host,
                     double* root_prior_host, void* stream);

/* GoEnv protocol on the G slots.  board_step: actions i32 [G] (-1 = leave the
 * slot alone); status i32 [G] gets 0 ok, 1 step after done, 2 invalid move,
 * 3 action out of range; winner f64 [G] gets GoEnv.winner() after the step.
 * status/winner may be NULL. */
int mzgo_board_reset(mzgo_engine* eng, void* stream);
int mzgo_board_step(mzgo_engine* eng, const int32_t* actions, int32_t* status, double* winner,
                    void* stream);
/* planes f64 [G][6][N][N] */
int mzgo_board_planes(mzgo_engine* eng, double* planes, void* stream);
/* Overwrite slot g's board (host data): stones i8 [N*N] (0/1 black/2 white),
 * invd u8 [N*N], meta i32 [4] (turn, passed, done, moves). */
int mzgo_board_set(mzgo_engine* eng, int g, const int8_t* stones_host, const uint8_t* invd_host,
                   const int32_t* meta_host, void* stream);

/* Self-play.  selfplay_reset starts a new game in every slot (epoch = RNG
 * generation of the games); selfplay_move plays one move in every unfinished
 * slot.  selfplay_counters (host u64 [8], synchronises; cumulative over the
 * engine's life): [0] simulations run, [1] moves played, [2] games finished,
 * [3] slots still playing now, [4] dynamics 3x3 convs run by searches (one per
 * expansion with direct_dynamics, one per new parent node when factored;
 * tower engines: dynamics towers evaluated, speculative batch entries that
 * were never used included),
 * [5] of those, parent convs shared with the workgroups of games that had
 * already ended (9x9 whole-game launches: the epoch tail), [6] prior rows
 * formed by searches (a node's child priors + child row written to HBM: every
 * eagerly expanded child, and a lazily expanded one -- the lazy policy head --
 * only when a select first reaches it; 0 on tower engines), [7] self-play
 * game workgroups started (every slot's workgroup of every launch counts one
 * when it begins: mzgo_stream_wait_started's count), [8] epoch-tail helper
 * workgroups whose bounded wait for a job expired (they stop helping; records
 * are unaffected).  counters_host must hold 9 values.  An expired
 * mzgo_stream_wait_started gate is reported here (MZGO_EHIP, once). */
int mzgo_selfplay_reset(mzgo_engine* eng, int epoch, void* stream);
int mzgo_selfplay_move(mzgo_engine* eng, void* stream);
/* Up to ``moves`` consecutive moves of every unfinished slot in ONE launch
 * (each slot stops at its game's end); the records and RNG streams are those
 * of ``moves`` mzgo_selfplay_move calls.  moves = max_moves plays whole games.
 * Tower engines (tower = 1) run a move as a sequence of launches; for
 * moves > 4 they read the slots' status every 4 moves (BLOCKING: the stream is
 * synchronised there, so such a call cannot be captured in a HIP graph) and
 * stop enqueueing once every game has ended -- the same records and counters
 * as ``moves`` single-move calls -- and synchronise once at the end of every
 * call, which reports an expired k_tconv_chain wait (MZGO_EHIP). */
int mzgo_selfplay_moves(mzgo_engine* eng, int moves, void* stream);

/* Arena (main.py:526-611, SelfPlayEvaluator): like mzgo_selfplay_move, but
 * game i (global id) is played between two networks -- eng's ("current",
 * turn 0) and opponent's ("best", turn 1); game i's first mover is turn
 * i % 2 and turns alternate.  Search, move rule and records are eng's
 * (use search_variant 1 for main.py's rules); opponent only lends its
 * weights (same board_size and latent_dim).  Replaces the evaluator's
 * MCTS(current/best net).run + argmax loop (main.py:548-568). */
int mzgo_arena_move(mzgo_engine* eng, mzgo_engine* opponent, void* stream);
/* ``moves`` arena moves per slot in one launch (as mzgo_selfplay_moves). */
int mzgo_arena_moves(mzgo_engine* eng, mzgo_engine* opponent, int moves, void* stream);
int mzgo_selfplay_counters(mzgo_engine* eng, uint64_t* counters_host, void* stream);

/* Move-parallel epoch (no reference counterpart; the schedule, not the
 * protocol): a multi-move mzgo_selfplay_moves under compat "reference"
 * (self_play.py's search) runs as two launches -- k_selfplay_boards, every
 * game's moves without their searches (observation, legal mask, action,
 * policy target, board step, reward: under compat "reference" the action
 * never reads the search), then k_search_queue, which runs every recorded
 * move's search (root value) from one work queue on one workgroup per CU.
 * The records are byte-identical to the game-per-workgroup launch
 * (MZGO_MOVE_PARALLEL=0 in the environment keeps that launch); the trees
 * left in the slots are then those of whatever searches ran last in each
 * queue slot, not one per game.  19x19 engines created under compat
 * "reference" hold a tree slot per CU for it (MZGO_MOVE_PARALLEL=0 at
 * creation: G slots).
 * mzgo_selfplay_set_timing(eng, 1) records HIP events around both launches
 * of every such call (0 stops and discards); mzgo_selfplay_launch_times
 * synchronises on them, writes up to ``cap`` (boards, queue) durations in
 * ms, stores the number recorded in *n_host and clears them. */
int mzgo_selfplay_set_timing(mzgo_engine* eng, int on);
int mzgo_selfplay_launch_times(mzgo_engine* eng, float* boards_ms, float* queue_ms, int cap, int* n_host);
/* DIAGNOSTIC (scripts/rccl_standin.py; not part of the self-play protocol, and
 * bench.py does not call it: it gathers every timed epoch's records in ONE
 * collective after the timed loop).  Enqueue on ``stream`` a gate that
 * completes once counter [7] (self-play workgroups started) reaches
 * ``target``: work queued behind it -- a collective -- cannot take a CU before
 * every workgroup of the self-play launch that brings the count to target is
 * resident (a self-play workgroup fills a CU's LDS).  The gate itself is one
 * wave without LDS, so it sits beside them; its wait is bounded (~seconds)
 * and an expiry is reported by the next mzgo_selfplay_counters call.  Tower
 * engines: MZGO_EINVAL (they never count started workgroups). */
int mzgo_stream_wait_started(mzgo_engine* eng, uint64_t target, void* stream);
/* Tower engines (tower = 1): report (synchronising) and reset the time spent
 * in the dynamics towers since the last call -- one HIP event pair around each
 * simulation step's 2*res_blocks+1 conv launches, on the launch stream -- then
 * switch the timing on (enable = 1) or off. */
int mzgo_tower_timing(mzgo_engine* eng, int enable, double* tower_ms_host, int64_t* towers_host);

/* Trainer backward of the dynamics conv (main.py:478-482's loss.backward()
 * through DynamicsNetwork.forward, main.py:97-103; replaces
 * torch.nn.grad.conv2d_input / conv2d_weight in the trainer's HIP autograd
 * Function).  Forward: out = relu(conv3x3(latent + emb[action]) + bias),
 * padding 1.  In: grad_out, out, latent [B][C][N][N] f32, action [B] i64,
 * emb [A][C], weight [C][C][3][3].  Out: grad_latent [B][C][N][N] (= the
 * conv input's gradient), grad_weight [C][C][3][3], grad_bias [C]; fp32 MFMA,
 * deterministic.  C a multiple of 16, 2 <= N <= 19; workspace of at least
 * mzgo_dyn_conv_backward_workspace(B, C) bytes (device). */
int mzgo_dyn_conv_backward_workspace(int B, int C, int64_t* bytes_host);
int mzgo_dyn_conv_backward(const float* grad_out, const float* out, const float* latent, const int64_t* action,
                           const float* emb, const float* weight, int B, int C, int N, float* grad_latent,
                           float* grad_weight, float* grad_bias, void* workspace, int64_t workspace_bytes,
                           void* stream);
/* Trainer: one 3x3 conv layer y = relu(conv3x3(x') + bias), padding 1, on
 * fp32 MFMA (main.py:72-84 RepresentationNetwork's conv1-3, main.py:97-103
 * DynamicsNetwork's conv), x' = x [B][Cin][N][N], or x + emb[action[b]]
 * broadcast over the board when emb ([A][Cin]) is given (the dynamics input).
 * Forward: the activation recomputation of the representation's hidden
 * layers (the engine's k_initial_inference keeps them on chip).  Backward:
 * from the saved output (ReLU mask y > 0) and input, grad_x [B][Cin][N][N]
 * (may be NULL: the first layer), grad_weight [Cout][Cin][3][3], grad_bias
 * [Cout]; deterministic (fixed summation order).  Replaces
 * torch.nn.grad.conv2d_input / conv2d_weight in the trainer's autograd
 * Functions.  Any Cin, Cout >= 1; 2 <= N <= 19; device workspace of at least
 * mzgo_conv3x3_backward_workspace(B, Cin, Cout) bytes. */
int mzgo_conv3x3_relu_forward(const float* x, const int64_t* action, const float* emb, const float* weight,
                              const float* bias, int B, int Cin, int Cout, int N, float* out, void* stream);
int mzgo_conv3x3_backward_workspace(int B, int Cin, int Cout, int64_t* bytes_host);
int mzgo_conv3x3_backward(const float* grad_out, const float* out, const float* x, const int64_t* action,
                          const float* emb, const float* weight, int B, int Cin, int Cout, int N, float* grad_x,
                          float* grad_weight, float* grad_bias, void* workspace, int64_t workspace_bytes,
                          void* stream);
/* Test hook: use injected Dirichlet samples f64 [G][max_moves][A] (device,
 * caller-owned, must outlive the moves) instead of the counter-RNG sampler;
 * NULL restores sampling. */
int mzgo_selfplay_inject_noise(mzgo_engine* eng, const double* noise);
/* Test hook (parity of the sampled-noise path): every self-play root's
 * normalised Dirichlet sample -- the one the counter-RNG sampler drew, or the
 * injected one -- written to dst f64 [G][max_moves][A] (device, caller-owned,
 * must outlive the moves) at (slot, move); NULL turns it off. */
int mzgo_selfplay_record_noise(mzgo_engine* eng, double* dst);
/* Test hook, tower engines (tower = 1): every node the searches evaluate,
 * written to dst f32 [G][S+1][A+2] (device, caller-owned) at (slot, node id)
 * as the tower produced it: the policy logits [A], then reward and value
 * (node 0: the representation's logits and value, reward 0).  With it a
 * CPU search driven by these outputs must rebuild the device tree exactly.
 * NULL turns it off. */
int mzgo_tower_record_nodes(mzgo_engine* eng, float* dst);

/* Copy slot g's game record to host buffers (synchronises ``stream``).
 * length: moves recorded; ended: 1 if the game ended by double pass; status.
 * stones i8 [M][N*N], invd u8 [M][N*N], flags u8 [M] (bit0 turn, bit1 passed,
 * bit2 done), action i32 [M], value f64 [M], policy f64 [M][A], reward f64 [M],
 * final_reward f64.  M = length; NULL pointers are skipped. */
int mzgo_records_export(mzgo_engine* eng, int g, int32_t* length_host, int32_t* status_host,
                        int8_t* stones_host, uint8_t* invd_host, uint8_t* flags_host,
                        int32_t* action_host, double* value_host, double* policy_host,
                        double* reward_host, double* final_reward_host, void* stream);

/* All slots' records packed into one DEVICE buffer (the multi-GPU trajectory
 * gather moves it with RCCL).  dst NULL: only report *bytes_needed.  Layout,
 * each field padded to 16 bytes, G slots, M = max_moves, C = N*N, A = C+1:
 *   stones i8 [G][M][C] | invd u8 [G][M][C] | flags u8 [G][M] | action i32 [G][M] |
 *   value f64 [G][M] | policy f64 [G][M][A] | reward f64 [G][M] |
 *   meta i32 [G][4] (turn, passed, done, length) | status i32 [G] | final_reward f64 [G] */
int mzgo_records_pack(mzgo_engine* eng, uint8_t* dst, int64_t capacity, int64_t* bytes_needed,
                      void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MZGO_H */
