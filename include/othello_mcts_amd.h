/*
 * othello_mcts_amd.h — C ABI of the MI355X-native othello_mcts engine.
 *
 * Plain pointers and sizes only (no torch / pybind types). Every entry point
 * names the reference interface it replaces (yunhao-qian/Othello-AlphaZero,
 * paths relative to cpp/src/). The Python package othello_mcts
 * (othello-alphazero_amd/othello_mcts) is a pybind11 layer over exactly these
 * functions; INTEGRATION.md shows the binding a maintainer of the reference
 * would add.
 *
 * Conventions
 *   - Return value: OAMD_OK (0) or an oamd_status; oamd_last_error() holds the
 *     message (thread-local). The pybind layer maps OAMD_INVALID_ARGUMENT to
 *     ValueError and OAMD_OUT_OF_RANGE to IndexError, like the reference's
 *     std::invalid_argument / std::out_of_range (othello_mcts.cpp, pybind11).
 *   - "dev" pointers are HIP device pointers on the engine's / net's device;
 *     "host" pointers are ordinary host memory.
 *   - `stream` is a hipStream_t (NULL = the legacy default stream).
 *   - Bit order: square i = row*8 + col, bitboard bit (63 - i) (position.h:275).
 *   - Actions: 0..63 squares, 64 = pass (position.h:402-408).
 */
#ifndef OTHELLO_MCTS_AMD_H
#define OTHELLO_MCTS_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OAMD_ABI_VERSION 1

typedef enum oamd_status {
    OAMD_OK = 0,
    OAMD_INVALID_ARGUMENT = 1, /* std::invalid_argument -> ValueError */
    OAMD_OUT_OF_RANGE = 2,     /* std::out_of_range     -> IndexError */
    OAMD_RUNTIME = 3,          /* HIP / device failure  -> RuntimeError */
    OAMD_CAPACITY = 4          /* node pool exhausted   -> RuntimeError */
} oamd_status;

const char *oamd_last_error(void);
int oamd_abi_version(void);
/* Hash of the sources the library was built from (16 hex digits; family
 * "resnet", "tree" or "all", else NULL): build.py compiles them in, and
 * othello_mcts.provenance compares them with the sources on disk. */
const char *oamd_source_hash(const char *family);
/* number of visible HIP devices (0 when no GPU) */
int oamd_device_count(int32_t *out);

/* ------------------------------------------------------------------------ */
/* Batched bitboards (device, bit-exact with position.h)                     */
/* ------------------------------------------------------------------------ */

/* Same memory layout as the engine's Position value type (40 bytes). */
typedef struct oamd_position {
    int32_t player; /* 1 black, 2 white, 0 terminal  (position.h:47) */
    int32_t reserved;
    uint64_t player1_discs;    /* position.h:53 */
    uint64_t player2_discs;    /* position.h:59 */
    uint64_t legal_moves;      /* position.h:74 */
    uint64_t next_legal_moves; /* position.h:148 (private in the reference) */
} oamd_position;

/* replaces othello::get_legal_moves (position.h:202-229), n boards */
int oamd_get_legal_moves(const uint64_t *player_discs_dev, const uint64_t *opponent_discs_dev,
                         uint64_t *out_dev, int64_t n, void *stream);
/* replaces othello::get_flips (position.h:231-262), n boards */
int oamd_get_flips(const uint64_t *move_mask_dev, const uint64_t *player_discs_dev,
                   const uint64_t *opponent_discs_dev, uint64_t *out_dev, int64_t n, void *stream);
/* replaces Position::apply_action (position.h:402-408, unchecked), n positions */
int oamd_apply_action(const oamd_position *in_dev, const int32_t *actions_dev,
                      oamd_position *out_dev, int64_t n, void *stream);
/* replaces Position::initial_position (position.h:264-272) */
int oamd_initial_position(oamd_position *out_host);

/* Scalar host forms of the same functions (the Python Position API and
 * get_legal_moves / get_flips, used by player.py:45-160). Same source as the
 * device kernels (csrc/bitboard.h, __host__ __device__). */
uint64_t oamd_host_legal_moves(uint64_t player_discs, uint64_t opponent_discs);
uint64_t oamd_host_flips(uint64_t move_mask, uint64_t player_discs, uint64_t opponent_discs);
void oamd_host_apply_action(const oamd_position *in_host, int32_t action, oamd_position *out_host);

/* ------------------------------------------------------------------------ */
/* Native network: replaces the Python NeuralNet callback                   */
/* (neural_net.h:15-29, othello_mcts.cpp:19-45) for AlphaZeroNet             */
/* (python/othello_alphazero/neural_net.py:138-172) in eval mode.            */
/* ------------------------------------------------------------------------ */

typedef enum oamd_dtype { OAMD_BF16 = 0, OAMD_FP16 = 1 } oamd_dtype;

typedef struct oamd_net_desc {
    int32_t in_channels;                /* 1 + 2 * history_size, <= 31 */
    int32_t conv_channels;              /* 128 or 256 */
    int32_t num_residual_blocks;        /* >= 0 */
    int32_t value_head_hidden_channels; /* >= 1 */
    int32_t num_squares;                /* must be 64 */
    int32_t num_actions;                /* must be 65 */
    int32_t dtype;                      /* oamd_dtype */
} oamd_net_desc;

typedef struct oamd_net oamd_net;

int oamd_net_create(int32_t device, const oamd_net_desc *desc, oamd_net **out);
int oamd_net_destroy(oamd_net *net);
/* Number of tensors oamd_net_load_state expects (= AlphaZeroNet.state_dict()
 * entries without num_batches_tracked), and the i-th key / element count. */
int oamd_net_state_size(const oamd_net *net, int32_t *n_tensors);
int oamd_net_state_key(const oamd_net *net, int32_t i, const char **key, int64_t *numel);
/* Host fp32 tensors in oamd_net_state_key order. BatchNorm (eval, eps 1e-5)
 * is folded into the preceding convolution; weights are packed into the
 * MFMA fragment layout and converted to the net's dtype. */
int oamd_net_load_state(oamd_net *net, const float *const *tensors_host, int32_t n_tensors);
/* features_dev: (rows, in_channels, 8, 8) fp32; policy_dev (rows, 65)
 * probabilities; value_dev (rows,) in [-1, 1]. */
int oamd_net_forward(oamd_net *net, const float *features_dev, int32_t rows, float *policy_dev,
                     float *value_dev, void *stream);

/* ------------------------------------------------------------------------ */
/* Search engine: G independent games, one tree per game in HBM.             */
/* Replaces othello::MCTS (mcts.h:35-216, mcts.cpp) and SearchThread         */
/* (search_thread.cpp); G = 1 is the reference's single-game object.         */
/* ------------------------------------------------------------------------ */

/* MCTS(...) constructor arguments (othello_mcts.cpp:89-112, keyword names
 * authoritative). torch_device / torch_pin_memory live in the Python layer. */
typedef struct oamd_search_config {
    int32_t history_size;    /* >= 1, <= 15 */
    int32_t num_simulations; /* >= 1 */
    int32_t num_threads;     /* >= 1: virtual search threads */
    int32_t batch_size;      /* >= 1: leaves per virtual thread per step */
    float c_puct_base;       /* > 0 */
    float c_puct_init;       /* >= 0 */
    float dirichlet_epsilon; /* in [0, 1] */
    float dirichlet_alpha;   /* >= 0 */
} oamd_search_config;

typedef struct oamd_engine oamd_engine;

/* node_capacity: nodes per game (0 = default 1<<20). Nodes are never freed
 * while a game lasts (history ancestors stay valid, mcts.cpp:140-165);
 * oamd_engine_reset recycles a game's pool. */
int oamd_engine_create(int32_t device, int32_t num_games, int64_t node_capacity,
                       const oamd_search_config *config, uint64_t seed, oamd_engine **out);
int oamd_engine_destroy(oamd_engine *e);
/* mcts.cpp:167-241 setters (validated; OAMD_INVALID_ARGUMENT with the
 * reference's messages) */
int oamd_engine_set_config(oamd_engine *e, const oamd_search_config *config);
int oamd_engine_get_config(const oamd_engine *e, oamd_search_config *config);
int oamd_engine_num_games(const oamd_engine *e, int32_t *out);
int oamd_engine_set_stream(oamd_engine *e, void *stream);
/* game = -1: all games. Resets to the initial position (mcts.cpp:40-43) and
 * reseeds the game's random stream with (seed, game). */
int oamd_engine_reset(oamd_engine *e, int32_t game, uint64_t seed);

/* Whole search for every active game with the native net
 * (MCTS::search, mcts.h:220-256). Outputs are optional (may be NULL):
 * simulations = leaf selections (sum over games), evaluations = NN rows of
 * non-terminal leaves. With both NULL the call returns once the search is
 * enqueued (stream order; the host does not wait), otherwise after it ends.
 * One game with num_threads > 1 runs thread by thread, each thread's ResNet
 * rows on a stream of their own while the next thread's tree work runs
 * (same results; OAMD_TREE_SPLIT=0 in the environment turns it off). */
int oamd_engine_search(oamd_engine *e, oamd_net *net, int64_t *simulations, int64_t *evaluations);
/* Work done since the engine was created (host outputs; waits for the
 * engine's stream): simulations (leaf selections) and evaluations (NN rows of
 * non-terminal leaves, BASELINE.md's n_eval) over every search, native or
 * step-wise. The reference counts neither; it builds no NN row for a terminal
 * leaf (search_thread.cpp:88-90). */
int oamd_engine_work_counters(oamd_engine *e, int64_t *simulations, int64_t *evaluations);
/* Tree shape since the engine was created (host outputs; waits for the
 * engine's stream): leaves selected (= simulations), the sum of their descent
 * depths (levels below the root, search_thread.cpp:64-67) and the deepest
 * descent. mean depth = depth_sum / leaves. */
int oamd_engine_descent_depths(oamd_engine *e, int64_t *leaves, int64_t *depth_sum, int32_t *depth_max);
/* Rows per ResNet launch in oamd_engine_search (0 = a whole pipeline group per
 * launch): a group's rows are evaluated by consecutive launches of at most
 * `rows` rows on its stream (the NN evaluation batch; configs[4] uses 2048).
 * Results do not depend on it. */
int oamd_engine_set_nn_batch(oamd_engine *e, int32_t rows);
/* Counts since the engine was created: grouped native searches enqueued (all
 * pipeline groups of one search count once), their NN rounds (steps + extra
 * rounds each), and the final backup-only k_tree launches of the timed
 * searches (the launches behind oamd_engine_tree_timing's backup_ms). */
int oamd_engine_round_counts(const oamd_engine *e, int64_t *searches, int64_t *rounds,
                             int64_t *final_launches);
/* enable = 1 (default): the reference's thread interleaving exactly — a
 * virtual thread whose batch is all terminal backs it up without an NN round
 * trip and selects again at once (search_thread.cpp:102-127), in the same
 * round. enable = 0: such a batch waits for its thread's next round like any
 * other (the round-robin of round 2): identical results until a batch is all
 * terminal (endgames), and no round longer than one batch per thread, so the
 * search rounds stay hidden behind the other pipeline group's ResNet launch
 * in sustained self-play. */
int oamd_engine_set_exact_interleaving(oamd_engine *e, int32_t enable);

/* Step-wise search for an external evaluator (the Python NeuralNet callback
 * path, othello_mcts.cpp:36-45). Rows: row = game * L + leaf, L =
 * num_threads * batch_size; virtual thread k of a game owns leaves
 * [k*batch_size, (k+1)*batch_size) (search_thread.cpp:59-128).
 *   begin -> steps;  repeat steps times: select, [features, evaluate,
 *   set_evaluation];  then backup once.
 * select backs up the previous round's batch of each thread right before that
 * thread selects its next batch: the interleaving the reference's threads
 * produce (search_thread.cpp:47-128 with mcts.h:242-251's FIFO NN service).
 * Calling backup after every select gives the lock-step order instead. */
int oamd_engine_search_begin(oamd_engine *e, int32_t *steps);
int oamd_engine_select(oamd_engine *e);
/* host_out[row] = 1 when the row needs the NN this round: a non-terminal leaf
 * of a batch that waits for its evaluation (a virtual thread whose batch was
 * all terminal backed it up without one and selected again,
 * search_thread.cpp:102-127; a thread that ran out of batches has none) */
int oamd_engine_leaf_flags(oamd_engine *e, uint8_t *host_out);
/* features_dev: (rows, 1 + 2H, 8, 8) fp32 of rows [row_begin, row_begin+rows) */
int oamd_engine_features(oamd_engine *e, float *features_dev, int32_t row_begin, int32_t rows);
int oamd_engine_set_evaluation(oamd_engine *e, const float *policy_dev, const float *value_dev,
                               int32_t row_begin, int32_t rows);
int oamd_engine_backup(oamd_engine *e);

/* Root queries (mcts.cpp:45-61, mcts.h:69-71). visits/q are in
 * legal_actions() order, arrays of >= 65 entries. */
typedef struct oamd_root_info {
    oamd_position position;
    int32_t num_children; /* 0 while the root is unexpanded */
    int32_t visit_count;  /* root N (includes virtual-loss increments) */
    int32_t overflow;     /* node pool exhausted during a search */
    int32_t reserved;
    int64_t node_count;
} oamd_root_info;

int oamd_engine_root_info(oamd_engine *e, int32_t game, oamd_root_info *info_host,
                          int32_t *visits_host, float *q_host);
/* Engine health (host outputs; waits for the engine's stream): number of
 * games whose node pool was exhausted (a leaf could not be expanded: the
 * search no longer follows the reference) and of games whose descent hit the
 * path-depth cap, since each game's last reset. Callers raise on nonzero. */
int oamd_engine_status(oamd_engine *e, int32_t *overflow_games, int32_t *depth_capped_games);
/* All games at once (device buffers): visits_dev (G, 65) and q_dev (G, 65)
 * indexed BY ACTION (0 where not a child), info_dev (G) */
int oamd_engine_root_stats(oamd_engine *e, int32_t *visits_dev, float *q_dev,
                           oamd_root_info *info_dev);
/* mcts.cpp:63-112: features (8, 1+2H, 8, 8) fp32, policy (8, 65) fp32, host.
 * OAMD_INVALID_ARGUMENT if the root is terminal or unexpanded. */
int oamd_engine_self_play_data(oamd_engine *e, int32_t game, float *features_host,
                               float *policy_host);
/* mcts.cpp:114-165 for one game (validated, reference messages) */
int oamd_engine_apply_action(oamd_engine *e, int32_t game, int32_t action);
/* Batched: actions_dev (G), -1 = leave the game as is (not validated). */
int oamd_engine_apply_actions(oamd_engine *e, const int32_t *actions_dev);

/* ------------------------------------------------------------------------ */
/* On-device self-play driver (train.py:404-452 per move, all games):        */
/* choose the move from root visits (temperature sampling for the first      */
/* `temperature_moves` plies, argmax with random tie-break afterwards), emit  */
/* the 8-fold training targets of the root (optional), apply the move, and   */
/* restart finished games from a random opening of up to                     */
/* `opening_moves` uniformly random plies.                                   */
/* ------------------------------------------------------------------------ */
typedef struct oamd_selfplay_config {
    int32_t temperature_moves; /* reference: 12 */
    float temperature;         /* reference: 1.0 */
    int32_t opening_moves;     /* random plies after a restart (0 = none) */
    int32_t emit_targets;      /* 1: write features/policy of every move */
} oamd_selfplay_config;

/* Per move, per game outputs (device, may be NULL):
 *   actions_dev (G) chosen action (-1 inactive); finished_dev (G): bits 0-1 =
 *   0 game continues, 1 draw, 2 black won, 3 white won (the game ended with
 *   this move and restarted); bit 2 = the root was unexpanded, no targets were
 *   written (the move was uniform); bit 3 = the game's node pool overflowed;
 *   features_dev (G, 8, 1+2H, 8, 8) and policy_dev (G, 8, 65) targets. */
int oamd_engine_selfplay_move(oamd_engine *e, const oamd_selfplay_config *cfg,
                              int32_t *actions_dev, int32_t *finished_dev, float *features_dev,
                              float *policy_dev);
/* n_moves self-play moves of every game with the native net: per move one
 * oamd_engine_search + oamd_engine_selfplay_move, identical results, but each
 * pipeline group chains its searches and moves on its own stream (no join
 * between moves: a group's move and next selection overlap the other groups'
 * ResNet launches). Enqueued only (stream order). per_move_outputs = 1: the
 * output buffers hold n_moves consecutive slices of the per-move shapes above
 * (move i at offset i x G rows); 0: every move overwrites the same slice.
 * Replaces the reference's per-move loop train.py:404-452 (_self_play). */
int oamd_engine_selfplay_steps(oamd_engine *e, oamd_net *net, const oamd_selfplay_config *cfg,
                               int32_t n_moves, int32_t per_move_outputs, int32_t *actions_dev,
                               int32_t *finished_dev, float *features_dev, float *policy_dev);
/* Reset every game to a random opening. */
int oamd_engine_random_openings(oamd_engine *e, int32_t max_moves, uint64_t seed);
/* The random-stream key of a game (DESIGN.md "Random streams"). */
int oamd_engine_game_key(oamd_engine *e, int32_t game, uint64_t *key_host);

/* Timing accumulated over the timed oamd_engine_search calls (HIP events on
 * the launching streams; a query waits for the searches still in flight):
 * total ms spent in the NN kernel, number of NN launches, rows launched
 * (terminal leaves included; oamd_engine_work_counters gives the rows that
 * needed an evaluation). */
int oamd_engine_nn_timing(const oamd_engine *e, float *nn_ms, int64_t *launches, int64_t *rows);
/* Busy time of the ResNet kernel: while timing is enabled, every ResNet
 * launch of a native search (all searches, all rounds, the chain-splitting
 * extra rounds included) records its execution interval in the kernel (first
 * workgroup start to last workgroup end, s_memrealtime); busy_ms is the union
 * of those intervals since timing was last enabled (ms some ResNet launch was
 * running; launches of different NN chains and pipeline groups overlap),
 * launches their count. The rows they evaluated are the difference of
 * oamd_engine_work_counters over the same window, so evals x FLOPs per row /
 * busy is the delivered rate. Waits for the device. */
int oamd_engine_nn_busy(const oamd_engine *e, float *busy_ms, int64_t *launches);
/* Same for the tree kernel (k_tree, one launch per search round and pipeline
 * group): select_ms = total ms of the rounds that select (each also backs up
 * the previous batch, thread by thread), backup_ms = total ms of the final
 * backup-only rounds (one per search and pipeline group). launches = timed
 * select rounds (k_tree launches: rounds x pipeline groups). Timed searches
 * record 4 HIP events per round and pipeline group on the group's stream. */
int oamd_engine_tree_timing(const oamd_engine *e, float *select_ms, float *backup_ms, int64_t *launches);
/* enable: 0 off, 1 time every search, N >= 2 time every N-th search (sampled:
 * a timed search's event packets lengthen the gaps between its launches).
 * The ResNet busy-time window (oamd_engine_nn_busy) restarts here and covers
 * every search while enable != 0; restarting waits for the device. */
int oamd_engine_enable_timing(oamd_engine *e, int32_t enable);

#ifdef __cplusplus
}
#endif

#endif /* OTHELLO_MCTS_AMD_H */
