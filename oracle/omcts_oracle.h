/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked, loaded or called by the
 * product (othello-alphazero_amd/). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it, and only as the checker / the timed
 * CPU baseline.
 *
 * Plain-C restatement of the reference's othello_mcts hot path
 * (yunhao-qian/Othello-AlphaZero, cpp/src/include + cpp/src/lib):
 *   - bitboard rules        position.h:151-272, 308-408
 *   - D4 action transform   transformation.h:40-81
 *   - NN input features     transformation.h:83-116 (+ position_iterator.h:24-71)
 *   - MCTS search           search_thread.cpp:47-260, mcts.h:220-256
 *   - root queries / reuse  mcts.cpp:40-165
 *
 * Pinning (see DESIGN.md "Oracle"): bitboard, transform table and features are
 * checked bit-exactly against vectors produced by the reference headers
 * themselves (oracle/_ref/ref_driver, fixtures in tests/golden/). The MCTS
 * search is pinned by the known-answer visit counts SURVEY.md §4 recorded from
 * the compiled reference (num_threads=1, dirichlet_epsilon=0). The reference's
 * own random sources (std::mt19937 seeded by std::random_device,
 * std::gamma_distribution) are not reproducible; this restatement replaces
 * them with the counter-based stream specified in DESIGN.md "Random streams",
 * which the HIP engine implements identically.
 */
#ifndef OMCTS_ORACLE_H
#define OMCTS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- bitboards (position.h) ------------------------------------------- */
typedef struct {
    int32_t player; /* 1 black, 2 white, 0 terminal */
    uint64_t p1, p2;
    uint64_t legal;      /* legal moves of the side to move */
    uint64_t next_legal; /* opponent's moves, set only when side to move must pass */
} orc_pos;

uint64_t orc_get_legal_moves(uint64_t me, uint64_t opp);
uint64_t orc_get_flips(uint64_t move, uint64_t me, uint64_t opp);
void orc_initial_position(orc_pos *out);
/* action 0..63 = square, 64 = pass; unchecked like Position::apply_action */
void orc_apply_action(const orc_pos *p, int action, orc_pos *out);
/* ascending square order, {64} when the side to move must pass, {} if terminal */
int orc_legal_actions(const orc_pos *p, int32_t *actions_out);
int orc_transform_action(int action, int t);
/* batched loops (n elements) for large-size parity checks */
void orc_legal_moves_n(const uint64_t *me, const uint64_t *opp, uint64_t *out, int64_t n);
void orc_flips_n(const uint64_t *mv, const uint64_t *me, const uint64_t *opp, uint64_t *out, int64_t n);
/* positions as 5 arrays: player (i32), p1, p2, legal, next_legal */
void orc_apply_action_n(const int32_t *player, const uint64_t *p1, const uint64_t *p2,
                        const uint64_t *legal, const uint64_t *next_legal, const int32_t *action,
                        int32_t *o_player, uint64_t *o_p1, uint64_t *o_p2, uint64_t *o_legal,
                        uint64_t *o_next, int64_t n);
/* features of a chain: chain[0] = current position, chain[1] its parent, ...
 * (n_chain entries); writes (1 + 2*history_size) * 64 floats */
void orc_features(const orc_pos *chain, int n_chain, int history_size, int t, float *out);

/* ---- random streams (DESIGN.md "Random streams"; shared spec with HIP) --- */
uint64_t orc_mix64(uint64_t z);
uint64_t orc_stream_key(uint64_t game_key, uint64_t event, uint32_t sub);
float orc_uniform(uint64_t stream_key, uint32_t k);
float orc_logf(float x);
float orc_expf(float x);
/* Gamma(alpha, 1) draw consuming uniforms of one stream */
float orc_gamma(uint64_t stream_key, float alpha);
float orc_cos2pi_sq(float v);

/* ---- MCTS (search_thread.cpp / mcts.cpp) ------------------------------ */
typedef void (*orc_nn_fn)(void *user, const float *features, int rows, int channels,
                          float *policy_out, float *value_out);

typedef struct orc_mcts orc_mcts;

orc_mcts *orc_mcts_create(int history_size, int num_simulations, int num_threads,
                          int batch_size, float c_puct_base, float c_puct_init,
                          float dirichlet_epsilon, float dirichlet_alpha,
                          uint64_t game_key);
void orc_mcts_destroy(orc_mcts *m);
void orc_mcts_reset_position(orc_mcts *m);
/* start from an arbitrary (reachable) position with the given history chain
 * (chain[0] = current, chain[1] = its predecessor, ...) */
void orc_mcts_reset_chain(orc_mcts *m, const orc_pos *chain, int n_chain);
void orc_mcts_position(const orc_mcts *m, orc_pos *out);
/* returns number of simulations (leaf selections) performed */
int orc_mcts_search(orc_mcts *m, orc_nn_fn nn, void *user);
int orc_mcts_num_children(const orc_mcts *m);
void orc_mcts_visit_counts(const orc_mcts *m, int32_t *out);
void orc_mcts_mean_action_values(const orc_mcts *m, float *out);
int32_t orc_mcts_root_visit_count(const orc_mcts *m);
/* 0 ok, 1 terminal root, 2 root not expanded; features 8*(1+2H)*64, policy 8*65 */
int orc_mcts_self_play_data(const orc_mcts *m, float *features, float *policy);
/* 0 ok, -1 out of range, -2 illegal action, -3 pass in terminal, -4 pass with moves */
int orc_mcts_apply_action(orc_mcts *m, int action);
int orc_mcts_node_count(const orc_mcts *m);
uint64_t orc_mcts_events(const orc_mcts *m);
/* train.py:421-430 move choice drawn like the on-device driver (one event) */
int orc_mcts_selfplay_action(orc_mcts *m, int ply, int temperature_moves, float temperature);

#ifdef __cplusplus
}
#endif

#endif
