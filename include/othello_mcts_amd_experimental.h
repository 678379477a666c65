/*
 * othello_mcts_amd_experimental.h — scheduling knobs and diagnostics of the
 * native engine, outside the product ABI (othello_mcts_amd.h).
 *
 * The product defaults (2 pipeline groups from 64 games, 2 NN chains, chain
 * budget 2 with up to 64 cuts, adaptive extra rounds with minimum 1, a
 * 128-workgroup grid for the extra rounds) were measured in DESIGN.md §7 and
 * need no setting. These setters exist for A/B measurements
 * (bench.py flags, tools/); none of them changes a result — every search
 * output is identical for every setting (tests/test_gpu_configs.py,
 * tests/test_gpu_resnet.py). The debug readers work only in diagnostic builds.
 * Not part of the reference's interface: nothing in othello_mcts.cpp:49-151
 * corresponds to them.
 */
#ifndef OTHELLO_MCTS_AMD_EXPERIMENTAL_H
#define OTHELLO_MCTS_AMD_EXPERIMENTAL_H

#include "othello_mcts_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Split the games into `groups` pipeline groups (own HIP streams) so that tree
 * kernels of one group overlap the NN launch of another (0 = auto: 2 groups
 * from 64 games, else 1; at most 8). Results do not depend on it. */
int oamd_engine_set_pipeline(oamd_engine *e, int32_t groups);
/* The pipeline groups' ResNet launches form `chains` chains (group k in chain
 * k % chains, 1..4, default 2): launches of one chain run one after another,
 * chains run concurrently (the default lets the two groups' launches overlap
 * at their ends). Results do not depend on it. */
int oamd_engine_set_nn_chains(oamd_engine *e, int32_t chains);
/* Native search with the exact interleaving: a virtual thread whose batches
 * come back all terminal selects again at once (search_thread.cpp:102-127),
 * which near a game's end can run a thread's whole remaining search inside one
 * round and hold its pipeline group's ResNet launch. After `budget`
 * re-selections in a round such a chain stops and the game's next round
 * resumes it exactly there (every game keeps its order of operations; only
 * round boundaries move), at most `cuts` times per search, at the cost of
 * up to `cuts` extra rounds per search (see the adaptive count below; never
 * more than T x steps / budget, the most cuts one game's search can use).
 * Default budget 2, cuts 64; budget 0 = never split. Results do not depend on
 * it. */
int oamd_engine_set_chain_split(oamd_engine *e, int32_t budget, int32_t cuts);
/* Adaptive extra rounds (default on, min_rounds 1): a grouped native search
 * runs X extra rounds and allows X cuts per game, X in [min(min_rounds,
 * cuts), cuts], following the search two back (read back without draining
 * the queue; the first two searches run min_rounds): X = cuts when some
 * root of that search was within 12 empty squares of the end (the endgame,
 * where all-terminal chains appear), else
 * the most cuts u any game used + min_rounds (2X + 2 + min_rounds when a
 * game ran out of cuts). Extra rounds past every game's last cut are empty
 * launches; a game that would need more cuts runs its last chain uncut.
 * enable = 0: X = cuts always. Scheduling only: results are identical. */
int oamd_engine_set_adaptive_extra_rounds(oamd_engine *e, int32_t enable, int32_t min_rounds);
/* Workgroups of the chain-splitting extra rounds' ResNet launches (default
 * 128; 0 = the regular grid, the list's capacity): those launches hold the
 * rows of lagging games only (none outside endgames), so a small grid loops
 * over them instead of dispatching ~1000 mostly empty workgroups between the
 * other NN chain's. Scheduling only: results are identical. */
int oamd_engine_set_extra_round_grid(oamd_engine *e, int32_t workgroups);
/* Diagnostics: copy the ResNet kernel's per-workgroup time stamps and cycle
 * sums (24 u64 per workgroup, resnet.hip kStampStride; see tools/nn_stamps.py)
 * of the last launch. Only in builds with OAMD_EXTRA_FLAGS=-DOAMD_STAMPS;
 * otherwise OAMD_INVALID_ARGUMENT. */
int oamd_debug_read_stamps(uint64_t *out, int64_t n);
/* Diagnostics: k_tree's phase cycle sums over every wave since the last reset
 * (tools/tree_stamps.py); reset != 0 zeroes them after the copy. Only in
 * builds with OAMD_EXTRA_FLAGS=-DOAMD_TREE_STAMPS; otherwise
 * OAMD_INVALID_ARGUMENT. */
int oamd_debug_tree_stamps(uint64_t *out, int64_t n, int32_t reset);

/* Free-running self-play in oamd_engine_selfplay_steps (default on): every
 * game plays its moves on its own — the round that completes a game's search
 * also runs its move and its next search's first round — so no game waits at
 * a move for the group's slowest one, and no extra rounds are run. Per game
 * the operations and their order are those of n x (oamd_engine_search +
 * oamd_engine_selfplay_move), and every output is identical; enable = 0 gives
 * the lock-step multi-move call (searches with chain-splitting extra rounds).
 * One game with num_threads > 1 (the thread-split schedule) is always
 * lock-step. */
int oamd_engine_set_free_running(oamd_engine *e, int32_t enable);

/* Diagnostics: the tree kernels' algorithmic work since the engine was
 * created (host outputs; waits for the engine's stream), the terms of the
 * byte model of SURVEY.md §8(d) that bench.py prices per k_tree launch:
 * descent levels (= the depth sum of oamd_engine_descent_depths), children
 * whose statistics those levels scanned, expansions, children created, and
 * tree kernel launches (k_tree, k_tree_wide, k_tree_free). Any pointer may be
 * NULL. */
int oamd_engine_tree_work(oamd_engine *e, int64_t *levels, int64_t *children_scanned, int64_t *expansions,
                          int64_t *children_created, int64_t *launches);

#ifdef __cplusplus
}
#endif

#endif /* OTHELLO_MCTS_AMD_EXPERIMENTAL_H */
