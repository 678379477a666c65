// Internal device-side data layout of the search engine (see DESIGN.md
// "Data layout in HBM"). Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bitboard.h"

namespace oamd {

constexpr int kMaxDepth = 128;  // path slots per leaf (2 per lane)
constexpr int kMaxHistory = 15; // in_channels = 1 + 2H <= 31
constexpr int kExploreTab = 1 << 20;
constexpr int kMaxLeaves = 1024;  // num_threads * batch_size per game and step

// Edge statistics of the edge INTO a node (search_node.h:26-40).
struct NodeStat {
    int32_t n;  // visit_count
    float w;    // total_action_value
    float q;    // mean_action_value
    float p;    // prior_probability (1.0f for a fresh root)
};

// Tree links. player mirrors the node position's player (0 = terminal).
struct NodeLink {
    int32_t first_child;  // local node id, -1 while unexpanded
    int32_t n_children;
    int32_t parent;       // local node id, -1 for a game's first position
    int32_t player;
};

struct NodePos {
    uint64_t p1, p2, legal, next_legal;
};

enum GameFlags : int32_t { kActive = 1, kOverflow = 2, kDepthCap = 4 };

struct GameState {
    int32_t root;
    int32_t count;   // nodes allocated in this game's pool
    int32_t flags;
    int32_t hist_n;  // valid entries of hist
    uint64_t key;    // random stream key of the game
    uint64_t event;  // next random event
    int32_t hist[16];  // strict ancestors of the root: parent, grandparent, ...
    int32_t ply;       // moves played since the last reset (self-play driver)
    int32_t resume;    // k_tree chain splitting: the virtual thread this game's next round starts at
    int32_t cuts;      // ... and the chains split so far in this search
    int32_t moves_left;  // free-running self-play (k_tree_free): moves this game still plays in the call
    int32_t fresh;       // ... 1: its next round starts a new search
    int32_t pad[2];
};

// Packed NN input row (FW uint64 words): word 0 = meta, then (p1, p2) of the
// leaf and its H-1 nearest ancestors, untransformed. meta bit 0 = player - 1,
// bits 8..10 = transform, bit 16 = row valid (non-terminal leaf).
__host__ __device__ inline int feature_words(int H) { return 2 + 2 * H; }

// k_tree per-thread state (EngineView::tstate): batches selected in this search
// in the low 31 bits (steps = ceil(S / L) has no upper limit), the batch
// waiting for the NN in bit 31
constexpr int32_t kTstateSel = 0x7FFFFFFF;
constexpr int32_t kTstatePend = (int32_t)0x80000000u;

struct EngineView {
    int32_t G, L, H, FW;
    int64_t cap;
    NodeLink* link;
    NodeStat* stat;
    NodePos* pos;
    GameState* games;
    int32_t* leaf;   // G*L
    int32_t* depth;  // G*L
    int32_t* trans;  // G*L
    int32_t* path;   // G*L*kMaxDepth
    uint64_t* feat;  // G*L*FW
    float* policy;   // G*L*65
    float* value;    // G*L
    const float* explore_tab;  // kExploreTab
    float c_base, c_init, eps, alpha;
    unsigned long long* counters;  // [0..11], tree.hip add_counters / count_launch
    int32_t* rowlist;  // G*L: evaluation lists (pipeline group k: from its first game's row)
    int32_t* tstate;   // G*L (entry g*L + t for virtual thread t): batches selected | kTstatePend
    int32_t steps;     // batches per virtual thread and search: ceil(num_simulations / L)
    int32_t B;         // batch_size (leaves per virtual thread and batch)
    int32_t terminal_skip;  // 1: an all-terminal batch is backed up at once and its thread selects
                            // again (the reference's interleaving); 0: it waits for its round
};

}  // namespace oamd
