// Search-tree kernels: one 64-lane wavefront per game.
//
// The reference runs num_threads CPU threads per game, each selecting
// batch_size leaves under a mutex with virtual loss, sending them through the
// NN and backing them up (search_thread.cpp:47-260). Here a round of a game
// (every thread backs up its previous batch and selects its next one, see
// k_tree) is one wave of k_tree followed by one row block of the NN launch;
// all games of the engine run in the same launches. Lanes parallelise what is parallel inside one game:
// the child scan of PUCT (lane = child), virtual loss and backup (lane = path
// depth), expansion (lane = square), feature gathers (lane = history slot).
// The sequential dependence between the L descents (each sees the previous
// descents' virtual losses) is kept exactly.
//
// Floating point: compiled with -ffp-contract=off and IEEE division/sqrt so
// that every PUCT score, virtual loss and backup is bit-identical to the
// reference's float arithmetic (search_thread.cpp:163-166, 198-249, 270-280).

#include <hip/hip_runtime.h>

#include "bitboard.h"
#include "engine.h"
#include "kernels.h"
#include "rng.h"

namespace oamd {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

#ifndef OAMD_CHAIN_PRIO
#define OAMD_CHAIN_PRIO 2
#endif

// Diagnostic build only (-DOAMD_TREE_STAMPS, tools/tree_stamps.py): cycle
// sums of k_tree's phases (s_memtime), per wave in LDS (k_tree blocks are one
// wave), added to g_tree_stamps when the wave ends. Nothing else reads them.
#ifdef OAMD_TREE_STAMPS
enum TreeStamp {
    kTsWaves, kTsCycles, kTsDescent, kTsLevels, kTsLeaves, kTsPost, kTsBackup, kTsBackedUp, kTsTerminal,
    kTsMaxCycles, kTsBatches, kTsSelect, kTsExpand, kTsPathW, kTsNoise, kTsRefill, kTsCount
};
__device__ unsigned long long g_tree_stamps[kTsCount];
__shared__ unsigned long long ts_acc[kTsCount];
#define TS_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define TS_ADD(i, x) do { if (lane_id() == 0) ts_acc[i] += (unsigned long long)(x); } while (0)
#else
#define TS_T(v) ((void)0)
#define TS_ADD(i, x) ((void)0)
#endif

__device__ __forceinline__ void wait_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Orders this wave's earlier global stores before its later loads of the same
// words, from any lane: the next descent / backup reads the statistics the
// previous one stored. A wavefront-scope fence: the AMDGPU memory model needs
// no wait for it on gfx950 (it emits none; a wave's vector memory operations
// reach the cache in order), so the stores' write-back overlaps the next
// descent's first loads instead of a vmcnt(0) drain per leaf.
// -DOAMD_TREE_DRAIN restores the vmcnt(0) drain (the A/B build that
// shows both orderings give identical results; tests/test_cpu_host.py checks
// in the ISA that k_tree reads no statistics through the scalar cache, which
// would not see these vector stores).
#ifdef OAMD_TREE_DRAIN
__device__ __forceinline__ void wave_order() { wait_stores(); }
#else
__device__ __forceinline__ void wave_order() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }
#endif

// Wave reductions with DPP (row_shr / row_bcast inclusive scan, the total ends
// in lane 63): a few cycles per step, where __shfl_xor compiles to a chain of
// ds_bpermute LDS round trips (the dominant cost of a k_select level).
template <int CTRL, int ROW_MASK, int BANK_MASK, typename T>
__device__ __forceinline__ T dpp_move(T x, T id) {
    return __builtin_bit_cast(T, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, id), __builtin_bit_cast(int, x),
                                                             CTRL, ROW_MASK, BANK_MASK, false));
}

template <typename T, typename Op>
__device__ __forceinline__ T wave_scan_last(T v, T id, Op op) {
    static_assert(sizeof(T) == 4, "32-bit lanes");
    T t = op(v, dpp_move<0x111, 0xF, 0xF>(v, id));  // row_shr:1
    t = op(t, dpp_move<0x112, 0xF, 0xF>(v, id));    // row_shr:2
    t = op(t, dpp_move<0x113, 0xF, 0xF>(v, id));    // row_shr:3
    t = op(t, dpp_move<0x114, 0xF, 0xE>(t, id));    // row_shr:4, banks 1-3
    t = op(t, dpp_move<0x118, 0xF, 0xC>(t, id));    // row_shr:8, banks 2-3
    t = op(t, dpp_move<0x142, 0xA, 0xF>(t, id));    // row_bcast:15 into rows 1, 3
    t = op(t, dpp_move<0x143, 0xC, 0xF>(t, id));    // row_bcast:31 into rows 2, 3
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t), 63));
}

__device__ __forceinline__ int wave_sum(int v) {
    return wave_scan_last(v, 0, [](int a, int b) { return a + b; });
}

__device__ __forceinline__ float wave_max(float v) {
    return wave_scan_last(v, -__builtin_inff(), [](float a, float b) { return fmaxf(a, b); });
}

// The same scans over the first n lanes only (lanes >= n hold the identity):
// with n <= 16 (almost every node: Othello positions rarely have more legal
// moves) row 0 holds them all, so the two row_bcast steps are skipped and the
// total is read from lane 15.
template <typename T, typename Op>
__device__ __forceinline__ T wave_scan_first_n(T v, T id, Op op, int n) {
    static_assert(sizeof(T) == 4, "32-bit lanes");
    T t = op(v, dpp_move<0x111, 0xF, 0xF>(v, id));  // row_shr:1
    t = op(t, dpp_move<0x112, 0xF, 0xF>(v, id));    // row_shr:2
    t = op(t, dpp_move<0x113, 0xF, 0xF>(v, id));    // row_shr:3
    t = op(t, dpp_move<0x114, 0xF, 0xE>(t, id));    // row_shr:4, banks 1-3
    t = op(t, dpp_move<0x118, 0xF, 0xC>(t, id));    // row_shr:8, banks 2-3
    if (n > 16) {
        t = op(t, dpp_move<0x142, 0xA, 0xF>(t, id));  // row_bcast:15 into rows 1, 3
        t = op(t, dpp_move<0x143, 0xC, 0xF>(t, id));  // row_bcast:31 into rows 2, 3
    }
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t), n > 16 ? 63 : 15));
}

__device__ __forceinline__ int wave_max_i(int v) {
    return wave_scan_last(v, (int)0x80000000, [](int a, int b) { return a > b ? a : b; });
}

// First lane holding the maximum (strict '>' scan in child order,
// search_thread.cpp:222,254): the max, then the lowest lane equal to it.
// Values are finite or -inf (no NaN).
__device__ __forceinline__ int wave_argmax_first(float v, int) {
    const float m = wave_max(v);
    const uint64_t eq = __ballot(v == m);
    return __ffsll((unsigned long long)eq) - 1;
}

// ... over the first n lanes (the others hold -inf)
__device__ __forceinline__ int wave_argmax_first_n(float v, int n) {
    const float m = wave_scan_first_n(v, -__builtin_inff(), [](float a, float b) { return fmaxf(a, b); }, n);
    const uint64_t eq = __ballot(v == m);
    return __ffsll((unsigned long long)eq) - 1;
}

__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
}
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__device__ __forceinline__ NodeStat load_stat(const NodeStat* s) {
    const int4 v = *reinterpret_cast<const int4*>(s);
    NodeStat r;
    r.n = v.x;
    r.w = __int_as_float(v.y);
    r.q = __int_as_float(v.z);
    r.p = __int_as_float(v.w);
    return r;
}

__device__ __forceinline__ void store_stat(NodeStat* s, const NodeStat& r) {
    *reinterpret_cast<int4*>(s) =
        make_int4(r.n, __float_as_int(r.w), __float_as_int(r.q), __float_as_int(r.p));
}

__device__ __forceinline__ NodeLink load_link(const NodeLink* l) {
    const int4 v = *reinterpret_cast<const int4*>(l);
    return NodeLink{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void store_link(NodeLink* l, const NodeLink& v) {
    *reinterpret_cast<int4*>(l) = make_int4(v.first_child, v.n_children, v.parent, v.player);
}

__device__ __forceinline__ Pos load_pos(const NodePos* p, int player) {
    Pos r;
    r.player = player;
    r.pad_ = 0;
    r.p1 = p->p1;
    r.p2 = p->p2;
    r.legal = p->legal;
    r.next_legal = p->next_legal;
    return r;
}

__device__ __forceinline__ void store_pos(NodePos* p, const Pos& v) {
    p->p1 = v.p1;
    p->p2 = v.p2;
    p->legal = v.legal;
    p->next_legal = v.next_legal;
}

// exploration_rate of search_thread.cpp:198-203, tabulated on the host with
// the host's logf so that it is bit-identical to the CPU reference.
__device__ __forceinline__ float explore_rate(const EngineView& E, int n) {
    if (n >= 0 && n < kExploreTab) return E.explore_tab[n];
    return logf(((float)(1 + n) + E.c_base) / E.c_base) + E.c_init;
}

// sqrt of the children's visit sum: IEEE correctly rounded on the device as on
// the host (HIP's default correctly-rounded fp32 sqrt, -fno-fast-math)
__device__ __forceinline__ float sqrt_count(const EngineView&, int n) { return sqrtf((float)n); }

// Square of the j-th legal action of a position (legal_actions order,
// position.h:308-326), computed by lane = square.
__device__ __forceinline__ int action_of_child(uint64_t legal, int j) {
    if (legal == 0) return 64;
    const int s = lane_id();
    const bool set = (legal >> (63 - s)) & 1ULL;
    const uint64_t before = s == 0 ? 0ULL : (legal & (~0ULL << (64 - s)));
    const bool hit = set && popcount64(before) == j;
    const uint64_t b = __ballot(hit);
    return b ? (__ffsll((unsigned long long)b) - 1) : 64;
}

// Child index of an action in legal_actions order (mcts.cpp:147-153).
__device__ __forceinline__ int child_index_of(uint64_t legal, int n_children, int action) {
    if (action == 0 || n_children <= 1 || action == 64) return 0;
    return popcount64(legal & (~0ULL << (64 - action)));
}

// Packed features of row r (position_iterator.h:24-71, transformation.h:83-116):
// a meta word (leaf player, symmetry, valid; 0 for a terminal leaf: no NN row)
// and the H positions leaf = path[d], its ancestors, then the game history.
// The meta word is written at the leaf; the positions are gathered for up to
// 64 / H leaves at once (flush_ancestors), so the selection loop does not wait
// for a position load per leaf.
__device__ __forceinline__ void write_feature_meta(const EngineView& E, int r, int leaf_player, int t,
                                                   bool valid) {
    if (lane_id() != 0) return;
    uint64_t* row = E.feat + (size_t)r * E.FW;
    row[0] = valid ? ((uint64_t)((leaf_player - 1) & 1) | ((uint64_t)t << 8) | (1ULL << 16)) : 0ULL;
    row[1] = 0;
}

// Node of position h = lane (< H) of a leaf at depth d: path[d - h] for h <= d,
// else hist[h - d - 1]; -1 past the history (a zero plane pair)
__device__ __forceinline__ int feature_ancestor(int d, int p0, int p1, int hist_node, int hist_n) {
    const int lane = lane_id();
    const int idx = d - lane;
    const int from_p0 = __shfl(p0, idx & 63);
    const int from_p1 = __shfl(p1, idx & 63);
    const int hj = lane - d - 1;
    const int from_h = __shfl(hist_node, hj & 63);
    int anc = -1;
    if (idx >= 0) anc = idx < 64 ? from_p0 : from_p1;
    else if (hj < hist_n) anc = from_h;
    return anc;
}

// Position planes of rows r0 .. r0 + n - 1: lane j = (leaf j / H, position
// j % H) holds its node in anc (from feature_ancestor); bit k of `valid` =
// row r0 + k has an NN row. One load round trip for all of them.
__device__ __forceinline__ void flush_ancestors(const EngineView& E, size_t base, int r0, int n, int anc,
                                                uint64_t valid) {
    const int lane = lane_id();
    const int k = lane / E.H, h = lane - k * E.H;
    if (k >= n || !((valid >> k) & 1ULL)) return;
    uint64_t a1 = 0, a2 = 0;
    if (anc >= 0) {
        const NodePos* np = E.pos + base + anc;
        a1 = np->p1;
        a2 = np->p2;
    }
    uint64_t* row = E.feat + (size_t)(r0 + k) * E.FW;
    row[2 + 2 * h] = a1;
    row[3 + 2 * h] = a2;
}

// Append the NN rows of non-terminal leaves among rows c0 + j (bit j of
// `valid`) to the group's evaluation list: one atomic per chunk of <= 64 rows
// reserves the slots, lane j writes row c0 + j. The ResNet launch reads the
// list, so terminal leaves cost it nothing (the reference builds no NN row for
// them, search_thread.cpp:88-90); the list order does not matter, every row's
// evaluation is independent of its place in a launch.
__device__ __forceinline__ void append_rows(const EngineView& E, int* cnt, int list_base, int c0, uint64_t valid) {
    const int n = popcount64(valid);
    if (n == 0) return;
    int slot = 0;
    if (lane_id() == 0) slot = atomicAdd(cnt, n);
    slot = readlane_i(slot, 0);
    const int lane = lane_id();
    if ((valid >> lane) & 1ULL)
        E.rowlist[list_base + slot + popcount64(valid & ((1ULL << lane) - 1ULL))] = c0 + lane;
}

// ---------------------------------------------------------------------------
// Selection: descents i in [i0, i1) with virtual loss (search_thread.cpp:59-100).
// cnt != nullptr: the non-terminal leaves' rows go to the evaluation list.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void select_range(const EngineView& E, int g, GameState* gs, size_t base,
                                             int i0, int i1, uint64_t& event, int hist_node,
                                             int hist_n, unsigned long long& sims,
                                             unsigned long long& evals, int* cnt, int list_base,
                                             unsigned long long& depth_sum, int& depth_max,
                                             unsigned long long& scan_sum) {
    const int lane = lane_id();
    const int root = gs->root;
    const uint64_t key = gs->key;
    // the root's link is fixed during one thread's selections (expansions happen
    // in that thread's backup, before this range); its N grows by one per
    // selected leaf (search_thread.cpp:78)
    const NodeLink root_link = load_link(E.link + base + root);
    int root_n = E.stat[base + root].n;
    uint64_t valid_rows = 0;  // bit i - c0: row i is an NN row (chunks of 64 rows from i0)
    int c0 = i0;
    // Root noise vectors drawn ahead: lane s * nz_nc + j holds the noise of
    // child j at event nz_base + s, for as many events as 64 lanes hold (a
    // selection followed by a non-terminal leaf's symmetry draw uses two, one
    // ending in a terminal leaf one); a selection past them draws again.
    // The noise is a function of (game key, event, child) only, so these are
    // the draws of the selections themselves.
    float nz_cache = 0.0f;
    uint64_t nz_base = ~0ULL;
    int nz_nc = 0;
    // feature positions of leaves f0 .. (up to 64 / H of them), flushed together
    const int per_flush = 64 / E.H;
    int f0 = i0, anc_rec = -1;
    uint64_t fvalid = 0;

    for (int i = i0; i < i1; ++i) {
        const int r = g * E.L + i;
        int node = root;
        int d = 0;
        int p0 = lane == 0 ? root : -1;  // path slot `lane`
        int p1 = -1;                     // path slot 64 + lane
        NodeLink lk = root_link;
        // exploration rate of `node` (from its N); for a chosen child it was
        // fetched by the child's lane at the previous level
        float er = explore_rate(E, root_n);
        TS_T(ts0);
        // One dependent memory round trip per level: the stats AND links of all
        // children are loaded together; the chosen child's link, N and
        // exploration rate come from its lane (readlane), not from a second load.
        while (!(lk.player == 0 || lk.n_children == 0) && d < kMaxDepth - 1) {
            const int nc = lk.n_children, fc = lk.first_child;
            scan_sum += (unsigned long long)nc;  // children whose stats this level reads
            int4 cs4 = make_int4(0, 0, 0, 0), cl4 = make_int4(0, 0, 0, 0);
            if (lane < nc) {
                cs4 = *reinterpret_cast<const int4*>(E.stat + base + fc + lane);
                cl4 = *reinterpret_cast<const int4*>(E.link + base + fc + lane);
            }
            // every child lane fetches its own exploration rate now, so the
            // chosen child's is ready for the next level (no dependent table read)
            const float er_child = lane < nc ? explore_rate(E, cs4.x) : 0.0f;
            int best = 0;
            if (nc > 1) {
                const NodeStat cs{cs4.x, __int_as_float(cs4.y), __int_as_float(cs4.z), __int_as_float(cs4.w)};
                const int total = wave_scan_first_n(lane < nc ? cs.n : 0, 0, [](int a, int b) { return a + b; }, nc);
                const float mult = er * sqrt_count(E, total);
                float prob = cs.p;
                if (node == root && E.eps > 0.0f) {
                    // fresh Dirichlet noise on every root selection (search_thread.cpp:230-249)
                    TS_T(tn0);
                    const int slots = 64 / nc;
                    const uint64_t off = event - nz_base;
                    if (nz_nc != nc || off >= (uint64_t)slots) {
                        TS_T(tr0);
                        nz_base = event;
                        nz_nc = nc;
                        const int sl = lane / nc, j = lane - sl * nc;
                        nz_cache = sl < slots ? gamma_draw(stream_key(key, event + (uint64_t)sl, (uint32_t)j), E.alpha)
                                              : 0.0f;
                        TS_T(tr1);
                        TS_ADD(kTsRefill, tr1 - tr0);
                    }
                    float noise = __shfl(nz_cache, ((int)(event - nz_base) * nc + lane) & 63);
                    if (lane >= nc) noise = 0.0f;
                    event += 1;
                    float nsum = 0.0f;
                    for (int j = 0; j < nc; ++j) nsum += readlane_f(noise, j);
                    if (nsum == 0.0f) nsum = 1.0f;
                    const float pm = 1.0f - E.eps;
                    const float nm = E.eps / nsum;
                    prob = cs.p * pm + noise * nm;
                    TS_T(tn1);
                    TS_ADD(kTsNoise, tn1 - tn0);
                }
                float ucb = cs.q + mult * prob / (1.0f + (float)cs.n);
                if (lane >= nc) ucb = -__builtin_inff();
                best = wave_argmax_first_n(ucb, nc);
            }  // a single child is taken without scoring (search_thread.cpp:194-196)
            const int child = fc + best;
            const int4 clk4 = make_int4(readlane_i(cl4.x, best), readlane_i(cl4.y, best),
                                        readlane_i(cl4.z, best), readlane_i(cl4.w, best));
            const float er_next = readlane_f(er_child, best);
            ++d;
            if (lane == (d & 63)) {
                if (d < 64) p0 = child;
                else p1 = child;
            }
            node = child;
            lk = NodeLink{clk4.x, clk4.y, clk4.z, clk4.w};
            er = er_next;
        }
        TS_T(ts1);
        TS_ADD(kTsDescent, ts1 - ts0);
        TS_ADD(kTsLevels, d);
        TS_ADD(kTsLeaves, 1);
        TS_ADD(kTsTerminal, lk.player == 0 ? 1 : 0);
        if (d == kMaxDepth - 1 && lk.player != 0 && lk.n_children != 0 && lane == 0)
            atomicOr(&gs->flags, (int)kDepthCap);
        // virtual loss on the path excluding the root (search_thread.cpp:69-76)
        if (lane >= 1 && lane <= d) {
            NodeStat s = load_stat(E.stat + base + p0);
            s.n += 1;
            s.w -= 1.0f;
            s.q = s.w / (float)s.n;
            store_stat(E.stat + base + p0, s);
        }
        if (64 + lane <= d) {
            NodeStat s = load_stat(E.stat + base + p1);
            s.n += 1;
            s.w -= 1.0f;
            s.q = s.w / (float)s.n;
            store_stat(E.stat + base + p1, s);
        }
        root_n += 1;
        if (lane == 0) E.stat[base + root].n = root_n;  // search_thread.cpp:78
        // record the path for the backup
        int* gp = E.path + (size_t)r * kMaxDepth;
        if (lane <= d) gp[lane] = p0;
        if (64 + lane <= d) gp[64 + lane] = p1;
        const bool valid = lk.player != 0;
        int t = 0;
        if (valid) {
            t = draw_transform(key, event);  // search_thread.cpp:92
            event += 1;
        }
        if (lane == 0) {
            E.leaf[r] = node;
            E.depth[r] = d;
            E.trans[r] = t;
        }
        write_feature_meta(E, r, lk.player, t, valid);
        {
            const int anc = feature_ancestor(d, p0, p1, hist_node, hist_n);
            const int k = i - f0;
            const int moved = __shfl(anc, (lane - k * E.H) & 63);
            if (lane >= k * E.H && lane < (k + 1) * E.H) anc_rec = moved;
            fvalid |= (uint64_t)(valid ? 1 : 0) << k;
            if (k == per_flush - 1 || i == i1 - 1) {
                flush_ancestors(E, base, g * E.L + f0, k + 1, anc_rec, fvalid);
                f0 = i + 1;
                fvalid = 0;
            }
        }
        sims += 1;
        evals += valid ? 1 : 0;
        depth_sum += (unsigned long long)d;
        depth_max = d > depth_max ? d : depth_max;
        if (cnt) {
            valid_rows |= (uint64_t)(valid ? 1 : 0) << (i - c0);
            if (i - c0 == 63 || i == i1 - 1) {
                append_rows(E, cnt, list_base, g * E.L + c0, valid_rows);
                valid_rows = 0;
                c0 = i + 1;
            }
        }
        wave_order();  // the next descent reads these statistics
        TS_T(ts2);
        TS_ADD(kTsPost, ts2 - ts1);
    }
}

// ---------------------------------------------------------------------------
// Expansion: the children of one position, four lanes per child.
// The reference computes each child with apply_action (position.h:328-363):
// flips in 8 directions, then the child's legal moves (8 directions), and the
// other side's when those are empty. Lane 4k + q works on child k and on the
// two opposite directions of magnitude {1, 7, 8, 9}[q] (edge masks as
// position.h:155-172); an OR over the child's 4 lanes completes each 8-way
// union. Exactly the same bit operations as bitboard.h's apply_action, 4x
// fewer instructions per expansion than one child per lane (16 children per
// pass; positions with more take a second pass).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t or_quad(uint64_t x) {
    // quad_perm [1,0,3,2], then [2,3,0,1]: every lane of a quad holds the quad's OR
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0xB1, 0xF, 0xF, false);
    hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0xB1, 0xF, 0xF, false);
    lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x4E, 0xF, 0xF, false);
    hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0x4E, 0xF, 0xF, false);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// opponent run from seed along << mag and >> mag (run_dir's 6 steps each)
__device__ __forceinline__ void runs_pair(uint64_t seed, uint64_t om, int mag, uint64_t& l, uint64_t& r) {
    l = om & (seed << mag);
    r = om & (seed >> mag);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        l |= om & (l << mag);
        r |= om & (r >> mag);
    }
}

// The k-th set square (ascending square index = descending bit) of a mask
__device__ __forceinline__ int kth_square(uint64_t mask, int k) {
    // bit-reverse so that square s is bit s, then select the k-th set bit from
    // the bottom by halving
    const uint32_t rlo = __builtin_bitreverse32((uint32_t)(mask >> 32));  // squares 0..31
    const uint32_t rhi = __builtin_bitreverse32((uint32_t)mask);          // squares 32..63
    int pos = 0;
    uint32_t x = rlo;
    int c = __builtin_popcount(rlo);
    if (k >= c) {
        k -= c;
        pos = 32;
        x = rhi;
    }
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        c = __builtin_popcount(x & ((1u << w) - 1u));
        if (k >= c) {
            k -= c;
            pos += w;
            x >>= w;
        }
    }
    return pos;
}

// Expand position P (not terminal, legal != 0) into children fc .. fc+nc-1 in
// legal_actions order (position.h:308-326), priors policy[transform(a, t)].
// pol_l: entry `lane` of the leaf's policy row (prefetched by backup_range)
__device__ __forceinline__ void expand_quads(const EngineView& E, size_t base, int leaf, const Pos& P, int fc,
                                             int nc, int t, float pol_l) {
    const int lane = lane_id();
    const int q = lane & 3;
    const int mag = q == 0 ? 1 : (q == 1 ? 7 : (q == 2 ? 8 : 9));
    const uint64_t dmask = q == 0 ? kNoLR : (q == 2 ? kNoTB : kNoEdge);
    const bool black = P.player == 1;
    const uint64_t me = black ? P.p1 : P.p2;
    const uint64_t opp = black ? P.p2 : P.p1;
    for (int k0 = 0; k0 < nc; k0 += 16) {
        const int k = k0 + (lane >> 2);
        const int sq = kth_square(P.legal, k < nc ? k : 0);
        const uint64_t move = 1ULL << (63 - sq);
        // flips (position.h:231-262): runs capped by an own disc
        uint64_t l, r;
        runs_pair(move, opp & dmask, mag, l, r);
        uint64_t f = (((l << mag) & me) ? l : 0ULL) | (((r >> mag) & me) ? r : 0ULL);
        f = or_quad(f);
        const uint64_t mine = me | move | f, theirs = opp & ~f;  // the mover's / the opponent's discs
        // the child's side to move is the opponent (position.h:349-362)
        runs_pair(theirs, mine & dmask, mag, l, r);
        uint64_t lg = or_quad((l << mag) | (r >> mag)) & ~(mine | theirs);
        uint64_t nx = 0;
        int player = 3 - P.player;
        if (lg == 0) {  // the child's mover must pass: the other side's moves
            runs_pair(mine, theirs & dmask, mag, l, r);
            nx = or_quad((l << mag) | (r >> mag)) & ~(mine | theirs);
            if (nx == 0) player = 0;
        }
        // the prior of a move (< 64) from the lane holding its transformed entry
        const float prior = __shfl(pol_l, transform_action(sq, t));
        if (q == 0 && k < nc) {
            Pos c;
            c.player = player;
            c.pad_ = 0;
            c.p1 = black ? mine : theirs;
            c.p2 = black ? theirs : mine;
            c.legal = lg;
            c.next_legal = nx;
            const int id = fc + k;
            store_link(E.link + base + id, NodeLink{-1, 0, leaf, c.player});
            store_stat(E.stat + base + id, NodeStat{0, 0.0f, 0.0f, prior});
            store_pos(E.pos + base + id, c);
        }
    }
}

// ---------------------------------------------------------------------------
// Expansion + backup of leaves [i0, i1) (search_thread.cpp:116-127, 130-190).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void backup_range(const EngineView& E, int g, size_t base, int i0, int i1,
                                             int& count, bool& overflow, unsigned& expansions) {
    const int lane = lane_id();
    TS_T(tb0);
    TS_ADD(kTsBackedUp, i1 - i0);
    // Leaves are processed in order (their backups share path nodes), but
    // everything a leaf needs except the path statistics is independent of
    // the earlier leaves: it is fetched for up to 64 leaves at once, one lane
    // per leaf. A chunk's prefetch starts after every earlier store of the
    // wave has completed, so links are current except for duplicates of a
    // leaf expanded earlier in the same chunk: those are found by a ballot
    // over the chunk's lanes (duplicates never expand again, search_thread.cpp:
    // 133-135, and use only the immutable player / parent of the link).
    for (int c0 = i0; c0 < i1; c0 += 64) {
        const int cend = i1 - c0 < 64 ? i1 - c0 : 64;
        const int cl = lane < cend ? lane : 0;
        const int rl = g * E.L + c0 + cl;
        const int leaf_v = E.leaf[rl];
        const int d_v = E.depth[rl];
        const int t_v = E.trans[rl];
        const float val_v = E.value[rl];
        const int4 lk_v = *reinterpret_cast<const int4*>(E.link + base + leaf_v);
        const NodePos pos_v = E.pos[base + leaf_v];
        bool expanded_here = false;  // lane j: leaf j of this chunk expanded its node
        // path and policy row (entry `lane`; the pass's entry 64 is read when used) of the chunk's first
        // leaf; each leaf prefetches the next one's (the ResNet launch that
        // wrote the rows has completed before this kernel started)
        int gp0 = 0, gp1 = 0;
        float pol_l = 0.0f;
        {
            const int* gp = E.path + (size_t)(g * E.L + c0) * kMaxDepth;
            const int d0 = readlane_i(d_v, 0);
            if (lane >= 1 && lane <= d0) gp0 = gp[lane];
            if (64 + lane <= d0) gp1 = gp[64 + lane];
            const float* pr = E.policy + (size_t)(g * E.L + c0) * 65;
            pol_l = pr[lane];
        }
        for (int j = 0; j < cend; ++j) {
            const int r = g * E.L + c0 + j;
            const int leaf = readlane_i(leaf_v, j);
            const int d = readlane_i(d_v, j);
            const int t = readlane_i(t_v, j);
            const NodeLink lk{readlane_i(lk_v.x, j), readlane_i(lk_v.y, j), readlane_i(lk_v.z, j),
                              readlane_i(lk_v.w, j)};
            const int path0 = gp0, path1 = gp1;
            const float polj = pol_l;
            if (j + 1 < cend) {  // next leaf's path and policy row, behind this leaf's work
                const int* gp = E.path + (size_t)(r + 1) * kMaxDepth;
                const int dn = readlane_i(d_v, j + 1);
                if (lane >= 1 && lane <= dn) gp0 = gp[lane];
                if (64 + lane <= dn) gp1 = gp[64 + lane];
                const float* pr = E.policy + (size_t)(r + 1) * 65;
                pol_l = pr[lane];
            }
            const bool already = __ballot(expanded_here && leaf_v == leaf) != 0;
            TS_T(te0);
            if (lk.player != 0 && lk.n_children == 0 && !already) {
                Pos P;
                P.player = lk.player;
                P.pad_ = 0;
                P.p1 = readlane_u64(pos_v.p1, j);
                P.p2 = readlane_u64(pos_v.p2, j);
                P.legal = readlane_u64(pos_v.legal, j);
                P.next_legal = readlane_u64(pos_v.next_legal, j);
                const int nc = P.legal ? popcount64(P.legal) : 1;
                if ((int64_t)count + nc > E.cap) {
                    overflow = true;  // leaf stays a leaf; value still backed up
                } else {
                    const int fc = count;
                    count += nc;
                    ++expansions;
                    if (P.legal) {
                        expand_quads(E, base, leaf, P, fc, nc, t, polj);
                    } else if (lane == 0) {  // the pass: one child (position.h:382-386)
                        const Pos c = apply_action(P, 64);
                        store_link(E.link + base + fc, NodeLink{-1, 0, leaf, c.player});
                        store_stat(E.stat + base + fc, NodeStat{0, 0.0f, 0.0f, E.policy[(size_t)r * 65 + 64]});
                        store_pos(E.pos + base + fc, c);
                    }
                    if (lane == 0) store_link(E.link + base + leaf, NodeLink{fc, nc, lk.parent, lk.player});
                    if (lane == j) expanded_here = true;
                }
            }
            TS_T(te1);
            TS_ADD(kTsExpand, te1 - te0);
            if (d > 0) {
                float v;
                if (lk.player != 0) {
                    v = -readlane_f(val_v, j);
                } else {
                    // terminal: score from the perspective of the parent's player
                    const NodeLink pl = load_link(E.link + base + lk.parent);
                    const uint64_t lp1 = readlane_u64(pos_v.p1, j);
                    const uint64_t lp2 = readlane_u64(pos_v.p2, j);
                    const uint64_t mine = pl.player == 1 ? lp1 : lp2;
                    const uint64_t theirs = pl.player == 1 ? lp2 : lp1;
                    const int a = popcount64(mine), b = popcount64(theirs);
                    v = a > b ? 1.0f : (a < b ? -1.0f : 0.0f);
                }
                // node at depth k receives v * (-1)^(d-k)  (sign flips walking up)
                if (lane >= 1 && lane <= d) {
                    const float vk = ((d - lane) & 1) ? -v : v;
                    NodeStat s = load_stat(E.stat + base + path0);
                    s.w += 1.0f + vk;
                    s.q = s.w / (float)s.n;
                    store_stat(E.stat + base + path0, s);
                }
                if (64 + lane <= d) {
                    const int k = 64 + lane;
                    const float vk = ((d - k) & 1) ? -v : v;
                    NodeStat s = load_stat(E.stat + base + path1);
                    s.w += 1.0f + vk;
                    s.q = s.w / (float)s.n;
                    store_stat(E.stat + base + path1, s);
                }
            }
            wave_order();  // the next leaf's backup reads these statistics
            TS_T(tw1);
            TS_ADD(kTsPathW, tw1 - te1);
        }
    }
    TS_T(tb1);
    TS_ADD(kTsBackup, tb1 - tb0);
}

// ---------------------------------------------------------------------------
// One round of the search schedule for every game (one wave per game).
//
// The reference runs T threads, each looping lock{select B leaves} -> NN ->
// lock{expand + backup B leaves}, with the calling thread serving NN requests
// FIFO (search_thread.cpp:47-128, mcts.h:220-256). The interleaving it
// produces (measured on the compiled reference, DESIGN.md "Search semantics")
// is a pipelined round-robin: after every thread selected its first batch,
// thread t backs up batch k and immediately selects batch k+1, then thread
// t+1 does the same. Round k of this kernel is therefore, for t = 0..T-1:
//     backup(thread t, batch k-1)   [do_backup]
//     select(thread t, batch k)     [do_select]
// Thread t's rows are consumed by its backup before its selection rewrites
// them. With T = 1 this is exactly the reference's sequential loop. Calling
// with do_backup only after every select gives the lock-step order instead.
// ---------------------------------------------------------------------------
// Capped at 96 VGPRs (amdgpu_num_vgpr counts the unified VGPR+AGPR file in
// units of 2 on gfx950) so that a tree wave fits beside the two 208-VGPR
// k_resnet_w8 waves of every SIMD (512 VGPRs): one pipeline group's tree round
// runs on the CUs that the other group's ResNet launch occupies. The cap costs
// 56 bytes per lane of spills (60 in k_tree_free); launches of at most
// kWideTreeGames games run k_tree_wide, the same round uncapped (114 VGPRs).
// Evaluation list (cnt_add != nullptr, the native search): the rows of
// non-terminal leaves this round selects are appended to E.rowlist[g0 * L ..]
// behind the counter *cnt_add; *cnt_reset (the counter of the next round,
// which no launch still reads) is zeroed by the group's first wave.
// Chain splitting (budget > 0, the native search): a thread whose batches
// come back all terminal selects again at once (the reference's order), and
// such a chain can run to the end of the thread's search inside one round,
// holding its pipeline group's NN launch. After `budget` re-selections in a
// round the game stops (at most `max_cuts` times per search) and its next
// round resumes exactly there, visiting the threads cyclically from that
// thread: every game still performs the same operations in the same order,
// only the round boundaries move. Each cut delays the game's remaining visits
// by at most one round, so the host runs max_cuts extra rounds. budget = 0:
// rounds always start at thread 0 (the step API and the single-game split).
// Per-wave work counters of one k_tree launch.
struct RoundAcc {
    unsigned long long sims = 0, evals = 0, depth_sum = 0;
    unsigned long long scan_sum = 0;  // children scanned over every descent level
    int depth_max = 0;
    unsigned expansions = 0;          // leaves expanded (children = the node count's growth)
};

// One round of game g's search schedule (see k_tree): virtual threads
// [t0, t1) visited cyclically from rp, each backing up its pending batch and
// selecting its next ones (chain splitting after `budget` re-selections, at
// most `max_cuts` cuts per search; cut_at = the thread whose chain stopped).
// Returns true when the search is complete after this round: every thread
// selected its `steps` batches and none waits for the NN (the reference's
// search has returned, mcts.h:252-255).
__device__ __forceinline__ bool search_round(const EngineView& E, int g, GameState* gs, size_t base, int t0,
                                             int t1, int B, bool do_backup, bool do_select, bool fresh, int rp,
                                             int budget, int max_cuts, int& cuts, bool& over, int& cut_at,
                                             uint64_t& event, int hist_node, int hist_n, int& count,
                                             bool& overflow, int* cnt_add, int list_base, RoundAcc& acc) {
    const int lane = lane_id();
    const int nt = t1 - t0;
    int chain = 0;  // re-selections after all-terminal batches in this round
    bool done = true;
    // a search's first round starts every thread fresh, also the ones a split
    // chain keeps it from visiting (their state is read from the next round on)
    // (strided: a search may run up to 1024 virtual threads)
    if (fresh && budget > 0)
        for (int t = t0 + lane; t < t1; t += 64) E.tstate[(size_t)g * E.L + t] = 0;
    for (int k = 0; k < nt && cut_at < 0; ++k) {
        const int t = t0 + (rp - t0 + k) % nt;
        // virtual thread t: batches selected so far in this search, and whether
        // its last batch waits for the NN (a search's first round starts fresh)
        int* ts = E.tstate + (size_t)g * E.L + t;
        const int st = fresh ? 0 : *ts;
        int sel = st & kTstateSel;
        bool pend = (st & kTstatePend) != 0;
        if (do_backup && pend) {
            backup_range(E, g, base, t * B, (t + 1) * B, count, overflow, acc.expansions);
            pend = false;
        }
        // the thread's next batch; one whose leaves are all terminal needs no NN
        // round trip (search_thread.cpp:102) and is backed up at once (:116-127),
        // then the thread selects again, up to `steps` batches per search
        bool again = false;  // the last batch was all terminal and is backed up
        while (do_select && !pend && sel < E.steps) {
            if (again && budget > 0 && chain >= budget) {
                if (cuts < max_cuts) {
                    cut_at = t;  // the next round continues this chain
                    ++cuts;
                    break;
                }
                over = true;  // no cut left: the chain runs on in this round
            }
            const unsigned long long ev0 = acc.evals;
            TS_T(tsel0);
            select_range(E, g, gs, base, t * B, (t + 1) * B, event, hist_node, hist_n, acc.sims, acc.evals, cnt_add,
                         list_base, acc.depth_sum, acc.depth_max, acc.scan_sum);
            TS_T(tsel1);
            TS_ADD(kTsSelect, tsel1 - tsel0);
            TS_ADD(kTsBatches, 1);
            ++sel;
            if (acc.evals != ev0 || !E.terminal_skip) {
                pend = true;
            } else {
                backup_range(E, g, base, t * B, (t + 1) * B, count, overflow, acc.expansions);
                again = true;
                ++chain;
#if OAMD_CHAIN_PRIO > 0
                // an all-terminal chain holds its pipeline group's round (and so
                // its NN launch): from its first re-selection on, this wave
                // issues ahead of the other group's ResNet waves (priority 1)
                if (chain == 1) __builtin_amdgcn_s_setprio(OAMD_CHAIN_PRIO);
#endif
            }
        }
        if (lane == 0) *ts = sel | (pend ? kTstatePend : 0);
        done = done && sel >= E.steps && !pend;
    }
    return done && cut_at < 0;
}

// The wave's work counters (lane 0): [0..1] this search (reset when a caller
// asks for them), [2..3] cumulative since the engine was created
// (oamd_engine_work_counters), [4..5] the searches that record timing events,
// [6] descent depths summed over every selected leaf, [7] the deepest descent
// (levels below the root; oamd_engine_descent_depths), and the tree kernels'
// algorithmic work (oamd_engine_tree_work): [8] children scanned over every
// descent level, [9] expansions, [10] children created, [11] tree launches
// (lane 0 of each launch's first wave). children: the game's node count
// growth this round (count_grown, no restart in between).
__device__ __forceinline__ void add_counters(const EngineView& E, const RoundAcc& acc, bool timed,
                                             unsigned children) {
    if (!E.counters) return;
    if (acc.sims) {
        atomicAdd(E.counters + 0, acc.sims);
        atomicAdd(E.counters + 1, acc.evals);
        atomicAdd(E.counters + 2, acc.sims);
        atomicAdd(E.counters + 3, acc.evals);
        if (timed) {
            atomicAdd(E.counters + 4, acc.sims);
            atomicAdd(E.counters + 5, acc.evals);
        }
        atomicAdd(E.counters + 6, acc.depth_sum);
        atomicMax(E.counters + 7, (unsigned long long)acc.depth_max);
        atomicAdd(E.counters + 8, acc.scan_sum);
    }
    if (acc.expansions) {
        atomicAdd(E.counters + 9, (unsigned long long)acc.expansions);
        atomicAdd(E.counters + 10, (unsigned long long)children);
    }
}

// counter [11]: one per tree launch (lane 0 of its first wave, before any
// early return of an inactive game)
__device__ __forceinline__ void count_launch(const EngineView& E) {
    if (E.counters && blockIdx.x == 0 && lane_id() == 0) atomicAdd(E.counters + 11, 1ULL);
}

__device__ __forceinline__ void tree_round_kernel(const EngineView& E, int g0, int do_backup, int do_select, int t0,
                                                  int t1, int B, int* cnt_add, int* cnt_reset, int fresh, int budget,
                                                  int max_cuts, int timed, int* cuts_out) {
    const int g = g0 + (int)blockIdx.x;
    const int lane = lane_id();
    if (cnt_reset && blockIdx.x == 0 && lane == 0) *cnt_reset = 0;
    count_launch(E);
    // cuts_out (adaptive extra rounds, capi.hip): [0] the most cuts any game
    // of the launch's group used in this search, [1] the fewest empty squares
    // of an active game's root; reset by the search's first round, set by its
    // final (backup-only) round
    if (cuts_out && fresh && blockIdx.x == 0 && lane == 0) {
        cuts_out[0] = 0;
        cuts_out[1] = 64;
    }
#ifdef OAMD_TREE_STAMPS
    if (lane < kTsCount) ts_acc[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    TS_T(tk0);
#endif
    GameState* gs = E.games + g;
    const size_t base = (size_t)g * E.cap;
    const int flags = gs->flags;
    if (!(flags & kActive)) {
        if (do_select) {
            for (int i = t0 * B; i < t1 * B; ++i) {
                const int r = g * E.L + i;
                if (lane == 0) {
                    E.leaf[r] = -1;
                    E.depth[r] = 0;
                    E.trans[r] = 0;
                }
                write_feature_meta(E, r, 1, 0, false);
            }
        }
        return;
    }
    uint64_t event = gs->event;
    const int hist_n = gs->hist_n;
    const int hist_node = lane < 16 ? gs->hist[lane] : -1;
    RoundAcc acc;
    int count = gs->count;
    const int count0 = count;
    bool overflow = false;
    const int rp = budget > 0 && !fresh ? gs->resume : t0;  // this round's first thread
    int cuts = budget > 0 && !fresh ? gs->cuts : 0;
    bool over = false;  // a chain went past the budget with every cut used
    int cut_at = -1;    // the thread whose chain this round stopped
    search_round(E, g, gs, base, t0, t1, B, do_backup != 0, do_select != 0, fresh != 0, rp, budget, max_cuts, cuts,
                 over, cut_at, event, hist_node, hist_n, count, overflow, cnt_add, g0 * E.L, acc);
    if (lane == 0) {
        if (budget > 0) {
            gs->resume = cut_at >= 0 ? cut_at : rp;
            // a search that ran out of cuts reports max_cuts + 1 (cuts_out)
            gs->cuts = over ? max_cuts + 1 : cuts;
        }
        if (cuts_out && !do_select) {
            const NodePos& rp = E.pos[base + gs->root];
            atomicMax(cuts_out, cuts);
            atomicMin(cuts_out + 1, 64 - __popcll(rp.p1 | rp.p2));
        }
        gs->event = event;
        gs->count = count;
        // atomic like select_range's kDepthCap: a plain read-modify-write of
        // the flags read at kernel start could drop that bit
        if (overflow) atomicOr(&gs->flags, (int)kOverflow);
#ifdef OAMD_TREE_STAMPS
        {
            TS_T(tk1);
            ts_acc[kTsWaves] = 1;
            ts_acc[kTsCycles] = tk1 - tk0;
            for (int i = 0; i < kTsCount; ++i) {
                if (i == kTsMaxCycles) atomicMax(&g_tree_stamps[i], tk1 - tk0);
                else atomicAdd(&g_tree_stamps[i], ts_acc[i]);
            }
        }
#endif
        add_counters(E, acc, timed != 0, (unsigned)(count - count0));
    }
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(48))) void k_tree(EngineView E, int g0, int do_backup,
                                                                                int do_select, int t0, int t1, int B,
                                                                                int* cnt_add, int* cnt_reset, int fresh,
                                                                                int budget, int max_cuts, int timed,
                                                                                int* cuts_out) {
    tree_round_kernel(E, g0, do_backup, do_select, t0, t1, B, cnt_add, cnt_reset, fresh, budget, max_cuts, timed,
                      cuts_out);
}

// The same round without the register cap (114 VGPRs, no spills) for launches
// of at most kWideTreeGames games (the single-game drop-in MCTS and other
// small engines): their NN launches leave most CUs free, so a tree wave needs
// no room beside ResNet waves, and its leaves' serial chain is the search's
// critical path.
constexpr int kWideTreeGames = 16;
__global__ __launch_bounds__(64) void k_tree_wide(EngineView E, int g0, int do_backup, int do_select, int t0, int t1,
                                                  int B, int* cnt_add, int* cnt_reset, int fresh, int budget,
                                                  int max_cuts, int timed, int* cuts_out) {
    tree_round_kernel(E, g0, do_backup, do_select, t0, t1, B, cnt_add, cnt_reset, fresh, budget, max_cuts, timed,
                      cuts_out);
}

// ---------------------------------------------------------------------------
// Packed -> fp32 features (B, 1+2H, 8, 8) for the external-evaluator path.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float plane_value(const uint64_t* row, int c, int sq_src) {
    if (c == 0) return (float)(row[0] & 1ULL);
    const uint64_t bb = row[1 + c];  // c = 1 + 2h -> word 2 + 2h; c = 2 + 2h -> 3 + 2h
    return (float)((bb >> (63 - sq_src)) & 1ULL);
}

__global__ __launch_bounds__(256) void k_features_f32(EngineView E, float* out, int row_begin,
                                                      int rows) {
    const int rr = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (rr >= rows) return;
    const int p = threadIdx.x & 63;
    const uint64_t* row = E.feat + (size_t)(row_begin + rr) * E.FW;
    const uint64_t meta = row[0];
    const bool valid = (meta >> 16) & 1ULL;
    const int t = (int)((meta >> 8) & 7ULL);
    const int src = inverse_transform(p, t);
    const int C = 1 + 2 * E.H;
    float* o = out + (size_t)rr * C * 64;
    for (int c = 0; c < C; ++c) o[c * 64 + p] = valid ? plane_value(row, c, src) : 0.0f;
}

__global__ __launch_bounds__(256) void k_set_evaluation(EngineView E, const float* policy,
                                                        const float* value, int row_begin,
                                                        int rows) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx < rows * 65) E.policy[(size_t)row_begin * 65 + idx] = policy[idx];
    if (idx < rows) E.value[row_begin + idx] = value[idx];
}

// 1 = the row is a non-terminal leaf of a batch that waits for the NN this
// round (a thread that ran out of batches, or whose last batch was all
// terminal, has none: its rows are stale)
__global__ __launch_bounds__(256) void k_leaf_flags(EngineView E, uint8_t* flags) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= E.G * E.L) return;
    const int g = r / E.L, t = (r % E.L) / E.B;
    const bool pend = (E.tstate[(size_t)g * E.L + t] & kTstatePend) != 0;
    flags[r] = (uint8_t)(pend && ((E.feat[(size_t)r * E.FW] >> 16) & 1ULL));
}

// ---------------------------------------------------------------------------
// Game state: reset, moves, root statistics, self-play targets
// ---------------------------------------------------------------------------
__device__ void init_game(const EngineView& E, int g, uint64_t seed) {
    GameState* gs = E.games + g;
    const size_t base = (size_t)g * E.cap;
    const Pos p = initial_position();
    store_link(E.link + base, NodeLink{-1, 0, -1, p.player});
    store_stat(E.stat + base, NodeStat{0, 0.0f, 0.0f, 1.0f});
    store_pos(E.pos + base, p);
    gs->root = 0;
    gs->count = 1;
    gs->flags = kActive;
    gs->hist_n = 0;
    gs->key = mix64(seed ^ mix64((uint64_t)g + 0x632BE59BD9B4E019ULL));
    gs->event = 0;
    gs->ply = 0;
    for (int k = 0; k < 16; ++k) gs->hist[k] = -1;
}

__global__ void k_reset(EngineView E, int game, uint64_t seed) {
    const int g = game >= 0 ? game : (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (g >= E.G || (game >= 0 && threadIdx.x + blockIdx.x != 0)) return;
    init_game(E, g, seed);
}

// Move the root of game g along `action` (mcts.cpp:114-165): into the existing
// child when the root is expanded, else into a fresh node. History = parents.
__device__ void move_root(const EngineView& E, int g, int action) {
    GameState* gs = E.games + g;
    const size_t base = (size_t)g * E.cap;
    const int root = gs->root;
    const NodeLink lk = load_link(E.link + base + root);
    int next;
    if (lk.n_children == 0) {
        if ((int64_t)gs->count + 1 > E.cap) {
            gs->flags |= kOverflow;
            return;
        }
        next = gs->count++;
        const Pos p = load_pos(E.pos + base + root, lk.player);
        const Pos c = apply_action(p, action);
        store_link(E.link + base + next, NodeLink{-1, 0, root, c.player});
        store_stat(E.stat + base + next, NodeStat{0, 0.0f, 0.0f, 1.0f});
        store_pos(E.pos + base + next, c);
    } else {
        const uint64_t legal = E.pos[base + root].legal;
        next = lk.first_child + child_index_of(legal, lk.n_children, action);
    }
    for (int k = 15; k > 0; --k) gs->hist[k] = gs->hist[k - 1];
    gs->hist[0] = root;
    gs->hist_n = gs->hist_n < 16 ? gs->hist_n + 1 : 16;
    gs->root = next;
    gs->ply += 1;
}

__global__ void k_apply_actions(EngineView E, const int32_t* actions) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= E.G) return;
    const int a = actions[g];
    if (a < 0 || !(E.games[g].flags & kActive)) return;
    move_root(E, g, a);
}

__global__ void k_apply_one(EngineView E, int g, int action) { move_root(E, g, action); }

// Root summary per game: info + visits/q indexed by action.
__global__ __launch_bounds__(64) void k_root_stats(EngineView E, int game_begin,
                                                   oamd_root_info* info, int32_t* visits,
                                                   float* q, int by_action) {
    const int g = game_begin + blockIdx.x;
    const int lane = lane_id();
    const GameState* gs = E.games + g;
    const size_t base = (size_t)g * E.cap;
    const int root = gs->root;
    const NodeLink lk = load_link(E.link + base + root);
    const NodePos rp = E.pos[base + root];
    const int nc = lk.n_children;
    int32_t* vo = visits + (size_t)blockIdx.x * 65;
    float* qo = q + (size_t)blockIdx.x * 65;
    if (by_action) {
        // lane = square; pass in slot 64
        vo[lane] = 0;
        qo[lane] = 0.0f;
        if (lane == 0) {
            vo[64] = 0;
            qo[64] = 0.0f;
        }
        __builtin_amdgcn_wave_barrier();
        if (nc > 0) {
            if (rp.legal) {
                if ((rp.legal >> (63 - lane)) & 1ULL) {
                    const int j = child_index_of(rp.legal, nc, lane);
                    const NodeStat s = load_stat(E.stat + base + lk.first_child + j);
                    vo[lane] = s.n;
                    qo[lane] = s.q;
                }
            } else if (lane == 0) {
                const NodeStat s = load_stat(E.stat + base + lk.first_child);
                vo[64] = s.n;
                qo[64] = s.q;
            }
        }
    } else if (lane < nc) {
        const NodeStat s = load_stat(E.stat + base + lk.first_child + lane);
        vo[lane] = s.n;
        qo[lane] = s.q;
    }
    if (lane == 0) {
        oamd_root_info& I = info[blockIdx.x];
        I.position.player = lk.player;
        I.position.reserved = 0;
        I.position.player1_discs = rp.p1;
        I.position.player2_discs = rp.p2;
        I.position.legal_moves = rp.legal;
        I.position.next_legal_moves = rp.next_legal;
        I.num_children = nc;
        I.visit_count = E.stat[base + root].n;
        I.overflow = (gs->flags & (kOverflow | kDepthCap)) ? gs->flags : 0;
        I.reserved = 0;
        I.node_count = gs->count;
    }
}

// 8-fold self-play targets of the root (mcts.cpp:63-112): features of the root
// under transform t (wave t of the block) and policy[transform(a,t)] = N_a/sum.
__device__ void write_targets(const EngineView& E, int g, int t, float* feat_out, float* pol_out) {
    const int lane = lane_id();
    const GameState* gs = E.games + g;
    const size_t base = (size_t)g * E.cap;
    const int root = gs->root;
    const NodeLink lk = load_link(E.link + base + root);
    const NodePos rp = E.pos[base + root];
    const int C = 1 + 2 * E.H;
    float* fo = feat_out + (size_t)t * C * 64;
    const int src = inverse_transform(lane, t);
    fo[lane] = (float)(lk.player - 1);
    for (int h = 0; h < E.H; ++h) {
        int node = -1;
        if (h == 0) node = root;
        else if (h - 1 < gs->hist_n) node = gs->hist[h - 1];
        float b = 0.0f, w = 0.0f;
        if (node >= 0) {
            const NodePos np = E.pos[base + node];
            b = (float)((np.p1 >> (63 - src)) & 1ULL);
            w = (float)((np.p2 >> (63 - src)) & 1ULL);
        }
        fo[(1 + 2 * h) * 64 + lane] = b;
        fo[(2 + 2 * h) * 64 + lane] = w;
    }
    float* po = pol_out + (size_t)t * 65;
    const int nc = lk.n_children;
    int n = 0;
    if (lane < nc) n = E.stat[base + lk.first_child + lane].n;
    int sum = wave_sum(n);
    if (sum == 0) sum = 1;
    po[lane] = 0.0f;
    if (lane == 0) po[64] = 0.0f;
    __builtin_amdgcn_wave_barrier();
    if (nc > 0) {
        if (rp.legal) {
            const int s = lane;
            const bool set = (rp.legal >> (63 - s)) & 1ULL;
            const int j = s == 0 ? 0 : popcount64(rp.legal & (~0ULL << (64 - s)));
            const int nj = __shfl(n, j & 63);
            if (set) po[transform_action(s, t)] = (float)nj / (float)sum;
        } else if (lane == 0) {
            po[64] = (float)n / (float)sum;
        }
    }
}

__global__ __launch_bounds__(512) void k_self_play_data(EngineView E, int g, float* feat_out,
                                                        float* pol_out) {
    write_targets(E, g, threadIdx.x >> 6, feat_out, pol_out);
}

// ---------------------------------------------------------------------------
// On-device self-play move (train.py:404-452): choose, emit targets, apply,
// restart finished games from a random opening.
// ---------------------------------------------------------------------------
__device__ void random_opening(const EngineView& E, int g, int max_moves) {
    // lane-0 sequential: k ~ U{0..max_moves} uniformly random legal plies
    GameState* gs = E.games + g;
    if (max_moves <= 0) return;
    const uint64_t ev = gs->event++;
    const uint64_t key = stream_key(gs->key, ev, 0);
    const int k = (int)(mix64(key) % (uint64_t)(max_moves + 1));
    for (int m = 0; m < k; ++m) {
        const size_t base = (size_t)g * E.cap;
        const int root = gs->root;
        const NodeLink lk = load_link(E.link + base + root);
        if (lk.player == 0) break;
        const NodePos rp = E.pos[base + root];
        const int na = rp.legal ? popcount64(rp.legal) : 1;
        const int pick = (int)(mix64(key + (uint64_t)(m + 1) * kGolden) % (uint64_t)na);
        int action = 64;
        if (rp.legal) {
            uint64_t rem = rp.legal;
            for (int s = 0, c = 0; s < 64; ++s) {
                if ((rem >> (63 - s)) & 1ULL) {
                    if (c == pick) {
                        action = s;
                        break;
                    }
                    ++c;
                }
            }
        }
        move_root(E, g, action);
    }
    gs->ply = 0;
}

__global__ void k_random_openings(EngineView E, int max_moves, uint64_t seed) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= E.G) return;
    init_game(E, g, seed);
    random_opening(E, g, max_moves);
}

constexpr int kFinNoTargets = 4, kFinOverflow = 8;

// One self-play move of game g (one wave): outputs at index g of the given
// per-move slices.
__device__ __forceinline__ void selfplay_move_game(const EngineView& E, const SelfplayParams& sp, int g,
                                                   int32_t* actions, int32_t* finished, float* feat_out,
                                                   float* pol_out) {
    const int lane = lane_id();
    GameState* gs = E.games + g;
    const size_t base = (size_t)g * E.cap;
    const int root = gs->root;
    const NodeLink lk = load_link(E.link + base + root);
    const NodePos rp = E.pos[base + root];
    const int nc = lk.n_children;
    // status bits reported with `finished` (selfplay.py): the root had no
    // searched children, so no targets were written (the reference's
    // self_play_data raises, mcts.cpp:69-71); the game's node pool overflowed
    const int status = (lk.player != 0 && nc == 0 ? kFinNoTargets : 0) |
                       (gs->flags & kOverflow ? kFinOverflow : 0);
    int action = -1;
    if (lk.player != 0) {
        const int na = rp.legal ? popcount64(rp.legal) : 1;
        int n = 0;
        if (lane < nc) n = E.stat[base + lk.first_child + lane].n;
        const uint64_t ev = gs->event;
        const float u = uniform(stream_key(gs->key, ev, 0), 0);
        int j = 0;
        if (nc == 0) {
            j = (int)(u * (float)na);  // unexpanded root: uniform over legal actions
            if (j >= na) j = na - 1;
        } else if (gs->ply < sp.temperature_moves) {
            // p ~ N^(1/temperature) (train.py:423-426); cdf search like numpy.random.choice
            const float w = lane < nc ? powf((float)n, 1.0f / sp.temperature) : 0.0f;
            float sum = 0.0f;
            float cdf = 0.0f;
            for (int k = 0; k < nc; ++k) {
                sum += readlane_f(w, k);
                if (k == lane) cdf = sum;
            }
            if (sum > 0.0f) {
                const float target = u * sum;
                const bool above = lane < nc && cdf > target;
                const uint64_t b = __ballot(above);
                j = b ? __ffsll((unsigned long long)b) - 1 : nc - 1;
            } else {
                j = (int)(u * (float)nc);
                if (j >= nc) j = nc - 1;
            }
        } else {
            // argmax with uniform random tie-break (train.py:428-430)
            int m = n;
            m = wave_max_i(m);
            const uint64_t ties = __ballot(lane < nc && n == m);
            const int nt = popcount64(ties);
            int k = (int)(u * (float)nt);
            if (k >= nt) k = nt - 1;
            uint64_t rem = ties;
            for (int x = 0; x < k; ++x) rem &= rem - 1;
            j = __ffsll((unsigned long long)rem) - 1;
        }
        action = action_of_child(rp.legal, j);
        if (sp.emit_targets && feat_out && nc > 0) {
            const int C = 1 + 2 * E.H;
            for (int t = 0; t < 8; ++t)
                write_targets(E, g, t, feat_out + (size_t)g * 8 * C * 64, pol_out + (size_t)g * 8 * 65);
        }
        if (lane == 0) {
            gs->event = ev + 1;
            move_root(E, g, action);
        }
    }
    __builtin_amdgcn_wave_barrier();
    wait_stores();
    int fin = 0;
    if (lane == 0) {
        const int r2 = gs->root;
        const NodeLink l2 = load_link(E.link + base + r2);
        if (l2.player == 0) {
            const NodePos p2 = E.pos[base + r2];
            const int b = popcount64(p2.p1), w = popcount64(p2.p2);
            fin = b > w ? 2 : (b < w ? 3 : 1);  // 1 draw, 2 black won, 3 white won
            const uint64_t key = gs->key;
            const uint64_t ev = gs->event;
            init_game(E, g, key ^ mix64(ev + 0xA5A5A5A5ULL));
            random_opening(E, g, sp.opening_moves);
        }
        if (actions) actions[g] = action;
        if (finished) finished[g] = fin | status;
    }
}

__global__ __launch_bounds__(64) void k_selfplay_move(EngineView E, SelfplayParams sp, int g0,
                                                      int32_t* actions, int32_t* finished,
                                                      float* feat_out, float* pol_out) {
    const int g = g0 + (int)blockIdx.x;
    const int lane = lane_id();
    GameState* gs = E.games + g;
    if (!(gs->flags & kActive)) {
        if (lane == 0) {
            if (actions) actions[g] = -1;
            if (finished) finished[g] = 0;
        }
        return;
    }
    selfplay_move_game(E, sp, g, actions, finished, feat_out, pol_out);
}

// ---------------------------------------------------------------------------
// Free-running self-play (oamd_engine_selfplay_steps, capi.hip): every game
// plays `n_moves` moves on its own; a round of this kernel is, per game, one
// round of its current search (search_round) and, in the round that completes
// the search, the move (selfplay_move_game: choice, 8-fold targets, apply,
// restart) and the first round of its next search. Per game the operations
// and their order are exactly those of n x (search + selfplay_move): the
// rounds of one search, then its move, then the next search's rounds (a chain
// cut only moves a round boundary, see k_tree). But no game waits for the
// others at a move: a game whose search needs more rounds (chains near its
// end) lags by those rounds while the others go on, so the group's ResNet
// launches stay full and no extra rounds are needed. The host enqueues rounds
// until `remaining` (games of the group with moves left) reads 0.
// ---------------------------------------------------------------------------
__global__ void k_free_begin(EngineView E, int g0, int ng, int n_moves, int32_t* remaining, int32_t* actions,
                             int32_t* finished, int per_move) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // *remaining zeroed by the caller
    if (i >= ng) return;
    const int g = g0 + i;
    GameState* gs = E.games + g;
    const bool active = (gs->flags & kActive) != 0 && n_moves > 0;
    gs->moves_left = active ? n_moves : 0;
    gs->fresh = 1;
    if (active) atomicAdd(remaining, 1);
    for (int m = 0; !active && m < (per_move ? n_moves : (n_moves > 0 ? 1 : 0)); ++m) {
        if (actions) actions[(size_t)m * E.G + g] = -1;
        if (finished) finished[(size_t)m * E.G + g] = 0;
    }
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(48))) void k_tree_free(
    EngineView E, int g0, int B, int* cnt_add, int* cnt_reset, int budget, int timed, SelfplayParams sp, int n_moves,
    int per_move, int32_t* actions, int32_t* finished, float* feat_out, float* pol_out, int32_t* remaining) {
    const int g = g0 + (int)blockIdx.x;
    const int lane = lane_id();
    if (cnt_reset && blockIdx.x == 0 && lane == 0) *cnt_reset = 0;
    count_launch(E);
    GameState* gs = E.games + g;
    const size_t base = (size_t)g * E.cap;
    int moves = gs->moves_left;
    if (moves <= 0) return;
    const int T = E.L / B;
    const bool fresh = gs->fresh != 0;
    uint64_t event = gs->event;
    int hist_n = gs->hist_n;
    int hist_node = lane < 16 ? gs->hist[lane] : -1;
    int count = gs->count;
    unsigned grown = 0;  // children created (the node count restarts with a finished game)
    int count0 = count;
    bool overflow = false;
    RoundAcc acc;
    int rp = fresh || budget <= 0 ? 0 : gs->resume;
    int cuts = fresh ? 0 : gs->cuts;
    bool over = false;
    int cut_at = -1;
    // no extra rounds to budget for: a game may cut its chains any number of times
    constexpr int kNoCap = 0x3FFFFFFF;
    const bool done = search_round(E, g, gs, base, 0, T, B, true, true, fresh, rp, budget, kNoCap, cuts, over, cut_at,
                                   event, hist_node, hist_n, count, overflow, cnt_add, g0 * E.L, acc);
    if (done) {
        // the search has returned: publish the wave's state, then the move
        // (k_selfplay_move's), which reads it from memory
        if (lane == 0) {
            gs->event = event;
            gs->count = count;
            if (overflow) atomicOr(&gs->flags, (int)kOverflow);
        }
        overflow = false;
        grown += (unsigned)(count - count0);
        __builtin_amdgcn_wave_barrier();
        wait_stores();
        const size_t slot = per_move ? (size_t)(n_moves - moves) * E.G : 0;
        const size_t C = 1 + 2 * (size_t)E.H;
        selfplay_move_game(E, sp, g, actions ? actions + slot : nullptr, finished ? finished + slot : nullptr,
                           feat_out ? feat_out + slot * 8 * C * 64 : nullptr, pol_out ? pol_out + slot * 8 * 65 : nullptr);
        --moves;
        __builtin_amdgcn_wave_barrier();
        wait_stores();  // (a compiler barrier too: the reloads below see the move's stores)
        event = gs->event;
        hist_n = gs->hist_n;
        hist_node = lane < 16 ? gs->hist[lane] : -1;
        count = gs->count;
        count0 = count;
        rp = 0;
        cuts = 0;
        cut_at = -1;
        if (moves > 0)  // the next search's first round, in this same round
            search_round(E, g, gs, base, 0, T, B, true, true, true, 0, budget, kNoCap, cuts, over, cut_at, event,
                         hist_node, hist_n, count, overflow, cnt_add, g0 * E.L, acc);
    }
    if (lane == 0) {
        gs->moves_left = moves;
        gs->fresh = 0;
        gs->resume = cut_at >= 0 ? cut_at : rp;
        gs->cuts = cuts;
        gs->event = event;
        gs->count = count;
        if (overflow) atomicOr(&gs->flags, (int)kOverflow);
        if (moves == 0 && remaining) atomicSub(remaining, 1);
        add_counters(E, acc, timed != 0, grown + (unsigned)(count - count0));
    }
}

// Games whose node pool overflowed / whose descent hit the depth cap (sticky
// flags since the game's last reset).
__global__ void k_status(EngineView E, int32_t* out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= E.G) return;
    const int f = E.games[g].flags;
    if (f & kOverflow) atomicAdd(out + 0, 1);
    if (f & kDepthCap) atomicAdd(out + 1, 1);
}

// ---------------------------------------------------------------------------
// Batched bitboards (position.h) — elementwise, one position per lane.
// ---------------------------------------------------------------------------
__global__ void k_legal_moves(const uint64_t* me, const uint64_t* opp, uint64_t* out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = legal_moves(me[i], opp[i]);
}

__global__ void k_flips(const uint64_t* mv, const uint64_t* me, const uint64_t* opp, uint64_t* out,
                        int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = flips(mv[i], me[i], opp[i]);
}

__global__ void k_apply_positions(const Pos* in, const int32_t* actions, Pos* out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = apply_action(in[i], actions[i]);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static inline unsigned blocks_for(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

void launch_tree(const EngineView& E, hipStream_t s, bool do_backup, bool do_select, int T, int B,
                 int g0, int ng, int t0, int t1, int* cnt_add, int* cnt_reset, bool fresh, int budget,
                 int max_cuts, bool timed, int* cuts_out) {
    if (ng < 0) ng = E.G - g0;
    if (t1 < 0) t1 = T;
    if (T * B != E.L || t0 < 0 || t1 > T || t0 >= t1) return;  // caller validated; never launch on a mismatched layout
    if (ng > 0 && (do_backup || do_select))
        hipLaunchKernelGGL(ng <= kWideTreeGames ? k_tree_wide : k_tree, dim3(ng), dim3(64), 0, s, E, g0,
                           (int)do_backup, (int)do_select, t0, t1, B, do_select ? cnt_add : nullptr, cnt_reset,
                           (int)fresh, budget, max_cuts, (int)timed, cuts_out);
}
void launch_features_f32(const EngineView& E, float* out, int row_begin, int rows, hipStream_t s) {
    if (rows > 0) hipLaunchKernelGGL(k_features_f32, dim3(blocks_for(rows, 4)), dim3(256), 0, s, E, out, row_begin, rows);
}
void launch_set_evaluation(const EngineView& E, const float* pol, const float* val, int row_begin,
                           int rows, hipStream_t s) {
    if (rows > 0)
        hipLaunchKernelGGL(k_set_evaluation, dim3(blocks_for((int64_t)rows * 65, 256)), dim3(256), 0, s, E,
                           pol, val, row_begin, rows);
}
void launch_leaf_flags(const EngineView& E, uint8_t* flags, hipStream_t s) {
    hipLaunchKernelGGL(k_leaf_flags, dim3(blocks_for((int64_t)E.G * E.L, 256)), dim3(256), 0, s, E, flags);
}
void launch_reset(const EngineView& E, int game, uint64_t seed, hipStream_t s) {
    if (game >= 0) hipLaunchKernelGGL(k_reset, dim3(1), dim3(1), 0, s, E, game, seed);
    else hipLaunchKernelGGL(k_reset, dim3(blocks_for(E.G, 64)), dim3(64), 0, s, E, -1, seed);
}
void launch_apply_actions(const EngineView& E, const int32_t* actions, hipStream_t s) {
    hipLaunchKernelGGL(k_apply_actions, dim3(blocks_for(E.G, 64)), dim3(64), 0, s, E, actions);
}
void launch_apply_one(const EngineView& E, int g, int action, hipStream_t s) {
    hipLaunchKernelGGL(k_apply_one, dim3(1), dim3(1), 0, s, E, g, action);
}
void launch_root_stats(const EngineView& E, int game_begin, int n_games, oamd_root_info* info,
                       int32_t* visits, float* q, int by_action, hipStream_t s) {
    hipLaunchKernelGGL(k_root_stats, dim3(n_games), dim3(64), 0, s, E, game_begin, info, visits, q, by_action);
}
void launch_self_play_data(const EngineView& E, int g, float* feat, float* pol, hipStream_t s) {
    hipLaunchKernelGGL(k_self_play_data, dim3(1), dim3(512), 0, s, E, g, feat, pol);
}
void launch_selfplay_move(const EngineView& E, const SelfplayParams& sp, int g0, int ng, int32_t* actions,
                          int32_t* finished, float* feat, float* pol, hipStream_t s) {
    if (ng > 0)
        hipLaunchKernelGGL(k_selfplay_move, dim3(ng), dim3(64), 0, s, E, sp, g0, actions, finished, feat, pol);
}
void launch_free_begin(const EngineView& E, int g0, int ng, int n_moves, int32_t* remaining, int32_t* actions,
                       int32_t* finished, int per_move, hipStream_t s) {
    if (ng > 0)
        hipLaunchKernelGGL(k_free_begin, dim3(blocks_for(ng, 256)), dim3(256), 0, s, E, g0, ng, n_moves, remaining,
                           actions, finished, per_move);
}
void launch_tree_free(const EngineView& E, hipStream_t s, int g0, int ng, int B, int* cnt_add, int* cnt_reset,
                      int budget, bool timed, const SelfplayParams& sp, int n_moves, int per_move, int32_t* actions,
                      int32_t* finished, float* feat, float* pol, int32_t* remaining) {
    if (ng > 0 && B > 0 && E.L % B == 0)
        hipLaunchKernelGGL(k_tree_free, dim3(ng), dim3(64), 0, s, E, g0, B, cnt_add, cnt_reset, budget, (int)timed, sp,
                           n_moves, per_move, actions, finished, feat, pol, remaining);
}
void launch_status(const EngineView& E, int32_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_status, dim3(blocks_for(E.G, 64)), dim3(64), 0, s, E, out);
}
void launch_random_openings(const EngineView& E, int max_moves, uint64_t seed, hipStream_t s) {
    hipLaunchKernelGGL(k_random_openings, dim3(blocks_for(E.G, 64)), dim3(64), 0, s, E, max_moves, seed);
}
void launch_legal_moves(const uint64_t* me, const uint64_t* opp, uint64_t* out, int64_t n, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(k_legal_moves, dim3(blocks_for(n, 256)), dim3(256), 0, s, me, opp, out, n);
}
void launch_flips(const uint64_t* mv, const uint64_t* me, const uint64_t* opp, uint64_t* out, int64_t n,
                  hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(k_flips, dim3(blocks_for(n, 256)), dim3(256), 0, s, mv, me, opp, out, n);
}
void launch_apply_positions(const Pos* in, const int32_t* actions, Pos* out, int64_t n, hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(k_apply_positions, dim3(blocks_for(n, 256)), dim3(256), 0, s, in, actions, out, n);
}

}  // namespace oamd

namespace oamd {
int tree_read_stamps(unsigned long long* out, long long n, int reset) {
#ifdef OAMD_TREE_STAMPS
    if (n > kTsCount) n = kTsCount;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tree_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[kTsCount] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tree_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess)
            return -1;
    }
    return 0;
#else
    (void)out;
    (void)n;
    (void)reset;
    return -2;
#endif
}
}  // namespace oamd
