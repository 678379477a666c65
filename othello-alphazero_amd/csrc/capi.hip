// C ABI (include/othello_mcts_amd.h): engine / net lifetime, validation with
// the reference's exception messages, host-side weight folding and packing,
// and the search step sequence. All compute is in tree.hip / resnet.hip.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/othello_mcts_amd.h"
#include "../../include/othello_mcts_amd_experimental.h"
#include "bitboard.h"

#include "engine.h"
#include "kernels.h"
#include "timing.h"

using namespace oamd;

constexpr int kMaxPipeline = 8;

// Host waits for a readback (the adaptive extra rounds' cut counts, the
// free-running call's remaining-games counters and its enqueue throttle):
// off the GPU's critical path (the reads are two chunks late), so the thread
// polls the event and sleeps 100 us between polls instead of spinning a CPU
// in hipEventSynchronize (which spins here even on blocking-sync events:
// bench.py's rank table read 1.0 CPU-s per s either way). The host budget of
// 8 ranks on one node is what it saves (cpu_s_per_s).
// OAMD_SPIN_SYNC=1: hipEventSynchronize (A/B only).
static bool spin_sync() {
    static const bool spin = [] {
        const char* v = std::getenv("OAMD_SPIN_SYNC");
        return v && v[0] == '1';
    }();
    return spin;
}
static unsigned readback_event_flags() {
    return hipEventDisableTiming | (spin_sync() ? 0u : (unsigned)hipEventBlockingSync);
}
static hipError_t host_wait(hipEvent_t ev) {
    if (spin_sync()) return hipEventSynchronize(ev);
    for (;;) {
        const hipError_t q = hipEventQuery(ev);
        if (q != hipErrorNotReady) return q;
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}
constexpr int kEvPerBlock = 4;  // timing events per (round, group): tree begin/end, NN begin/end
// device counters (k_tree): [0..1] sims / NN rows of the current search,
// [2..3] cumulative, [4..5] of timed searches, [6] summed descent depths,
// [7] deepest descent, [8..11] the tree work of oamd_engine_tree_work
// (children scanned, expansions, children created, tree launches)
constexpr int kCounters = 12;
// Order of the pipeline groups' NN launches within an NN chain (one chain:
// one after another, each owning every CU while the other groups' tree
// kernels run beside it). OAMD_NN_ORDER 1: a token event passed between the
// group streams; 2: all NN launches on one NN stream (a group's launch waits
// for its select, its backup for the launch); 0: unordered (A/B only). Kernel
// traces show the same gap between consecutive launches for 1 and 2 (~14 us,
// ~24 us with the timing events), and 1 measured 0.4 % faster in the bench.
// The default is one chain per group (2 groups, 2 chains): a group's launch
// starts as soon as its selection is done, so it fills the other launch's
// last-generation tail and the launch gap (bench +2.5-2.8 %, two boxes;
// DESIGN.md §7).
#ifndef OAMD_NN_ORDER
#define OAMD_NN_ORDER 1
#endif

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                  \
    do {                                                                              \
        hipError_t _e = (expr);                                                       \
        if (_e != hipSuccess)                                                         \
            return fail(OAMD_RUNTIME, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define LAUNCHCHK()                                                                       \
    do {                                                                                  \
        hipError_t _e = hipGetLastError();                                                \
        if (_e != hipSuccess) return fail(OAMD_RUNTIME, std::string("kernel launch: ") + hipGetErrorString(_e)); \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <typename T>
int dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) return OAMD_OK;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T));
    if (e != hipSuccess) return fail(OAMD_RUNTIME, std::string("hipMalloc: ") + hipGetErrorString(e));
    return OAMD_OK;
}

template <typename T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

std::string fstr(float v) { return std::to_string(v); }

// mcts.cpp:167-241 (messages verbatim) + the native engine's own limits
int validate_config(const oamd_search_config* c) {
    if (c->history_size < 1)
        return fail(OAMD_INVALID_ARGUMENT,
                    "Expected history_size >= 1, but got " + std::to_string(c->history_size) + ".");
    if (c->history_size > kMaxHistory)
        return fail(OAMD_INVALID_ARGUMENT, "Expected history_size <= 15 (native engine limit), but got " +
                                               std::to_string(c->history_size) + ".");
    if (c->num_simulations < 1)
        return fail(OAMD_INVALID_ARGUMENT, "Expected num_simulations >= 1, but got " +
                                               std::to_string(c->num_simulations) + ".");
    if (c->num_threads < 1)
        return fail(OAMD_INVALID_ARGUMENT,
                    "Expected num_threads >= 1, but got " + std::to_string(c->num_threads) + ".");
    if (c->batch_size < 1)
        return fail(OAMD_INVALID_ARGUMENT,
                    "Expected batch_size >= 1, but got " + std::to_string(c->batch_size) + ".");
    if ((int64_t)c->num_threads * c->batch_size > kMaxLeaves)
        return fail(OAMD_INVALID_ARGUMENT,
                    "Expected num_threads * batch_size <= 1024 (native engine limit), but got " +
                        std::to_string((int64_t)c->num_threads * c->batch_size) + ".");
    if (!(c->c_puct_base > 0.0f))
        return fail(OAMD_INVALID_ARGUMENT, "Expected c_puct_base > 0.0, but got " + fstr(c->c_puct_base) + ".");
    if (!(c->c_puct_init >= 0.0f))
        return fail(OAMD_INVALID_ARGUMENT, "Expected c_puct_init >= 0.0, but got " + fstr(c->c_puct_init) + ".");
    if (!(0.0f <= c->dirichlet_epsilon && c->dirichlet_epsilon <= 1.0f))
        return fail(OAMD_INVALID_ARGUMENT, "Expected 0.0 <= dirichlet_epsilon <= 1.0, but got " +
                                               fstr(c->dirichlet_epsilon) + ".");
    if (!(c->dirichlet_alpha >= 0.0f))
        return fail(OAMD_INVALID_ARGUMENT,
                    "Expected dirichlet_alpha >= 0.0, but got " + fstr(c->dirichlet_alpha) + ".");
    return OAMD_OK;
}

}  // namespace

// ===========================================================================
// engine
// ===========================================================================
struct oamd_engine {
    int device = 0;
    int G = 0;
    int64_t cap = 0;
    oamd_search_config cfg{};
    hipStream_t stream = nullptr;
    uint64_t seed = 0;

    NodeLink* link = nullptr;
    NodeStat* stat = nullptr;
    NodePos* pos = nullptr;
    GameState* games = nullptr;
    // per-row buffers (sized for rows_cap rows)
    int64_t rows_cap = 0;
    int fw_cap = 0;
    int32_t* leaf = nullptr;
    int32_t* depth = nullptr;
    int32_t* trans = nullptr;
    int32_t* path = nullptr;
    uint64_t* feat = nullptr;
    float* policy = nullptr;
    float* value = nullptr;
    uint8_t* flags = nullptr;
    // evaluation lists of the native search (tree.hip append_rows): the rows of
    // non-terminal leaves per pipeline group, and two counters per group (the
    // round being evaluated, the next round's)
    int32_t* rowlist = nullptr;
    int32_t* rowcount = nullptr;
    int32_t* tstate = nullptr;  // per game and virtual thread: batches selected, pending (k_tree)
    float* explore_tab = nullptr;
    unsigned long long* counters = nullptr;
    int32_t* status_dev = nullptr;  // [0] games with pool overflow, [1] depth-capped games
    // query scratch
    oamd_root_info* info_dev = nullptr;
    int32_t* visits_dev = nullptr;
    float* q_dev = nullptr;
    float* spd_dev = nullptr;  // self-play data scratch (8*(1+2H)*64 + 8*65)
    // search state
    int steps_left = 0;
    int steps_total = 0;  // of the step-wise search begun by oamd_engine_search_begin
    bool exact_interleaving = true;  // oamd_engine_set_exact_interleaving
    // native search, exact interleaving: an all-terminal chain stops after
    // chain_budget re-selections in a round, at most X <= chain_cuts times
    // per search (k_tree), X extra rounds per search (pick_extra_rounds).
    // budget 0 = never split
    int chain_budget = 2;
    int chain_cuts = 64;
    // adaptive extra rounds (pick_extra_rounds): a grouped search runs X in
    // [min(adapt_min, chain_cuts), chain_cuts] extra rounds (and allows X
    // cuts), X following the search two back. adapt_on = false: always
    // chain_cuts
    static constexpr int kCutSlots = 4;
    bool adapt_on = true;
    int adapt_min = 1;
    int adapt_x = -1;        // the last X picked from a measurement (-1: none yet: the minimum)
    // endgame threshold: at most this many empty squares on some game's root
    // (two moves before the search) -> X = chain_cuts; raised past every root
    // whose search needed cuts
    static constexpr int kEndgameEmpties = 12;
    int adapt_empties = kEndgameEmpties;
    int64_t adapt_seq = 0;   // grouped searches enqueued with a cuts slot
    // [kCutSlots][kMaxPipeline][2] per search and group: most cuts, fewest root empties
    int32_t* cuts_dev = nullptr;
    int32_t* cuts_host = nullptr;  // pinned copies
    int cut_x[kCutSlots] = {-1, -1, -1, -1};  // X of the search in the slot (-1: slot empty)
    int cut_groups[kCutSlots] = {};
    hipEvent_t cuts_ev[kCutSlots][kMaxPipeline] = {};
    // allocated into locals and published only when every allocation
    // succeeded (a failure leaves nothing half-initialised behind)
    int ensure_cut_slots() {
        if (cuts_dev) return OAMD_OK;
        int32_t* dev = nullptr;
        int32_t* host = nullptr;
        hipEvent_t evs[kCutSlots][kMaxPipeline] = {};
        int rc = dalloc(&dev, (size_t)2 * kCutSlots * kMaxPipeline);
        if (!rc && hipHostMalloc((void**)&host, sizeof(int32_t) * 2 * kCutSlots * kMaxPipeline) != hipSuccess)
            rc = fail(OAMD_RUNTIME, "cut slots: hipHostMalloc failed");
        for (auto& row : evs)
            for (auto& x : row)
                if (!rc && hipEventCreateWithFlags(&x, readback_event_flags()) != hipSuccess)
                    rc = fail(OAMD_RUNTIME, "cut slots: hipEventCreate failed");
        if (rc) {
            for (auto& row : evs)
                for (auto x : row)
                    if (x) (void)hipEventDestroy(x);
            if (host) (void)hipHostFree(host);
            dfree(dev);
            return rc;
        }
        cuts_host = host;
        std::memcpy(cuts_ev, evs, sizeof(evs));
        cuts_dev = dev;
        return OAMD_OK;
    }
    // free-running self-play (oamd_engine_selfplay_steps, tree.hip k_tree_free):
    // games play their moves without waiting for each other; the host enqueues
    // rounds until every group's remaining-games counter (read back two chunks
    // late, pinned memory behind events) is 0
    bool free_running = true;
    // base chunks wait for the chunk two back before they are enqueued
    // (OAMD_SPIN_SYNC=1: no wait, A/B only)
    bool throttle_enqueue = !spin_sync();
    static constexpr int kFreeSlots = 4;
    static constexpr int kFreeTailRounds = 4;
    int32_t* remaining_dev = nullptr;   // [kMaxPipeline]
    int32_t* remaining_host = nullptr;  // [kFreeSlots][kMaxPipeline], pinned
    hipEvent_t free_ev[kFreeSlots][kMaxPipeline] = {};
    int ensure_free_slots() {
        if (remaining_dev) return OAMD_OK;
        int32_t* dev = nullptr;
        int32_t* host = nullptr;
        hipEvent_t evs[kFreeSlots][kMaxPipeline] = {};
        int rc = dalloc(&dev, (size_t)kMaxPipeline);
        if (!rc && hipHostMalloc((void**)&host, sizeof(int32_t) * kFreeSlots * kMaxPipeline) != hipSuccess)
            rc = fail(OAMD_RUNTIME, "free-running slots: hipHostMalloc failed");
        for (auto& row : evs)
            for (auto& x : row)
                if (!rc && hipEventCreateWithFlags(&x, readback_event_flags()) != hipSuccess)
                    rc = fail(OAMD_RUNTIME, "free-running slots: hipEventCreate failed");
        if (rc) {
            for (auto& row : evs)
                for (auto x : row)
                    if (x) (void)hipEventDestroy(x);
            if (host) (void)hipHostFree(host);
            dfree(dev);
            return rc;
        }
        remaining_host = host;
        std::memcpy(free_ev, evs, sizeof(evs));
        remaining_dev = dev;
        return OAMD_OK;
    }
    // workgroups of an extra round's ResNet launch (0 = the regular grid)
    int extra_grid = 128;
    int step_phase = 0;  // 1 = a selected round awaits its backup (step API)
    // pipeline groups (0 = auto) and their streams / fork-join events
    int pipeline = 0;
    // rows per k_resnet launch (0 = one launch per group and step); a group's
    // rows are evaluated by consecutive launches on its stream
    int nn_batch = 0;
    int n_pipe_streams = 0;
    int n_events = 0;  // sel_ev / nn_ev pairs created
    hipStream_t pipe_stream[kMaxPipeline] = {};
    hipEvent_t fork_ev = nullptr;
    // NN tokens: the pipeline groups' ResNet launches form nn_chains chains
    // (group k in chain k % nn_chains); launches of one chain run one after
    // another, chains run concurrently (1 = every launch serialised)
    static constexpr int kMaxChains = 4;
    hipEvent_t nn_token[kMaxChains] = {};
    int nn_chains = 2;
    hipStream_t nn_stream = nullptr;
    hipEvent_t sel_ev[kMaxPipeline] = {};
    hipEvent_t nn_ev[kMaxPipeline] = {};
    hipEvent_t join_ev[kMaxPipeline] = {};
    // timing: kEvPerBlock events per (step, group) of a search, in two pools used in
    // turn, so a search never waits for the previous one's events; a pool is
    // summed (waiting for its last event) before reuse or on a timing query
    bool timing = false;
    int timing_stride = 1;     // time every timing_stride-th search (sampled timing)
    int64_t search_count = 0;
    std::vector<hipEvent_t> ev[2];
    int ev_blocks[2] = {0, 0};  // pending (round, group) blocks per pool
    int ev_final[2] = {0, 0};   // first block of the backup-only final round
    int ev_K[2] = {1, 1};       // groups per round of those blocks
    int ev_nn_groups[2] = {1, 1};  // groups (0 .. n-1) whose NN launches carry events
    int64_t ev_launches[2] = {0, 0};  // k_resnet launches inside those blocks
    int64_t ev_rows[2] = {0, 0};
    // NN busy time (oamd_engine_nn_busy): while timing is enabled, EVERY
    // ResNet launch of a native search records its execution interval
    // (kernel-side span, launch_resnet_packed: ~start, end in 100 MHz ticks)
    // in a window of slots, zeroed when allocated and when the window
    // restarts; the busy time is the union over the whole window (launches of
    // the pipeline groups' searches overlap in time, and the groups drift
    // apart over whole games, so per-search unions would count shared time
    // twice). A search's slots are contiguous: [group][round][launch], in one
    // chunk of at least kSpanChunk slots (larger when one search needs more).
    // Chunks that no search reserves in any more are copied to the host once
    // (span_ticks); a window of more than kSpanWindow slots stops recording
    // and makes oamd_engine_nn_busy fail (its launches would be missing).
    static constexpr int64_t kSpanChunk = 1 << 15;    // slots (2 x u64) per chunk
    static constexpr int64_t kSpanWindow = 1 << 23;   // most slots of one window (128 MiB)
    struct SpanChunk {
        unsigned long long* p = nullptr;
        int64_t cap = 0, used = 0;
    };
    std::vector<SpanChunk> span_chunks;
    int64_t span_slots = 0;     // slots reserved in this window
    int64_t span_dropped = 0;   // launches of this window that found no slot
    size_t span_copied = 0;     // leading chunks already folded into span_ticks
    std::vector<std::pair<long long, long long>> span_ticks;  // their intervals (ticks)
    int ev_cur = 0;
    float nn_ms = 0.0f;
    float select_ms = 0.0f;
    float backup_ms = 0.0f;
    int64_t nn_launches = 0;
    int64_t tree_launches = 0;  // timed select rounds (one k_tree launch per round and group)
    int64_t tree_final_launches = 0;  // timed final backup-only rounds (x groups)
    int64_t grouped_searches = 0, grouped_rounds = 0;  // oamd_engine_round_counts
    int64_t nn_rows = 0;

    int resolve_timing(int p) {
        const int n = ev_blocks[p];
        if (!n) return OAMD_OK;
        // NN launch intervals relative to the search's first event: their
        // union is the time some ResNet launch ran (launches of different NN
        // chains overlap; with one chain the union is the sum of durations)
        for (int i = 0; i < n; ++i) {
            const hipEvent_t* b = &ev[p][kEvPerBlock * i];
            float ms = 0.0f;
            // blocks of different groups end on different streams; the final
            // round records no NN events
            const bool nn = i < ev_final[p] && i % ev_K[p] < ev_nn_groups[p];
            HIPCHK(hipEventSynchronize(b[1]));
            if (nn) HIPCHK(hipEventSynchronize(b[3]));
            HIPCHK(hipEventElapsedTime(&ms, b[0], b[1]));
            (i < ev_final[p] ? select_ms : backup_ms) += ms;
            if (nn) {
                HIPCHK(hipEventElapsedTime(&ms, b[2], b[3]));
                nn_ms += ms;
            }
        }

        nn_launches += ev_launches[p];
        tree_launches += ev_final[p];
        tree_final_launches += n - ev_final[p];
        nn_rows += ev_rows[p];
        ev_blocks[p] = 0;
        return OAMD_OK;
    }
    int resolve_all_timing() {
        int rc = resolve_timing(ev_cur ^ 1);
        return rc ? rc : resolve_timing(ev_cur);
    }
    // n contiguous span slots for one search (nullptr when timing is off)
    int reserve_spans(int64_t n, unsigned long long** out) {
        *out = nullptr;
        if (!timing || n <= 0) return OAMD_OK;
        if (span_slots + n > kSpanWindow) {  // not recorded: nn_busy reports it
            span_dropped += n;
            return OAMD_OK;
        }
        if (span_chunks.empty() || span_chunks.back().used + n > span_chunks.back().cap) {
            SpanChunk c;
            c.cap = std::max(kSpanChunk, n);
            if (int rc = dalloc(&c.p, (size_t)2 * c.cap)) return rc;
            if (hipMemset(c.p, 0, sizeof(unsigned long long) * 2 * c.cap) != hipSuccess) {
                dfree(c.p);
                return fail(OAMD_RUNTIME, "span window: hipMemset failed");
            }
            span_chunks.push_back(c);
        }
        SpanChunk& c = span_chunks.back();
        *out = c.p + 2 * c.used;
        c.used += n;
        span_slots += n;
        return OAMD_OK;
    }
    // restart the window: every launch that may still write a slot is done
    int reset_spans() {
        if (span_chunks.empty() && !span_dropped) return OAMD_OK;
        HIPCHK(hipDeviceSynchronize());
        for (auto& c : span_chunks) dfree(c.p);
        span_chunks.clear();
        span_slots = span_dropped = 0;
        span_copied = 0;
        span_ticks.clear();
        return OAMD_OK;
    }
    // the window's recorded intervals (ticks); waits for the device
    int span_intervals(std::vector<std::pair<long long, long long>>* iv) {
        HIPCHK(hipDeviceSynchronize());  // every launch of the window has written its slot
        auto read = [&](const SpanChunk& c, std::vector<std::pair<long long, long long>>* to) -> int {
            std::vector<unsigned long long> sp((size_t)2 * c.used);
            if (c.used)
                HIPCHK(hipMemcpy(sp.data(), c.p, sizeof(unsigned long long) * 2 * c.used, hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < c.used; ++i)  // start stored complemented (an atomicMin on zeroed slots)
                if (sp[2 * i + 1]) to->emplace_back((long long)~sp[2 * i], (long long)sp[2 * i + 1]);
            return OAMD_OK;
        };
        // chunks before the last one are complete: fold them in once
        for (; span_copied + 1 < span_chunks.size(); ++span_copied) {
            if (int rc = read(span_chunks[span_copied], &span_ticks)) return rc;
            dfree(span_chunks[span_copied].p);
        }
        *iv = span_ticks;
        if (!span_chunks.empty())
            if (int rc = read(span_chunks.back(), iv)) return rc;
        return OAMD_OK;
    }

    int L() const { return cfg.num_threads * cfg.batch_size; }
    // thread-split schedule for one game (OAMD_TREE_SPLIT=0 in the environment: off)
    static bool tree_split() {
        static const bool v = [] {
            const char* e = getenv("OAMD_TREE_SPLIT");
            return e ? atoi(e) != 0 : true;
        }();
        return v;
    }
    // K group streams (2 in the single-game thread split) and their events; the
    // thread split needs a select / NN event pair per virtual thread (nev >= K)
    int ensure_streams(int K, int nev) {
        if (K <= 1 && nev <= 1) return OAMD_OK;
        if (!fork_ev) HIPCHK(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
        for (int c = 0; c < kMaxChains; ++c)
            if (!nn_token[c]) HIPCHK(hipEventCreateWithFlags(&nn_token[c], hipEventDisableTiming));
        if (!nn_stream) HIPCHK(hipStreamCreateWithFlags(&nn_stream, hipStreamNonBlocking));
        while (n_pipe_streams < K) {
            const int k = n_pipe_streams;
            HIPCHK(hipStreamCreateWithFlags(&pipe_stream[k], hipStreamNonBlocking));
            HIPCHK(hipEventCreateWithFlags(&join_ev[k], hipEventDisableTiming));
            ++n_pipe_streams;
        }
        while (n_events < nev) {
            const int k = n_events;
            // sel_ev only orders kernels of this device (the split schedule's tree
            // operations): no system-scope fence (its host-visibility cache
            // maintenance) on the cross-stream path of every round
            HIPCHK(hipEventCreateWithFlags(&sel_ev[k], hipEventDisableTiming | hipEventDisableSystemFence));
            HIPCHK(hipEventCreateWithFlags(&nn_ev[k], hipEventDisableTiming));
            ++n_events;
        }
        return OAMD_OK;
    }
    int FW() const { return feature_words(cfg.history_size); }

    EngineView view() const {
        EngineView E;
        E.G = G;
        E.L = L();
        E.H = cfg.history_size;
        E.FW = FW();
        E.cap = cap;
        E.link = link;
        E.stat = stat;
        E.pos = pos;
        E.games = games;
        E.leaf = leaf;
        E.depth = depth;
        E.trans = trans;
        E.path = path;
        E.feat = feat;
        E.policy = policy;
        E.value = value;
        E.explore_tab = explore_tab;
        E.c_base = cfg.c_puct_base;
        E.c_init = cfg.c_puct_init;
        E.eps = cfg.dirichlet_epsilon;
        E.alpha = cfg.dirichlet_alpha;
        E.counters = counters;
        E.rowlist = rowlist;
        E.tstate = tstate;
        E.steps = (cfg.num_simulations + L() - 1) / L();
        E.B = cfg.batch_size;
        E.terminal_skip = exact_interleaving ? 1 : 0;
        return E;
    }

    int alloc_rows() {
        const int64_t rows = (int64_t)G * L();
        const int fw = FW();
        if (rows <= rows_cap && fw <= fw_cap) return OAMD_OK;
        dfree(leaf);
        dfree(depth);
        dfree(trans);
        dfree(path);
        dfree(feat);
        dfree(policy);
        dfree(value);
        dfree(flags);
        dfree(rowlist);
        dfree(tstate);
        int rc;
        if ((rc = dalloc(&leaf, rows)) || (rc = dalloc(&depth, rows)) || (rc = dalloc(&trans, rows)) ||
            (rc = dalloc(&path, rows * kMaxDepth)) || (rc = dalloc(&feat, rows * fw)) ||
            (rc = dalloc(&policy, rows * 65)) || (rc = dalloc(&value, rows)) || (rc = dalloc(&flags, rows)) ||
            (rc = dalloc(&rowlist, rows)) || (rc = dalloc(&tstate, rows)))
            return rc;
        HIPCHK(hipMemset(policy, 0, rows * 65 * sizeof(float)));
        HIPCHK(hipMemset(value, 0, rows * sizeof(float)));
        rows_cap = rows;
        fw_cap = fw;
        return OAMD_OK;
    }

    // exploration_rate table with the HOST's logf (bit-identical to the
    // reference's std::log(float), search_thread.cpp:198-203)
    int build_tables() {
        std::vector<float> ex(kExploreTab);
        for (int n = 0; n < kExploreTab; ++n)
            ex[n] = std::log(((float)(1 + n) + cfg.c_puct_base) / cfg.c_puct_base) + cfg.c_puct_init;
        HIPCHK(hipMemcpy(explore_tab, ex.data(), ex.size() * sizeof(float), hipMemcpyHostToDevice));
        return OAMD_OK;
    }

    ~oamd_engine() {
        DeviceGuard dg(device);
        dfree(link);
        dfree(stat);
        dfree(pos);
        dfree(games);
        dfree(leaf);
        dfree(depth);
        dfree(trans);
        dfree(path);
        dfree(feat);
        dfree(policy);
        dfree(value);
        dfree(flags);
        dfree(rowlist);
        dfree(tstate);
        dfree(rowcount);
        dfree(explore_tab);
        dfree(counters);
        dfree(status_dev);
        dfree(info_dev);
        dfree(visits_dev);
        dfree(q_dev);
        dfree(spd_dev);
        for (auto& pool : ev)
            for (auto e : pool) (void)hipEventDestroy(e);
        for (auto& c : span_chunks) dfree(c.p);
        if (cuts_dev) {
            (void)hipDeviceSynchronize();  // no copy into cuts_host in flight
            dfree(cuts_dev);
            (void)hipHostFree(cuts_host);
            for (auto& row : cuts_ev)
                for (auto x : row) (void)hipEventDestroy(x);
        }
        if (remaining_dev) {
            (void)hipDeviceSynchronize();  // no copy into remaining_host in flight
            dfree(remaining_dev);
            (void)hipHostFree(remaining_host);
            for (auto& row : free_ev)
                for (auto x : row) (void)hipEventDestroy(x);
        }
        for (int k = 0; k < n_pipe_streams; ++k) {
            (void)hipStreamDestroy(pipe_stream[k]);
            (void)hipEventDestroy(join_ev[k]);
        }
        for (int k = 0; k < n_events; ++k) {
            (void)hipEventDestroy(sel_ev[k]);
            (void)hipEventDestroy(nn_ev[k]);
        }
        if (fork_ev) (void)hipEventDestroy(fork_ev);
        for (int c = 0; c < kMaxChains; ++c)
            if (nn_token[c]) (void)hipEventDestroy(nn_token[c]);
        if (nn_stream) (void)hipStreamDestroy(nn_stream);
    }
};

// ===========================================================================
// net
// ===========================================================================
struct oamd_net {
    int device = 0;
    oamd_net_desc desc{};
    uint16_t* w = nullptr;
    float* bias = nullptr;
    float* head = nullptr;
    uint16_t* hconv = nullptr;
    bool loaded = false;
    std::vector<std::string> keys;
    std::vector<int64_t> numel;

    NetView view() const {
        NetView N;
        N.cin = desc.in_channels;
        N.C = desc.conv_channels;
        N.R = desc.num_residual_blocks;
        N.hidden = desc.value_head_hidden_channels;
        N.dtype = desc.dtype;
        N.w = w;
        N.bias = bias;
        N.head = head;
        N.hconv = hconv;
        return N;
    }
    ~oamd_net() {
        DeviceGuard dg(device);
        dfree(w);
        dfree(bias);
        dfree(head);
        dfree(hconv);
    }
};

extern "C" {

const char* oamd_last_error(void) { return g_err.c_str(); }
int oamd_abi_version(void) { return OAMD_ABI_VERSION; }

// build.py passes the source hashes (othello_mcts/provenance.py)
#ifndef OAMD_SOURCE_HASH_ALL
#define OAMD_SOURCE_HASH_ALL "unknown"
#define OAMD_SOURCE_HASH_RESNET "unknown"
#define OAMD_SOURCE_HASH_TREE "unknown"
#endif
const char* oamd_source_hash(const char* family) {
    if (!family) return nullptr;
    if (!std::strcmp(family, "all")) return OAMD_SOURCE_HASH_ALL;
    if (!std::strcmp(family, "resnet")) return OAMD_SOURCE_HASH_RESNET;
    if (!std::strcmp(family, "tree")) return OAMD_SOURCE_HASH_TREE;
    return nullptr;
}

int oamd_device_count(int32_t* out) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return OAMD_OK;
}

// ---------------------------------------------------------------- bitboards
int oamd_get_legal_moves(const uint64_t* me, const uint64_t* opp, uint64_t* out, int64_t n, void* stream) {
    if (n < 0) return fail(OAMD_INVALID_ARGUMENT, "n must be >= 0");
    launch_legal_moves(me, opp, out, n, (hipStream_t)stream);
    LAUNCHCHK();
    return OAMD_OK;
}

int oamd_get_flips(const uint64_t* mv, const uint64_t* me, const uint64_t* opp, uint64_t* out, int64_t n,
                   void* stream) {
    if (n < 0) return fail(OAMD_INVALID_ARGUMENT, "n must be >= 0");
    launch_flips(mv, me, opp, out, n, (hipStream_t)stream);
    LAUNCHCHK();
    return OAMD_OK;
}

int oamd_apply_action(const oamd_position* in, const int32_t* actions, oamd_position* out, int64_t n,
                      void* stream) {
    static_assert(sizeof(oamd_position) == sizeof(Pos), "layout");
    if (n < 0) return fail(OAMD_INVALID_ARGUMENT, "n must be >= 0");
    launch_apply_positions(reinterpret_cast<const Pos*>(in), actions, reinterpret_cast<Pos*>(out), n,
                           (hipStream_t)stream);
    LAUNCHCHK();
    return OAMD_OK;
}

int oamd_initial_position(oamd_position* out) {
    const Pos p = initial_position();
    std::memcpy(out, &p, sizeof(Pos));
    return OAMD_OK;
}

uint64_t oamd_host_legal_moves(uint64_t me, uint64_t opp) { return legal_moves(me, opp); }
uint64_t oamd_host_flips(uint64_t mv, uint64_t me, uint64_t opp) { return flips(mv, me, opp); }
void oamd_host_apply_action(const oamd_position* in, int32_t action, oamd_position* out) {
    Pos p;
    std::memcpy(&p, in, sizeof(Pos));
    const Pos c = apply_action(p, action);
    std::memcpy(out, &c, sizeof(Pos));
}

// ---------------------------------------------------------------- net
int oamd_net_create(int32_t device, const oamd_net_desc* d, oamd_net** out) {
    *out = nullptr;
    if (d->in_channels < 1 || d->in_channels > 31)
        return fail(OAMD_INVALID_ARGUMENT, "in_channels must be in [1, 31], got " + std::to_string(d->in_channels));
    if (d->conv_channels != 128 && d->conv_channels != 256)
        return fail(OAMD_INVALID_ARGUMENT,
                    "conv_channels must be 128 or 256 for the native net, got " + std::to_string(d->conv_channels));
    if (d->num_residual_blocks < 0)
        return fail(OAMD_INVALID_ARGUMENT, "num_residual_blocks must be >= 0");
    if (d->value_head_hidden_channels < 1 || d->value_head_hidden_channels > 1024)
        return fail(OAMD_INVALID_ARGUMENT, "value_head_hidden_channels must be in [1, 1024] for the native net, got " +
                                               std::to_string(d->value_head_hidden_channels));
    if (d->num_squares != 64 || d->num_actions != 65)
        return fail(OAMD_INVALID_ARGUMENT, "num_squares must be 64 and num_actions 65");
    if (d->dtype != OAMD_BF16 && d->dtype != OAMD_FP16)
        return fail(OAMD_INVALID_ARGUMENT, "dtype must be OAMD_BF16 or OAMD_FP16");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(OAMD_RUNTIME, "no HIP device available");
    if (device < 0 || device >= n) return fail(OAMD_INVALID_ARGUMENT, "bad device ordinal");
    DeviceGuard dg(device);
    auto* net = new oamd_net();
    net->device = device;
    net->desc = *d;
    const int C = d->conv_channels, R = d->num_residual_blocks, hid = d->value_head_hidden_channels;
    int rc;
    if ((rc = dalloc(&net->w, resnet_packed_weight_alloc_elems(C, R))) ||
        (rc = dalloc(&net->bias, (size_t)(1 + 2 * R) * C)) ||
        (rc = dalloc(&net->head, resnet_head_floats(C, hid))) ||
        (rc = dalloc(&net->hconv, resnet_hconv_elems(C)))) {
        delete net;
        return rc;
    }
    // state_dict keys (neural_net.py:9-172), num_batches_tracked omitted
    auto conv = [&](const std::string& p, int64_t cout, int64_t cin, int64_t k) {
        net->keys.push_back(p + ".weight");
        net->numel.push_back(cout * cin * k * k);
        net->keys.push_back(p + ".bias");
        net->numel.push_back(cout);
    };
    auto bn = [&](const std::string& p, int64_t c) {
        for (const char* s : {".weight", ".bias", ".running_mean", ".running_var"}) {
            net->keys.push_back(p + s);
            net->numel.push_back(c);
        }
    };
    auto lin = [&](const std::string& p, int64_t fin, int64_t fout) {
        net->keys.push_back(p + ".weight");
        net->numel.push_back(fin * fout);
        net->keys.push_back(p + ".bias");
        net->numel.push_back(fout);
    };
    conv("conv_block.conv", C, d->in_channels, 3);
    bn("conv_block.norm", C);
    for (int i = 0; i < R; ++i) {
        const std::string p = "residual_blocks." + std::to_string(i);
        conv(p + ".conv1", C, C, 3);
        bn(p + ".norm1", C);
        conv(p + ".conv2", C, C, 3);
        bn(p + ".norm2", C);
    }
    conv("policy_head.conv", 2, C, 1);
    bn("policy_head.norm", 2);
    lin("policy_head.linear", 128, 65);
    conv("value_head.conv", 1, C, 1);
    bn("value_head.norm", 1);
    lin("value_head.linear1", 64, hid);
    lin("value_head.linear2", hid, 1);
    *out = net;
    return OAMD_OK;
}

int oamd_net_destroy(oamd_net* net) {
    delete net;
    return OAMD_OK;
}

int oamd_net_state_size(const oamd_net* net, int32_t* n) {
    *n = (int32_t)net->keys.size();
    return OAMD_OK;
}

int oamd_net_state_key(const oamd_net* net, int32_t i, const char** key, int64_t* numel) {
    if (i < 0 || i >= (int32_t)net->keys.size()) return fail(OAMD_OUT_OF_RANGE, "state index out of range");
    *key = net->keys[i].c_str();
    *numel = net->numel[i];
    return OAMD_OK;
}

static uint16_t f32_to_bf16_rne(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

static uint16_t f32_to_f16(float f) {
    _Float16 h = (_Float16)f;
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
}

int oamd_net_load_state(oamd_net* net, const float* const* t, int32_t n_tensors) {
    if (n_tensors != (int32_t)net->keys.size())
        return fail(OAMD_INVALID_ARGUMENT, "expected " + std::to_string(net->keys.size()) + " tensors, got " +
                                               std::to_string(n_tensors));
    const auto& d = net->desc;
    const int C = d.conv_channels, R = d.num_residual_blocks, hid = d.value_head_hidden_channels;
    const double eps = 1e-5;  // torch.nn.BatchNorm2d default
    int ti = 0;
    std::vector<uint16_t> packed(resnet_packed_weight_elems(C, R));
    std::vector<float> bias((size_t)(1 + 2 * R) * C);
    size_t ks_global = 0;
    // fold BN into a 3x3 conv and pack in MFMA A-fragment order, K-step by K-step
    // (resnet_kstep): [ks][ntile][lane][8]; lane holds output channel
    // resnet_out_channel(ntile, lane&15) and input channels cb*32 + 8*chunk(lane>>4) + j
    auto pack_conv = [&](int layer, int cin, bool first) {
        const float* W = t[ti++];
        const float* b = t[ti++];
        const float* g = t[ti++];
        const float* be = t[ti++];
        const float* mu = t[ti++];
        const float* var = t[ti++];
        std::vector<double> scale(C);
        for (int n = 0; n < C; ++n) {
            scale[n] = (double)g[n] / std::sqrt((double)var[n] + eps);
            bias[(size_t)layer * C + n] = (float)(((double)b[n] - (double)mu[n]) * scale[n] + (double)be[n]);
        }
        const int nk = resnet_ksteps(C, first);
        for (int i = 0; i < nk; ++i) {
            int tap, cb;
            bool pad;
            resnet_kstep(C, first, i, &tap, &cb, &pad);
            const size_t ks = ks_global + (size_t)i;
            for (int nt = 0; nt < C / 16; ++nt)
                for (int lane = 0; lane < 64; ++lane)
                    for (int j = 0; j < 8; ++j) {
                        const int ci = cb * 32 + 8 * resnet_kgroup_chunk(lane >> 4) + j;
                        const int n = resnet_out_channel(nt, lane & 15);
                        double v = 0.0;
                        if (!pad && ci < cin) v = (double)W[((size_t)n * cin + ci) * 9 + tap] * scale[n];
                        const size_t idx = (((ks * (C / 16) + nt) * 64) + lane) * 8 + j;
                        packed[idx] = d.dtype == OAMD_BF16 ? f32_to_bf16_rne((float)v) : f32_to_f16((float)v);
                    }
        }
        ks_global += (size_t)nk;
    };
    pack_conv(0, d.in_channels, true);
    for (int i = 0; i < R; ++i) {
        pack_conv(1 + 2 * i, C, false);
        pack_conv(2 + 2 * i, C, false);
    }
    // heads (fp32; 1x1 conv + BN folded)
    std::vector<float> head(resnet_head_floats(C, hid));
    const int HL_pcw = 0, HL_pcb = HL_pcw + 2 * C, HL_vcw = HL_pcb + 2, HL_vcb = HL_vcw + C,
              HL_plw = HL_vcb + 1, HL_plb = HL_plw + 128 * 65, HL_v1w = HL_plb + 65, HL_v1b = HL_v1w + 64 * hid,
              HL_v2w = HL_v1b + hid, HL_v2b = HL_v2w + hid;
    {
        const float* W = t[ti++];
        const float* b = t[ti++];
        const float* g = t[ti++];
        const float* be = t[ti++];
        const float* mu = t[ti++];
        const float* var = t[ti++];
        for (int c = 0; c < 2; ++c) {
            const double s = (double)g[c] / std::sqrt((double)var[c] + eps);
            for (int ch = 0; ch < C; ++ch) head[HL_pcw + c * C + ch] = (float)((double)W[c * C + ch] * s);
            head[HL_pcb + c] = (float)(((double)b[c] - (double)mu[c]) * s + (double)be[c]);
        }
        const float* LW = t[ti++];
        const float* LB = t[ti++];
        for (int a = 0; a < 65; ++a) {
            for (int i = 0; i < 128; ++i) head[HL_plw + i * 65 + a] = LW[a * 128 + i];
            head[HL_plb + a] = LB[a];
        }
    }
    {
        const float* W = t[ti++];
        const float* b = t[ti++];
        const float* g = t[ti++];
        const float* be = t[ti++];
        const float* mu = t[ti++];
        const float* var = t[ti++];
        const double s = (double)g[0] / std::sqrt((double)var[0] + eps);
        for (int ch = 0; ch < C; ++ch) head[HL_vcw + ch] = (float)((double)W[ch] * s);
        head[HL_vcb] = (float)(((double)b[0] - (double)mu[0]) * s + (double)be[0]);
        const float* W1 = t[ti++];
        const float* B1 = t[ti++];
        for (int j = 0; j < hid; ++j) {
            for (int sq = 0; sq < 64; ++sq) head[HL_v1w + sq * hid + j] = W1[j * 64 + sq];
            head[HL_v1b + j] = B1[j];
        }
        const float* W2 = t[ti++];
        const float* B2 = t[ti++];
        for (int j = 0; j < hid; ++j) head[HL_v2w + j] = W2[j];
        head[HL_v2b] = B2[0];
    }
    // 1x1 head convs (folded) in MFMA A-fragment order: lane holds row lane&15
    // (0, 1 = policy channels, 2 = value, else 0) and input channels
    // cb*32 + 8*chunk(lane>>4) + j, matching the tower's B fragments
    std::vector<uint16_t> hconv(resnet_hconv_elems(C));
    for (int cb = 0; cb < C / 32; ++cb)
        for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 8; ++j) {
                const int r = lane & 15, ci = cb * 32 + 8 * resnet_kgroup_chunk(lane >> 4) + j;
                const float v = r < 2 ? head[HL_pcw + r * C + ci] : (r == 2 ? head[HL_vcw + ci] : 0.0f);
                hconv[((size_t)cb * 64 + lane) * 8 + j] = d.dtype == OAMD_BF16 ? f32_to_bf16_rne(v) : f32_to_f16(v);
            }
    DeviceGuard dg(net->device);
    // searches run the ResNet on non-blocking streams, which a plain hipMemcpy
    // does not order against: let every launch still reading these buffers
    // finish before they are overwritten (a weight refresh between searches)
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(net->hconv, hconv.data(), hconv.size() * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(net->w, packed.data(), packed.size() * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(net->w + packed.size(), 0,
                     (resnet_packed_weight_alloc_elems(C, R) - packed.size()) * sizeof(uint16_t)));
    HIPCHK(hipMemcpy(net->bias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(net->head, head.data(), head.size() * 4, hipMemcpyHostToDevice));
    net->loaded = true;
    return OAMD_OK;
}

int oamd_net_forward(oamd_net* net, const float* features, int32_t rows, float* policy, float* value,
                     void* stream) {
    if (!net->loaded) return fail(OAMD_INVALID_ARGUMENT, "net weights not loaded");
    if (rows < 0) return fail(OAMD_INVALID_ARGUMENT, "rows must be >= 0");
    DeviceGuard dg(net->device);
    launch_resnet_f32(net->view(), features, rows, policy, value, (hipStream_t)stream);
    LAUNCHCHK();
    return OAMD_OK;
}

// ---------------------------------------------------------------- engine
int oamd_engine_create(int32_t device, int32_t num_games, int64_t node_capacity, const oamd_search_config* cfg,
                       uint64_t seed, oamd_engine** out) {
    *out = nullptr;
    int rc = validate_config(cfg);
    if (rc) return rc;
    if (num_games < 1) return fail(OAMD_INVALID_ARGUMENT, "num_games must be >= 1");
    if (node_capacity == 0) node_capacity = (int64_t)1 << 20;
    if (node_capacity < 128 || node_capacity > ((int64_t)1 << 30))
        return fail(OAMD_INVALID_ARGUMENT, "node_capacity must be in [128, 2^30]");
    if ((int64_t)num_games * node_capacity > ((int64_t)1 << 36))
        return fail(OAMD_INVALID_ARGUMENT, "num_games * node_capacity too large");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(OAMD_RUNTIME, "no HIP device available");
    if (device < 0 || device >= n) return fail(OAMD_INVALID_ARGUMENT, "bad device ordinal");
    DeviceGuard dg(device);
    auto* e = new oamd_engine();
    e->device = device;
    e->G = num_games;
    e->cap = node_capacity;
    e->cfg = *cfg;
    e->seed = seed;
    const size_t nodes = (size_t)num_games * node_capacity;
    if ((rc = dalloc(&e->link, nodes)) || (rc = dalloc(&e->stat, nodes)) || (rc = dalloc(&e->pos, nodes)) ||
        (rc = dalloc(&e->games, num_games)) || (rc = dalloc(&e->explore_tab, kExploreTab)) || (rc = dalloc(&e->counters, kCounters)) ||
        (rc = dalloc(&e->rowcount, 2 * kMaxPipeline)) ||
        (rc = dalloc(&e->status_dev, 2)) || (rc = dalloc(&e->info_dev, num_games)) || (rc = dalloc(&e->visits_dev, (size_t)num_games * 65)) ||
        (rc = dalloc(&e->q_dev, (size_t)num_games * 65)) ||
        (rc = dalloc(&e->spd_dev, (size_t)8 * (1 + 2 * kMaxHistory) * 64 + 8 * 65)) || (rc = e->alloc_rows()) ||
        (rc = e->build_tables())) {
        delete e;
        return rc;
    }
    if (hipMemset(e->counters, 0, kCounters * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(e->rowcount, 0, 2 * kMaxPipeline * sizeof(int32_t)) != hipSuccess) {
        delete e;
        return fail(OAMD_RUNTIME, "engine init: counter memset failed");
    }
    launch_reset(e->view(), -1, seed, nullptr);
    hipError_t le = hipGetLastError();
    if (le != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        delete e;
        return fail(OAMD_RUNTIME, std::string("engine init: ") + hipGetErrorString(le));
    }
    *out = e;
    return OAMD_OK;
}

int oamd_engine_destroy(oamd_engine* e) {
    delete e;
    return OAMD_OK;
}

int oamd_engine_set_config(oamd_engine* e, const oamd_search_config* cfg) {
    int rc = validate_config(cfg);
    if (rc) return rc;
    DeviceGuard dg(e->device);
    const bool tabs = cfg->c_puct_base != e->cfg.c_puct_base || cfg->c_puct_init != e->cfg.c_puct_init;
    HIPCHK(hipStreamSynchronize(e->stream));
    e->cfg = *cfg;
    if ((rc = e->alloc_rows())) return rc;
    if (tabs && (rc = e->build_tables())) return rc;
    e->step_phase = 0;
    e->steps_left = 0;
    return OAMD_OK;
}

int oamd_engine_get_config(const oamd_engine* e, oamd_search_config* cfg) {
    *cfg = e->cfg;
    return OAMD_OK;
}

int oamd_engine_num_games(const oamd_engine* e, int32_t* out) {
    *out = e->G;
    return OAMD_OK;
}

int oamd_engine_set_stream(oamd_engine* e, void* stream) {
    e->stream = (hipStream_t)stream;
    return OAMD_OK;
}

int oamd_engine_reset(oamd_engine* e, int32_t game, uint64_t seed) {
    if (game < -1 || game >= e->G) return fail(OAMD_OUT_OF_RANGE, "game index out of range");
    DeviceGuard dg(e->device);
    launch_reset(e->view(), game, seed, e->stream);
    LAUNCHCHK();
    e->step_phase = 0;
    e->steps_left = 0;
    return OAMD_OK;
}

int oamd_engine_search_begin(oamd_engine* e, int32_t* steps) {
    const int L = e->L();
    e->steps_left = (e->cfg.num_simulations + L - 1) / L;  // search_thread.cpp:50-52
    e->steps_total = e->steps_left;
    e->step_phase = 0;
    if (steps) *steps = e->steps_left;
    return OAMD_OK;
}

int oamd_engine_select(oamd_engine* e) {
    if (e->steps_left <= 0)
        return fail(OAMD_INVALID_ARGUMENT, "select called out of order (search_begin first)");
    DeviceGuard dg(e->device);
    // a pending round is backed up thread by thread, each thread selecting its
    // next batch right after its backup (the reference's interleaving, k_tree)
    launch_tree(e->view(), e->stream, e->step_phase == 1, true, e->cfg.num_threads, e->cfg.batch_size, 0, -1, 0, -1,
                nullptr, nullptr, e->steps_left == e->steps_total);
    LAUNCHCHK();
    e->step_phase = 1;
    e->steps_left -= 1;
    return OAMD_OK;
}

int oamd_engine_leaf_flags(oamd_engine* e, uint8_t* host_out) {
    DeviceGuard dg(e->device);
    launch_leaf_flags(e->view(), e->flags, e->stream);
    LAUNCHCHK();
    HIPCHK(hipMemcpyAsync(host_out, e->flags, (size_t)e->G * e->L(), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return OAMD_OK;
}

int oamd_engine_features(oamd_engine* e, float* out, int32_t row_begin, int32_t rows) {
    if (row_begin < 0 || rows < 0 || (int64_t)row_begin + rows > (int64_t)e->G * e->L())
        return fail(OAMD_OUT_OF_RANGE, "row range out of range");
    DeviceGuard dg(e->device);
    launch_features_f32(e->view(), out, row_begin, rows, e->stream);
    LAUNCHCHK();
    return OAMD_OK;
}

int oamd_engine_set_evaluation(oamd_engine* e, const float* pol, const float* val, int32_t row_begin,
                               int32_t rows) {
    if (row_begin < 0 || rows < 0 || (int64_t)row_begin + rows > (int64_t)e->G * e->L())
        return fail(OAMD_OUT_OF_RANGE, "row range out of range");
    DeviceGuard dg(e->device);
    launch_set_evaluation(e->view(), pol, val, row_begin, rows, e->stream);
    LAUNCHCHK();
    return OAMD_OK;
}

int oamd_engine_backup(oamd_engine* e) {
    if (e->step_phase != 1) return fail(OAMD_INVALID_ARGUMENT, "backup called before select");
    DeviceGuard dg(e->device);
    launch_tree(e->view(), e->stream, true, false, e->cfg.num_threads, e->cfg.batch_size);
    LAUNCHCHK();
    e->step_phase = 0;
    return OAMD_OK;
}

int oamd_engine_enable_timing(oamd_engine* e, int32_t enable) {
    if (enable < 0) return fail(OAMD_INVALID_ARGUMENT, "enable_timing: expected >= 0");
    DeviceGuard dg(e->device);
    if (int rc = e->reset_spans()) return rc;
    e->timing = enable != 0;
    e->timing_stride = enable > 1 ? enable : 1;
    e->search_count = 0;
    return OAMD_OK;
}

int oamd_engine_nn_timing(const oamd_engine* ce, float* nn_ms, int64_t* launches, int64_t* rows) {
    oamd_engine* e = const_cast<oamd_engine*>(ce);  // pending events are summed here
    if (int rc = e->resolve_all_timing()) return rc;
    if (nn_ms) *nn_ms = e->nn_ms;
    if (launches) *launches = e->nn_launches;
    if (rows) *rows = e->nn_rows;
    return OAMD_OK;
}

int oamd_engine_nn_busy(const oamd_engine* ce, float* busy_ms, int64_t* launches) {
    oamd_engine* e = const_cast<oamd_engine*>(ce);
    DeviceGuard dg(e->device);
    if (e->span_dropped)
        return fail(OAMD_RUNTIME, "nn_busy: the timing window outgrew its " + std::to_string(oamd_engine::kSpanWindow) +
                                      " slots; " + std::to_string(e->span_dropped) +
                                      " launches were not recorded (restart it with oamd_engine_enable_timing)");
    std::vector<std::pair<long long, long long>> iv;
    if (int rc = e->span_intervals(&iv)) return rc;
    // 100 MHz ticks -> ms, once for the whole union
    if (busy_ms) *busy_ms = (float)(interval_union(iv) * 1e-5);
    // the launches that ran (a search reserves slots for the most launches of
    // any group per round; groups of unequal size may leave some unused)
    if (launches) *launches = (int64_t)iv.size();
    return OAMD_OK;
}

int oamd_engine_tree_timing(const oamd_engine* ce, float* select_ms, float* backup_ms, int64_t* launches) {
    oamd_engine* e = const_cast<oamd_engine*>(ce);
    if (int rc = e->resolve_all_timing()) return rc;
    if (select_ms) *select_ms = e->select_ms;
    if (backup_ms) *backup_ms = e->backup_ms;
    if (launches) *launches = e->tree_launches;
    return OAMD_OK;
}

// Pipeline groups of a native search: the games split into K contiguous
// groups, each on its own stream, so one group's tree kernels (latency-bound,
// a wave per game) run while another group's ResNet launch owns the MFMA
// units. Games are independent, so the results are identical for every K.
struct GroupPlan {
    int K = 1;
    hipStream_t st[kMaxPipeline] = {};
    int g0[kMaxPipeline] = {}, ng[kMaxPipeline] = {};
};

static int native_search_checks(const oamd_engine* e, const oamd_net* net) {
    if (!net || !net->loaded) return fail(OAMD_INVALID_ARGUMENT, "native net not loaded");
    if (net->device != e->device) return fail(OAMD_INVALID_ARGUMENT, "net and engine on different devices");
    if (net->desc.in_channels != 1 + 2 * e->cfg.history_size)
        return fail(OAMD_INVALID_ARGUMENT, "net in_channels != 1 + 2 * history_size");
    return OAMD_OK;
}

static GroupPlan plan_groups(oamd_engine* e) {
    GroupPlan P;
    int K = e->pipeline > 0 ? e->pipeline : (e->G >= 64 ? 2 : 1);
    if (K > e->G) K = e->G;
    if (K > kMaxPipeline) K = kMaxPipeline;
    P.K = K;
    for (int k = 0; k < K; ++k) {
        P.g0[k] = (int)((int64_t)e->G * k / K);
        P.ng[k] = (int)((int64_t)e->G * (k + 1) / K) - P.g0[k];
        P.st[k] = K == 1 ? e->stream : e->pipe_stream[k];
    }
    return P;
}

// Extra rounds of a native grouped search (chain splitting, k_tree): the
// reference's interleaving only
static int extra_rounds(const oamd_engine* e) {
    if (!e->exact_interleaving || e->chain_budget <= 0) return 0;
    // a cut follows >= budget all-terminal batches of its round, and a search
    // has T x steps batches per game: no game can use more cuts than that
    const int64_t batches = (int64_t)e->cfg.num_threads * ((e->cfg.num_simulations + e->L() - 1) / e->L());
    return (int)std::min<int64_t>(e->chain_cuts, batches / e->chain_budget);
}

// Extra rounds X of the next grouped search. Fixed: chain_cuts. Adaptive: a
// game cut c times finishes by round steps + c, so the extra rounds past the
// most cuts any game used are empty launches, while a game that would need
// more than X cuts runs its last chain uncut (same results, but a round of up
// to ~10 ms that holds its group's NN launch). X follows the search two back
// (done by now: the previous one is still queued, so the read-back does not
// drain the queue): its most cuts and the fewest empty squares of its roots.
static int pick_extra_rounds(oamd_engine* e, int* X) {
    *X = extra_rounds(e);
    if (*X == 0 || !e->adapt_on) return OAMD_OK;
    if (int rc = e->ensure_cut_slots()) return rc;
    const int64_t q = e->adapt_seq - 2;
    const int s = q >= 0 ? (int)(q % oamd_engine::kCutSlots) : 0;
    if (q >= 0 && e->cut_x[s] >= 0) {
        int used = 0, empties = 64;
        for (int k = 0; k < e->cut_groups[s]; ++k) {
            HIPCHK(host_wait(e->cuts_ev[s][k]));
            used = std::max(used, (int)e->cuts_host[2 * (s * kMaxPipeline + k)]);
            empties = std::min(empties, (int)e->cuts_host[2 * (s * kMaxPipeline + k) + 1]);
        }
        // the cuts come with the endgame: outside it no chain outlasts the
        // budget (used = 0), within ~9 empty squares of the end a game's whole
        // search can be all terminal (used = 12 of 50 batches per thread at
        // budget 4; profiles/r04/ab/adaptive_demand_log.txt). The root loses
        // one empty square per move, so the fewest empties two searches back
        // announce the endgame before it starts; a search that needed cuts
        // raises the threshold past its root. Outside the endgame X = the
        // cuts used + the minimum, or 2X + 2 when a game ran out of cuts
        // (k_tree reports X + 1: X = 0 still counts the chains that would
        // have been split)
        // the raised threshold decays by one per search without cuts back to
        // kEndgameEmpties (a mid-game chain must not pin the full
        // count for the engine's lifetime)
        if (used > 0) e->adapt_empties = std::max(e->adapt_empties, empties + 3);
        else if (e->adapt_empties > oamd_engine::kEndgameEmpties) --e->adapt_empties;
        if (empties <= e->adapt_empties) e->adapt_x = e->chain_cuts;
        else e->adapt_x = (used > e->cut_x[s] ? 2 * e->cut_x[s] + 2 : used) + e->adapt_min;
        static const bool plog = getenv("OAMD_ADAPT_LOG") != nullptr;
        if (plog)
            fprintf(stderr, "adapt search %lld X %d used %d empties %d\n", (long long)q, e->cut_x[s], used, empties);
        e->cut_x[s] = -1;
    }
    // the first two searches (nothing read back yet) run the minimum: games
    // usually start from an opening, and a game that needs more cuts only
    // runs a longer round
    *X = e->adapt_x >= 0 ? std::clamp(e->adapt_x, std::min(e->adapt_min, *X), *X) : std::min(e->adapt_min, *X);
    return OAMD_OK;
}

// ResNet launches per group and round (the most of any group: nn_batch splits
// a group's rows into consecutive launches)
static int launches_per_group_round(const oamd_engine* e, const GroupPlan& P) {
    int n = 1;
    for (int k = 0; k < P.K; ++k) {
        const int grows = P.ng[k] * e->L(), cb = e->nn_batch > 0 ? e->nn_batch : grows;
        n = std::max(n, (grows + cb - 1) / cb);
    }
    return n;
}

// Sampled timing of one search: claim the current event pool (every
// timing_stride-th search), sized for NB blocks per round and `steps` NN
// rounds (steps + extra rounds) plus the final backup-only round.
static int timing_begin(oamd_engine* e, int steps, int NB, bool* timed) {
    *timed = e->timing && (e->search_count++ % e->timing_stride) == 0;
    if (!*timed) return OAMD_OK;
    const int pool = e->ev_cur;
    if (int rc = e->resolve_timing(pool)) return rc;

    while ((int)e->ev[pool].size() < kEvPerBlock * (steps + 1) * NB) {
        hipEvent_t x;
        HIPCHK(hipEventCreate(&x));
        e->ev[pool].push_back(x);
    }
    return OAMD_OK;
}

static void timing_end(oamd_engine* e, int steps, int NB, bool split, const GroupPlan& P) {
    const int pool = e->ev_cur;
    e->ev_blocks[pool] = (steps + 1) * NB;
    e->ev_final[pool] = steps * NB;
    e->ev_K[pool] = NB;
    e->ev_nn_groups[pool] = NB;
    int64_t nl = 0, rows = 0;
    if (split) {
        nl = e->cfg.num_threads;
        rows = e->L();
    }
    for (int k = 0; !split && k < e->ev_nn_groups[pool]; ++k) {
        const int grows = P.ng[k] * e->L(), cb = e->nn_batch > 0 ? e->nn_batch : grows;
        nl += (grows + cb - 1) / cb;
        rows += grows;
    }
    e->ev_launches[pool] = (int64_t)steps * nl;
    e->ev_rows[pool] = (int64_t)steps * rows;
    e->ev_cur ^= 1;
}

// Timing of R free-running rounds (every round has NN launches, none is a
// backup-only final round)
static void timing_end_rounds(oamd_engine* e, int R, const GroupPlan& P) {
    const int pool = e->ev_cur;
    e->ev_blocks[pool] = R * P.K;
    e->ev_final[pool] = R * P.K;
    e->ev_K[pool] = P.K;
    e->ev_nn_groups[pool] = P.K;
    int64_t nl = 0, rows = 0;
    for (int k = 0; k < P.K; ++k) {
        const int grows = P.ng[k] * e->L(), cb = e->nn_batch > 0 ? e->nn_batch : grows;
        nl += (grows + cb - 1) / cb;
        rows += grows;
    }
    e->ev_launches[pool] = (int64_t)R * nl;
    e->ev_rows[pool] = (int64_t)R * rows;
    e->ev_cur ^= 1;
}

// The rounds of one native search over the groups of P, enqueued on the group
// streams (already forked from the engine stream). chained: the groups'
// streams carry on from a previous search of the same call (a multi-move
// self-play call), so its first NN launch also waits for the NN token.

static int enqueue_group_rounds(oamd_engine* e, const NetView& N, const GroupPlan& P, int steps, int X, bool timed,
                                bool chained) {
    const EngineView E = e->view();
    const int K = P.K, L = e->L();
    const int T = e->cfg.num_threads, B = e->cfg.batch_size;
    const int pool = e->ev_cur;
    const int nch = e->nn_chains < K ? e->nn_chains : K;
    // chain splitting (k_tree): X extra rounds (pick_extra_rounds) absorb the
    // rounds a split chain delays its game by; only the reference's
    // interleaving has chains
    // (X = 0 picked by the adaptive count keeps the budget: k_tree reports
    // the chains it could not split)
    const bool splitting = extra_rounds(e) > 0;
    const int budget = splitting ? e->chain_budget : 0;
    const int S = steps + X;
    // adaptive X: each group's most cuts, into this search's slot
    const bool adapt = splitting && e->adapt_on;
    const int cs = (int)(e->adapt_seq % oamd_engine::kCutSlots);
    ++e->grouped_searches;
    e->grouped_rounds += S;
    if (adapt) {
        e->cut_x[cs] = X;
        e->cut_groups[cs] = K;
        ++e->adapt_seq;
    }
    // rounds 0..S (k_tree): round s backs up what the previous rounds selected
    // and selects, thread by thread; the NN evaluates round s's selections
    // between rounds s and s+1; the last round only backs up. A timed search
    // records events for every round, the extra ones included, and counts the
    // NN rows of every round (counters [4..5]): launches, rows and busy time
    // of a timed search cover the same launches (steps + X)
    const int nlg = launches_per_group_round(e, P);
    unsigned long long* span = nullptr;  // this search's busy-time slots (timing on)
    if (int rc = e->reserve_spans((int64_t)K * S * nlg, &span)) return rc;
    for (int s = 0; s <= S; ++s) {
        for (int k = 0; k < K; ++k) {
            const size_t r0 = (size_t)P.g0[k] * L;
            hipStream_t sk = P.st[k];
            hipEvent_t* ev = timed ? &e->ev[pool][kEvPerBlock * (s * K + k)] : nullptr;
            if (ev) HIPCHK(hipEventRecord(ev[0], sk));
            // evaluation list of group k: round s fills counter s % 2 and zeroes
            // the other one (which round s-1's launch, done by now, read); the
            // final round zeroes counter 0 for the next search's round 0
            int* cnt = e->rowcount + 2 * k;
            int* cuts = adapt ? e->cuts_dev + 2 * (cs * kMaxPipeline + k) : nullptr;
            launch_tree(E, sk, s > 0, s < S, T, B, P.g0[k], P.ng[k], 0, -1, s < S ? cnt + (s & 1) : nullptr,
                        s < S ? cnt + ((s + 1) & 1) : cnt, s == 0, budget, X, timed,
                        s == 0 || s == S ? cuts : nullptr);
            if (ev) HIPCHK(hipEventRecord(ev[1], sk));
            if (s == S) {
                if (adapt) {
                    HIPCHK(hipMemcpyAsync(e->cuts_host + 2 * (cs * kMaxPipeline + k), cuts, 2 * sizeof(int32_t),
                                          hipMemcpyDeviceToHost, sk));
                    HIPCHK(hipEventRecord(e->cuts_ev[cs][k], sk));
                }
                continue;
            }
            // the groups' NN launches run one after another (OAMD_NN_ORDER)
            hipStream_t ns = sk;
            if (K > 1 && OAMD_NN_ORDER == 2) {
                ns = e->nn_stream;
                HIPCHK(hipEventRecord(e->sel_ev[k], sk));
                HIPCHK(hipStreamWaitEvent(ns, e->sel_ev[k], 0));
            } else if (K > 1 && OAMD_NN_ORDER == 1 && (s > 0 || k >= nch || chained)) {
                HIPCHK(hipStreamWaitEvent(sk, e->nn_token[k % nch], 0));
            }
            if (ev) HIPCHK(hipEventRecord(ev[2], ns));
            const int grows = P.ng[k] * L;
            const int cb = e->nn_batch > 0 ? e->nn_batch : grows;
            // the extra rounds evaluate lagging games only: a small looping grid
            const int max_wgs = s >= steps ? e->extra_grid : 0;
            for (int r = 0, j = 0; r < grows; r += cb, ++j)
                launch_resnet_packed(N, E.feat, E.FW, E.H, std::min(cb, grows - r), E.policy, E.value, ns,
                                     E.rowlist + r0 + r, cnt + (s & 1), r,
                                     span ? span + (size_t)2 * ((k * S + s) * nlg + j) : nullptr, max_wgs);
            if (ev) HIPCHK(hipEventRecord(ev[3], ns));
            if (K > 1 && OAMD_NN_ORDER == 2) {
                HIPCHK(hipEventRecord(e->nn_ev[k], ns));
                HIPCHK(hipStreamWaitEvent(sk, e->nn_ev[k], 0));
            } else if (K > 1 && OAMD_NN_ORDER == 1) {
                HIPCHK(hipEventRecord(e->nn_token[k % nch], sk));
            }
        }
    }
    return OAMD_OK;
}

static int fork_groups(oamd_engine* e, const GroupPlan& P) {
    if (P.K > 1) {  // fork from the caller's stream
        HIPCHK(hipEventRecord(e->fork_ev, e->stream));
        for (int k = 0; k < P.K; ++k) HIPCHK(hipStreamWaitEvent(P.st[k], e->fork_ev, 0));
    }
    return OAMD_OK;
}

static int join_groups(oamd_engine* e, const GroupPlan& P) {
    if (P.K > 1) {  // join back into the caller's stream
        for (int k = 0; k < P.K; ++k) {
            HIPCHK(hipEventRecord(e->join_ev[k], P.st[k]));
            HIPCHK(hipStreamWaitEvent(e->stream, e->join_ev[k], 0));
        }
    }
    return OAMD_OK;
}

int oamd_engine_search(oamd_engine* e, oamd_net* net, int64_t* sims, int64_t* evals) {
    if (int rc = native_search_checks(e, net)) return rc;
    DeviceGuard dg(e->device);
    const int L = e->L();
    const int steps = (e->cfg.num_simulations + L - 1) / L;
    const EngineView E = e->view();
    const NetView N = net->view();
    GroupPlan P = plan_groups(e);
    const int K = P.K;
    const int T = e->cfg.num_threads, B = e->cfg.batch_size;
    // One game with T > 1 virtual threads (the drop-in MCTS, latency mode):
    // virtual thread t's tree operations (backup of its batch s-1 + selection
    // of batch s) and its ResNet launches alternate on a stream of its own, so
    // thread t's rows are evaluated while the tree kernel backs up and selects
    // for thread t+1 (the overlap the reference gets from its T threads,
    // search_thread.cpp:59-128). The tree operations keep the order of one
    // launch per round (thread 0 .. T-1, round by round) through an event
    // from each to the next, so results are identical; an operation waits
    // across streams only for the previous thread's tree operation, which ends
    // while this thread's ResNet launch still runs (a ResNet launch waiting
    // across streams for its selection, and a selection for its thread's
    // launch, each cost ~13 us of queue latency per round).
    const bool split = e->G == 1 && K == 1 && T > 1 && T <= kMaxPipeline && e->tree_split();
    const int NB = split ? T : K;  // timing blocks per round
    int rc = split ? e->ensure_streams(T, T) : e->ensure_streams(K, K);
    if (rc) return rc;
    if (!split) P = plan_groups(e);  // the group streams exist now
    if (sims || evals) HIPCHK(hipMemsetAsync(e->counters, 0, 2 * sizeof(unsigned long long), e->stream));
    // sampled timing: per (round, group) kEvPerBlock events: tree begin/end, NN
    // begin/end (on the NN stream, after its waits; not in the final round)
    bool timed = false;
    int X = 0;
    if (!split && (rc = pick_extra_rounds(e, &X))) return rc;
    const int rounds = steps + X;  // NN rounds
    if ((rc = timing_begin(e, rounds, NB, &timed))) return rc;
    const int pool = e->ev_cur;
    unsigned long long* span = nullptr;  // busy-time slots [thread][round] of the split schedule
    if (split && (rc = e->reserve_spans((int64_t)T * steps, &span))) return rc;
    if (split) {  // every thread stream after the caller's stream
        HIPCHK(hipEventRecord(e->fork_ev, e->stream));
        for (int t = 0; t < T; ++t) HIPCHK(hipStreamWaitEvent(e->pipe_stream[t], e->fork_ev, 0));
    }
    for (int s = 0; split && s <= steps; ++s) {
        for (int t = 0; t < T; ++t) {
            hipEvent_t* ev = timed ? &e->ev[pool][kEvPerBlock * (s * T + t)] : nullptr;
            hipStream_t ts = e->pipe_stream[t];  // after this thread's batch s-1 evaluation (stream order)
            if (s > 0 || t > 0)  // after the previous tree operation (thread t-1, or T-1 of round s-1)
                HIPCHK(hipStreamWaitEvent(ts, e->sel_ev[t > 0 ? t - 1 : T - 1], 0));
            if (ev) HIPCHK(hipEventRecord(ev[0], ts));
            launch_tree(E, ts, s > 0, s < steps, T, B, 0, 1, t, t + 1, nullptr, nullptr, s == 0, 0, 0, timed);
            if (ev) HIPCHK(hipEventRecord(ev[1], ts));
            HIPCHK(hipEventRecord(e->sel_ev[t], ts));
            if (s == steps) continue;
            if (ev) HIPCHK(hipEventRecord(ev[2], ts));
            launch_resnet_packed(N, E.feat + (size_t)t * B * E.FW, E.FW, E.H, B, E.policy + (size_t)t * B * 65,
                                 E.value + (size_t)t * B, ts, nullptr, nullptr, 0,
                                 span ? span + (size_t)2 * (t * steps + s) : nullptr);
            if (ev) HIPCHK(hipEventRecord(ev[3], ts));
        }
    }
    if (split) {  // the caller's stream after every thread stream
        for (int t = 0; t < T; ++t) {
            HIPCHK(hipEventRecord(e->join_ev[t], e->pipe_stream[t]));
            HIPCHK(hipStreamWaitEvent(e->stream, e->join_ev[t], 0));
        }
    }
    if (!split) {
        if ((rc = fork_groups(e, P))) return rc;
        if ((rc = enqueue_group_rounds(e, N, P, steps, X, timed, false))) return rc;
    }
    LAUNCHCHK();
    if (!split && (rc = join_groups(e, P))) return rc;
    if (timed) timing_end(e, rounds, NB, split, P);
    // without counters requested the search is left in flight (stream order)
    if (sims || evals) {
        unsigned long long c[2] = {0, 0};
        HIPCHK(hipMemcpyAsync(c, e->counters, sizeof(c), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        if (sims) *sims = (int64_t)c[0];
        if (evals) *evals = (int64_t)c[1];
    }
    e->step_phase = 0;
    e->steps_left = 0;
    return OAMD_OK;
}

int oamd_engine_work_counters(oamd_engine* e, int64_t* sims, int64_t* evals) {
    DeviceGuard dg(e->device);
    unsigned long long c[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(c, e->counters + 2, sizeof(c), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (sims) *sims = (int64_t)c[0];
    if (evals) *evals = (int64_t)c[1];
    return OAMD_OK;
}

int oamd_engine_descent_depths(oamd_engine* e, int64_t* leaves, int64_t* depth_sum, int32_t* depth_max) {
    DeviceGuard dg(e->device);
    unsigned long long c[kCounters] = {};
    HIPCHK(hipMemcpyAsync(c, e->counters, sizeof(c), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (leaves) *leaves = (int64_t)c[2];
    if (depth_sum) *depth_sum = (int64_t)c[6];
    if (depth_max) *depth_max = (int32_t)c[7];
    return OAMD_OK;
}

int oamd_engine_tree_work(oamd_engine* e, int64_t* levels, int64_t* scanned, int64_t* expansions, int64_t* created,
                          int64_t* launches) {
    DeviceGuard dg(e->device);
    unsigned long long c[kCounters] = {};
    HIPCHK(hipMemcpyAsync(c, e->counters, sizeof(c), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (levels) *levels = (int64_t)c[6];
    if (scanned) *scanned = (int64_t)c[8];
    if (expansions) *expansions = (int64_t)c[9];
    if (created) *created = (int64_t)c[10];
    if (launches) *launches = (int64_t)c[11];
    return OAMD_OK;
}

int oamd_engine_set_pipeline(oamd_engine* e, int32_t groups) {
    if (groups < 0 || groups > kMaxPipeline)
        return fail(OAMD_INVALID_ARGUMENT, "pipeline groups must be in [0, " + std::to_string(kMaxPipeline) + "]");
    e->pipeline = groups;
    return OAMD_OK;
}

int oamd_debug_read_stamps(uint64_t* out, int64_t n) {
    if (!out || n < 0) return fail(OAMD_INVALID_ARGUMENT, "stamps: bad buffer");
    const int rc = resnet_read_stamps(reinterpret_cast<unsigned long long*>(out), (long long)n);
    if (rc == -2) return fail(OAMD_INVALID_ARGUMENT, "built without OAMD_STAMPS");
    return rc ? fail(OAMD_RUNTIME, "stamp copy failed") : OAMD_OK;
}

int oamd_debug_tree_stamps(uint64_t* out, int64_t n, int32_t reset) {
    if (!out || n < 0) return fail(OAMD_INVALID_ARGUMENT, "tree stamps: bad buffer");
    const int rc = tree_read_stamps(reinterpret_cast<unsigned long long*>(out), (long long)n, reset);
    if (rc == -2) return fail(OAMD_INVALID_ARGUMENT, "built without OAMD_TREE_STAMPS");
    return rc ? fail(OAMD_RUNTIME, "tree stamp copy failed") : OAMD_OK;
}

int oamd_engine_set_nn_chains(oamd_engine* e, int32_t chains) {
    if (chains < 1 || chains > oamd_engine::kMaxChains)
        return fail(OAMD_INVALID_ARGUMENT, "nn chains must be in [1, " + std::to_string(oamd_engine::kMaxChains) + "]");
    e->nn_chains = chains;
    return OAMD_OK;
}

int oamd_engine_set_chain_split(oamd_engine* e, int32_t budget, int32_t cuts) {
    if (budget < 0 || cuts < 0 || cuts > 64) return fail(OAMD_INVALID_ARGUMENT, "chain split: budget >= 0, cuts in [0, 64]");
    e->chain_budget = budget;
    e->chain_cuts = cuts;
    return OAMD_OK;
}

int oamd_engine_set_adaptive_extra_rounds(oamd_engine* e, int32_t enable, int32_t min_rounds) {
    if (min_rounds < 0 || min_rounds > 64) return fail(OAMD_INVALID_ARGUMENT, "adaptive extra rounds: min in [0, 64]");
    e->adapt_on = enable != 0;
    e->adapt_min = min_rounds;
    e->adapt_x = -1;  // the next two searches run the minimum
    e->adapt_empties = oamd_engine::kEndgameEmpties;
    for (int& x : e->cut_x) x = -1;
    return OAMD_OK;
}

int oamd_engine_round_counts(const oamd_engine* ce, int64_t* searches, int64_t* rounds, int64_t* final_launches) {
    oamd_engine* e = const_cast<oamd_engine*>(ce);  // pending events are summed here
    if (int rc = e->resolve_all_timing()) return rc;
    if (searches) *searches = e->grouped_searches;
    if (rounds) *rounds = e->grouped_rounds;
    if (final_launches) *final_launches = e->tree_final_launches;
    return OAMD_OK;
}

int oamd_engine_set_extra_round_grid(oamd_engine* e, int32_t workgroups) {
    if (workgroups < 0) return fail(OAMD_INVALID_ARGUMENT, "extra-round grid must be >= 0");
    e->extra_grid = workgroups;
    return OAMD_OK;
}

int oamd_engine_set_exact_interleaving(oamd_engine* e, int32_t enable) {
    e->exact_interleaving = enable != 0;
    return OAMD_OK;
}

int oamd_engine_set_nn_batch(oamd_engine* e, int32_t rows) {
    if (rows < 0) return fail(OAMD_INVALID_ARGUMENT, "nn batch rows must be >= 0");
    e->nn_batch = rows;
    return OAMD_OK;
}

int oamd_engine_root_info(oamd_engine* e, int32_t game, oamd_root_info* info, int32_t* visits, float* q) {
    if (game < 0 || game >= e->G) return fail(OAMD_OUT_OF_RANGE, "game index out of range");
    DeviceGuard dg(e->device);
    launch_root_stats(e->view(), game, 1, e->info_dev, e->visits_dev, e->q_dev, 0, e->stream);
    LAUNCHCHK();
    oamd_root_info tmp;
    HIPCHK(hipMemcpyAsync(&tmp, e->info_dev, sizeof(tmp), hipMemcpyDeviceToHost, e->stream));
    int32_t v[65];
    float qq[65];
    HIPCHK(hipMemcpyAsync(v, e->visits_dev, sizeof(v), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(qq, e->q_dev, sizeof(qq), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (info) *info = tmp;
    const int nc = tmp.num_children;
    if (visits) std::memcpy(visits, v, sizeof(int32_t) * nc);
    if (q) std::memcpy(q, qq, sizeof(float) * nc);
    return OAMD_OK;
}

int oamd_engine_status(oamd_engine* e, int32_t* overflow_games, int32_t* depth_capped_games) {
    DeviceGuard dg(e->device);
    HIPCHK(hipMemsetAsync(e->status_dev, 0, 2 * sizeof(int32_t), e->stream));
    launch_status(e->view(), e->status_dev, e->stream);
    LAUNCHCHK();
    int32_t h[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(h, e->status_dev, sizeof(h), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (overflow_games) *overflow_games = h[0];
    if (depth_capped_games) *depth_capped_games = h[1];
    return OAMD_OK;
}

int oamd_engine_root_stats(oamd_engine* e, int32_t* visits_dev, float* q_dev, oamd_root_info* info_dev) {
    DeviceGuard dg(e->device);
    launch_root_stats(e->view(), 0, e->G, info_dev ? info_dev : e->info_dev, visits_dev ? visits_dev : e->visits_dev,
                      q_dev ? q_dev : e->q_dev, 1, e->stream);
    LAUNCHCHK();
    return OAMD_OK;
}

int oamd_engine_self_play_data(oamd_engine* e, int32_t game, float* features, float* policy) {
    oamd_root_info info;
    int rc = oamd_engine_root_info(e, game, &info, nullptr, nullptr);
    if (rc) return rc;
    if (info.position.player == 0)
        return fail(OAMD_INVALID_ARGUMENT, "Self-play data cannot be generated from a terminal position.");
    if (info.num_children == 0) return fail(OAMD_INVALID_ARGUMENT, "The root node has not been expanded yet.");
    DeviceGuard dg(e->device);
    const int C = 1 + 2 * e->cfg.history_size;
    float* fd = e->spd_dev;
    float* pd = e->spd_dev + (size_t)8 * C * 64;
    launch_self_play_data(e->view(), game, fd, pd, e->stream);
    LAUNCHCHK();
    HIPCHK(hipMemcpyAsync(features, fd, sizeof(float) * 8 * C * 64, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(policy, pd, sizeof(float) * 8 * 65, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return OAMD_OK;
}

int oamd_engine_apply_action(oamd_engine* e, int32_t game, int32_t action) {
    if (game < 0 || game >= e->G) return fail(OAMD_OUT_OF_RANGE, "game index out of range");
    if (!(0 <= action && action < 65))
        return fail(OAMD_OUT_OF_RANGE, "Expected 0 <= action < 65, but got " + std::to_string(action) + ".");
    oamd_root_info info;
    int rc = oamd_engine_root_info(e, game, &info, nullptr, nullptr);
    if (rc) return rc;
    if (action == 64) {
        if (info.position.player == 0)
            return fail(OAMD_INVALID_ARGUMENT, "Pass is not allowed in a terminal position.");
        if (info.position.legal_moves != 0)
            return fail(OAMD_INVALID_ARGUMENT, "Pass is not allowed when there are legal moves.");
    } else if (((1ULL << (63 - action)) & info.position.legal_moves) == 0) {
        return fail(OAMD_INVALID_ARGUMENT, std::to_string(action) + " is not a legal action.");
    }
    if (info.node_count + 1 > e->cap) return fail(OAMD_CAPACITY, "node pool exhausted");
    DeviceGuard dg(e->device);
    launch_apply_one(e->view(), game, action, e->stream);
    LAUNCHCHK();
    return OAMD_OK;
}

int oamd_engine_apply_actions(oamd_engine* e, const int32_t* actions_dev) {
    DeviceGuard dg(e->device);
    launch_apply_actions(e->view(), actions_dev, e->stream);
    LAUNCHCHK();
    return OAMD_OK;
}

int oamd_engine_selfplay_move(oamd_engine* e, const oamd_selfplay_config* cfg, int32_t* actions_dev,
                              int32_t* finished_dev, float* features_dev, float* policy_dev) {
    if (cfg->temperature_moves < 0 || !(cfg->temperature > 0.0f) || cfg->opening_moves < 0)
        return fail(OAMD_INVALID_ARGUMENT, "bad self-play config");
    if (cfg->emit_targets && (!features_dev || !policy_dev))
        return fail(OAMD_INVALID_ARGUMENT, "emit_targets needs features and policy buffers");
    SelfplayParams sp{cfg->temperature_moves, cfg->temperature, cfg->opening_moves, cfg->emit_targets};
    DeviceGuard dg(e->device);
    launch_selfplay_move(e->view(), sp, 0, e->G, actions_dev, finished_dev, features_dev, policy_dev, e->stream);
    LAUNCHCHK();
    return OAMD_OK;
}

// Free-running self-play: n_moves moves of every game, each game on its own
// (tree.hip k_tree_free). Rounds are enqueued in chunks: one per move's worth
// of rounds (steps + 1 for the first search, steps for each later one: a
// schedule estimate only — a search whose batches are all terminal can
// re-select several times in one round and finish sooner, and such a game
// simply plays its next move in the same call), then tail chunks of
// kFreeTailRounds rounds until the group's remaining-games counter, copied to
// pinned memory after every chunk and read two chunks late (so the read never
// drains the queue), is 0. The
// tail chunks' ResNet launches use the small looping grid (extra_grid): only
// lagging games have rows then. Returns once the last chunk is enqueued.
static int selfplay_steps_free(oamd_engine* e, oamd_net* net, const oamd_selfplay_config* cfg, int n_moves,
                               int per_move, int32_t* actions, int32_t* finished, float* feat, float* pol) {
    if (int rc = e->ensure_free_slots()) return rc;
    GroupPlan P = plan_groups(e);
    const int K = P.K, L = e->L();
    const int T = e->cfg.num_threads, B = e->cfg.batch_size;
    const int steps = (e->cfg.num_simulations + L - 1) / L;
    const EngineView E = e->view();
    const NetView N = net->view();
    const SelfplayParams sp{cfg->temperature_moves, cfg->temperature, cfg->opening_moves, cfg->emit_targets};
    const int budget = e->exact_interleaving && e->chain_budget > 0 ? e->chain_budget : 0;
    const int nch = e->nn_chains < K ? e->nn_chains : K;
    const int nlg = launches_per_group_round(e, P);
    if (int rc = fork_groups(e, P)) return rc;
    int64_t round = 0;
    // everything between the fork and the join; on an error the groups are
    // still joined into the caller's stream, so that nothing the caller
    // enqueues next overlaps the rounds already in the group streams
    auto rounds = [&]() -> int {
        for (int k = 0; k < K; ++k) {
            HIPCHK(hipMemsetAsync(e->rowcount + 2 * k, 0, 2 * sizeof(int32_t), P.st[k]));
            HIPCHK(hipMemsetAsync(e->remaining_dev + k, 0, sizeof(int32_t), P.st[k]));
            launch_free_begin(E, P.g0[k], P.ng[k], n_moves, e->remaining_dev + k, actions, finished, per_move, P.st[k]);
        }
        bool gdone[kMaxPipeline] = {};
        const int64_t base_rounds = n_moves > 0 ? (int64_t)n_moves * steps + 1 : 0;
        // a round completes at least one batch of every game still playing (or
        // its move): a generous bound that only a kernel fault could exceed
        const int64_t max_rounds = base_rounds + (int64_t)n_moves * ((int64_t)T * steps + 2) + 4 * oamd_engine::kFreeTailRounds;
        for (int64_t chunk = 0; n_moves > 0; ++chunk) {
            int R;
            const bool tail = round >= base_rounds;
            if (!tail) {
                R = (int)std::min<int64_t>(round == 0 ? steps + 1 : steps, base_rounds - round);
                // keep at most two chunks (~two moves of GPU work) queued ahead:
                // wait (blocking, the thread sleeps) for chunk - 2 to finish.
                // Enqueuing every move at once filled the hardware queues and
                // the host spun a CPU in the launch calls for the whole call
                // (host budget)
                if (chunk >= 2 && e->throttle_enqueue) {
                    const int slot = (int)((chunk - 2) % oamd_engine::kFreeSlots);
                    for (int k = 0; k < K; ++k) HIPCHK(host_wait(e->free_ev[slot][k]));
                }
            } else {
                if (chunk >= 2) {  // chunk - 2's readback: done by now while chunk - 1 is queued
                    const int slot = (int)((chunk - 2) % oamd_engine::kFreeSlots);
                    for (int k = 0; k < K; ++k) {
                        if (gdone[k]) continue;
                        HIPCHK(host_wait(e->free_ev[slot][k]));
                        if (e->remaining_host[slot * kMaxPipeline + k] == 0) gdone[k] = true;
                    }
                }
                bool all = true;
                for (int k = 0; k < K; ++k) all = all && gdone[k];
                if (all) break;
                if (round >= max_rounds) return fail(OAMD_RUNTIME, "free-running self-play did not finish");
                R = oamd_engine::kFreeTailRounds;
            }
            bool timed = false;
            if (!tail) {
                if (int rc = timing_begin(e, R, K, &timed)) return rc;
            }
            const int pool = e->ev_cur;
            unsigned long long* span = nullptr;
            if (int rc = e->reserve_spans((int64_t)K * R * nlg, &span)) return rc;
            for (int s = 0; s < R; ++s) {
                const int64_t r = round + s;
                for (int k = 0; k < K; ++k) {
                    if (gdone[k]) continue;
                    hipStream_t sk = P.st[k];
                    hipEvent_t* ev = timed ? &e->ev[pool][kEvPerBlock * (s * K + k)] : nullptr;
                    int* cnt = e->rowcount + 2 * k;
                    if (ev) HIPCHK(hipEventRecord(ev[0], sk));
                    launch_tree_free(E, sk, P.g0[k], P.ng[k], B, cnt + (r & 1), cnt + ((r + 1) & 1), budget, timed, sp,
                                     n_moves, per_move, actions, finished, feat, pol, e->remaining_dev + k);
                    if (ev) HIPCHK(hipEventRecord(ev[1], sk));
                    if (K > 1 && (r > 0 || k >= nch)) HIPCHK(hipStreamWaitEvent(sk, e->nn_token[k % nch], 0));
                    if (ev) HIPCHK(hipEventRecord(ev[2], sk));
                    const int grows = P.ng[k] * L;
                    const int cb = e->nn_batch > 0 ? e->nn_batch : grows;
                    const size_t r0 = (size_t)P.g0[k] * L;
                    for (int rr = 0, j = 0; rr < grows; rr += cb, ++j)
                        launch_resnet_packed(N, E.feat, E.FW, E.H, std::min(cb, grows - rr), E.policy, E.value, sk,
                                             E.rowlist + r0 + rr, cnt + (r & 1), rr,
                                             span ? span + (size_t)2 * ((k * R + s) * nlg + j) : nullptr,
                                             tail ? e->extra_grid : 0);
                    if (ev) HIPCHK(hipEventRecord(ev[3], sk));
                    if (K > 1) HIPCHK(hipEventRecord(e->nn_token[k % nch], sk));
                }
            }
            const int slot = (int)(chunk % oamd_engine::kFreeSlots);
            for (int k = 0; k < K; ++k) {
                if (gdone[k]) continue;
                HIPCHK(hipMemcpyAsync(e->remaining_host + slot * kMaxPipeline + k, e->remaining_dev + k, sizeof(int32_t),
                                      hipMemcpyDeviceToHost, P.st[k]));
                HIPCHK(hipEventRecord(e->free_ev[slot][k], P.st[k]));
            }
            if (timed) timing_end_rounds(e, R, P);
            round += R;
        }
        // the next search (or call) starts with empty evaluation lists
        for (int k = 0; k < K; ++k) HIPCHK(hipMemsetAsync(e->rowcount + 2 * k, 0, 2 * sizeof(int32_t), P.st[k]));
        LAUNCHCHK();
        return OAMD_OK;
    };
    const int rc = rounds();
    const int jrc = join_groups(e, P);
    e->step_phase = 0;
    e->steps_left = 0;
    if (rc) return rc;
    e->grouped_searches += n_moves;
    e->grouped_rounds += round;
    return jrc;
}

int oamd_engine_set_free_running(oamd_engine* e, int32_t enable) {
    e->free_running = enable != 0;
    return OAMD_OK;
}

int oamd_engine_selfplay_steps(oamd_engine* e, oamd_net* net, const oamd_selfplay_config* cfg, int32_t n_moves,
                               int32_t per_move_outputs, int32_t* actions_dev, int32_t* finished_dev,
                               float* features_dev, float* policy_dev) {
    if (n_moves < 0) return fail(OAMD_INVALID_ARGUMENT, "n_moves must be >= 0");
    if (cfg->temperature_moves < 0 || !(cfg->temperature > 0.0f) || cfg->opening_moves < 0)
        return fail(OAMD_INVALID_ARGUMENT, "bad self-play config");
    if (cfg->emit_targets && (!features_dev || !policy_dev))
        return fail(OAMD_INVALID_ARGUMENT, "emit_targets needs features and policy buffers");
    if (int rc = native_search_checks(e, net)) return rc;
    DeviceGuard dg(e->device);
    const int G = e->G, C = 1 + 2 * e->cfg.history_size;
    // move i's outputs: the i-th slice of per-move buffers, or the same G-game buffers every move
    auto out = [&](int i, auto* p, int64_t per_game) { return p ? p + (per_move_outputs ? (int64_t)i * G * per_game : 0) : p; };
    GroupPlan P = plan_groups(e);
    const int T = e->cfg.num_threads;
    const bool split = G == 1 && P.K == 1 && T > 1 && T <= kMaxPipeline && e->tree_split();
    if (!split && e->free_running) {
        if (int rc = e->ensure_streams(P.K, P.K)) return rc;
        return selfplay_steps_free(e, net, cfg, n_moves, per_move_outputs, actions_dev, finished_dev, features_dev,
                                   policy_dev);
    }
    if (split || P.K == 1) {  // one stream: the plain sequence of calls
        for (int i = 0; i < n_moves; ++i) {
            if (int rc = oamd_engine_search(e, net, nullptr, nullptr)) return rc;
            if (int rc = oamd_engine_selfplay_move(e, cfg, out(i, actions_dev, 1), out(i, finished_dev, 1),
                                                   out(i, features_dev, 8 * C * 64), out(i, policy_dev, 8 * 65)))
                return rc;
        }
        return OAMD_OK;
    }
    if (int rc = e->ensure_streams(P.K, P.K)) return rc;
    P = plan_groups(e);
    const int L = e->L();
    const int steps = (e->cfg.num_simulations + L - 1) / L;
    const EngineView E = e->view();
    const NetView N = net->view();
    SelfplayParams sp{cfg->temperature_moves, cfg->temperature, cfg->opening_moves, cfg->emit_targets};
    // Each group runs its own chain of searches and moves on its stream: its
    // move and the next search's first selection overlap the other groups'
    // last ResNet launches instead of waiting for a join after every move.
    // Per game the kernels and their order are those of search + move calls.
    int rc = fork_groups(e, P);
    for (int i = 0; !rc && i < n_moves; ++i) {
        bool timed = false;
        int X = 0;
        if ((rc = pick_extra_rounds(e, &X))) break;
        if ((rc = timing_begin(e, steps + X, P.K, &timed))) break;
        if ((rc = enqueue_group_rounds(e, N, P, steps, X, timed, i > 0))) break;
        for (int k = 0; k < P.K; ++k)
            launch_selfplay_move(E, sp, P.g0[k], P.ng[k], out(i, actions_dev, 1), out(i, finished_dev, 1),
                                 out(i, features_dev, 8 * C * 64), out(i, policy_dev, 8 * 65), P.st[k]);
        if (timed) timing_end(e, steps + X, P.K, false, P);
    }
    if (rc) return rc;
    LAUNCHCHK();
    if ((rc = join_groups(e, P))) return rc;
    e->step_phase = 0;
    e->steps_left = 0;
    return OAMD_OK;
}

int oamd_engine_random_openings(oamd_engine* e, int32_t max_moves, uint64_t seed) {
    if (max_moves < 0) return fail(OAMD_INVALID_ARGUMENT, "max_moves must be >= 0");
    DeviceGuard dg(e->device);
    launch_random_openings(e->view(), max_moves, seed, e->stream);
    LAUNCHCHK();
    return OAMD_OK;
}

int oamd_engine_game_key(oamd_engine* e, int32_t game, uint64_t* key) {
    if (game < 0 || game >= e->G) return fail(OAMD_OUT_OF_RANGE, "game index out of range");
    DeviceGuard dg(e->device);
    HIPCHK(hipMemcpyAsync(key, &e->games[game].key, sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return OAMD_OK;
}

}  // extern "C"
