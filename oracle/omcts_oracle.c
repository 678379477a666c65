/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see omcts_oracle.h). Plain-C restatement
 * of the reference othello_mcts path; every function cites the reference
 * file:line it follows. Compiled with -ffp-contract=off (see Makefile).
 */
#include "omcts_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================= */
/* Bitboards — position.h                                                  */
/* ======================================================================= */

/* position.h:155-172 */
#define NO_LR 0x7E7E7E7E7E7E7E7EULL
#define NO_TB 0x00FFFFFFFFFFFF00ULL
#define NO_EDGE (NO_LR & NO_TB)

/* position.h:153 STRIDES = {-9,-8,-7,-1,1,7,8,9}; positive stride = >>, negative = << */
static const int k_stride[8] = {-9, -8, -7, -1, 1, 7, 8, 9};
static const uint64_t k_mask[8] = {NO_EDGE, NO_TB, NO_EDGE, NO_LR, NO_LR, NO_EDGE, NO_TB, NO_EDGE};

static uint64_t shift_dir(uint64_t m, int d) {
    int s = k_stride[d];
    return s > 0 ? (m >> s) : (m << (-s));
}

/* position.h:186-196: seed run + 5 propagation steps */
static uint64_t potential_flips(uint64_t seed, uint64_t opp, int d) {
    uint64_t o = opp & k_mask[d];
    uint64_t f = o & shift_dir(seed, d);
    for (int i = 0; i < 5; ++i) f |= o & shift_dir(f, d);
    return f;
}

/* position.h:202-229 */
uint64_t orc_get_legal_moves(uint64_t me, uint64_t opp) {
    uint64_t legal = 0;
    for (int d = 0; d < 8; ++d) legal |= shift_dir(potential_flips(me, opp, d), d);
    return legal & ~(me | opp);
}

/* position.h:231-262 */
uint64_t orc_get_flips(uint64_t move, uint64_t me, uint64_t opp) {
    uint64_t flips = 0;
    for (int d = 0; d < 8; ++d) {
        uint64_t f = potential_flips(move, opp, d);
        if (shift_dir(f, d) & me) flips |= f;
    }
    return flips;
}

/* position.h:264-272 */
void orc_initial_position(orc_pos *out) {
    out->player = 1;
    out->p1 = 0x0000000810000000ULL;
    out->p2 = 0x0000001008000000ULL;
    out->legal = orc_get_legal_moves(out->p1, out->p2);
    out->next_legal = 0;
}

/* position.h:328-363 (move), 382-386 (pass), 402-408 (dispatch) */
void orc_apply_action(const orc_pos *p, int action, orc_pos *out) {
    if (action == 64) {
        out->player = 3 - p->player;
        out->p1 = p->p1;
        out->p2 = p->p2;
        out->legal = p->next_legal;
        out->next_legal = 0;
        return;
    }
    uint64_t move = 1ULL << (63 - action);
    uint64_t p1 = p->p1, p2 = p->p2;
    uint64_t *me = p->player == 1 ? &p1 : &p2;
    uint64_t *opp = p->player == 1 ? &p2 : &p1;
    uint64_t flips = orc_get_flips(move, *me, *opp);
    *me |= move | flips;
    *opp &= ~flips;
    int player = 3 - p->player;
    uint64_t legal = orc_get_legal_moves(*opp, *me);
    uint64_t next_legal = 0;
    if (legal == 0) {
        next_legal = orc_get_legal_moves(*me, *opp);
        if (next_legal == 0) player = 0;
    }
    out->player = player;
    out->p1 = p1;
    out->p2 = p2;
    out->legal = legal;
    out->next_legal = next_legal;
}

/* position.h:308-326 */
int orc_legal_actions(const orc_pos *p, int32_t *actions_out) {
    if (p->player == 0) return 0;
    if (p->legal == 0) {
        actions_out[0] = 64;
        return 1;
    }
    int n = 0;
    for (int a = 0; a < 64; ++a)
        if (p->legal & (1ULL << (63 - a))) actions_out[n++] = a;
    return n;
}

void orc_legal_moves_n(const uint64_t *me, const uint64_t *opp, uint64_t *out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) out[i] = orc_get_legal_moves(me[i], opp[i]);
}

void orc_flips_n(const uint64_t *mv, const uint64_t *me, const uint64_t *opp, uint64_t *out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) out[i] = orc_get_flips(mv[i], me[i], opp[i]);
}

void orc_apply_action_n(const int32_t *player, const uint64_t *p1, const uint64_t *p2,
                        const uint64_t *legal, const uint64_t *next_legal, const int32_t *action,
                        int32_t *o_player, uint64_t *o_p1, uint64_t *o_p2, uint64_t *o_legal,
                        uint64_t *o_next, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        orc_pos p = {player[i], p1[i], p2[i], legal[i], next_legal[i]}, c;
        orc_apply_action(&p, action[i], &c);
        o_player[i] = c.player;
        o_p1[i] = c.p1;
        o_p2[i] = c.p2;
        o_legal[i] = c.legal;
        o_next[i] = c.next_legal;
    }
}

/* transformation.h:40-57: optional horizontal flip (t odd), then t/2
 * clockwise rotations (row,col) -> (col, 7-row); pass is fixed. */
int orc_transform_action(int action, int t) {
    if (action == 64) return 64;
    int row = action / 8, col = action % 8;
    if (t % 2 == 1) col = 7 - col;
    for (int i = 0; i < t / 2; ++i) {
        int r = row;
        row = col;
        col = 7 - r;
    }
    return row * 8 + col;
}

/* transformation.h:83-116 */
void orc_features(const orc_pos *chain, int n_chain, int history_size, int t, float *out) {
    float plane0 = (float)chain[0].player - 1.0f;
    for (int s = 0; s < 64; ++s) out[s] = plane0;
    out += 64;
    for (int i = 0; i < history_size; ++i) {
        if (i >= n_chain) {
            memset(out, 0, 128 * sizeof(float));
        } else {
            for (int s = 0; s < 64; ++s) {
                int ts = orc_transform_action(s, t);
                uint64_t m = 1ULL << (63 - s);
                out[ts] = (chain[i].p1 & m) ? 1.0f : 0.0f;
                out[64 + ts] = (chain[i].p2 & m) ? 1.0f : 0.0f;
            }
        }
        out += 128;
    }
}

/* ======================================================================= */
/* Random streams — DESIGN.md "Random streams". Replaces the reference's    */
/* std::mt19937 + std::gamma_distribution (search_thread.h:77-79,         */
/* search_thread.cpp:22-24, draws at :92 and :233)                          */
/* ======================================================================= */

#define GOLDEN 0x9E3779B97F4A7C15ULL
#define EVENT_MUL 0xD1B54A32D192ED03ULL

uint64_t orc_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

uint64_t orc_stream_key(uint64_t game_key, uint64_t event, uint32_t sub) {
    return orc_mix64(orc_mix64(game_key ^ (event * EVENT_MUL)) + (uint64_t)(sub + 1) * GOLDEN);
}

/* exact float in (0,1): (2m+1) * 2^-24, m = top 23 bits */
float orc_uniform(uint64_t stream_key, uint32_t k) {
    uint64_t x = orc_mix64(stream_key + (uint64_t)(k + 1) * GOLDEN);
    uint32_t m = (uint32_t)(x >> 41);
    return (float)(2u * m + 1u) * 5.9604644775390625e-08f;
}

static float as_float(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static uint32_t as_uint(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

/* Portable natural log for positive normal floats (spec, not libm). */
float orc_logf(float x) {
    uint32_t b = as_uint(x);
    int e = (int)((b >> 23) & 0xffu) - 127;
    float m = as_float((b & 0x7fffffu) | 0x3f800000u);
    if (m > 1.41421356f) {
        m = m * 0.5f;
        e = e + 1;
    }
    float s = (m - 1.0f) / (m + 1.0f);
    float s2 = s * s;
    float p = 0.0909090936f;            /* 1/11 */
    p = 0.111111112f + s2 * p;          /* 1/9 */
    p = 0.142857149f + s2 * p;          /* 1/7 */
    p = 0.200000003f + s2 * p;          /* 1/5 */
    p = 0.333333343f + s2 * p;          /* 1/3 */
    float t = s2 * p;
    float logm = 2.0f * s + (2.0f * s) * t;
    float fe = (float)e;
    return fe * 0.693145752f + (fe * 1.42860677e-06f + logm);
}

/* Portable exp (spec, not libm); flushes below 2^-126 to 0. */
float orc_expf(float x) {
    if (x < -87.0f) return 0.0f;
    if (x > 88.0f) return as_float(0x7f800000u);
    float kf = floorf(x * 1.44269502f + 0.5f);
    int k = (int)kf;
    float r = (x - kf * 0.693145752f) - kf * 1.42860677e-06f;
    float p = 0.00138888892f;           /* 1/720 */
    p = 0.00833333377f + r * p;         /* 1/120 */
    p = 0.0416666679f + r * p;          /* 1/24 */
    p = 0.166666672f + r * p;           /* 1/6 */
    p = 0.5f + r * p;
    p = 1.0f + r * p;
    p = 1.0f + r * p;
    if (k < -126) return 0.0f;
    return p * as_float((uint32_t)(k + 127) << 23);
}

/* cos^2(2 pi v), v in (0,1), folded to [0, pi/4] (rng.h cos2pi_sq) */
float orc_cos2pi_sq(float v) {
    float t = 2.0f * v;
    t = t - floorf(t);
    if (t > 0.5f) t = 1.0f - t;
    float c;
    if (t < 0.25f) {
        float x = 3.14159274f * t;
        float x2 = x * x;
        c = 1.0f + x2 * (-0.5f + x2 * (0.0416666679f + x2 * (-0.00138888892f + x2 * 2.48015876e-05f)));
    } else {
        float x = 3.14159274f * (0.5f - t);
        float x2 = x * x;
        c = x * (1.0f + x2 * (-0.166666672f + x2 * (0.00833333377f + x2 * -0.000198412701f)));
    }
    return c * c;
}

/* Gamma(alpha,1). alpha = 1/2: Z^2/2 in Box-Muller form, -ln(U) cos^2(2 pi V)
 * (no rejection). Otherwise Marsaglia–Tsang; alpha<1 via the U^(1/alpha)
 * boost; normal deviates by the Marsaglia polar method. Every loop is bounded
 * so the GPU wave always terminates; the bounded fallbacks are part of the
 * spec. (rng.h gamma_draw) */
float orc_gamma(uint64_t key, float alpha) {
    if (!(alpha > 0.0f)) return 0.0f;
    if (alpha == 0.5f) return -orc_logf(orc_uniform(key, 0)) * orc_cos2pi_sq(orc_uniform(key, 1));
    uint32_t k = 0;
    int boost = alpha < 1.0f;
    float a = boost ? alpha + 1.0f : alpha;
    float d = a - 0.333333343f;
    float c = 1.0f / sqrtf(9.0f * d);
    float g = d;
    for (int it = 0; it < 16; ++it) {
        float u = 0.0f, s = 0.5f;
        int ok = 0;
        for (int j = 0; j < 16; ++j) {
            float uu = 2.0f * orc_uniform(key, k) - 1.0f;
            float vv = 2.0f * orc_uniform(key, k + 1) - 1.0f;
            k += 2;
            float ss = uu * uu + vv * vv;
            if (ss < 1.0f && ss > 0.0f) {
                u = uu;
                s = ss;
                ok = 1;
                break;
            }
        }
        if (!ok) u = 0.5f;
        float x = u * sqrtf((-2.0f * orc_logf(s)) / s);
        float v = 1.0f + c * x;
        if (v <= 0.0f) continue;
        v = (v * v) * v;
        float uu = orc_uniform(key, k);
        k += 1;
        float x2 = x * x;
        float x4 = x2 * x2;
        if (uu < 1.0f - 0.0331f * x4) {
            g = d * v;
            break;
        }
        if (orc_logf(uu) < 0.5f * x2 + d * ((1.0f - v) + orc_logf(v))) {
            g = d * v;
            break;
        }
    }
    if (boost) {
        float ub = orc_uniform(key, 63);
        g = g * orc_expf(orc_logf(ub) / alpha);
    }
    return g;
}

/* ======================================================================= */
/* MCTS — search_node.h, search_thread.cpp, mcts.h/.cpp                     */
/* ======================================================================= */

typedef struct {
    orc_pos pos;
    int32_t parent;      /* -1 for the initial position (search_node.h:20) */
    int32_t first_child; /* children are contiguous (legal_actions order) */
    int32_t n_children;
    int32_t n;           /* visit_count       search_node.h:28 */
    float w;             /* total_action_value */
    float q;             /* mean_action_value */
    float p;             /* prior_probability, default 1.0f (search_node.h:40) */
} onode;

struct orc_mcts {
    int history_size, num_simulations, num_threads, batch_size;
    float c_puct_base, c_puct_init, eps, alpha;
    onode *nodes;
    int count, cap;
    int root;
    uint64_t key, event;
    int channels;
    float *features, *policy, *value;
    int32_t *leaves, *trans;
};

static int new_node(orc_mcts *m, const orc_pos *pos, int parent) {
    if (m->count == m->cap) {
        m->cap = m->cap ? m->cap * 2 : 1024;
        m->nodes = (onode *)realloc(m->nodes, (size_t)m->cap * sizeof(onode));
    }
    onode *n = &m->nodes[m->count];
    n->pos = *pos;
    n->parent = parent;
    n->first_child = -1;
    n->n_children = 0;
    n->n = 0;
    n->w = 0.0f;
    n->q = 0.0f;
    n->p = 1.0f;
    return m->count++;
}

static void alloc_buffers(orc_mcts *m) {
    int rows = m->num_threads * m->batch_size;
    m->channels = 1 + 2 * m->history_size;
    free(m->features);
    free(m->policy);
    free(m->value);
    free(m->leaves);
    free(m->trans);
    m->features = (float *)calloc((size_t)rows * m->channels * 64, sizeof(float));
    m->policy = (float *)calloc((size_t)rows * 65, sizeof(float));
    m->value = (float *)calloc((size_t)rows, sizeof(float));
    m->leaves = (int32_t *)calloc((size_t)rows, sizeof(int32_t));
    m->trans = (int32_t *)calloc((size_t)rows, sizeof(int32_t));
}

orc_mcts *orc_mcts_create(int history_size, int num_simulations, int num_threads,
                          int batch_size, float c_puct_base, float c_puct_init,
                          float dirichlet_epsilon, float dirichlet_alpha, uint64_t game_key) {
    orc_mcts *m = (orc_mcts *)calloc(1, sizeof(orc_mcts));
    m->history_size = history_size;
    m->num_simulations = num_simulations;
    m->num_threads = num_threads;
    m->batch_size = batch_size;
    m->c_puct_base = c_puct_base;
    m->c_puct_init = c_puct_init;
    m->eps = dirichlet_epsilon;
    m->alpha = dirichlet_alpha;
    m->key = game_key;
    alloc_buffers(m);
    orc_mcts_reset_position(m);
    return m;
}

void orc_mcts_destroy(orc_mcts *m) {
    if (!m) return;
    free(m->nodes);
    free(m->features);
    free(m->policy);
    free(m->value);
    free(m->leaves);
    free(m->trans);
    free(m);
}

/* mcts.cpp:40-43 */
void orc_mcts_reset_position(orc_mcts *m) {
    orc_pos p;
    orc_initial_position(&p);
    m->count = 0;
    m->root = new_node(m, &p, -1);
    m->event = 0;
}

void orc_mcts_reset_chain(orc_mcts *m, const orc_pos *chain, int n_chain) {
    m->count = 0;
    int parent = -1;
    for (int i = n_chain - 1; i >= 0; --i) parent = new_node(m, &chain[i], parent);
    m->root = parent;
    m->event = 0;
}

void orc_mcts_position(const orc_mcts *m, orc_pos *out) { *out = m->nodes[m->root].pos; }

/* search_thread.cpp:192-260 */
static int choose_best_child(orc_mcts *m, int node) {
    onode *nd = &m->nodes[node];
    int nc = nd->n_children, fc = nd->first_child;
    if (nc == 1) return fc;
    float exploration_rate =
        logf(((float)(1 + nd->n) + m->c_puct_base) / m->c_puct_base) + m->c_puct_init;
    int total = 0;
    for (int i = 0; i < nc; ++i) total += m->nodes[fc + i].n;
    float ucb_multiplier = exploration_rate * sqrtf((float)total);

    if (!(node == m->root && m->eps > 0.0f)) {
        int best = 0;
        float best_ucb = 0.0f;
        for (int i = 0; i < nc; ++i) {
            onode *c = &m->nodes[fc + i];
            float ucb = c->q + ucb_multiplier * c->p / (1.0f + (float)c->n);
            if (i == 0 || ucb > best_ucb) {
                best = i;
                best_ucb = ucb;
            }
        }
        return fc + best;
    }
    /* Dirichlet noise re-sampled on every root selection (search_thread.cpp:230-249) */
    uint64_t ev = m->event++;
    float noise[64];
    float noise_sum = 0.0f;
    for (int i = 0; i < nc; ++i) {
        noise[i] = orc_gamma(orc_stream_key(m->key, ev, (uint32_t)i), m->alpha);
        noise_sum += noise[i];
    }
    if (noise_sum == 0.0f) noise_sum = 1.0f;
    float pm = 1.0f - m->eps;
    float nm = m->eps / noise_sum;
    int best = 0;
    float best_ucb = 0.0f;
    for (int i = 0; i < nc; ++i) {
        onode *c = &m->nodes[fc + i];
        float prob = c->p * pm + noise[i] * nm;
        float ucb = c->q + ucb_multiplier * prob / (1.0f + (float)c->n);
        if (i == 0 || ucb > best_ucb) {
            best = i;
            best_ucb = ucb;
        }
    }
    return fc + best;
}

static void leaf_features(orc_mcts *m, int leaf, int t, float *out) {
    orc_pos chain[64];
    int n = 0;
    for (int x = leaf; x >= 0 && n < m->history_size; x = m->nodes[x].parent)
        chain[n++] = m->nodes[x].pos;
    orc_features(chain, n, m->history_size, t, out);
}

/* search_thread.cpp:130-190 */
static void expand_and_backward(orc_mcts *m, int leaf, int t, const float *policy,
                                const float *value) {
    onode *lf = &m->nodes[leaf];
    if (lf->pos.player != 0 && lf->n_children == 0) {
        int32_t acts[65];
        orc_pos parent_pos = lf->pos;
        int na = orc_legal_actions(&parent_pos, acts);
        int first = m->count;
        for (int i = 0; i < na; ++i) {
            orc_pos c;
            orc_apply_action(&parent_pos, acts[i], &c);
            int id = new_node(m, &c, leaf);
            m->nodes[id].p = policy[orc_transform_action(acts[i], t)];
        }
        lf = &m->nodes[leaf];
        lf->first_child = first;
        lf->n_children = na;
    }
    float v;
    if (lf->pos.player != 0) {
        v = -value[0];
    } else {
        const onode *par = &m->nodes[lf->parent];
        uint64_t mine = par->pos.player == 1 ? lf->pos.p1 : lf->pos.p2;
        uint64_t theirs = par->pos.player == 1 ? lf->pos.p2 : lf->pos.p1;
        int a = __builtin_popcountll(mine), b = __builtin_popcountll(theirs);
        v = a > b ? 1.0f : (a < b ? -1.0f : 0.0f);
    }
    for (int x = leaf; x != m->root; x = m->nodes[x].parent) {
        onode *c = &m->nodes[x];
        c->w += 1.0f + v;
        c->q = c->w / (float)c->n;
        v = -v;
    }
}

/* One descent of a virtual thread's leaf i (search_thread.cpp:62-79):
 * PUCT walk to a terminal or unexpanded node, virtual loss on the path below
 * the root, root N+1, and the leaf's symmetry draw (:92). */
static void select_leaf(orc_mcts *m, int i) {
    int node = m->root;
    while (!(m->nodes[node].pos.player == 0 || m->nodes[node].n_children == 0))
        node = choose_best_child(m, node);
    m->leaves[i] = node;
    for (int x = node; x != m->root; x = m->nodes[x].parent) {
        onode *c = &m->nodes[x];
        c->n += 1;
        c->w -= 1.0f;
        c->q = c->w / (float)c->n;
    }
    m->nodes[m->root].n += 1;
    if (m->nodes[node].pos.player != 0) {
        uint64_t ev = m->event++;
        m->trans[i] = (int32_t)(orc_mix64(orc_stream_key(m->key, ev, 0)) >> 61);
    } else {
        m->trans[i] = 0;
    }
}

/* Features of thread th's batch and its NN call (search_thread.cpp:84-110;
 * skipped when every leaf of the batch is terminal, :102). */
static void evaluate_thread(orc_mcts *m, int th, orc_nn_fn nn, void *user) {
    int B = m->batch_size, C = m->channels;
    int any = 0;
    for (int j = 0; j < B; ++j) {
        int i = th * B + j;
        float *f = m->features + (size_t)i * C * 64;
        if (m->nodes[m->leaves[i]].pos.player == 0) {
            memset(f, 0, (size_t)C * 64 * sizeof(float));
            continue;
        }
        any = 1;
        leaf_features(m, m->leaves[i], m->trans[i], f);
    }
    if (any)
        nn(user, m->features + (size_t)th * B * C * 64, B, C, m->policy + (size_t)th * B * 65,
           m->value + (size_t)th * B);
}

static int batch_any_live(const orc_mcts *m, int th) {
    for (int j = 0; j < m->batch_size; ++j)
        if (m->nodes[m->leaves[th * m->batch_size + j]].pos.player != 0) return 1;
    return 0;
}

static void backup_thread(orc_mcts *m, int th) {
    for (int j = 0; j < m->batch_size; ++j) {
        int i = th * m->batch_size + j;
        expand_and_backward(m, m->leaves[i], m->trans[i], m->policy + (size_t)i * 65, m->value + i);
    }
}

/* Thread th selects its next batches (search_thread.cpp:60-81) until one has
 * a non-terminal leaf, which then waits for the NN; a batch whose leaves are
 * all terminal needs no NN round trip (:102) and is backed up at once
 * (:116-127) before the thread selects again. At most `steps` batches per
 * thread and search (:47-57). */
static void select_thread(orc_mcts *m, int th, int steps, int *sel, int *pend) {
    while (sel[th] < steps) {
        for (int j = 0; j < m->batch_size; ++j) select_leaf(m, th * m->batch_size + j);
        ++sel[th];
        if (batch_any_live(m, th)) {
            pend[th] = 1;
            return;
        }
        backup_thread(m, th);
    }
}

/* Schedule of the reference's T threads x B leaves (search_thread.cpp:47-128,
 * mcts.h:220-256). Each thread runs ceil(S / (T*B)) batches of
 * lock{select B} -> NN round trip -> lock{expand + backup B}; the calling
 * thread serves NN requests in FIFO order. The interleaving the reference
 * produces in practice (measured over repeated runs of the compiled
 * reference, DESIGN.md "Search semantics") is the pipelined round-robin
 *
 *     S_0(1) S_1(1) .. S_{T-1}(1)  then, for k = 1..n, for t = 0..T-1:
 *     B_t(k) S_t(k+1)
 *
 * (S = select a batch, B = back it up): a thread whose NN result arrives
 * backs up and immediately selects its next batch while the NN serves the
 * next thread; a thread whose selected batch is all terminal skips the NN and
 * backs up and selects again right away (select_thread), so near the end of a
 * game threads run ahead of each other. With T = 1 this is exactly the
 * reference's sequential loop. */
int orc_mcts_search(orc_mcts *m, orc_nn_fn nn, void *user) {
    int T = m->num_threads, B = m->batch_size, L = T * B;
    int steps = (m->num_simulations + L - 1) / L;
    int sel[1024], pend[1024];
    for (int t = 0; t < T; ++t) sel[t] = pend[t] = 0;
    for (int t = 0; t < T; ++t) select_thread(m, t, steps, sel, pend);
    for (;;) {
        int any = 0;
        for (int t = 0; t < T; ++t)
            if (pend[t]) {
                any = 1;
                evaluate_thread(m, t, nn, user);
            }
        if (!any) break;
        for (int t = 0; t < T; ++t)
            if (pend[t]) {
                backup_thread(m, t);
                pend[t] = 0;
                select_thread(m, t, steps, sel, pend);
            }
    }
    return steps * L;
}

int orc_mcts_num_children(const orc_mcts *m) { return m->nodes[m->root].n_children; }

/* mcts.cpp:45-52 */
void orc_mcts_visit_counts(const orc_mcts *m, int32_t *out) {
    const onode *r = &m->nodes[m->root];
    for (int i = 0; i < r->n_children; ++i) out[i] = m->nodes[r->first_child + i].n;
}

/* mcts.cpp:54-61 */
void orc_mcts_mean_action_values(const orc_mcts *m, float *out) {
    const onode *r = &m->nodes[m->root];
    for (int i = 0; i < r->n_children; ++i) out[i] = m->nodes[r->first_child + i].q;
}

int32_t orc_mcts_root_visit_count(const orc_mcts *m) { return m->nodes[m->root].n; }

/* mcts.cpp:63-112 */
int orc_mcts_self_play_data(const orc_mcts *m, float *features, float *policy) {
    const onode *r = &m->nodes[m->root];
    if (r->pos.player == 0) return 1;
    if (r->n_children == 0) return 2;
    int32_t acts[65];
    int na = orc_legal_actions(&r->pos, acts);
    int sum = 0;
    for (int i = 0; i < r->n_children; ++i) sum += m->nodes[r->first_child + i].n;
    if (sum == 0) sum = 1;
    int C = m->channels;
    for (int t = 0; t < 8; ++t) {
        leaf_features((orc_mcts *)m, m->root, t, features + (size_t)t * C * 64);
        float *pol = policy + t * 65;
        for (int a = 0; a < 65; ++a) pol[a] = 0.0f;
        for (int i = 0; i < na; ++i)
            pol[orc_transform_action(acts[i], t)] =
                (float)m->nodes[r->first_child + i].n / (float)sum;
    }
    return 0;
}

/* mcts.cpp:114-165 */
int orc_mcts_apply_action(orc_mcts *m, int action) {
    onode *r = &m->nodes[m->root];
    if (!(0 <= action && action < 65)) return -1;
    if (action == 64) {
        if (r->pos.player == 0) return -3;
        if (r->pos.legal != 0) return -4;
    } else if (((1ULL << (63 - action)) & r->pos.legal) == 0) {
        return -2;
    }
    if (r->n_children == 0) {
        orc_pos c;
        orc_apply_action(&r->pos, action, &c);
        m->root = new_node(m, &c, m->root);
        return 0;
    }
    int idx = 0;
    if (action != 0 && r->n_children > 1)
        idx = __builtin_popcountll(r->pos.legal & (~0ULL << (64 - action)));
    m->root = r->first_child + idx;
    return 0;
}

int orc_mcts_node_count(const orc_mcts *m) { return m->count; }
uint64_t orc_mcts_events(const orc_mcts *m) { return m->event; }

/* The self-play move choice of train.py:421-430 as the on-device driver
 * (tree.hip k_selfplay_move) draws it from one event of the game's stream:
 * for ply < temperature_moves sample a child with p ~ N^(1/temperature) by a
 * sequential float cdf (numpy.random.choice's rule); afterwards argmax of N
 * with a uniform random tie-break; an unexpanded root picks a legal action
 * uniformly. Returns the action (not applied). */
int orc_mcts_selfplay_action(orc_mcts *m, int ply, int temperature_moves, float temperature) {
    const onode *r = &m->nodes[m->root];
    if (r->pos.player == 0) return -1;
    int32_t acts[65];
    orc_pos rp = r->pos;
    int na = orc_legal_actions(&rp, acts);
    int nc = r->n_children;
    uint64_t ev = m->event++;
    float u = orc_uniform(orc_stream_key(m->key, ev, 0), 0);
    int j = 0;
    if (nc == 0) {
        j = (int)(u * (float)na);
        if (j >= na) j = na - 1;
    } else if (ply < temperature_moves) {
        float cdf[64], sum = 0.0f;
        for (int k = 0; k < nc; ++k) {
            sum += powf((float)m->nodes[r->first_child + k].n, 1.0f / temperature);
            cdf[k] = sum;
        }
        if (sum > 0.0f) {
            float target = u * sum;
            j = nc - 1;
            for (int k = 0; k < nc; ++k)
                if (cdf[k] > target) {
                    j = k;
                    break;
                }
        } else {
            j = (int)(u * (float)nc);
            if (j >= nc) j = nc - 1;
        }
    } else {
        int mx = 0, nt = 0;
        for (int k = 0; k < nc; ++k)
            if (m->nodes[r->first_child + k].n > mx) mx = m->nodes[r->first_child + k].n;
        for (int k = 0; k < nc; ++k) nt += m->nodes[r->first_child + k].n == mx;
        int pick = (int)(u * (float)nt);
        if (pick >= nt) pick = nt - 1;
        for (int k = 0; k < nc; ++k)
            if (m->nodes[r->first_child + k].n == mx && pick-- == 0) {
                j = k;
                break;
            }
    }
    return acts[j];
}
