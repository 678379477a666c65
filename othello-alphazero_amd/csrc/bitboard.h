// 64-bit Othello bitboards for CDNA4 waves and for the host API.
//
// Semantics follow the reference game core (cpp/src/include/position.h):
//   square i = row*8 + col, bit (63 - i); a1 = square 0 = bit 63   (position.h:275)
//   direction strides {-9,-8,-7,-1,1,7,8,9}: positive -> >>, negative -> <<  (:153,174-184)
//   per-direction edge masks drop wrap-around files/ranks                  (:155-172)
//   opponent runs: seed step + 5 propagation steps                        (:186-196)
//   legal moves  (:202-229), flips (:231-262), apply move/pass (:328-386)
// The code is written once and compiled for both the host (Position API of
// the Python surface) and gfx950 (batched kernels, tree expansion), so the
// two can never drift apart.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define OAMD_HD __host__ __device__ __forceinline__

namespace oamd {

constexpr uint64_t kNoLR = 0x7E7E7E7E7E7E7E7EULL;
constexpr uint64_t kNoTB = 0x00FFFFFFFFFFFF00ULL;
constexpr uint64_t kNoEdge = kNoLR & kNoTB;

// Position value type: player 1 = black to move, 2 = white, 0 = terminal.
struct Pos {
    int32_t player;
    int32_t pad_;
    uint64_t p1, p2;
    uint64_t legal;       // moves of the side to move
    uint64_t next_legal;  // opponent's moves, only set when the side to move must pass
};

template <int S>
OAMD_HD uint64_t shift_by(uint64_t m) {
    if constexpr (S > 0) return m >> S;
    else return m << (-S);
}

// Dumb7fill-style run in one direction; 6 steps cover runs of up to 6 discs.
template <int S>
OAMD_HD uint64_t run_dir(uint64_t seed, uint64_t opp_masked) {
    uint64_t f = opp_masked & shift_by<S>(seed);
    f |= opp_masked & shift_by<S>(f);
    f |= opp_masked & shift_by<S>(f);
    f |= opp_masked & shift_by<S>(f);
    f |= opp_masked & shift_by<S>(f);
    f |= opp_masked & shift_by<S>(f);
    return f;
}

OAMD_HD uint64_t legal_moves(uint64_t me, uint64_t opp) {
    const uint64_t oe = opp & kNoEdge, otb = opp & kNoTB, olr = opp & kNoLR;
    uint64_t m = 0;
    m |= shift_by<-9>(run_dir<-9>(me, oe));
    m |= shift_by<-8>(run_dir<-8>(me, otb));
    m |= shift_by<-7>(run_dir<-7>(me, oe));
    m |= shift_by<-1>(run_dir<-1>(me, olr));
    m |= shift_by<1>(run_dir<1>(me, olr));
    m |= shift_by<7>(run_dir<7>(me, oe));
    m |= shift_by<8>(run_dir<8>(me, otb));
    m |= shift_by<9>(run_dir<9>(me, oe));
    return m & ~(me | opp);
}

template <int S>
OAMD_HD uint64_t capped(uint64_t move, uint64_t me, uint64_t opp_masked) {
    uint64_t f = run_dir<S>(move, opp_masked);
    return (shift_by<S>(f) & me) ? f : 0ULL;
}

OAMD_HD uint64_t flips(uint64_t move, uint64_t me, uint64_t opp) {
    const uint64_t oe = opp & kNoEdge, otb = opp & kNoTB, olr = opp & kNoLR;
    return capped<-9>(move, me, oe) | capped<-8>(move, me, otb) | capped<-7>(move, me, oe) |
           capped<-1>(move, me, olr) | capped<1>(move, me, olr) | capped<7>(move, me, oe) |
           capped<8>(move, me, otb) | capped<9>(move, me, oe);
}

OAMD_HD Pos initial_position() {
    Pos p;
    p.player = 1;
    p.pad_ = 0;
    p.p1 = 0x0000000810000000ULL;
    p.p2 = 0x0000001008000000ULL;
    p.legal = legal_moves(p.p1, p.p2);
    p.next_legal = 0;
    return p;
}

// Unchecked, like Position::apply_action (position.h:402-408).
OAMD_HD Pos apply_action(const Pos& p, int action) {
    Pos c;
    c.pad_ = 0;
    if (action == 64) {
        c.player = 3 - p.player;
        c.p1 = p.p1;
        c.p2 = p.p2;
        c.legal = p.next_legal;
        c.next_legal = 0;
        return c;
    }
    const uint64_t move = 1ULL << (63 - action);
    const bool black = p.player == 1;
    uint64_t me = black ? p.p1 : p.p2;
    uint64_t opp = black ? p.p2 : p.p1;
    const uint64_t f = flips(move, me, opp);
    me |= move | f;
    opp &= ~f;
    c.p1 = black ? me : opp;
    c.p2 = black ? opp : me;
    c.player = 3 - p.player;
    c.legal = legal_moves(opp, me);
    c.next_legal = 0;
    if (c.legal == 0) {
        c.next_legal = legal_moves(me, opp);
        if (c.next_legal == 0) c.player = 0;
    }
    return c;
}

OAMD_HD int popcount64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __popcll(x);
#else
    return __builtin_popcountll(x);
#endif
}

// Number of legal actions (children of an expanded node): {} terminal, {64} pass.
OAMD_HD int num_actions(const Pos& p) {
    if (p.player == 0) return 0;
    return p.legal ? popcount64(p.legal) : 1;
}

// D4 transform of an action (transformation.h:40-57): optional horizontal
// flip (t odd), then t/2 clockwise rotations (row,col) -> (col, 7-row).
OAMD_HD int transform_action(int action, int t) {
    if (action == 64) return 64;
    int row = action >> 3, col = action & 7;
    if (t & 1) col = 7 - col;
    for (int i = 0; i < (t >> 1); ++i) {
        const int r = row;
        row = col;
        col = 7 - r;
    }
    return row * 8 + col;
}

// Inverse map: square s' of the transformed board shows original square
// inverse_transform(s', t), i.e. transform_action(inverse_transform(s', t), t) == s'.
OAMD_HD int inverse_transform(int sq, int t) {
    int row = sq >> 3, col = sq & 7;
    for (int i = 0; i < (t >> 1); ++i) {  // undo clockwise rotations
        const int c = col;
        col = row;
        row = 7 - c;
    }
    if (t & 1) col = 7 - col;
    return row * 8 + col;
}

}  // namespace oamd
