// Launchers shared between the kernel translation units and the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/othello_mcts_amd.h"
#include "bitboard.h"
#include "engine.h"

namespace oamd {

struct SelfplayParams {
    int32_t temperature_moves;
    float temperature;
    int32_t opening_moves;
    int32_t emit_targets;
};

// tree.hip
// One search round for games [g0, g0 + ng) (ng < 0: to the end): for each
// virtual thread t in [t0, t1) (t1 < 0: T), back up its previous batch
// (do_backup), then select its next B leaves (do_select). T * B must equal
// E.L. cnt_add: append the selected non-terminal rows to the evaluation list
// E.rowlist[g0 * L ..] behind this counter; cnt_reset: the counter to zero
// (the next round's). fresh: the search's first round (every virtual thread
// starts with no batch selected). See tree.hip k_tree.
void launch_tree(const EngineView& E, hipStream_t s, bool do_backup, bool do_select, int T, int B,
                 int g0 = 0, int ng = -1, int t0 = 0, int t1 = -1, int* cnt_add = nullptr,
                 int* cnt_reset = nullptr, bool fresh = false, int budget = 0, int max_cuts = 0,
                 bool timed = false, int* cuts_out = nullptr);
void launch_features_f32(const EngineView& E, float* out, int row_begin, int rows, hipStream_t s);
void launch_set_evaluation(const EngineView& E, const float* pol, const float* val, int row_begin,
                           int rows, hipStream_t s);
void launch_leaf_flags(const EngineView& E, uint8_t* flags, hipStream_t s);
void launch_reset(const EngineView& E, int game, uint64_t seed, hipStream_t s);
void launch_apply_actions(const EngineView& E, const int32_t* actions, hipStream_t s);
void launch_apply_one(const EngineView& E, int g, int action, hipStream_t s);
void launch_root_stats(const EngineView& E, int game_begin, int n_games, oamd_root_info* info,
                       int32_t* visits, float* q, int by_action, hipStream_t s);
void launch_self_play_data(const EngineView& E, int g, float* feat, float* pol, hipStream_t s);
void launch_selfplay_move(const EngineView& E, const SelfplayParams& sp, int g0, int ng, int32_t* actions,
                          int32_t* finished, float* feat, float* pol, hipStream_t s);
void launch_random_openings(const EngineView& E, int max_moves, uint64_t seed, hipStream_t s);
// Free-running self-play (tree.hip k_tree_free): begin sets every game of the
// group to play n_moves moves starting with a fresh search and counts them in
// *remaining; each round runs one search round per game, a game's move in the
// round its search completes, and its next search's first round after it.
// *remaining must be zeroed before begin (stream order).
void launch_free_begin(const EngineView& E, int g0, int ng, int n_moves, int32_t* remaining, int32_t* actions,
                       int32_t* finished, int per_move, hipStream_t s);
void launch_tree_free(const EngineView& E, hipStream_t s, int g0, int ng, int B, int* cnt_add, int* cnt_reset,
                      int budget, bool timed, const SelfplayParams& sp, int n_moves, int per_move, int32_t* actions,
                      int32_t* finished, float* feat, float* pol, int32_t* remaining);
void launch_status(const EngineView& E, int32_t* out, hipStream_t s);
void launch_legal_moves(const uint64_t* me, const uint64_t* opp, uint64_t* out, int64_t n,
                        hipStream_t s);
void launch_flips(const uint64_t* mv, const uint64_t* me, const uint64_t* opp, uint64_t* out,
                  int64_t n, hipStream_t s);
void launch_apply_positions(const Pos* in, const int32_t* actions, Pos* out, int64_t n,
                            hipStream_t s);

// resnet.hip
struct NetView {
    int32_t cin;     // real input channels (1 + 2H)
    int32_t C;       // conv channels
    int32_t R;       // residual blocks
    int32_t hidden;  // value head hidden units
    int32_t dtype;   // oamd_dtype
    const uint16_t* w;   // packed conv weights, all layers, fragment order
    const float* bias;   // folded conv bias, (1 + 2R) * C
    const float* head;   // head parameters, see resnet.hip
    const uint16_t* hconv;  // 1x1 head convs (BN folded), MFMA A fragments: [C/32][lane][8]
};

// features: packed engine rows (fw words per row, history H) or fp32 planes.
// Packed rows with an evaluation list (rowlist != nullptr): the launch
// evaluates rows rowlist[0 .. min(rows, *rowcount - list_off)) (absolute row
// indices into feat / policy / value); without one, rows 0 .. rows-1.
// max_wgs > 0: at most that many workgroups, looping over the board groups
// (the chain-splitting extra rounds' nearly empty launches).
// span != nullptr (timed searches): the launch records its execution interval
// in span[0] = ~(earliest workgroup start), span[1] = latest workgroup end
// (s_memrealtime, 100 MHz ticks; zero-initialised by the caller)
void launch_resnet_packed(const NetView& N, const uint64_t* feat, int fw, int H, int rows,
                          float* policy, float* value, hipStream_t s, const int32_t* rowlist = nullptr,
                          const int32_t* rowcount = nullptr, int list_off = 0,
                          unsigned long long* span = nullptr, int max_wgs = 0);
void launch_resnet_f32(const NetView& N, const float* feat, int rows, float* policy, float* value,
                       hipStream_t s);
size_t resnet_packed_weight_elems(int C, int R);
size_t resnet_packed_weight_alloc_elems(int C, int R);  // + the zero pad the stream may run into
size_t resnet_head_floats(int C, int hidden);
// elements of the packed 1x1 head-conv fragments (NetView::hconv)
inline size_t resnet_hconv_elems(int C) { return (size_t)(C / 32) * 64 * 8; }
// diagnostic stamp buffer (OAMD_STAMPS builds; -2 otherwise), see resnet.hip
int resnet_read_stamps(unsigned long long* out, long long n);
int tree_read_stamps(unsigned long long* out, long long n, int reset);
// Weight K-step schedule shared by the kernel and the host packer: a K-step is
// one 3x3 tap x 32 input channels. K-steps per conv (first conv: input zero-
// padded to 32 channels, 9 K-steps rounded up to whole weight stages with
// zero-weight K-steps); tap and 32-channel block of K-step i (pad = all-zero).
int resnet_ksteps(int C, bool first);
void resnet_kstep(int C, bool first, int i, int* tap, int* cb, bool* pad);
// 8-channel chunk (0..3 within a K-step) that MFMA k-group kg (= lane >> 4) reads
int resnet_kgroup_chunk(int kg);
// output channel of row `row` (0..15) of MFMA output-channel tile `tile` (weights packing)
int resnet_out_channel(int tile, int row);

}  // namespace oamd
