// Fused AlphaZeroNet forward (python/othello_alphazero/neural_net.py:138-172,
// eval mode) for gfx950: one launch evaluates a batch of boards end to end.
//
// Work decomposition (DESIGN.md "ResNet kernel"):
//   * a 512-thread workgroup (8 waves, 2 per SIMD) owns BOARDS = 512/C boards
//     (4 boards at C=128, 2 boards at C=256) and runs the whole tower + both
//     heads on them; activations never leave LDS;
//   * each 3x3 conv is an implicit GEMM  out[ch][pos] = W[ch][K] x X[K][pos],
//     K = 9 taps x C_in, on v_mfma_f32_16x16x32_{bf16,f16} with the WEIGHTS as
//     the A operand: an accumulator lane then holds 4 consecutive output
//     channels of one position, so the epilogue writes 8 contiguous bytes;
//     throughput geometries: wave (wm, wn) owns 32 channels (wn) x rows 0-7
//     of board pair wm (edge-row tiles, see wide_cb / edge_tile_row);
//     small-batch geometry: C/8 channels x the 64 positions of the board;
//   * K is walked in K-steps of one tap x 32 input channels. Weights (BatchNorm
//     folded, packed on the host in fragment order) stream once per workgroup
//     through a 3-slot LDS ring by LDS-DMA (global_load_lds_dwordx4); a 16 KiB
//     slot holds one stage = 256/C K-steps. Stage s+2 is issued at the barrier
//     that opens stage s+1, so fragment reads always overlap MFMAs;
//   * ONE activation buffer per workgroup, updated in place: each board is a
//     zero-bordered 10x10 grid of rows of 2C+16 bytes ([position][channel]).
//     The border makes every 3x3 tap read `lane base + uniform offset` (no
//     per-read address arithmetic, no masking), and with the 16-byte row pad,
//     the position->lane map kTilePos and the k-group->chunk map kgroup_chunk
//     the 16 lanes of every ds_read_b128 lane group hit 16 distinct LDS slots
//     for every tap (verified exhaustively in tests/test_cpu_host.py);
//   * accumulators start from the folded bias (+ the residual skip for the
//     second conv of a block, carried in registers from the first conv's
//     epilogue), so the epilogue is cvt_pk + packed-i16 ReLU + one ds_write_b64;
//   * heads: both 1x1 convs of a board as one small MFMA GEMM, the Linear
//     layers k-split in fp32 over every board of the workgroup, softmax(65),
//     tanh (heads()).

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "bitboard.h"
#include "kernels.h"

namespace oamd {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) short i16x2_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int kLdsBytes = 160 * 1024;
#ifdef OAMD_STAMPS
constexpr int kMaxStampWgs = 1 << 16;
// u64 per workgroup: 0-15 wave 0's stamps (tools/nn_stamps.py), 16-22 cycle
// sums over all 8 waves: step-start lgkmcnt waits, stage-open vmcnt waits,
// stage barriers, epilogue first barrier / stores / second barrier + reads,
// tower cycles
constexpr int kStampStride = 24;
#endif
// Weight stream: 16 KiB stages (2 K-steps at C=128, 1 at C=256) in a 3-slot
// LDS ring (the small-batch geometry: 4 slots), refilled by LDS-DMA. 8 KiB
// stages in a 6-slot ring measured 3 % slower (DESIGN.md §6 lists every
// measured alternative: register staging, early stage opening, staggered or
// prioritised waves, other DMA placements, 128-channel tiles, ...).
constexpr int kStageBytes = 16384;
// throughput geometries: stage bytes and ring slots per channel count.
// Edge-row boards without their never-read top / bottom border rows leave
// room for a fourth 16 KiB slot or for 32 KiB stages. Same box, 4096 rows
// (profiles/r03/ab): C=256 with 4 slots (3 stages in flight) 6.60 ms vs 6.75
// with 3; 32 KiB stages in 2 slots (one barrier per 2 K-steps) 7.13-7.22 vs
// 6.69. C=128: 4 slots 0.81-0.83 vs 0.78, 32 KiB stages 0.83-0.84 vs 0.78.
#ifndef OAMD_C128_STAGE
#define OAMD_C128_STAGE 16384
#endif
#ifndef OAMD_C128_RING
#define OAMD_C128_RING 3
#endif
#ifndef OAMD_C256_STAGE
#define OAMD_C256_STAGE 16384
#endif
#ifndef OAMD_C256_RING
#define OAMD_C256_RING 4
#endif
// C=256 throughput geometry: weight fragments go from global memory (L2)
// straight into a per-wave register queue 3 K-steps ahead of their MFMAs
// instead of through the LDS ring (GeoT::DIRECT): no stage barriers (the ring
// needs one per K-step at C=256). Same box, 4096 rows (profiles/r03/ab):
// 6.385 ms vs 6.725 with the ring; a 2-deep queue 6.51; 6- and 8-deep queues
// spill. At C=128 (one barrier per 2 K-steps, and the two board pairs' waves
// of a channel block fetch the same fragments) the queue measured 1.3 %
// slower than the ring: 0.807-0.809 vs 0.794-0.798 ms.
constexpr int kWeightQueue = 4;
constexpr int kStageBytesMax = 32768;
__host__ __device__ constexpr int stage_bytes(int C) { return C == 256 ? OAMD_C256_STAGE : OAMD_C128_STAGE; }
// k_resnet_w8 register cap: gfx950 counts the unified VGPR+AGPR file, the
// backend doubles this value: 2 x 104 = 208 VGPRs, so one 96-VGPR k_tree wave
// fits beside the two ResNet waves of a SIMD
#ifndef OAMD_VGPR_CAP
#define OAMD_VGPR_CAP 104
#endif
// Tower K order and tiling (throughput geometries; DESIGN.md §6 "wide wave
// tiles"): a wave owns 32 output channels x 128 positions, i.e. rows 0-7 of a
// pair of boards (C=128) or of both boards (C=256), as 8 MFMA tiles of one
// board row each (edge_tile_row). Per dx and 32-channel block the K-steps run
// (cb, dy) = (c,-1) (c,0) (c,+1): tile m at dy reads board row m + dy, so the
// three dy taps of one (dx, block) read the 8 board rows once into a register
// window, and tile 0 at dy = -1 and tile 7 at dy = +1 read only the zero
// border: those MFMAs are left out at compile time (8.3 % of the tower's).
// The order is one function shared by the host weight packer and every
// geometry (the small-batch one reads every fragment), so all geometries are
// bit-identical.
__host__ __device__ constexpr int wide_cb(int J) { return J / 3; }
__host__ __device__ constexpr int wide_dy(int J) { return J % 3 - 1; }
// window rows (bit i = board row i - 1) K-step J needs first: rows 0-6 at
// dy = -1, row 7 at dy = 0
__host__ __device__ constexpr int wide_new(int J) { return J % 3 == 0 ? 0xFE : (J % 3 == 1 ? 0x100 : 0); }
// Epilogue without its first barrier (OAMD_EPI_NOBAR, round 6; tower layers
// of the C=128 edge-row geometry, which has a weight ring): the layer's last
// (dx, block) reads its whole window, rows 0-7, at its first K-step, so every
// activation read of the layer is issued before the barrier that opens the
// layer's last stage; after it no wave reads the layer's input, and a wave
// overwrites its outputs in place as soon as its own MFMAs are done (the
// wait at the first barrier was 1.5 % of the tower's cycles).
// The last stage's weight slot is refilled after the second (post-store)
// barrier instead. Same box, 4096 rows, interleaved, bit-identical:
// 0.787-0.796 vs 0.796-0.808 ms. Not for the register-queue geometry
// (C=256, DIRECT): it has no stage barriers, so nothing orders the other
// waves' last reads before a store (its outputs differed when tried).
#ifndef OAMD_EPI_NOBAR
#define OAMD_EPI_NOBAR 1
#endif
template <bool ENABLE>
__host__ __device__ constexpr int wide_new_last(int J, int NJ) {
    return !ENABLE || J < NJ - 3 ? wide_new(J) : (J % 3 == 0 ? 0x1FE : 0);
}

// Head parameter buffer layout (fp32), filled by oamd_net_load_state (capi.hip).
struct HeadLayout {
    int pcw, pcb, vcw, vcb, plw, plb, v1w, v1b, v2w, v2b, total;
    __host__ __device__ HeadLayout(int C, int hidden) {
        pcw = 0;                 // [2][C]
        pcb = pcw + 2 * C;       // [2]
        vcw = pcb + 2;           // [C]
        vcb = vcw + C;           // [1]
        plw = vcb + 1;           // [128][65]  (transposed linear weight)
        plb = plw + 128 * 65;    // [65]
        v1w = plb + 65;          // [64][hidden] (transposed)
        v1b = v1w + 64 * hidden; // [hidden]
        v2w = v1b + hidden;      // [hidden]
        v2b = v2w + hidden;      // [1]
        total = v2b + 1;
    }
};

size_t resnet_head_floats(int C, int hidden) { return (size_t)HeadLayout(C, hidden).total; }

// ---- K-step schedule (shared with the host packer) --------------------------
__host__ __device__ constexpr int ksteps_per_stage(int C) {
    return stage_bytes(C) / (32 * C * 2);
}
__host__ __device__ constexpr int ksteps_first(int C) {
    return (9 + ksteps_per_stage(C) - 1) / ksteps_per_stage(C) * ksteps_per_stage(C);
}
__host__ __device__ constexpr int ksteps_tower(int C) { return 9 * (C / 32); }
__host__ __device__ constexpr int kgroup_chunk(int kg) { return ((kg & 1) << 1) | (kg >> 1); }
// Output channel computed by row 4 * kg + k of MFMA channel tile `tile` (an
// accumulator lane of k-group kg holds rows 4 kg .. 4 kg + 3): the tiles 2j and
// 2j + 1 of a 32-channel block interleave in groups of 4, so a lane's 8
// accumulator channels of the pair are contiguous (channels 32j + 8kg .. +7)
// and the epilogue stores them with one ds_write_b128. The host packs every
// conv's weights and the kernel loads every bias in this order; activations
// stay in plain channel order.
__host__ __device__ constexpr int out_chan(int tile, int kg, int k) {
    return 32 * (tile >> 1) + 8 * kg + 4 * (tile & 1) + k;
}

int resnet_ksteps(int C, bool first) { return first ? ksteps_first(C) : ksteps_tower(C); }
void resnet_kstep(int C, bool first, int i, int* tap, int* cb, bool* pad) {
    if (first) {
        *tap = i < 9 ? i : 8;
        *cb = 0;
        *pad = i >= 9;
    } else {  // the tower's wide order: per dx, (cb, dy) = (c,-1) (c,0) (c,+1)
        const int dxi = i / (3 * (C / 32)), J = i % (3 * (C / 32));
        *tap = dxi + 3 * (wide_dy(J) + 1);
        *cb = wide_cb(J);
        *pad = false;
    }
}
int resnet_kgroup_chunk(int kg) { return kgroup_chunk(kg); }
int resnet_out_channel(int tile, int row) { return out_chan(tile, row >> 2, row & 3); }
size_t resnet_packed_weight_elems(int C, int R) {
    return (size_t)(ksteps_first(C) + 2 * R * ksteps_tower(C)) * 32 * C;
}
// + a zero pad of 4 stages: the weight stream runs up to AHEAD (<= 3) stages
// past the last one (issue_stage_dma)
size_t resnet_packed_weight_alloc_elems(int C, int R) { return resnet_packed_weight_elems(C, R) + 4 * kStageBytesMax / 2; }

// ---- activation layout --------------------------------------------------------
// padded row of board position p = 8y + x inside its board's 10x10 grid
__host__ __device__ constexpr int pad_row(int p) { return ((p >> 3) + 1) * 10 + (p & 7) + 1; }

// kTilePos.p[16m + n]: board position held by B-fragment column n of position
// tile m. Tile m takes, for every residue r = pad_row mod 16 (each residue
// occurs exactly 4 times on the 8x8 board), the m-th position of that residue;
// columns n in {0-3, 12-15} carry the odd residues, n in {4-11} the even ones.
// With chunk offsets kgroup_chunk = {0,2,1,3} every ds_read_b128 lane group
// then covers the 16 slots of a 256-byte bank row exactly once.
struct TilePos {
    unsigned char p[64];
};
constexpr TilePos make_tile_pos() {
    TilePos t{};
    for (int n = 0; n < 16; ++n) {
        const int k = n < 4 ? n : (n < 12 ? n - 4 : n - 8);
        const int r = (n < 4 || n >= 12) ? 2 * k + 1 : 2 * k;
        int m = 0;
        for (int p = 0; p < 64; ++p)
            if (pad_row(p) % 16 == r) t.p[16 * (m++) + n] = (unsigned char)p;
    }
    return t;
}
__constant__ TilePos kTilePos = make_tile_pos();

// Edge-row tiling (G::EDGE): layout row of B-fragment column j of position tile
// m for position group q (wave / WN). Group q = (pair P, half h): tile m is
// board row y = 4h + m of boards P and P + NPAIR (NPAIR * BROWS = 8 mod 16 rows
// apart, so the tile's 16 squares cover every residue of the layout row mod 16
// once). Columns 0-3 / 12-15 take the odd-residue squares of board P /
// P + NPAIR, columns 4-7 / 8-11 the even ones: the kTilePos split, so the
// kgroup_chunk map keeps every ds_read_b128 lane group on 16 distinct slots
// (tests/test_cpu_host.py restates and checks it for every tap). Edge-row
// boards keep no top / bottom border rows (G::ROW0 = 0): the MFMAs of tile 0
// at dy = -1 and tile 7 at dy = +1 are left out, so rows -1 and 8 are never
// read; the left / right border columns stay (zero) in every row.
template <class G>
__host__ __device__ constexpr int edge_tile_row(int q, int m, int j) {
    constexpr int NP = G::NPAIR > 0 ? G::NPAIR : 1;
    const int P = q % NP, h = q / NP;
    const int y = 4 * h + m;
    const int r0 = (P * G::BROWS + G::ROW0 + y * 10 + 1) & 15;
    const int oddcol = (j < 4 || j >= 12) ? 1 : 0;
    const int b = j < 8 ? P : P + NP;
    const int x = 2 * (j & 3) + ((r0 & 1) ^ oddcol);
    return b * G::BROWS + G::ROW0 + y * 10 + x + 1;
}

// Workgroup geometry: C channels, BOARDS boards per workgroup, WC output
// channels per wave (NT = WC/16 MFMA tiles), at most RING_MAX weight slots of
// STAGE bytes (a whole number of K-steps; the packed weights are K-step
// granular, so any stage size reads the same buffer).
template <int C_, int BOARDS_, int WC_, int RING_MAX_, int STAGE_ = stage_bytes(C_), int PW_ = 64>
struct GeoT {
    static constexpr int C = C_;
    static constexpr int BOARDS = BOARDS_;
    static constexpr int WC = WC_;
    static constexpr int NT = WC / 16;
    static constexpr int WN = C / WC;           // waves along output channels
    static constexpr int PW = PW_;                      // positions per wave
    static constexpr int MT = PW / 16;                  // MFMA position tiles per wave
    static constexpr int WAVES = BOARDS * 64 / PW * WN;
    static constexpr int WPB = WAVES / BOARDS;          // waves per board (heads)
    static constexpr int THREADS = WAVES * 64;
    static constexpr int RP = 2 * C + 16;       // row pitch (bytes)
    // board stride in rows (10x10 padded board); with two boards per workgroup
    // 104, so the two boards of an edge tile sit 8 rows apart modulo 16
    static constexpr int NPAIR = BOARDS / 2;
    // edge-row wave tiles (32 channels x rows 0-7 of a board pair)
    static constexpr bool EDGE = BOARDS >= 2 && BOARDS % 2 == 0 && WC_ == 32 && PW_ == 128;
    // layout row of board row y, column x (x = -1, 8: the zero border) is
    // b * BROWS + ROW0 + 10 y + x + 1. Edge-row boards: 8 rows of 10 (no top /
    // bottom border), BROWS = 84 / 88 so the boards of a tile pair sit 8 rows
    // apart mod 16; other geometries: the full 10 x 10 bordered board
    static constexpr int ROW0 = EDGE ? 0 : 10;
    static constexpr int BROWS = !EDGE ? 100 : (NPAIR == 1 ? 88 : 84);
    __host__ __device__ static constexpr int prow(int p) { return ROW0 + (p >> 3) * 10 + (p & 7) + 1; }
    static constexpr int ACT_BYTES = BOARDS * BROWS * RP;
    // DIRECT: no weight ring during the tower (its LDS stays allocated as the
    // heads' scratch); WQ = K-steps of weight fragments held per wave
    static constexpr bool DIRECT = EDGE && C == 256;
    static constexpr int WQ = kWeightQueue;
    static constexpr int KSTEP_BYTES = 32 * C * 2;
    static constexpr int STAGE = STAGE_;
    static constexpr int KS = STAGE / KSTEP_BYTES;
    static constexpr int DPT = STAGE / 16 / THREADS;         // DMAs per thread per stage
    static constexpr int RING_FIT = (kLdsBytes - ACT_BYTES) / STAGE;
    static constexpr int RING = RING_FIT < RING_MAX_ ? RING_FIT : RING_MAX_;  // weight ring slots
    static constexpr int LDS = ACT_BYTES + RING * STAGE;
    // The barrier that opens stage s issues stage s + AHEAD. Every wave has
    // retired its reads of stage s-1 before that barrier (the per-step
    // lgkmcnt(0) fence), so s-1's slot is free and AHEAD = RING - 1 stages fly
    // while one is read.
    static constexpr int AHEAD = RING - 1;
    // SPLIT_DMA (8 waves, 2 K-steps per stage): a wave issues the first of its
    // two LDS-DMA pieces of a stage at the barrier that opens the stage before
    // it and the second one at that stage's second K-step, so the weight reads
    // behind a barrier never queue behind two DMA issues (-2.5 %, DESIGN.md
    // §6); otherwise all of a wave's pieces go out at the barrier.
    static constexpr bool SPLIT_DMA = WAVES == 8 && KS == 2 && DPT == 2;
    // vmcnt at a stage-opening barrier, and after an epilogue's (or the
    // prologue's) issue: with SPLIT_DMA only the newest stage's first piece
    static constexpr int VM_OPEN = (AHEAD - 1) * DPT;
    static constexpr int VM_LAYER = SPLIT_DMA ? AHEAD * DPT - 1 : AHEAD * DPT;
    // which of this wave's pieces an opening issues (-1 all, 0 the first) and
    // the stage's second K-step issues (1, SPLIT_DMA only)
    static constexpr int OPEN_PART = SPLIT_DMA ? 0 : -1;
    static constexpr int MID_PART = 1;
    static_assert(RING >= 2 && LDS <= kLdsBytes && STAGE == KS * KSTEP_BYTES, "LDS budget");
    static_assert(KS == 1 || KS == 2 || KS == 4, "K-steps per stage");
    static_assert(ksteps_first(C) % KS == 0 && ksteps_tower(C) % KS == 0, "whole stages per layer");
    static_assert(THREADS >= BOARDS * 64 && DPT >= 1 && VM_LAYER <= 63, "decomposition");
    static_assert(!EDGE || ((NPAIR * BROWS) % 16 == 8 && WAVES == 8), "edge tiles: pair boards 8 rows apart mod 16");
    static_assert(!DIRECT || ((3 * (C / 32)) % WQ == 0 && WQ >= 2), "register queue: whole queues per dx");
};
// throughput geometry: 512 positions x C channels per workgroup, 8 waves of
// 32 channels x 128 positions (edge-row tiles)
template <int C>
using Geo = GeoT<C, 512 / C, 32, C == 128 ? OAMD_C128_RING : OAMD_C256_RING, stage_bytes(C), 128>;
// small-batch geometry (latency): one board per workgroup, 8 waves of C/8
// channels, so a handful of rows spreads over as many CUs as boards. 8 waves
// take 0.098 ms per 16-32 rows against 0.107 with 4 (two same-box pairs,
// bit-identical): in this regime the per-K-step chain of one wave, not the
// fragment reads per MFMA, sets the time; a 4-, 6- or 8-slot ring measured
// equal
template <int C>
using GeoS = GeoT<C, 1, C / 8, 4, kStageBytes>;

template <int DT>
__device__ __forceinline__ uint32_t to_act(float v) {
    if constexpr (DT == OAMD_BF16) {
        return __builtin_bit_cast(uint16_t, (__bf16)v);
    } else {
        return __builtin_bit_cast(uint16_t, (_Float16)v);
    }
}

template <int DT>
__device__ __forceinline__ float from_act(uint32_t u) {
    if constexpr (DT == OAMD_BF16) {
        return __uint_as_float(u << 16);
    } else {
        return (float)__builtin_bit_cast(_Float16, (uint16_t)u);
    }
}

// relu(round(a)), relu(round(b)) packed: v_cvt_pk_{bf16,f16}_f32 (RNE) + v_pk_max_i16
// (a 16-bit float is negative exactly when its bit pattern is a negative i16)
template <int DT>
__device__ __forceinline__ uint32_t pack_relu(float a, float b) {
    i16x2_t s;
    if constexpr (DT == OAMD_BF16) {
        s = __builtin_bit_cast(i16x2_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
    } else {
        s = __builtin_bit_cast(i16x2_t, __builtin_convertvector((f32x2_t){a, b}, f16x2_t));
    }
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(s, (i16x2_t){0, 0}));
}

template <int DT>
__device__ __forceinline__ f32x4_t mfma(u32x4_t a, u32x4_t b, f32x4_t c) {
    if constexpr (DT == OAMD_BF16) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                       __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
    } else {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a),
                                                      __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
    }
}

enum InputKind { kPacked = 0, kF32 = 1 };

// Rows of a launch: without a list, rows 0 .. rows-1; with the search's
// evaluation list (tree.hip append_rows), entry i < rows is row list[i]. The
// launch's grid covers the list's capacity; the entries filled this round are
// counted on the device (resnet_body turns that count into `rows`).
struct RowMap {
    const int32_t* list;
    const int32_t* count;  // filled entries + off (list entries before this launch)
    int off;
    int rows;
    unsigned long long* span;  // launch interval (launch_resnet_packed), or nullptr
};
// row of launch entry r (= workgroup row0 + board), -1 past the end
__device__ __forceinline__ int map_row(const RowMap& M, int r) {
    if (r >= M.rows) return -1;
    return M.list ? M.list[r] : r;
}

// Fragments of one K-step: 4 weight tiles (A: 16 channels x 32 K) and
// 4 activation tiles (B: 32 K x 16 positions).
template <int NT, int MT = 4>
struct Frags {
    u32x4_t w[NT];
    u32x4_t x[MT];
};

// uniform byte offset of the first conv's K-step i (tap-major, tap 8 repeated
// as the zero-weight pad step) relative to the lane bases
template <int C>
__device__ __forceinline__ int first_kstep_offset(int i) {
    const int tap = i < 9 ? i : 8;
    const int dy = tap / 3 - 1, dx = tap - 3 * (tap / 3) - 1;
    return (dy * 10 + dx) * Geo<C>::RP;
}
// ... and of the tower's K-step 0 (dx = -1, dy = -1, channel block 0)
template <int C>
__device__ __forceinline__ int tower_kstep0_offset() {
    return (-10 - 1) * Geo<C>::RP;
}

// ds_read the fragments of one K-step: wk = its weights in the ring (uniform),
// aoff = the K-step's uniform offset; rd[m] / wl are per-lane bases
template <int NT, int MT>
__device__ __forceinline__ void load_wfrags(Frags<NT, MT>& f, const unsigned char* wk, int wl) {
    const unsigned char* wp = wk + wl;
#pragma unroll
    for (int n = 0; n < NT; ++n) f.w[n] = *reinterpret_cast<const u32x4_t*>(wp + n * 1024);
}

template <int NT, int MT>
__device__ __forceinline__ void load_xfrags(Frags<NT, MT>& f, const unsigned char* act, int aoff, const int (&rd)[MT]) {
    const unsigned char* ap = act + aoff;
#pragma unroll
    for (int m = 0; m < MT; ++m) f.x[m] = *reinterpret_cast<const u32x4_t*>(ap + rd[m]);
}

template <int NT, int MT>
__device__ __forceinline__ void load_frags(Frags<NT, MT>& f, const unsigned char* act, const unsigned char* wk,
                                           int aoff, const int (&rd)[MT], int wl) {
    load_wfrags(f, wk, wl);
    load_xfrags(f, act, aoff, rd);
}

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>), in order
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (N > 0) {
        static_for<N - 1>(f);
        f(std::integral_constant<int, N - 1>{});
    }
}

template <int DT, int NT, int MT>
__device__ __forceinline__ void mfma_frags(f32x4_t (&acc)[NT][MT], const Frags<NT, MT>& f) {
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[n][m] = mfma<DT>(f.w[n], f.x[m], acc[n][m]);
}

// LDS-DMA of the weight stage at `src` into ring slot `slot`. The stream
// pointer advances by one stage per opening (a loop-carried scalar: the
// compiler cannot hoist every stage's address to the top of a layer); stages
// past the last one read the zero pad behind the packed weights
// (resnet_packed_weight_alloc_elems) into a slot nobody reads any more, so
// the issue stays branch-free and the vmcnt bookkeeping uniform.
// PART: -1 = all of this wave's pieces of the stage; 0 / 1 = its first /
// second piece (G::SPLIT_DMA).
template <class G, int PART = -1>
__device__ __forceinline__ void issue_stage_dma(const unsigned char* src, unsigned char* ring, int slot, int tid) {
    unsigned char* dst = ring + slot * G::STAGE;
    const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int i = 0; i < G::DPT; ++i) {
        if (PART >= 0 && i != PART) continue;
        const int q = i * G::THREADS + wave * 64;  // first 16-byte chunk of this wave's piece
        __builtin_amdgcn_global_load_lds(src + (size_t)(q + lane) * 16, (lds_void_t*)(dst + q * 16), 16, 0, 0);
    }
}

// s_waitcnt vmcnt(N): all but this wave's N youngest LDS-DMA / global ops done
// (gfx9 encoding: vmcnt[3:0], expcnt[6:4] = 7, lgkmcnt[11:8] = 15: no wait on those)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);  // vmcnt[3:0], vmcnt[5:4] at 15:14
    asm volatile("" ::: "memory");
}

// Workgroup barrier that keeps LDS-DMA in flight: __syncthreads()' fence would
// add vmcnt(0). This wave's LDS accesses complete first (lgkmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Policy and value heads, all waves of the workgroup together (called by every
// thread; barriers inside). The Linear layers run k-split with every board on
// every lane, so a workgroup reads each head weight once (not once per board):
//   phase 1  both 1x1 convs + BN + ReLU of a board as one MFMA GEMM
//            (16 rows: 2 policy, 1 value, 13 zero) on one wave per board;
//            results go to `scratch`, the drained weight ring;
//   phase 2  partial dot products over 32-input chunks, lane = output unit,
//            one task per (chunk, 64-unit slice);
//   phase 3  per board: chunks summed in a fixed order, policy logit 64 (a
//            reduction over squares), softmax(65) / ReLU, Linear(hidden->1), tanh.
// Every output's arithmetic order is independent of BOARDS / WAVES, so all
// geometries produce identical bits.
constexpr int kMaxValueHidden = 1024;  // scratch budget (capi.hip validates)
template <int B>
__host__ __device__ constexpr int head_scratch_floats(int hidden) {
    return 128 * B + 64 * B + 4 * B * 64 + 2 * B * ((hidden + 63) / 64) * 64;
}

#ifdef OAMD_STAMPS
// Diagnostic build only (tools/nn_stamps.py): per workgroup, wave 0 lane 0
// records s_memrealtime (100 MHz) at kernel entry, after the prologue barrier,
// after the tower, and at exit, plus s_memtime cycles across the tower and the
// hardware id of its CU. Nothing else reads this buffer.
__device__ unsigned long long g_oamd_stamps[kMaxStampWgs * kStampStride];
__device__ __forceinline__ void stamp(int slot, int wave, int lane) {
    if (wave == 0 && lane == 0 && blockIdx.x < kMaxStampWgs) {
        __builtin_amdgcn_sched_barrier(0);
        g_oamd_stamps[blockIdx.x * kStampStride + slot] = __builtin_amdgcn_s_memrealtime();
        if (slot == 1 || slot == 2) g_oamd_stamps[blockIdx.x * kStampStride + 4 + slot] = __builtin_amdgcn_s_memtime();
        if (slot == 0) {
            unsigned id;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
            unsigned xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            g_oamd_stamps[blockIdx.x * kStampStride + 4] = ((unsigned long long)xcc << 32) | id;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}
#define OAMD_STAMP(slot) stamp(slot, wave, lane)
#else
#define OAMD_STAMP(slot) ((void)0)
#endif

// acc[b] += sum_k w[k] x[k][b], k in order; x in LDS ([k][B], broadcast reads),
// in chunks of 8 inputs so the reads of one chunk are live at a time
template <int B>
__device__ __forceinline__ void dot32(float (&acc)[B], const float (&w)[32], const float* x) {
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 8) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = k0; k < k0 + 8; ++k)
#pragma unroll
            for (int b = 0; b < B; ++b) acc[b] = __builtin_fmaf(w[k], x[k * B + b], acc[b]);
    }
}

template <class G, int DT>
__device__ __forceinline__ void heads(const NetView& N, const unsigned char* act, unsigned char* scratch, int wave,
                                      int lane, int row0, const RowMap& M, float* __restrict__ policy,
                                      float* __restrict__ value) {
    constexpr int C = G::C;
    constexpr int B = G::BOARDS;
    constexpr int NW = G::WAVES;
    static_assert(head_scratch_floats<B>(kMaxValueHidden) * 4 <= G::RING * G::STAGE, "head scratch");
    // opaque to the optimiser: keeps the heads' lane-derived addresses from
    // being hoisted to the kernel start and held live through the tower
    asm volatile("" : "+v"(lane));
    const HeadLayout HL(C, N.hidden);
    const float* hp = N.head;
    const int hid = N.hidden;
    const int nvs = (hid + 63) / 64;  // 64-unit slices of the value hidden layer
    float* sp = reinterpret_cast<float*>(scratch);  // [128][B] policy conv outputs (k = c*64 + square)
    float* sv = sp + 128 * B;                       // [64][B]  value conv outputs
    float* pp = sv + 64 * B;                        // [4][B][64] policy partials
    float* pv = pp + 4 * B * 64;                    // [2][B][nvs*64] value partials

    // Linear weights of this wave's phase-2 task (one column of 32 inputs per
    // lane): task t < 4 covers policy inputs 32t.., task 4 + 2q + c value
    // units 64q.. over inputs 32c... Issued first, so their global round trip
    // overlaps the conv-weight copy and phase 1.
    auto task_weights = [&](int task, float (&wv)[32]) {
        const float* w;
        int stride;
        if (task < 4) {
            w = hp + HL.plw + task * 32 * 65 + lane;
            stride = 65;
        } else {
            const int t = task - 4, c = t & 1, j = (t >> 1) * 64 + lane;
            w = hp + HL.v1w + c * 32 * hid + (j < hid ? j : hid - 1);
            stride = hid;
        }
#pragma unroll
        for (int k = 0; k < 32; ++k) wv[k] = w[k * stride];
    };
    const int ntask = 4 + 2 * nvs;
    float wv[32];
    // waves without phase-1 work issue their first task's weights now
    if (wave % G::WPB != 0 && wave < ntask) task_weights(wave, wv);
    OAMD_STAMP(8);
    // phase 1: both 1x1 convs of a board as one small MFMA GEMM on the wave
    // that owns the board's first channel block: A = folded head conv weights
    // (rows 0, 1 = policy channels, row 2 = value, rows 3-15 zero; packed in
    // fragment order on the host), B = the tower output at the centre tap.
    if (wave % G::WPB == 0) {
        const int b = wave / G::WPB;
        u32x4_t hw[C / 32];
#pragma unroll
        for (int cb = 0; cb < C / 32; ++cb)
            hw[cb] = *reinterpret_cast<const u32x4_t*>(N.hconv + ((size_t)cb * 64 + lane) * 8);
        int rd[4];
#pragma unroll
        for (int m = 0; m < 4; ++m)
            rd[m] = (b * G::BROWS + G::prow(kTilePos.p[16 * m + (lane & 15)])) * G::RP + kgroup_chunk(lane >> 4) * 16;
        f32x4_t d[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) d[m] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int cb = 0; cb < C / 32; ++cb)
#pragma unroll
            for (int m = 0; m < 4; ++m)
                d[m] = mfma<DT>(hw[cb], *reinterpret_cast<const u32x4_t*>(act + rd[m] + cb * 64), d[m]);
        if (lane < 16) {  // rows 0-3 of output column `lane` of each position tile
            const float pb0 = hp[HL.pcb + 0], pb1 = hp[HL.pcb + 1], vb = hp[HL.vcb];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int pos = kTilePos.p[16 * m + lane];
                sp[pos * B + b] = fmaxf(d[m][0] + pb0, 0.0f);
                sp[(64 + pos) * B + b] = fmaxf(d[m][1] + pb1, 0.0f);
                sv[pos * B + b] = fmaxf(d[m][2] + vb, 0.0f);
            }
        }
    }
    __syncthreads();
    OAMD_STAMP(9);
    for (int task = wave; task < ntask; task += NW) {
        float acc[B];
#pragma unroll
        for (int b = 0; b < B; ++b) acc[b] = 0.0f;
        if (task != wave || wave % G::WPB == 0) task_weights(task, wv);
        if (task < 4) {  // policy Linear(128->64 of 65), inputs 32*task ..
            const float* x = sp + task * 32 * B;
            dot32<B>(acc, wv, x);
#pragma unroll
            for (int b = 0; b < B; ++b) pp[(task * B + b) * 64 + lane] = acc[b];
        } else {  // value Linear(64->hidden), units 64*q + lane, inputs 32*c ..
            const int t = task - 4, c = t & 1, q = t >> 1;
            const int j = q * 64 + lane;
            const float* x = sv + c * 32 * B;
            dot32<B>(acc, wv, x);
#pragma unroll
            for (int b = 0; b < B; ++b) pv[(c * B + b) * nvs * 64 + j] = acc[b];
        }
    }
    __syncthreads();
    OAMD_STAMP(10);
    for (int job = wave; job < 2 * B; job += NW) {
        const int b = job % B;
        const int gr = map_row(M, row0 + b);
        if (gr < 0) continue;
        if (job < B) {
            const float o = hp[HL.plb + lane] + (((pp[(0 * B + b) * 64 + lane] + pp[(1 * B + b) * 64 + lane]) +
                                                  pp[(2 * B + b) * 64 + lane]) +
                                                 pp[(3 * B + b) * 64 + lane]);
            // policy logit 64: a reduction over squares (lane = square)
            const float u0 = hp[HL.plw + lane * 65 + 64], u1 = hp[HL.plw + (64 + lane) * 65 + 64];
            float o64 = __builtin_fmaf(u1, sp[(64 + lane) * B + b], u0 * sp[lane * B + b]);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) o64 += __shfl_xor(o64, off);
            o64 += hp[HL.plb + 64];
            float m = o;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
            m = fmaxf(m, o64);
            const float e = __expf(o - m);
            const float e64 = __expf(o64 - m);
            float ssum = e;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) ssum += __shfl_xor(ssum, off);
            ssum += e64;
            const float inv = 1.0f / ssum;
            policy[(size_t)gr * 65 + lane] = e * inv;
            if (lane == 0) policy[(size_t)gr * 65 + 64] = e64 * inv;
        } else {
            // Linear(hidden->1) over ReLU(Linear(64->hidden)), tanh
            float part = 0.0f;
            for (int q = 0; q < nvs; ++q) {
                const int j = q * 64 + lane;
                if (j < hid) {
                    const float h = hp[HL.v1b + j] + (pv[(0 * B + b) * nvs * 64 + j] + pv[(1 * B + b) * nvs * 64 + j]);
                    part = __builtin_fmaf(fmaxf(h, 0.0f), hp[HL.v2w + j], part);
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
            if (lane == 0) value[gr] = tanhf(part + hp[HL.v2b]);
        }
    }
}

template <class G>
__device__ __forceinline__ void load_bias(float4 (&bv)[G::NT], const NetView& N, int layer, int wn, int lane) {
#pragma unroll
    for (int n = 0; n < G::NT; ++n)
        bv[n] = *reinterpret_cast<const float4*>(N.bias + (size_t)layer * G::C + out_chan(wn * G::NT + n, lane >> 4, 0));
}

template <class G, int DT, int IN>
__device__ __forceinline__ void resnet_body(NetView N, const void* __restrict__ feat_in, int fw, int H, RowMap M,
                                            float* __restrict__ policy, float* __restrict__ value, int wg) {
    constexpr int C = G::C;
    constexpr int kNT = G::NT;
    constexpr int kMT = G::MT;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* act = smem;
    unsigned char* ring = smem + G::ACT_BYTES;

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    const int wm = wave / G::WN;  // position group of this wave (EDGE: edge_tile_row; else its board)
    const int wn = wave % G::WN;  // 32-channel block of this wave
    const int kg = lane >> 4;
    const int row0 = wg * G::BOARDS;  // this workgroup's first board of the launch
    if (M.list) {  // entries filled this round (a uniform scalar load)
        const int filled = *M.count - M.off;
        M.rows = filled < M.rows ? (filled > 0 ? filled : 0) : M.rows;
        // a workgroup past the filled entries has nothing to do: it leaves
        // before its first weight DMA (the launch's grid is the list capacity)
        if (row0 >= M.rows) return;
    }
    OAMD_STAMP(0);
#ifdef OAMD_STAMPS
    // epilogue cycle sums: first barrier, stores, second barrier + first reads
    unsigned long long ep_sum[3] = {0, 0, 0}, ep_t = 0;
    unsigned long long wt_sum[3] = {0, 0, 0};  // lgkmcnt, vmcnt, stage barrier waits
    // a step's stamps (s_memtime, an SMEM read counted in lgkmcnt) are read
    // only after the NEXT step's lgkmcnt(0), which the kernel waits for anyway:
    // consuming one earlier would drain the fragment reads in flight and
    // change what is measured. pw[0] = before the step's lgkmcnt(0), [1]
    // after it, [2] after the stage-open vmcnt wait, [3] after the barrier
    unsigned long long pw[4] = {0, 0, 0, 0};
    bool pw_on = false, pw_open = false;
#define OAMD_EP_MARK(k)                                                          \
    do {                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                       \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();              \
        if ((k) > 0) ep_sum[(k) - 1] += t_ - ep_t;                               \
        ep_t = t_;                                                               \
        __builtin_amdgcn_sched_barrier(0);                                       \
    } while (0)
#define OAMD_T() __builtin_amdgcn_s_memtime()
#define OAMD_STEP_WAIT(stmt)                                                     \
    do {                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                       \
        const unsigned long long w0_ = OAMD_T();                                 \
        stmt;                                                                    \
        if (pw_on) {                                                             \
            wt_sum[0] += pw[1] - pw[0];                                          \
            if (pw_open) {                                                       \
                wt_sum[1] += pw[2] - pw[1];                                      \
                wt_sum[2] += pw[3] - pw[2];                                      \
            }                                                                    \
        }                                                                        \
        pw[0] = w0_;                                                             \
        pw[1] = OAMD_T();                                                        \
        pw_on = true;                                                            \
        pw_open = false;                                                         \
        __builtin_amdgcn_sched_barrier(0);                                       \
    } while (0)
#define OAMD_OPEN_WAIT(vmstmt, barstmt)                                          \
    do {                                                                         \
        vmstmt;                                                                  \
        pw[2] = OAMD_T();                                                        \
        barstmt;                                                                 \
        pw[3] = OAMD_T();                                                        \
        pw_open = true;                                                          \
    } while (0)
#else
#define OAMD_EP_MARK(k) ((void)0)
#define OAMD_STEP_WAIT(stmt) stmt
#define OAMD_OPEN_WAIT(vmstmt, barstmt) \
    do {                                 \
        vmstmt;                          \
        barstmt;                         \
    } while (0)
#endif
    const unsigned char* wsrc = reinterpret_cast<const unsigned char*>(N.w);

    // weight stream starts right away: stages 0 .. AHEAD (with SPLIT_DMA the
    // newest stage's second piece goes out at stage 0's second K-step)
    const unsigned char* wcur = wsrc + G::AHEAD * G::STAGE;  // the newest stage issued
    if constexpr (!G::DIRECT) {
#pragma unroll
        for (int s = 0; s < G::AHEAD; ++s) issue_stage_dma<G>(wsrc + s * G::STAGE, ring, s, tid);
        issue_stage_dma<G, G::OPEN_PART>(wcur, ring, G::AHEAD, tid);
    }

    float4 bv[kNT];  // folded bias of this lane's output channels (current layer)
    load_bias<G>(bv, N, 0, wn, lane);

    // per-lane bases: fragment reads (row of position tile m + k-group chunk),
    // epilogue writes (row + k-group's 8-byte half chunk), weight fragments
    // (edge-row tiles: tile m is board row m, one lane base + m x 10 rows, so
    // every tile's offset folds into the LDS instructions' immediates)
    int rd[kMT], wr[kMT];
    const int erow0 = G::EDGE ? edge_tile_row<G>(wm, 0, lane & 15) * G::RP : 0;
#pragma unroll
    for (int m = 0; m < kMT; ++m) {
        const int rowb = G::EDGE ? erow0 + m * 10 * G::RP
                                 : (wm * G::BROWS + G::prow(kTilePos.p[16 * m + (lane & 15)])) * G::RP;
        rd[m] = rowb + kgroup_chunk(kg) * 16;
        wr[m] = rowb;
    }
    const int wl = (wn * kNT * 64 + lane) * 16;

    // DIRECT: K-step g's weight fragments live in wq[g % WQ]; the K-step whose
    // MFMAs a step issues loads K-step g + WQ - 1 (the stream pointer wgp is
    // uniform, the lane's fragment offset wl). The packed weights run on
    // through the first conv's pad step and every layer, so g counts K-steps
    // over the whole network (tower layers start at g = WOFF mod WQ); loads
    // past the last K-step read the zero pad behind the weights.
    constexpr int WQ = G::DIRECT ? G::WQ : 1;
    constexpr int WOFF = ksteps_first(C) % WQ;
    u32x4_t wq[WQ][kNT];
    const unsigned char* wgp = wsrc;
    auto wload = [&](auto SLOT) {
        constexpr int q = decltype(SLOT)::value % WQ;
#pragma unroll
        for (int n = 0; n < kNT; ++n) wq[q][n] = *reinterpret_cast<const u32x4_t*>(wgp + wl + n * 1024);
        wgp += G::KSTEP_BYTES;
    };
    if constexpr (G::DIRECT) static_for<WQ - 1>([&](auto I) { wload(I); });

    // ---------------- zero border rows; input planes -> channels 0..31 ------
    // border cells per board: bordered boards 10 top + 10 bottom + 16 side,
    // edge-row boards only the 16 side cells (x = -1, 8 of rows 0-7)
    constexpr int NBC = G::ROW0 ? 36 : 16;
    for (int w = tid; w < G::BOARDS * NBC * (C / 8); w += G::THREADS) {
        const int c = w % (C / 8), k = (w / (C / 8)) % NBC, b = w / (C / 8) / NBC;
        const int r = G::ROW0 ? (k < 10 ? k : (k < 20 ? 80 + k : ((k - 20) >> 1) * 10 + 10 + ((k & 1) ? 9 : 0)))
                              : (k >> 1) * 10 + ((k & 1) ? 9 : 0);
        *reinterpret_cast<u32x4_t*>(act + (b * G::BROWS + r) * G::RP + c * 16) = u32x4_t{0u, 0u, 0u, 0u};
    }
    if (tid < G::BOARDS * 64) {
        const int b = tid >> 6, p = tid & 63;
        const int gr = map_row(M, row0 + b);
        const uint32_t one = to_act<DT>(1.0f);
        uint32_t words[16];  // 32 channels as 16-bit pairs
        // one global round trip per board: the wave of board b (lane = square)
        // issues all its input loads before using any of them
        if constexpr (IN == kPacked) {
            uint32_t mask = 0;  // bit c = channel c is 1 (c < 31)
            if (gr >= 0) {      // wave-uniform
                // lane j holds word j of the row (fw = 2 + 2H <= 32 words)
                const uint64_t* fr = reinterpret_cast<const uint64_t*>(feat_in) + (size_t)gr * fw;
                const uint64_t wj = fr[p < fw ? p : fw - 1];
                const uint32_t lo = (uint32_t)wj, hi = (uint32_t)(wj >> 32);
                auto word = [&](int j) {
                    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, j) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)lo, j);
                };
                const uint64_t meta = word(0);
                if ((meta >> 16) & 1ULL) {
                    const int t = (int)((meta >> 8) & 7ULL);
                    const int src = inverse_transform(p, t);
                    mask = (uint32_t)(meta & 1ULL);
                    for (int h = 0; h < H; ++h) {
                        mask |= (uint32_t)((word(2 + 2 * h) >> (63 - src)) & 1ULL) << (1 + 2 * h);
                        mask |= (uint32_t)((word(3 + 2 * h) >> (63 - src)) & 1ULL) << (2 + 2 * h);
                    }
                }
            }
#pragma unroll
            for (int w = 0; w < 16; ++w) {
                const uint32_t lo = ((mask >> (2 * w)) & 1u) ? one : 0u;
                const uint32_t hi = ((mask >> (2 * w + 1)) & 1u) ? one : 0u;
                words[w] = lo | (hi << 16);
            }
        } else {
            float v[32];
#pragma unroll
            for (int c = 0; c < 32; ++c) v[c] = 0.0f;
            if (gr >= 0) {  // wave-uniform; channel index clamped so all 32 loads issue at once
                const float* fr = reinterpret_cast<const float*>(feat_in) + (size_t)gr * N.cin * 64;
#pragma unroll
                for (int c = 0; c < 32; ++c) v[c] = fr[(c < N.cin ? c : N.cin - 1) * 64 + p];
            }
#pragma unroll
            for (int w = 0; w < 16; ++w) {
                const int c0 = 2 * w, c1 = 2 * w + 1;
                const uint32_t lo = c0 < N.cin ? to_act<DT>(v[c0]) : 0u;
                const uint32_t hi = c1 < N.cin ? to_act<DT>(v[c1]) : 0u;
                words[w] = lo | (hi << 16);
            }
        }
        unsigned char* dst = act + (b * G::BROWS + G::prow(p)) * G::RP;
#pragma unroll
        for (int c = 0; c < 4; ++c)
            *reinterpret_cast<u32x4_t*>(dst + c * 16) =
                u32x4_t{words[4 * c], words[4 * c + 1], words[4 * c + 2], words[4 * c + 3]};
    }

    f32x4_t acc[kNT][kMT];
    u32x2_t skip[kNT][kMT];  // residual (block input) of this lane's outputs

    Frags<kNT, kMT> fa, fb;
    // edge-row tiles: the activation fragments of the current / next channel
    // block come from register windows of board rows (fa / fb carry weights)
    constexpr bool kWide = G::EDGE;
    u32x4_t win0[kWide ? 9 : 1], win1[kWide ? 9 : 1];
    // window base: this lane's column, board row -1, dx = -1
    const int sb0 = rd[0] - 10 * G::RP - G::RP;
    int slot = 0;  // ring slot of the stage holding the current K-step

    OAMD_STAMP(7);
    if constexpr (IN == kPacked) {
        // Terminal leaves need no evaluation: the reference builds no NN row
        // for them and skips a thread's NN call when its whole batch is
        // terminal (search_thread.cpp:83-111); their policy / value rows are
        // never read (backup_range scores them from the discs). A workgroup
        // whose boards are all terminal (or past the end) therefore stops
        // here, once its weight DMAs have landed (the LDS they write is
        // released with the workgroup). Scalar loads of uniform addresses.
        bool live = false;
#pragma unroll
        for (int b = 0; b < G::BOARDS; ++b) {
            const int gr = map_row(M, row0 + b);
            if (gr >= 0) live |= ((reinterpret_cast<const uint64_t*>(feat_in)[(size_t)gr * fw] >> 16) & 1ULL) != 0;
        }
        if (!live) {
            wait_vm<0>();
            return;
        }
    }
    // stage 0 and the input planes must be visible (bias loads are older than the DMAs)
    if constexpr (!G::DIRECT) wait_vm<G::VM_LAYER>();
    lds_barrier();
    // the first conv's K-step 0 (tap 0, dy = -1: edge-row geometries skip tile 0)
    if constexpr (!G::DIRECT) load_wfrags(fa, ring, wl);
#pragma unroll
    for (int m = kWide ? 1 : 0; m < kMT; ++m)
        fa.x[m] = *reinterpret_cast<const u32x4_t*>(act + first_kstep_offset<C>(0) + rd[m]);
    OAMD_STAMP(1);
#ifdef OAMD_STAMPS
    const unsigned long long tower_t0 = __builtin_amdgcn_s_memtime();
#endif
    // throughput geometry: every ResNet wave issues ahead of the other pipeline
    // group's co-resident tree waves (SQ arbitration): bench C2 4.42-4.47 vs
    // 4.31-4.36 M sims/s (four same-box pairs on two boxes), launch 0.90-0.91
    // vs 0.92-0.935 ms (the standalone speed), the tree round 0.46 vs 0.34 ms
    // and still hidden behind the other group's launch
    if constexpr (G::BOARDS > 1) __builtin_amdgcn_s_setprio(1);

    const int nlayers = 1 + 2 * N.R;
    // one conv layer: KIND 0 = first conv, 1 = a block's first conv (saves the
    // block input as skip), 2 = a block's second conv (adds skip). Instantiated
    // per kind so `skip` is live only from conv1's epilogue to conv2's start.
    auto conv = [&](auto KIND, int layer) {
        constexpr int kind = decltype(KIND)::value;
        constexpr bool first = kind == 0;
        constexpr int nk = first ? ksteps_first(C) : ksteps_tower(C);

        // accumulators start at bias (+ block input for the block's second conv)
#pragma unroll
        for (int n = 0; n < kNT; ++n)
#pragma unroll
            for (int m = 0; m < kMT; ++m) {
                f32x4_t a = f32x4_t{bv[n].x, bv[n].y, bv[n].z, bv[n].w};
                if constexpr (kind == 2) {
                    const u32x2_t r = skip[n][m];
                    a[0] += from_act<DT>(r.x & 0xffffu);
                    a[1] += from_act<DT>(r.x >> 16);
                    a[2] += from_act<DT>(r.y & 0xffffu);
                    a[3] += from_act<DT>(r.y >> 16);
                }
                acc[n][m] = a;
            }

        // step: load K-step i1's fragments into nxt, then MFMAs on cur (K-step
        // i1-1). KIS: i1's K-step within its stage (0: i1 opens a new stage ->
        // DMA wait + barrier, ring advances). TILES = xlo | xhi << 4 | mlo << 8 |
        // mhi << 12: position tiles [xlo, xhi) of nxt are read and MFMAs run on
        // tiles [mlo, mhi) of cur (edge-row geometries leave out the border
        // tiles of the first conv). xoff: uniform byte offset of the next
        // K-step's activation rows/channels
        auto step = [&](auto KIS, auto TILES, auto GI, const Frags<kNT, kMT>& cur, Frags<kNT, kMT>& nxt, int xoff) {
            constexpr int kis = decltype(KIS)::value;
            constexpr int gi = decltype(GI)::value;  // cur's K-step (DIRECT: first conv only)
            constexpr bool open = kis == 0 && !G::DIRECT;
            constexpr int tl = decltype(TILES)::value;
            constexpr int xlo = tl & 15, xhi = (tl >> 4) & 15, mlo = (tl >> 8) & 15, mhi = (tl >> 12) & 15;
            // keep each step's MFMAs (on cur) with the fragment reads they hide:
            // without this fence the scheduler may hoist the next step's MFMAs over
            // the barrier right behind their reads and drain lgkmcnt each step
            __builtin_amdgcn_sched_barrier(0);
            // cur's reads (issued a step ago) are done: retire them before
            // issuing nxt's, or 16 outstanding reads overflow the 4-bit lgkmcnt
            // and the compiler drains nxt's reads too
            OAMD_STEP_WAIT(__builtin_amdgcn_s_waitcnt(0xC07F));  // lgkmcnt(0)
            // activation fragments do not depend on the stage barrier (the
            // layer's input is fixed): issued before it, their latency overlaps
            // the barrier wait (+3.6 %)
            {
                const unsigned char* ap = act + xoff;
#pragma unroll
                for (int m = xlo; m < xhi; ++m) nxt.x[m] = *reinterpret_cast<const u32x4_t*>(ap + rd[m]);
            }
            if constexpr (open) {
                // open the next stage: it has landed (this wave's DMAs, then
                // everyone's via the barrier), and the slot of the stage before the
                // current one is drained by all waves: the newest stage goes there
                OAMD_OPEN_WAIT(wait_vm<G::VM_OPEN>(), __builtin_amdgcn_s_barrier());
                const int sp = (slot + G::AHEAD + 1) % G::RING;  // (g + 1 + AHEAD) % RING
                wcur += G::STAGE;
                issue_stage_dma<G, G::OPEN_PART>(wcur, ring, sp, tid);
                slot = slot == G::RING - 1 ? 0 : slot + 1;
            } else if constexpr (G::SPLIT_DMA && !G::DIRECT) {
                // the rest of the newest stage (its slot was freed by the barrier
                // that opened the current stage)
                int sa = slot + G::AHEAD;
                sa = sa >= G::RING ? sa - G::RING : sa;
                issue_stage_dma<G, G::MID_PART>(wcur, ring, sa, tid);
            }
            if constexpr (G::DIRECT) wload(std::integral_constant<int, gi + WQ - 1>{});
            else load_wfrags(nxt, ring + slot * G::STAGE + kis * G::KSTEP_BYTES, wl);
#pragma unroll
            for (int n = 0; n < kNT; ++n)
#pragma unroll
                for (int m = mlo; m < mhi; ++m) {
                    if constexpr (G::DIRECT) acc[n][m] = mfma<DT>(wq[gi % WQ][n], cur.x[m], acc[n][m]);
                    else acc[n][m] = mfma<DT>(cur.w[n], cur.x[m], acc[n][m]);
                }
            // fine interleave of the step's fragment reads with its MFMAs (one
            // read, then a share of the MFMAs; +2.5 %): a stage-opening step has
            // only its weight reads after the barrier
            if constexpr (G::DIRECT) {
                constexpr int nds = xhi - xlo;
                constexpr int nm = kNT * (mhi - mlo);
                static_for<nds>([&](auto I) {
                    constexpr int i = decltype(I)::value;
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, (i + 1) * nm / nds - i * nm / nds, 0);
                });
            } else if constexpr (kMT != 4) {
                constexpr int nds = open ? kNT : kNT + (xhi - xlo);
                constexpr int nm = kNT * (mhi - mlo);
                static_for<nds>([&](auto I) {
                    constexpr int i = decltype(I)::value;
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, (i + 1) * nm / nds - i * nm / nds, 0);
                });
            } else {
                constexpr int nds = open ? 4 : 8;
                static_for<nds>([&](auto) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 16 / nds, 0);
                });
            }
        };
        // all tiles read and multiplied
        using AllTiles = std::integral_constant<int, kMT << 4 | kMT << 12>;
        if constexpr (first) {
            // tap-major, K-step i = tap min(i, 8) (the pad steps repeat tap 8
            // with zero weights); edge-row geometries leave out tile 0 at
            // dy = -1 and tile 7 at dy = +1 (rows -1 and 8 are not in the layout)
            auto tiles = [](int i) {
                const int dy = (i < 9 ? i : 8) / 3 - 1;
                const int lo = kWide && dy < 0 ? 1 : 0, hi = kWide && dy > 0 ? kMT - 1 : kMT;
                return lo | hi << 4 | lo << 8 | hi << 12;
            };
            static_for<nk - 1>([&](auto II) {
                constexpr int i1 = decltype(II)::value + 1;  // the K-step this step loads
                constexpr int tl = (tiles(i1) & 0xFF) | (tiles(i1 - 1) & 0xFF00);
                using GI = std::integral_constant<int, i1 - 1>;
                if constexpr (i1 % 2 == 1) step(std::integral_constant<int, i1 % G::KS>{},
                                                std::integral_constant<int, tl>{}, GI{}, fa, fb, first_kstep_offset<C>(i1));
                else step(std::integral_constant<int, i1 % G::KS>{}, std::integral_constant<int, tl>{}, GI{}, fb, fa,
                          first_kstep_offset<C>(i1));
            });
            constexpr int ml = tiles(nk - 1) >> 8 & 15, mh = tiles(nk - 1) >> 12 & 15;
            const Frags<kNT, kMT>& last = (nk - 1) % 2 == 1 ? fb : fa;
            if constexpr (G::DIRECT) wload(std::integral_constant<int, nk - 1 + WQ - 1>{});
#pragma unroll
            for (int n = 0; n < kNT; ++n)
#pragma unroll
                for (int m = ml; m < mh; ++m) {
                    if constexpr (G::DIRECT) acc[n][m] = mfma<DT>(wq[(nk - 1) % WQ][n], last.x[m], acc[n][m]);
                    else acc[n][m] = mfma<DT>(last.w[n], last.x[m], acc[n][m]);
                }
        } else if constexpr (kWide) {
            constexpr int KPT = C / 32;
            static_assert(kNT == 2 && kMT == 8 && KPT % 2 == 0 && (3 * KPT) % G::KS == 0, "wide geometry");
            constexpr int NJ = 3 * KPT;     // K-steps per dx
            constexpr int RS = 10 * G::RP;  // one board row
            // K-step J = (cb J/3, dy J%3 - 1) of the dx: tiles mlo..mhi-1 from
            // window rows m + 1 + dy (tile 0 at dy = -1 and tile 7 at dy = +1
            // read the zero border: left out, every wave alike); reads the
            // window rows K-step J + 1 needs (at sbn: the next dx's base when
            // J = NJ - 1) and its weights
            auto wstep = [&](auto JJ, auto LASTDX, const Frags<kNT, kMT>& wc, Frags<kNT, kMT>& wn, int sbn) {
                constexpr int J = decltype(JJ)::value;
                constexpr int Jn = (J + 1) % NJ;
                constexpr bool open = Jn % G::KS == 0 && !G::DIRECT;
                // rows of the window K-step Jn needs first (the layer's last dx:
                // wide_new_last, OAMD_EPI_NOBAR)
                constexpr int newmask =
                    decltype(LASTDX)::value ? wide_new_last<OAMD_EPI_NOBAR && !G::DIRECT>(Jn, NJ) : wide_new(Jn);
                constexpr int dy = wide_dy(J), cbn = wide_cb(Jn), nnew = __builtin_popcount(newmask);
                constexpr int mlo = dy < 0 ? 1 : 0, mhi = dy > 0 ? 7 : 8;
                auto& Wc = [&]() -> u32x4_t(&)[9] {
                    if constexpr (wide_cb(J) % 2 == 0) return win0; else return win1;
                }();
                auto& Wn = [&]() -> u32x4_t(&)[9] {
                    if constexpr (cbn % 2 == 0) return win0; else return win1;
                }();
                __builtin_amdgcn_sched_barrier(0);
                OAMD_STEP_WAIT(__builtin_amdgcn_s_waitcnt(0xC07F));  // lgkmcnt(0): wc / Wc have landed
                static_for<9>([&](auto I) {
                    constexpr int i = decltype(I)::value;
                    if constexpr ((newmask >> i) & 1)
                        Wn[i] = *reinterpret_cast<const u32x4_t*>(act + sbn + i * RS + cbn * 64);
                });
                if constexpr (open) {
                    OAMD_OPEN_WAIT(wait_vm<G::VM_OPEN>(), __builtin_amdgcn_s_barrier());
                    const int sp = (slot + G::AHEAD + 1) % G::RING;
                    wcur += G::STAGE;
                    issue_stage_dma<G, G::OPEN_PART>(wcur, ring, sp, tid);
                    slot = slot == G::RING - 1 ? 0 : slot + 1;
                } else if constexpr (G::SPLIT_DMA && !G::DIRECT) {
                    int sa = slot + G::AHEAD;
                    sa = sa >= G::RING ? sa - G::RING : sa;
                    issue_stage_dma<G, G::MID_PART>(wcur, ring, sa, tid);
                }
                if constexpr (G::DIRECT) wload(std::integral_constant<int, WOFF + J + WQ - 1>{});
                else load_wfrags(wn, ring + slot * G::STAGE + (Jn % G::KS) * G::KSTEP_BYTES, wl);
#pragma unroll
                for (int n = 0; n < kNT; ++n)
#pragma unroll
                    for (int m = mlo; m < mhi; ++m) {
                        if constexpr (G::DIRECT) acc[n][m] = mfma<DT>(wq[(WOFF + J) % WQ][n], Wc[m + 1 + dy], acc[n][m]);
                        else acc[n][m] = mfma<DT>(wc.w[n], Wc[m + 1 + dy], acc[n][m]);
                    }
                constexpr int nds = G::DIRECT ? nnew : (open ? kNT : kNT + nnew);
                constexpr int nm = kNT * (mhi - mlo);
                static_for<nds>([&](auto I) {
                    constexpr int i = decltype(I)::value;
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, (i + 1) * nm / nds - i * nm / nds, 0);
                });
            };
            auto dx_wide = [&](int dxi, auto LASTDX) {
                constexpr bool lastdx = decltype(LASTDX)::value;
                const int sb = sb0 + dxi * G::RP;
                static_for<lastdx ? NJ - 1 : NJ>([&](auto JJ) {
                    constexpr int J = decltype(JJ)::value;
                    const int sbn = J == NJ - 1 ? sb + G::RP : sb;
                    if constexpr (J % 2 == 0) wstep(JJ, LASTDX, fa, fb, sbn);
                    else wstep(JJ, LASTDX, fb, fa, sbn);
                });
                if constexpr (lastdx) {
                    // the layer's last K-step = (last block, dy +1) in fb / win1
                    if constexpr (G::DIRECT) wload(std::integral_constant<int, WOFF + NJ - 1 + WQ - 1>{});
#pragma unroll
                    for (int n = 0; n < kNT; ++n)
#pragma unroll
                        for (int m = 0; m < 7; ++m) {
                            if constexpr (G::DIRECT) acc[n][m] = mfma<DT>(wq[(WOFF + NJ - 1) % WQ][n], win1[m + 2], acc[n][m]);
                            else acc[n][m] = mfma<DT>(fb.w[n], win1[m + 2], acc[n][m]);
                        }
                }
            };
#pragma nounroll
            for (int dxi = 0; dxi < 2; ++dxi) dx_wide(dxi, std::false_type{});
            dx_wide(2, std::true_type{});
        } else {
            // the tower's order without edge tiles (small-batch geometry):
            // generic steps, every K-step's fragments read
            constexpr int KPT = C / 32;
            static_assert(KPT % 2 == 0, "whole block pairs");
            constexpr int NJ = 3 * KPT;
            auto xoff_of = [](int dxi, int J) { return (wide_dy(J) * 10 + dxi - 1) * G::RP + wide_cb(J) * 64; };
            auto dx_steps = [&](int dxi, auto LASTDX) {
                constexpr bool lastdx = decltype(LASTDX)::value;
                static_for<lastdx ? NJ - 1 : NJ>([&](auto JJ) {
                    constexpr int J = decltype(JJ)::value;
                    using KIS = std::integral_constant<int, (J + 1) % G::KS>;
                    const int xo = J == NJ - 1 ? xoff_of(dxi + 1, 0) : xoff_of(dxi, J + 1);
                    if constexpr (J % 2 == 0) step(KIS{}, AllTiles{}, std::integral_constant<int, 0>{}, fa, fb, xo);
                    else step(KIS{}, AllTiles{}, std::integral_constant<int, 0>{}, fb, fa, xo);
                });
            };
#pragma nounroll
            for (int dxi = 0; dxi < 2; ++dxi) dx_steps(dxi, std::false_type{});
            dx_steps(2, std::true_type{});
            mfma_frags<DT>(acc, fb);  // the layer's last K-step
        }

        // ---------------- epilogue: ReLU, in place --------------------------
        // stages g+1 .. (next layer's) are in flight; the next layer's bias is
        // loaded before the next DMA so the counted wait below covers it
        const bool more = layer + 1 < nlayers;
        if (more) load_bias<G>(bv, N, layer + 1, wn, lane);
#ifdef OAMD_STAMPS
        // the layer's last step: its stamps are complete once the epilogue mark waits
        OAMD_STEP_WAIT(asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"));
        pw_on = false;
#endif
        OAMD_EP_MARK(0);
        // OAMD_EPI_NOBAR: no wave reads this layer's input after the barrier that
        // opened its last stage (wide_new_last), so the stores need no barrier;
        // the last stage's slot is refilled after the post-store barrier
        constexpr bool nobar = OAMD_EPI_NOBAR && kWide && !first && !G::DIRECT;
        const int last_slot = slot;  // the slot of the layer's last stage
        if constexpr (!nobar) {
            lds_barrier();  // every wave is done reading this layer's input and its last stage
        }
        OAMD_EP_MARK(1);
        if constexpr (!G::DIRECT && !nobar) {
            wcur += G::STAGE;
            issue_stage_dma<G, G::OPEN_PART>(wcur, ring, (slot + G::AHEAD + 1) % G::RING, tid);
        }
        if constexpr (kNT == 2) {
            // the wave's two channel tiles hold 8 contiguous channels per lane
            // (out_chan): one 16-byte store (and skip read) per position tile
            const int co = 2 * out_chan(wn * 2, kg, 0);
#pragma unroll
            for (int m = 0; m < kMT; ++m) {
                u32x4_t* p = reinterpret_cast<u32x4_t*>(act + wr[m] + co);
                if constexpr (kind == 1) {  // block input, needed by conv2
                    const u32x4_t v = *p;
                    skip[0][m] = u32x2_t{v.x, v.y};
                    skip[1][m] = u32x2_t{v.z, v.w};
                }
                const f32x4_t a = acc[0][m], b = acc[1][m];
                *p = u32x4_t{pack_relu<DT>(a[0], a[1]), pack_relu<DT>(a[2], a[3]), pack_relu<DT>(b[0], b[1]),
                             pack_relu<DT>(b[2], b[3])};
            }
        } else {
#pragma unroll
            for (int n = 0; n < kNT; ++n)
#pragma unroll
                for (int m = 0; m < kMT; ++m) {
                    u32x2_t* p = reinterpret_cast<u32x2_t*>(act + wr[m] + 2 * out_chan(wn * kNT + n, kg, 0));
                    if constexpr (kind == 1) skip[n][m] = *p;  // block input, needed by conv2
                    const f32x4_t a = acc[n][m];
                    *p = u32x2_t{pack_relu<DT>(a[0], a[1]), pack_relu<DT>(a[2], a[3])};
                }
        }
        slot = slot == G::RING - 1 ? 0 : slot + 1;
        OAMD_EP_MARK(2);
        if (more) {
            // the next layer's first stage has landed (later may fly; with
            // nobar the epilogue's DMA is not issued yet: one fewer in flight)
            if constexpr (!G::DIRECT) wait_vm<nobar ? G::VM_LAYER - 1 : G::VM_LAYER>();
            lds_barrier();  // ... and this layer's output is complete
            if constexpr (!G::DIRECT && nobar) {
                // every wave is past its last K-step: the last stage's slot is free
                wcur += G::STAGE;
                issue_stage_dma<G, G::OPEN_PART>(wcur, ring, (last_slot + G::AHEAD + 1) % G::RING, tid);
            }
            if constexpr (kWide) {
                if constexpr (!G::DIRECT) load_wfrags(fa, ring + slot * G::STAGE, wl);
#pragma unroll
                for (int i = 1; i < 8; ++i) win0[i] = *reinterpret_cast<const u32x4_t*>(act + sb0 + i * 10 * G::RP);
            } else {
                load_frags(fa, act, ring + slot * G::STAGE, tower_kstep0_offset<C>(), rd, wl);
            }
#ifdef OAMD_STAMPS
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
        }
        OAMD_EP_MARK(3);
    };
    conv(std::integral_constant<int, 0>{}, 0);
    for (int blk = 0; blk < N.R; ++blk) {
        conv(std::integral_constant<int, 1>{}, 1 + 2 * blk);
        conv(std::integral_constant<int, 2>{}, 2 + 2 * blk);
    }
    __syncthreads();  // also drains this wave's trailing ring DMAs: the ring is free
    OAMD_STAMP(2);
#ifdef OAMD_STAMPS
    const unsigned long long tower_cyc = __builtin_amdgcn_s_memtime() - tower_t0;
#endif
#ifdef OAMD_STAMPS
    if (wave == 0 && lane == 0 && blockIdx.x < kMaxStampWgs)
        for (int i = 0; i < 3; ++i) g_oamd_stamps[blockIdx.x * kStampStride + 11 + i] = ep_sum[i];
    if (lane == 0 && blockIdx.x < kMaxStampWgs) {
        unsigned long long* q = g_oamd_stamps + blockIdx.x * kStampStride + 16;
        for (int i = 0; i < 3; ++i) atomicAdd(q + i, wt_sum[i]);
        for (int i = 0; i < 3; ++i) atomicAdd(q + 3 + i, ep_sum[i]);
        atomicAdd(q + 6, tower_cyc);
    }
#endif
    heads<G, DT>(N, act, ring, wave, lane, row0, M, policy, value);
    OAMD_STAMP(3);
}

// Every geometry is 8 waves (2 per SIMD), capped at 208 VGPRs: that leaves 96
// of a SIMD's 512 for one k_tree wave (<= 96 VGPRs, no LDS), so the other
// pipeline group's tree kernel co-resides with this kernel instead of waiting
// for a CU. amdgpu_num_vgpr counts in units of the unified VGPR+AGPR file on
// gfx950 (the backend doubles it), hence OAMD_VGPR_CAP = 104; build.py checks
// the resulting allocation.
template <class G, int DT, int IN>
__global__ __launch_bounds__(512) __attribute__((amdgpu_num_vgpr(OAMD_VGPR_CAP))) void k_resnet_w8(
    NetView N, const void* __restrict__ feat_in, int fw, int H, RowMap M, float* __restrict__ policy,
    float* __restrict__ value) {
    // timed searches: the launch's execution interval over all its workgroups
    // (the union of these intervals is the bench's busy time; a HIP event pair
    // would add the dispatch latency of every launch, which near-empty
    // endgame launches nobody overlaps make visible). Every early return of
    // resnet_body is workgroup-uniform, so all threads meet at the barrier.
    if (M.span && threadIdx.x == 0) atomicMax(M.span, ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
    resnet_body<G, DT, IN>(N, feat_in, fw, H, M, policy, value, blockIdx.x);
    if (M.span) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(M.span + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}

// The chain-splitting extra rounds' launches (lagging games' rows only, none
// outside endgames) on a small grid that loops over the list's board groups:
// the regular grid (the list's capacity, ~1000 workgroups of 139 KB of LDS)
// would put each of its empty workgroups on a CU for a moment, between the
// other NN chain's workgroups. Same per-board arithmetic, bit-identical.
template <class G, int DT, int IN>
__global__ __launch_bounds__(512) __attribute__((amdgpu_num_vgpr(OAMD_VGPR_CAP))) void k_resnet_w8_loop(
    NetView N, const void* __restrict__ feat_in, int fw, int H, RowMap M, float* __restrict__ policy,
    float* __restrict__ value) {
    if (M.span && threadIdx.x == 0) atomicMax(M.span, ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
    int rows = M.rows;
    if (M.list) {
        const int filled = *M.count - M.off;
        rows = filled < rows ? (filled > 0 ? filled : 0) : rows;
    }
    for (int wg = blockIdx.x; wg * G::BOARDS < rows; wg += gridDim.x) {
        resnet_body<G, DT, IN>(N, feat_in, fw, H, M, policy, value, wg);
        __syncthreads();  // the heads' scratch (the drained ring) is read before the next group's DMA
    }
    if (M.span) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(M.span + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}

template <class G, int DT, int IN>
static void launch_t(const NetView& N, const void* feat, int fw, int H, const RowMap& M, float* pol, float* val,
                     hipStream_t s, int max_wgs) {
    const int rows = M.rows;
    static_assert(G::THREADS == 512, "k_resnet_w8 geometries");
    const unsigned grid = (unsigned)((rows + G::BOARDS - 1) / G::BOARDS);
    constexpr auto kern = &k_resnet_w8<G, DT, IN>;
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  G::LDS);
        configured = true;
    }
    if constexpr (IN == kPacked) {
        if (max_wgs > 0 && grid > (unsigned)max_wgs) {
            constexpr auto lk = &k_resnet_w8_loop<G, DT, IN>;
            static bool lconfigured = false;
            if (!lconfigured) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(lk),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
                lconfigured = true;
            }
            hipLaunchKernelGGL(lk, dim3(max_wgs), dim3(G::THREADS), G::LDS, s, N, feat, fw, H, M, pol, val);
            return;
        }
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(G::THREADS), G::LDS, s, N, feat, fw, H, M, pol, val);
}

// Below kSmallBatchRows rows the throughput geometry would leave most CUs idle
// and its per-workgroup latency (4 or 2 boards through the whole tower) sets
// the call's latency: one board per workgroup instead. The K order and MFMA
// tiling per output are the same, so results are bit-identical.
constexpr int kSmallBatchRows = 1024;

template <int IN>
static void dispatch(const NetView& N, const void* feat, int fw, int H, const RowMap& M, float* pol, float* val,
                     hipStream_t s, int max_wgs = 0) {
    const int rows = M.rows;
    if (rows <= 0) return;
    const bool small = rows < kSmallBatchRows;
    const bool fp16 = N.dtype == OAMD_FP16;
    if (N.C == 128) {
        if (small) {
            if (fp16) launch_t<GeoS<128>, OAMD_FP16, IN>(N, feat, fw, H, M, pol, val, s, max_wgs);
            else launch_t<GeoS<128>, OAMD_BF16, IN>(N, feat, fw, H, M, pol, val, s, max_wgs);
        } else {
            if (fp16) launch_t<Geo<128>, OAMD_FP16, IN>(N, feat, fw, H, M, pol, val, s, max_wgs);
            else launch_t<Geo<128>, OAMD_BF16, IN>(N, feat, fw, H, M, pol, val, s, max_wgs);
        }
    } else {
        if (small) {
            if (fp16) launch_t<GeoS<256>, OAMD_FP16, IN>(N, feat, fw, H, M, pol, val, s, max_wgs);
            else launch_t<GeoS<256>, OAMD_BF16, IN>(N, feat, fw, H, M, pol, val, s, max_wgs);
        } else {
            if (fp16) launch_t<Geo<256>, OAMD_FP16, IN>(N, feat, fw, H, M, pol, val, s, max_wgs);
            else launch_t<Geo<256>, OAMD_BF16, IN>(N, feat, fw, H, M, pol, val, s, max_wgs);
        }
    }
}

void launch_resnet_packed(const NetView& N, const uint64_t* feat, int fw, int H, int rows,
                          float* policy, float* value, hipStream_t s, const int32_t* rowlist,
                          const int32_t* rowcount, int list_off, unsigned long long* span, int max_wgs) {
    dispatch<kPacked>(N, feat, fw, H, RowMap{rowlist, rowcount, list_off, rows, span}, policy, value, s, max_wgs);
}

void launch_resnet_f32(const NetView& N, const float* feat, int rows, float* policy, float* value,
                       hipStream_t s) {
    dispatch<kF32>(N, feat, 0, 0, RowMap{nullptr, nullptr, 0, rows, nullptr}, policy, value, s);
}

int resnet_read_stamps(unsigned long long* out, long long n) {
#ifdef OAMD_STAMPS
    if (n > (long long)kMaxStampWgs * kStampStride) n = (long long)kMaxStampWgs * kStampStride;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_oamd_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? 0
               : -1;
#else
    (void)out;
    (void)n;
    return -2;
#endif
}

}  // namespace oamd
