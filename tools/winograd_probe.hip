// Winograd F(2x2, 3x3) probe for the C=128 tower — a
// MEASUREMENT, not product code: nothing in othello_mcts loads it.
//
// The question it answers: can a Winograd tower, fused in LDS like
// k_resnet_w8 (csrc/resnet.hip), beat the direct tower by >= 15 %? The probe
// runs `layers` 128 -> 128 3x3 convolutions (bias, ReLU, a residual every
// second layer, as neural_net.py:32-65's blocks) over a batch of 8x8 boards,
// activations resident in LDS for the whole tower, and is timed against the
// direct kernel's tower (tools/winograd_probe.py). It is optimistic by
// construction: no first conv, no heads, weights from L2 straight into a
// per-wave register queue (no LDS ring, no stage barriers).
//
// Geometry (the one that fits; DESIGN.md §10 has the budget):
//   * 2 boards per 512-thread workgroup (8 waves, 2 per SIMD). A board's 16
//     output tiles of 2x2 are one MFMA column block, so wave w (16 output
//     channels) keeps 2 boards x 16 transform points x 4 = 128 accumulator
//     VGPRs — 4 boards would need 256, the whole register file of a wave at
//     two waves per SIMD;
//   * LDS: spatial activations [board][64 pos][128 ch] (272-byte rows, 34 KB)
//     and the transformed inputs of one 32-channel block
//     V[board][xi][tile][32 ch] (80-byte rows, conflict-free b128 reads, 40 KB);
//   * per 32-channel block cb: barrier, V = B^T d B for 2 boards x 16 tiles x
//     32 channels (one lane per (board, tile, channel pair): 16 loads, 64
//     fp32 adds, 16 stores), barrier, then per transform point xi one
//     v_mfma_f32_16x16x32_bf16 per board (A = U[xi] fragment of the wave's 16
//     channels, B = V[board][xi]);
//   * epilogue in registers: a lane holds, for its tile and 4 output
//     channels, all 16 points, so Y = A^T M A is in-lane (24 adds per
//     channel), + bias (+ the block's skip, carried in registers), ReLU,
//     ds_write_b64 of 4 channels per output position.
// U = G g G^T (bf16) is packed on the host in fragment order:
// [layer][cb][xi][out-block][lane][8].
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;
typedef __attribute__((ext_vector_type(2))) short i16x2_t;

namespace {
constexpr int kC = 128;
constexpr int kNB = 2;          // boards per workgroup
constexpr int kSRow = 136;      // bf16 per spatial row: 128 + 8 pad (272 B)
constexpr int kVRow = 40;       // bf16 per V row: 32 + 8 pad (80 B)
#ifndef WP_Q
#define WP_Q 4                  // weight fragment queue depth (fragments ahead; 8 spills)
#endif
constexpr int kQ = WP_Q;

__device__ __forceinline__ float lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}
__device__ __forceinline__ uint32_t pack2_relu(float a, float b) {
    const i16x2_t s = __builtin_bit_cast(i16x2_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(s, (i16x2_t){0, 0}));
}
__device__ __forceinline__ f32x4_t mfma(u32x4_t a, u32x4_t b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}
__device__ __forceinline__ void barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}
}  // namespace

// x, out: [boards][64][128] bf16 (channel last); U: packed fragments, layers x
// 64 x 8 of 1 KB + kQ zero fragments of pad; bias: [layers][128] fp32
extern "C" __global__ __launch_bounds__(512) void k_wino_probe(const uint16_t* __restrict__ x,
                                                              const u32x4_t* __restrict__ U,
                                                              const float* __restrict__ bias,
                                                              uint16_t* __restrict__ out, int boards, int layers) {
    __shared__ __attribute__((aligned(16))) uint16_t S[kNB * 64 * kSRow];
    __shared__ __attribute__((aligned(16))) uint16_t V[kNB * 16 * 16 * kVRow];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int b0 = blockIdx.x * kNB;
    for (int i = tid; i < kNB * 64 * 16; i += 512) {
        const int b = i >> 10, p = (i >> 4) & 63, c8 = i & 15;
        u32x4_t v = {0, 0, 0, 0};
        if (b0 + b < boards) v = *reinterpret_cast<const u32x4_t*>(x + ((size_t)(b0 + b) * 64 + p) * kC + c8 * 8);
        *reinterpret_cast<u32x4_t*>(S + (b * 64 + p) * kSRow + c8 * 8) = v;
    }
    // MFMA roles: 16 output channels per wave, column = tile, k-group kg
    const int ob = wave, tile = lane & 15, kg = lane >> 4;
    const int ty = tile >> 2, tx = tile & 3;
    // transform roles: (board, tile, channel pair)
    const int tb = tid >> 8, ttile = (tid >> 4) & 15, cp = tid & 15;
    const int tty = ttile >> 2, ttx = ttile & 3;
    // weight stream: fragment f (= (layer * 4 + cb) * 16 + xi) of out-block ob
    const u32x4_t* uw = U + (size_t)ob * 64 + lane;
    u32x4_t q[kQ];
#pragma unroll
    for (int i = 0; i < kQ; ++i) q[i] = uw[(size_t)i * 512];
    size_t f = 0;
    uint32_t skip[kNB][8];
    for (int layer = 0; layer < layers; ++layer) {
        f32x4_t acc[kNB][16];
#pragma unroll
        for (int b = 0; b < kNB; ++b)
#pragma unroll
            for (int xi = 0; xi < 16; ++xi) acc[b][xi] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        for (int cb = 0; cb < 4; ++cb) {
            barrier();  // V is free, S holds the layer input
#ifndef WP_SKIP_TRANSFORM  // attribution builds: MFMAs on stale V
            {
                // d: 4 x 4 inputs of the tile (2 channels packed), zero outside the board
                float d0[4][4], d1[4][4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = 2 * tty - 1 + i, c = 2 * ttx - 1 + j;
                        uint32_t u = 0;
                        if (r >= 0 && r < 8 && c >= 0 && c < 8)
                            u = *reinterpret_cast<const uint32_t*>(S + (tb * 64 + r * 8 + c) * kSRow + cb * 32 + 2 * cp);
                        d0[i][j] = lo(u);
                        d1[i][j] = hi(u);
                    }
                float t0[4][4], t1[4][4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {  // B^T d: rows
                    t0[0][j] = d0[0][j] - d0[2][j];
                    t0[1][j] = d0[1][j] + d0[2][j];
                    t0[2][j] = d0[2][j] - d0[1][j];
                    t0[3][j] = d0[1][j] - d0[3][j];
                    t1[0][j] = d1[0][j] - d1[2][j];
                    t1[1][j] = d1[1][j] + d1[2][j];
                    t1[2][j] = d1[2][j] - d1[1][j];
                    t1[3][j] = d1[1][j] - d1[3][j];
                }
                uint16_t* vb = V + ((tb * 16) * 16 + ttile) * kVRow + 2 * cp;
#pragma unroll
                for (int i = 0; i < 4; ++i) {  // (B^T d) B: columns
                    const float a0 = t0[i][0] - t0[i][2], a1 = t0[i][1] + t0[i][2];
                    const float a2 = t0[i][2] - t0[i][1], a3 = t0[i][1] - t0[i][3];
                    const float c0 = t1[i][0] - t1[i][2], c1 = t1[i][1] + t1[i][2];
                    const float c2 = t1[i][2] - t1[i][1], c3 = t1[i][1] - t1[i][3];
                    *reinterpret_cast<uint32_t*>(vb + (4 * i + 0) * 16 * kVRow) = pack2(a0, c0);
                    *reinterpret_cast<uint32_t*>(vb + (4 * i + 1) * 16 * kVRow) = pack2(a1, c1);
                    *reinterpret_cast<uint32_t*>(vb + (4 * i + 2) * 16 * kVRow) = pack2(a2, c2);
                    *reinterpret_cast<uint32_t*>(vb + (4 * i + 3) * 16 * kVRow) = pack2(a3, c3);
                }
            }
#endif
            barrier();  // V ready
#pragma unroll
            for (int xi = 0; xi < 16; ++xi) {
                const u32x4_t a = q[xi % kQ];
                q[xi % kQ] = uw[(f + kQ) * 512];
                ++f;
#pragma unroll
                for (int b = 0; b < kNB; ++b) {
                    const u32x4_t bv = *reinterpret_cast<const u32x4_t*>(V + ((b * 16 + xi) * 16 + tile) * kVRow + kg * 8);
                    acc[b][xi] = mfma(a, bv, acc[b][xi]);
                }
            }
        }
        // epilogue: Y = A^T M A in-lane, + bias (+ skip on odd layers), ReLU, in place
#ifdef WP_SKIP_EPILOGUE  // attribution builds: one store per board keeps the MFMAs live
#pragma unroll
        for (int b = 0; b < kNB; ++b) {
            f32x4_t s = acc[b][0];
#pragma unroll
            for (int xi = 1; xi < 16; ++xi) s += acc[b][xi];
            *reinterpret_cast<u32x2_t*>(S + (b * 64 + tile) * kSRow + ob * 16 + kg * 4) =
                (u32x2_t){pack2_relu(s[0], s[1]), pack2_relu(s[2], s[3])};
        }
        continue;
#endif
        const bool second = (layer & 1) != 0;
        const float* bl = bias + (size_t)layer * kC + ob * 16 + kg * 4;
        const float bi[4] = {bl[0], bl[1], bl[2], bl[3]};
#pragma unroll
        for (int b = 0; b < kNB; ++b) {
            float y[4][4];  // [output position a*2+c][channel k]
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float m[4][4];
#pragma unroll
                for (int xi = 0; xi < 16; ++xi) m[xi >> 2][xi & 3] = acc[b][xi][k];
                float s0[4], s1[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    s0[j] = m[0][j] + m[1][j] + m[2][j];
                    s1[j] = m[1][j] - m[2][j] - m[3][j];
                }
                y[0][k] = s0[0] + s0[1] + s0[2] + bi[k];
                y[1][k] = s0[1] - s0[2] - s0[3] + bi[k];
                y[2][k] = s1[0] + s1[1] + s1[2] + bi[k];
                y[3][k] = s1[1] - s1[2] - s1[3] + bi[k];
            }
#pragma unroll
            for (int pq = 0; pq < 4; ++pq) {
                const int p = (2 * ty + (pq >> 1)) * 8 + 2 * tx + (pq & 1);
                uint16_t* sp = S + (b * 64 + p) * kSRow + ob * 16 + kg * 4;
                if (second) {  // the block's skip: its input, read by this lane before conv1 overwrote it
                    y[pq][0] += lo(skip[b][2 * pq]);
                    y[pq][1] += hi(skip[b][2 * pq]);
                    y[pq][2] += lo(skip[b][2 * pq + 1]);
                    y[pq][3] += hi(skip[b][2 * pq + 1]);
                } else {
                    const u32x2_t s = *reinterpret_cast<const u32x2_t*>(sp);
                    skip[b][2 * pq] = s.x;
                    skip[b][2 * pq + 1] = s.y;
                }
                *reinterpret_cast<u32x2_t*>(sp) = (u32x2_t){pack2_relu(y[pq][0], y[pq][1]), pack2_relu(y[pq][2], y[pq][3])};
            }
        }
    }
    barrier();
    for (int i = tid; i < kNB * 64 * 16; i += 512) {
        const int b = i >> 10, p = (i >> 4) & 63, c8 = i & 15;
        if (b0 + b < boards)
            *reinterpret_cast<u32x4_t*>(out + ((size_t)(b0 + b) * 64 + p) * kC + c8 * 8) =
                *reinterpret_cast<const u32x4_t*>(S + (b * 64 + p) * kSRow + c8 * 8);
    }
}

extern "C" int wino_probe_launch(const void* x, const void* U, const float* bias, void* out, int boards, int layers,
                                 void* stream) {
    const int wgs = (boards + kNB - 1) / kNB;
    hipLaunchKernelGGL(k_wino_probe, dim3(wgs), dim3(512), 0, (hipStream_t)stream, (const uint16_t*)x,
                       (const u32x4_t*)U, bias, (uint16_t*)out, boards, layers);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int wino_probe_queue() { return kQ; }
