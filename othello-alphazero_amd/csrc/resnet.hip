// Fused AlphaZeroNet forward (python/othello_alphazero/neural_net.py:138-172,
// eval mode) for gfx950: one launch evaluates a batch of boards end to end.
//
// Work decomposition (DESIGN.md "ResNet kernel"):
//   * a 512-thread workgroup (8 waves, 2 per SIMD) owns BOARDS = 512/C boards
//     (4 boards = 256 positions at C=128, 2 boards at C=256) and runs the whole
//     tower + both heads on them; activations never leave LDS;
//   * each 3x3 conv is an implicit GEMM  M = 64*BOARDS positions,
//     N = C output channels, K = 9 taps x C_in, on v_mfma_f32_16x16x32_{bf16,f16};
//     wave (wm, wn) owns the 64x64 output tile of board wm, columns wn*64..;
//   * weights (BatchNorm folded, packed on the host in MFMA fragment order) are
//     streamed once per workgroup per K-step (32 x C) through a 2-stage LDS
//     ring with register staging, so L2 traffic is 1x per workgroup;
//   * activations are bf16/fp16 in LDS, [position][channel] rows of 2C bytes
//     with a 16-byte-chunk XOR swizzle (chunk ^ (row & 15)) so the 16 rows an
//     MFMA A-fragment reads land in distinct LDS slots; zero padding of the
//     3x3 taps at the board edge is a predicated load;
//   * epilogue: + folded bias, (+ residual from LDS), ReLU, round to the
//     activation dtype, written back in place (conv2 overwrites the block
//     input element it just consumed as the skip);
//   * heads (1x1 convs, Linear layers, softmax(65), tanh) run in fp32 on VALU,
//     one wave per (board, head).

#include <hip/hip_runtime.h>

#include "bitboard.h"
#include "kernels.h"

namespace oamd {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

constexpr int kThreads = 512;

// Head parameter buffer layout (fp32), see pack in capi.hip.
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

// K-steps: first conv 9 (C_in padded to 32), each tower conv 9 * C/32.
__host__ __device__ inline int ksteps_first() { return 9; }
__host__ __device__ inline int ksteps_tower(int C) { return 9 * (C / 32); }
size_t resnet_packed_weight_elems(int C, int R) {
    return (size_t)(ksteps_first() + 2 * R * ksteps_tower(C)) * 32 * C;
}

template <int DT>
__device__ __forceinline__ uint16_t to_act(float v) {
    if constexpr (DT == OAMD_BF16) {
        return __builtin_bit_cast(uint16_t, (__bf16)v);
    } else {
        return __builtin_bit_cast(uint16_t, (_Float16)v);
    }
}

template <int DT>
__device__ __forceinline__ float from_act(uint16_t u) {
    if constexpr (DT == OAMD_BF16) {
        return __uint_as_float((uint32_t)u << 16);
    } else {
        return (float)__builtin_bit_cast(_Float16, u);
    }
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

// byte offset of (row, 8-channel chunk) in an activation buffer with rows of 2C bytes
template <int C>
__device__ __forceinline__ int act_chunk_off(int row, int chunk) {
    return row * (2 * C) + ((chunk ^ (row & 15)) << 4);
}

template <int C>
__device__ __forceinline__ int act_elem_off(int row, int ch) {
    return act_chunk_off<C>(row, ch >> 3) + ((ch & 7) << 1);
}

enum InputKind { kPacked = 0, kF32 = 1 };

template <int C, int DT, int IN>
__global__ __launch_bounds__(kThreads) void k_resnet(NetView N, const void* __restrict__ feat_in,
                                                    int fw, int H, int rows,
                                                    float* __restrict__ policy,
                                                    float* __restrict__ value) {
    constexpr int BOARDS = 512 / C;
    constexpr int ROWS = BOARDS * 64;
    constexpr int WN = 8 / BOARDS;      // waves along N
    constexpr int ACT_BYTES = ROWS * C * 2;
    constexpr int STAGE_BYTES = 32 * C * 2;
    constexpr int STAGE_U4 = STAGE_BYTES / 16 / kThreads;  // uint4 per thread per stage
    static_assert(STAGE_U4 >= 1, "stage too small");

    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* act0 = smem;
    unsigned char* act1 = smem + ACT_BYTES;
    unsigned char* stage = smem + 2 * ACT_BYTES;

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    const int wm = wave / WN;  // board of this wave
    const int wn = wave % WN;
    const int row0 = blockIdx.x * BOARDS;  // first board of the tile

    // ---------------- input planes -> act1 (C_in padded to 32 channels) -------
    if (tid < ROWS) {
        const int b = tid >> 6, p = tid & 63;
        const int gr = row0 + b;
        uint16_t v[32];
        const uint16_t one = to_act<DT>(1.0f);
        if constexpr (IN == kPacked) {
            uint32_t mask = 0;  // bit c = channel c is 1
            if (gr < rows) {
                const uint64_t* fr = reinterpret_cast<const uint64_t*>(feat_in) + (size_t)gr * fw;
                const uint64_t meta = fr[0];
                if ((meta >> 16) & 1ULL) {
                    const int t = (int)((meta >> 8) & 7ULL);
                    const int src = inverse_transform(p, t);
                    mask = (uint32_t)(meta & 1ULL);
                    for (int h = 0; h < H; ++h) {
                        mask |= (uint32_t)((fr[2 + 2 * h] >> (63 - src)) & 1ULL) << (1 + 2 * h);
                        mask |= (uint32_t)((fr[3 + 2 * h] >> (63 - src)) & 1ULL) << (2 + 2 * h);
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < 32; ++c) v[c] = ((mask >> c) & 1u) ? one : (uint16_t)0;
        } else {
            const float* fr = reinterpret_cast<const float*>(feat_in) + (size_t)gr * N.cin * 64;
            const bool ok = gr < rows;
#pragma unroll
            for (int c = 0; c < 32; ++c)
                v[c] = (ok && c < N.cin) ? to_act<DT>(fr[c * 64 + p]) : (uint16_t)0;
        }
#pragma unroll
        for (int ch = 0; ch < 4; ++ch) {
            u32x4_t w;
            w.x = (uint32_t)v[8 * ch + 0] | ((uint32_t)v[8 * ch + 1] << 16);
            w.y = (uint32_t)v[8 * ch + 2] | ((uint32_t)v[8 * ch + 3] << 16);
            w.z = (uint32_t)v[8 * ch + 4] | ((uint32_t)v[8 * ch + 5] << 16);
            w.w = (uint32_t)v[8 * ch + 6] | ((uint32_t)v[8 * ch + 7] << 16);
            *reinterpret_cast<u32x4_t*>(act1 + act_chunk_off<C>(tid, ch)) = w;
        }
    }

    // ---------------- weight stream: register-staged 2-stage ring ------------
    const u32x4_t* wg = reinterpret_cast<const u32x4_t*>(N.w);
    const int total_ks = ksteps_first() + 2 * N.R * ksteps_tower(C);
    u32x4_t wreg[STAGE_U4];
#pragma unroll
    for (int u = 0; u < STAGE_U4; ++u) wreg[u] = wg[(size_t)u * kThreads + tid];
#pragma unroll
    for (int u = 0; u < STAGE_U4; ++u)
        *reinterpret_cast<u32x4_t*>(stage + ((size_t)u * kThreads + tid) * 16) = wreg[u];
    __syncthreads();

    f32x4_t acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    int ks = 0;  // global K-step counter (drives the weight ring)
    const int nlayers = 1 + 2 * N.R;
    for (int layer = 0; layer < nlayers; ++layer) {
        const bool first = layer == 0;
        const bool conv2 = !first && ((layer - 1) & 1);
        unsigned char* act_in = first ? act1 : (conv2 ? act1 : act0);
        unsigned char* act_out = first ? act0 : (conv2 ? act0 : act1);
        const int CB = first ? 1 : C / 32;

        for (int tap = 0; tap < 9; ++tap) {
            const int dy = tap / 3 - 1, dx = tap % 3 - 1;
            int a_row[4];
            bool a_ok[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int s = m * 16 + (lane & 15);
                const int yy = (s >> 3) + dy, xx = (s & 7) + dx;
                a_ok[m] = (unsigned)yy < 8u && (unsigned)xx < 8u;
                a_row[m] = wm * 64 + (a_ok[m] ? yy * 8 + xx : s);
            }
            for (int cb = 0; cb < CB; ++cb) {
                // prefetch the next K-step's weights into registers
                const bool more = ks + 1 < total_ks;
                if (more) {
#pragma unroll
                    for (int u = 0; u < STAGE_U4; ++u)
                        wreg[u] = wg[(size_t)(ks + 1) * (STAGE_BYTES / 16) + (size_t)u * kThreads + tid];
                }
                const unsigned char* st = stage + (ks & 1) * STAGE_BYTES;
                u32x4_t a[4], b[4];
                const int chunk = cb * 4 + (lane >> 4);
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const u32x4_t v =
                        *reinterpret_cast<const u32x4_t*>(act_in + act_chunk_off<C>(a_row[m], chunk));
                    a[m] = a_ok[m] ? v : u32x4_t{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (int n = 0; n < 4; ++n)
                    b[n] = *reinterpret_cast<const u32x4_t*>(st + (((wn * 4 + n) * 64) + lane) * 16);
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int n = 0; n < 4; ++n) acc[m][n] = mfma<DT>(a[m], b[n], acc[m][n]);
                if (more) {
#pragma unroll
                    for (int u = 0; u < STAGE_U4; ++u)
                        *reinterpret_cast<u32x4_t*>(stage + ((ks + 1) & 1) * STAGE_BYTES +
                                                    ((size_t)u * kThreads + tid) * 16) = wreg[u];
                }
                __syncthreads();
                ++ks;
            }
        }

        // ---------------- epilogue: bias (+ skip) + ReLU -> act_out ------------
        const float* bias = N.bias + (size_t)layer * C;
        float bcol[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) bcol[n] = bias[wn * 64 + n * 16 + (lane & 15)];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int col = wn * 64 + n * 16 + (lane & 15);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int row = wm * 64 + m * 16 + (lane >> 4) * 4 + j;
                    float v = acc[m][n][j] + bcol[n];
                    const int off = act_elem_off<C>(row, col);
                    if (conv2) v += from_act<DT>(*reinterpret_cast<const uint16_t*>(act0 + off));
                    v = fmaxf(v, 0.0f);
                    *reinterpret_cast<uint16_t*>(act_out + off) = to_act<DT>(v);
                }
                acc[m][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            }
        }
        __syncthreads();
    }

    // ---------------- heads (fp32, VALU), final activations in act0 ---------
    const HeadLayout HL(C, N.hidden);
    const float* hp = N.head;
    const int b = wave % BOARDS;
    const int gr = row0 + b;
    if (wave >= 2 * BOARDS || gr >= rows) return;
    const int row = b * 64 + lane;
    if (wave < BOARDS) {
        // policy head: 1x1 conv (C->2) + BN + ReLU, flatten c*64+s, Linear(128->65), softmax
        float h0 = hp[HL.pcb + 0], h1 = hp[HL.pcb + 1];
        for (int c8 = 0; c8 < C / 8; ++c8) {
            const u32x4_t v = *reinterpret_cast<const u32x4_t*>(act0 + act_chunk_off<C>(row, c8));
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float x = from_act<DT>((uint16_t)(w4[e >> 1] >> ((e & 1) * 16)));
                h0 += x * hp[HL.pcw + c8 * 8 + e];
                h1 += x * hp[HL.pcw + C + c8 * 8 + e];
            }
        }
        h0 = fmaxf(h0, 0.0f);
        h1 = fmaxf(h1, 0.0f);
        const float* plw = hp + HL.plw;
        float o = hp[HL.plb + lane];
        float o64 = hp[HL.plb + 64];
        for (int s = 0; s < 64; ++s) {
            const float x0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h0), s));
            const float x1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h1), s));
            o += plw[s * 65 + lane] * x0 + plw[(64 + s) * 65 + lane] * x1;
            o64 += plw[s * 65 + 64] * x0 + plw[(64 + s) * 65 + 64] * x1;
        }
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
        // value head: 1x1 conv (C->1) + BN + ReLU, Linear(64->hidden), ReLU, Linear(hidden->1), tanh
        float v = hp[HL.vcb];
        for (int c8 = 0; c8 < C / 8; ++c8) {
            const u32x4_t q = *reinterpret_cast<const u32x4_t*>(act0 + act_chunk_off<C>(row, c8));
            const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float x = from_act<DT>((uint16_t)(w4[e >> 1] >> ((e & 1) * 16)));
                v += x * hp[HL.vcw + c8 * 8 + e];
            }
        }
        v = fmaxf(v, 0.0f);
        const float* v1w = hp + HL.v1w;
        float part = 0.0f;
        for (int j0 = 0; j0 < N.hidden; j0 += 64) {
            const bool ok = j0 + lane < N.hidden;
            const int j = ok ? j0 + lane : N.hidden - 1;
            float hj = hp[HL.v1b + j];
            for (int s = 0; s < 64; ++s) {
                const float xs = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), s));
                hj += v1w[s * N.hidden + j] * xs;
            }
            hj = fmaxf(hj, 0.0f);
            part += ok ? hj * hp[HL.v2w + j] : 0.0f;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
        if (lane == 0) value[gr] = tanhf(part + hp[HL.v2b]);
    }
}

template <int C>
static size_t lds_bytes() {
    return (size_t)2 * (512 / C) * 64 * C * 2 + 2 * 32 * C * 2;
}

template <int C, int DT, int IN>
static void launch_t(const NetView& N, const void* feat, int fw, int H, int rows, float* pol,
                     float* val, hipStream_t s) {
    constexpr int BOARDS = 512 / C;
    const unsigned grid = (unsigned)((rows + BOARDS - 1) / BOARDS);
    const size_t lds = lds_bytes<C>();
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_resnet<C, DT, IN>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        configured = true;
    }
    hipLaunchKernelGGL((k_resnet<C, DT, IN>), dim3(grid), dim3(kThreads), lds, s, N, feat, fw, H,
                       rows, pol, val);
}

template <int IN>
static void dispatch(const NetView& N, const void* feat, int fw, int H, int rows, float* pol,
                     float* val, hipStream_t s) {
    if (rows <= 0) return;
    if (N.C == 128) {
        if (N.dtype == OAMD_FP16) launch_t<128, OAMD_FP16, IN>(N, feat, fw, H, rows, pol, val, s);
        else launch_t<128, OAMD_BF16, IN>(N, feat, fw, H, rows, pol, val, s);
    } else {
        if (N.dtype == OAMD_FP16) launch_t<256, OAMD_FP16, IN>(N, feat, fw, H, rows, pol, val, s);
        else launch_t<256, OAMD_BF16, IN>(N, feat, fw, H, rows, pol, val, s);
    }
}

void launch_resnet_packed(const NetView& N, const uint64_t* feat, int fw, int H, int rows,
                          float* policy, float* value, hipStream_t s) {
    dispatch<kPacked>(N, feat, fw, H, rows, policy, value, s);
}

void launch_resnet_f32(const NetView& N, const float* feat, int rows, float* policy, float* value,
                       hipStream_t s) {
    dispatch<kF32>(N, feat, 0, 0, rows, policy, value, s);
}

}  // namespace oamd
