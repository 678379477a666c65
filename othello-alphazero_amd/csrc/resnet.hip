// Fused AlphaZeroNet forward (python/othello_alphazero/neural_net.py:138-172,
// eval mode) for gfx950: one launch evaluates a batch of boards end to end.
//
// Work decomposition (DESIGN.md "ResNet kernel"):
//   * a 512-thread workgroup (8 waves, 2 per SIMD) owns BOARDS = 512/C boards
//     (4 boards = 256 positions at C=128, 2 boards at C=256) and runs the whole
//     tower + both heads on them; activations never leave LDS;
//   * each 3x3 conv is an implicit GEMM  out[ch][pos] = W[ch][K] x X[K][pos],
//     K = 9 taps x C_in, on v_mfma_f32_16x16x32_{bf16,f16} with the WEIGHTS as
//     the A operand: an accumulator lane then holds 4 consecutive output
//     channels of one position, so the epilogue writes 8 contiguous bytes;
//     wave (wm, wn) owns 64 channels (wn) x 64 positions (board wm);
//   * weights (BatchNorm folded, packed on the host in MFMA fragment order) are
//     streamed once per workgroup through a 3-slot LDS ring by LDS-DMA
//     (global_load_lds_dwordx4), one slot = one tap x 64 input channels; the
//     slot for stage g+2 is issued while stage g computes, and the single
//     barrier per stage sits between the two K=32 halves of the stage so the
//     fragment reads of the next half always overlap MFMAs;
//   * ONE activation buffer per workgroup, updated in place: [position][channel]
//     rows of 2C bytes, 16-byte chunks XOR-swizzled by (row & 15) so the 16
//     positions of an MFMA fragment hit distinct LDS slots; the residual skip
//     is held in registers from conv1's epilogue to conv2's;
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
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int kThreads = 512;
constexpr int kRing = 3;  // weight ring slots
// LDS byte offset past any workgroup allocation (max 160 KiB): ds_read returns 0
constexpr int kLdsZeroOff = 0x3FFF0;

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

// A stage = one tap x 64 input channels = 2 K-steps of 32. The first conv's
// input is zero-padded to 64 channels (9 stages), tower convs have 9 * C/64.
__host__ __device__ inline int stages_first() { return 9; }
__host__ __device__ inline int stages_tower(int C) { return 9 * (C / 64); }
size_t resnet_packed_weight_elems(int C, int R) {
    return (size_t)(stages_first() + 2 * R * stages_tower(C)) * 64 * C;
}
int resnet_first_cin_pad() { return 64; }

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

// byte offset of (row, 8-channel chunk) in the activation buffer (rows of 2C bytes)
template <int C>
__device__ __forceinline__ int act_chunk_off(int row, int chunk) {
    return row * (2 * C) + ((chunk ^ (row & 15)) << 4);
}

enum InputKind { kPacked = 0, kF32 = 1 };

// Fragments of one K=32 step: 4 weight tiles (A: 16 channels x 32 K) and
// 4 activation tiles (B: 32 K x 16 positions).
struct Frags {
    u32x4_t w[4];
    u32x4_t x[4];
};

template <int C>
struct Geo {
    static constexpr int BOARDS = 512 / C;
    static constexpr int ROWS = BOARDS * 64;
    static constexpr int WN = 8 / BOARDS;           // waves along output channels
    static constexpr int ACT_BYTES = ROWS * C * 2;  // 64 KB for both C
    static constexpr int STAGE_BYTES = 64 * C * 2;  // 16 KB (C=128) / 32 KB (C=256)
    static constexpr int DMA_PER_THREAD = STAGE_BYTES / 16 / kThreads;
    static constexpr int LDS = ACT_BYTES + kRing * STAGE_BYTES;
};

// ds_read the fragments of K-step `sub` (0/1) of a stage.
template <int C>
__device__ __forceinline__ void load_frags(Frags& f, const unsigned char* act, const unsigned char* slot,
                                           int sub, int cb64, const int (&xrow)[4], const bool (&xok)[4],
                                           int wn, int lane) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
        f.w[n] = *reinterpret_cast<const u32x4_t*>(slot + ((sub * (C / 16) + wn * 4 + n) * 64 + lane) * 16);
    const int chunk = cb64 * 8 + sub * 4 + (lane >> 4);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        // Off-board taps (the 3x3 zero padding) read beyond the workgroup's LDS
        // allocation, which returns zeros: no data-dependent select, so the
        // compiler never has to wait for these reads before the next MFMAs.
        const int off = xok[m] ? act_chunk_off<C>(xrow[m], chunk) : kLdsZeroOff;
        f.x[m] = *reinterpret_cast<const u32x4_t*>(act + off);
    }
}

template <int DT>
__device__ __forceinline__ void mfma_frags(f32x4_t (&acc)[4][4], const Frags& f) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[n][m] = mfma<DT>(f.w[n], f.x[m], acc[n][m]);
}

// positions (rows of the activation buffer) feeding tap (dy, dx) for the 4
// position tiles of this lane; out-of-board taps read a valid row and zero it
__device__ __forceinline__ void tap_rows(int tap, int wm, int lane, int (&xrow)[4], bool (&xok)[4]) {
    const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int s = m * 16 + (lane & 15);
        const int yy = (s >> 3) + dy, xx = (s & 7) + dx;
        xok[m] = (unsigned)yy < 8u && (unsigned)xx < 8u;
        xrow[m] = wm * 64 + (xok[m] ? yy * 8 + xx : s);
    }
}

template <int C>
__device__ __forceinline__ void issue_stage_dma(const unsigned char* wsrc, unsigned char* ring, int g,
                                                int total, int tid) {
    using G = Geo<C>;
    if (g >= total) return;
    const unsigned char* src = wsrc + (size_t)g * G::STAGE_BYTES;
    unsigned char* dst = ring + (g % kRing) * G::STAGE_BYTES;
    const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int i = 0; i < G::DMA_PER_THREAD; ++i) {
        const int q = i * kThreads + wave * 64;  // first 16-byte chunk of this wave's piece
        __builtin_amdgcn_global_load_lds(src + (size_t)(q + lane) * 16, (lds_void_t*)(dst + q * 16), 16, 0, 0);
    }
}

__device__ __forceinline__ void wait_dma_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// all but the youngest stage's DMAs complete
template <int C>
__device__ __forceinline__ void wait_dma_stage() {
    if constexpr (Geo<C>::DMA_PER_THREAD == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
}

template <int C, int DT>
__device__ void heads(const NetView& N, const unsigned char* act, int wave, int lane, int row0, int rows,
                      float* __restrict__ policy, float* __restrict__ value) {
    constexpr int BOARDS = Geo<C>::BOARDS;
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
            const u32x4_t v = *reinterpret_cast<const u32x4_t*>(act + act_chunk_off<C>(row, c8));
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float x = from_act<DT>((w4[e >> 1] >> ((e & 1) * 16)) & 0xffffu);
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
            const u32x4_t q = *reinterpret_cast<const u32x4_t*>(act + act_chunk_off<C>(row, c8));
            const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float x = from_act<DT>((w4[e >> 1] >> ((e & 1) * 16)) & 0xffffu);
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

template <int C, int DT, int IN>
__global__ __launch_bounds__(kThreads) void k_resnet(NetView N, const void* __restrict__ feat_in,
                                                    int fw, int H, int rows,
                                                    float* __restrict__ policy,
                                                    float* __restrict__ value) {
    using G = Geo<C>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* act = smem;
    unsigned char* ring = smem + G::ACT_BYTES;

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    const int wm = wave / G::WN;  // board of this wave
    const int wn = wave % G::WN;  // 64-channel block of this wave
    const int row0 = blockIdx.x * G::BOARDS;
    const unsigned char* wsrc = reinterpret_cast<const unsigned char*>(N.w);
    const int total = stages_first() + 2 * N.R * stages_tower(C);

    // weight stream starts right away (two stages ahead)
    issue_stage_dma<C>(wsrc, ring, 0, total, tid);
    issue_stage_dma<C>(wsrc, ring, 1, total, tid);

    // ---------------- input planes -> act channels 0..63 ---------------------
    if (tid < G::ROWS) {
        const int b = tid >> 6, p = tid & 63;
        const int gr = row0 + b;
        const uint32_t one = to_act<DT>(1.0f);
        uint32_t words[32];  // 64 channels as 16-bit pairs
        if constexpr (IN == kPacked) {
            uint32_t mask = 0;  // bit c = channel c is 1 (c < 31)
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
            for (int w = 0; w < 32; ++w) {
                const uint32_t lo = (w < 16 && ((mask >> (2 * w)) & 1u)) ? one : 0u;
                const uint32_t hi = (w < 16 && ((mask >> (2 * w + 1)) & 1u)) ? one : 0u;
                words[w] = lo | (hi << 16);
            }
        } else {
            const float* fr = reinterpret_cast<const float*>(feat_in) + (size_t)gr * N.cin * 64;
            const bool ok = gr < rows;
#pragma unroll
            for (int w = 0; w < 32; ++w) {
                const int c0 = 2 * w, c1 = 2 * w + 1;
                const uint32_t lo = (ok && c0 < N.cin) ? to_act<DT>(fr[c0 * 64 + p]) : 0u;
                const uint32_t hi = (ok && c1 < N.cin) ? to_act<DT>(fr[c1 * 64 + p]) : 0u;
                words[w] = lo | (hi << 16);
            }
        }
#pragma unroll
        for (int ch = 0; ch < 8; ++ch)
            *reinterpret_cast<u32x4_t*>(act + act_chunk_off<C>(tid, ch)) =
                u32x4_t{words[4 * ch], words[4 * ch + 1], words[4 * ch + 2], words[4 * ch + 3]};
    }

    f32x4_t acc[4][4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[n][m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    u32x2_t skip[4][4];  // residual (block input) of this lane's 64 outputs
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int m = 0; m < 4; ++m) skip[n][m] = u32x2_t{0u, 0u};

    Frags fa, fb;
    int xrow[4];
    bool xok[4];

    // first stage of layer 0: its DMA and the input planes must be visible
    wait_dma_all();
    __syncthreads();
    tap_rows(0, wm, lane, xrow, xok);
    load_frags<C>(fa, act, ring, 0, 0, xrow, xok, wn, lane);

    int g = 0;  // global stage index (weight ring position)
    const int nlayers = 1 + 2 * N.R;
    for (int layer = 0; layer < nlayers; ++layer) {
        const int S = layer == 0 ? stages_first() : stages_tower(C);
        const int per_tap = S / 9;  // 64-channel blocks per tap
        float4 bv[4];               // folded bias of this lane's 16 output channels
#pragma unroll
        for (int n = 0; n < 4; ++n)
            bv[n] = *reinterpret_cast<const float4*>(N.bias + (size_t)layer * C + wn * 64 + n * 16 +
                                                     (lane >> 4) * 4);
        // Stages 0..S-2 share one branch-free body (the waitcnt pass then counts
        // the outstanding LDS reads exactly and never drains to lgkmcnt(0)).
        int slot_i = g % kRing;
        for (int s = 0; s + 1 < S; ++s, ++g) {
            const int cb64 = s % per_tap;
            const unsigned char* slot = ring + slot_i * G::STAGE_BYTES;
            // second K-step of this stage; its reads overlap the first MFMAs
            load_frags<C>(fb, act, slot, 1, cb64, xrow, xok, wn, lane);
            mfma_frags<DT>(acc, fa);
            // stage g+1 landed (issued one stage ago); stage g-1 drained by all waves
            wait_dma_all();
            __builtin_amdgcn_s_barrier();
            issue_stage_dma<C>(wsrc, ring, g + 2, total, tid);
            slot_i = slot_i == kRing - 1 ? 0 : slot_i + 1;
            tap_rows((s + 1) / per_tap, wm, lane, xrow, xok);
            load_frags<C>(fa, act, ring + slot_i * G::STAGE_BYTES, 0, (s + 1) % per_tap, xrow, xok, wn, lane);
            mfma_frags<DT>(acc, fb);
        }
        {  // last stage of the layer
            load_frags<C>(fb, act, ring + slot_i * G::STAGE_BYTES, 1, (S - 1) % per_tap, xrow, xok, wn, lane);
            mfma_frags<DT>(acc, fa);
            mfma_frags<DT>(acc, fb);
            ++g;
        }

        // ---------------- epilogue: bias (+ skip) + ReLU, in place ------------
        // g is now the first stage of the next layer (its DMA is in flight)
        __syncthreads();  // every wave is done reading this layer's input and stage g-1
        issue_stage_dma<C>(wsrc, ring, g + 1, total, tid);  // hidden behind the epilogue
        const bool is_conv1 = layer > 0 && ((layer - 1) & 1) == 0;
        const bool is_conv2 = layer > 0 && ((layer - 1) & 1) == 1;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int ch = wn * 64 + n * 16 + (lane >> 4) * 4;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int row = wm * 64 + m * 16 + (lane & 15);
                const int off = act_chunk_off<C>(row, ch >> 3) + (ch & 7) * 2;
                u32x2_t* p = reinterpret_cast<u32x2_t*>(act + off);
                float v0 = acc[n][m][0] + bv[n].x, v1 = acc[n][m][1] + bv[n].y;
                float v2 = acc[n][m][2] + bv[n].z, v3 = acc[n][m][3] + bv[n].w;
                if (is_conv1) skip[n][m] = *p;  // block input, needed by conv2's epilogue
                if (is_conv2) {
                    const u32x2_t r = skip[n][m];
                    v0 += from_act<DT>(r.x & 0xffffu);
                    v1 += from_act<DT>(r.x >> 16);
                    v2 += from_act<DT>(r.y & 0xffffu);
                    v3 += from_act<DT>(r.y >> 16);
                }
                v0 = fmaxf(v0, 0.f);
                v1 = fmaxf(v1, 0.f);
                v2 = fmaxf(v2, 0.f);
                v3 = fmaxf(v3, 0.f);
                *p = u32x2_t{to_act<DT>(v0) | (to_act<DT>(v1) << 16), to_act<DT>(v2) | (to_act<DT>(v3) << 16)};
                acc[n][m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            }
        }
        if (layer + 1 < nlayers) {
            wait_dma_stage<C>();  // stage g has landed (stage g+1 may still fly)
            __syncthreads();      // ... and this layer's output is complete
            tap_rows(0, wm, lane, xrow, xok);
            load_frags<C>(fa, act, ring + (g % kRing) * G::STAGE_BYTES, 0, 0, xrow, xok, wn, lane);
        }
    }
    __syncthreads();
    heads<C, DT>(N, act, wave, lane, row0, rows, policy, value);
}

template <int C, int DT, int IN>
static void launch_t(const NetView& N, const void* feat, int fw, int H, int rows, float* pol,
                     float* val, hipStream_t s) {
    using G = Geo<C>;
    const unsigned grid = (unsigned)((rows + G::BOARDS - 1) / G::BOARDS);
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_resnet<C, DT, IN>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
        configured = true;
    }
    hipLaunchKernelGGL((k_resnet<C, DT, IN>), dim3(grid), dim3(kThreads), G::LDS, s, N, feat, fw, H,
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
