// Measurement probe (not product code): the bf16 / fp16 MFMA rate this MI355X
// holds under a sustained load, to read k_resnet_w8's roofline fraction against.
//
// k_mfma_loop: 512-thread workgroups (8 waves, 2 per SIMD, like k_resnet_w8),
// each wave runs ITERS K-steps of the ResNet's tile shape — 2 weight (A) x 8
// position (B) fragments, 16 independent v_mfma_f32_16x16x32_bf16
// accumulators — on operands held in registers (MODE 0) or with the 8 B
// fragments re-read from LDS every K-step by ds_read_b128 (MODE 1, the
// ResNet's fragment traffic without its barriers, DMA and epilogues), in bf16
// and (f16_*) fp16. The operands come from a buffer of random values in
// [-1, 1) (or zeros) so the data toggles the way real activations do. Prints
// one JSON line per configuration: TFLOP/s over >= 2 s of back-to-back
// launches after a warm-up.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/_build/mfma_ceiling tools/mfma_ceiling.hip
//   tools/_build/mfma_ceiling [regs_random,f16_regs_random,...]
// (bench.py runs the bf16 / fp16 register probes after its timed regions)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr int kIters = 2048;  // K-steps per wave per launch

template <int F16>
__device__ __forceinline__ f32x4_t mfma(u32x4_t a, u32x4_t b, f32x4_t c) {
    if constexpr (F16)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0, 0,
                                                       0);
}

template <int MODE, int F16 = 0>
__global__ __launch_bounds__(512) void k_mfma_loop(const u32x4_t* __restrict__ src, float* __restrict__ out) {
    __shared__ u32x4_t lds[8 * 512];  // 64 KiB: 8 B fragments per wave slot
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u32x4_t* s = src + ((size_t)blockIdx.x * 512 + tid) * 10 % ((1 << 20) - 16);  // + 10 fragments stay inside
    u32x4_t a[2], b[8];
    for (int i = 0; i < 2; ++i) a[i] = s[i];
    for (int i = 0; i < 8; ++i) b[i] = s[2 + i];
    if constexpr (MODE == 1) {
        for (int i = 0; i < 8; ++i) lds[i * 512 + tid] = b[i];
        __syncthreads();
    }
    f32x4_t acc[2][8];
    for (int n = 0; n < 2; ++n)
        for (int m = 0; m < 8; ++m) acc[n][m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < kIters; ++it) {
        if constexpr (MODE == 1) {
            // this K-step's B fragments from LDS (a neighbour's slot, so the
            // reads are not loop-invariant)
            const int o = ((it & 7) * 64 + lane + wave * 64) & 511;
#pragma unroll
            for (int i = 0; i < 8; ++i) b[i] = lds[i * 512 + o];
        }
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int m = 0; m < 8; ++m)
                acc[n][m] = mfma<F16>(a[n], b[m], acc[n][m]);
        if constexpr (MODE == 0) {
            // keep the operands from being treated as loop-invariant constants
            asm volatile("" : "+v"(a[0]), "+v"(a[1]));
        }
    }
    float t = 0.f;
    for (int n = 0; n < 2; ++n)
        for (int m = 0; m < 8; ++m) t += acc[n][m][0] + acc[n][m][1] + acc[n][m][2] + acc[n][m][3];
    out[(size_t)blockIdx.x * 512 + tid] = t;
}

static const char* g_only = nullptr;  // argv[1]: comma-separated probe names to run (default: all)
static bool wanted(const char* name) {
    if (!g_only) return true;
    const size_t n = strlen(name);
    for (const char* p = g_only; (p = strstr(p, name)) != nullptr; p += n)
        if ((p == g_only || p[-1] == ',') && (p[n] == ',' || p[n] == 0)) return true;
    return false;
}

template <int MODE, int F16 = 0>
static void run(const char* name, const u32x4_t* d_src, float* d_out, int grid) {
    if (!wanted(name)) return;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_mfma_loop<MODE, F16>), dim3(grid), dim3(512), 0, 0, d_src, d_out);
    CHECK(hipDeviceSynchronize());
    // >= 2 s of back-to-back launches before the timed window (the clock settles)
    auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 2.0) {
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_mfma_loop<MODE, F16>), dim3(grid), dim3(512), 0, 0, d_src, d_out);
        CHECK(hipDeviceSynchronize());
    }
    const int reps = 50;
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_mfma_loop<MODE, F16>), dim3(grid), dim3(512), 0, 0, d_src, d_out);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double flops = (double)reps * grid * 8 /*waves*/ * kIters * 16 /*MFMAs*/ * 16384.0;
    printf("{\"probe\": \"%s\", \"grid\": %d, \"ms_per_launch\": %.4f, \"TFLOP_s\": %.1f, \"frac_of_2.5PF\": %.4f}\n", name,
           grid, ms / reps, flops / (ms * 1e-3) / 1e12, flops / (ms * 1e-3) / 2.5e15);
    fflush(stdout);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    if (argc > 1) g_only = argv[1];
    const size_t n = (size_t)1 << 20;  // 16 MiB of operands
    std::vector<u32x4_t> h(n);
    // random bf16 in [-1, 1) (the magnitude of folded conv weights / ReLU
    // activations), from a fixed LCG
    unsigned long long x = 0x9E3779B97F4A7C15ULL;
    for (size_t i = 0; i < n; ++i) {
        unsigned int w[4];
        for (int k = 0; k < 4; ++k) {
            unsigned short hv[2];
            for (int j = 0; j < 2; ++j) {
                x = x * 6364136223846793005ULL + 1442695040888963407ULL;
                float f = (float)((x >> 40) & 0xFFFFFF) / 8388608.0f - 1.0f;
                unsigned int u;
                memcpy(&u, &f, 4);
                hv[j] = (unsigned short)(u >> 16);
            }
            w[k] = hv[0] | ((unsigned int)hv[1] << 16);
        }
        h[i] = u32x4_t{w[0], w[1], w[2], w[3]};
    }
    // the same values as fp16 (configs[4]'s dtype)
    std::vector<u32x4_t> hf(n);
    x = 0x9E3779B97F4A7C15ULL;
    for (size_t i = 0; i < n; ++i) {
        unsigned int w[4];
        for (int k = 0; k < 4; ++k) {
            unsigned short hv[2];
            for (int j = 0; j < 2; ++j) {
                x = x * 6364136223846793005ULL + 1442695040888963407ULL;
                const _Float16 f = (_Float16)((float)((x >> 40) & 0xFFFFFF) / 8388608.0f - 1.0f);
                memcpy(&hv[j], &f, 2);
            }
            w[k] = hv[0] | ((unsigned int)hv[1] << 16);
        }
        hf[i] = u32x4_t{w[0], w[1], w[2], w[3]};
    }
    u32x4_t *d_rand, *d_zero, *d_randf;
    float* d_out;
    const int grid = 1024;  // 4 workgroups per CU, like a 4096-row ResNet launch
    CHECK(hipMalloc(&d_rand, n * sizeof(u32x4_t)));
    CHECK(hipMalloc(&d_zero, n * sizeof(u32x4_t)));
    CHECK(hipMalloc(&d_randf, n * sizeof(u32x4_t)));
    CHECK(hipMemcpy(d_randf, hf.data(), n * sizeof(u32x4_t), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&d_out, (size_t)grid * 512 * sizeof(float)));
    CHECK(hipMemcpy(d_rand, h.data(), n * sizeof(u32x4_t), hipMemcpyHostToDevice));
    CHECK(hipMemset(d_zero, 0, n * sizeof(u32x4_t)));
    run<0>("regs_random", d_rand, d_out, grid);
    run<1>("lds_b_random", d_rand, d_out, grid);
    run<0>("regs_zero", d_zero, d_out, grid);
    run<1>("lds_b_zero", d_zero, d_out, grid);
    run<0, 1>("f16_regs_random", d_randf, d_out, grid);
    run<1, 1>("f16_lds_b_random", d_randf, d_out, grid);
    CHECK(hipFree(d_rand));
    CHECK(hipFree(d_zero));
    CHECK(hipFree(d_randf));
    CHECK(hipFree(d_out));
    return 0;
}
