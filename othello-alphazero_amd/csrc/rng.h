// Counter-based random streams for the search (DESIGN.md "Random streams").
//
// The reference draws its per-leaf symmetry (search_thread.cpp:92) and its
// root Dirichlet noise (search_thread.cpp:230-236) from std::mt19937 seeded by
// std::random_device — unreproducible by design. This engine replaces that
// with a random-access stream so every wave can draw independently:
//   stream_key(game_key, event, sub) -> uniform(stream_key, k), k = 0,1,...
// One "event" per random decision of a game (a leaf's transform, a root
// selection's noise vector, a move choice); "sub" separates the children of
// one noise vector. The Gamma sampler and the log/exp/cos^2 it uses are
// written in plain IEEE float operations (no libm beyond the exact floorf, no
// FMA contraction: this file must be compiled with -ffp-contract=off) so that
// host and device produce the same bits. The test oracle (oracle/omcts_oracle.c) restates the same spec.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bitboard.h"

namespace oamd {

constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ULL;
constexpr uint64_t kEventMul = 0xD1B54A32D192ED03ULL;

OAMD_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

OAMD_HD uint64_t stream_key(uint64_t game_key, uint64_t event, uint32_t sub) {
    return mix64(mix64(game_key ^ (event * kEventMul)) + (uint64_t)(sub + 1) * kGolden);
}

// Exact float in (0,1): (2m+1) * 2^-24 with m the top 23 bits.
OAMD_HD float uniform(uint64_t key, uint32_t k) {
    const uint64_t x = mix64(key + (uint64_t)(k + 1) * kGolden);
    const uint32_t m = (uint32_t)(x >> 41);
    return (float)(2u * m + 1u) * 5.9604644775390625e-08f;
}

// Symmetry draw for a leaf: top three bits of the event's stream key.
OAMD_HD int draw_transform(uint64_t game_key, uint64_t event) {
    return (int)(mix64(stream_key(game_key, event, 0)) >> 61);
}

OAMD_HD float bits_to_float(uint32_t u) { return __builtin_bit_cast(float, u); }
OAMD_HD uint32_t float_to_bits(float f) { return __builtin_bit_cast(uint32_t, f); }

OAMD_HD float plogf(float x) {
    const uint32_t b = float_to_bits(x);
    int e = (int)((b >> 23) & 0xffu) - 127;
    float m = bits_to_float((b & 0x7fffffu) | 0x3f800000u);
    if (m > 1.41421356f) {
        m = m * 0.5f;
        e = e + 1;
    }
    const float s = (m - 1.0f) / (m + 1.0f);
    const float s2 = s * s;
    float p = 0.0909090936f;
    p = 0.111111112f + s2 * p;
    p = 0.142857149f + s2 * p;
    p = 0.200000003f + s2 * p;
    p = 0.333333343f + s2 * p;
    const float t = s2 * p;
    const float logm = 2.0f * s + (2.0f * s) * t;
    const float fe = (float)e;
    return fe * 0.693145752f + (fe * 1.42860677e-06f + logm);
}

OAMD_HD float pexpf(float x) {
    if (x < -87.0f) return 0.0f;
    if (x > 88.0f) return bits_to_float(0x7f800000u);
    const float kf = floorf(x * 1.44269502f + 0.5f);
    const int k = (int)kf;
    const float r = (x - kf * 0.693145752f) - kf * 1.42860677e-06f;
    float p = 0.00138888892f;
    p = 0.00833333377f + r * p;
    p = 0.0416666679f + r * p;
    p = 0.166666672f + r * p;
    p = 0.5f + r * p;
    p = 1.0f + r * p;
    p = 1.0f + r * p;
    if (k < -126) return 0.0f;
    return p * bits_to_float((uint32_t)(k + 127) << 23);
}

// cos^2(2 pi v) for v in (0, 1): folded to an argument x in [0, pi/4] of a
// sine or cosine polynomial (plain float operations, as plogf)
OAMD_HD float cos2pi_sq(float v) {
    float t = 2.0f * v;
    t = t - floorf(t);              // cos^2(pi t), period 1
    if (t > 0.5f) t = 1.0f - t;     // symmetric about 1/2: t in [0, 1/2]
    float c;
    if (t < 0.25f) {                // cos(pi t), pi t in [0, pi/4)
        const float x = 3.14159274f * t;
        const float x2 = x * x;
        c = 1.0f + x2 * (-0.5f + x2 * (0.0416666679f + x2 * (-0.00138888892f + x2 * 2.48015876e-05f)));
    } else {                        // sin(pi (1/2 - t)), pi (1/2 - t) in [0, pi/4]
        const float x = 3.14159274f * (0.5f - t);
        const float x2 = x * x;
        c = x * (1.0f + x2 * (-0.166666672f + x2 * (0.00833333377f + x2 * -0.000198412701f)));
    }
    return c * c;
}

// Gamma(alpha, 1). alpha = 1/2 (the default Dirichlet alpha): Z^2 / 2 for a
// standard normal Z in Box-Muller form, -ln(U) cos^2(2 pi V), with no
// rejection loop (a wave's lanes all finish together). Otherwise
// Marsaglia–Tsang with the alpha < 1 boost; bounded loops.
OAMD_HD float gamma_draw(uint64_t key, float alpha) {
    if (!(alpha > 0.0f)) return 0.0f;
    if (alpha == 0.5f) return -plogf(uniform(key, 0)) * cos2pi_sq(uniform(key, 1));
    uint32_t k = 0;
    const bool boost = alpha < 1.0f;
    const float a = boost ? alpha + 1.0f : alpha;
    const float d = a - 0.333333343f;
    const float c = 1.0f / sqrtf(9.0f * d);
    float g = d;
    for (int it = 0; it < 16; ++it) {
        float u = 0.0f, s = 0.5f;
        bool ok = false;
        for (int j = 0; j < 16; ++j) {
            const float uu = 2.0f * uniform(key, k) - 1.0f;
            const float vv = 2.0f * uniform(key, k + 1) - 1.0f;
            k += 2;
            const float ss = uu * uu + vv * vv;
            if (ss < 1.0f && ss > 0.0f) {
                u = uu;
                s = ss;
                ok = true;
                break;
            }
        }
        if (!ok) u = 0.5f;
        const float x = u * sqrtf((-2.0f * plogf(s)) / s);
        float v = 1.0f + c * x;
        if (v <= 0.0f) continue;
        v = (v * v) * v;
        const float uu = uniform(key, k);
        k += 1;
        const float x2 = x * x;
        const float x4 = x2 * x2;
        if (uu < 1.0f - 0.0331f * x4) {
            g = d * v;
            break;
        }
        if (plogf(uu) < 0.5f * x2 + d * ((1.0f - v) + plogf(v))) {
            g = d * v;
            break;
        }
    }
    if (boost) {
        const float ub = uniform(key, 63);
        g = g * pexpf(plogf(ub) / alpha);
    }
    return g;
}

}  // namespace oamd
