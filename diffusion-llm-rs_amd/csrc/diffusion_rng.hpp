// diffusion_rng.hpp -- the seeded N(0,1) stream of the diffusion steps (device side).
//
// Element e of stream (seed, offset = 0): Philox4x32-10 keyed by (seed lo, seed hi) on the counter
// (e / 4 as 64 bits, 0, 0) gives r0..r3; Box-Muller on (r0, r1) -> z0, z1 and (r2, r3) -> z2, z3;
// element e is z_{e % 4}.  Every floating-point step is a single correctly rounded + - * / or
// sqrt (this file is compiled with -ffp-contract=off): ln by exponent split + atanh series,
// sin/cos by quadrant + Taylor polynomial on [0, pi/2).  That makes the stream reproducible bit
// for bit by any IEEE binary32 host (the CPU oracle checks exactly that).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dllm {
namespace rng {

__device__ __forceinline__ void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c[0], hi0 = __umulhi(0xD2511F53u, c[0]);
        const uint32_t lo1 = 0xCD9E8D57u * c[2], hi1 = __umulhi(0xCD9E8D57u, c[2]);
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// ln(u) for u in (0, 1].
__device__ __forceinline__ float ln01(float u) {
    const uint32_t bits = __float_as_uint(u);
    int e = static_cast<int>((bits >> 23) & 0xffu) - 127;
    float m = __uint_as_float((bits & 0x007fffffu) | 0x3f800000u);   // [1, 2)
    if (m > 0x1.6a09e6p+0f) {
        m = m * 0.5f;
        e += 1;
    }
    const float s = (m - 1.0f) / (m + 1.0f);
    const float s2 = s * s;
    float p = 0x1.3b13b2p-4f;          // 1/13
    p = 0x1.745d18p-4f + s2 * p;       // 1/11
    p = 0x1.c71c72p-4f + s2 * p;       // 1/9
    p = 0x1.24924ap-3f + s2 * p;       // 1/7
    p = 0x1.99999ap-3f + s2 * p;       // 1/5
    p = 0x1.555556p-2f + s2 * p;       // 1/3
    p = 1.0f + s2 * p;
    return static_cast<float>(e) * 0x1.62e430p-1f + (2.0f * s) * p;
}

__device__ __forceinline__ void box_muller(uint32_t ra, uint32_t rb, float &z0, float &z1) {
    const float u1 = static_cast<float>((ra >> 8) + 1u) * 0x1p-24f;
    const float u2 = static_cast<float>(rb >> 8) * 0x1p-24f;
    const float rad = __builtin_sqrtf(-2.0f * ln01(u1));
    const float v = u2 * 4.0f;
    const int q = static_cast<int>(v);
    const float phi = (v - static_cast<float>(q)) * 0x1.921fb6p+0f;
    const float x2 = phi * phi;
    float sp = 1.0f - x2 * 0x1.a41a42p-8f;   // 1/156
    sp = 1.0f - x2 * 0x1.29e412p-7f * sp;    // 1/110
    sp = 1.0f - x2 * 0x1.c71c72p-7f * sp;    // 1/72
    sp = 1.0f - x2 * 0x1.861862p-6f * sp;    // 1/42
    sp = 1.0f - x2 * 0x1.99999ap-5f * sp;    // 1/20
    sp = 1.0f - x2 * 0x1.555556p-3f * sp;    // 1/6
    const float sn = phi * sp;
    float cp = 1.0f - x2 * 0x1.f07c20p-8f;   // 1/132
    cp = 1.0f - x2 * 0x1.6c16c2p-7f * cp;    // 1/90
    cp = 1.0f - x2 * 0x1.24924ap-6f * cp;    // 1/56
    cp = 1.0f - x2 * 0x1.111112p-5f * cp;    // 1/30
    cp = 1.0f - x2 * 0x1.555556p-4f * cp;    // 1/12
    cp = 1.0f - x2 * 0.5f * cp;              // 1/2
    const float c = q == 0 ? cp : q == 1 ? -sn : q == 2 ? -cp : sn;
    const float s = q == 0 ? sn : q == 1 ? cp : q == 2 ? -sn : -cp;
    z0 = rad * c;
    z1 = rad * s;
}

// The four normals of Philox block `blk` (stream elements 4 blk .. 4 blk + 3).
__device__ __forceinline__ void normal4(uint64_t seed, uint64_t blk, float (&z)[4]) {
    uint32_t c[4] = {static_cast<uint32_t>(blk), static_cast<uint32_t>(blk >> 32), 0u, 0u};
    philox4x32_10(c, static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
    box_muller(c[0], c[1], z[0], z[1]);
    box_muller(c[2], c[3], z[2], z[3]);
}

}  // namespace rng
}  // namespace dllm
