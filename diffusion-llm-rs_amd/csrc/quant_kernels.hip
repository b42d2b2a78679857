// quant_kernels.hip -- HBM-bound quantize / dequantize / pack kernels for gfx950 (MI355X).
//
// Every kernel is a bit-exact restatement of a reference Rust loop (cited per kernel), built with
// -ffp-contract=off so that no separately rounded Rust f32 op pair is fused into an FMA.
// Layout: elements are processed in "octets" of 8 consecutive values: 8 codes of b bits are
// exactly b bytes of the LSB-first packed bitstream (include/dllm_quant.h), so a thread owns
// whole bytes and no two threads ever touch the same output byte.
#include "common.hpp"

#include <algorithm>
#include <cstring>
#include <cstdlib>

namespace dllm {
namespace {

constexpr int kBlock = 256;

#ifndef DLLM_QMAP_OCTET
#define DLLM_QMAP_OCTET 0
#endif

// ---------------------------------------------------------------------------------------------
// Octet load / store helpers
// ---------------------------------------------------------------------------------------------
struct F8 { float v[8]; };

// Loads the 8 floats of octet `o` (cnt = number of valid elements, <= 8).  vec: x is 16-B aligned.
__device__ __forceinline__ F8 load_octet(const float *__restrict__ x, size_t o, int cnt, bool vec) {
    F8 r;
    const float *p = x + o * 8;
    if (vec && cnt == 8) {
        float4 a = *reinterpret_cast<const float4 *>(p);
        float4 b = *reinterpret_cast<const float4 *>(p + 4);
        r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
        r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) r.v[i] = (i < cnt) ? p[i] : 0.0f;
    }
    return r;
}

// Packs 8 codes (each < 2^bits) into the low 8*bits bits of a u64, LSB-first.
__device__ __forceinline__ uint64_t pack_octet(const uint32_t (&c)[8], int bits) {
    uint64_t w = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) w |= static_cast<uint64_t>(c[i]) << (i * bits);
    return w;
}

// Writes the octet's codes: packed -> `bits` bytes (fewer for a partial tail octet),
// unpacked -> one byte per code.
__device__ __forceinline__ void store_codes(uint8_t *__restrict__ out, size_t o, int cnt, const uint32_t (&c)[8],
                                            int bits, bool packed, bool vec) {
    if (packed) {
        uint64_t w = pack_octet(c, bits);
        uint8_t *p = out + o * bits;
        if (cnt == 8 && vec) {
            switch (bits) {
            case 1: *p = static_cast<uint8_t>(w); return;
            case 2: *reinterpret_cast<uint16_t *>(p) = static_cast<uint16_t>(w); return;
            case 4: *reinterpret_cast<uint32_t *>(p) = static_cast<uint32_t>(w); return;
            case 8: *reinterpret_cast<uint64_t *>(p) = w; return;
            default: break;
            }
        }
        int nbytes = (cnt * bits + 7) / 8;
        for (int i = 0; i < nbytes; ++i) p[i] = static_cast<uint8_t>(w >> (8 * i));
    } else {
        uint8_t *p = out + o * 8;
        if (cnt == 8 && vec) {
            uint64_t w = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) w |= static_cast<uint64_t>(c[i]) << (8 * i);
            *reinterpret_cast<uint64_t *>(p) = w;
        } else {
            for (int i = 0; i < cnt; ++i) p[i] = static_cast<uint8_t>(c[i]);
        }
    }
}

// Reads the octet's codes back (inverse of store_codes).
__device__ __forceinline__ void load_codes(const uint8_t *__restrict__ q, size_t o, int cnt, int bits, bool packed,
                                           bool vec, uint32_t (&c)[8]) {
    uint64_t w = 0;
    if (packed) {
        const uint8_t *p = q + o * bits;
        if (cnt == 8 && vec && (bits == 1 || bits == 2 || bits == 4 || bits == 8)) {
            switch (bits) {
            case 1: w = *p; break;
            case 2: w = *reinterpret_cast<const uint16_t *>(p); break;
            case 4: w = *reinterpret_cast<const uint32_t *>(p); break;
            default: w = *reinterpret_cast<const uint64_t *>(p); break;
            }
        } else {
            int nbytes = (cnt * bits + 7) / 8;
            for (int i = 0; i < nbytes; ++i) w |= static_cast<uint64_t>(p[i]) << (8 * i);
        }
        const uint32_t mask = (1u << bits) - 1u;
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] = static_cast<uint32_t>(w >> (i * bits)) & mask;
    } else {
        const uint8_t *p = q + o * 8;
        if (cnt == 8 && vec) {
            w = *reinterpret_cast<const uint64_t *>(p);
        } else {
            for (int i = 0; i < cnt; ++i) w |= static_cast<uint64_t>(p[i]) << (8 * i);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] = static_cast<uint32_t>(w >> (8 * i)) & 0xFFu;
    }
}

__device__ __forceinline__ void store_f8(void *__restrict__ out, int dtype, size_t o, int cnt, const float (&y)[8],
                                         bool vec) {
    if (dtype == DLLM_F32) {
        float *p = static_cast<float *>(out) + o * 8;
        if (cnt == 8 && vec) {
            *reinterpret_cast<float4 *>(p) = make_float4(y[0], y[1], y[2], y[3]);
            *reinterpret_cast<float4 *>(p + 4) = make_float4(y[4], y[5], y[6], y[7]);
        } else {
            for (int i = 0; i < cnt; ++i) p[i] = y[i];
        }
    } else {
        __half *p = static_cast<__half *>(out) + o * 8;
        if (cnt == 8 && vec) {
            union { __half h[8]; uint4 u; } pk;
#pragma unroll
            for (int i = 0; i < 8; ++i) pk.h[i] = __float2half_rn(y[i]);
            *reinterpret_cast<uint4 *>(p) = pk.u;
        } else {
            for (int i = 0; i < cnt; ++i) p[i] = __float2half_rn(y[i]);
        }
    }
}

__device__ __forceinline__ int octet_count(size_t o, size_t n) {
    size_t rem = n - o * 8;
    return rem >= 8 ? 8 : static_cast<int>(rem);
}

// ---------------------------------------------------------------------------------------------
// K1: global max/min fold (diffuse-llm-rs/src/quantization.rs:41-46).  f32::max / f32::min
// ignore NaN and are order-independent on the remaining values, so a tree reduction gives the
// Rust fold's result exactly (the sign of a zero extremum never reaches the outputs).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void block_minmax(float &mx, float &mn, float *smem /* 2*kBlock/64 */) {
    mx = wave_max(mx);
    mn = wave_min(mn);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { smem[w] = mx; smem[kBlock / 64 + w] = mn; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < kBlock / 64; ++i) { mx = fmaxf(mx, smem[i]); mn = fminf(mn, smem[kBlock / 64 + i]); }
    }
}

// Block `b` of `nb` folds its grid-stride share of x into partials[b] = {max, min}.
__device__ __forceinline__ void minmax_body(const float *__restrict__ x, size_t n, size_t head,
                                            float2 *__restrict__ partials, unsigned b, unsigned nb, float *smem) {
    float mx = -INFINITY, mn = INFINITY;
    const size_t gid = b * static_cast<size_t>(kBlock) + threadIdx.x;
    const size_t stride = static_cast<size_t>(nb) * kBlock;
    if (gid < head) { float v = x[gid]; mx = fmaxf(mx, v); mn = fminf(mn, v); }
    const size_t nv = (n - head) / 4;
    const float4 *x4 = reinterpret_cast<const float4 *>(x + head);
    size_t i = gid;
    // 4 independent float4 loads in flight per thread per trip.
    for (; i + 3 * stride < nv; i += 4 * stride) {
        float4 a = x4[i], b = x4[i + stride], c = x4[i + 2 * stride], d = x4[i + 3 * stride];
        mx = fmaxf(mx, fmaxf(fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)), fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w))));
        mx = fmaxf(mx, fmaxf(fmaxf(fmaxf(c.x, c.y), fmaxf(c.z, c.w)), fmaxf(fmaxf(d.x, d.y), fmaxf(d.z, d.w))));
        mn = fminf(mn, fminf(fminf(fminf(a.x, a.y), fminf(a.z, a.w)), fminf(fminf(b.x, b.y), fminf(b.z, b.w))));
        mn = fminf(mn, fminf(fminf(fminf(c.x, c.y), fminf(c.z, c.w)), fminf(fminf(d.x, d.y), fminf(d.z, d.w))));
    }
    for (; i < nv; i += stride) {
        float4 a = x4[i];
        mx = fmaxf(mx, fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)));
        mn = fminf(mn, fminf(fminf(a.x, a.y), fminf(a.z, a.w)));
    }
    const size_t tail0 = head + nv * 4;
    if (gid < n - tail0) { float v = x[tail0 + gid]; mx = fmaxf(mx, v); mn = fminf(mn, v); }
    block_minmax(mx, mn, smem);
    if (threadIdx.x == 0) partials[b] = make_float2(mx, mn);
}

__global__ void __launch_bounds__(kBlock) minmax_partial_kernel(const float *__restrict__ x, size_t n, size_t head,
                                                                float2 *__restrict__ partials) {
    __shared__ float smem[2 * kBlock / 64];
    minmax_body(x, n, head, partials, blockIdx.x, gridDim.x, smem);
}

// (scale, zp) from the extremes exactly as quantization.rs:49-56.
__device__ __forceinline__ void params_of(float mx, float mn, int bits, float &scale_out, float &zp_out) {
    const float q_min = 0.0f;
    const float q_max = static_cast<float>(1u << bits) - 1.0f;     // :50
    float scale = (mx - mn) / (q_max - q_min);                      // :52
    if (scale == 0.0f) scale = 1.0f;                                // :53
    const float zpf = q_min - mn / scale;                           // :55
    const uint32_t zp = rs_as_u8(roundf(rs_clamp(zpf, q_min, q_max)));  // :56
    scale_out = scale;
    zp_out = static_cast<float>(zp);                                // :67
}

__device__ __forceinline__ void write_params(float mx, float mn, int bits, float *params) {
    params_of(mx, mn, bits, params[0], params[1]);
}

// Params of width `bits` from caller-held extremes stats[2] = {min, max} (sharded quantize_tensor).
__global__ void params_from_extremes_kernel(const float *__restrict__ stats, int bits, float *__restrict__ params) {
    if (threadIdx.x == 0) write_params(stats[1], stats[0], bits, params);
}

// Reduces the partials and writes the params of width `bits` (and of `bits_b` when nonzero:
// the extremes do not depend on the width).
__global__ void __launch_bounds__(kBlock) quant_params_kernel(const float2 *__restrict__ partials, int np, int bits,
                                                              float *__restrict__ params, int bits_b = 0,
                                                              float *__restrict__ params_b = nullptr) {
    __shared__ float smem[2 * kBlock / 64];
    float mx = -INFINITY, mn = INFINITY;
    for (int i = threadIdx.x; i < np; i += kBlock) { float2 p = partials[i]; mx = fmaxf(mx, p.x); mn = fminf(mn, p.y); }
    block_minmax(mx, mn, smem);
    if (threadIdx.x == 0) {
        write_params(mx, mn, bits, params);
        if (bits_b) write_params(mx, mn, bits_b, params_b);
    }
}

// ---------------------------------------------------------------------------------------------
// K2 fast path: the quantize map of quantization.rs:59-65 for packed 1/2/4/8-bit codes, with the
// params reduction (:41-56) folded into every block's prologue and a cheaper exact division.
// ---------------------------------------------------------------------------------------------
// x / s exactly as the IEEE division (what Rust's `x / scale` computes), in three FMA-pipe ops
// instead of the ~10 of the v_div_scale/v_div_fmas/v_div_fixup sequence.  Markstein's theorem:
// with r = RN(1/s), q0 = RN(x r) is faithful, the residual e = x - q0 s is exact (one fma), and
// q1 = RN(q0 + e r) = RN(x / s) -- provided nothing over- or underflows.  The callers only use
// it for s in [2^-64, 2^64] (checked per tensor; otherwise the plain division runs):
//  * |x/s| >= 2^-25 implies |x| >= 2^-89, so q0, e (>= ~|x| 2^-24) and q1 are normal and exact as
//    the theorem needs.  A quotient below 2^-25 cannot move a code: round(q) = 0 when zp = 0, and
//    q + zp rounds to zp when zp >= 1, for the exact and the corrected quotient alike.
//  * x = +-inf or a quotient that overflows gives e = -+inf and q1 = NaN: the select keeps q0 =
//    +-inf, whose code (clamped to q_max) equals the code of the IEEE quotient.  x = NaN -> NaN.
// The identity is also checked exhaustively over all 2^24 significands of x for 96 sampled divisor
// significands (tests/test_quantize_division.py, 1.6e9 quotients) and bit-exactly on the device by
// the a1 parity tests.
__device__ __forceinline__ bool markstein_ok(float s) { return s >= 0x1p-64f && s <= 0x1p64f; }

template <bool kFast>
__device__ __forceinline__ float div_scale(float x, float s, float r) {
    if constexpr (!kFast) {
        return x / s;
    } else {
        const float q0 = x * r;
        const float e = __builtin_fmaf(-q0, s, x);
        const float q1 = __builtin_fmaf(e, r, q0);
        return q1 != q1 ? q0 : q1;
    }
}

// (round(t) as i32).clamp(0, hi) with Rust's round-half-away-from-zero: trunc(t), plus one when
// the (exact) fraction t - trunc(t) is >= 0.5; negatives and NaN give 0, +inf gives hi.
__device__ __forceinline__ uint32_t code_of(float t, uint32_t hi) {
    const float tr = __builtin_truncf(t);
    const float c = fminf(fmaxf(tr, 0.0f), static_cast<float>(hi));
    const uint32_t u = static_cast<uint32_t>(c) + ((t - tr) >= 0.5f ? 1u : 0u);
    return u > hi ? hi : u;
}

// Every block folds the min/max partials (order-independent, so each block gets the same
// extremes bit for bit) and broadcasts them through LDS.
__device__ __forceinline__ void fold_partials(const float2 *__restrict__ partials, int np, float *smem, float &mx,
                                              float &mn) {
    mx = -INFINITY;
    mn = INFINITY;
    for (int i = threadIdx.x; i < np; i += kBlock) { float2 p = partials[i]; mx = fmaxf(mx, p.x); mn = fminf(mn, p.y); }
    block_minmax(mx, mn, smem);
    if (threadIdx.x == 0) { smem[0] = mx; smem[1] = mn; }
    __syncthreads();
    mx = smem[0];
    mn = smem[1];
}

template <int B>
__device__ __forceinline__ void store_packed(uint8_t *__restrict__ out, size_t o, const uint32_t (&c)[8]) {
    if constexpr (B == 8) {
        const uint32_t lo = c[0] | (c[1] << 8) | (c[2] << 16) | (c[3] << 24);
        const uint32_t hi = c[4] | (c[5] << 8) | (c[6] << 16) | (c[7] << 24);
        *reinterpret_cast<uint2 *>(out + o * 8) = make_uint2(lo, hi);
    } else {
        uint32_t w = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) w |= c[i] << (i * B);
        if constexpr (B == 4) *reinterpret_cast<uint32_t *>(out + o * 4) = w;
        else if constexpr (B == 2) *reinterpret_cast<uint16_t *>(out + o * 2) = static_cast<uint16_t>(w);
        else out[o] = static_cast<uint8_t>(w);
    }
}

template <int BA, int BB, bool kFast>
__device__ __forceinline__ void quantize_fused_body(const float *__restrict__ x, size_t n, uint8_t *__restrict__ out_a,
                                                    uint8_t *__restrict__ out_b, float sa, float za, float sb,
                                                    float zb) {
    const float ra = 1.0f / sa, rb = BB ? 1.0f / sb : 0.0f;
    constexpr uint32_t ha = (1u << BA) - 1u, hb = BB ? (1u << BB) - 1u : 0u;
    const size_t nfull = n / 8;
    const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    auto one = [&](size_t o, const float4 &p0, const float4 &p1) {
        const float v[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
        uint32_t ca[8], cb[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            ca[i] = code_of(div_scale<kFast>(v[i], sa, ra) + za, ha);   // :61-64
            if constexpr (BB != 0) cb[i] = code_of(div_scale<kFast>(v[i], sb, rb) + zb, hb);
        }
        store_packed<BA>(out_a, o, ca);
        if constexpr (BB != 0) store_packed<BB>(out_b, o, cb);
    };
    size_t o = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x;
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    for (; o + stride < nfull; o += 2 * stride) {       // two octets in flight per thread
        const float4 a0 = x4[2 * o], a1 = x4[2 * o + 1];
        const float4 b0 = x4[2 * (o + stride)], b1 = x4[2 * (o + stride) + 1];
        one(o, a0, a1);
        one(o + stride, b0, b1);
    }
    if (o < nfull) one(o, x4[2 * o], x4[2 * o + 1]);
    if (blockIdx.x == 0 && threadIdx.x == 0 && n % 8) {  // partial tail octet
        const size_t ot = nfull;
        const int cnt = static_cast<int>(n - ot * 8);
        uint32_t ca[8] = {0, 0, 0, 0, 0, 0, 0, 0}, cb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < cnt; ++i) {
            const float v = x[ot * 8 + i];
            ca[i] = code_of(div_scale<kFast>(v, sa, ra) + za, ha);
            if constexpr (BB != 0) cb[i] = code_of(div_scale<kFast>(v, sb, rb) + zb, hb);
        }
        store_codes(out_a, ot, cnt, ca, BA, true, false);
        if constexpr (BB != 0) store_codes(out_b, ot, cnt, cb, BB, true, false);
    }
}


// The same map with every load instruction one contiguous KiB: a wave takes chunks of 512 float4
// (2048 values); lane l holds float4s l, l + 64, ..., l + 448 of the chunk (8 loads in flight),
// codes its 4 values into a 4B-bit field and stores it at the field's place in the packed stream
// (B = 8: 4 bytes, 4: 2, 2: 1; B = 1: the nibbles of lanes 2i and 2i + 1 make one byte).  Octets
// past the last whole chunk (and the partial tail octet) go through quantize_fused_body's code.
template <int B>
__device__ __forceinline__ void store_quad(uint8_t *__restrict__ out, size_t f, uint32_t w, int lane) {
    if constexpr (B == 8) {
        *reinterpret_cast<uint32_t *>(out + f * 4) = w;
    } else if constexpr (B == 4) {
        *reinterpret_cast<uint16_t *>(out + f * 2) = static_cast<uint16_t>(w);
    } else if constexpr (B == 2) {
        out[f] = static_cast<uint8_t>(w);
    } else {
        const uint32_t other = static_cast<uint32_t>(__shfl_xor(static_cast<int>(w), 1, 64));
        if ((lane & 1) == 0) out[f >> 1] = static_cast<uint8_t>(w | (other << 4));
    }
}

template <int BA, int BB, bool kFast>
__device__ __forceinline__ void quantize_coalesced_body(const float *__restrict__ x, size_t n,
                                                        uint8_t *__restrict__ out_a, uint8_t *__restrict__ out_b,
                                                        float sa, float za, float sb, float zb, unsigned b,
                                                        unsigned nb) {
    const float ra = 1.0f / sa, rb = BB ? 1.0f / sb : 0.0f;
    constexpr uint32_t ha = (1u << BA) - 1u, hb = BB ? (1u << BB) - 1u : 0u;
    constexpr int kWaves = kBlock / 64;
    const int lane = threadIdx.x & 63;
    const size_t nchunk = n / 2048;
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    const size_t W = static_cast<size_t>(nb) * kWaves;
    for (size_t c = static_cast<size_t>(b) * kWaves + (threadIdx.x >> 6); c < nchunk; c += W) {
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = x4[c * 512 + j * 64 + lane];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
            uint32_t wa = 0, wb = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                wa |= code_of(div_scale<kFast>(e[i], sa, ra) + za, ha) << (i * BA);   // :61-64
                if constexpr (BB != 0) wb |= code_of(div_scale<kFast>(e[i], sb, rb) + zb, hb) << (i * BB);
            }
            const size_t f = c * 512 + j * 64 + lane;
            store_quad<BA>(out_a, f, wa, lane);
            if constexpr (BB != 0) store_quad<BB>(out_b, f, wb, lane);
        }
    }
    // the octets after the last whole chunk, then the partial tail octet
    const size_t nfull = n / 8;
    const size_t stride = static_cast<size_t>(nb) * kBlock;
    for (size_t o = nchunk * 256 + b * static_cast<size_t>(kBlock) + threadIdx.x; o < nfull; o += stride) {
        const float4 p0 = x4[2 * o], p1 = x4[2 * o + 1];
        const float e[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
        uint32_t ca[8], cb[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            ca[i] = code_of(div_scale<kFast>(e[i], sa, ra) + za, ha);
            if constexpr (BB != 0) cb[i] = code_of(div_scale<kFast>(e[i], sb, rb) + zb, hb);
        }
        store_packed<BA>(out_a, o, ca);
        if constexpr (BB != 0) store_packed<BB>(out_b, o, cb);
    }
    if (b == 0 && threadIdx.x == 0 && n % 8) {
        const int cnt = static_cast<int>(n - nfull * 8);
        uint32_t ca[8] = {0, 0, 0, 0, 0, 0, 0, 0}, cb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < cnt; ++i) {
            const float v = x[nfull * 8 + i];
            ca[i] = code_of(div_scale<kFast>(v, sa, ra) + za, ha);
            if constexpr (BB != 0) cb[i] = code_of(div_scale<kFast>(v, sb, rb) + zb, hb);
        }
        store_codes(out_a, nfull, cnt, ca, BA, true, false);
        if constexpr (BB != 0) store_codes(out_b, nfull, cnt, cb, BB, true, false);
    }
}

// quantize_tensor (and the pair of widths of KVCacheEntry::update) after minmax_partial_kernel:
// x 16-B aligned, packed codes (out 8-B aligned); block 0 publishes the params.
template <int BA, int BB>
__global__ void __launch_bounds__(kBlock) quantize_fused_kernel(const float *__restrict__ x, size_t n,
                                                                const float2 *__restrict__ partials, int np,
                                                                uint8_t *__restrict__ out_a, float *__restrict__ params_a,
                                                                uint8_t *__restrict__ out_b,
                                                                float *__restrict__ params_b) {
    __shared__ float smem[2 * kBlock / 64];
    float mx, mn, sa, za, sb = 1.0f, zb = 0.0f;
    fold_partials(partials, np, smem, mx, mn);
    params_of(mx, mn, BA, sa, za);
    if constexpr (BB != 0) params_of(mx, mn, BB, sb, zb);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        params_a[0] = sa; params_a[1] = za;
        if constexpr (BB != 0) { params_b[0] = sb; params_b[1] = zb; }
    }
#if DLLM_QMAP_OCTET   // A/B build: the round-3 octet-per-thread loads (two 32-B-strided float4 per lane)
    if (markstein_ok(sa) && (BB == 0 || markstein_ok(sb)))
        quantize_fused_body<BA, BB, true>(x, n, out_a, out_b, sa, za, sb, zb);
    else
        quantize_fused_body<BA, BB, false>(x, n, out_a, out_b, sa, za, sb, zb);
#else
    if (markstein_ok(sa) && (BB == 0 || markstein_ok(sb)))
        quantize_coalesced_body<BA, BB, true>(x, n, out_a, out_b, sa, za, sb, zb, blockIdx.x, gridDim.x);
    else
        quantize_coalesced_body<BA, BB, false>(x, n, out_a, out_b, sa, za, sb, zb, blockIdx.x, gridDim.x);
#endif
}

// ---------------------------------------------------------------------------------------------
// Both tensors of one KV-cache quantization (QuantizedKVCacheEntry::new, quantization.rs:140-157,
// and KVCacheEntry::update's two widths, lib.rs:241-276) as a few launches of one job kernel.  The
// blocks of a launch are dealt round-robin to its jobs (block i -> job i % jobs), so a map job
// whose x still sits in the Infinity Cache (read by the previous launch's min/max) runs beside a
// min/max job streaming the other tensor from HBM:
//   min/max K  |  map K (params folded from K's partials) + min/max V  |  map V.
// A map job takes its extremes from min/max partials, or from {-min, max} already reduced over
// the ranks of a head-sharded cache (dllm_quantize_kv_with_extremes).
// ---------------------------------------------------------------------------------------------
struct MapJob {
    const float *x;
    size_t n;
    uint8_t *out_a, *out_b;
    float *params_a, *params_b;
    const float2 *partials;   // extremes from these min/max partials (np of them) ...
    int np;
    const float *red;         // ... or from {-min, max} (red != nullptr)
};
struct MinmaxJob {
    const float *x;
    size_t n, head;
    float2 *partials;
    unsigned nb;              // blocks (= partials written)
};
struct KVJobs {
    MapJob map[2];
    MinmaxJob mm[2];
    int nmap, nmm;
    unsigned nbq;             // blocks per map job
};

template <int BA, int BB>
__global__ void __launch_bounds__(kBlock) kv_jobs_kernel(const KVJobs J) {
    __shared__ float smem[2 * kBlock / 64];
    const int jobs = J.nmap + J.nmm;
    const int role = static_cast<int>(blockIdx.x % jobs);
    const unsigned idx = blockIdx.x / jobs;
    if (role >= J.nmap) {
        const MinmaxJob &m = J.mm[role - J.nmap];
        if (idx < m.nb) minmax_body(m.x, m.n, m.head, m.partials, idx, m.nb, smem);
        return;
    }
    const MapJob &q = J.map[role];
    if (idx >= J.nbq) return;
    float mx, mn, sa, za, sb = 1.0f, zb = 0.0f;
    if (q.red) {
        mn = -q.red[0];
        mx = q.red[1];
    } else {
        fold_partials(q.partials, q.np, smem, mx, mn);
    }
    params_of(mx, mn, BA, sa, za);
    if constexpr (BB != 0) params_of(mx, mn, BB, sb, zb);
    if (idx == 0 && threadIdx.x == 0) {
        q.params_a[0] = sa; q.params_a[1] = za;
        if constexpr (BB != 0) { q.params_b[0] = sb; q.params_b[1] = zb; }
    }
    if (markstein_ok(sa) && (BB == 0 || markstein_ok(sb)))
        quantize_coalesced_body<BA, BB, true>(q.x, q.n, q.out_a, q.out_b, sa, za, sb, zb, idx, J.nbq);
    else
        quantize_coalesced_body<BA, BB, false>(q.x, q.n, q.out_a, q.out_b, sa, za, sb, zb, idx, J.nbq);
}

// {-min_K, max_K, -min_V, max_V} from the two tensors' min/max partials (dllm_kv_extremes).
__global__ void __launch_bounds__(kBlock) kv_red_kernel(const float2 *__restrict__ pk, int nk,
                                                        const float2 *__restrict__ pv, int nv, float *__restrict__ red) {
    __shared__ float smem[2 * kBlock / 64];
    float mx, mn;
    fold_partials(pk, nk, smem, mx, mn);
    if (threadIdx.x == 0) { red[0] = -mn; red[1] = mx; }
    __syncthreads();
    fold_partials(pv, nv, smem, mx, mn);
    if (threadIdx.x == 0) { red[2] = -mn; red[3] = mx; }
}

// Params of width `bits` from {-min, max} (the generic fallback of dllm_quantize_kv_with_extremes).
__global__ void params_from_red_kernel(const float *__restrict__ red, int bits, float *__restrict__ params) {
    if (threadIdx.x == 0) write_params(red[1], -red[0], bits, params);
}

// ---------------------------------------------------------------------------------------------
// K2: quantize map (quantization.rs:59-65) fused with packing (a6).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) quantize_tensor_kernel(const float *__restrict__ x, size_t n, int bits,
                                                                 int packed, uint8_t *__restrict__ out,
                                                                 const float *__restrict__ params, int vec_in,
                                                                 int vec_out) {
    const float scale = params[0], zp = params[1];
    const int hi = (1 << bits) - 1;
    const size_t noct = (n + 7) / 8;
    for (size_t o = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; o < noct;
         o += static_cast<size_t>(gridDim.x) * kBlock) {
        const int cnt = octet_count(o, n);
        F8 v = load_octet(x, o, cnt, vec_in);
        uint32_t c[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float t = v.v[i] / scale;       // IEEE division (separately rounded)
            t = t + zp;                     // separately rounded add
            c[i] = (i < cnt) ? rs_round_i32_clamp(t, hi) : 0u;
        }
        store_codes(out, o, cnt, c, bits, packed, vec_out);
    }
}

// K2 at two widths of the same x: one read, two code sets (each width's arithmetic exactly K2's).
__global__ void __launch_bounds__(kBlock) quantize_pair_kernel(const float *__restrict__ x, size_t n, int bits_a,
                                                               int bits_b, int packed, uint8_t *__restrict__ out_a,
                                                               uint8_t *__restrict__ out_b,
                                                               const float *__restrict__ params_a,
                                                               const float *__restrict__ params_b, int vec_in,
                                                               int vec_out_a, int vec_out_b) {
    const float sa = params_a[0], za = params_a[1], sb = params_b[0], zb = params_b[1];
    const int ha = (1 << bits_a) - 1, hb = (1 << bits_b) - 1;
    const size_t noct = (n + 7) / 8;
    for (size_t o = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; o < noct;
         o += static_cast<size_t>(gridDim.x) * kBlock) {
        const int cnt = octet_count(o, n);
        F8 v = load_octet(x, o, cnt, vec_in);
        uint32_t ca[8], cb[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float ta = v.v[i] / sa + za;
            const float tb = v.v[i] / sb + zb;
            ca[i] = (i < cnt) ? rs_round_i32_clamp(ta, ha) : 0u;
            cb[i] = (i < cnt) ? rs_round_i32_clamp(tb, hb) : 0u;
        }
        store_codes(out_a, o, cnt, ca, bits_a, packed, vec_out_a);
        store_codes(out_b, o, cnt, cb, bits_b, packed, vec_out_b);
    }
}

// ---------------------------------------------------------------------------------------------
// K3: dequantize (quantization.rs:81-85): y = (q as f32 - zp) * scale.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) dequantize_kernel(const uint8_t *__restrict__ q, size_t n, int bits,
                                                            int packed, const float *__restrict__ params, float s_arg,
                                                            float z_arg, void *__restrict__ out, int dtype, int vec_in,
                                                            int vec_out) {
    const float scale = params ? params[0] : s_arg;
    const float zp = params ? params[1] : z_arg;
    const size_t noct = (n + 7) / 8;
    for (size_t o = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; o < noct;
         o += static_cast<size_t>(gridDim.x) * kBlock) {
        const int cnt = octet_count(o, n);
        uint32_t c[8];
        load_codes(q, o, cnt, bits, packed, vec_in, c);
        float y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float d = static_cast<float>(c[i]) - zp;
            y[i] = d * scale;
        }
        store_f8(out, dtype, o, cnt, y, vec_out);
    }
}

// a6 standalone: codes (one per byte) <-> packed bitstream.
__global__ void __launch_bounds__(kBlock) pack_kernel(const uint8_t *__restrict__ codes, size_t n, int bits,
                                                      uint8_t *__restrict__ packed, int vec_in, int vec_out) {
    const size_t noct = (n + 7) / 8;
    const uint32_t mask = (1u << bits) - 1u;
    for (size_t o = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; o < noct;
         o += static_cast<size_t>(gridDim.x) * kBlock) {
        const int cnt = octet_count(o, n);
        uint32_t c[8];
        load_codes(codes, o, cnt, 8, false, vec_in, c);
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] &= mask;
        store_codes(packed, o, cnt, c, bits, true, vec_out);
    }
}

__global__ void __launch_bounds__(kBlock) unpack_kernel(const uint8_t *__restrict__ packed, size_t n, int bits,
                                                        uint8_t *__restrict__ codes, int vec_in, int vec_out) {
    const size_t noct = (n + 7) / 8;
    for (size_t o = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; o < noct;
         o += static_cast<size_t>(gridDim.x) * kBlock) {
        const int cnt = octet_count(o, n);
        uint32_t c[8];
        load_codes(packed, o, cnt, bits, true, vec_in, c);
        store_codes(codes, o, cnt, c, 8, false, vec_out);
    }
}

// ---------------------------------------------------------------------------------------------
// a4: DefaultQuantizer (quantization/src/quantize.rs:111-154, :172-184).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) default_quantize_kernel(const float *__restrict__ x, size_t n, float scale,
                                                                  float zp, float lo, float hi,
                                                                  uint8_t *__restrict__ out, int vec_in, int vec_out) {
    const size_t noct = (n + 7) / 8;
    for (size_t o = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; o < noct;
         o += static_cast<size_t>(gridDim.x) * kBlock) {
        const int cnt = octet_count(o, n);
        F8 v = load_octet(x, o, cnt, vec_in);
        uint32_t c[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float t = v.v[i] / scale;
            t = t + zp;
            t = fminf(fmaxf(t, lo), hi);    // .max(min).min(max): NaN -> lo (:119-121)
            c[i] = rs_as_u8(roundf(t));     // .round(), then `q as u8` (:122, :150)
        }
        store_codes(out, o, cnt, c, 8, false, vec_out);
    }
}

// ---------------------------------------------------------------------------------------------
// a8-ii BitQuantizer (prefill-kvquant-rs/lib.rs:39-53) and its row-batched forms.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bitq(float x, float scale, float zp, float max_val) {
    float s = (x - zp) / scale;
    return rs_as_u8(rs_clamp(s, 0.0f, max_val));
}

__global__ void __launch_bounds__(kBlock) bit_quantize_kernel(const float *__restrict__ x, size_t n, float scale,
                                                              float zp, float max_val, uint8_t *__restrict__ out,
                                                              int vec_in, int vec_out) {
    const size_t noct = (n + 7) / 8;
    for (size_t o = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; o < noct;
         o += static_cast<size_t>(gridDim.x) * kBlock) {
        const int cnt = octet_count(o, n);
        F8 v = load_octet(x, o, cnt, vec_in);
        uint32_t c[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] = bitq(v.v[i], scale, zp, max_val);
        store_codes(out, o, cnt, c, 8, false, vec_out);
    }
}

__global__ void __launch_bounds__(kBlock) bit_dequantize_kernel(const uint8_t *__restrict__ q, size_t n, float scale,
                                                                float zp, void *__restrict__ out, int dtype, int vec_in,
                                                                int vec_out) {
    const size_t noct = (n + 7) / 8;
    for (size_t o = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; o < noct;
         o += static_cast<size_t>(gridDim.x) * kBlock) {
        const int cnt = octet_count(o, n);
        uint32_t c[8];
        load_codes(q, o, cnt, 8, false, vec_in, c);
        float y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float p = static_cast<float>(c[i]) * scale;   // lib.rs:50, no FMA
            y[i] = p + zp;
        }
        store_f8(out, dtype, o, cnt, y, vec_out);
    }
}

// PrefillKVQuant::quantize_vectors: the per-row (bits, scale) cycle table, passed by value.
constexpr int kCycleMax = 64;
struct CycleTable {
    float scale[kCycleMax];
    float max_val[kCycleMax];
};

// One block per (row, chunk); rows r = r0 + j*rstride (j = blockIdx.y).
__global__ void __launch_bounds__(kBlock) quantize_rows_cycle_kernel(const float *__restrict__ x, size_t rows,
                                                                     size_t dim, int ncycle, CycleTable tab,
                                                                     uint8_t *__restrict__ out) {
    const size_t r = blockIdx.y;
    if (r >= rows) return;
    const int slot = static_cast<int>(r % static_cast<size_t>(ncycle));
    const float scale = tab.scale[slot], max_val = tab.max_val[slot];
    const float *xr = x + r * dim;
    uint8_t *orow = out + r * dim;
    for (size_t i = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; i < dim;
         i += static_cast<size_t>(gridDim.x) * kBlock)
        orow[i] = static_cast<uint8_t>(bitq(xr[i], scale, 0.0f, max_val));
}

// a8-iii compress_vector (diffusion_prefill/src/prefill_kv.rs:104-121): one block per row.
__global__ void __launch_bounds__(kBlock) compress_rows_kernel(const float *__restrict__ x, size_t dim, float levels,
                                                               uint8_t *__restrict__ out, float *__restrict__ scales,
                                                               float *__restrict__ zps) {
    __shared__ float smem[2 * kBlock / 64];
    __shared__ float sp[2];
    const size_t r = blockIdx.x;
    const float *xr = x + r * dim;
    float mx = -INFINITY, mn = INFINITY;
    for (size_t i = threadIdx.x; i < dim; i += kBlock) { float v = xr[i]; mx = fmaxf(mx, v); mn = fminf(mn, v); }
    block_minmax(mx, mn, smem);
    if (threadIdx.x == 0) {
        const float scale = (mx - mn) / levels;   // :107
        sp[0] = scale; sp[1] = mn;                 // :108 zero_point = min
        scales[r] = scale; zps[r] = mn;
    }
    __syncthreads();
    const float scale = sp[0], zp = sp[1];
    uint8_t *orow = out + r * dim;
    for (size_t i = threadIdx.x; i < dim; i += kBlock) orow[i] = static_cast<uint8_t>(bitq(xr[i], scale, zp, levels));
}

__global__ void __launch_bounds__(kBlock) decompress_rows_kernel(const uint8_t *__restrict__ q, size_t rows, size_t dim,
                                                                 const float *__restrict__ scales,
                                                                 const float *__restrict__ zps,
                                                                 float *__restrict__ out) {
    const size_t total = rows * dim;
    for (size_t i = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; i < total;
         i += static_cast<size_t>(gridDim.x) * kBlock) {
        const size_t r = i / dim;
        float p = static_cast<float>(q[i]) * scales[r];
        out[i] = p + zps[r];
    }
}

// ---------------------------------------------------------------------------------------------
// a10: CalibrationData::update (quantization/src/calibrate.rs:42-69) on the device.
// ---------------------------------------------------------------------------------------------
// seed: the fold's start value, f32::MAX for calibrate.rs:43 (MIN/MAX seeds), +inf for the
// adaptive quantizer's exact extremes.
__global__ void __launch_bounds__(kBlock) calib_fold_kernel(const float2 *__restrict__ partials, int np,
                                                            float *__restrict__ stats, float seed) {
    __shared__ float smem[2 * kBlock / 64];
    float mx = -seed, mn = seed;
    for (int i = threadIdx.x; i < np; i += kBlock) { float2 p = partials[i]; mx = fmaxf(mx, p.x); mn = fminf(mn, p.y); }
    block_minmax(mx, mn, smem);
    if (threadIdx.x == 0) {
        stats[0] = fminf(stats[0], mn);   // :47
        stats[1] = fmaxf(stats[1], mx);   // :48
    }
}

__global__ void __launch_bounds__(kBlock) calib_hist_kernel(const float *__restrict__ x, size_t n,
                                                            const float *__restrict__ stats,
                                                            unsigned long long *__restrict__ hist, int num_bins,
                                                            int use_lds) {
    extern __shared__ unsigned int lhist[];
    const float mn = stats[0], mx = stats[1];
    if (!(mx > mn)) return;                                   // :59
    const float bw = (mx - mn) / static_cast<float>(num_bins); // :60
    if (use_lds) {
        for (int b = threadIdx.x; b < num_bins; b += kBlock) lhist[b] = 0u;
        __syncthreads();
    }
    for (size_t i = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; i < n;
         i += static_cast<size_t>(gridDim.x) * kBlock) {
        const float v = x[i];
        if (v >= mn && v <= mx) {                             // :62
            float f = floorf((v - mn) / bw);                  // :63
            unsigned long long b = (f > 0.0f) ? static_cast<unsigned long long>(f) : 0ull;  // `as usize`
            if (f >= 18446744073709551616.0f) b = ~0ull;
            if (b > static_cast<unsigned long long>(num_bins - 1)) b = num_bins - 1;        // :64
            if (use_lds) atomicAdd(&lhist[b], 1u);
            else atomicAdd(&hist[b], 1ull);
        }
    }
    if (use_lds) {
        __syncthreads();
        for (int b = threadIdx.x; b < num_bins; b += kBlock)
            if (lhist[b]) atomicAdd(&hist[b], static_cast<unsigned long long>(lhist[b]));
    }
}

// ---------------------------------------------------------------------------------------------
// 8f rank 4: AdaptiveQuantizer (diffuse-llm-rs/src/quantization.rs:178-235).
// ---------------------------------------------------------------------------------------------
// compute_params (:206-217): query(0.0/1.0).unwrap_or(0.0/1.0); scale without a zero guard;
// zp = round(-min / scale).clamp(0, q_max) -- round first, NaN passes the clamp.
__global__ void adaptive_params_kernel(const float *__restrict__ stats, int has_samples, uint32_t bits,
                                       float *__restrict__ params) {
    if (threadIdx.x != 0) return;
    const float mn = has_samples ? stats[0] : 0.0f;
    const float mx = has_samples ? stats[1] : 1.0f;
    const float q_max = static_cast<float>(1u << bits) - 1.0f;  // :212
    const float scale = (mx - mn) / q_max;                        // :213
    const float m = -mn;
    params[0] = scale;
    params[1] = rs_clamp(roundf(m / scale), 0.0f, q_max);         // :214
}

// quantize (:220-234), one code per byte: (round(x/scale + zp) as i32).clamp(0, hi) as u8, where
// hi = q_max as i32 and `as u8` keeps the low byte (bits > 8).  Four elements per thread.
__global__ void __launch_bounds__(kBlock) adaptive_quantize_kernel(const float *__restrict__ x, size_t n, int hi,
                                                                   const float *__restrict__ params,
                                                                   uint8_t *__restrict__ out) {
    const float scale = params[0], zp = params[1];
    const size_t nq = (n + 3) / 4;
    for (size_t o = blockIdx.x * static_cast<size_t>(kBlock) + threadIdx.x; o < nq;
         o += static_cast<size_t>(gridDim.x) * kBlock) {
        const size_t i0 = 4 * o;
        uint32_t word = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (i0 + j < n) {
                float t = x[i0 + j] / scale;
                t = t + zp;
                word |= (rs_round_i32_clamp(t, hi) & 0xffu) << (8 * j);
            }
        }
        if (i0 + 4 <= n) {
            if ((reinterpret_cast<uintptr_t>(out + i0) & 3) == 0) {
                *reinterpret_cast<uint32_t *>(out + i0) = word;
                continue;
            }
        }
        for (int j = 0; j < 4 && i0 + j < n; ++j) out[i0 + j] = static_cast<uint8_t>(word >> (8 * j));
    }
}

inline bool aligned(const void *p, size_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

#ifndef DLLM_GRID_CAP   // A/B builds: every streaming quantization kernel on at most this many blocks
#define DLLM_GRID_CAP 0
#endif
constexpr unsigned kCapOr(unsigned c) { return DLLM_GRID_CAP ? DLLM_GRID_CAP : c; }
inline unsigned octet_grid(size_t n) { return grid_for((n + 7) / 8, kBlock, kCapOr(kCUs * 16)); }

constexpr unsigned kMinmaxBlocks = kCapOr(1024);

inline int launch_minmax(const float *x, size_t n, float2 *partials, unsigned nblk, hipStream_t st) {
    size_t head = 0;
    if (aligned(x, 4)) head = ((16 - (reinterpret_cast<uintptr_t>(x) & 15)) & 15) / 4;
    else return fail(DLLM_ERR_INVALID_PARAMS, "x must be 4-byte aligned");
    if (head > n) head = n;
    minmax_partial_kernel<<<nblk, kBlock, 0, st>>>(x, n, head, partials);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

inline unsigned minmax_blocks(size_t n) { return grid_for((n + 15) / 16, kBlock, kMinmaxBlocks); }

// Lab build only: DLLM_QUANT_GENERIC=1 selects the generic two-kernel path (A/B measurement).  The
// product library reads no environment; its generic path runs for x not 16-byte aligned.
#ifndef DLLM_LAB
#define DLLM_LAB 0
#endif
inline bool fused_disabled() {
#if DLLM_LAB
    const char *e = std::getenv("DLLM_QUANT_GENERIC");
    return e && e[0] == '1';
#else
    return false;
#endif
}

inline bool fused_width(int b) { return b == 1 || b == 2 || b == 4 || b == 8; }

// Grid of quantize_fused_kernel: two full octets per thread per trip, at most 8 blocks per CU
// (all resident, so the prologue's 8 KiB partials read overlaps other blocks' streaming).
inline unsigned fused_grid(size_t n) { return grid_for((n / 8 + 1) / 2, kBlock, kCapOr(kCUs * 8)); }

template <int BA>
int launch_fused_b(const float *x, size_t n, const float2 *partials, int np, uint8_t *out_a, float *params_a, int bb,
                   uint8_t *out_b, float *params_b, hipStream_t st) {
    const unsigned g = fused_grid(n);
    switch (bb) {
    case 0: quantize_fused_kernel<BA, 0><<<g, kBlock, 0, st>>>(x, n, partials, np, out_a, params_a, out_b, params_b); break;
    case 1: quantize_fused_kernel<BA, 1><<<g, kBlock, 0, st>>>(x, n, partials, np, out_a, params_a, out_b, params_b); break;
    case 2: quantize_fused_kernel<BA, 2><<<g, kBlock, 0, st>>>(x, n, partials, np, out_a, params_a, out_b, params_b); break;
    case 4: quantize_fused_kernel<BA, 4><<<g, kBlock, 0, st>>>(x, n, partials, np, out_a, params_a, out_b, params_b); break;
    default: quantize_fused_kernel<BA, 8><<<g, kBlock, 0, st>>>(x, n, partials, np, out_a, params_a, out_b, params_b); break;
    }
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

// bits_b = 0: one width.  Preconditions: fused_width(bits_a) (and bits_b), x 16-B and outs 8-B aligned.
inline int launch_fused(const float *x, size_t n, const float2 *partials, int np, int bits_a, uint8_t *out_a,
                        float *params_a, int bits_b, uint8_t *out_b, float *params_b, hipStream_t st) {
    switch (bits_a) {
    case 1: return launch_fused_b<1>(x, n, partials, np, out_a, params_a, bits_b, out_b, params_b, st);
    case 2: return launch_fused_b<2>(x, n, partials, np, out_a, params_a, bits_b, out_b, params_b, st);
    case 4: return launch_fused_b<4>(x, n, partials, np, out_a, params_a, bits_b, out_b, params_b, st);
    default: return launch_fused_b<8>(x, n, partials, np, out_a, params_a, bits_b, out_b, params_b, st);
    }
}

}  // namespace

#if DLLM_LAB
// lab/quant_resident.hip (lab build only): quantize_tensor of one or two tensors in one HBM read
// (returns 1, launching nothing, when they do not fit on chip or the shape is outside its
// preconditions).
int launch_quantize_resident(const float *const *x, const size_t *n, int nt, const int *bits, uint8_t *const *out,
                             float *const *params, void *ws, size_t ws_bytes, hipStream_t st);
#endif

namespace {

#if DLLM_LAB
// The single pass pays one grid-wide hand-off (a few us): below 4 Mi values per tensor the two
// passes (both in the Infinity Cache) are as fast.
constexpr size_t kResidentMin = size_t(1) << 22;
#endif

// One or two tensors at one or two widths through the single-pass resident kernel; 0 = launched,
// 1 = not applicable (the caller runs the multi-pass path), else an error code.  An A/B of the lab
// build (DLLM_QUANT_RESIDENT=1): measured slower than the two passes at every size it holds
// (8192 x 4096: 60 vs 49 us), so the product runs the two-pass kernels and
// does not contain the resident kernel.
inline int try_resident(int nt, const float *x0, size_t n0, const float *x1, size_t n1, int ba, int bb,
                        uint8_t *o0a, float *p0a, uint8_t *o0b, float *p0b, uint8_t *o1a, float *p1a, uint8_t *o1b,
                        float *p1b, void *ws, size_t wsb, hipStream_t st) {
#if DLLM_LAB
    const char *e = std::getenv("DLLM_QUANT_RESIDENT");
    if (!(e && e[0] == '1') || !fused_width(ba) || (bb && !fused_width(bb))) return 1;
    if (n0 < kResidentMin || (nt > 1 && n1 < kResidentMin)) return 1;
    const float *x[2] = {x0, x1};
    const size_t n[2] = {n0, n1};
    const int bits[2] = {ba, bb};
    uint8_t *out[4] = {o0a, o0b, o1a, o1b};
    float *params[4] = {p0a, p0b, p1a, p1b};
    return launch_quantize_resident(x, n, nt, bits, out, params, ws, wsb, st);
#else
    (void)nt; (void)x0; (void)n0; (void)x1; (void)n1; (void)ba; (void)bb; (void)o0a; (void)p0a; (void)o0b;
    (void)p0b; (void)o1a; (void)p1a; (void)o1b; (void)p1b; (void)ws; (void)wsb; (void)st;
    return 1;
#endif
}

template <int BA>
int launch_kv_jobs_b(const KVJobs &J, int bb, unsigned grid, hipStream_t st) {
    switch (bb) {
    case 0: kv_jobs_kernel<BA, 0><<<grid, kBlock, 0, st>>>(J); break;
    case 1: kv_jobs_kernel<BA, 1><<<grid, kBlock, 0, st>>>(J); break;
    case 2: kv_jobs_kernel<BA, 2><<<grid, kBlock, 0, st>>>(J); break;
    case 4: kv_jobs_kernel<BA, 4><<<grid, kBlock, 0, st>>>(J); break;
    default: kv_jobs_kernel<BA, 8><<<grid, kBlock, 0, st>>>(J); break;
    }
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

// One launch of kv_jobs_kernel: every job gets `per` blocks (map jobs J.nbq, min/max jobs their nb).
int launch_kv_jobs(KVJobs J, int ba, int bb, hipStream_t st) {
    unsigned per = J.nmap ? J.nbq : 0;
    for (int i = 0; i < J.nmm; ++i) per = std::max(per, J.mm[i].nb);
    const unsigned grid = per * static_cast<unsigned>(J.nmap + J.nmm);
    switch (ba) {
    case 1: return launch_kv_jobs_b<1>(J, bb, grid, st);
    case 2: return launch_kv_jobs_b<2>(J, bb, grid, st);
    case 4: return launch_kv_jobs_b<4>(J, bb, grid, st);
    default: return launch_kv_jobs_b<8>(J, bb, grid, st);
    }
}

inline size_t minmax_head(const float *x, size_t n) {
    size_t head = ((16 - (reinterpret_cast<uintptr_t>(x) & 15)) & 15) / 4;
    return head > n ? n : head;
}

inline MinmaxJob minmax_job(const float *x, size_t n, float2 *partials) {
    return MinmaxJob{x, n, minmax_head(x, n), partials, minmax_blocks(n)};
}

inline MapJob map_job(const float *x, size_t n, uint8_t *oa, float *pa, uint8_t *ob, float *pb,
                      const float2 *partials, int np, const float *red) {
    return MapJob{x, n, oa, ob, pa, pb, partials, np, red};
}

}  // namespace
}  // namespace dllm

using namespace dllm;

// =============================================================================================
// C-ABI
// =============================================================================================
extern "C" {

size_t dllm_quantize_tensor_workspace(size_t n) { return sizeof(float2) * minmax_blocks(n); }

size_t dllm_quantize_kv_workspace(size_t n_k, size_t n_v) {
    return sizeof(float2) * (minmax_blocks(n_k) + minmax_blocks(n_v));
}

int dllm_quantize_kv(const float *k, size_t n_k, const float *v, size_t n_v, uint8_t bits_a, uint8_t bits_b,
                     int packed, uint8_t *k_a, float *kp_a, uint8_t *v_a, float *vp_a, uint8_t *k_b, float *kp_b,
                     uint8_t *v_b, float *vp_b, void *workspace, size_t workspace_bytes, dllm_stream_t stream) {
    if (bits_a < 1 || bits_a > 8 || bits_b > 8) return fail(DLLM_ERR_INVALID_PARAMS, "Bits must be between 1 and 8");
    const bool two = bits_b != 0;
    if (!kp_a || !vp_a || (two && (!kp_b || !vp_b)) || (n_k && (!k || !k_a || (two && !k_b))) ||
        (n_v && (!v || !v_a || (two && !v_b))))
        return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    const unsigned nbk = minmax_blocks(n_k), nbv = minmax_blocks(n_v);
    if (!workspace || workspace_bytes < sizeof(float2) * (nbk + nbv))
        return fail(DLLM_ERR_INVALID_PARAMS, "workspace too small (see dllm_quantize_kv_workspace)");
    float2 *pk = static_cast<float2 *>(workspace), *pv = pk + nbk;
    const bool fast = packed && n_k && n_v && fused_width(bits_a) && (!two || fused_width(bits_b)) &&
                      aligned(k, 16) && aligned(v, 16) && aligned(k_a, 8) && aligned(v_a, 8) &&
                      (!two || (aligned(k_b, 8) && aligned(v_b, 8))) && !fused_disabled();
    if (fast) {   // lab A/B: one HBM read, K and V together when both fit on chip
        const int rr = try_resident(2, k, n_k, v, n_v, bits_a, bits_b, k_a, kp_a, k_b, kp_b, v_a, vp_a, v_b, vp_b,
                                    workspace, workspace_bytes, as_stream(stream));
        if (rr != 1) return rr;
    }
    // per tensor, two passes each (min/max | map with the params folded in): measured as fast as or
    // faster than one launch mapping K beside V's min/max (C4 98.5 vs 99.8 us; C5's pair 44.2 vs
    // 49.1 us, profiles/r04_quant/), with the same bits
    int rc = two ? dllm_quantize_tensor_pair(k, n_k, bits_a, bits_b, packed, k_a, kp_a, k_b, kp_b, pk,
                                             sizeof(float2) * nbk, stream)
                 : dllm_quantize_tensor(k, n_k, bits_a, packed, k_a, kp_a, pk, sizeof(float2) * nbk, stream);
    if (rc) return rc;
    return two ? dllm_quantize_tensor_pair(v, n_v, bits_a, bits_b, packed, v_a, vp_a, v_b, vp_b, pv,
                                           sizeof(float2) * nbv, stream)
               : dllm_quantize_tensor(v, n_v, bits_a, packed, v_a, vp_a, pv, sizeof(float2) * nbv, stream);
}

int dllm_kv_extremes(const float *k, size_t n_k, const float *v, size_t n_v, float *red, void *workspace,
                     size_t workspace_bytes, dllm_stream_t stream) {
    if (!red || (n_k && !k) || (n_v && !v)) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    if ((n_k && !aligned(k, 4)) || (n_v && !aligned(v, 4))) return fail(DLLM_ERR_INVALID_PARAMS, "x must be 4-byte aligned");
    const unsigned nbk = minmax_blocks(n_k), nbv = minmax_blocks(n_v);
    if (!workspace || workspace_bytes < sizeof(float2) * (nbk + nbv))
        return fail(DLLM_ERR_INVALID_PARAMS, "workspace too small (see dllm_quantize_kv_workspace)");
    float2 *pk = static_cast<float2 *>(workspace), *pv = pk + nbk;
    hipStream_t st = as_stream(stream);
    KVJobs J{};
    if (n_k) J.mm[J.nmm++] = minmax_job(k, n_k, pk);
    if (n_v) J.mm[J.nmm++] = minmax_job(v, n_v, pv);
    if (J.nmm) {
        const int rc = launch_kv_jobs(J, 1, 0, st);
        if (rc) return rc;
    }
    kv_red_kernel<<<1, kBlock, 0, st>>>(pk, n_k ? static_cast<int>(nbk) : 0, pv, n_v ? static_cast<int>(nbv) : 0, red);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_quantize_kv_with_extremes(const float *k, size_t n_k, const float *v, size_t n_v, const float *red,
                                   uint8_t bits_a, uint8_t bits_b, int packed, uint8_t *k_a, float *kp_a,
                                   uint8_t *v_a, float *vp_a, uint8_t *k_b, float *kp_b, uint8_t *v_b, float *vp_b,
                                   dllm_stream_t stream) {
    if (bits_a < 1 || bits_a > 8 || bits_b > 8) return fail(DLLM_ERR_INVALID_PARAMS, "Bits must be between 1 and 8");
    const bool two = bits_b != 0;
    if (!red || !kp_a || !vp_a || (two && (!kp_b || !vp_b)) || (n_k && (!k || !k_a || (two && !k_b))) ||
        (n_v && (!v || !v_a || (two && !v_b))))
        return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    hipStream_t st = as_stream(stream);
    const bool fast = packed && n_k && n_v && fused_width(bits_a) && (!two || fused_width(bits_b)) &&
                      aligned(k, 16) && aligned(v, 16) && aligned(k_a, 8) && aligned(v_a, 8) &&
                      (!two || (aligned(k_b, 8) && aligned(v_b, 8))) && !fused_disabled();
    if (!fast) {
        const float *rk = red, *rv = red + 2;
        for (int t = 0; t < 2; ++t) {
            const float *x = t ? v : k, *r = t ? rv : rk;
            const size_t n = t ? n_v : n_k;
            uint8_t *oa = t ? v_a : k_a, *ob = t ? v_b : k_b;
            float *pa = t ? vp_a : kp_a, *pb = t ? vp_b : kp_b;
            params_from_red_kernel<<<1, 64, 0, st>>>(r, bits_a, pa);
            DLLM_LAUNCH_CHECK();
            if (two) {
                params_from_red_kernel<<<1, 64, 0, st>>>(r, bits_b, pb);
                DLLM_LAUNCH_CHECK();
            }
            const int rc = two ? dllm_quantize_tensor_pair_with_params(x, n, bits_a, bits_b, packed, pa, pb, oa, ob, stream)
                               : dllm_quantize_tensor_with_params(x, n, bits_a, packed, pa, oa, stream);
            if (rc) return rc;
        }
        return DLLM_OK;
    }
    KVJobs J{};
    J.map[0] = map_job(k, n_k, k_a, kp_a, k_b, kp_b, nullptr, 0, red);
    J.map[1] = map_job(v, n_v, v_a, vp_a, v_b, vp_b, nullptr, 0, red + 2);
    J.nmap = 2; J.nbq = fused_grid(std::max(n_k, n_v));
    return launch_kv_jobs(J, bits_a, bits_b, st);
}

int dllm_quantize_tensor(const float *x, size_t n, uint8_t bits, int packed, uint8_t *out, float *params_out,
                         void *workspace, size_t workspace_bytes, dllm_stream_t stream) {
    if (bits < 1 || bits > 8) return fail(DLLM_ERR_INVALID_PARAMS, "Bits must be between 1 and 8");
    if (!params_out || (n && (!x || !out))) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    const unsigned nblk = minmax_blocks(n);
    if (!workspace || workspace_bytes < sizeof(float2) * nblk)
        return fail(DLLM_ERR_INVALID_PARAMS, "workspace too small (see dllm_quantize_tensor_workspace)");
    hipStream_t st = as_stream(stream);
    float2 *partials = static_cast<float2 *>(workspace);
    if (n && packed) {
        const int rr = try_resident(1, x, n, nullptr, 0, bits, 0, out, params_out, nullptr, nullptr, nullptr, nullptr,
                                    nullptr, nullptr, workspace, workspace_bytes, st);
        if (rr != 1) return rr;
    }
    if (n) {
        int rc = launch_minmax(x, n, partials, nblk, st);
        if (rc) return rc;
        if (packed && fused_width(bits) && aligned(x, 16) && aligned(out, 8) && !fused_disabled())
            return launch_fused(x, n, partials, static_cast<int>(nblk), bits, out, params_out, 0, nullptr, nullptr,
                                st);
    }
    quant_params_kernel<<<1, kBlock, 0, st>>>(partials, n ? static_cast<int>(nblk) : 0, bits, params_out);
    DLLM_LAUNCH_CHECK();
    if (n) {
        quantize_tensor_kernel<<<octet_grid(n), kBlock, 0, st>>>(x, n, bits, packed, out, params_out,
                                                                 aligned(x, 16), aligned(out, 8));
        DLLM_LAUNCH_CHECK();
    }
    return DLLM_OK;
}

int dllm_quantize_tensor_pair(const float *x, size_t n, uint8_t bits_a, uint8_t bits_b, int packed, uint8_t *out_a,
                              float *params_a, uint8_t *out_b, float *params_b, void *workspace,
                              size_t workspace_bytes, dllm_stream_t stream) {
    if (bits_a < 1 || bits_a > 8 || bits_b < 1 || bits_b > 8)
        return fail(DLLM_ERR_INVALID_PARAMS, "Bits must be between 1 and 8");
    if (!params_a || !params_b || (n && (!x || !out_a || !out_b))) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    const unsigned nblk = minmax_blocks(n);
    if (!workspace || workspace_bytes < sizeof(float2) * nblk)
        return fail(DLLM_ERR_INVALID_PARAMS, "workspace too small (see dllm_quantize_tensor_workspace)");
    hipStream_t st = as_stream(stream);
    float2 *partials = static_cast<float2 *>(workspace);
    if (n && packed) {
        const int rr = try_resident(1, x, n, nullptr, 0, bits_a, bits_b, out_a, params_a, out_b, params_b, nullptr,
                                    nullptr, nullptr, nullptr, workspace, workspace_bytes, st);
        if (rr != 1) return rr;
    }
    if (n) {
        int rc = launch_minmax(x, n, partials, nblk, st);
        if (rc) return rc;
        if (packed && fused_width(bits_a) && fused_width(bits_b) && aligned(x, 16) && aligned(out_a, 8) &&
            aligned(out_b, 8) && !fused_disabled())
            return launch_fused(x, n, partials, static_cast<int>(nblk), bits_a, out_a, params_a, bits_b, out_b,
                                params_b, st);
    }
    quant_params_kernel<<<1, kBlock, 0, st>>>(partials, n ? static_cast<int>(nblk) : 0, bits_a, params_a, bits_b,
                                              params_b);
    DLLM_LAUNCH_CHECK();
    if (n) {
        quantize_pair_kernel<<<octet_grid(n), kBlock, 0, st>>>(x, n, bits_a, bits_b, packed, out_a, out_b, params_a,
                                                               params_b, aligned(x, 16), aligned(out_a, 8),
                                                               aligned(out_b, 8));
        DLLM_LAUNCH_CHECK();
    }
    return DLLM_OK;
}

static int dequant_common(const uint8_t *q, size_t n, uint8_t bits, int packed, const float *params, float s,
                          float z, void *out, int out_dtype, dllm_stream_t stream) {
    if (bits < 1 || bits > 8) return fail(DLLM_ERR_INVALID_PARAMS, "Bits must be between 1 and 8");
    if (out_dtype != DLLM_F32 && out_dtype != DLLM_F16) return fail(DLLM_ERR_UNSUPPORTED, "out_dtype");
    if (!n) return DLLM_OK;
    if (!q || !out) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    dequantize_kernel<<<octet_grid(n), kBlock, 0, as_stream(stream)>>>(q, n, bits, packed, params, s, z, out,
                                                                       out_dtype, aligned(q, 8), aligned(out, 16));
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_dequantize_tensor(const uint8_t *q, size_t n, uint8_t bits, int packed, const float *params, void *out,
                           int out_dtype, dllm_stream_t stream) {
    if (!params) return fail(DLLM_ERR_INVALID_PARAMS, "params is null");
    return dequant_common(q, n, bits, packed, params, 0.f, 0.f, out, out_dtype, stream);
}

int dllm_dequantize_tensor_scalar(const uint8_t *q, size_t n, uint8_t bits, int packed, float scale, float zp,
                                  void *out, int out_dtype, dllm_stream_t stream) {
    return dequant_common(q, n, bits, packed, nullptr, scale, zp, out, out_dtype, stream);
}

float dllm_compression_ratio(size_t numel, size_t len, uint8_t bits) {
    const size_t original = numel * 4;                      // quantization.rs:121
    const size_t compressed = (len * bits + 7) / 8;         // :122
    return static_cast<float>(original) / static_cast<float>(compressed);
}

size_t dllm_packed_bytes(size_t n, uint8_t bits) { return (n * bits + 7) / 8; }

int dllm_pack(const uint8_t *codes, size_t n, uint8_t bits, uint8_t *packed, dllm_stream_t stream) {
    if (bits < 1 || bits > 8) return fail(DLLM_ERR_INVALID_PARAMS, "bits must be in 1..=8");
    if (!n) return DLLM_OK;
    pack_kernel<<<octet_grid(n), kBlock, 0, as_stream(stream)>>>(codes, n, bits, packed, aligned(codes, 8),
                                                                 aligned(packed, 8));
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_unpack(const uint8_t *packed, size_t n, uint8_t bits, uint8_t *codes, dllm_stream_t stream) {
    if (bits < 1 || bits > 8) return fail(DLLM_ERR_INVALID_PARAMS, "bits must be in 1..=8");
    if (!n) return DLLM_OK;
    unpack_kernel<<<octet_grid(n), kBlock, 0, as_stream(stream)>>>(packed, n, bits, codes, aligned(packed, 8),
                                                                   aligned(codes, 8));
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_default_quantize(const float *x, size_t n, int qtype, float scale, int32_t zero_point, uint8_t *out,
                          dllm_stream_t stream) {
    float lo, hi;
    switch (qtype) {   // quantize.rs:139-144
    case DLLM_QT_INT8: lo = -128.f; hi = 127.f; break;
    case DLLM_QT_INT4: lo = -8.f; hi = 7.f; break;
    case DLLM_QT_BINARY: lo = 0.f; hi = 1.f; break;
    case DLLM_QT_FLOAT8: lo = -127.f; hi = 127.f; break;
    default: return fail(DLLM_ERR_UNSUPPORTED, "unknown QuantizationType");
    }
    if (!n) return DLLM_OK;
    default_quantize_kernel<<<octet_grid(n), kBlock, 0, as_stream(stream)>>>(
        x, n, scale, static_cast<float>(zero_point), lo, hi, out, aligned(x, 16), aligned(out, 8));
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_default_dequantize(const uint8_t *q, size_t n, float scale, int32_t zero_point, float *out,
                            dllm_stream_t stream) {
    // quantize.rs:179-181 == quantization.rs:81-85 with zp = zero_point as f32.
    return dequant_common(q, n, 8, 0, nullptr, scale, static_cast<float>(zero_point), out, DLLM_F32, stream);
}

int dllm_calib_update(const float *x, size_t n, float *stats, uint64_t *histogram, size_t num_bins, void *workspace,
                      size_t workspace_bytes, dllm_stream_t stream) {
    if (!stats) return fail(DLLM_ERR_INVALID_PARAMS, "stats is null");
    if (!n) return DLLM_OK;
    const unsigned nblk = minmax_blocks(n);
    if (!workspace || workspace_bytes < sizeof(float2) * nblk)
        return fail(DLLM_ERR_INVALID_PARAMS, "workspace too small (see dllm_quantize_tensor_workspace)");
    hipStream_t st = as_stream(stream);
    float2 *partials = static_cast<float2 *>(workspace);
    int rc = launch_minmax(x, n, partials, nblk, st);
    if (rc) return rc;
    calib_fold_kernel<<<1, kBlock, 0, st>>>(partials, static_cast<int>(nblk), stats, 3.40282347e+38f);
    DLLM_LAUNCH_CHECK();
    if (num_bins && histogram) {
        if (num_bins > 0x7fffffff) return fail(DLLM_ERR_INVALID_PARAMS, "num_bins too large");
        const int use_lds = num_bins <= 16384;
        calib_hist_kernel<<<grid_for(n, kBlock, kCUs * 4), kBlock, use_lds ? num_bins * 4 : 0, st>>>(
            x, n, stats, reinterpret_cast<unsigned long long *>(histogram), static_cast<int>(num_bins), use_lds);
        DLLM_LAUNCH_CHECK();
    }
    return DLLM_OK;
}

int dllm_adaptive_update(const float *x, size_t n, float *stats, void *workspace, size_t workspace_bytes,
                         dllm_stream_t stream) {
    if (!stats || (n && !x)) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    if (!n) return DLLM_OK;
    const unsigned nblk = minmax_blocks(n);
    if (!workspace || workspace_bytes < sizeof(float2) * nblk)
        return fail(DLLM_ERR_INVALID_PARAMS, "workspace too small (see dllm_quantize_tensor_workspace)");
    hipStream_t st = as_stream(stream);
    float2 *partials = static_cast<float2 *>(workspace);
    int rc = launch_minmax(x, n, partials, nblk, st);
    if (rc) return rc;
    calib_fold_kernel<<<1, kBlock, 0, st>>>(partials, static_cast<int>(nblk), stats, INFINITY);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_adaptive_compute_params(const float *stats, int has_samples, uint32_t bits, float *params,
                                 dllm_stream_t stream) {
    if (bits > 31) return fail(DLLM_ERR_INVALID_PARAMS, "1u32 << bits overflows");
    if (!params || (has_samples && !stats)) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    adaptive_params_kernel<<<1, 64, 0, as_stream(stream)>>>(stats, has_samples ? 1 : 0, bits, params);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_adaptive_quantize(const float *x, size_t n, uint32_t bits, const float *params, int packed, uint8_t *out,
                           dllm_stream_t stream) {
    if (bits > 31) return fail(DLLM_ERR_INVALID_PARAMS, "1u32 << bits overflows");
    if (packed && (bits < 1 || bits > 8)) return fail(DLLM_ERR_INVALID_PARAMS, "packed output needs 1 <= bits <= 8");
    if (!params || (n && (!x || !out))) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    if (!n) return DLLM_OK;
    hipStream_t st = as_stream(stream);
    if (bits >= 1 && bits <= 8) {
        // Same map as quantize_tensor (quantization.rs:61-64 == :225-230), hi = 2^bits - 1.
        quantize_tensor_kernel<<<octet_grid(n), kBlock, 0, st>>>(x, n, bits, packed, out, params, aligned(x, 16),
                                                                 aligned(out, 8));
    } else {
        const float qf = static_cast<float>(1u << bits) - 1.0f;
        const int hi = qf >= 2147483648.0f ? INT32_MAX : static_cast<int>(qf);   // `q_max as i32`
        adaptive_quantize_kernel<<<grid_for((n + 3) / 4, kBlock, kCUs * 16), kBlock, 0, st>>>(x, n, hi, params, out);
    }
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_calib_compute_params(float mn, float mx, size_t total_samples, uint8_t bits, int symmetric, float *scale,
                              int32_t *zero_point) {
    // quantization/src/calibrate.rs:72-110 (host scalar arithmetic, IEEE f32, no contraction).
    if (total_samples == 0) return fail(DLLM_ERR_CALIBRATION_REQUIRED, "Calibration data required");
    if (bits > 31) return fail(DLLM_ERR_INVALID_PARAMS, "2u32.pow(bits) overflows");
    volatile float num_levels = static_cast<float>(1u << bits);
    volatile float range = mx - mn;
    if (range <= 1.1920929e-07f) { *scale = 1.0f; *zero_point = 0; return DLLM_OK; }
    auto as_i32 = [](float f) -> int32_t {
        if (f != f) return 0;
        if (f >= 2147483648.0f) return INT32_MAX;
        if (f <= -2147483648.0f) return INT32_MIN;
        return static_cast<int32_t>(f);
    };
    if (symmetric) {
        volatile float ma = std::max(std::fabs(mx), std::fabs(mn));
        volatile float t = ma * 2.0f;
        volatile float s = t / (num_levels - 1.0f);
        *scale = s;
        *zero_point = as_i32(num_levels / 2.0f - 1.0f);
    } else {
        volatile float s = range / (num_levels - 1.0f);
        volatile float q = -mn / s;
        *scale = s;
        *zero_point = as_i32(std::round(static_cast<float>(q)));
    }
    return DLLM_OK;
}

int dllm_bit_quantize(const float *x, size_t n, uint32_t bits, float scale, float zero_point, uint8_t *out,
                      dllm_stream_t stream) {
    if (bits > 30) return fail(DLLM_ERR_INVALID_PARAMS, "(1 << bits) - 1 overflows i32");
    if (!n) return DLLM_OK;
    const float max_val = static_cast<float>((1 << bits) - 1);
    bit_quantize_kernel<<<octet_grid(n), kBlock, 0, as_stream(stream)>>>(x, n, scale, zero_point, max_val, out,
                                                                         aligned(x, 16), aligned(out, 8));
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_bit_dequantize(const uint8_t *q, size_t n, float scale, float zero_point, void *out, int out_dtype,
                        dllm_stream_t stream) {
    if (out_dtype != DLLM_F32 && out_dtype != DLLM_F16) return fail(DLLM_ERR_UNSUPPORTED, "out_dtype");
    if (!n) return DLLM_OK;
    bit_dequantize_kernel<<<octet_grid(n), kBlock, 0, as_stream(stream)>>>(q, n, scale, zero_point, out, out_dtype,
                                                                           aligned(q, 8), aligned(out, 16));
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_quantize_vectors(const float *x, size_t rows, size_t dim, const uint8_t *cfg_bits, size_t ncfg,
                          const uint8_t *req_bits, size_t nreq, uint8_t *out, uint8_t *out_bits,
                          dllm_stream_t stream) {
    if (nreq == 0 || rows == 0) return DLLM_OK;   // zip(cycle of empty) yields nothing (lib.rs:132)
    if (!req_bits || (ncfg && !cfg_bits)) return fail(DLLM_ERR_INVALID_PARAMS, "null config");
    // Validate every row's quantizer index first: the reference panics mid-loop on the first
    // out-of-bounds quantizers[bits/2] (lib.rs:133); we launch nothing in that case.
    for (size_t j = 0; j < nreq && j < rows; ++j) {
        const size_t qi = req_bits[j] / 2;
        if (qi >= ncfg) return fail(DLLM_ERR_INVALID_PARAMS, "index out of bounds: quantizers[bits / 2]");
        if (cfg_bits[qi] > 30 || req_bits[j] > 30) return fail(DLLM_ERR_INVALID_PARAMS, "shift overflow");
    }
    if (out_bits)
        for (size_t r = 0; r < rows; ++r) out_bits[r] = req_bits[r % nreq];
    const size_t ncycle = std::min(nreq, rows);
    hipStream_t st = as_stream(stream);
    const unsigned gx = grid_for(dim, kBlock, 64);
    // Rows are processed in chunks of kCycleMax cycle slots; for nreq <= kCycleMax one launch.
    if (ncycle <= static_cast<size_t>(kCycleMax)) {
        CycleTable tab{};
        for (size_t j = 0; j < ncycle; ++j) {
            const uint32_t cb = cfg_bits[req_bits[j] / 2];
            tab.scale[j] = 1.0f / static_cast<float>((1 << cb) - 1);          // lib.rs:106
            tab.max_val[j] = static_cast<float>((1 << req_bits[j]) - 1);       // lib.rs:41
        }
        for (size_t r0 = 0; r0 < rows; r0 += 65535) {
            const size_t nr = std::min<size_t>(65535, rows - r0);
            // Cycle position of row r0 + j is (r0 + j) % nreq; r0 is a multiple of 65535, so
            // rotate the table for this chunk.
            CycleTable rt{};
            for (size_t j = 0; j < ncycle; ++j) {
                const size_t s = (r0 + j) % nreq;
                rt.scale[j] = tab.scale[s]; rt.max_val[j] = tab.max_val[s];
            }
            quantize_rows_cycle_kernel<<<dim3(gx, nr), kBlock, 0, st>>>(x + r0 * dim, nr, dim,
                                                                      static_cast<int>(ncycle), rt, out + r0 * dim);
            DLLM_LAUNCH_CHECK();
        }
    } else {
        // Long cycles: one launch per row with that row's quantizer (rare configuration).
        for (size_t r = 0; r < rows; ++r) {
            const uint8_t b = req_bits[r % nreq];
            const uint32_t cb = cfg_bits[b / 2];
            const float scale = 1.0f / static_cast<float>((1 << cb) - 1);
            bit_quantize_kernel<<<grid_for((dim + 7) / 8, kBlock, 64), kBlock, 0, st>>>(
                x + r * dim, dim, scale, 0.0f, static_cast<float>((1 << b) - 1), out + r * dim, aligned(x + r * dim, 16),
                aligned(out + r * dim, 8));
            DLLM_LAUNCH_CHECK();
        }
    }
    return DLLM_OK;
}

int dllm_compress_vectors(const float *x, size_t rows, size_t dim, uint8_t bits, uint8_t *out, float *scales,
                          float *zps, dllm_stream_t stream) {
    if (bits > 31) return fail(DLLM_ERR_INVALID_PARAMS, "1u32 << bits overflows");
    if (!rows) return DLLM_OK;
    if (rows > 0x7fffffff) return fail(DLLM_ERR_INVALID_PARAMS, "too many rows");
    const float levels = static_cast<float>((1u << bits) - 1u);
    compress_rows_kernel<<<static_cast<unsigned>(rows), kBlock, 0, as_stream(stream)>>>(x, dim, levels, out, scales,
                                                                                        zps);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_decompress_vectors(const uint8_t *q, size_t rows, size_t dim, const float *scales, const float *zps,
                            float *out, dllm_stream_t stream) {
    if (!rows || !dim) return DLLM_OK;
    decompress_rows_kernel<<<grid_for(rows * dim, kBlock, kCUs * 16), kBlock, 0, as_stream(stream)>>>(
        q, rows, dim, scales, zps, out);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

// ---- quantize_tensor split at its reduction (a tensor sharded over ranks) -------
int dllm_tensor_extremes(const float *x, size_t n, float *stats, void *workspace, size_t workspace_bytes,
                         dllm_stream_t stream) {
    // The fold of quantization.rs:41-46 (NaN-ignoring max/min), into caller-seeded stats.
    return dllm_adaptive_update(x, n, stats, workspace, workspace_bytes, stream);
}

int dllm_quantize_params_from_extremes(const float *stats, uint8_t bits, float *params, dllm_stream_t stream) {
    if (bits < 1 || bits > 8) return fail(DLLM_ERR_INVALID_PARAMS, "Bits must be between 1 and 8");
    if (!stats || !params) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    params_from_extremes_kernel<<<1, 64, 0, as_stream(stream)>>>(stats, bits, params);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_quantize_tensor_pair_with_params(const float *x, size_t n, uint8_t bits_a, uint8_t bits_b, int packed,
                                          const float *params_a, const float *params_b, uint8_t *out_a, uint8_t *out_b,
                                          dllm_stream_t stream) {
    // quantization.rs:59-65 at two widths with given device params, one read of x (the head-sharded
    // KVCacheEntry::update: both copies from one all-reduced pair of extremes).
    if (bits_a < 1 || bits_a > 8 || bits_b < 1 || bits_b > 8)
        return fail(DLLM_ERR_INVALID_PARAMS, "Bits must be between 1 and 8");
    if (!params_a || !params_b || (n && (!x || !out_a || !out_b))) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    if (!aligned(x, 4)) return fail(DLLM_ERR_INVALID_PARAMS, "x must be 4-byte aligned");
    if (!n) return DLLM_OK;
    quantize_pair_kernel<<<octet_grid(n), kBlock, 0, as_stream(stream)>>>(x, n, bits_a, bits_b, packed, out_a, out_b,
                                                                          params_a, params_b, aligned(x, 16),
                                                                          aligned(out_a, 8), aligned(out_b, 8));
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_quantize_tensor_with_params(const float *x, size_t n, uint8_t bits, int packed, const float *params,
                                     uint8_t *out, dllm_stream_t stream) {
    if (bits < 1 || bits > 8) return fail(DLLM_ERR_INVALID_PARAMS, "Bits must be between 1 and 8");
    // quantization.rs:61-64 with the params of :49-56 (== the adaptive map for 1 <= bits <= 8).
    return dllm_adaptive_quantize(x, n, bits, params, packed, out, stream);
}

}  // extern "C"
