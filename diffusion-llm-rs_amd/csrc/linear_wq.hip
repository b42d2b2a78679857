// linear_wq.hip -- group-quantized linear layer for gfx950 (MI355X).
//
// Replaces SimpleDiffusionModel::forward = x.dot(W) + b (diffuse-llm-rs/src/lib.rs:806-813) with
// W quantized per (output column n, K-group g) by quantize_tensor (quantization.rs:38-68) and
// dequantized (quantization.rs:81-85) inside the GEMM.
//
// Device weight layout ("fragment-major", private to this file; canonical form is the packed
// [K][N] bitstream of include/dllm_quant.h, converted bit-exactly in both directions):
//   For the 32x32x16 f16 MFMA the A operand (W^ transposed: n on the lane) of lane l is
//   W^[k = 8*(l>>5) + j][n = l&31], j = 0..7.  Per (n-tile nt of 32 columns, k64 slab) the 64
//   lanes' codes for the slab's 4 k16-substeps are stored lane-major, `bits` 32-bit words per
//   lane: ((nt*(K/64) + k64)*64 + lane)*bits + w.  One wave therefore fetches a slab with one
//   fully coalesced dwordx4 (int4) / dwordx2 (int2) / 2x dwordx4 (int8) per lane.
//   Inside a word: pair P = w*(16/bits) + p (p = 0..16/bits-1) = (substep s = P/4, v = P%4)
//   holds fragment elements (2v, 2v+1) at bits [bits*p, ...) and [16 + bits*p, ...), so
//   ((word >> bits*p) & mask2) | 0x64006400 is the f16 pair (1024 + q_2v, 1024 + q_2v+1).
//   Per (group, column) one u32 `sz` = f16 pair {-(1024 + zp), f16(scale)}:
//   f16(q - zp) is exact (|q - zp| < 2048), then one f16 rounding of (q - zp) * f16(scale).
#include "linear_common.hpp"
#include "stamp.hpp"
#include "diffusion_rng.hpp"
#if DLLM_LAB
#include "dllm_quant_lab.h"   // the lab build's extra entry point
#endif

#ifndef DLLM_LAB
#define DLLM_LAB 0
#endif
// Horner-form exact GEMM: 1 = half of the reps are rescaled in the tail of the group's last stage
// (the next group's ratios travel with that stage), half at the head of the group's first stage.
#ifndef DLLM_EXACT_HORNER
#define DLLM_EXACT_HORNER 0
#endif
#ifndef DLLM_HORNER_SPLIT
#define DLLM_HORNER_SPLIT 0
#endif
// Horner form: 1 = the ratios travel only with a group's first stage (one LDS-DMA per two stages).
#ifndef DLLM_HORNER_HR_GF
#define DLLM_HORNER_HR_GF 0
#endif
#if DLLM_HORNER_HR_GF && DLLM_HORNER_SPLIT
#error "DLLM_HORNER_SPLIT reads the next group's ratios in every group's second stage"
#endif

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <map>
#include <tuple>
#include <cstring>
#include <mutex>
#include <new>
#include <type_traits>


struct dllm_linear {
    size_t K = 0, N = 0, Npad = 0, G = 0, group = 0;
    int bits = 0;
    int device = 0;
    int precision = DLLM_PRECISION_EXACT;
    uint32_t *wdev = nullptr;     // prefill layout (32x32x16 fragments)
    uint32_t *wdec = nullptr;     // decode layout (16x16x32 fragments)
    uint32_t *sz = nullptr;       // [G][Npad] f16 pairs {-(1024 + zp), f16(scale)}
    float *sf = nullptr;          // [G][Npad] f32 scales (exact-weight kernels; export), 0 in the padding
    float *bias = nullptr;        // [Npad]
    float *hr = nullptr;          // [G + 1][Npad] Horner ratios s_{g-1} / s_g (Horner-form shapes with valid scales)
    int hstate = 0;               // Horner form: 0 not applicable, 1 valid (hr kept), 2 not valid for these scales
    bool prefill_only = false;    // DLLM_LINEAR_PREFILL_ONLY: no decode layout; M <= 64 runs the prefill kernels
#if DLLM_LAB   // measurement knobs of the lab build (dllm_linear_set_kernel_variant)
    uint32_t *w16 = nullptr;      // 16x16x32 prefill layout (wq_gemm16_kernel)
    int variant = -1;             // prefill schedule variant (-1: product policy)
    int dlab = 0;                 // decode-kernel ablation mask
    int dcfg = 0;                 // decode (NT, nsplit) override
    int rlab = 0;                 // ring-kernel ablation mask
    int pplab = 0;                // ping-pong-kernel ablation mask
#endif
};

namespace dllm {
namespace {



inline size_t canon_words(size_t K, size_t N, int bits) { return (K * N * bits + 31) / 32; }

// ---------------------------------------------------------------------------------------------
// Weight quantization: one thread per (group g, column n).  Column reads are coalesced across
// the wave (consecutive n).  Codes go into the canonical bitstream by atomicOr (b | 32, so no
// code straddles a word); the buffer is zeroed first.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) quantize_weights_kernel(const float *__restrict__ W, size_t K, size_t N,
                                                               int bits, int group, uint32_t *__restrict__ canon,
                                                               float *__restrict__ scales,
                                                               uint8_t *__restrict__ zps) {
    const size_t n = blockIdx.x * static_cast<size_t>(256) + threadIdx.x;
    const size_t g = blockIdx.y;
    if (n >= N) return;
    const size_t k0 = g * group;
    const size_t len = std::min<size_t>(group, K - k0);
    float mx = -INFINITY, mn = INFINITY;                      // quantization.rs:41-46
    for (size_t k = 0; k < len; ++k) { float v = W[(k0 + k) * N + n]; mx = fmaxf(mx, v); mn = fminf(mn, v); }
    const float q_max = static_cast<float>(1u << bits) - 1.0f;
    float scale = (mx - mn) / (q_max - 0.0f);                 // :52
    if (scale == 0.0f) scale = 1.0f;                          // :53
    const float zpf = 0.0f - mn / scale;                      // :55
    const uint32_t zp = rs_as_u8(roundf(rs_clamp(zpf, 0.0f, q_max)));   // :56
    const float zpf32 = static_cast<float>(zp);
    scales[g * N + n] = scale;
    zps[g * N + n] = static_cast<uint8_t>(zp);
    const int hi = (1 << bits) - 1;
    for (size_t k = 0; k < len; ++k) {                        // :59-65
        float t = W[(k0 + k) * N + n] / scale;
        t = t + zpf32;
        const uint32_t q = rs_round_i32_clamp(t, hi);
        const size_t bit = ((k0 + k) * N + n) * bits;
        if (q) atomicOr(&canon[bit >> 5], q << (bit & 31));
    }
}

// Same results as quantize_weights_kernel without its per-code atomics (N % 4 == 0, group <= 128):
// lane = 16 r + c of a wave owns column quad c (4 columns, one float4 per row) and rows
// [32 r, 32 r + 32) of the group, held in registers between the two passes; the group's extremes
// (order-independent NaN-ignoring folds, so identical to the serial fold) are combined across the
// 4 row quarters by two xor-shuffles, and each lane writes whole canonical bytes (4 codes of a row).
__global__ void __launch_bounds__(256) quantize_weights4_kernel(const float *__restrict__ W, size_t K, size_t N,
                                                                int bits, int group, uint32_t *__restrict__ canon,
                                                                float *__restrict__ scales,
                                                                uint8_t *__restrict__ zps) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t n = (static_cast<size_t>(blockIdx.x) * 4 + wave) * 64 + 4 * (lane & 15);
    const size_t g = blockIdx.y;
    const size_t k0 = g * group;
    const int len = static_cast<int>(std::min<size_t>(group, K - k0));
    const int r0 = 32 * (lane >> 4);
    const bool col_ok = n < N;
    float4 v[32];
    float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, mn[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const bool ok = col_ok && r0 + i < len;
        v[i] = ok ? *reinterpret_cast<const float4 *>(W + (k0 + r0 + i) * N + n) : make_float4(NAN, NAN, NAN, NAN);
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) {                              // quantization.rs:41-46
        mx[0] = fmaxf(mx[0], v[i].x); mn[0] = fminf(mn[0], v[i].x);
        mx[1] = fmaxf(mx[1], v[i].y); mn[1] = fminf(mn[1], v[i].y);
        mx[2] = fmaxf(mx[2], v[i].z); mn[2] = fminf(mn[2], v[i].z);
        mx[3] = fmaxf(mx[3], v[i].w); mn[3] = fminf(mn[3], v[i].w);
    }
    float scale[4], zpf32[4];
    const float q_max = static_cast<float>(1u << bits) - 1.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        mx[j] = fmaxf(mx[j], __shfl_xor(mx[j], 16, 64));
        mx[j] = fmaxf(mx[j], __shfl_xor(mx[j], 32, 64));
        mn[j] = fminf(mn[j], __shfl_xor(mn[j], 16, 64));
        mn[j] = fminf(mn[j], __shfl_xor(mn[j], 32, 64));
        float sc = (mx[j] - mn[j]) / (q_max - 0.0f);            // :52
        if (sc == 0.0f) sc = 1.0f;                              // :53
        const float zpf = 0.0f - mn[j] / sc;                    // :55
        const uint32_t zp = rs_as_u8(roundf(rs_clamp(zpf, 0.0f, q_max)));   // :56
        scale[j] = sc;
        zpf32[j] = static_cast<float>(zp);
    }
    if (!col_ok) return;
    if (r0 == 0) {
        *reinterpret_cast<float4 *>(scales + g * N + n) = make_float4(scale[0], scale[1], scale[2], scale[3]);
        const uint32_t zq = static_cast<uint32_t>(zpf32[0]) | (static_cast<uint32_t>(zpf32[1]) << 8) |
                            (static_cast<uint32_t>(zpf32[2]) << 16) | (static_cast<uint32_t>(zpf32[3]) << 24);
        *reinterpret_cast<uint32_t *>(zps + g * N + n) = zq;
    }
    const int hi = (1 << bits) - 1;
    uint8_t *cb = reinterpret_cast<uint8_t *>(canon);
#pragma unroll
    for (int i = 0; i < 32; ++i) {                              // :59-65
        if (r0 + i >= len) continue;
        const float e[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float t = e[j] / scale[j];
            t = t + zpf32[j];
            w |= rs_round_i32_clamp(t, hi) << (j * bits);
        }
        const size_t byte = ((k0 + r0 + i) * N + n) * bits / 8;
        if (bits == 2) cb[byte] = static_cast<uint8_t>(w);
        else if (bits == 4) *reinterpret_cast<uint16_t *>(cb + byte) = static_cast<uint16_t>(w);
        else *reinterpret_cast<uint32_t *>(cb + byte) = w;
    }
}

__device__ __forceinline__ uint32_t canon_code(const uint32_t *__restrict__ canon, size_t k, size_t n, size_t N,
                                               int bits) {
    const size_t bit = (k * N + n) * bits;
    return (canon[bit >> 5] >> (bit & 31)) & ((1u << bits) - 1u);
}

// Canonical -> fragment-major.  One thread per (column n < Npad, k64 slab); pad columns get 0.
__global__ void __launch_bounds__(256) build_fragments_kernel(const uint32_t *__restrict__ canon, size_t K, size_t N,
                                                              size_t Npad, int bits, uint32_t *__restrict__ wdev) {
    const size_t n = blockIdx.x * static_cast<size_t>(256) + threadIdx.x;
    const size_t kt = blockIdx.y;
    if (n >= Npad) return;
    const size_t nk = K / 64, nt = n >> 5;
    const int pairs_per_word = 16 / bits;
    for (int h = 0; h < 2; ++h) {
        const size_t lane = (n & 31) + 32 * h;
        uint32_t *dst = wdev + ((nt * nk + kt) * 64 + lane) * bits;
        for (int w = 0; w < bits; ++w) {
            uint32_t word = 0;
            for (int p = 0; p < pairs_per_word; ++p) {
                const int P = w * pairs_per_word + p, s = P >> 2, v = P & 3;
                const size_t k = kt * 64 + s * 16 + 8 * h + 2 * v;
                uint32_t lo = 0, hi = 0;
                if (n < N) { lo = canon_code(canon, k, n, N, bits); hi = canon_code(canon, k + 1, n, N, bits); }
                word |= (lo << (bits * p)) | (hi << (16 + bits * p));
            }
            dst[w] = word;
        }
    }
}

#if DLLM_LAB   // the 16x16x32 prefill weight layout (lab variants 8, 11)
#include "lab/wq_fragments16.inc"
#endif

// Code (k, n) from the fragment-major (prefill) layout: lane (n & 31) + 32 ((k % 16) / 8) of the
// (n / 32, k / 64) slab, pair P = 4 ((k % 64) / 16) + (k % 8) / 2, bit bits (P % (16/bits)) + 16 (k & 1).
__device__ __forceinline__ uint32_t wdev_code(const uint32_t *__restrict__ wdev, size_t k, size_t n, size_t nk,
                                              int bits) {
    const size_t ppw = 16 / bits, kk = k % 64, lane = (n & 31) + 32 * ((kk % 16) / 8);
    const size_t P = 4 * (kk / 16) + (kk % 8) / 2;
    const uint32_t word = wdev[(((n >> 5) * nk + k / 64) * 64 + lane) * bits + P / ppw];
    return (word >> (bits * (P % ppw) + 16 * (k & 1))) & ((1u << bits) - 1u);
}

// Prefill layout -> decode layout, the second weight layout, built lazily by the first decode-shaped
// call.  Word w of lane (n & 15) + 16 o in the (n / 16, 128-deep slab) tile holds 16/bits code pairs
// (k, k + 1), k = slab 128 + 32 (P / 4) + 8 o + 2 (P % 4).  One thread per (column n < Npad, slab).
__global__ void __launch_bounds__(256) build_decode_from_wdev_kernel(const uint32_t *__restrict__ wdev, size_t K,
                                                                     size_t Npad, int bits, uint32_t *__restrict__ wdec) {
    const size_t n = blockIdx.x * static_cast<size_t>(256) + threadIdx.x;
    const size_t slab = blockIdx.y;
    if (n >= Npad) return;
    const size_t nk = K / 64, nslab = (K + 127) / 128, nt = n >> 4;
    const int pairs_per_word = 16 / bits;
    for (int o = 0; o < 4; ++o) {
        const size_t lane = (n & 15) + 16 * o;
        uint32_t *dst = wdec + ((nt * nslab + slab) * 64 + lane) * bits;
        for (int w = 0; w < bits; ++w) {
            uint32_t word = 0;
            for (int p = 0; p < pairs_per_word; ++p) {
                const int P = w * pairs_per_word + p, t = P >> 2, v = P & 3;
                const size_t k = slab * 128 + t * 32 + 8 * o + 2 * v;
                uint32_t lo = 0, hi = 0;
                if (k < K) { lo = wdev_code(wdev, k, n, nk, bits); hi = wdev_code(wdev, k + 1, n, nk, bits); }
                word |= (lo << (bits * p)) | (hi << (16 + bits * p));
            }
            dst[w] = word;
        }
    }
}

// Export of the per-(group, column) parameters from the device copies: scale = sf (f32, exact),
// zp = -(1024 + zp) of the sz pair's low half (exact in f16).
__global__ void __launch_bounds__(256) export_params_kernel(const float *__restrict__ sf, const uint32_t *__restrict__ sz,
                                                            size_t G, size_t N, size_t Npad, float *__restrict__ scales,
                                                            uint8_t *__restrict__ zps) {
    const size_t n = blockIdx.x * static_cast<size_t>(256) + threadIdx.x;
    const size_t g = blockIdx.y;
    if (n >= N) return;
    if (scales) scales[g * N + n] = sf[g * Npad + n];
    if (zps) {
        const _Float16 nz = __builtin_bit_cast(_Float16, static_cast<uint16_t>(sz[g * Npad + n] & 0xFFFFu));
        zps[g * N + n] = static_cast<uint8_t>(-static_cast<float>(nz) - 1024.0f);
    }
}

// Fragment-major (prefill layout) -> canonical packed bytes: one thread per output byte; code
// (k, n) sits in wdev word ((n/32 * K/64 + k/64) * 64 + lane) * bits + P / (16/bits), lane =
// (n & 31) + 32 ((k % 16) / 8), pair P = 4 ((k % 64) / 16) + (k % 8) / 2, at bit
// bits (P % (16/bits)) + 16 (k & 1).  Inverse of build_fragments_kernel (export round trip test).
__global__ void __launch_bounds__(256) export_codes_kernel(const uint32_t *__restrict__ wdev, size_t K, size_t N,
                                                           int bits, uint8_t *__restrict__ out, size_t nbytes) {
    const size_t nk = K / 64, per_byte = 8 / bits;
    for (size_t B = blockIdx.x * static_cast<size_t>(256) + threadIdx.x; B < nbytes;
         B += static_cast<size_t>(gridDim.x) * 256) {
        uint32_t byte = 0;
        for (size_t e = 0; e < per_byte; ++e) {
            const size_t i = B * per_byte + e;
            if (i >= K * N) break;
            byte |= wdev_code(wdev, i / N, i % N, nk, bits) << (bits * e);
        }
        out[B] = static_cast<uint8_t>(byte);
    }
}

__global__ void __launch_bounds__(256) build_sz_kernel(const float *__restrict__ scales, const uint8_t *__restrict__ zps,
                                                       size_t G, size_t N, size_t Npad, uint32_t *__restrict__ sz) {
    const size_t n = blockIdx.x * static_cast<size_t>(256) + threadIdx.x;
    const size_t g = blockIdx.y;
    if (n >= Npad) return;
    float s = 0.0f, nz = -1024.0f;
    if (n < N) { s = scales[g * N + n]; nz = -(1024.0f + static_cast<float>(zps[g * N + n])); }
    union { _Float16 h[2]; uint32_t u; } pk;
    pk.h[0] = static_cast<_Float16>(nz);   // exact (integer < 2048)
    pk.h[1] = static_cast<_Float16>(s);    // RNE
    sz[g * Npad + n] = pk.u;
}

__global__ void __launch_bounds__(256) build_sf_kernel(const float *__restrict__ scales, size_t G, size_t N,
                                                       size_t Npad, float *__restrict__ sf) {
    const size_t n = blockIdx.x * static_cast<size_t>(256) + threadIdx.x;
    const size_t g = blockIdx.y;
    if (n < Npad) sf[g * Npad + n] = n < N ? scales[g * N + n] : 0.0f;
}

// Horner ratios hr[g][n] = s_{g-1} / s_g (hr[0][n] = 1; padding columns 1) for the HORNER GEMM, and
// *unsafe = 1 when some column's scales are not all finite normal f32 or span more than 2^64 (the
// rescaled accumulator could overflow or lose its exponent range there).
__global__ void __launch_bounds__(256) build_horner_kernel(const float *__restrict__ sf, size_t G, size_t N,
                                                           size_t Npad, float *__restrict__ hr, int *__restrict__ unsafe) {
    const size_t n = blockIdx.x * static_cast<size_t>(256) + threadIdx.x;
    if (n >= Npad) return;
    float mn = __builtin_inff(), mx = 0.0f, prev = 1.0f;
    bool bad = false;
    for (size_t g = 0; g < G; ++g) {
        const float s = n < N ? sf[g * Npad + n] : 1.0f;
        bad |= !(s >= 1.17549435e-38f && s <= 3.40282347e+38f);
        mn = fminf(mn, s);
        mx = fmaxf(mx, s);
        hr[g * Npad + n] = g ? prev / s : 1.0f;
        prev = s;
    }
    hr[G * Npad + n] = 1.0f;   // past the last group (read by the split schedule's last stage)
    if (bad || mx > mn * 0x1p64f) atomicOr(unsafe, 1);
}

__global__ void __launch_bounds__(256) cast_f32_f16_kernel(const float *__restrict__ x, size_t n,
                                                           __half *__restrict__ y) {
    const size_t n4 = n / 4;
    const size_t stride = static_cast<size_t>(gridDim.x) * 256;
    for (size_t i = blockIdx.x * static_cast<size_t>(256) + threadIdx.x; i < n4; i += stride) {
        float4 v = reinterpret_cast<const float4 *>(x)[i];
        union { __half h[4]; uint2 u; } pk;
        pk.h[0] = __float2half_rn(v.x); pk.h[1] = __float2half_rn(v.y);
        pk.h[2] = __float2half_rn(v.z); pk.h[3] = __float2half_rn(v.w);
        reinterpret_cast<uint2 *>(y)[i] = pk.u;
    }
    for (size_t i = n4 * 4 + blockIdx.x * static_cast<size_t>(256) + threadIdx.x; i < n; i += stride)
        y[i] = __float2half_rn(x[i]);
}

// The epilogue of a reduced row-parallel partial (dllm_bias_cast): out[m][n] = y[m][n] + bias[n]
// (f32 add, the reference's `+ &self.bias` after the dot, lib.rs:812), stored in f32 or RNE f16.
template <typename YT>
__global__ void __launch_bounds__(256) bias_cast_kernel(const float *__restrict__ y, size_t M, size_t N,
                                                        const float *__restrict__ bias, YT *__restrict__ out,
                                                        int vec) {
    const size_t stride = static_cast<size_t>(gridDim.x) * 256;
    const size_t t0 = blockIdx.x * static_cast<size_t>(256) + threadIdx.x;
    if (vec) {   // N % 4 == 0 and 16-B aligned rows: 4 outputs per thread
        const size_t q = N / 4, total = M * q;
        for (size_t i = t0; i < total; i += stride) {
            const size_t n = (i % q) * 4;
            const float4 v = reinterpret_cast<const float4 *>(y)[i];
            const float4 b = bias ? *reinterpret_cast<const float4 *>(bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
            store4<YT>(out + i * 4, v.x + b.x, v.y + b.y, v.z + b.z, v.w + b.w);
        }
        return;
    }
    for (size_t i = t0; i < M * N; i += stride) store1<YT>(out + i, y[i] + (bias ? bias[i % N] : 0.0f));
}

// Row coefficient table: out[m] = coef[m / rps] (3 floats each).
__global__ void __launch_bounds__(256) expand_coef_kernel(const float *__restrict__ coef, size_t M, size_t rps,
                                                          float *__restrict__ out) {
    for (size_t m = blockIdx.x * static_cast<size_t>(256) + threadIdx.x; m < M; m += static_cast<size_t>(gridDim.x) * 256) {
        const float *c = coef + 3 * (m / rps);
        out[3 * m] = c[0];
        out[3 * m + 1] = c[1];
        out[3 * m + 2] = c[2];
    }
}

// Loads a lane's BITS weight words (one 16-B or 8-B vector).
template <int BITS>
__device__ __forceinline__ void load_words(uint32_t (&w)[BITS], const uint32_t *__restrict__ p) {
    if constexpr (BITS == 4) {
        uint4 v = *reinterpret_cast<const uint4 *>(p);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else if constexpr (BITS == 2) {
        uint2 v = *reinterpret_cast<const uint2 *>(p);
        w[0] = v.x; w[1] = v.y;
    } else {
        uint4 a = *reinterpret_cast<const uint4 *>(p), b = *reinterpret_cast<const uint4 *>(p + 4);
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
        w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    }
}

#if DLLM_LAB   // the round-1 prefill GEMM schedules (lab variants 0-3)
#include "lab/wq_gemm_round1.inc"
#endif

// ---------------------------------------------------------------------------------------------
// Big-tile prefill GEMM (used when it still fills the chip): block tile 256 (m) x 256 (n), 8 waves
// side by side in n (wave tile 256 x 32 as above), so each X tile is shared by 8 waves (half the
// LDS-DMA per FLOP of the 128-column tile).  Three LDS stages in a ring: stage kt+2 is issued
// while kt is computed, the end-of-step wait is a COUNTED vmcnt that leaves kt+2's DMAs in flight
// across the raw s_barrier (never __syncthreads, whose fence would drain them).
// ---------------------------------------------------------------------------------------------
// Ring GEMM: block tile (32 MR) x (32 NW), NW*KG waves.  Wave (cw, kg) = (wave % NW, wave / NW)
// owns output columns n0 + 32 cw .. +32 for all 32 MR rows and, of every 64-deep k-step, the
// 4/KG substeps kg*4/KG ..: KG = 2 puts two waves on each SIMD at the same tile count (the 128-row
// tiles of mid-M shapes run one block per CU), their two accumulators summed through the stage
// LDS at the end (fixed order).  SPLIT: as wq_gemm_kernel (slab partial, no bias).
//
// HORNER (exact weights, group 128, KG = 1, no K split): the MFMA A operand is the exact integer
// q - zp (dequant_exact) and the f32 group scales enter in Horner form.  With r_g = s_{g-1} / s_g
// (hr[g][n], f32; r_0 = 1) the accumulator is rescaled at the head of every group,
//   acc <- acc * r_g + T_g   (T_g = the group's MFMA sum),
// so after the last group G-1 acc = sum_g T_g s_g / s_{G-1}, and the epilogue multiplies by
// s_{G-1} (sf).  Each term carries at most G f32 roundings of its ratio product (relative
// <= G 2^-24).  There is no transient per-group accumulator (the fold form needs one beside acc),
// so the 256 x 256 tile fits at two waves per SIMD.  Valid only where every scale is a finite
// normal f32 and max_g s / min_g s <= 2^64 per column (build_horner_kernel decides per handle).
template <int BITS, typename YT, int NW = 8, int MR = kMReps, bool SPLIT = false, int KG = 1, int LAB = 0,
          int EPI = 0, bool HORNER = false>
__global__ void __launch_bounds__(NW * KG * 64, (NW * KG == 8 || MR == 8) ? 1 : 2)
wq_gemm8_kernel(const __half *__restrict__ X, int M, int K, const uint32_t *__restrict__ wdev,
                const uint32_t *__restrict__ sz, const float *__restrict__ bias, YT *__restrict__ Y, int N, int Npad,
                int group, int nbm, int nbn, int nsplit = 1, float *__restrict__ ws = nullptr,
                PSampleEpi epi = PSampleEpi{}, const float *__restrict__ hr = nullptr,
                const float *__restrict__ sf = nullptr) {
    using SL = StageLayout8<BITS, NW, MR, KG>;
    constexpr int kBMt = 32 * MR, kBNt = 32 * NW, kWT = NW * KG, kSub = 4 / KG;
    static_assert(SL::kXRounds >= 1 && 4 * MR % kWT == 0, "X staging must split evenly over the waves");
    static_assert(!HORNER || (KG == 1 && !SPLIT && NW == 8 && LAB == 0), "Horner form: one k-group, whole K");
    // HORNER: the group's ratios r_g (256 columns f32) follow the scale dwords in every stage.
    constexpr int kHR = SL::kBytes, kStBytes = SL::kBytes + (HORNER ? 1024 : 0);
    __shared__ __attribute__((aligned(16))) uint8_t st0[kStBytes];
    __shared__ __attribute__((aligned(16))) uint8_t st1[kStBytes];
    __shared__ __attribute__((aligned(16))) uint8_t st2[kStBytes];

    // K-slice outermost, so the blocks an XCD holds share the slice's X rows in its L2.
    const int nb = nbm * nbn * nsplit, orig = blockIdx.x;
    const int xcd = orig % kXCDs, q8 = nb / kXCDs, r8 = nb % kXCDs;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / kXCDs;
    const int ks = wgid / (nbm * nbn), tile = wgid % (nbm * nbn);
    const int bm = tile / nbn, bn = tile % nbn;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cw = wave % NW, kg = wave / NW;
    const int m0 = bm * kBMt, n0 = bn * kBNt;
    const unsigned nk_all = static_cast<unsigned>(K) / kBK;
    const unsigned nk = nk_all / static_cast<unsigned>(nsplit);   // k-steps of this K slice
    const unsigned kt0 = static_cast<unsigned>(ks) * nk;
    const unsigned kpg = static_cast<unsigned>(group) / kBK;
    const unsigned nt = static_cast<unsigned>(n0 + cw * 32) >> 5;

    // X: kXRounds rounds of kWT KiB (kWT waves x 64 lanes x 16 B); round i, wave w covers rows
    // 8 (kWT i + w) .. +8.
    const int chunk_st = lane & 7;
    const __half *xsrc[SL::kXRounds];
#pragma unroll
    for (int i = 0; i < SL::kXRounds; ++i) {
        const int row = (i * kWT + wave) * 8 + (lane >> 3);
        int grow = m0 + row;
        grow = grow < M ? grow : M - 1;
        const int c = chunk_st ^ ((row >> 1) & 7);
        xsrc[i] = X + static_cast<size_t>(grow) * K + c * 8;
    }
    const uint32_t *wsrc = wdev + (static_cast<size_t>(nt) * nk_all * 64 + lane) * BITS;
    // Scales: one 16-B LDS-DMA per block per k-step (wave szw; 4 columns per lane) instead of one
    // 256-B DMA per wave: each LDS-DMA costs its wave ~60-185 issue cycles whatever its size.
    const int szw = KG == 1 ? 0 : NW;
    const bool has_w = KG == 1 || kg == 0, has_sz = wave == szw, has_hr = HORNER && wave == 1;
    const uint32_t *szsrc = sz + n0 + 4 * (lane & (8 * NW - 1));
    const float *hrsrc = HORNER ? hr + n0 + 4 * lane : nullptr;

    const uint32_t wv = static_cast<uint32_t>(wave), cwv = static_cast<uint32_t>(cw);
    // A stage is kXRounds + 2 pieces: X rounds, the weight words, the scale dword (pieces a wave
    // does not own under KG = 2 are empty), issued as one burst at the top of a k-step.  Spreading
    // the pieces over the substeps (to hide each DMA's issue cost) measured slower: the later
    // issue shortens the landing slack before the counted wait two steps on.  HORNER: + the
    // group's ratios (wave 1).
    constexpr int kPieces = SL::kXRounds + 2 + (HORNER ? 1 : 0);
    auto piece = [&](uint8_t *sb, unsigned kt, int p, bool with_hr) {
        const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(sb));
        kt += kt0;
        if (p < SL::kXRounds) {
            if constexpr (!(LAB & 1)) glds16_asm(xsrc[p] + kt * kBK, base + wv * 1024 + p * kWT * 1024);
            return;
        }
        if constexpr (LAB & 2) return;
        if (p == SL::kXRounds) {
            if (has_w) {
                const uint32_t *wp = wsrc + static_cast<size_t>(kt) * 64 * BITS;
                const uint32_t wb = base + SL::kX + cwv * (64 * BITS * 4);
                if constexpr (BITS == 4) {
                    glds16_asm(wp, wb);
                } else if constexpr (BITS == 8) {
                    glds16_asm(wp, wb);
                    glds16_asm(wp + 4, wb + 64 * 16);
                } else {
                    glds4_asm(wp, wb);
                    glds4_asm(wp + 1, wb + 256);
                }
            }
        } else if (p == SL::kXRounds + 1) {
            if (has_sz) glds16_asm(szsrc + (kt / kpg) * Npad, base + SL::kX + SL::kW);
        } else if (has_hr && with_hr) {
            // SPLIT: a group's second stage carries the NEXT group's ratios (row G = 1 after the last)
            glds16_asm(hrsrc + (kt / kpg + (DLLM_HORNER_SPLIT ? (kt & 1) : 0)) * Npad, base + kHR);
        }
    };
    // with_hr (DLLM_HORNER_HR_GF): the stage opens a group, so its ratios travel with it
    auto stage = [&](uint8_t *sb, unsigned kt, bool with_hr = true) {
#pragma unroll
        for (int p = 0; p < kPieces; ++p) piece(sb, kt, p, with_hr);
    };
    // Counted wait leaving the newest stage's DMAs (this wave's own count) in flight.
    auto wait_prev = [&](bool newest_hr = true) {
        if (has_w && (has_sz || (has_hr && newest_hr))) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SL::kXRounds + SL::kWOps + 1) : "memory");
        else if (has_w) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SL::kXRounds + SL::kWOps) : "memory");
        else if (has_sz) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SL::kXRounds + 1) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SL::kXRounds) : "memory");
    };

    float16_t acc[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[r][e] = 0.0f;

    const int hsel = lane >> 5;
    const int rowx = ((lane & 31) >> 1) & 7;
    // This wave's substeps: kg * kSub + j, j < kSub (fragment offsets selected once, uniform).
    int soff[kSub];
#pragma unroll
    for (int j = 0; j < kSub; ++j) {
        const int s = kg * kSub + j;
        soff[j] = (lane & 31) * (kBK * 2) + ((((2 * s + hsel) ^ rowx)) << 4);
    }

    half8_t bconst = half8_t{(_Float16)lane, 1, 1, 1, 1, 1, 1, (_Float16)wave};
    asm volatile("" : "+v"(bconst));
    auto read_b = [&](half8_t (&b)[MR], const uint8_t *sb, int j) {
        if constexpr (LAB & 8) {   // measurement only: loop-invariant B fragments, no LDS reads
#pragma unroll
            for (int r = 0; r < MR; ++r) b[r] = bconst;
            return;
        }
#pragma unroll
        for (int r = 0; r < MR; ++r) b[r] = *reinterpret_cast<const half8_t *>(sb + soff[j] + r * 32 * kBK * 2);
    };
    auto mfma8 = [&](const half8_t &a, const half8_t (&b)[MR]) {
#pragma unroll
        for (int r = 0; r < MR; ++r) acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b[r], acc[r], 0, 0, 0);
    };
    // Compute stage `sb`; stage `pf` receives k-step kt+2.  gf_tag (HORNER): the stage opens a group.
    auto step = [&](const uint8_t *sb, uint8_t *pf, unsigned kt, auto gf_tag) {
        constexpr bool GF = HORNER && decltype(gf_tag)::value;
        const bool issue = kt + 2 < nk;
        if (!(LAB & 32) && issue) stage(pf, kt + 2, !DLLM_HORNER_HR_GF || GF);   // kt + 2 has kt's group phase
        if constexpr (LAB & 4) {   // measurement only: the ring and its waits without any compute
            if (issue) wait_prev();
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            return;
        }
        uint32_t w[BITS];
        lds_words<BITS>(w, sb + SL::kX + cw * (64 * BITS * 4), lane);
        if constexpr (KG == 2) {
            // Substeps 2 kg + j of the slab words = substeps j of the words shifted by kg * BITS/2.
#pragma unroll
            for (int i = 0; i < BITS / 2; ++i) w[i] = kg ? w[BITS / 2 + i] : w[i];
        }
        half2_t nz, sc;
        split_sz(*reinterpret_cast<const uint32_t *>(sb + SL::kX + SL::kW + (cw * 32 + (lane & 31)) * 4), nz, sc);
        // HORNER: exact integer fragments; at a group's head the lane's 16 column ratios
        // (columns 4 hsel + 8 qd + (0..3) of the wave's 32, as the accumulator registers).
        ExactConsts ec;
        float4 r4[4];
        if constexpr (HORNER) ec = exact_consts(nz);
        if constexpr (GF || (HORNER && DLLM_HORNER_SPLIT)) {
            const float *rl = reinterpret_cast<const float *>(sb + kHR) + cw * 32 + 4 * hsel;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) r4[qd] = *reinterpret_cast<const float4 *>(rl + 8 * qd);
        }
        auto deq = [&](int j) {
            if constexpr (HORNER) return dequant_exact<BITS>(w, j, ec);
            else return dequant_frag<BITS>(w, j, nz, sc);
        };
        half8_t bA[MR], bB[MR];
        read_b(bA, sb, 0);
        if constexpr (LAB & 32) {   // measurement: head-of-step LDS reads drained before the DMAs issue
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (issue) stage(pf, kt + 2);
        }
        half8_t aA = deq(0), aB;
        constexpr int kRH = (HORNER && DLLM_HORNER_SPLIT) ? MR / 2 : MR;   // reps rescaled at the group's head
        auto rescale = [&](int r) {
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                acc[r][4 * qd + 0] *= r4[qd].x;
                acc[r][4 * qd + 1] *= r4[qd].y;
                acc[r][4 * qd + 2] *= r4[qd].z;
                acc[r][4 * qd + 3] *= r4[qd].w;
            }
        };
        auto sub = [&](half8_t (&bc)[MR], half8_t (&bn)[MR], const half8_t &ac, half8_t &an, int j) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
            if (j < kSub - 1) {
                read_b(bn, sb, j + 1);
                an = deq(j + 1);
            }
            if (GF && j == 0) {
                // acc <- acc * r_g right before the group's first MFMA of each rep; scalar v_mul_f32
                // (the file is built without the SLP vectorizer: v_pk_mul_f32 costs far more beside
                // MFMAs, MI355X_MICROARCH.md filler prices)
#pragma unroll
                for (int r = 0; r < MR; ++r) {
                    if (r < kRH) rescale(r);
                    acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ac, bc[r], acc[r], 0, 0, 0);
                }
                // rep i + 1's rescale issues beside rep i's MFMA (one rep of slack before its use)
                __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
#pragma unroll
                for (int i = 0; i < MR; ++i) {
                    if (i + 1 < kRH) __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // MFMA rep i
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, kRH < MR ? 2 : 1, 0);
                }
            } else if (HORNER && kRH < MR && !GF && j == kSub - 1) {
                // the group's last substep: reps kRH.. take the next group's ratio after their last
                // MFMA of this group (rep r's rescale beside rep r + 2's MFMA)
                mfma8(ac, bc);
#pragma unroll
                for (int r = kRH; r < MR; ++r) rescale(r);
#pragma unroll
                for (int i = 0; i < MR; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    if (i >= kRH + 2) __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
                }
            } else {
                mfma8(ac, bc);
#pragma unroll
                for (int i = 0; i < MR; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                }
            }
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
        };
        sub(bA, bB, aA, aB, 0);
        sub(bB, bA, aB, aA, 1);
        if constexpr (kSub == 4) {
            sub(bA, bB, aA, aB, 2);
            sub(bB, bA, aB, aA, 3);
        }
        // Stage kt+1 must have landed; kt+2's DMAs may stay in flight across the barrier.
        if (issue && !(LAB & 16)) wait_prev(!DLLM_HORNER_HR_GF || GF);
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    stage(st0, 0);
    if (nk > 1) stage(st1, 1, !DLLM_HORNER_HR_GF || !HORNER);
    if (nk > 1) wait_prev(!DLLM_HORNER_HR_GF || !HORNER);
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    using GFt = std::integral_constant<bool, true>;
    using GFf = std::integral_constant<bool, false>;
    if constexpr (HORNER) {
        // group = 2 k-steps, ring period 3: unroll 6 so each step's buffer and group phase are static
        for (unsigned kt = 0; kt < nk; kt += 6) {
            step(st0, st2, kt, GFt{});
            if (kt + 1 < nk) step(st1, st0, kt + 1, GFf{});
            if (kt + 2 < nk) step(st2, st1, kt + 2, GFt{});
            if (kt + 3 < nk) step(st0, st2, kt + 3, GFf{});
            if (kt + 4 < nk) step(st1, st0, kt + 4, GFt{});
            if (kt + 5 < nk) step(st2, st1, kt + 5, GFf{});
        }
        // acc = sum_g T_g s_g / s_{G-1}: times the last group's scales
        const float *sl = sf + static_cast<size_t>(nk / 2 - 1) * Npad + n0 + cw * 32 + 4 * hsel;
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
            const float4 s = *reinterpret_cast<const float4 *>(sl + 8 * qd);
#pragma unroll
            for (int r = 0; r < MR; ++r) {
                acc[r][4 * qd + 0] *= s.x;
                acc[r][4 * qd + 1] *= s.y;
                acc[r][4 * qd + 2] *= s.z;
                acc[r][4 * qd + 3] *= s.w;
            }
        }
    } else {
        for (unsigned kt = 0; kt < nk; kt += 3) {
            step(st0, st2, kt, GFf{});
            if (kt + 1 < nk) step(st1, st0, kt + 1, GFf{});
            if (kt + 2 < nk) step(st2, st1, kt + 2, GFf{});
        }
    }

    if constexpr (KG == 2) {
        // k-group 1 hands its accumulators to k-group 0 through the (now idle) stage buffers,
        // three m-reps per pass (one 16-KiB rep image per stage array), float4-lane-linear.
        static_assert(NW * 64 * 16 * 4 <= SL::kBytes, "a rep image must fit one stage array");
        uint8_t *bufs[3] = {st0, st1, st2};
#pragma unroll
        for (int r0 = 0; r0 < MR; r0 += 3) {
            if (kg == 1) {
#pragma unroll
                for (int u = 0; u < 3; ++u) {
                    if (r0 + u >= MR) break;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        *reinterpret_cast<float4 *>(bufs[u] + ((q * NW + cw) * 64 + lane) * 16) =
                            make_float4(acc[r0 + u][4 * q], acc[r0 + u][4 * q + 1], acc[r0 + u][4 * q + 2],
                                        acc[r0 + u][4 * q + 3]);
                }
            }
            __syncthreads();
            if (kg == 0) {
#pragma unroll
                for (int u = 0; u < 3; ++u) {
                    if (r0 + u >= MR) break;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float4 o = *reinterpret_cast<const float4 *>(bufs[u] + ((q * NW + cw) * 64 + lane) * 16);
                        acc[r0 + u][4 * q] += o.x;
                        acc[r0 + u][4 * q + 1] += o.y;
                        acc[r0 + u][4 * q + 2] += o.z;
                        acc[r0 + u][4 * q + 3] += o.w;
                    }
                }
            }
            __syncthreads();
        }
        if (kg != 0) return;
    }

    const int nb0 = n0 + cw * 32 + 4 * hsel;
    if constexpr (SPLIT) {
        float *slab = ws + static_cast<size_t>(ks) * M * Npad;
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            const int m = m0 + r * 32 + (lane & 31);
            if (m >= M) continue;
            float *prow = slab + static_cast<size_t>(m) * Npad + nb0;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd)
                *reinterpret_cast<float4 *>(prow + 8 * qd) =
                    make_float4(acc[r][4 * qd + 0], acc[r][4 * qd + 1], acc[r][4 * qd + 2], acc[r][4 * qd + 3]);
        }
        return;
    }
    float4 bv[4];
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) bv[qd] = *reinterpret_cast<const float4 *>(bias + nb0 + 8 * qd);
    if constexpr (EPI == 1) {
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            const int m = m0 + r * 32 + (lane & 31);
            if (m >= M) continue;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                if (nb0 + 8 * qd >= N) continue;
                psample4(epi, m, nb0 + 8 * qd, N, acc[r][4 * qd + 0] + bv[qd].x, acc[r][4 * qd + 1] + bv[qd].y,
                         acc[r][4 * qd + 2] + bv[qd].z, acc[r][4 * qd + 3] + bv[qd].w);
            }
        }
        return;
    }
    const bool full = (m0 + kBMt <= M) && (n0 + kBNt <= N) && (N % 4) == 0;
    if (full) {
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            YT *yrow = Y + static_cast<size_t>(m0 + r * 32 + (lane & 31)) * N + nb0;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd)
                store4<YT>(yrow + 8 * qd, acc[r][4 * qd + 0] + bv[qd].x, acc[r][4 * qd + 1] + bv[qd].y,
                           acc[r][4 * qd + 2] + bv[qd].z, acc[r][4 * qd + 3] + bv[qd].w);
        }
    } else {
        const bool vec_ok = (N % 4) == 0;
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            const int m = m0 + r * 32 + (lane & 31);
            if (m >= M) continue;
            YT *yrow = Y + static_cast<size_t>(m) * N;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd)
                store_out4<YT>(yrow, bias, nb0 + 8 * qd, N, vec_ok, acc[r][4 * qd + 0], acc[r][4 * qd + 1],
                               acc[r][4 * qd + 2], acc[r][4 * qd + 3]);
        }
    }
}

#if DLLM_LAB   // the 256 x 256 ring / ping-pong GEMM schedules (lab variants 4-15)
#include "lab/wq_ring256.inc"
#endif

#ifndef DLLM_DECODE_XL
#define DLLM_DECODE_XL 1
#endif

// ---------------------------------------------------------------------------------------------
// Decode GEMM (small M, weight-streaming / HBM-bound): one block per 16 NT-column group and
// K-slice (grid Npad/(16 NT) x nsplit), 8 waves split the block's K-slice by 128-deep slabs,
// 16x16x32 f16 MFMA with the weight as A (16 columns per n16 tile) and MT 16-token tiles of X as
// B, then the 8 wave partials are summed through LDS in wave order.  NT > 1 reuses each X
// fragment for NT weight tiles: at M = 64 a 16-column block reads 512 KiB of X from L2 for 32 KiB
// of weight, so the per-CU load path, not HBM, bounded the NT = 1 kernel.  With nsplit > 1 each
// K-slice writes an f32 slab and splitk_reduce_kernel sums the slabs in slice order (+ bias):
// deterministic, no atomics.
// Decode layout: [n16 tile][k128 slab][lane][BITS words], lane l = (n & 15) + 16 * ((k % 32) / 8),
// word/pair order as the prefill layout with the 32-deep step t in place of the substep.
// ---------------------------------------------------------------------------------------------
typedef float float4_t __attribute__((ext_vector_type(4)));
constexpr int kDecWaves = 8;
#if DLLM_STAMP
// phase stamps of wq_decode_kernel (stamp build only): 0 entry, 1 + 2 r / 2 + 2 r round r's loads
// issued / its MFMAs issued, kEpi the wave partials in LDS, kEnd exit
DLLM_STAMP_BUFFER(g_stamp_dec);
#endif

// EXACT (1: group 64, 2: group >= 128): the MFMA A operand is the exact integer (q - zp)
// (linear_exact.hip) and each slab's partial is folded into the accumulator with the f32 scales of
// its group(s) (group 64: two folds per 128-deep slab; group >= 128: one).  With one group per
// slab every lane's own {zp} dword is already its column's for all four 32-deep steps, so EXACT = 2
// skips the per-step ds_bpermute (an LDS round trip on the dequant's critical path).
// XL (M <= 16, NT = 1, EXACT = 2, one K-slice, every wave owning a slab): the block's X rows
// [M][K], one zero row and its columns' zero-point pairs and scales for every group are staged once
// in LDS (dynamic, xl_lds_bytes) by LDS-DMA -- 1 KiB per instruction -- instead of each wave
// fetching its own 16-B fragments per slab.  At M = 1 fifteen of sixteen fragment lanes were out of
// range and the scales were 4-16x redundant: 224 vector-memory instructions per CU for 32 KiB of
// weight words, which bounded the decode layer by the per-CU load issue rate, not by HBM
// (profiles/r05_midm).  With XL a CU issues the 32 weight loads, 8 X chunks and 16 scale rows --
// which measured no faster at M <= 8 (the layer waits on the weight stream's latency, not on load
// issue), and 7 % faster at M = 16, where the 16 lanes of a fragment are all in range; the product
// uses it for M 9..16.
template <int BITS, typename YT, int MT, int NT = 1, bool SPLIT = false, int LAB = 0, int EXACT = 0, int DW = kDecWaves,
          bool XL = false>
__global__ void __launch_bounds__(DW * 64)
wq_decode_kernel(const __half *__restrict__ X, int M, int K, const uint32_t *__restrict__ wdec,
                 const uint32_t *__restrict__ sz, const float *__restrict__ bias, YT *__restrict__ Y, int N, int Npad,
                 int group, int nsplit = 1, float *__restrict__ ws = nullptr, const float *__restrict__ sf = nullptr) {
    // Slabs in flight per wave: every load of a round (W words, scales, X fragments) is issued
    // before the first MFMA, so a round costs one memory latency, not one per 32-deep step.
    // The load phase has no branch and every loop bound is wave-uniform (scalar wave index): a
    // per-lane branch around a load makes the compiler wait for it at the join, which serialises
    // the rounds into one HBM latency per slab.  Rows >= M, steps past K and the clamped duplicate
    // slabs of the last round read X through a buffer resource with an out-of-range offset, which
    // returns zeros without a memory access; X is thereby also free of per-lane selects.
    // Rounds of slabs in flight per wave, sized to the registers one slab's operands take.
    constexpr int kPerSlab = NT * BITS + NT + 16 * MT + (EXACT ? 8 * NT : 0);
    constexpr int kDepth0 = NT == 1 ? (MT <= 2 ? 4 : 2) : (128 / kPerSlab < 1 ? 1 : (128 / kPerSlab > 4 ? 4 : 128 / kPerSlab));
    constexpr int kDepth = DW > 8 && kDepth0 > 2 ? 2 : kDepth0;   // 16 waves: 2 slabs each at K = 4096
    constexpr uint32_t kOOB = 0x80000000u;
    __shared__ __attribute__((aligned(16))) float red[DW * MT * NT * 64 * 4];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    DLLM_STAMP_RT(g_stamp_dec, stamp::kRtEntry);
    DLLM_STAMP_AT(g_stamp_dec, 0);
    DLLM_STAMP_IDS(g_stamp_dec);
    const int n0 = blockIdx.x * 16 * NT;
    const int nslab = (K + 127) / 128;
    // this block's K-slice: slabs [s_beg, s_end)
    const int s_beg = static_cast<int>(static_cast<long>(blockIdx.y) * nslab / nsplit);
    const int s_end = static_cast<int>(static_cast<long>(blockIdx.y + 1) * nslab / nsplit);
    const uint32_t *wbase = wdec + (static_cast<size_t>(blockIdx.x) * NT * nslab * 64 + lane) * BITS;
    const size_t wtile = static_cast<size_t>(nslab) * 64 * BITS;   // words per n16 tile
    // Scales: one dword per lane per slab and tile, lane l fetching (column l & 15, 32-deep step
    // l >> 4); step t's value for column c is then pulled from lane c + 16 t.
    const uint32_t *szcol = sz + n0 + (lane & 15);
    const int sz_step = lane >> 4;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<__half *>(X), 0, static_cast<int>(static_cast<size_t>(M) * K * 2), 0x00020000);
    uint32_t xoff[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = mt * 16 + (lane & 15);
        xoff[mt] = m < M ? static_cast<uint32_t>((m * K + 8 * (lane >> 4)) * 2) : kOOB;
    }
    // The epilogue's bias is fetched now, behind the weight stream, not after the reduction.
    float4 bv[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
        bv[nt] = SPLIT ? float4{0.f, 0.f, 0.f, 0.f}
                       : *reinterpret_cast<const float4 *>(bias + n0 + 16 * nt + 4 * (lane >> 4));

    static_assert(!XL || (MT == 1 && NT == 1 && EXACT == 2 && !SPLIT && LAB == 0), "XL: M <= 16, one tile, group >= 128");
    extern __shared__ __attribute__((aligned(16))) uint8_t xl_lds[];
    const int xl_pitch = K * 2 + 16;   // rows 16 B apart in bank order: the 16 rows of a fragment read hit 64 banks
    uint32_t xl_row = 0, xl_zero = 0;  // XL: this lane's fragment base (its token row, or the zero row)
    int xl_sz = 0, xl_sf = 0;          // XL: LDS offsets of the zero-point pair rows and the scale rows
    if constexpr (XL) {
        auto u = [](uint32_t v) { return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v))); };
        const uint32_t base = lds_addr(xl_lds);
        const int cpr = K / 512;   // 1-KiB chunks per X row
        for (int c = wave; c < M * cpr; c += DW) {
            const int row = c / cpr, cc = c - row * cpr;
            blds16_asm(xrs, static_cast<uint32_t>(lane * 16), u(static_cast<uint32_t>((row * K + cc * 512) * 2)),
                       u(base + static_cast<uint32_t>(row * xl_pitch + cc * 1024)));
        }
        // zero-point pairs then scales: ng rows of the block's 16 columns; one DMA moves 4 rows
        const int ng = K / group, nq = (ng + 3) / 4;
        xl_sz = (M + 1) * xl_pitch;
        xl_sf = xl_sz + nq * 256;
        const uint32_t pv = static_cast<uint32_t>(((lane >> 4) * Npad + (lane & 15)) * 4);
        const uint32_t prange = static_cast<uint32_t>((static_cast<size_t>(ng) * Npad - n0) * 4);
        // descriptor fields through readfirstlane: the asm's "s" operand needs them provably uniform
        auto uptr = [](const void *p) {
            const uint64_t v = reinterpret_cast<uint64_t>(p);
            const uint64_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v)));
            const uint64_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v >> 32)));
            return reinterpret_cast<void *>((hi << 32) | lo);
        };
        const int pr = __builtin_amdgcn_readfirstlane(static_cast<int>(prange));
        const __amdgpu_buffer_rsrc_t szr = __builtin_amdgcn_make_buffer_rsrc(uptr(sz + n0), 0, pr, 0x00020000);
        const __amdgpu_buffer_rsrc_t sfr = __builtin_amdgcn_make_buffer_rsrc(uptr(sf + n0), 0, pr, 0x00020000);
        // (two loops, one descriptor each: a select between them is not provably uniform)
        for (int j = wave; j < nq; j += DW)
            blds4_asm(szr, pv, u(static_cast<uint32_t>(4 * j * Npad * 4)), u(base + static_cast<uint32_t>(xl_sz + j * 256)));
        for (int j = wave; j < nq; j += DW)
            blds4_asm(sfr, pv, u(static_cast<uint32_t>(4 * j * Npad * 4)), u(base + static_cast<uint32_t>(xl_sf + j * 256)));
        for (int c = tid; c < K / 8; c += DW * 64)
            *reinterpret_cast<uint4 *>(xl_lds + M * xl_pitch + c * 16) = uint4{0u, 0u, 0u, 0u};
        xl_zero = static_cast<uint32_t>(M * xl_pitch + 16 * (lane >> 4));
        xl_row = (lane & 15) < M ? static_cast<uint32_t>((lane & 15) * xl_pitch + 16 * (lane >> 4)) : xl_zero;
    }

    float4_t acc[NT][MT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = float4_t{0.f, 0.f, 0.f, 0.f};

    const bool g64 = EXACT == 1;    // two groups per 128-deep slab
    int round = 0;
    for (int base = s_beg + wave; base < s_end; base += DW * kDepth, ++round) {
        uint32_t w[kDepth][NT][BITS];
        uint32_t szl[kDepth][NT];
        half8_t xb[kDepth][4][MT];
        float4 sfl[kDepth][NT][EXACT ? 2 : 1];
#pragma unroll
        for (int i = 0; i < kDepth; ++i) {
            const int slab_raw = base + i * DW;
            const int slab = min(slab_raw, s_end - 1);
            const int ks = min(slab * 128 + sz_step * 32, K - 32);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                if constexpr (LAB & 4) {
#pragma unroll
                    for (int j = 0; j < BITS; ++j) w[i][nt][j] = lane * 0x01010101u + j + slab;
                } else {
                    load_words<BITS>(w[i][nt], wbase + nt * wtile + static_cast<size_t>(slab) * 64 * BITS);
                }
                if constexpr (XL) continue;   // scales from LDS below
                if constexpr (LAB & 2) szl[i][nt] = 0x3c00e400u + ks;
                else szl[i][nt] = szcol[static_cast<size_t>(ks / group) * Npad + 16 * nt];
                if constexpr (EXACT) {
                    // scales of this lane's 4 columns for the slab's group (group 64: both halves)
                    const int nb0 = n0 + 16 * nt + 4 * (lane >> 4);
                    const int g0 = (slab * 128) / group, g1 = g64 ? min(g0 + 1, (K - 1) / group) : g0;
                    sfl[i][nt][0] = *reinterpret_cast<const float4 *>(sf + static_cast<size_t>(g0) * Npad + nb0);
                    sfl[i][nt][1] = *reinterpret_cast<const float4 *>(sf + static_cast<size_t>(g1) * Npad + nb0);
                }
            }
            if constexpr (XL) continue;   // X fragments from LDS below
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int k = slab_raw * 128 + t * 32;
                const bool step_ok = slab_raw < s_end && k < K;
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    if constexpr (LAB & 1) {
                        xb[i][t][mt] = half8_t{(_Float16)k, 1, 1, 1, 1, 1, 1, (_Float16)lane};
                    } else {
                        const uint32_t off = step_ok ? xoff[mt] + static_cast<uint32_t>(k * 2) : kOOB;
                        xb[i][t][mt] = __builtin_bit_cast(
                            half8_t, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
                    }
                }
            }
        }
        // Keep the scheduler from sinking the loads back next to their MFMAs (it does so to cut
        // register pressure, which turns the round into one serial latency per fragment).
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (XL) {
            if (round == 0) {
                // The block's LDS-DMAs must land before any wave reads X / scales from LDS.  The
                // round's weight loads were issued after them, but how many VMEM instructions
                // load_words becomes is the compiler's choice (it may split or merge them), so a
                // count that leaves them in flight could under-wait: drain everything, once.
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int i = 0; i < kDepth; ++i) {
                const int slab_raw = base + i * DW;
                const int slab = min(slab_raw, s_end - 1);
                const uint32_t lb = (slab_raw < s_end ? xl_row : xl_zero) + static_cast<uint32_t>(slab * 256);
#pragma unroll
                for (int t = 0; t < 4; ++t) xb[i][t][0] = *reinterpret_cast<const half8_t *>(xl_lds + lb + t * 64);
                const int g = (slab * 128) / group;
                szl[i][0] = *reinterpret_cast<const uint32_t *>(xl_lds + xl_sz + (g * 16 + (lane & 15)) * 4);
                sfl[i][0][0] = sfl[i][0][1] =
                    *reinterpret_cast<const float4 *>(xl_lds + xl_sf + (g * 16 + 4 * (lane >> 4)) * 4);
            }
        }
        DLLM_STAMP_AT(g_stamp_dec, round < 20 ? 1 + 2 * round : -1);
        if constexpr (EXACT) {
#pragma unroll
            for (int i = 0; i < kDepth; ++i) {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    float4_t tacc[MT];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const uint32_t szv = EXACT == 2 ? szl[i][nt] : static_cast<uint32_t>(
                            __builtin_amdgcn_ds_bpermute(((lane & 15) + 16 * t) * 4, static_cast<int>(szl[i][nt])));
                        const half2_t p = __builtin_bit_cast(half2_t, szv);
                        const half8_t a = dequant_exact<BITS>(w[i][nt], t, exact_consts(half2_t{p[0], p[0]}));
                        const bool first = t == 0 || (t == 2 && g64);
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
                            tacc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                                a, xb[i][t][mt], first ? float4_t{0.f, 0.f, 0.f, 0.f} : tacc[mt], 0, 0, 0);
                        if (t == 3 || (t == 1 && g64)) {
                            const float4 sv = sfl[i][nt][t == 3 && g64 ? 1 : 0];
#pragma unroll
                            for (int mt = 0; mt < MT; ++mt) {
                                acc[nt][mt][0] = __builtin_fmaf(sv.x, tacc[mt][0], acc[nt][mt][0]);
                                acc[nt][mt][1] = __builtin_fmaf(sv.y, tacc[mt][1], acc[nt][mt][1]);
                                acc[nt][mt][2] = __builtin_fmaf(sv.z, tacc[mt][2], acc[nt][mt][2]);
                                acc[nt][mt][3] = __builtin_fmaf(sv.w, tacc[mt][3], acc[nt][mt][3]);
                            }
                        }
                    }
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < kDepth; ++i) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) {
                        const uint32_t szv = static_cast<uint32_t>(
                            __builtin_amdgcn_ds_bpermute(((lane & 15) + 16 * t) * 4, static_cast<int>(szl[i][nt])));
                        half2_t nz, sc;
                        split_sz(szv, nz, sc);
                        const half8_t a = dequant_frag<BITS>(w[i][nt], t, nz, sc);
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
                            acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, xb[i][t][mt], acc[nt][mt], 0, 0, 0);
                    }
                }
            }
        }
        DLLM_STAMP_AT(g_stamp_dec, round < 20 ? 2 + 2 * round : -1);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
            *reinterpret_cast<float4_t *>(red + ((wave * MT * NT + nt * MT + mt) * 64 + lane) * 4) = acc[nt][mt];
    __syncthreads();
    DLLM_STAMP_AT(g_stamp_dec, stamp::kEpi);
    // Wave j sums the 8 partials of tiles j, j + 8, ... (tile = nt * MT + mt) in wave order.
    for (int tile = wave; tile < MT * NT; tile += DW) {
        float4_t s = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int w = 0; w < DW; ++w)
            s += *reinterpret_cast<const float4_t *>(red + ((w * MT * NT + tile) * 64 + lane) * 4);
        const int nt = tile / MT, mt = tile % MT;
        const int m = mt * 16 + (lane & 15);
        const int nb0 = n0 + 16 * nt + 4 * (lane >> 4);
        if constexpr (SPLIT) {
            // slab [split][M][Npad]; Npad covers every column of the block
            if (m < M)
                *reinterpret_cast<float4_t *>(ws + (static_cast<size_t>(blockIdx.y) * M + m) * Npad + nb0) = s;
        } else if (m < M && nb0 < N) {
            // bias of this tile: bv[nt] (nt is wave-uniform, select without dynamic indexing)
            float4 b = bv[0];
#pragma unroll
            for (int j = 1; j < NT; ++j)
                if (nt == j) b = bv[j];
            YT *yrow = Y + static_cast<size_t>(m) * N;
            const float y0 = s[0] + b.x, y1 = s[1] + b.y, y2 = s[2] + b.z, y3 = s[3] + b.w;
            if ((N % 4) == 0) {
                store4<YT>(yrow + nb0, y0, y1, y2, y3);
            } else {
                store1<YT>(yrow + nb0, y0);
                if (nb0 + 1 < N) store1<YT>(yrow + nb0 + 1, y1);
                if (nb0 + 2 < N) store1<YT>(yrow + nb0 + 2, y2);
                if (nb0 + 3 < N) store1<YT>(yrow + nb0 + 3, y3);
            }
        }
    }
    DLLM_STAMP_AT(g_stamp_dec, stamp::kEnd);
    DLLM_STAMP_RT(g_stamp_dec, stamp::kRtEnd);
}
#if DLLM_STAMP
}  // namespace
DLLM_STAMP_READER(dllm_stamp_read_dec, g_stamp_dec)
namespace {
#endif

constexpr int kDecodeMaxM = 64;

// XL decode (M <= 16): dynamic LDS of X rows + zero row (2K + 16 B each) + pair and scale rows
// (256 B per 4 groups each), within the CU's 160 KiB beside the 8 KiB partial-sum buffer.
constexpr size_t kXlLdsMax = 160 * 1024 - kDecWaves * 64 * 4 * 4;
inline size_t xl_lds_bytes(int M, int K, int group) {
    const size_t nq = static_cast<size_t>((K / group + 3) / 4);
    return static_cast<size_t>(M + 1) * (2 * static_cast<size_t>(K) + 16) + 2 * nq * 256;
}

// Exact-weight kernels apply when the group tiles K (a stage never straddles two groups).
inline bool use_exact(const dllm_linear *h) {
    return h->precision == DLLM_PRECISION_EXACT &&
           exact_gemm_supported(1, static_cast<int>(h->K), static_cast<int>(h->Npad), static_cast<int>(h->group));
}

// Decode tile policy: (NT, nsplit) per M bucket, chosen from the M-sweep.
// Measured (scripts/decode_sweep.py, 48-layer graph, K = N = 4096 int4, us per layer;
// profiles/r01_decode_tiles): up to M = 32 the one-tile kernel wins (M 1/16/32: 5.1/6.9/10.7;
// the slab combine's extra launch costs ~4.7 us and NT = 4 without a split leaves 64 blocks whose
// per-CU load rate bounds the stream); at M 33..64 X re-reads dominate and NT 4 x 4 K-slices
// wins (M 64: 13.8 vs 18.6).
inline void decode_policy(int M, int &nt, int &nsplit) {
    nt = nsplit = M > 32 ? 4 : 1;
}

template <int BITS, typename YT, int MT, int NT, int EXACT>
int launch_decode_nt(const dllm_linear *h, const __half *X, int M, YT *Y, int nsplit, hipStream_t st) {
    const unsigned nbx = static_cast<unsigned>(h->Npad / (16 * NT));
    const int K = static_cast<int>(h->K), N = static_cast<int>(h->N);
    const int Np = static_cast<int>(h->Npad), gr = static_cast<int>(h->group);
    const int nslab = (K + 127) / 128;
    nsplit = std::max(1, std::min(nsplit, nslab));
    if (nsplit == 1) {
#if DLLM_DECODE_XL
        if constexpr (MT == 1 && NT == 1 && EXACT == 2) {
            const size_t bytes = xl_lds_bytes(M, K, gr);
            // M 9..16 only: M = 16 6.75 vs 7.25 us per layer in the 40-layer chain, M = 1 / 2 / 4 / 8
            // 5.16 / 5.34 / 5.58 / 6.00 vs 5.18 / 5.38 / 5.47 / 5.94 (profiles/r05_decode_xl/): fewer
            // load instructions do not shorten the M <= 8 layer, whose time is the weight stream's
            // latency, and the DMA wait + barrier before the first MFMA costs a little there.
            if (M > 8 && K % 512 == 0 && nslab >= kDecWaves && bytes <= kXlLdsMax) {
                auto *kern = &wq_decode_kernel<BITS, YT, 1, 1, false, 0, 2, kDecWaves, true>;
                // the dynamic-LDS limit, set once per device (a bit per device id; a process may drive
                // several GPUs)
                static std::atomic<uint64_t> attr_set{0};
                int dev = 0;
                if (hipGetDevice(&dev) != hipSuccess) return fail(DLLM_ERR_HIP, "decode XL device");
                const uint64_t bit = dev < 64 ? (uint64_t{1} << dev) : 0;
                if (!bit || !(attr_set.load(std::memory_order_acquire) & bit)) {
                    if (hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                            static_cast<int>(kXlLdsMax)) != hipSuccess)
                        return fail(DLLM_ERR_HIP, "decode XL LDS attribute");
                    attr_set.fetch_or(bit, std::memory_order_acq_rel);
                }
                kern<<<nbx, kDecWaves * 64, bytes, st>>>(X, M, K, h->wdec, h->sz, h->bias, Y, N, Np, gr, 1, nullptr, h->sf);
                DLLM_LAUNCH_CHECK();
                return DLLM_OK;
            }
        }
#endif
#if DLLM_LAB
        if constexpr (MT * NT <= 2) {
            if (h->variant == 306) {   // lab A/B: 16 waves per block (two slabs each at K = 4096)
                wq_decode_kernel<BITS, YT, MT, NT, false, 0, EXACT, 16><<<nbx, 16 * 64, 0, st>>>(
                    X, M, K, h->wdec, h->sz, h->bias, Y, N, Np, gr, 1, nullptr, h->sf);
                DLLM_LAUNCH_CHECK();
                return DLLM_OK;
            }
        }
#endif
        wq_decode_kernel<BITS, YT, MT, NT, false, 0, EXACT><<<nbx, kDecWaves * 64, 0, st>>>(
            X, M, K, h->wdec, h->sz, h->bias, Y, N, Np, gr, 1, nullptr, h->sf);
        DLLM_LAUNCH_CHECK();
        return DLLM_OK;
    }
    float *ws = device_workspace(st, static_cast<size_t>(nsplit) * M * h->Npad * sizeof(float));
    if (!ws) return DLLM_ERR_HIP;
    wq_decode_kernel<BITS, YT, MT, NT, true, 0, EXACT><<<dim3(nbx, static_cast<unsigned>(nsplit)), kDecWaves * 64, 0, st>>>(
        X, M, K, h->wdec, h->sz, h->bias, Y, N, Np, gr, nsplit, ws, h->sf);
    DLLM_LAUNCH_CHECK();
    const size_t q = static_cast<size_t>(M) * (h->Npad / 4);
    const unsigned rb = static_cast<unsigned>(std::min<size_t>((q + 255) / 256, 4 * kCUs));
    splitk_reduce_kernel<YT><<<rb, 256, 0, st>>>(ws, nsplit, M, N, Np, h->bias, Y, PSampleEpi{});
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

template <int BITS, typename YT, int MT, int EXACT>
int launch_decode_mt(const dllm_linear *h, const __half *X, int M, YT *Y, int nt, int nsplit, hipStream_t st) {
    switch (nt) {
    case 2: return launch_decode_nt<BITS, YT, MT, 2, EXACT>(h, X, M, Y, nsplit, st);
    case 4: return launch_decode_nt<BITS, YT, MT, 4, EXACT>(h, X, M, Y, nsplit, st);
    default: return launch_decode_nt<BITS, YT, MT, 1, EXACT>(h, X, M, Y, nsplit, st);
    }
}

template <int BITS, typename YT, int EXACT>
int launch_decode_x(const dllm_linear *h, const __half *X, size_t M, YT *Y, int nt, int nsplit, hipStream_t st) {
    const int Mi = static_cast<int>(M);
    if (M <= 16) return launch_decode_mt<BITS, YT, 1, EXACT>(h, X, Mi, Y, nt, nsplit, st);
    if (M <= 32) return launch_decode_mt<BITS, YT, 2, EXACT>(h, X, Mi, Y, nt, nsplit, st);
    return launch_decode_mt<BITS, YT, 4, EXACT>(h, X, Mi, Y, nt, nsplit, st);
}

#if DLLM_LAB
template <int BITS, typename YT>
int launch_decode_lab(const dllm_linear *h, const __half *X, size_t M, YT *Y, hipStream_t st) {
    const unsigned nb = static_cast<unsigned>(h->Npad / 16);
    const int Mi = static_cast<int>(M), K = static_cast<int>(h->K), N = static_cast<int>(h->N);
    const int Np = static_cast<int>(h->Npad), gr = static_cast<int>(h->group);
    switch (h->dlab) {
#define DLLM_DLAB(L) case L: wq_decode_kernel<BITS, YT, 1, 1, false, L><<<nb, kDecWaves * 64, 0, st>>>(X, Mi, K, h->wdec, h->sz, h->bias, Y, N, Np, gr); break;
        DLLM_DLAB(1) DLLM_DLAB(2) DLLM_DLAB(3) DLLM_DLAB(4) DLLM_DLAB(5) DLLM_DLAB(6) DLLM_DLAB(7)
#undef DLLM_DLAB
        default: break;
    }
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}
#endif

// Both code layouts are built by the handle's create (finish_linear), so a forward call never
// allocates, builds or synchronises, and behaves the same inside and outside stream capture.
int ensure_decode_layout(const dllm_linear *h, hipStream_t) {
    return h->wdec ? DLLM_OK : fail(DLLM_ERR_INVALID_PARAMS, "linear handle has no decode layout");
}

template <int BITS, typename YT>
int launch_decode(const dllm_linear *h, const __half *X, size_t M, YT *Y, hipStream_t st) {
    if (const int rc = ensure_decode_layout(h, st)) return rc;
    int nt, nsplit;
    decode_policy(static_cast<int>(M), nt, nsplit);
#if DLLM_LAB
    if (M <= 16 && h->dlab != 0) return launch_decode_lab<BITS, YT>(h, X, M, Y, st);
    if (h->dcfg > 0) {   // dcfg = 16 log2(NT) + log2(nsplit) + 1
        nt = 1 << ((h->dcfg - 1) / 16);
        nsplit = 1 << ((h->dcfg - 1) % 16);
    }
#endif
    // the column group must tile Npad (a multiple of 128)
    while (nt > 1 && h->Npad % (16 * nt)) nt /= 2;
    if (use_exact(h)) {
        if (h->group == 64) return launch_decode_x<BITS, YT, 1>(h, X, M, Y, nt, nsplit, st);
        return launch_decode_x<BITS, YT, 2>(h, X, M, Y, nt, nsplit, st);
    }
    return launch_decode_x<BITS, YT, 0>(h, X, M, Y, nt, nsplit, st);
}

// 3-stage-ring GEMM (rounded weights) with tile (32 MR) x (32 NW), K optionally split into nsplit slices.
template <int BITS, typename YT, int NW, int MR, int KG = 1, int EPI = 0>
int launch_ring(const dllm_linear *h, const __half *X, int M, YT *Y, hipStream_t st, int nsplit,
                const PSampleEpi *epi = nullptr) {
    const int nbm = (M + 32 * MR - 1) / (32 * MR), nbn = static_cast<int>(h->Npad / (32 * NW));
    const unsigned nb = static_cast<unsigned>(nbm * nbn * nsplit);
    const PSampleEpi ep = epi ? *epi : PSampleEpi{};
#if DLLM_LAB
    if (EPI == 0 && h->rlab != 0 && nsplit == 1) {   // measurement only
        switch (h->rlab) {
#define DLLM_RLAB(L)                                                                                              \
    case L:                                                                                                       \
        wq_gemm8_kernel<BITS, YT, NW, MR, false, KG, L><<<nb, NW * KG * 64, 0, st>>>(                           \
            X, M, (int)h->K, h->wdev, h->sz, h->bias, Y, (int)h->N, (int)h->Npad, (int)h->group, nbm, nbn);   \
        break;
            DLLM_RLAB(1) DLLM_RLAB(2) DLLM_RLAB(3) DLLM_RLAB(4) DLLM_RLAB(5) DLLM_RLAB(6) DLLM_RLAB(7)
            DLLM_RLAB(8) DLLM_RLAB(9) DLLM_RLAB(10) DLLM_RLAB(11) DLLM_RLAB(16) DLLM_RLAB(20) DLLM_RLAB(32)
            DLLM_RLAB(40)
#undef DLLM_RLAB
            default: break;
        }
        DLLM_LAUNCH_CHECK();
        return DLLM_OK;
    }
#endif
    if (nsplit == 1) {
        wq_gemm8_kernel<BITS, YT, NW, MR, false, KG, 0, EPI><<<nb, NW * KG * 64, 0, st>>>(
            X, M, (int)h->K, h->wdev, h->sz, h->bias, Y, (int)h->N, (int)h->Npad, (int)h->group, nbm, nbn, 1,
            nullptr, ep);
        DLLM_LAUNCH_CHECK();
        return DLLM_OK;
    }
    float *ws = device_workspace(st, static_cast<size_t>(nsplit) * M * h->Npad * sizeof(float));
    if (!ws) return DLLM_ERR_HIP;
    wq_gemm8_kernel<BITS, YT, NW, MR, true, KG><<<nb, NW * KG * 64, 0, st>>>(
        X, M, (int)h->K, h->wdev, h->sz, h->bias, Y, (int)h->N, (int)h->Npad, (int)h->group, nbm, nbn, nsplit, ws);
    DLLM_LAUNCH_CHECK();
    const size_t q = static_cast<size_t>(M) * (h->Npad / 4);
    const unsigned rb = static_cast<unsigned>(std::min<size_t>((q + 255) / 256, 4 * kCUs));
    splitk_reduce_kernel<YT, EPI><<<rb, 256, 0, st>>>(ws, nsplit, M, (int)h->N, (int)h->Npad, h->bias, Y, ep);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

#if DLLM_LAB   // launchers of the lab schedules
#include "lab/wq_lab_launch.inc"
#endif

// Rounded-weight (DLLM_PRECISION_F16W) tile policy: the largest tile that still gives >= 256
// blocks -- 256 x 256 (8 waves), 256 x 128 (8 waves, two k-groups) -- below that 128 x 128 tiles
// (two k-groups) with K split until ~200+ blocks (slab partials + ordered combine).
template <int BITS, typename YT, int EPI = 0>
int launch_rounded(const dllm_linear *h, const __half *X, int M, YT *Y, hipStream_t st,
                   const PSampleEpi *epi = nullptr) {
    const int np = static_cast<int>(h->Npad);
    const int mb256 = (M + 255) / 256, mb128 = (M + 127) / 128;
    if (np % 256 == 0 && mb256 * (np / 256) >= kCUs) return launch_ring<BITS, YT, 8, 8, 1, EPI>(h, X, M, Y, st, 1, epi);
    if (mb256 * (np / 128) >= kCUs) return launch_ring<BITS, YT, 4, 8, 2, EPI>(h, X, M, Y, st, 1, epi);
    const int tiles = mb128 * (np / 128);
    const int nk = static_cast<int>(h->K / kBK);
    int nsplit = 1;
    while (tiles * nsplit < 200 && nsplit < 8 && nk % (2 * nsplit) == 0 && nk / (2 * nsplit) >= 4) nsplit *= 2;
    return launch_ring<BITS, YT, 4, 4, 2, EPI>(h, X, M, Y, st, nsplit, epi);
}

// Exact-weight GEMM in Horner form (wq_gemm8_kernel<..., HORNER>, 256 x 256 tiles): for int4 g128
// on grids of >= 256 such tiles.  The ratios and their validity are decided once, by the handle's
// create (finish_linear); a handle whose scales fail the check runs the fold-form exact kernels.
#if DLLM_LAB
inline bool lab_horner128() {
    static const bool on = std::getenv("DLLM_LAB_HORNER128") != nullptr;
    return on;
}
#endif

// int4 and (256 x 256 tiles only: horner_ready) int2 codes, group 128.
inline bool horner_shape(const dllm_linear *h) {
    return h->precision == DLLM_PRECISION_EXACT && (h->bits == 4 || h->bits == 2) && h->group == 128 &&
           h->K % 128 == 0 && h->Npad % 256 == 0;
}

// The handle's Horner ratios are valid (decided at create, immutable afterwards).
inline bool ensure_horner(const dllm_linear *h, hipStream_t) { return h->hstate == 1; }

// DLLM_POLICY_ROUNDS (product; 0 = the earlier full-round thresholds, A/B): a grid short of a round
// takes the larger tiles when the alternative needs more rounds -- a 256 x 256 Horner round takes
// about two 128 x 256 PC rounds, a 128 x 256 PC round about 1.78 two-k-group 128 x 128 rounds
// (58.6 vs 33 us at K 4096).  N 4096, 40-layer chain (profiles/r06_tiles/policy_rounds_ab.jsonl):
// M 1100 / 1280 / 1536 / 1800: 63.2 / 61.0 / 62.1 / 68.2 -> 56.8 / 52.3 / 53.2 / 59.0 us (128 x 256
// PC tiles short of a round), M 2304 / 2560 / 3072 / 3584: 106.5 / 106.7 / 107.7 / 112.6 -> 97.3 /
// 97.3 / 98.4 / 104.0 us (256 x 256 Horner tiles short of a round), M 2048 and 4096 unchanged.
#ifndef DLLM_POLICY_ROUNDS
#define DLLM_POLICY_ROUNDS 1
#endif
bool horner_ready(const dllm_linear *hc, int M, hipStream_t st) {
    const int np = static_cast<int>(hc->Npad);
    if (!horner_shape(hc)) return false;
    // rounds of 256 tiles: a 256 x 256 round takes about two 128 x 256 rounds, so the Horner grid
    // must not need more rounds than half the fold form's (M = 4300: 2 vs 3 rounds -> fold form)
    const int t256 = ((M + 255) / 256) * (np / 256), t128 = ((M + 127) / 128) * (np / 256);
#if DLLM_LAB
    if (hc->variant == 14) return false;   // lab A/B: the fold-form exact policy
    if (lab_horner128()) {                 // lab A/B: Horner form on 128 x 256 tiles
        if (t128 < kCUs) return false;
    } else
#endif
    if ((!DLLM_POLICY_ROUNDS && t256 < kCUs) || 2 * ((t256 + kCUs - 1) / kCUs) > (t128 + kCUs - 1) / kCUs)
        return false;
    return ensure_horner(hc, st);
}

// The Horner kernel on 128-token tiles (wq_horner16_kernel<..., TB = 8>, x 256 columns, 128-deep
// stages), for grids where the 256 x 256 Horner grid leaves CUs idle but 128 x 256 tiles fill a round
// (M = 2048 at N = 4096; the 2-GPU column shard, M = 4096 x N 2048).  Lab A/B only (variant 323):
// against the fold form on those grids it measured -2.8 % on one box and +8 % on another (M = 2048:
// 64.9 vs 66.7 us, 72.5 vs 67.0 us; profiles/r04_horner/), so the fold form stays the product path.
// Returns the tile rows, 0 = not applicable.
#if DLLM_LAB
int horner_rows(const dllm_linear *hc, int M) {
    const int np = static_cast<int>(hc->Npad);
    if (hc->variant != 323 || hc->bits != 4 || !horner_shape(hc) || hc->hstate != 1) return 0;
    if (((M + 127) / 128) * (np / 256) >= kCUs) return 128;
    return 0;
}
#endif

// The KG2 Horner kernel (256 x 128 tiles, two k-groups): where neither the 256 x 256 Horner grid
// nor the fold form's 128 x 256 grid fills a round but the 256 x 128 grid does (N = 4096: M
// 1793..1920; measured at M = 1800: 69.2 vs 74.9 us).  At M = 2048 the 128 x 256 fold grid fills
// the chip and is as fast (68.5 vs 69.6 us: KG2 stages two K-halves' X slices, 72 KiB per k-step
// against 24 KiB for the same MFMAs; profiles/r03_kg2/).
bool horner_kg2_ready(const dllm_linear *hc, int M) {
    const int np = static_cast<int>(hc->Npad);
    if (!(hc->precision == DLLM_PRECISION_EXACT && hc->bits == 4 && hc->group == 128 && hc->K % 256 == 0 &&
          np % 128 == 0 && hc->hstate == 1))
        return false;
#if DLLM_LAB
    if (hc->variant == 14 || hc->variant == 28) return false;   // lab A/B: the fold-form exact policy
#endif
    const int t256 = ((M + 255) / 256) * (np / 256), tk = ((M + 255) / 256) * (np / 128);
    const int t128 = ((M + 127) / 128) * (np / 256);
    return t256 < kCUs && t128 < kCUs && tk >= kCUs;
}

// The producer / consumer Horner kernel (128 x 256 tiles, linear_pc.hip): where the 256 x 256
// Horner grid does not fill a round and the 128 x 256 grid does (N = 4096: M 1921..4096 minus the
// Horner grid's own range; M = 2048 = config C2 and the C5 layers; the 2-GPU column shard).
#ifndef DLLM_HORNER_PC
#define DLLM_HORNER_PC 1
#endif
bool horner_pc_ready(const dllm_linear *hc, int M, hipStream_t st) {
#if DLLM_HORNER_PC
    const int np = static_cast<int>(hc->Npad);
    if (hc->bits != 4 || !horner_shape(hc) || hc->hstate != 1) return false;
#if DLLM_LAB
    if (hc->variant == 14 || hc->variant == 28) return false;   // lab A/B: the fold-form exact policy
#endif
    const int t128 = ((M + 127) / 128) * (np / 256);
    if (horner_ready(hc, M, st)) return false;
    if (t128 >= kCUs) return true;
    if (!DLLM_POLICY_ROUNDS || np % 128 != 0 || hc->K % 256 != 0) return false;
    const int tk = ((M + 127) / 128) * (np / 128);   // the two-k-group 128 x 128 grid
    return 178 * ((t128 + kCUs - 1) / kCUs) <= 100 * ((tk + kCUs - 1) / kCUs);
#else
    (void)hc; (void)M; (void)st;
    return false;
#endif
}

// The two-k-group PC kernel (rows x 128 tiles, linear_pc.hip): where none of the larger Horner grids
// fills a round, 128- or 64-row tiles by rounds x tile time (below) (128: the 4-GPU
// column shard M = 4096 x N 1024, M = 2048 x N 2048, M = 1024 x N 4096: 34.8 -> 32.3 us; 64: M = 512
// x N 4096 and the 8-GPU shard 4096 x 512: 22.1 -> 21.5 us).  32-row tiles (DLLM_PC_KG2_SMALL, A/B)
// lose to the 4-k-group fold tiles at mid M (M 256: 17.1 vs 14.3 us; profiles/r06_tiles/).  Returns
// the tile rows, 0 = not applicable.
#ifndef DLLM_HORNER_PC_KG2
#define DLLM_HORNER_PC_KG2 1
#endif
// A 64-row grid of at least 3/4 of a round takes the two-k-group PC kernel: M 321..448 at N 4096
// (192..224 tiles) ran 21.3 / 21.4 us at M 384 / 448 against 21.8 / 23.4 for the 4-k-group fold
// tiles of mid M; at 5/8 of a round (M 300, 160 tiles) the fold tiles stay faster (21.4 vs 22.8 us;
// profiles/r06_tiles/pc_kg2_fill_ab.jsonl, 40-layer chain).
#ifndef DLLM_PC_KG2_MINFILL
#define DLLM_PC_KG2_MINFILL (3 * kCUs / 4)
#endif
#ifndef DLLM_PC_KG2_SMALL   // 64- and 32-token tiles too
#define DLLM_PC_KG2_SMALL 0
#endif
bool horner_kg2_ready(const dllm_linear *hc, int M);
int horner_pc_kg2_rows(const dllm_linear *hc, int M, hipStream_t st) {
#if DLLM_HORNER_PC_KG2
    const int np = static_cast<int>(hc->Npad);
    if (!(hc->precision == DLLM_PRECISION_EXACT && hc->bits == 4 && hc->group == 128 && hc->K % 256 == 0 &&
          np % 128 == 0 && hc->hstate == 1))
        return 0;
#if DLLM_LAB
    if (hc->variant == 14 || hc->variant == 28) return 0;   // lab A/B: the fold-form exact policy
#endif
    if (horner_ready(hc, M, st) || horner_pc_ready(hc, M, st) || horner_kg2_ready(hc, M)) return 0;
#if DLLM_PC_KG2_SMALL
    for (int rows = 128; rows >= 32; rows /= 2) {
        const int t = ((M + rows - 1) / rows) * (np / 128);
        if (t >= 2 * kCUs) return 0;
        if (t >= DLLM_PC_KG2_MINFILL) return rows;
    }
    return 0;
#else
    // A 128-row tile takes ~1.55x a 64-row one (33 vs 21 us at K 4096: the 4- and 8-GPU shards), so
    // a grid of 128-row tiles short of a round still beats two rounds of 64-row tiles, and a single
    // round of 64-row tiles beats one of 128-row tiles.  N 4096: M 513..768 now take 128-row tiles
    // (M 700 / 768: 42.1 / 39.1 -> 33.3 / 30.5 us in the 40-layer chain; they took 64-row tiles in
    // 1.1 - 1.5 rounds) and M 321..448 64-row tiles (a 64-row grid of fewer than
    // DLLM_PC_KG2_MINFILL tiles leaves mid M to the fold tiles); profiles/r06_tiles/pc_kg2_fill_ab.jsonl, pc_kg2_policy_ab.jsonl.
    const int t128 = ((M + 127) / 128) * (np / 128), t64 = ((M + 63) / 64) * (np / 128);
    if (t128 >= 2 * kCUs) return 0;   // the larger tiles of the other kernels fill the chip
    if (t128 >= kCUs || t64 > kCUs) return 128;
    return t64 >= DLLM_PC_KG2_MINFILL ? 64 : 0;
#endif
#else
    (void)hc; (void)M; (void)st;
    return 0;
#endif
}

template <typename YT, int EPI>
int launch_horner(const dllm_linear *h, const __half *X, int M, YT *Y, hipStream_t st, const PSampleEpi *epi) {
#if DLLM_LAB
    const PSampleEpi ep = epi ? *epi : PSampleEpi{};
    if (lab_horner128() && h->bits == 4) {
        const int nbm = (M + 127) / 128, nbn = static_cast<int>(h->Npad / 256);
        wq_gemm8_kernel<4, YT, 8, 4, false, 1, 0, EPI, true><<<static_cast<unsigned>(nbm * nbn), 512, 0, st>>>(
            X, M, (int)h->K, h->wdev, h->sz, h->bias, Y, (int)h->N, (int)h->Npad, (int)h->group, nbm, nbn, 1, nullptr,
            ep, h->hr, h->sf);
        DLLM_LAUNCH_CHECK();
        return DLLM_OK;
    }
    if (h->variant == 24 && h->bits == 4) {   // lab A/B: the round-2 Horner kernel (wq_gemm8_kernel<..., HORNER>)
        const int nbm = (M + 255) / 256, nbn = static_cast<int>(h->Npad / 256);
        wq_gemm8_kernel<4, YT, 8, 8, false, 1, 0, EPI, true><<<static_cast<unsigned>(nbm * nbn), 512, 0, st>>>(
            X, M, (int)h->K, h->wdev, h->sz, h->bias, Y, (int)h->N, (int)h->Npad, (int)h->group, nbm, nbn, 1, nullptr,
            ep, h->hr, h->sf);
        DLLM_LAUNCH_CHECK();
        return DLLM_OK;
    }
#endif
    HornerGemmArgs a{X, M, (int)h->K, h->wdev, h->sz, h->hr, h->sf, h->bias, Y, (int)h->N, (int)h->Npad, epi};
    a.bits = static_cast<int>(h->bits);
#if DLLM_LAB
    if (h->variant >= 25 && h->variant <= 27) a.lab = h->variant - 24;   // lab A/B (see HornerGemmArgs::lab)
    if (h->variant >= 29 && h->variant <= 31) a.lab = h->variant - 25;   // lab ablations 4..6
    if (h->variant >= 303 && h->variant <= 304) a.lab = h->variant - 295;   // lab ablations 8, 9 (DMA)
    if (h->variant >= 310 && h->variant <= 312) a.lab = h->variant - 300;   // lab XCD groupings (10..12)
    if ((h->variant >= 314 && h->variant <= 321) || (h->variant >= 324 && h->variant <= 328)) a.lab = h->variant - 300;   // lab: MFMA only / DMA only / burst DMA / ...
    if (h->variant == 305) a.lab = 7;   // lab ablation: no stores, rescale; one dequant and B read per k-step
    if (h->variant >= 340 && h->variant <= 345) a.lab = h->variant - 300;   // product-kernel ablations / A/B (40..45)
#endif
    return launch_horner_gemm(a, std::is_same<YT, float>::value ? 1 : 0, st);
}

inline ExactGemmArgs exact_args(const dllm_linear *h, const __half *X, int M, void *Y, const PSampleEpi *epi) {
    ExactGemmArgs a{h->bits, X, M, (int)h->K, h->wdev, h->sz, h->sf, h->bias, Y, (int)h->N, (int)h->Npad,
                    (int)h->group, epi};
#if DLLM_LAB
    a.tm = h->variant == 15 ? 1 : 0;
    a.lab_policy = h->variant == 28 ? 1 : (h->variant >= 300 && h->variant <= 302 ? h->variant - 298 : (h->variant == 329 ? 5 : (h->variant == 330 ? 6 : (h->variant == 331 ? 7 : 0))));
#endif
    return a;
}

// Prefill (M > kDecodeMaxM) dispatch: exact-weight kernels (default precision) or the rounded ring.
template <int BITS, typename YT, int EPI = 0>
int launch_prefill_auto(const dllm_linear *h, const __half *X, int M, YT *Y, hipStream_t st,
                        const PSampleEpi *epi = nullptr) {
#if DLLM_LAB
    // lab A/B: 4 = the rounded policy, 14 / 15 = exact (128 x 256 / tile-major 256 x 256), others
    // = the round-1 schedules; -1 (default) = the product policy below
    if (h->variant == 4) return launch_rounded<BITS, YT, EPI>(h, X, M, Y, st, epi);
    if ((h->variant == 14 || h->variant == 15) && exact_gemm_supported(M, (int)h->K, (int)h->Npad, (int)h->group))
        return launch_exact_gemm(exact_args(h, X, M, Y, epi), std::is_same<YT, float>::value ? 1 : 0, st);
    if (h->variant >= 0) {
        const int rc = launch_lab_variant<BITS, YT, EPI>(h, X, M, Y, st, epi);
        if (rc >= 0) return rc;
    }
#endif
    if (use_exact(h)) {
        if ((BITS == 4 || BITS == 2) && horner_ready(h, M, st)) return launch_horner<YT, EPI>(h, X, M, Y, st, epi);
        if (BITS == 4 && horner_pc_ready(h, M, st)) {
            const HornerGemmArgs a{X, M, (int)h->K, h->wdev, h->sz, h->hr, h->sf, h->bias, Y, (int)h->N,
                                   (int)h->Npad, epi};
            return launch_horner_pc_gemm(a, std::is_same<YT, float>::value ? 1 : 0, st);
        }
        if (BITS == 4 && horner_kg2_ready(h, M)) {
            const HornerGemmArgs a{X, M, (int)h->K, h->wdev, h->sz, h->hr, h->sf, h->bias, Y, (int)h->N,
                                   (int)h->Npad, epi};
            return launch_horner_kg2_gemm(a, std::is_same<YT, float>::value ? 1 : 0, st);
        }
        if (const int rows = BITS == 4 ? horner_pc_kg2_rows(h, M, st) : 0) {
            const HornerGemmArgs a{X, M, (int)h->K, h->wdev, h->sz, h->hr, h->sf, h->bias, Y, (int)h->N,
                                   (int)h->Npad, epi};
            return launch_horner_pc_kg2_gemm(a, rows, std::is_same<YT, float>::value ? 1 : 0, st);
        }
#if DLLM_LAB
        if (const int rows = BITS == 4 ? horner_rows(h, M) : 0) {   // lab A/B 323 only
            const HornerGemmArgs a{X, M, (int)h->K, h->wdev, h->sz, h->hr, h->sf, h->bias, Y, (int)h->N,
                                   (int)h->Npad, epi};
            return launch_horner_rows_gemm(a, rows, std::is_same<YT, float>::value ? 1 : 0, st);
        }
#endif
        ExactGemmArgs a = exact_args(h, X, M, Y, epi);
#if DLLM_EXACT_HORNER   // A/B build: the 128 x 256 exact tiles in Horner form too
        if (BITS == 4 && ensure_horner(h, st)) a.hr = h->hr;
#endif
        return launch_exact_gemm(a, std::is_same<YT, float>::value ? 1 : 0, st);
    }
    return launch_rounded<BITS, YT, EPI>(h, X, M, Y, st, epi);
}

template <int BITS, typename YT>
int launch_gemm_t(const dllm_linear *h, const __half *X, size_t M, YT *Y, hipStream_t st) {
    if (M <= static_cast<size_t>(kDecodeMaxM) && h->wdec) return launch_decode<BITS, YT>(h, X, M, Y, st);
    return launch_prefill_auto<BITS, YT>(h, X, static_cast<int>(M), Y, st);
}

template <int BITS>
int psample_fused(dllm_linear *h, const __half *Xh, int M, const PSampleEpi &ep, hipStream_t st) {
    return launch_prefill_auto<BITS, float, 1>(h, Xh, M, ep.x_prev, st, &ep);
}

template <int BITS>
int launch_gemm(const dllm_linear *h, const __half *X, size_t M, void *Y, int y_dtype, hipStream_t st) {
    if (y_dtype == DLLM_F32) return launch_gemm_t<BITS, float>(h, X, M, static_cast<float *>(Y), st);
    return launch_gemm_t<BITS, __half>(h, X, M, static_cast<__half *>(Y), st);
}

void free_linear(dllm_linear *h) {
    if (!h) return;
    (void)hipFree(h->wdev); (void)hipFree(h->wdec); (void)hipFree(h->sz); (void)hipFree(h->sf);
    (void)hipFree(h->bias); (void)hipFree(h->hr);
#if DLLM_LAB
    (void)hipFree(h->w16);
#endif
    delete h;
}

int check_shape(size_t K, size_t N, uint8_t bits, size_t group, int flags) {
    const int precision = flags & ~DLLM_LINEAR_PREFILL_ONLY;
    if (bits != 2 && bits != 4 && bits != 8)
        return fail(DLLM_ERR_UNSUPPORTED, "linear layer supports bits in {2, 4, 8}");
    if (K == 0 || N == 0) return fail(DLLM_ERR_SHAPE_MISMATCH, "K and N must be >= 1");
    if (K % kBK) return fail(DLLM_ERR_SHAPE_MISMATCH, "K must be a multiple of 64");
    if (group == 0 || group % kBK) return fail(DLLM_ERR_INVALID_PARAMS, "group must be a positive multiple of 64");
    if (K > (1u << 30) || N > (1u << 30)) return fail(DLLM_ERR_SHAPE_MISMATCH, "dimension too large");
    if (precision != DLLM_PRECISION_EXACT && precision != DLLM_PRECISION_F16W)
        return fail(DLLM_ERR_INVALID_PARAMS, "precision must be DLLM_PRECISION_EXACT or DLLM_PRECISION_F16W");
    return DLLM_OK;
}

int alloc_linear(size_t K, size_t N, uint8_t bits, size_t group, int flags, dllm_linear **out) {
    dllm_linear *h = new (std::nothrow) dllm_linear();
    if (!h) return fail(DLLM_ERR_HIP, "out of host memory");
    h->K = K; h->N = N; h->bits = bits; h->group = group;
    h->precision = flags & ~DLLM_LINEAR_PREFILL_ONLY;
    h->prefill_only = (flags & DLLM_LINEAR_PREFILL_ONLY) != 0;
    h->Npad = (N + kBN - 1) / kBN * kBN;
    h->G = (K + group - 1) / group;
    (void)hipGetDevice(&h->device);
    auto A = [&](void **p, size_t bytes) { return hipMalloc(p, std::max<size_t>(bytes, 16)); };
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = A(reinterpret_cast<void **>(&h->wdev), h->Npad * K * bits / 8);
    if (e == hipSuccess && !h->prefill_only)
        e = A(reinterpret_cast<void **>(&h->wdec), h->Npad * ((K + 127) / 128) * 128 * bits / 8);
    if (e == hipSuccess) e = A(reinterpret_cast<void **>(&h->sz), h->G * h->Npad * 4);
    if (e == hipSuccess) e = A(reinterpret_cast<void **>(&h->sf), h->G * h->Npad * 4);
    if (e == hipSuccess) e = A(reinterpret_cast<void **>(&h->bias), h->Npad * 4);
#if DLLM_LAB
    if (e == hipSuccess) e = A(reinterpret_cast<void **>(&h->w16), h->Npad * K * bits / 8);
#endif
    if (e != hipSuccess) {
        free_linear(h);
        return fail(DLLM_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    *out = h;
    return DLLM_OK;
}

// Device layouts from the canonical codes (`canon`, u32-addressable, ceil(K N bits / 32) words)
// and the scales / zero points [G][N] (all three only read by these launches): the prefill and
// decode code layouts, the {zp, scale} pairs, the f32 scales and, for the Horner-form shapes, the
// ratios with their validity flag.  Ends with one synchronisation of `st` (create is synchronous:
// the flag decides the handle's kernel once, and the caller's temporaries may be freed after it).
int finish_linear(dllm_linear *h, const uint32_t *canon, const float *scales, const uint8_t *zps, const float *bias,
                  hipStream_t st) {
    DLLM_HIP_TRY(hipMemsetAsync(h->bias, 0, h->Npad * 4, st));
    if (bias) DLLM_HIP_TRY(hipMemcpyAsync(h->bias, bias, h->N * 4, hipMemcpyDeviceToDevice, st));
    dim3 gf(static_cast<unsigned>((h->Npad + 255) / 256), static_cast<unsigned>(h->K / 64));
    build_fragments_kernel<<<gf, 256, 0, st>>>(canon, h->K, h->N, h->Npad, h->bits, h->wdev);
    DLLM_LAUNCH_CHECK();
#if DLLM_LAB
    build_fragments16_kernel<<<gf, 256, 0, st>>>(canon, h->K, h->N, h->Npad, h->bits, h->w16);
    DLLM_LAUNCH_CHECK();
#endif
    if (h->wdec) {
        dim3 gd(static_cast<unsigned>((h->Npad + 255) / 256), static_cast<unsigned>((h->K + 127) / 128));
        build_decode_from_wdev_kernel<<<gd, 256, 0, st>>>(h->wdev, h->K, h->Npad, h->bits, h->wdec);
        DLLM_LAUNCH_CHECK();
    }
    dim3 gs(static_cast<unsigned>((h->Npad + 255) / 256), static_cast<unsigned>(h->G));
    build_sz_kernel<<<gs, 256, 0, st>>>(scales, zps, h->G, h->N, h->Npad, h->sz);
    DLLM_LAUNCH_CHECK();
    build_sf_kernel<<<gs, 256, 0, st>>>(scales, h->G, h->N, h->Npad, h->sf);
    DLLM_LAUNCH_CHECK();
    int *flag = nullptr, unsafe = 1;
    if (horner_shape(h)) {
        DLLM_HIP_TRY(hipMalloc(reinterpret_cast<void **>(&h->hr), (h->G + 1) * h->Npad * 4));
        DLLM_HIP_TRY(hipMalloc(reinterpret_cast<void **>(&flag), sizeof(int)));
        hipError_t e = hipMemsetAsync(flag, 0, sizeof(int), st);
        if (e == hipSuccess) {
            build_horner_kernel<<<static_cast<unsigned>((h->Npad + 255) / 256), 256, 0, st>>>(h->sf, h->G, h->N,
                                                                                               h->Npad, h->hr, flag);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(&unsafe, flag, sizeof(int), hipMemcpyDeviceToHost, st);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(st);
            (void)hipFree(flag);
            return fail(DLLM_ERR_HIP, std::string("Horner ratios: ") + hipGetErrorString(e));
        }
    }
    const hipError_t e = hipStreamSynchronize(st);
    (void)hipFree(flag);
    if (e != hipSuccess) return fail(DLLM_ERR_HIP, std::string("linear create: ") + hipGetErrorString(e));
    if (h->hr) {
        h->hstate = unsafe ? 2 : 1;
        if (unsafe) {   // the fold form runs; the ratios are not kept
            (void)hipFree(h->hr);
            h->hr = nullptr;
        }
    }
    return DLLM_OK;
}

// Device temporaries of one create (the canonical codes, scales and zero points): owned by that
// create alone, released after finish_linear's synchronisation.
struct CreateTemps {
    void *p[2] = {nullptr, nullptr};
    ~CreateTemps() {
        for (void *q : p) (void)hipFree(q);
    }
    template <typename T>
    T *alloc(int i, size_t bytes) {
        return hipMalloc(&p[i], std::max<size_t>(bytes, 16)) == hipSuccess ? static_cast<T *>(p[i]) : nullptr;
    }
};

}  // namespace
}  // namespace dllm

using namespace dllm;

extern "C" {

int dllm_linear_create_ex(const float *W, const float *bias, size_t K, size_t N, uint8_t bits, size_t group,
                          int precision, dllm_linear_t *out, dllm_stream_t stream) {
    if (!out || !W) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    int rc = check_shape(K, N, bits, group, precision);
    if (rc) return rc;
    dllm_linear *h = nullptr;
    if ((rc = alloc_linear(K, N, bits, group, precision, &h))) return rc;
    hipStream_t st = as_stream(stream);
    // The canonical codes, scales and zero points only live for the creation (its own buffers).
    const size_t cbytes = canon_words(K, N, bits) * 4;
    CreateTemps tmp;
    uint32_t *canon = tmp.alloc<uint32_t>(0, cbytes);
    float *scales = tmp.alloc<float>(1, h->G * N * 4 + h->G * N);   // scales [G][N] f32, then zps u8
    if (!canon || !scales) { free_linear(h); return fail(DLLM_ERR_HIP, "hipMalloc (create temporaries)"); }
    uint8_t *zps = reinterpret_cast<uint8_t *>(scales + h->G * N);
    hipError_t e = hipMemsetAsync(canon, 0, cbytes, st);
    if (e != hipSuccess) { free_linear(h); return fail(DLLM_ERR_HIP, hipGetErrorString(e)); }
    if (N % 4 == 0 && group <= 128 && (bits == 2 || bits == 4 || bits == 8) &&
        (reinterpret_cast<uintptr_t>(W) & 15) == 0) {
        dim3 g(static_cast<unsigned>((N + 255) / 256), static_cast<unsigned>(h->G));
        quantize_weights4_kernel<<<g, 256, 0, st>>>(W, K, N, bits, static_cast<int>(group), canon, scales, zps);
    } else {
        dim3 g(static_cast<unsigned>((N + 255) / 256), static_cast<unsigned>(h->G));
        quantize_weights_kernel<<<g, 256, 0, st>>>(W, K, N, bits, static_cast<int>(group), canon, scales, zps);
    }
    if (hipGetLastError() != hipSuccess) { free_linear(h); return fail(DLLM_ERR_HIP, "quantize_weights launch"); }
    if ((rc = finish_linear(h, canon, scales, zps, bias, st))) { free_linear(h); return rc; }
    *out = h;
    return DLLM_OK;
}

int dllm_linear_create(const float *W, const float *bias, size_t K, size_t N, uint8_t bits, size_t group,
                       dllm_linear_t *out, dllm_stream_t stream) {
    return dllm_linear_create_ex(W, bias, K, N, bits, group, DLLM_PRECISION_EXACT, out, stream);
}

int dllm_linear_create_quantized_ex(const uint8_t *packed_codes, const float *scales, const uint8_t *zps,
                                    const float *bias, size_t K, size_t N, uint8_t bits, size_t group, int precision,
                                    dllm_linear_t *out, dllm_stream_t stream) {
    if (!out || !packed_codes || !scales || !zps) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    int rc = check_shape(K, N, bits, group, precision);
    if (rc) return rc;
    dllm_linear *h = nullptr;
    if ((rc = alloc_linear(K, N, bits, group, precision, &h))) return rc;
    hipStream_t st = as_stream(stream);
    // The caller's bitstream is read through u32 words: stage it in a zero-padded workspace.
    const size_t nbytes = (K * N * bits + 7) / 8, cbytes = canon_words(K, N, bits) * 4;
    CreateTemps tmp;
    uint32_t *canon = tmp.alloc<uint32_t>(0, cbytes);
    if (!canon) { free_linear(h); return fail(DLLM_ERR_HIP, "hipMalloc (create temporaries)"); }
    hipError_t e = hipMemsetAsync(canon, 0, cbytes, st);
    if (e == hipSuccess) e = hipMemcpyAsync(canon, packed_codes, nbytes, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) { free_linear(h); return fail(DLLM_ERR_HIP, hipGetErrorString(e)); }
    if ((rc = finish_linear(h, canon, scales, zps, bias, st))) { free_linear(h); return rc; }
    *out = h;
    return DLLM_OK;
}

int dllm_linear_create_quantized(const uint8_t *packed_codes, const float *scales, const uint8_t *zps,
                                 const float *bias, size_t K, size_t N, uint8_t bits, size_t group,
                                 dllm_linear_t *out, dllm_stream_t stream) {
    return dllm_linear_create_quantized_ex(packed_codes, scales, zps, bias, K, N, bits, group, DLLM_PRECISION_EXACT,
                                           out, stream);
}

// f16 view of X: as given, or cast from f32 through the per-(device, stream) staging workspace
// (slot 3): calls on one stream run in order, so they can share it, and calls on distinct streams
// never touch each other's (a handle keeps no mutable state).
static int prepare_x(dllm_linear *h, const void *X, size_t M, int x_dtype, hipStream_t st, const __half **Xh) {
    *Xh = static_cast<const __half *>(X);
    if (x_dtype != DLLM_F32) return DLLM_OK;
    const size_t need = M * h->K;
    __half *xs = reinterpret_cast<__half *>(device_workspace(st, need * sizeof(__half), 3));
    if (!xs) return DLLM_ERR_HIP;
    cast_f32_f16_kernel<<<grid_for(need / 4 + 1, 256, kCUs * 8), 256, 0, st>>>(static_cast<const float *>(X), need, xs);
    DLLM_LAUNCH_CHECK();
    *Xh = xs;
    return DLLM_OK;
}

int dllm_bias_cast(const float *y, size_t M, size_t N, const float *bias, void *out, int out_dtype,
                   dllm_stream_t stream) {
    if (out_dtype != DLLM_F32 && out_dtype != DLLM_F16) return fail(DLLM_ERR_UNSUPPORTED, "dtype must be DLLM_F32 or DLLM_F16");
    if (M == 0 || N == 0) return DLLM_OK;
    if (!y || !out) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    if (out_dtype == DLLM_F16 && static_cast<const void *>(y) == out)
        return fail(DLLM_ERR_INVALID_PARAMS, "an f16 output cannot alias the f32 input");
    const int vec = (N % 4 == 0) && ((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(bias) |
                                      reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    hipStream_t st = as_stream(stream);
    const unsigned g = grid_for(vec ? M * N / 4 : M * N, 256, kCUs * 8);
    if (out_dtype == DLLM_F32)
        bias_cast_kernel<float><<<g, 256, 0, st>>>(y, M, N, bias, static_cast<float *>(out), vec);
    else
        bias_cast_kernel<__half><<<g, 256, 0, st>>>(y, M, N, bias, static_cast<__half *>(out), vec);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_linear_forward(dllm_linear_t h, const void *X, size_t M, int x_dtype, void *Y, int y_dtype,
                        dllm_stream_t stream) {
    if (!h) return fail(DLLM_ERR_INVALID_PARAMS, "null handle");
    if ((x_dtype != DLLM_F32 && x_dtype != DLLM_F16) || (y_dtype != DLLM_F32 && y_dtype != DLLM_F16))
        return fail(DLLM_ERR_UNSUPPORTED, "dtype must be DLLM_F32 or DLLM_F16");
    if (M == 0) return DLLM_OK;
    if (!X || !Y) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    if (M > (1u << 30)) return fail(DLLM_ERR_SHAPE_MISMATCH, "M too large");
    if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(Y) & 15))
        return fail(DLLM_ERR_INVALID_PARAMS, "X and Y must be 16-byte aligned");
    hipStream_t st = as_stream(stream);
    const __half *Xh = nullptr;
    if (const int rc = prepare_x(h, X, M, x_dtype, st, &Xh)) return rc;
    switch (h->bits) {
    case 2: return launch_gemm<2>(h, Xh, M, Y, y_dtype, st);
    case 4: return launch_gemm<4>(h, Xh, M, Y, y_dtype, st);
    case 8: return launch_gemm<8>(h, Xh, M, Y, y_dtype, st);
    default: return fail(DLLM_ERR_UNSUPPORTED, "bits");
    }
}

int dllm_linear_forward_psample(dllm_linear_t h, const void *X, size_t M, int x_dtype, const float *x_t,
                                const float *coef, size_t rows_per_sample, int add_noise, uint64_t seed,
                                uint64_t offset, const float *noise, float *x_prev, dllm_stream_t stream) {
    return dllm_linear_forward_psample_ex(h, X, M, x_dtype, x_t, coef, rows_per_sample, add_noise, seed, offset,
                                          noise, x_prev, nullptr, stream);
}

int dllm_linear_forward_psample_ex(dllm_linear_t h, const void *X, size_t M, int x_dtype, const float *x_t,
                                   const float *coef, size_t rows_per_sample, int add_noise, uint64_t seed,
                                   uint64_t offset, const float *noise, float *x_prev, void *x_prev_f16,
                                   dllm_stream_t stream) {
    if (!h) return fail(DLLM_ERR_INVALID_PARAMS, "null handle");
    if (x_dtype != DLLM_F32 && x_dtype != DLLM_F16) return fail(DLLM_ERR_UNSUPPORTED, "x_dtype");
    if (M == 0) return DLLM_OK;
    if (!X || !x_t || !coef || !x_prev || rows_per_sample == 0) return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    if (M > (1u << 30)) return fail(DLLM_ERR_SHAPE_MISMATCH, "M too large");
    if (h->N % 4) return fail(DLLM_ERR_UNSUPPORTED, "fused p_sample needs N % 4 == 0");
    if (offset % 4) return fail(DLLM_ERR_INVALID_PARAMS, "offset must be a multiple of 4");
    if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(x_t) | reinterpret_cast<uintptr_t>(x_prev) |
         reinterpret_cast<uintptr_t>(noise) | reinterpret_cast<uintptr_t>(x_prev_f16)) & 15)
        return fail(DLLM_ERR_INVALID_PARAMS, "X, x_t, noise, x_prev and x_prev_f16 must be 16-byte aligned");
    hipStream_t st = as_stream(stream);
    const __half *Xh = nullptr;
    if (const int rc = prepare_x(h, X, M, x_dtype, st, &Xh)) return rc;
    bool fused = M > static_cast<size_t>(kDecodeMaxM);
#if DLLM_LAB
    fused = fused && !((h->variant >= 0 && h->variant <= 3) || h->variant == 5 || h->variant == 6);
#endif
    if (!fused) {
        // Paths without the fused epilogue: f32 eps through a per-stream workspace, then p_sample
        // (the same eps bits, hence the same result as the fused form on that path).
        float *eps = device_workspace(st, M * h->N * sizeof(float), 1);
        if (!eps) return DLLM_ERR_HIP;
        int rc = DLLM_OK;
        switch (h->bits) {
        case 2: rc = launch_gemm<2>(h, Xh, M, eps, DLLM_F32, st); break;
        case 4: rc = launch_gemm<4>(h, Xh, M, eps, DLLM_F32, st); break;
        default: rc = launch_gemm<8>(h, Xh, M, eps, DLLM_F32, st); break;
        }
        if (rc) return rc;
        // Per-row coefficients: expand the per-sample table when samples span several rows.
        if (rows_per_sample != 1) {
            float *rc3 = device_workspace(st, M * 3 * sizeof(float), 2);
            if (!rc3) return DLLM_ERR_HIP;
            expand_coef_kernel<<<grid_for(M, 256, kCUs), 256, 0, st>>>(coef, M, rows_per_sample, rc3);
            DLLM_LAUNCH_CHECK();
            coef = rc3;
        }
        if (const int prc = dllm_p_sample(x_t, eps, noise, coef, M, h->N, add_noise, seed, offset, x_prev, stream))
            return prc;
        if (x_prev_f16) {
            const size_t n = M * h->N;
            cast_f32_f16_kernel<<<grid_for(n / 4 + 1, 256, kCUs * 8), 256, 0, st>>>(x_prev, n,
                                                                                     static_cast<__half *>(x_prev_f16));
            DLLM_LAUNCH_CHECK();
        }
        return DLLM_OK;
    }
    const PSampleEpi ep{x_t, coef, static_cast<int>(rows_per_sample), add_noise ? 1 : 0, seed, offset, x_prev, noise,
                        static_cast<__half *>(x_prev_f16)};
    switch (h->bits) {
    case 2: return psample_fused<2>(h, Xh, (int)M, ep, st);
    case 4: return psample_fused<4>(h, Xh, (int)M, ep, st);
    case 8: return psample_fused<8>(h, Xh, (int)M, ep, st);
    default: return fail(DLLM_ERR_UNSUPPORTED, "bits");
    }
}

int dllm_linear_export(dllm_linear_t h, uint8_t *packed_codes, float *scales, uint8_t *zps, dllm_stream_t stream) {
    if (!h) return fail(DLLM_ERR_INVALID_PARAMS, "null handle");
    hipStream_t st = as_stream(stream);
    if (packed_codes) {
        const size_t nbytes = (h->K * h->N * h->bits + 7) / 8;
        export_codes_kernel<<<grid_for(nbytes, 256, kCUs * 16), 256, 0, st>>>(h->wdev, h->K, h->N, h->bits,
                                                                               packed_codes, nbytes);
        DLLM_LAUNCH_CHECK();
    }
    if (scales || zps) {
        dim3 gs(static_cast<unsigned>((h->N + 255) / 256), static_cast<unsigned>(h->G));
        export_params_kernel<<<gs, 256, 0, st>>>(h->sf, h->sz, h->G, h->N, h->Npad, scales, zps);
        DLLM_LAUNCH_CHECK();
    }
    return DLLM_OK;
}

int dllm_linear_info(dllm_linear_t h, size_t *K, size_t *N, uint8_t *bits, size_t *group) {
    if (!h) return fail(DLLM_ERR_INVALID_PARAMS, "null handle");
    if (K) *K = h->K;
    if (N) *N = h->N;
    if (bits) *bits = static_cast<uint8_t>(h->bits);
    if (group) *group = h->group;
    return DLLM_OK;
}

int dllm_linear_precision(dllm_linear_t h) {
    if (!h) {
        fail(DLLM_ERR_INVALID_PARAMS, "null handle");
        return -1;
    }
    return h->precision;
}

size_t dllm_linear_weight_bytes(dllm_linear_t h) {
    if (!h) return 0;
    // one layout is read per forward: the packed codes + one 4-B {zp, scale} word per (group, column)
    // (+ the 4-B f32 scale on the exact-weight path)
    return h->Npad * h->K * h->bits / 8 + h->G * h->Npad * (use_exact(h) ? 8 : 4);
}

size_t dllm_linear_device_bytes(dllm_linear_t h) {
    if (!h) return 0;
    size_t b = h->Npad * h->K * h->bits / 8 + h->G * h->Npad * 8 + h->Npad * 4;   // wdev, sz + sf, bias
    if (h->wdec) b += h->Npad * ((h->K + 127) / 128) * 128 * h->bits / 8;         // decode layout
    if (h->hr) b += (h->G + 1) * h->Npad * 4;                                         // Horner ratios (valid ones)
#if DLLM_LAB
    b += h->Npad * h->K * h->bits / 8;
#endif
    return b;
}

#if DLLM_LAB
int dllm_linear_set_kernel_variant(dllm_linear_t h, int variant) {
    if (!h) return fail(DLLM_ERR_INVALID_PARAMS, "null handle");
    if (variant >= 200 && variant < 264) {   // decode (NT, nsplit) override (measurement only)
        h->dcfg = variant - 199;
        return DLLM_OK;
    }
    if (variant >= 16 && variant < 24) {   // decode ablation mask (measurement only)
        h->dlab = variant - 16;
        return DLLM_OK;
    }
    if (variant >= 32 && variant < 96) {   // ring-kernel ablation mask (measurement only)
        h->rlab = variant - 32;
        return DLLM_OK;
    }
    if (variant >= 100 && variant < 196) {   // ping-pong ablation: 100 / 132 / 164 + lab -> variant 9 / 10 / 11
        h->variant = 9 + (variant - 100) / 32;
        h->pplab = (variant - 100) % 32;
        return DLLM_OK;
    }
    if (variant < -1 || (variant > 15 && (variant < 24 || variant > 31) && (variant < 300 || variant > 331 || variant == 313) &&
                         (variant < 340 || variant > 345)))
        return fail(DLLM_ERR_INVALID_PARAMS, "variant must be -1..15, 24..31, 300..312, 314..331 or 340..345 (16..23, 32..95, 100..195, 200..263: ablations)");
    h->variant = variant;
    h->dlab = h->rlab = h->pplab = h->dcfg = 0;
    return DLLM_OK;
}
#endif

int dllm_linear_destroy(dllm_linear_t h) {
    free_linear(h);
    return DLLM_OK;
}

}  // extern "C"
