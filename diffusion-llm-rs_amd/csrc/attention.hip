// attention.hip -- quantized-KV dequant-attention for gfx950 (a9, build-defined consumer).
//
// The reference dequantizes the per-tensor-quantized K and V of its cache every timestep
// (QuantizedKVCacheEntry::dequantize_keys/values, diffuse-llm-rs/src/quantization.rs:160-175) and
// hands them to DiffusionModel::forward_with_cache (diffuse-llm-rs/src/lib.rs:910-915).  Here the
// dequantization y = (q - zp) * scale (a2) is fused into a flash-style bidirectional SDPA,
// O = softmax(Q K^T / sqrt(D)) V per head.  Because K and V each carry ONE per-tensor scale,
//   Q K^T = s_k * (Q (q_k - z_k)^T)   and   P V = s_v * (P (q_v - z_v)),
// so only the exact integers (q - z) are staged (exact in f16) and the scales fold into the softmax
// exponent and the final normalisation: fewer roundings than dequantizing to f16 first.
//
// Layout: Q, O f16 [S][H][D]; K, V codes in the canonical packed bitstream of the flattened
// [S][H][D] tensor (one per-tensor {scale, zp} pair each, on the device), D = 128.
// Workgroup = 8 waves = 256 queries of one head; every 64-key block of K and V is staged once in
// LDS (K as [key][d], V transposed as [d][key]) and shared by the 8 waves.
// Per wave (32 queries): S^T = K Q^T with 32x32x16 f16 MFMA (keys in registers, the query on the
// lane, so the softmax row reductions are lane-local plus one cross-half shuffle), then O = P V with
// the S^T accumulator converted in place to the A operand (no LDS round trip for P).  The O rescale
// is skipped when no query's running max moved (exact: the factor is then 1).
// Software pipeline: iteration kb issues S^T of block kb+1 on the matrix pipe and runs the
// softmax of block kb on the VALU meanwhile, then P V of block kb.  K is therefore staged two
// blocks ahead and V one block ahead, each in its own two-buffer ring; one barrier per block; no
// buffer is written in the iteration that reads it.
// Dequantize once (v4): every (head, 64-key block) of K and V is unpacked to the exact f16 (q - z)
// image of its LDS tiles ONCE, by kv_stage_kernel, into a workspace; the attention loop then
// streams those images into LDS with LDS-DMA (no VALU).  Unpacking inside the attention loop
// repeated it for each of a head's S/256 query workgroups (32x at S = 8192) and cost ~30 % of the
// kernel (measured by ablation: DLLM_ATTN_LAB=2).
#include "common.hpp"

#ifndef DLLM_LAB
#define DLLM_LAB 0
#endif

#include <cstdlib>

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float float16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

#ifndef DLLM_ATTN_MF16_ABL
#define DLLM_ATTN_MF16_ABL 0
#endif
#if DLLM_ATTN_MF16_ABL
// A/B build only (results wrong, timing only): kv_attention5's 32x32x16 MFMAs each replaced by two
// 16x16x32 on the same operands -- the MFMA shape's effect on the held clock.
__device__ __forceinline__ float16_t attn_mf16_abl(const half8_t &a, const half8_t &b, float16_t c) {
    typedef float fx4 __attribute__((ext_vector_type(4)));
    typedef float fx8 __attribute__((ext_vector_type(8)));
    fx4 c0 = __builtin_shufflevector(c, c, 0, 1, 2, 3), c1 = __builtin_shufflevector(c, c, 4, 5, 6, 7);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c1, 0, 0, 0);
    const fx8 lo = __builtin_shufflevector(c0, c1, 0, 1, 2, 3, 4, 5, 6, 7);
    const fx8 hi = __builtin_shufflevector(c, c, 8, 9, 10, 11, 12, 13, 14, 15);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
}
#define ATTN5_MFMA(a, b, c) attn_mf16_abl((a), (b), (c))
#else
#define ATTN5_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_f16((a), (b), (c), 0, 0, 0)
#endif

namespace dllm {
namespace {

constexpr int kD = 128;          // head dim
constexpr int kKB = 64;          // keys per block
constexpr int kWaves = 8;
constexpr int kQT = 32 * kWaves; // queries per workgroup
constexpr int kKRow = kD + 8;    // K row stride (halves): 272 B, conflict-free b128 fragment reads
constexpr int kVRow = kKB + 8;   // Vt row stride (halves): 144 B

template <int NB>
struct AttnSmemN {
    _Float16 k[NB][kKB][kKRow];   // NB x 17 KiB
    _Float16 vt[NB][kD][kVRow];   // NB x 18 KiB
    float bcast[kWaves][32];      // per-wave per-query factors (alpha, then 1/l)
};
using AttnSmem = AttnSmemN<2>;

// Workspace image of one (head, key block): the K tile then the transposed V tile, byte for byte
// the LDS layout (row padding included), so one 1-KiB LDS-DMA piece per wave-instruction moves it.
constexpr int kKImg = kKB * kKRow * 2;          // 17408 B = 17 pieces
constexpr int kVImg = kD * kVRow * 2;           // 18432 B = 18 pieces
constexpr int kImg = kKImg + kVImg;
static_assert(kKImg % 1024 == 0 && kVImg % 1024 == 0, "images must be whole 1-KiB DMA pieces");

// Codes of one thread's share of a block, loaded to registers ahead of the MFMAs.
// K: thread t < 256 owns key t>>2, dims 32*(t&3) .. +32 (one row chunk).
// V: thread t >= 256 owns keys 4*((t-256)>>4) .. +4, dims 8*((t-256)&15) .. +8 (a 4x8 micro-tile).
template <int BITS>
struct Raw {
    uint32_t w[BITS == 4 ? 4 : 8];
};

// 32-bit byte offsets through buffer resources: keys at or past S read as 0 (out of range, no
// memory access) instead of being clamped, and no 64-bit address math per block.
template <int BITS>
__device__ __forceinline__ void load_raw(Raw<BITS> &r, __amdgpu_buffer_rsrc_t krs, __amdgpu_buffer_rsrc_t vrs,
                                         int tid, int jk, int jv, int H, int h) {
    constexpr int kRowB = kD * BITS / 8;   // packed bytes per (key, head) row
    if (tid < 256) {
        const int key = tid >> 2, d0 = 32 * (tid & 3);
        const uint32_t off = static_cast<uint32_t>(((jk + key) * H + h) * kRowB + d0 * BITS / 8);
        if constexpr (BITS == 4) {
            const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(krs, off, 0, 0));
            r.w[0] = v.x; r.w[1] = v.y; r.w[2] = v.z; r.w[3] = v.w;
        } else {
            const uint4 a = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(krs, off, 0, 0));
            const uint4 b = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(krs, off + 16, 0, 0));
            r.w[0] = a.x; r.w[1] = a.y; r.w[2] = a.z; r.w[3] = a.w; r.w[4] = b.x; r.w[5] = b.y; r.w[6] = b.z; r.w[7] = b.w;
        }
    } else {
        const int t = tid - 256, k4 = 4 * (t >> 4), d0 = 8 * (t & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t off = static_cast<uint32_t>(((jv + k4 + i) * H + h) * kRowB + d0 * BITS / 8);
            if constexpr (BITS == 4) {
                r.w[i] = __builtin_amdgcn_raw_buffer_load_b32(vrs, off, 0, 0);
            } else {
                const uint2 v = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(vrs, off, 0, 0));
                r.w[2 * i] = v.x; r.w[2 * i + 1] = v.y;
            }
        }
    }
}

// Position of key k (0..15) within its 16-key group of the V image: bits 2 and 3 swapped.
__host__ __device__ constexpr int kv_pos(int k) { return (k & 3) | ((k & 4) << 1) | ((k & 8) >> 1); }

// Code c (0..7) of an 8-code group of the thread's raw words, as the f16 pair trick input.
template <int BITS>
__device__ __forceinline__ half2_t pair_qz(uint32_t lo_word_codes, int shift, half2_t nz) {
    // (code_a at bit shift, code_b at bit shift + BITS) -> f16 pair (1024 + code) - (1024 + z)
    const uint32_t m = (1u << BITS) - 1u;
    const uint32_t a = (lo_word_codes >> shift) & m, b = (lo_word_codes >> (shift + BITS)) & m;
    const uint32_t t = (a | (b << 16)) | 0x64006400u;
    return __builtin_bit_cast(half2_t, t) + nz;   // exact
}

// Position of key k (0..31) within its 32-key group of the 16x16x32 kernel's V image (lab A/B,
// lab/attn16.inc): key
// 16 a + 4 g + i at 8 g + 4 a + i, so that the 8 keys a P V B-fragment lane of group g needs
// ({4 g .. 4 g + 3, 16 + 4 g .. 16 + 4 g + 3}, the two 16-key score blocks' rows of that lane group)
// sit in one 16-B run.
__host__ __device__ constexpr int kv_pos16(int k) { return 8 * ((k >> 2) & 3) + 4 * ((k >> 4) & 1) + (k & 3); }

// VL16: the V image in kv_pos16 order (kv_attention16_kernel); else kv_pos (kv_attention5_kernel).
template <int BITS, bool VL16 = false>
__device__ __forceinline__ void store_raw(const Raw<BITS> &r, _Float16 (&bk)[kKB][kKRow], _Float16 (&bvt)[kD][kVRow],
                                          int tid, half2_t kz, half2_t vz) {
    constexpr int CPW = 32 / BITS;   // codes per word
    if (tid < 256) {
        const int key = tid >> 2, d0 = 32 * (tid & 3);
#pragma unroll
        for (int g = 0; g < 4; ++g) {   // 4 x 8 codes -> 4 x b128 stores
            half8_t out;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int c = 8 * g + 2 * p;   // code index within the 32
                const half2_t v = pair_qz<BITS>(r.w[c / CPW], BITS * (c % CPW), kz);
                out[2 * p] = v[0];
                out[2 * p + 1] = v[1];
            }
            *reinterpret_cast<half8_t *>(&bk[key][d0 + 8 * g]) = out;
        }
    } else {
        const int t = tid - 256, k4 = 4 * (t >> 4), d0 = 8 * (t & 15);
        _Float16 v[4][8];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int c = 2 * p;
                const uint32_t word = (BITS == 4) ? r.w[i] : r.w[2 * i + (c / CPW)];
                const half2_t x = pair_qz<BITS>(word, BITS * (c % CPW), vz);
                v[i][2 * p] = x[0];
                v[i][2 * p + 1] = x[1];
            }
        // transposed, 4 consecutive keys of one dim per 8-B store, at the key position of the V
        // image: keys 4..7 and 8..11 of every 16 swap places (kv_pos), so that the 8 keys a PV
        // fragment lane needs (16 s + 4 hh + {0..3, 8..11}) sit in one 16-B run.
        const int kp4 = VL16 ? (k4 & ~31) | kv_pos16(k4 & 31) : (k4 & ~15) | kv_pos(k4 & 15);
#pragma unroll
        for (int dd = 0; dd < 8; ++dd)
            *reinterpret_cast<half4_t *>(&bvt[d0 + dd][kp4]) = half4_t{v[0][dd], v[1][dd], v[2][dd], v[3][dd]};
    }
}

// Pre-pass: unpack block kb of head h to its LDS image (through LDS, so the stores to the
// workspace are coalesced 16-B rows).  Keys past S read as code 0 (buffer range check); the
// attention kernel masks their scores and their P is 0.
template <int BITS, bool VL16 = false>
__global__ void __launch_bounds__(512) kv_stage_kernel(const uint8_t *__restrict__ Kq, const float *__restrict__ kp,
                                                      const uint8_t *__restrict__ Vq, const float *__restrict__ vp,
                                                      int S, int H, int nkb, uint8_t *__restrict__ img) {
    __shared__ __attribute__((aligned(16))) _Float16 tk[kKB][kKRow];
    __shared__ __attribute__((aligned(16))) _Float16 tv[kD][kVRow];
    const int tid = threadIdx.x, kb = blockIdx.x, h = blockIdx.y;
    const _Float16 nkz = static_cast<_Float16>(-(1024.0f + kp[1]));
    const _Float16 nvz = static_cast<_Float16>(-(1024.0f + vp[1]));
    const half2_t kz{nkz, nkz}, vz{nvz, nvz};
    const int nbytes = static_cast<int>(static_cast<size_t>(S) * H * kD * BITS / 8);
    const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(Kq), 0, nbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(Vq), 0, nbytes, 0x00020000);
    Raw<BITS> raw;
    load_raw<BITS>(raw, krs, vrs, tid, kb * kKB, kb * kKB, H, h);
    store_raw<BITS, VL16>(raw, tk, tv, tid, kz, vz);
    __syncthreads();
    uint8_t *dst = img + (static_cast<size_t>(h) * nkb + kb) * kImg;
    const uint4 *sk = reinterpret_cast<const uint4 *>(&tk[0][0]);
    const uint4 *sv = reinterpret_cast<const uint4 *>(&tv[0][0]);
    for (int i = tid; i < kKImg / 16; i += 512) reinterpret_cast<uint4 *>(dst)[i] = sk[i];
    for (int i = tid; i < kVImg / 16; i += 512) reinterpret_cast<uint4 *>(dst + kKImg)[i] = sv[i];
}

#if DLLM_LAB   // attention v4 (the unscheduled form of v5; A/B and ablation masks)
#include "lab/attn_v4.inc"
#endif

// Row reductions across the two lane halves (lane l and l ^ 32 hold the two key halves of one
// query): v_permlane32_swap (VALU) instead of a ds_bpermute round trip through the LDS unit.
// Both halves compute the same expression of the same two values, so they agree bit for bit.
__device__ __forceinline__ float swap_halves_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float swap_halves_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// v5: the same algorithm and LDS ring as kv_attention_kernel with an explicit in-wave schedule:
// S^T of block kb+1 and the softmax of block kb share one scheduling region, the MFMAs paced by
// sched_group_barrier with softmax VALU and K-fragment reads in their gaps (hipcc had issued the
// 16 QK MFMAs back to back and then the whole softmax); the max and sum reductions are trees
// (depth 5 instead of 32-long chains); the k-loop is unrolled by two so the score register sets
// swap roles instead of being copied.
//
// STAG (A/B, lab case 198): waves 4-7 (group B, the second wave of each SIMD) run half a k-block behind
// waves 0-3 (group A), so that on every SIMD one wave's region 1 (QK MFMAs + the softmax's exp /
// max / sum VALU) overlaps the other's region 2 (P V MFMAs, little VALU) instead of both waves
// reaching the softmax together.  One barrier per half block (group B enters through one extra,
// group A leaves through one extra); K and V rings of THREE buffers each (K(j), V(j) in buffer
// j % 3, 105 KiB).  Half-block interval 2 kb: A runs R1(kb), B R2(kb - 1); interval 2 kb + 1: A
// R2(kb), B R1(kb).  Group A stages K(kb + 2) at the start of its R1(kb) (the buffer's previous
// block, K(kb - 1), was last read by B in interval 2 kb - 3) and waits for it before the barrier
// ending interval 2 kb + 1 (first read by A in 2 kb + 2); group B stages V(kb + 2) at the start
// of its R1(kb) (V(kb - 1) last read by B in 2 kb) and waits for it before the barrier ending
// interval 2 kb + 2 (first read by A in 2 kb + 5).  Same arithmetic per query as STAG = false:
// the outputs are bit-identical.
// DLLM_ATTN_BDMA = 1: K / V staging through a buffer descriptor with compile-time pieces (C4: 1.005
// -> 0.971 ms and 1.037 -> 1.017 ms on two boxes, bit-identical; a one-M0-save burst of the two
// whole rounds measured slower than this, profiles/r05_bdma/).
#ifndef DLLM_ATTN_BDMA
#define DLLM_ATTN_BDMA 1
#endif
constexpr bool kAttnBdma = DLLM_ATTN_BDMA != 0;

template <int LAB = 0, bool STAG = false>
__global__ void __launch_bounds__(kWaves * 64)
kv_attention5_kernel(const _Float16 *__restrict__ Q, const uint8_t *__restrict__ img, const float *__restrict__ kp,
                    const float *__restrict__ vp, int S, int H, _Float16 *__restrict__ O) {
    constexpr int NB = STAG ? 3 : 2;
    const int nkb = (S + kKB - 1) / kKB;
    __shared__ __attribute__((aligned(16))) AttnSmemN<NB> sm;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = blockIdx.y;
    const int q0 = blockIdx.x * kQT + wave * 32;
    const int ql = lane & 31, hh = lane >> 5;
    const float ks = kp[0], vs = vp[0];
    // exp2 domain, K scale folded in: p = exp2(c * raw - m), c = log2(e) * s_k / sqrt(D).
    const float c = 1.4426950408889634f * ks / sqrtf(static_cast<float>(kD));

    // Q^T fragments (B operand of S^T = K Q^T): lane holds Q[q = q0 + ql][d = 16 t + 8 hh + j].
    half8_t qf[kD / 16];
    {
        const int qrow = min(q0 + ql, S - 1);
        const _Float16 *qp = Q + (static_cast<size_t>(qrow) * H + h) * kD + 8 * hh;
#pragma unroll
        for (int t = 0; t < kD / 16; ++t) qf[t] = *reinterpret_cast<const half8_t *>(qp + 16 * t);
    }

    float16_t o[kD / 32];   // O tiles: d-tile dt, lane = d (within tile), rows = query via regs
#pragma unroll
    for (int dt = 0; dt < kD / 32; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[dt][e] = 0.0f;
    float m_run = -INFINITY, l_run = 0.0f;   // for query q0 + ql (same in both lane halves)

    // S^T (2 x 32 keys x 32 queries) of a staged K block: st[u][r] is key 32u + (r&3) + 8(r>>2) + 4hh
    // of the block, query q0 + ql.
    auto qk = [&](float16_t (&st)[2], const _Float16 (&kb_)[kKB][kKRow]) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int e = 0; e < 16; ++e) st[u][e] = 0.0f;
#pragma unroll
            for (int t = 0; t < kD / 16; ++t) {
                const half8_t kf = *reinterpret_cast<const half8_t *>(&kb_[32 * u + ql][16 * t + 8 * hh]);
                st[u] = ATTN5_MFMA(kf, qf[t], st[u]);
            }
        }
    };

    // LDS-DMA of the workspace images: wave w moves pieces w, w + 8, ... (1 KiB each).
    const uint8_t *himg = img + static_cast<size_t>(h) * nkb * kImg + lane * 16;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(wave);
    // pieces p0, p0 + step, ... of an image (the whole workgroup: wv, 8; one group: wv % 4, 4)
    // BDMA: the whole-workgroup form through a buffer descriptor of the head's images -- the block
    // and piece in the scalar offset, one fixed per-lane offset, the pieces unrolled at compile time
    // -- instead of a run-time loop of global_load_lds with a 64-bit address add per piece.
    const __amdgpu_buffer_rsrc_t irs = raw_rsrc(img + static_cast<size_t>(h) * nkb * kImg);
    auto u = [](uint32_t v) { return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v))); };
    auto dma_b = [&](uint32_t off0, uint32_t dst0, auto n_tag) __attribute__((always_inline)) {
        constexpr int n = decltype(n_tag)::value;
#pragma unroll
        for (int i = 0; i < (n + kWaves - 1) / kWaves; ++i) {
            const uint32_t p = wv + kWaves * i;
            if ((i + 1) * kWaves <= n || p < static_cast<uint32_t>(n))
                blds16_asm(irs, static_cast<uint32_t>(lane * 16), u(off0 + p * 1024), u(dst0 + p * 1024));
        }
    };
    auto dma_k = [&](int blk, int buf, uint32_t p0 = 0xffffffffu, uint32_t step = kWaves) {
        const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_addr(&sm.k[buf][0][0]));
        if (kAttnBdma && p0 == 0xffffffffu && step == kWaves) {
            dma_b(static_cast<uint32_t>(blk * kImg), dst, std::integral_constant<int, kKImg / 1024>{});
            return;
        }
        const uint8_t *src = himg + static_cast<size_t>(blk) * kImg;
        for (uint32_t p = p0 == 0xffffffffu ? wv : p0; p < kKImg / 1024; p += step) glds16_asm(src + p * 1024, dst + p * 1024);
    };
    auto dma_v = [&](int blk, int buf, uint32_t p0 = 0xffffffffu, uint32_t step = kWaves) {
        const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_addr(&sm.vt[buf][0][0]));
        if (kAttnBdma && p0 == 0xffffffffu && step == kWaves) {
            dma_b(static_cast<uint32_t>(blk * kImg + kKImg), dst, std::integral_constant<int, kVImg / 1024>{});
            return;
        }
        const uint8_t *src = himg + static_cast<size_t>(blk) * kImg + kKImg;
        for (uint32_t p = p0 == 0xffffffffu ? wv : p0; p < kVImg / 1024; p += step) glds16_asm(src + p * 1024, dst + p * 1024);
    };
    const bool grp_b = STAG && wave >= kWaves / 2;
    auto raw_barrier = []() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // Prologue: K and V of block 0 and K of block 1 staged (STAG: and V of block 1); S^T of block 0.
    dma_k(0, 0);
    dma_v(0, 0);
    if (nkb > 1) dma_k(1, 1);
    if (STAG && nkb > 1) dma_v(1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // One k-block: DMAs of the blocks ahead, then region 1 (S^T of block kb+1 on the matrix pipe,
    // the softmax of block kb on the VALU in the MFMA gaps), the O rescale (rare), region 2 (P V of
    // block kb with the V fragment reads and the P conversion in the gaps), one barrier.  The
    // scores of the next block land in `sn`; the caller swaps the two register sets.
    auto iter = [&](float16_t (&st)[2], float16_t (&sn)[2], int kb) {
        const int j0 = kb * kKB;
        const bool more1 = kb + 1 < nkb, more2 = kb + 2 < nkb;
        // Staging of K(kb+2) and V(kb+1): LDS-DMA as in v4 (default), or (LAB & 64, A/B) register
        // loads now and LDS writes at the end of the block (each wave owns the 1-KiB pieces wave,
        // wave + 8, wave + 16 of each image: a plain 16-B load and a ds_write_b128 per piece).
        // Measured at S 8192 H 32: LDS-DMA 1111 us, register staging 1176 us.
        u32x4_t kr[3], vr[3];
        if constexpr (STAG) {
            if (more2) {
                if (!grp_b) dma_k(kb + 2, (kb + 2) % 3, wv, kWaves / 2);
                else dma_v(kb + 2, (kb + 2) % 3, wv - kWaves / 2, kWaves / 2);
            }
        } else if constexpr (!(LAB & 2)) {
            if constexpr (!(LAB & 64)) {
                if (more2) dma_k(kb + 2, kb & 1);
                if (more1) dma_v(kb + 1, (kb + 1) & 1);
            } else {
                // Branch-free (a load under a branch makes hipcc wait for it at once): past the last
                // block the last block is re-staged into a free buffer, and piece indices past an
                // image's end repeat its last piece (several waves then store the same bytes).
                const uint8_t *ks_ = himg + static_cast<size_t>(min(kb + 2, nkb - 1)) * kImg;
                const uint8_t *vs_ = himg + static_cast<size_t>(min(kb + 1, nkb - 1)) * kImg + kKImg;
                // The loads are inline asm so that hipcc, which would sink them next to their
                // stores and wait for them there, leaves them where they are; their one wait
                // (vmcnt(0), naming every destination) precedes the LDS stores at the block's end.
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const uint8_t *kp_ = ks_ + min(static_cast<int>(wv) + 8 * i, kKImg / 1024 - 1) * 1024;
                    const uint8_t *vp_ = vs_ + min(static_cast<int>(wv) + 8 * i, kVImg / 1024 - 1) * 1024;
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(kr[i]) : "v"(kp_) : "memory");
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(vr[i]) : "v"(vp_) : "memory");
                }
            }
        }
        if (__builtin_expect(j0 + kKB > S, 0)) {   // last, partial block only (a real branch)
            asm volatile("" ::: "memory");
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = j0 + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * hh;
                    st[u][r] = key < S ? st[u][r] : -INFINITY;
                }
        }
        // ---- region 1.  After the last block the K buffer is stale: sn is computed and dropped.
        const auto &kn = sm.k[(kb + 1) % NB];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int e = 0; e < 16; ++e) sn[u][e] = 0.0f;
#pragma unroll
            for (int t = 0; t < kD / 16; ++t) {
                const half8_t kf = *reinterpret_cast<const half8_t *>(&kn[32 * u + ql][16 * t + 8 * hh]);
                if constexpr (LAB & 8) {   // measurement only: no QK MFMAs (reads kept live)
                    asm volatile("" ::"v"(kf));
                    sn[u][t] += 1.0f;
                } else {
                    sn[u] = ATTN5_MFMA(kf, qf[t], sn[u]);
                }
            }
        }
        float alpha = 1.0f;
        if constexpr (LAB & 1) {   // measurement only: no softmax (P = raw scores)
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(st[u][r]));
        } else {
        float mt[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) mt[r] = fmaxf(st[0][r], st[1][r]);
#pragma unroll
        for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
            for (int r = 0; r < w; ++r) mt[r] = fmaxf(mt[r], mt[r + w]);
        const float mloc = swap_halves_max(mt[0]);
        const float m_new = fmaxf(m_run, mloc * c);
        // raw v_exp_f32 (P below 2^-126 is 0 in the f16 P anyway); exp2(0) = 1 exactly.
        alpha = __builtin_amdgcn_exp2f(m_run - m_new);
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) st[u][r] = __builtin_amdgcn_exp2f(fmaf(st[u][r], c, -m_new));
        m_run = m_new;
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 1);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
            __builtin_amdgcn_sched_group_barrier(0x002, 5, 1);
        }
        // Keep the softmax in region 1: without these the compiler sinks the 32 exponentials (and
        // their fmas) past the O-rescale branch into region 2, where they run back to back ahead of
        // the P V MFMAs while region 1's S^T MFMAs go without VALU fillers.
        if constexpr (!(LAB & 1) && !(LAB & 512)) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(st[u][r]));
        }
        if constexpr (STAG) raw_barrier();   // the half-block barrier
        // ---- rescale O rows by their query's alpha, only if some query's max moved ----
        if (!(LAB & 1) && !__all(alpha == 1.0f)) {
            if (hh == 0) sm.bcast[wave][ql] = alpha;
            __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 a4 = *reinterpret_cast<const float4 *>(&sm.bcast[wave][8 * g + 4 * hh]);
#pragma unroll
                for (int dt = 0; dt < kD / 32; ++dt) {
                    o[dt][4 * g + 0] *= a4.x; o[dt][4 * g + 1] *= a4.y;
                    o[dt][4 * g + 2] *= a4.z; o[dt][4 * g + 3] *= a4.w;
                }
            }
        }
        // ---- region 2: O += P (q_v - z_v), the P^T accumulator as the A operand ----
        // Static priority 1 over region 2 (P V MFMAs): a SIMD whose other wave is in its softmax VALU
        // keeps issuing MFMAs (measured at S 8192, H 32: 1.0447 vs 1.0645 ms; LAB & 256 drops it, A/B).
        if constexpr (!(LAB & 256)) __builtin_amdgcn_s_setprio(1);
        const auto &vt = sm.vt[kb % NB];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            const int u = s2 >> 1, sl = s2 & 1;
            half8_t pa;
#pragma unroll
            for (int j = 0; j < 8; ++j) pa[j] = static_cast<_Float16>(st[u][8 * sl + j]);
#pragma unroll
            for (int dt = 0; dt < kD / 32; ++dt) {
                // element j <-> key 16s + 8(j>>2) + 4hh + (j&3), d = 32dt + ql
                // one 16-B read: keys 16s + 4hh + {0..3, 8..11} are adjacent in the kv_pos layout
                const half8_t vb = *reinterpret_cast<const half8_t *>(&vt[32 * dt + ql][16 * s2 + 8 * hh]);
                if constexpr (LAB & 4) {   // measurement only: no PV MFMAs (operands kept live)
                    asm volatile("" ::"v"(vb), "v"(pa));
                } else {
                    o[dt] = ATTN5_MFMA(pa, vb, o[dt]);
                }
            }
        }
        // the row sum of P rides in region 2's gaps (only l_run needs it)
        float ls[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) ls[r] = st[0][r] + st[1][r];
#pragma unroll
        for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
            for (int r = 0; r < w; ++r) ls[r] = ls[r] + ls[r + w];
        l_run = l_run * alpha + swap_halves_sum(ls[0]);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 2);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 2);
            __builtin_amdgcn_sched_group_barrier(0x002, 5, 2);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
        }
        if constexpr (!(LAB & 256)) __builtin_amdgcn_s_setprio(0);
        if constexpr (!(LAB & 2) && (LAB & 64)) {
            asm volatile("s_waitcnt vmcnt(0)"
                         : "+v"(kr[0]), "+v"(kr[1]), "+v"(kr[2]), "+v"(vr[0]), "+v"(vr[1]), "+v"(vr[2])
                         :
                         : "memory");
            uint8_t *kd = reinterpret_cast<uint8_t *>(&sm.k[kb & 1][0][0]) + lane * 16;
            uint8_t *vd = reinterpret_cast<uint8_t *>(&sm.vt[(kb + 1) & 1][0][0]) + lane * 16;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                *reinterpret_cast<u32x4_t *>(kd + min(static_cast<int>(wv) + 8 * i, kKImg / 1024 - 1) * 1024) = kr[i];
                *reinterpret_cast<u32x4_t *>(vd + min(static_cast<int>(wv) + 8 * i, kVImg / 1024 - 1) * 1024) = vr[i];
            }
        }
        if constexpr (STAG) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            raw_barrier();
        } else {
            if constexpr (!(LAB & 16)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if constexpr (!(LAB & 32)) __syncthreads();
        }
    };
    // LAB & 128 (A/B): static priority 1 for the second-dispatched half (waves 4-7), which
    // otherwise loses every VALU arbitration to its older SIMD partner (MI355X_MICROARCH.md, two
    // waves per SIMD, item 4).
    if constexpr (LAB & 128) {
        if (wave >= kWaves / 2) __builtin_amdgcn_s_setprio(1);
    }
    float16_t sa[2], sb[2];
    qk(sa, sm.k[0]);
    if (grp_b) raw_barrier();   // group B enters half a block behind
    for (int kb = 0; kb < nkb; kb += 2) {
        iter(sa, sb, kb);
        if (kb + 1 < nkb) iter(sb, sa, kb + 1);
    }
    if (STAG && !grp_b) raw_barrier();   // group A joins group B's last barrier

    // ---- normalise (1/l and the V scale) and store: o[dt][r] -> query q0 + (r&3) + 8(r>>2) + 4hh ----
    if (hh == 0) sm.bcast[wave][ql] = vs / l_run;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    if constexpr (!(LAB & (4096 | 32)) && !STAG) {
        // The wave's 32 x 128 f16 tile goes through the drained K/V ring (every wave passed the loop's
        // last barrier, so nothing reads it any more; rows padded to 272 B so the two half-waves'
        // rows land 16 banks apart) and leaves as whole 256-B rows in 16-B lane pieces: 8 global
        // stores per lane instead of 64 two-byte ones (guide T21).
        static_assert(kWaves * 32 * kKRow * 2 <= sizeof(sm.k) + sizeof(sm.vt), "O staging must fit the K/V ring");
        _Float16 *tile = reinterpret_cast<_Float16 *>(&sm) + wave * 32 * kKRow;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 inv = *reinterpret_cast<const float4 *>(&sm.bcast[wave][8 * g + 4 * hh]);
            const float iv[4] = {inv.x, inv.y, inv.z, inv.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 8 * g + 4 * hh + i;
#pragma unroll
                for (int dt = 0; dt < kD / 32; ++dt)
                    tile[r * kKRow + 32 * dt + ql] = static_cast<_Float16>(o[dt][4 * g + i] * iv[i]);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int c = it * 64 + lane, r = c >> 4, cc = c & 15;
            if (q0 + r < S)
                *reinterpret_cast<u32x4_t *>(O + (static_cast<size_t>(q0 + r) * H + h) * kD + 8 * cc) =
                    *reinterpret_cast<const u32x4_t *>(tile + r * kKRow + 8 * cc);
        }
        return;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 inv = *reinterpret_cast<const float4 *>(&sm.bcast[wave][8 * g + 4 * hh]);
        const float iv[4] = {inv.x, inv.y, inv.z, inv.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q = q0 + 8 * g + 4 * hh + i;
            if (q >= S) continue;
            _Float16 *op = O + (static_cast<size_t>(q) * H + h) * kD + ql;
#pragma unroll
            for (int dt = 0; dt < kD / 32; ++dt) op[32 * dt] = static_cast<_Float16>(o[dt][4 * g + i] * iv[i]);
        }
    }
}


#if DLLM_LAB   // producer/consumer attention (A/B against v5; measured slower, profiles/r06_attn/)
#include "lab/attn_pc.inc"
#endif

#if DLLM_LAB   // attention on 16x16x32 MFMAs (A/B against v5)
#include "lab/attn16.inc"
#endif

#if DLLM_LAB   // attention v6 (one wave per SIMD; A/B against v5)
#include "lab/attn_v6.inc"
#endif
}  // namespace
}  // namespace dllm

using namespace dllm;


extern "C" int dllm_kv_attention(const void *Q, const uint8_t *Kq, const float *k_params, const uint8_t *Vq,
                                 const float *v_params, uint8_t bits, size_t S, size_t H, size_t D, void *O,
                                 dllm_stream_t stream) {
    if (D != kD) return fail(DLLM_ERR_UNSUPPORTED, "dllm_kv_attention: head dim must be 128");
    if (bits != 4 && bits != 8) return fail(DLLM_ERR_UNSUPPORTED, "dllm_kv_attention: bits must be 4 or 8");
    if (S == 0 || H == 0) return DLLM_OK;
    if (!Q || !Kq || !Vq || !k_params || !v_params || !O) return fail(DLLM_ERR_INVALID_PARAMS, "null pointer");
    if (S * H * D * bits / 8 >= (size_t{1} << 31) || H > 65535)
        return fail(DLLM_ERR_SHAPE_MISMATCH, "K/V codes must stay below 2 GiB (32-bit buffer offsets)");
    if ((reinterpret_cast<uintptr_t>(Kq) & 15) || (reinterpret_cast<uintptr_t>(Vq) & 15) ||
        (reinterpret_cast<uintptr_t>(Q) & 15) || (reinterpret_cast<uintptr_t>(O) & 15))
        return fail(DLLM_ERR_INVALID_PARAMS, "Q, O, K and V codes must be 16-byte aligned");   // O: 16-B row stores
    hipStream_t st = as_stream(stream);
    const int nkb = static_cast<int>((S + kKB - 1) / kKB);
    // the attention kernel stages a head's f16 K / V images through one buffer descriptor with
    // 32-bit offsets (blk * kImg): a head's images must stay below 2 GiB too (~560 B per key, so
    // S past ~3.8 M keys at small H would pass the code-size check above)
    if (static_cast<size_t>(nkb) * kImg >= (size_t{1} << 31))
        return fail(DLLM_ERR_SHAPE_MISMATCH, "a head's K/V images must stay below 2 GiB (32-bit buffer offsets)");
    uint8_t *img = reinterpret_cast<uint8_t *>(device_workspace(st, static_cast<size_t>(H) * nkb * kImg, 8));
    if (!img) return DLLM_ERR_HIP;
    dim3 sgrid(static_cast<unsigned>(nkb), static_cast<unsigned>(H));
#if DLLM_LAB
    const int lab = [] { const char *e = getenv("DLLM_ATTN_LAB"); return e ? atoi(e) : 0; }();
    if (lab == 16) {   // the 16x16x32 kernel (A/B): its V image in kv_pos16 order
        if (bits == 4) kv_stage_kernel<4, true><<<sgrid, 512, 0, st>>>(Kq, k_params, Vq, v_params, (int)S, (int)H, nkb, img);
        else kv_stage_kernel<8, true><<<sgrid, 512, 0, st>>>(Kq, k_params, Vq, v_params, (int)S, (int)H, nkb, img);
    } else
#endif
    if (bits == 4)
        kv_stage_kernel<4><<<sgrid, 512, 0, st>>>(Kq, k_params, Vq, v_params, (int)S, (int)H, nkb, img);
    else
        kv_stage_kernel<8><<<sgrid, 512, 0, st>>>(Kq, k_params, Vq, v_params, (int)S, (int)H, nkb, img);
    DLLM_LAUNCH_CHECK();
    dim3 grid(static_cast<unsigned>((S + kQT - 1) / kQT), static_cast<unsigned>(H));
    const _Float16 *Qh = static_cast<const _Float16 *>(Q);
    _Float16 *Oh = static_cast<_Float16 *>(O);
#if DLLM_LAB
    // DLLM_ATTN_LAB (lab build only, measurement; results are garbage when set): 1 no softmax, 2 no
    // K/V staging, 4 no PV MFMAs, 8 no QK MFMAs (on the v4 kernel); 100: the v4 kernel itself
    // (valid results); 100 + mask: the same masks on the v5 kernel, plus 16 no vmcnt wait at the
    // end of a k-block, 32 no barrier there, 64 register staging instead of LDS-DMA (valid
    // results); 200 (+ mask): v6.  Read per call so that a script can A/B the schedules in one process.
    switch (lab) {
        case 16:   // the 16x16x32 kernel (A/B)
            kv_attention16_kernel<<<grid, kWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh);
            break;
#define DLLM_ALAB(L) case L: kv_attention_kernel<L><<<grid, kWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh); break;
        DLLM_ALAB(1) DLLM_ALAB(2) DLLM_ALAB(3) DLLM_ALAB(4) DLLM_ALAB(5) DLLM_ALAB(6) DLLM_ALAB(7)
        DLLM_ALAB(8) DLLM_ALAB(12) DLLM_ALAB(13) DLLM_ALAB(14) DLLM_ALAB(15)
#undef DLLM_ALAB
        case 100:   // the v4 schedule (A/B)
            kv_attention_kernel<0><<<grid, kWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh);
            break;
#define DLLM_ALAB5(L) case 100 + L: kv_attention5_kernel<L><<<grid, kWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh); break;
        DLLM_ALAB5(1) DLLM_ALAB5(2) DLLM_ALAB5(4) DLLM_ALAB5(8) DLLM_ALAB5(12) DLLM_ALAB5(13) DLLM_ALAB5(3) DLLM_ALAB5(16)
        DLLM_ALAB5(48) DLLM_ALAB5(50) DLLM_ALAB5(64) DLLM_ALAB5(128)
#undef DLLM_ALAB5
        case 200:   // v6: 4 waves x 64 queries (A/B)
            kv_attention6_kernel<0><<<grid, kW6 * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh);
            break;
#define DLLM_ALAB6(L) case 200 + L: kv_attention6_kernel<L><<<grid, kW6 * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh); break;
        DLLM_ALAB6(2) DLLM_ALAB6(4) DLLM_ALAB6(8)
#undef DLLM_ALAB6
        case 302:   // the product without the region-2 priority (A/B; bit-identical)
            kv_attention5_kernel<256, false><<<grid, kWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh);
            break;
        case 4196:   // the product with the round-2 epilogue, 64 two-byte stores per lane (A/B; bit-identical)
            kv_attention5_kernel<4096, false><<<grid, kWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh);
            break;
        case 612:   // the product without the region-1 softmax pins (A/B; bit-identical)
            kv_attention5_kernel<512, false><<<grid, kWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh);
            break;
        case 700:   // the producer/consumer kernel (A/B; bit-identical)
            kv_attention_pc_kernel<<<grid, kPcAttnWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh);
            break;
        case 198:   // the staggered schedule (A/B; bit-identical)
            kv_attention5_kernel<0, true><<<grid, kWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh);
            break;
        default:
            kv_attention5_kernel<0, false><<<grid, kWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh);
            break;
    }
#else
    kv_attention5_kernel<0, false><<<grid, kWaves * 64, 0, st>>>(Qh, img, k_params, v_params, (int)S, (int)H, Oh);
#endif
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}
