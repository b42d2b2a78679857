// linear_horner.hip -- the exact-weight int4 g128 GEMM in Horner form on 256 x 256 tiles: the
// default kernel of the headline shape (M = K = N = 4096) and of every int4 g128 layer whose
// 256 x 256 grid fills the chip.
//
// Replaces SimpleDiffusionModel::forward = x.dot(W) + b (diffuse-llm-rs/src/lib.rs:806-813) with
// W quantized per (column n, 128-row group g) by quantize_tensor (quantization.rs:38-68); the
// weight is the reference's f32 a2 value (q - zp) * s (quantization.rs:81-85): the MFMA A operand
// is the exact integer q - zp (f16) and the f32 group scale enters in Horner form,
//   acc <- acc * r_g + T_g,  r_g = s_{g-1} / s_g (hr[g][n], r_0 = 1),  T_g = sum_{k in g} X (q - zp),
// so after the last group acc = sum_g T_g s_g / s_{G-1} and the epilogue multiplies by s_{G-1}.
// The handle's create checks that every column's scales allow the form (linear_wq.hip).
//
// Structure (Y^T = W^T X^T: the accumulator's lane is the token, 4 consecutive registers are 4
// consecutive columns): block 256 tokens x 256 columns, 8 waves side by side in n (2 per SIMD),
// wave tile 32 columns x 256 tokens (acc = 8 x 16 f32).  Per 64-deep k-step a stage holds the X
// tile (32 KiB, XOR-swizzled 16-B chunks), the 8 waves' weight words (8 KiB) and, on a group's
// first k-step, the group's {zp, scale} pairs and ratios (2 KiB); 3 stages in a ring, stage kt+2
// issued while kt computes, one counted vmcnt wait and one raw s_barrier per k-step.
//
// Against wq_gemm8_kernel<..., HORNER> (linear_wq.hip, the same arithmetic and schedule, bit for bit)
// this kernel cuts the instruction stream around the MFMAs, which two waves per SIMD must share:
//   * a stage is ONE inline-asm burst per wave: buffer_load_dwordx4 ... lds with fixed per-lane
//     VGPR offsets and the k-step in an SGPR offset, M0 stepped by s_add between the DMAs (the LDS
//     destinations of a wave's X pieces and its weight words are 8 KiB apart), saved/restored once
//     per burst -- no per-DMA address VALU, no per-DMA M0 save/restore, no integer division;
//   * the group's {zp, scale} and ratios travel only with its first stage, and the zero-point
//     constants of dequant_exact are built once per group.
#include "linear_common.hpp"

#include <type_traits>

#ifndef DLLM_LAB
#define DLLM_LAB 0
#endif

namespace dllm {
namespace {

constexpr int kHW = 8 * 1024;                 // 8 waves x 64 lanes x 16 B of weight words
constexpr int kHG = 2048;                     // sz (1 KiB) + ratios (1 KiB), group-first stages

// One wave's stage burst: 4 X pieces (rows (8 i + wave) 8 ..) and its weight words, LDS-DMA
// through buffer descriptors.  lds0 = this wave's first X destination; the next pieces follow at
// +8 KiB (X piece i at wave * 1 KiB + i * 8 KiB, the weight words at 32 KiB + wave * 1 KiB).
__device__ __forceinline__ void horner_burst(__amdgpu_buffer_rsrc_t xr, uint32_t x0, uint32_t x1, uint32_t x2,
                                             uint32_t x3, uint32_t sx, __amdgpu_buffer_rsrc_t wr, uint32_t wo,
                                             uint32_t sw, uint32_t lds0) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %9\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %5, %6 offen lds\n\t"
        "s_add_u32 m0, m0, 0x2000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %5, %6 offen lds\n\t"
        "s_add_u32 m0, m0, 0x2000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %3, %5, %6 offen lds\n\t"
        "s_add_u32 m0, m0, 0x2000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %4, %5, %6 offen lds\n\t"
        "s_add_u32 m0, m0, 0x2000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %7, %8, %10 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(x0), "v"(x1), "v"(x2), "v"(x3), "s"(xr), "s"(sx), "v"(wo), "s"(wr), "s"(lds0), "s"(sw)
        : "memory");
}

// (wq_horner16_kernel: MODE bit 10 = half 1's A fragments built right after substep 1 (product);
// bit 11 = a non-group-first step's words and half-0 A fragments built at the end of the step
// before (lab A/B 325, not adopted).)
// MODE bit 0: the staggered schedule (product).  Lab ablations only (results wrong, timing only):
// bit 1 no output stores; bit 2 no Horner rescale; bit 3 one dequant per k-step instead of four;
// bit 4 one B fragment read per k-step instead of four; bit 5 no X DMA (weight words only); bit 6
// no DMA at all; bit 7 no MFMA (the DMA ring, waits and barriers alone).  Bit 8 (product): the
// stage's DMA pieces spread one per MFMA pair over the second half k-step instead of one burst
// (bit-identical; 124.9 -> 123.6 us at M = 4096 in one process, profiles/r04_horner/).
#if DLLM_LAB   // the round-3 kernel (32x32x16 MFMAs), lab variant 321 and the ablation harness
#include "lab/horner_r3.inc"
#endif

// ---------------------------------------------------------------------------------------------
// KG2 Horner GEMM: 256-token x 128-column tiles for grids where 256 x 256 tiles leave CUs idle
// (M = 2048 at N = 4096, 11 of the 12 GEMMs of a C5 step: 128 tiles of 256 x 256, 256 of
// 256 x 128; a 2-GPU column shard at M = 4096 likewise).  8 waves = 4 column waves (32 columns x
// 256 tokens each, wq_horner_kernel's wave tile, acc = 8 x 16 f32) x 2 k-groups: k-group kg runs the
// Horner chain over the groups of K-half kg (the ratio at a half's first group multiplies a zero
// accumulator), so each SIMD holds one wave of each k-group and every wave does the same work per
// k-step as in wq_horner_kernel.  A stage holds k-step kt of both halves: the two X slices
// (2 x 32 KiB), the 8 waves' weight words (8 KiB) and, on a group's first k-step, both halves'
// {zp, scale} pairs and ratios (4 x 512 B, each loaded twice by a 64-lane DMA); 2 stages in a ring
// (152 KiB), stage kt + 1 issued while kt computes, one vmcnt(0) + barrier per k-step.
// Epilogue: Y = acc0 s_{G/2-1} + acc1 s_{G-1} + b.  K-group 1 hands its scaled accumulator to its
// column partner through the drained ring, k-group 0 adds it (P0 + P1, a fixed order), and all 8
// waves store the f16 tile as coalesced 16-B rows.
constexpr int kKX = 256 * kBK * 2;              // one K-half's X slice per stage (32 KiB)
constexpr int kKW = 8 * 1024;                   // 8 waves x 1 KiB of weight words
constexpr int kKG = 4 * 1024;                   // 2 halves x (sz, ratios) x 1 KiB (mirrored halves)
constexpr int kKStage = 2 * kKX + kKW + kKG;    // 77824 B; 2 stages = 152 KiB

// One wave's stage burst: 8 X pieces (its k-group's slice, pieces 4 i + nw: rows (4 i + nw) 8 ..,
// 4 KiB apart in LDS) and its weight words.
__device__ __forceinline__ void kg2_burst(__amdgpu_buffer_rsrc_t xr, const uint32_t (&xo)[8], uint32_t sx,
                                          __amdgpu_buffer_rsrc_t wr, uint32_t wo, uint32_t sw, uint32_t lds_x,
                                          uint32_t lds_w) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %13\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %9, %10 offen lds\n\t"
        "s_add_u32 m0, m0, 0x1000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %9, %10 offen lds\n\t"
        "s_add_u32 m0, m0, 0x1000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %3, %9, %10 offen lds\n\t"
        "s_add_u32 m0, m0, 0x1000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %4, %9, %10 offen lds\n\t"
        "s_add_u32 m0, m0, 0x1000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %5, %9, %10 offen lds\n\t"
        "s_add_u32 m0, m0, 0x1000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %6, %9, %10 offen lds\n\t"
        "s_add_u32 m0, m0, 0x1000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %7, %9, %10 offen lds\n\t"
        "s_add_u32 m0, m0, 0x1000\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %8, %9, %10 offen lds\n\t"
        "s_mov_b32 m0, %14\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %11, %12, %15 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(xo[0]), "v"(xo[1]), "v"(xo[2]), "v"(xo[3]), "v"(xo[4]), "v"(xo[5]), "v"(xo[6]), "v"(xo[7]),
          "s"(xr), "s"(sx), "v"(wo), "s"(wr), "s"(lds_x), "s"(lds_w), "s"(sw)
        : "memory");
}

template <typename YT, int EPI>
__global__ void __launch_bounds__(512, 1)
wq_horner_kg2_kernel(const __half *__restrict__ X, int M, int K, const uint32_t *__restrict__ wdev,
                     const uint32_t *__restrict__ sz, const float *__restrict__ hr, const float *__restrict__ sf,
                     const float *__restrict__ bias, YT *__restrict__ Y, int N, int Npad, int nbm, int nbn,
                     PSampleEpi epi) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kKStage];

    // XCD-aware bijective remap (as wq_horner_kernel): an XCD's 32 concurrent tiles are one
    // 256-row block x 32 column blocks at N = 4096, so its L2 holds one X row block.
    const int nb = nbm * nbn, orig = blockIdx.x;
    const int xcd = orig % kXCDs, q8 = nb / kXCDs, r8 = nb % kXCDs;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / kXCDs;
    const int bm = tile / nbn, bn = tile % nbn;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int kg = wave >> 2, nw = wave & 3;
    const int m0 = bm * 256, n0 = bn * 128;
    const int nk = K / kBK, nk2 = nk / 2;   // k-steps per K-half (even: K % 256 == 0)
    const int kofs = kg * nk2;              // this k-group's first k-step

    uint32_t xo[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int row = (i * 4 + nw) * 8 + (lane >> 3);
        const int rrow = (m0 + row < M ? m0 + row : M - 1) - m0;   // rows past M re-read row M - 1
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        xo[i] = static_cast<uint32_t>((rrow * K + c * 8) * 2);
    }
    const __amdgpu_buffer_rsrc_t xr = raw_rsrc(X + static_cast<size_t>(m0) * K);
    const uint32_t nt = static_cast<uint32_t>(n0 + 32 * nw) >> 5;
    const __amdgpu_buffer_rsrc_t wr = raw_rsrc(wdev + static_cast<size_t>(nt) * nk * 64 * 4);
    const uint32_t wo = static_cast<uint32_t>(lane * 16);
    // group data: column wave 0 of each k-group stages the {zp, scale} pairs of columns n0 .. n0+127,
    // column wave 1 the ratios; lanes 32..63 repeat lanes 0..31 (a full 64-lane DMA, no exec mask)
    const __amdgpu_buffer_rsrc_t gr =
        raw_rsrc(nw == 0 ? static_cast<const void *>(sz + n0) : static_cast<const void *>(hr + n0));
    const bool has_g = nw < 2;
    const uint32_t go = static_cast<uint32_t>((lane & 31) * 16);
    const uint32_t sbase = __builtin_amdgcn_readfirstlane(lds_addr(smem));

    auto stage = [&](int slot, int kt, bool gf) __attribute__((always_inline)) {
        const uint32_t base = sbase + static_cast<uint32_t>(slot * kKStage);
        const int ka = kofs + kt;
        kg2_burst(xr, xo, static_cast<uint32_t>(ka * kBK * 2), wr, wo, static_cast<uint32_t>(ka * 1024),
                  base + static_cast<uint32_t>(kg * kKX + nw * 1024), base + static_cast<uint32_t>(2 * kKX + wave * 1024));
        if (gf && has_g)
            blds16_asm(gr, go, static_cast<uint32_t>((ka >> 1) * Npad * 4),
                       base + static_cast<uint32_t>(2 * kKX + kKW + kg * 2048 + nw * 1024));
    };

    float16_t acc[8];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[r][e] = 0.0f;

    const int hsel = lane >> 5;
    const int rowx = ((lane & 31) >> 1) & 7;
    int soff[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) soff[s] = (lane & 31) * (kBK * 2) + ((((2 * s + hsel) ^ rowx)) << 4);

    auto read_b = [&](half8_t (&b)[8], const uint8_t *sb, int s) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 8; ++r) b[r] = *reinterpret_cast<const half8_t *>(sb + soff[s] + r * 32 * kBK * 2);
    };

    ExactConsts ec;
    uint32_t w[4];
    float4 r4[4];
    half8_t bA[8], bB[8], aA, aB;
    auto sub = [&](const uint8_t *sb, half8_t (&bc)[8], half8_t (&bn)[8], const half8_t &ac, half8_t &an, int j,
                   bool gf) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        if (j < 3) {
            read_b(bn, sb, j + 1);
            an = dequant_exact<4>(w, j + 1, ec);
        }
        if (gf && j == 0) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
#pragma unroll
                for (int qd = 0; qd < 4; ++qd) {
                    acc[r][4 * qd + 0] *= r4[qd].x;
                    acc[r][4 * qd + 1] *= r4[qd].y;
                    acc[r][4 * qd + 2] *= r4[qd].z;
                    acc[r][4 * qd + 3] *= r4[qd].w;
                }
                acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ac, bc[r], acc[r], 0, 0, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (i + 1 < 8) __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
            }
        } else {
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ac, bc[r], acc[r], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            }
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto barrier = []() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // One k-step of this k-group's half on ring slot `slot`; slot ^ 1 receives k-step kt + 1
    // (the slot's previous k-step, kt - 1, was read before the barrier that ended it).
    auto step = [&](int slot, int kt, auto gf_tag) __attribute__((always_inline)) {
        constexpr bool GF = decltype(gf_tag)::value;
        if (kt + 1 < nk2) stage(slot ^ 1, kt + 1, !GF);   // kt + 1 opens a group iff kt does not
        const uint8_t *st8 = smem + slot * kKStage;
        const uint8_t *sb = st8 + kg * kKX;
        {
            const uint4 v = *reinterpret_cast<const uint4 *>(st8 + 2 * kKX + wave * 1024 + lane * 16);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        }
        if constexpr (GF) {
            const uint8_t *gb = st8 + 2 * kKX + kKW + kg * 2048;
            half2_t nz, sc;
            split_sz(*reinterpret_cast<const uint32_t *>(gb + (nw * 32 + (lane & 31)) * 4), nz, sc);
            ec = exact_consts(nz);
            const float *rl = reinterpret_cast<const float *>(gb + 1024) + nw * 32 + 4 * hsel;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) r4[qd] = *reinterpret_cast<const float4 *>(rl + 8 * qd);
        }
        read_b(bA, sb, 0);
        aA = dequant_exact<4>(w, 0, ec);
        sub(sb, bA, bB, aA, aB, 0, GF);
        sub(sb, bB, bA, aB, aA, 1, GF);
        sub(sb, bA, bB, aA, aB, 2, GF);
        sub(sb, bB, bA, aB, aA, 3, GF);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // k-step kt + 1 landed
        barrier();
    };

    stage(0, 0, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    using GFt = std::integral_constant<bool, true>;
    using GFf = std::integral_constant<bool, false>;
    for (int kt = 0; kt < nk2; kt += 2) {   // group = 2 k-steps = the 2-slot ring period
        step(0, kt, GFt{});
        step(1, kt + 1, GFf{});
    }

    // this half's partial sum: acc times the half's last group scales
    const int nb0 = n0 + nw * 32 + 4 * hsel;
    const float *sl = sf + static_cast<size_t>((kofs + nk2) / 2 - 1) * Npad + nb0;
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
        const float4 s = *reinterpret_cast<const float4 *>(sl + 8 * qd);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            acc[r][4 * qd + 0] *= s.x;
            acc[r][4 * qd + 1] *= s.y;
            acc[r][4 * qd + 2] *= s.z;
            acc[r][4 * qd + 3] *= s.w;
        }
    }
    // k-group 1 -> LDS (the ring is drained: every DMA waited for, every wave past the last
    // barrier); 4 column waves x 8 reps x 4 x 1 KiB = 128 KiB, one 16-B piece per lane
    float4 *part = reinterpret_cast<float4 *>(smem);
    if (kg == 1) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int qd = 0; qd < 4; ++qd)
                part[((nw * 8 + r) * 4 + qd) * 64 + lane] =
                    make_float4(acc[r][4 * qd + 0], acc[r][4 * qd + 1], acc[r][4 * qd + 2], acc[r][4 * qd + 3]);
    }
    __syncthreads();
    if (kg == 0) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                const float4 v = part[((nw * 8 + r) * 4 + qd) * 64 + lane];
                acc[r][4 * qd + 0] = acc[r][4 * qd + 0] + v.x;
                acc[r][4 * qd + 1] = acc[r][4 * qd + 1] + v.y;
                acc[r][4 * qd + 2] = acc[r][4 * qd + 2] + v.z;
                acc[r][4 * qd + 3] = acc[r][4 * qd + 3] + v.w;
            }
    }
    __syncthreads();
    float4 bv[4];
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) bv[qd] = *reinterpret_cast<const float4 *>(bias + nb0 + 8 * qd);
    if constexpr (EPI == 1) {
        if (kg != 0) return;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
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
    const bool full = (m0 + 256 <= M) && (n0 + 128 <= N) && (N % 8) == 0;
    if constexpr (std::is_same<YT, __half>::value) {
        if (full) {
            // k-group 0 writes the f16 tile image (256 rows x 256 B, 16-B chunks XORed with the
            // row), then all 8 waves store 4 whole rows per instruction
            uint8_t *img = smem;
            if (kg == 0) {
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const int t = r * 32 + (lane & 31);
#pragma unroll
                    for (int qd = 0; qd < 4; ++qd) {
                        const int pc = (nw * 4 + qd) ^ (t & 15);
                        union { __half h[4]; uint2 u; } pk;
                        pk.h[0] = __float2half_rn(acc[r][4 * qd + 0] + bv[qd].x);
                        pk.h[1] = __float2half_rn(acc[r][4 * qd + 1] + bv[qd].y);
                        pk.h[2] = __float2half_rn(acc[r][4 * qd + 2] + bv[qd].z);
                        pk.h[3] = __float2half_rn(acc[r][4 * qd + 3] + bv[qd].w);
                        *reinterpret_cast<uint2 *>(img + t * 256 + pc * 16 + hsel * 8) = pk.u;
                    }
                }
            }
            __syncthreads();
            const int c = lane & 15;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int t = (i * 8 + wave) * 4 + (lane >> 4);
                const uint4 v = *reinterpret_cast<const uint4 *>(img + t * 256 + ((c ^ (t & 15)) * 16));
                *reinterpret_cast<uint4 *>(Y + static_cast<size_t>(m0 + t) * N + n0 + 8 * c) = v;
            }
            return;
        }
    }
    if (kg != 0) return;
    const bool vec_ok = (N % 4) == 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int m = m0 + r * 32 + (lane & 31);
        if (m >= M) continue;
        YT *yrow = Y + static_cast<size_t>(m) * N;
#pragma unroll
        for (int qd = 0; qd < 4; ++qd)
            store_out4<YT>(yrow, bias, nb0 + 8 * qd, N, vec_ok, acc[r][4 * qd + 0], acc[r][4 * qd + 1],
                           acc[r][4 * qd + 2], acc[r][4 * qd + 3]);
    }
}

// ---------------------------------------------------------------------------------------------
// The same Horner GEMM on 16x16x32 MFMAs (the product kernel since round 4).  Same block tile, ring,
// stage bursts, stagger, spread DMA pieces and weight layout as wq_horner_kernel; per wave the
// 32 columns x 256 tokens are 2 column blocks x 16 token blocks of 16 x 16 (acc = 32 x 4 f32, the
// same 128 registers).  Why: at equal FLOPs and cycles the chip holds a higher clock on the
// 16x16x32 shape (MI355X_MICROARCH.md, DVFS give-back item 7) -- the shape-only lab ablation of the
// round-3 schedule ran 121.7 -> 112.7 us at M = K = N = 4096 (profiles/r04_horner/).
// A operand: the prefill layout gives lane L column L & 31 and k-chunks 2s + (L >> 5) (8 deep) of
// substep word s; dequant_exact turns words s = 2h, 2h + 1 into two f16 fragments and ONE
// v_permlane16_swap per VGPR pair regroups them into the 16x16x32 A fragments of half h: column
// block 0 (columns 0..15: lane rows R0..R3 hold k-chunks 4h + {0, 2, 1, 3}) and column block 1
// (columns 16..31, the same chunks).  B operand: token 16 tb + (lane & 15), the k-chunk of the
// lane's row in the same order, one ds_read_b128 from the swizzled X tile.  D: lane holds columns
// 16 cb + 4 (lane >> 4) + i of token 16 tb + (lane & 15), so the Horner ratios, the last group's
// scales and the bias are one float4 per column block.
typedef float fx4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// The f16 tile (acc * s + b) through the drained ring as 16-B row chunks, passes of 128 tokens.
template <int TB>
__device__ __forceinline__ void store_tile16_f16_lds(uint8_t *img, const fx4_t (&acc)[TB][2], const float4 (&bv)[2],
                                                     __half *Y, int N, int m0, int n0, int wave, int lane) {
    constexpr int kRowB = 512, kCpr = 32;
    const int row16 = lane & 15, rq = lane >> 4;
    constexpr int kTPP = TB < 8 ? TB : 8;   // token blocks per pass (128 rows at most)
#pragma unroll
    for (int p = 0; p < TB / kTPP; ++p) {
#pragma unroll
        for (int i = 0; i < kTPP; ++i) {
            const int t = 16 * i + row16;
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                const int pc = (4 * wave + 2 * cb + (rq >> 1)) ^ (t & (kCpr - 1));
                const fx4_t &a = acc[kTPP * p + i][cb];
                const float4 &b = bv[cb];
                union { __half h[4]; uint2 u; } pk;
                pk.h[0] = __float2half_rn(a[0] + b.x);
                pk.h[1] = __float2half_rn(a[1] + b.y);
                pk.h[2] = __float2half_rn(a[2] + b.z);
                pk.h[3] = __float2half_rn(a[3] + b.w);
                *reinterpret_cast<uint2 *>(img + t * kRowB + pc * 16 + (rq & 1) * 8) = pk.u;
            }
        }
        __syncthreads();
        const int c = lane % kCpr;
#pragma unroll
        for (int t0 = wave * 2; t0 < 16 * kTPP; t0 += 16) {
            const int t = t0 + lane / kCpr;
            const uint4 v = *reinterpret_cast<const uint4 *>(img + t * kRowB + ((c ^ (t & (kCpr - 1))) * 16));
#if DLLM_NT_STORE
            typedef unsigned int u4nt __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(u4nt{v.x, v.y, v.z, v.w},
                                        reinterpret_cast<u4nt *>(Y + static_cast<size_t>(m0 + 16 * kTPP * p + t) * N + n0 + 8 * c));
#else
            *reinterpret_cast<uint4 *>(Y + static_cast<size_t>(m0 + 16 * kTPP * p + t) * N + n0 + 8 * c) = v;
#endif
        }
        __syncthreads();
    }
}

// TB = 16: 256-token tiles (the M = 4096 grid), a stage = one 64-deep k-step.  TB = 8: 128-token
// tiles (grids where 256 x 256 tiles leave CUs idle and 128 x 256 fill them: M = 2048 at N = 4096,
// the 2-GPU column shard at M = 4096), a stage = one 128-deep group (two k-steps: X 2 x 16 KiB,
// weight words 2 x 8 KiB) so that a stage carries the same 64 MFMAs per wave as at TB = 16 and the
// 3-stage ring hides the same DMA latency.  Either way a stage is 4 substeps of 16 MFMAs:
// TB = 16: substep j = (half j >> 1, token blocks 8 (j & 1) ..); TB = 8: (k-step j >> 1, half j & 1).
template <int TB>
struct H16 {
    static_assert(TB == 16 || TB == 8, "256- or 128-token tiles");
    static constexpr int kKPS = 16 / TB;                  // 64-deep k-steps per stage
    static constexpr int kXB = 32 * 1024;                  // X bytes per stage (kKPS sub-tiles of 16 TB rows x 64)
    static constexpr int kXSub = kXB / kKPS;               // one k-step's X sub-tile
    static constexpr int kWB = kKPS * kHW;                 // weight words per stage
    static constexpr int kStage = kXB + kWB + kHG;         // 43008 / 51200 B
    static constexpr int kNX = TB / 4;                     // X pieces per wave per k-step sub-tile
    static constexpr int kPieces = kKPS * (kNX + 1) + 1;   // DMA pieces per stage (X, W, group data)
};

template <typename YT, int EPI, int MODE, int TB = 16, int BITS = 4>
__global__ void __launch_bounds__(512, 1)
wq_horner16_kernel(const __half *__restrict__ X, int M, int K, const uint32_t *__restrict__ wdev,
                   const uint32_t *__restrict__ sz, const float *__restrict__ hr, const float *__restrict__ sf,
                   const float *__restrict__ bias, YT *__restrict__ Y, int N, int Npad, int nbm, int nbn,
                   PSampleEpi epi) {
    constexpr bool STAG = MODE & 1;
    // BITS = 2 (int2 g128, 256-token tiles only): a wave's weight words of the k-step pair (2u, 2u + 1)
    // are one 1-KiB piece of the code layout (k-step 2u's 64 lanes x 8 B, then 2u + 1's); every stage
    // moves its pair's piece (twice per pair: int2's 4 MiB of words at 4096^2 read twice, the int4
    // stage's bytes) and reads its own half, so the ring, the pieces per stage and the waits are int4's.
    static_assert(BITS == 4 || (BITS == 2 && TB == 16), "int4, or int2 on 256-token tiles");
    using L = H16<TB>;
    constexpr int kStage = L::kStage, kXB = L::kXB, kKPS = L::kKPS;
    __shared__ __attribute__((aligned(16))) uint8_t smem[3 * kStage];

    // XCD-aware bijective remap (as wq_horner_kernel)
    const int nb = nbm * nbn, orig = blockIdx.x;
    const int xcd = orig % kXCDs, q8 = nb / kXCDs, r8 = nb % kXCDs;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / kXCDs;
    const int bm = tile / nbn, bn = tile % nbn;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m0 = bm * 16 * TB, n0 = bn * 256;
    const int nk = K / kBK;              // 64-deep k-steps
    const int ns = nk / kKPS;            // stages

    uint32_t xo[L::kNX];
#pragma unroll
    for (int i = 0; i < L::kNX; ++i) {
        const int row = (i * 8 + wave) * 8 + (lane >> 3);
        const int rrow = (m0 + row < M ? m0 + row : M - 1) - m0;
        const int c = (lane & 7) ^ ((row >> 1) & 5);   // X chunk swizzle: see soff below
        xo[i] = static_cast<uint32_t>((rrow * K + c * 8) * 2);
    }
    const __amdgpu_buffer_rsrc_t xr = raw_rsrc(X + static_cast<size_t>(m0) * K);
    const uint32_t nt = static_cast<uint32_t>(n0 + 32 * wave) >> 5;
    const __amdgpu_buffer_rsrc_t wr = raw_rsrc(wdev + static_cast<size_t>(nt) * nk * 64 * BITS);
    auto wsoff = [](int kstep) { return static_cast<uint32_t>(BITS == 4 ? kstep * 1024 : (kstep & ~1) * 512); };
    const uint32_t wo = static_cast<uint32_t>(lane * 16);
    const __amdgpu_buffer_rsrc_t gr =
        raw_rsrc(wave == 0 ? static_cast<const void *>(sz + n0) : static_cast<const void *>(hr + n0));
    const bool has_g = wave < 2;
    const uint32_t sbase = __builtin_amdgcn_readfirstlane(lds_addr(smem));

    // DMA piece p of stage st into ring slot `slot`: X pieces (sub-tile p / kNX, piece p % kNX), then
    // the weight words of each k-step, then (group-first stages, waves 0 and 1) the group data.
    auto piece = [&](int p, int slot, int st, bool gf) __attribute__((always_inline)) {
        const uint32_t base = sbase + static_cast<uint32_t>(slot * kStage);
        constexpr int nxp = kKPS * L::kNX;
        if (p < nxp) {
            const int kk = p / L::kNX, i = p % L::kNX;
            blds16_asm(xr, xo[i], static_cast<uint32_t>((st * kKPS + kk) * kBK * 2),
                       base + static_cast<uint32_t>(kk * L::kXSub + wave * 1024 + i * 0x2000));
        } else if (p < nxp + kKPS) {
            const int kk = p - nxp;
            blds16_asm(wr, wo, wsoff(st * kKPS + kk),
                       base + static_cast<uint32_t>(kXB + kk * kHW + wave * 1024));
        } else if (p == nxp + kKPS && gf && has_g) {
            blds16_asm(gr, wo, static_cast<uint32_t>(((st * kKPS) >> 1) * Npad * 4),
                       base + static_cast<uint32_t>(kXB + L::kWB + wave * 1024));
        }
    };
    auto stage = [&](int slot, int st, bool gf) __attribute__((always_inline)) {
        if constexpr (TB == 16) {
            horner_burst(xr, xo[0], xo[1], xo[2], xo[3], static_cast<uint32_t>(st * kBK * 2), wr, wo,
                         wsoff(st), sbase + static_cast<uint32_t>(slot * kStage + wave * 1024));
            piece(L::kPieces - 1, slot, st, gf);
        } else {
#pragma unroll
            for (int p = 0; p < L::kPieces; ++p) piece(p, slot, st, gf);
        }
    };

    fx4_t acc[TB][2];
#pragma unroll
    for (int t = 0; t < TB; ++t)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) acc[t][cb] = fx4_t{0.f, 0.f, 0.f, 0.f};

    const int row16 = lane & 15, rq = lane >> 4;
    const int cq = ((rq & 1) << 1) | (rq >> 1);   // k-chunk of lane row rq after the swap: 0, 2, 1, 3
    // LDS slot of chunk g in row r: g ^ ((r >> 1) & 5).  With the lane rows' chunks 4h + {0, 2, 1, 3}
    // this makes each ds_read_b128 lane group (16 lanes: 8 rows of one lane row, 8 of another whose
    // chunk differs by 2) hit 16 distinct 16-B bank slots; the (r >> 1) & 7 swizzle of the 32x32
    // kernel maps them 2-way onto 8.
    int soff[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) soff[h] = row16 * (kBK * 2) + (((4 * h + cq) ^ ((row16 >> 1) & 5)) << 4);

    // substep j -> (k-step kk of the stage, half h, first token block tb0)
    auto sj_kk = [](int j) { return TB == 16 ? 0 : (j >> 1); };
    auto sj_h = [](int j) { return TB == 16 ? (j >> 1) : (j & 1); };
    auto sj_tb0 = [](int j) { return TB == 16 ? 8 * (j & 1) : 0; };
    // B fragments of substep j
    auto read_b = [&](half8_t (&b)[8], const uint8_t *sb, int j) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            b[i] = *reinterpret_cast<const half8_t *>(sb + sj_kk(j) * L::kXSub + soff[sj_h(j)] +
                                                      (sj_tb0(j) + i) * 16 * kBK * 2);
    };

    ExactConsts ec;
    uint32_t w[BITS];
    float4 r4[2];
    half8_t bA[8], bB[8], a00, a01, a10, a11;
    // par: the k-step's parity (BITS = 2: which half of the pair's piece)
    auto load_w = [&](const uint8_t *sb, int kk, int par) __attribute__((always_inline)) {
        if constexpr (BITS == 4) {
            (void)par;
            const uint4 v = *reinterpret_cast<const uint4 *>(sb + kXB + kk * kHW + wave * 1024 + lane * 16);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else {
            const uint2 v = *reinterpret_cast<const uint2 *>(sb + kXB + kk * kHW + wave * 1024 + par * 512 + lane * 8);
            w[0] = v.x; w[1] = v.y;
        }
    };
    // A fragments of half h (words 2h, 2h + 1) for column blocks 0 and 1
    auto make_a = [&](int h, half8_t &c0, half8_t &c1) __attribute__((always_inline)) {
        u32x4_t u0 = __builtin_bit_cast(u32x4_t, dequant_exact<BITS>(w, 2 * h, ec));
        u32x4_t u1 = __builtin_bit_cast(u32x4_t, dequant_exact<BITS>(w, 2 * h + 1, ec));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const auto r = __builtin_amdgcn_permlane16_swap(u0[e], u1[e], false, false);
            u0[e] = r[0];
            u1[e] = r[1];
        }
        c0 = __builtin_bit_cast(half8_t, u0);
        c1 = __builtin_bit_cast(half8_t, u1);
    };
    bool a_done = false;   // MODE bit 3 (lab ablation): the A fragments are built in the first step only
    // MODE bit 8: the pending stage's pieces, issued between MFMA quarters of substeps 2 and 3
    int pend_slot = 0, pend_st = 0;
    bool pend_gf = false, pend_on = false;
    constexpr int kPPS = (L::kPieces + 1) / 2;   // pieces per late substep (3 / 4)
    auto mma = [&](int t, int cb, const half8_t &a, const half8_t &b) __attribute__((always_inline)) {
        acc[t][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[t][cb], 0, 0, 0);
    };
    auto rescale = [&](int t) __attribute__((always_inline)) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
            acc[t][cb][0] *= r4[cb].x;
            acc[t][cb][1] *= r4[cb].y;
            acc[t][cb][2] *= r4[cb].z;
            acc[t][cb][3] *= r4[cb].w;
        }
    };
    // Substep j: 16 MFMAs (8 token blocks x both column blocks); the next substep's B fragments and
    // the A fragments it needs (TB = 16: half 1's after substep 1, see step; TB = 8: the next
    // substep's, built during this one).
    auto sub = [&](const uint8_t *sb, half8_t (&bc)[8], half8_t (&bn)[8], int j, bool gf) __attribute__((always_inline)) {
        const int tb0 = sj_tb0(j);
        const bool use1 = TB == 16 ? (j >= 2) : (j & 1);
        const half8_t &a0 = use1 ? a10 : a00;
        const half8_t &a1 = use1 ? a11 : a01;
        __builtin_amdgcn_sched_barrier(0);
        if ((MODE & 1024) == 0 && TB == 16 && j == 2 && !((MODE & 8) && a_done)) {   // lab A/B: half 1's A fragments at substep 2
            make_a(1, a10, a11);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (TB == 8 && j == 1) load_w(sb, 1, 1);   // k-step 1's words (k-step 0's last use was in substep 0)
        __builtin_amdgcn_s_setprio(1);
        if (TB == 8 && j < 3) {   // the next substep's A fragments beside this substep's MFMAs
            if (j & 1) make_a(0, a00, a01);
            else make_a(1, a10, a11);
        }
        if ((MODE & 256) != 0 && j >= 2) {
            // quarters of 4 MFMAs (2 token blocks), each with 2 of the next substep's B reads, and a
            // DMA piece between quarters
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (j < 3) {
                    const uint8_t *nb = sb + sj_kk(j + 1) * L::kXSub + soff[sj_h(j + 1)] + sj_tb0(j + 1) * 16 * kBK * 2;
                    bn[2 * q] = *reinterpret_cast<const half8_t *>(nb + (2 * q) * 16 * kBK * 2);
                    bn[2 * q + 1] = *reinterpret_cast<const half8_t *>(nb + (2 * q + 1) * 16 * kBK * 2);
                }
                mma(tb0 + 2 * q, 0, a0, bc[2 * q]);
                mma(tb0 + 2 * q, 1, a1, bc[2 * q]);
                mma(tb0 + 2 * q + 1, 0, a0, bc[2 * q + 1]);
                mma(tb0 + 2 * q + 1, 1, a1, bc[2 * q + 1]);
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                __builtin_amdgcn_sched_barrier(0);
                if (pend_on && q < kPPS) piece(kPPS * (j - 2) + q, pend_slot, pend_st, pend_gf);
                __builtin_amdgcn_sched_barrier(0);
            }
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            return;
        }
        if (j < 3) read_b(bn, sb, j + 1);
        if (gf && (TB == 16 ? j < 2 : j == 0)) {
            // acc <- acc * r_g right before each token block's first MFMA of the group (block i + 1's
            // rescale beside block i's MFMAs)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr ((MODE & 4) == 0) rescale(tb0 + i);   // (bit 2: lab ablation, no rescale)
                mma(tb0 + i, 0, a0, bc[i]);
                mma(tb0 + i, 1, a1, bc[i]);
            }
            __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (i + 1 < 8) __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                mma(tb0 + i, 0, a0, bc[i]);
                mma(tb0 + i, 1, a1, bc[i]);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            }
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto barrier = []() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // Waits until at most the pieces of one stage (the one issued in this stage's second half) are
    // outstanding: 5 / 6 (TB = 16, + the group data) or 6 / 7 (TB = 8).
    auto wait_one_stage = [&](bool gf) __attribute__((always_inline)) {
        if constexpr (TB == 16) {
            if (gf && has_g) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        } else {
            if (gf && has_g) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        }
    };
    const bool grp_b = STAG && wave >= 4;
    // One stage on ring slot `slot` (stage si); slot (si + 2) % 3 receives stage si + 2.  GF: the stage
    // opens a group (every stage at TB = 8; TB = 16: even k-steps, so si + 2 opens one iff si does).
    auto step = [&](int slot, int si, auto gf_tag) __attribute__((always_inline)) {
        constexpr bool GF = decltype(gf_tag)::value;
        const bool issue = (MODE & 64) == 0 && si + 2 < ns;   // (bit 6: lab ablation, no DMA after the prologue)
        if (!STAG && issue) stage((slot + 2) % 3, si + 2, GF);
        const uint8_t *sb = smem + slot * kStage;
        // MODE bit 11 (TB = 16): a non-group-first step's words and half-0 A fragments were built at
        // the end of the step before (the wave's own weight-word DMA is complete after its vmcnt
        // wait; the zero points are the group's), so they overlap that step's MFMA drain
        constexpr bool kEarly = (MODE & 2048) != 0 && TB == 16;
        if (!(kEarly && !GF)) load_w(sb, 0, si & 1);
        if constexpr (GF) {
            half2_t nz, sc;
            split_sz(*reinterpret_cast<const uint32_t *>(sb + kXB + L::kWB + (wave * 32 + (lane & 31)) * 4), nz, sc);
            ec = exact_consts(nz);
            const float *rl = reinterpret_cast<const float *>(sb + kXB + L::kWB + 1024) + wave * 32 + 4 * rq;
            r4[0] = *reinterpret_cast<const float4 *>(rl);
            r4[1] = *reinterpret_cast<const float4 *>(rl + 16);
        }
        read_b(bA, sb, 0);
        if (!(kEarly && !GF) && !((MODE & 8) && a_done)) make_a(0, a00, a01);   // (bit 3: lab ablation, A once)
        sub(sb, bA, bB, 0, GF);
        sub(sb, bB, bA, 1, GF);
        if constexpr (TB == 16 && (MODE & 1024) != 0) {
            // half 1's A fragments right behind substep 1's MFMAs (their registers free once those
            // issue): the dequant runs while the MFMAs drain and the wave reaches the barrier
            if (!((MODE & 8) && a_done)) make_a(1, a10, a11);
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr ((MODE & 8) != 0) a_done = true;
        if constexpr (STAG) {
            if (grp_b) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            barrier();
            if constexpr ((MODE & 256) != 0) {
                pend_on = issue;
                pend_slot = (slot + 2) % 3;
                pend_st = si + 2;
                pend_gf = GF;
            } else if (issue) {
                stage((slot + 2) % 3, si + 2, GF);
            }
        }
        sub(sb, bA, bB, 2, GF);
        sub(sb, bB, bA, 3, GF);
        if (!grp_b) {
            if (issue) wait_one_stage(GF);
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if constexpr (kEarly && GF) {   // the next (same-group) step's words and half-0 A fragments
            __builtin_amdgcn_sched_barrier(0);
            load_w(smem + ((slot + 1) % 3) * kStage, 0, (si + 1) & 1);
            make_a(0, a00, a01);
            __builtin_amdgcn_sched_barrier(0);
        }
        barrier();
    };

    stage(0, 0, true);
    stage(1, 1, TB == 8);
    wait_one_stage(TB == 8);   // stage 0 landed (stage 1's pieces in flight)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (grp_b) barrier();
    using GFt = std::integral_constant<bool, true>;
    using GFf = std::integral_constant<bool, false>;
    if constexpr (TB == 16) {
        // group = 2 k-steps, ring period 3: unroll 6 so each step's slot and group phase are static
        for (int si = 0; si < ns; si += 6) {
            step(0, si, GFt{});
            step(1, si + 1, GFf{});
            if (si + 2 < ns) {
                step(2, si + 2, GFt{});
                step(0, si + 3, GFf{});
            }
            if (si + 4 < ns) {
                step(1, si + 4, GFt{});
                step(2, si + 5, GFf{});
            }
        }
    } else {
        for (int si = 0; si < ns; si += 3) {
            step(0, si, GFt{});
            if (si + 1 < ns) step(1, si + 1, GFt{});
            if (si + 2 < ns) step(2, si + 2, GFt{});
        }
    }
    if (STAG && !grp_b) barrier();

    // acc = sum_g T_g s_g / s_{G-1}: times the last group's scales, then the bias
    const int nc0 = n0 + wave * 32 + 4 * rq;   // + 16 cb: the lane's 4 columns of column block cb
    const float *sl = sf + static_cast<size_t>(nk / 2 - 1) * Npad + nc0;
    float4 bv[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
        const float4 s = *reinterpret_cast<const float4 *>(sl + 16 * cb);
        bv[cb] = *reinterpret_cast<const float4 *>(bias + nc0 + 16 * cb);
#pragma unroll
        for (int t = 0; t < TB; ++t) {
            acc[t][cb][0] *= s.x;
            acc[t][cb][1] *= s.y;
            acc[t][cb][2] *= s.z;
            acc[t][cb][3] *= s.w;
        }
    }
    if constexpr ((MODE & 2) != 0) {   // lab ablation: keep the results live, store nothing
#pragma unroll
        for (int t = 0; t < TB; ++t)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) asm volatile("" ::"v"(acc[t][cb]));
        return;
    }
    if constexpr (EPI == 1) {
#pragma unroll
        for (int t = 0; t < TB; ++t) {
            const int m = m0 + 16 * t + row16;
            if (m >= M) continue;
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                if (nc0 + 16 * cb >= N) continue;
                psample4(epi, m, nc0 + 16 * cb, N, acc[t][cb][0] + bv[cb].x, acc[t][cb][1] + bv[cb].y,
                         acc[t][cb][2] + bv[cb].z, acc[t][cb][3] + bv[cb].w);
            }
        }
        return;
    }
    const bool full = (m0 + 16 * TB <= M) && (n0 + 256 <= N) && (N % 4) == 0;
    if constexpr (std::is_same<YT, __half>::value && (MODE & 4096) == 0) {   // (bit 12, lab A/B: 8-B stores from registers)
        if (full && (N % 8) == 0) {   // coalesced 16-B row stores through the drained ring
            store_tile16_f16_lds<TB>(smem, acc, bv, Y, N, m0, n0, wave, lane);
            return;
        }
    }
    if (full) {
#pragma unroll
        for (int t = 0; t < TB; ++t) {
            YT *yrow = Y + static_cast<size_t>(m0 + 16 * t + row16) * N + nc0;
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
                store4<YT>(yrow + 16 * cb, acc[t][cb][0] + bv[cb].x, acc[t][cb][1] + bv[cb].y,
                           acc[t][cb][2] + bv[cb].z, acc[t][cb][3] + bv[cb].w);
        }
    } else {
        const bool vec_ok = (N % 4) == 0;
#pragma unroll
        for (int t = 0; t < TB; ++t) {
            const int m = m0 + 16 * t + row16;
            if (m >= M) continue;
            YT *yrow = Y + static_cast<size_t>(m) * N;
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
                store_out4<YT>(yrow, bias, nc0 + 16 * cb, N, vec_ok, acc[t][cb][0], acc[t][cb][1], acc[t][cb][2],
                               acc[t][cb][3]);
        }
    }
}

template <int MODE, int TB = 16, int BITS = 4>
void launch_horner16_t(const HornerGemmArgs &a, int y_f32, hipStream_t st) {
    const int nbm = (a.M + 16 * TB - 1) / (16 * TB), nbn = a.Npad / 256;
    const unsigned nb = static_cast<unsigned>(nbm * nbn);
    const PSampleEpi ep = a.epi ? *a.epi : PSampleEpi{};
    if (a.epi)
        wq_horner16_kernel<float, 1, MODE, TB, BITS><<<nb, 512, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                               a.epi->x_prev, a.N, a.Npad, nbm, nbn, ep);
    else if (y_f32)
        wq_horner16_kernel<float, 0, MODE, TB, BITS><<<nb, 512, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                               static_cast<float *>(a.Y), a.N, a.Npad, nbm, nbn, ep);
    else
        wq_horner16_kernel<__half, 0, MODE, TB, BITS><<<nb, 512, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                                static_cast<__half *>(a.Y), a.N, a.Npad, nbm, nbn, ep);
}

}  // namespace

int launch_horner_kg2_gemm(const HornerGemmArgs &a, int y_f32, hipStream_t st) {
    const int nbm = (a.M + 255) / 256, nbn = a.Npad / 128;
    const unsigned nb = static_cast<unsigned>(nbm * nbn);
    const PSampleEpi ep = a.epi ? *a.epi : PSampleEpi{};
    if (a.epi)
        wq_horner_kg2_kernel<float, 1><<<nb, 512, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                          a.epi->x_prev, a.N, a.Npad, nbm, nbn, ep);
    else if (y_f32)
        wq_horner_kg2_kernel<float, 0><<<nb, 512, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                          static_cast<float *>(a.Y), a.N, a.Npad, nbm, nbn, ep);
    else
        wq_horner_kg2_kernel<__half, 0><<<nb, 512, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                           static_cast<__half *>(a.Y), a.N, a.Npad, nbm, nbn, ep);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

#if DLLM_LAB   // launchers and A/B dispatch of the lab Horner variants
#include "lab/horner_lab_launch.inc"
#endif

int launch_horner_gemm(const HornerGemmArgs &a, int y_f32, hipStream_t st) {
#if DLLM_LAB
    if (a.lab && a.bits == 4) return launch_horner_lab(a, y_f32, st);
#endif
    if (a.bits == 2) launch_horner16_t<1 | 256 | 1024, 16, 2>(a, y_f32, st);
    else launch_horner16_t<1 | 256 | 1024>(a, y_f32, st);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

}  // namespace dllm
