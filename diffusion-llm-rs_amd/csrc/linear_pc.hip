// linear_pc.hip -- the exact-weight int4 g128 GEMM in Horner form on 128-token x 256-column tiles
// with PRODUCER / CONSUMER waves: the kernel of the grids where 256 x 256 tiles leave CUs idle and
// 128 x 256 tiles fill a round (M = 2048 at N = 4096: config C2 and 11 of the 12 GEMMs of a C5
// step; the 2-GPU column shard M = 4096 x N 2048).
//
// Replaces SimpleDiffusionModel::forward = x.dot(W) + b (diffuse-llm-rs/src/lib.rs:806-813) with W
// quantized per (column n, 128-row group g) by quantize_tensor (quantization.rs:38-68), the weight
// being the reference's f32 a2 value (q - zp) * s (quantization.rs:81-85): the MFMA A operand is the
// exact integer q - zp (f16) and the f32 scale enters in Horner form (linear_horner.hip):
//   acc <- acc * r_g + T_g,  r_g = s_{g-1} / s_g,  T_g = sum_{k in g} X (q - zp),
// and the epilogue multiplies by s_{G-1}.  Same arithmetic, fragment maps and weight layout as
// wq_horner16_kernel, so the bits equal that kernel's on the same tile shape.
//
// Why producer waves: in the kernels where every wave issues its own share of the stage's LDS-DMA,
// each 1-KiB piece costs the issuing wave ~60-185 cycles of issue (MI355X_MICROARCH.md, LDS-DMA
// piece row), and that time is lost to its MFMA stream: on the 128-token tiles the load issue and
// the MFMA issue were measured to serialise (4-GPU shard: loads alone 28.9 us, MFMAs alone 29.1,
// together 37.7; profiles/r05_shard/).  Here 12 waves share the block: 8 CONSUMER waves (two per
// SIMD; wave tile 32 columns x 128 tokens, 16x16x32 MFMAs) never issue a global load, and 4
// PRODUCER waves (one per SIMD) issue every DMA piece of the stage ring and never compute.  A
// stage = one 128-row group: the X tile of two 64-deep k-steps (2 x 16 KiB), the consumers' weight
// words (2 x 8 KiB) and the group's {zp, scale} pairs and ratios (2 KiB); 3 stages in a ring.  Per
// stage: the producers issue stage s + 2 into the slot the consumers left at the last barrier,
// wait (counted vmcnt) until stage s + 1 has landed and join the barrier; the consumers compute
// stage s and join the barrier.  One s_barrier per stage for all 12 waves.
//
// Register budget: 12 waves = 3 per SIMD, so every wave gets at most 168 VGPRs.  The consumers fit
// by streaming the B fragments in half-substep buffers (4 token blocks, 16 VGPRs) instead of whole
// double-buffered substeps (64 VGPRs).
#include "linear_common.hpp"

#include <type_traits>

// DLLM_PC_ABL = 4 (128 x 256 kernel): the consumers build their A fragments in the first stage only (no
// dequant VALU after it).
// DLLM_PC_ABL (A/B builds only, results wrong, timing only): 1 = the producers issue no DMA after
// the prologue (the consumers' compute + barriers alone); 2 = the consumers issue no MFMA (operands
// kept live: loads + VALU + LDS reads + barriers); 3 = the consumers only join the barriers (the
// producers' DMA stream alone).
#ifndef DLLM_PC_ABL
#define DLLM_PC_ABL 0
#endif
// DLLM_PC_STAG = 1: consumer waves 4..7 (each SIMD's second consumer) run half a stage behind waves
// 0..3, with a barrier for all 12 waves at every half stage, so a SIMD's two consumers do not reach
// their stage-opening LDS reads and dequant (the MFMA pipe's idle head) together.  The ring keeps 3
// slots: stage u + 2 is issued at the start of half step 2u + 1 into the slot whose last reader (the
// late half) finished at half step 2u, and must land by the end of half step 2u + 3.
#ifndef DLLM_PC_STAG
#define DLLM_PC_STAG 1
#endif
#ifndef DLLM_PC_KG2_STAG   // the same stagger in the two-k-group kernel (k-group 1 behind k-group 0)
#define DLLM_PC_KG2_STAG DLLM_PC_STAG
#endif
// DLLM_PC_MF: the consumers' MFMA shape.  16: 16x16x32 (wq_horner16_kernel's fragments; per wave 2
// column blocks x 8 token blocks); 32: 32x32x16 (per wave 4 token reps of 32 x 32, A fragments
// straight from the prefill layout's words -- no permlane swap -- and half the MFMA issue per flop).
#ifndef DLLM_PC_MF
#define DLLM_PC_MF 16
#endif
// DLLM_PC_BFULL = 1 (16x16x32): a substep's 8 B fragments double-buffered whole (64 VGPRs, the
// next substep's read beside this one's 16 MFMAs) instead of half-substep buffers (32 VGPRs).
#ifndef DLLM_PC_BFULL
#define DLLM_PC_BFULL 0
#endif

namespace dllm {
namespace {

typedef float fx4p_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4p_t __attribute__((ext_vector_type(4)));

constexpr int kPcCons = 8;                        // consumer waves (2 per SIMD)
constexpr int kPcProd = 4;                        // producer waves (1 per SIMD)
constexpr int kPcThreads = (kPcCons + kPcProd) * 64;
constexpr int kPcRows = 128;                      // tokens per tile
constexpr int kPcXSub = kPcRows * kBK * 2;        // one 64-deep k-step's X sub-tile (16 KiB)
constexpr int kPcXB = 2 * kPcXSub;                // X per stage (32 KiB)
constexpr int kPcW1 = kPcCons * 1024;             // one k-step's weight words (8 KiB)
constexpr int kPcWB = 2 * kPcW1;
constexpr int kPcG = 2048;                        // group data: sz pairs (1 KiB) + ratios (1 KiB)
constexpr int kPcStage = kPcXB + kPcWB + kPcG;    // 51200 B; 3 stages = 150 KiB
constexpr int kPcRing = 3;
// DMA pieces a producer issues per stage: 4 X row blocks x 2 k-steps, 2 consumers' words x 2
// k-steps, and (producers 0 / 1) the group's sz pairs / ratios
constexpr int kPcPieces = 4 * 2 + 2 * 2;

template <typename YT, int EPI, int MF>
__global__ void __launch_bounds__(kPcThreads, 1)
wq_horner_pc_kernel(const __half *__restrict__ X, int M, int K, const uint32_t *__restrict__ wdev,
                    const uint32_t *__restrict__ sz, const float *__restrict__ hr, const float *__restrict__ sf,
                    const float *__restrict__ bias, YT *__restrict__ Y, int N, int Npad, int nbm, int nbn,
                    PSampleEpi epi) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kPcRing * kPcStage];

    // XCD-aware bijective remap, then tiles in groups of 4 row blocks, column-major inside a group:
    // the 32 tiles an XCD runs at once are 4 row blocks x 8 column blocks (4 MiB of X + 4 MiB of
    // weight words through its L2 at K = 4096, against 10 MiB for 2 x 16)
    const int nb = nbm * nbn, orig = blockIdx.x;
    const int xcd = orig % kXCDs, q8 = nb / kXCDs, r8 = nb % kXCDs;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / kXCDs;
    constexpr int kGM = 4;
    const int grp = tile / (kGM * nbn), first = grp * kGM, gm = min(kGM, nbm - first);
    const int in_grp = tile - grp * kGM * nbn;
    const int bm = first + in_grp % gm, bn = in_grp / gm;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m0 = bm * kPcRows, n0 = bn * 256;
    const int nk = K / kBK;    // 64-deep k-steps
    const int ns = nk / 2;     // stages = 128-row groups
    const uint32_t sbase = __builtin_amdgcn_readfirstlane(lds_addr(smem));
    const bool full = (m0 + kPcRows <= M) && (n0 + 256 <= N) && (N % 8) == 0;
    constexpr bool kHalfY = std::is_same<YT, __half>::value && EPI == 0;

    if (wave >= kPcCons) {
        // ---------------- producer p: X row blocks p + 4 j of both k-steps, the weight words of
        // consumer waves 2p and 2p + 1, and (p = 0 / 1) the group's sz pairs / ratios
        const int p = wave - kPcCons;
        uint32_t xo[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = (p + 4 * j) * 8 + (lane >> 3);
            const int rrow = (m0 + row < M ? m0 + row : M - 1) - m0;   // rows past M re-read row M - 1
            const int c = (lane & 7) ^ ((row >> 1) & (MF == 16 ? 5 : 7));   // the consumers' chunk swizzle
            xo[j] = static_cast<uint32_t>((rrow * K + c * 8) * 2);
        }
        const __amdgpu_buffer_rsrc_t xr = raw_rsrc(X + static_cast<size_t>(m0) * K);
        const uint32_t nt0 = static_cast<uint32_t>(n0 + 64 * p) >> 5;   // consumer 2p's 32-column tile
        const __amdgpu_buffer_rsrc_t wr0 = raw_rsrc(wdev + static_cast<size_t>(nt0) * nk * 64 * 4);
        const __amdgpu_buffer_rsrc_t wr1 = raw_rsrc(wdev + static_cast<size_t>(nt0 + 1) * nk * 64 * 4);
        const __amdgpu_buffer_rsrc_t gr =
            raw_rsrc(p == 0 ? static_cast<const void *>(sz + n0) : static_cast<const void *>(hr + n0));
        const bool has_g = p < 2;
        const uint32_t vo = static_cast<uint32_t>(lane * 16);
        auto stage = [&](int slot, int st) __attribute__((always_inline)) {
            const uint32_t base = sbase + static_cast<uint32_t>(slot * kPcStage);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const uint32_t sx = static_cast<uint32_t>((2 * st + kk) * kBK * 2);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    blds16_asm(xr, xo[j], sx, base + static_cast<uint32_t>(kk * kPcXSub + (p + 4 * j) * 1024));
                const uint32_t sw = static_cast<uint32_t>((2 * st + kk) * 1024);
                blds16_asm(wr0, vo, sw, base + static_cast<uint32_t>(kPcXB + kk * kPcW1 + (2 * p) * 1024));
                blds16_asm(wr1, vo, sw, base + static_cast<uint32_t>(kPcXB + kk * kPcW1 + (2 * p + 1) * 1024));
            }
            if (has_g)
                blds16_asm(gr, vo, static_cast<uint32_t>(st * Npad * 4),
                           base + static_cast<uint32_t>(kPcXB + kPcWB + p * 1024));
        };
        // until only the newest stage's pieces are in flight
        auto wait_one = [&]() __attribute__((always_inline)) {
            if (has_g) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPcPieces + 1) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPcPieces) : "memory");
        };
        stage(0, 0);
        if (ns > 1) {
            stage(1, 1);
            wait_one();   // stage 0 landed
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
#if DLLM_PC_STAG
        int slot = 2;
        for (int u = 0; u < ns; ++u) {
            __builtin_amdgcn_s_barrier();   // end of half step 2u (the early consumers' first half)
            if (u + 2 < ns && DLLM_PC_ABL != 1) {
                stage(slot, u + 2);   // slot of stage u - 1: its late readers finished at half step 2u
                wait_one();           // stage u + 1 landed (the early consumers open it at half step 2u + 2)
                slot = slot == kPcRing - 1 ? 0 : slot + 1;
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();   // end of half step 2u + 1
        }
        __builtin_amdgcn_s_barrier();       // end of half step 2 ns (the late consumers' last half)
#else
        int slot = 2;
        for (int s = 0; s < ns; ++s) {
            if (s + 2 < ns && DLLM_PC_ABL != 1) {
                stage(slot, s + 2);   // the slot stage s - 1 used: read before the last barrier
                wait_one();           // stage s + 1 landed
                slot = slot == kPcRing - 1 ? 0 : slot + 1;
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();
        }
#endif
        if (!(kHalfY && full)) return;
        // the coalesced f16 epilogue: the consumers write the tile image, every wave stores rows
        __syncthreads();
        const int c = lane & 31;
        for (int i = wave; i < kPcRows / 2; i += kPcCons + kPcProd) {
            const int t = 2 * i + (lane >> 5);
            const uint4 v = *reinterpret_cast<const uint4 *>(smem + t * 512 + ((c ^ (t & 31)) * 16));
            typedef unsigned int u4nt __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(u4nt{v.x, v.y, v.z, v.w},
                                        reinterpret_cast<u4nt *>(Y + static_cast<size_t>(m0 + t) * N + n0 + 8 * c));
        }
        return;
    }

    if constexpr (MF == 32) {
        // ---------------- consumer wave (32x32x16): columns n0 + 32 wave .. + 32, tokens as 4 reps
        // of 32; acc[r] reg e = (token 32 r + (lane & 31), column 32 wave + 4 hsel + 8 (e >> 2) + (e & 3))
        float16_t acc[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[r][e] = 0.0f;
        const int hsel = lane >> 5;
        const int rowx = ((lane & 31) >> 1) & 7;
        int soff[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) soff[j] = (lane & 31) * (kBK * 2) + (((2 * j + hsel) ^ rowx) << 4);
        ExactConsts ec;
        uint32_t w0[4], w1[4];
        float4 r4[4];
        half8_t bA[4], bB[4], aA, aB;
        // substep v = 0..7: k-step v >> 2, 16-deep step v & 3
        auto read_b = [&](half8_t (&b)[4], const uint8_t *sb, int v) __attribute__((always_inline)) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                b[r] = *reinterpret_cast<const half8_t *>(sb + (v >> 2) * kPcXSub + soff[v & 3] + r * 32 * kBK * 2);
        };
        auto deq = [&](int v) __attribute__((always_inline)) {
            return v < 4 ? dequant_exact<4>(w0, v & 3, ec) : dequant_exact<4>(w1, v & 3, ec);
        };
        auto mma = [&](int r, const half8_t &a, const half8_t &b) __attribute__((always_inline)) {
#if DLLM_PC_ABL == 2 || DLLM_PC_ABL == 3
            asm volatile("" ::"v"(a), "v"(b));
            asm volatile("" : "+v"(acc[r]));
#else
            acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[r], 0, 0, 0);
#endif
        };
        auto rescale = [&](int r) __attribute__((always_inline)) {
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                acc[r][4 * qd + 0] *= r4[qd].x;
                acc[r][4 * qd + 1] *= r4[qd].y;
                acc[r][4 * qd + 2] *= r4[qd].z;
                acc[r][4 * qd + 3] *= r4[qd].w;
            }
        };
        // substep v: 4 MFMAs (the token reps) on bc / ac beside the next substep's B reads and dequant;
        // v = 0 rescales each rep right before its first MFMA of the group
        auto sub = [&](const uint8_t *sb, half8_t (&bc)[4], half8_t (&bn)[4], const half8_t &ac, half8_t &an, int v)
            __attribute__((always_inline)) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
            if (v < 7) {
                read_b(bn, sb, v + 1);
                an = deq(v + 1);
            }
            if (v == 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    rescale(r);
                    mma(r, ac, bc[r]);
                }
                __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (i + 1 < 4) __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) mma(r, ac, bc[r]);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                }
            }
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
        };
        auto step = [&](int slot) __attribute__((always_inline)) {
            const uint8_t *sb = smem + slot * kPcStage;
#if DLLM_PC_ABL == 3
            asm volatile("" : "+v"(acc[0]));
            __builtin_amdgcn_s_barrier();
            return;
#endif
            {
                const uint4 v0 = *reinterpret_cast<const uint4 *>(sb + kPcXB + wave * 1024 + lane * 16);
                const uint4 v1 = *reinterpret_cast<const uint4 *>(sb + kPcXB + kPcW1 + wave * 1024 + lane * 16);
                w0[0] = v0.x; w0[1] = v0.y; w0[2] = v0.z; w0[3] = v0.w;
                w1[0] = v1.x; w1[1] = v1.y; w1[2] = v1.z; w1[3] = v1.w;
            }
            {
                const uint8_t *gb = sb + kPcXB + kPcWB;
                half2_t nz, sc;
                split_sz(*reinterpret_cast<const uint32_t *>(gb + (wave * 32 + (lane & 31)) * 4), nz, sc);
                ec = exact_consts(nz);
                const float *rl = reinterpret_cast<const float *>(gb + 1024) + wave * 32 + 4 * hsel;
#pragma unroll
                for (int qd = 0; qd < 4; ++qd) r4[qd] = *reinterpret_cast<const float4 *>(rl + 8 * qd);
            }
            read_b(bA, sb, 0);
            aA = deq(0);
            sub(sb, bA, bB, aA, aB, 0);
            sub(sb, bB, bA, aB, aA, 1);
            sub(sb, bA, bB, aA, aB, 2);
            sub(sb, bB, bA, aB, aA, 3);
#if DLLM_PC_STAG
            __builtin_amdgcn_s_barrier();   // the half-stage barrier
            __builtin_amdgcn_sched_barrier(0);
#endif
            sub(sb, bA, bB, aA, aB, 4);
            sub(sb, bB, bA, aB, aA, 5);
            sub(sb, bA, bB, aA, aB, 6);
            sub(sb, bB, bA, aB, aA, 7);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
        };

        __builtin_amdgcn_s_barrier();   // stage 0 landed (the producers' prologue wait)
        __builtin_amdgcn_sched_barrier(0);
#if DLLM_PC_STAG
        const bool late = wave >= kPcCons / 2;
        if (late) __builtin_amdgcn_s_barrier();
#endif
        for (int s = 0; s < ns; s += kPcRing) {
            step(0);
            if (s + 1 < ns) step(1);
            if (s + 2 < ns) step(2);
        }
#if DLLM_PC_STAG
        if (!late) __builtin_amdgcn_s_barrier();
#endif
        // acc = sum_g T_g s_g / s_{G-1}: times the last group's scales, then the bias
        const int nb0 = n0 + wave * 32 + 4 * hsel;   // + 8 qd: the lane's 4 columns of quad qd
        const float *sl = sf + static_cast<size_t>(ns - 1) * Npad + nb0;
        float4 bv[4];
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
            const float4 sv = *reinterpret_cast<const float4 *>(sl + 8 * qd);
            bv[qd] = *reinterpret_cast<const float4 *>(bias + nb0 + 8 * qd);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                acc[r][4 * qd + 0] *= sv.x;
                acc[r][4 * qd + 1] *= sv.y;
                acc[r][4 * qd + 2] *= sv.z;
                acc[r][4 * qd + 3] *= sv.w;
            }
        }
        if constexpr (EPI == 1) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + 32 * r + (lane & 31);
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
        if constexpr (kHalfY) {
            if (full) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int t = 32 * r + (lane & 31);
#pragma unroll
                    for (int qd = 0; qd < 4; ++qd) {
                        const int pc = (4 * wave + qd) ^ (t & 31);
                        union { __half h[4]; uint2 u; } pk;
                        pk.h[0] = __float2half_rn(acc[r][4 * qd + 0] + bv[qd].x);
                        pk.h[1] = __float2half_rn(acc[r][4 * qd + 1] + bv[qd].y);
                        pk.h[2] = __float2half_rn(acc[r][4 * qd + 2] + bv[qd].z);
                        pk.h[3] = __float2half_rn(acc[r][4 * qd + 3] + bv[qd].w);
                        *reinterpret_cast<uint2 *>(smem + t * 512 + pc * 16 + hsel * 8) = pk.u;
                    }
                }
                __syncthreads();
                const int c = lane & 31;
                for (int i = wave; i < kPcRows / 2; i += kPcCons + kPcProd) {
                    const int t = 2 * i + (lane >> 5);
                    const uint4 v = *reinterpret_cast<const uint4 *>(smem + t * 512 + ((c ^ (t & 31)) * 16));
                    typedef unsigned int u4nt __attribute__((ext_vector_type(4)));
                    __builtin_nontemporal_store(u4nt{v.x, v.y, v.z, v.w},
                                                reinterpret_cast<u4nt *>(Y + static_cast<size_t>(m0 + t) * N + n0 + 8 * c));
                }
                return;
            }
        }
        const bool vec_ok = (N % 4) == 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 32 * r + (lane & 31);
            if (m >= M) continue;
            YT *yrow = Y + static_cast<size_t>(m) * N;
#pragma unroll
            for (int qd = 0; qd < 4; ++qd)
                store_out4<YT>(yrow, bias, nb0 + 8 * qd, N, vec_ok, acc[r][4 * qd + 0], acc[r][4 * qd + 1],
                               acc[r][4 * qd + 2], acc[r][4 * qd + 3]);
        }
        return;
    } else {
    // ---------------- consumer wave: columns n0 + 32 wave .. + 32, all 128 tokens
    fx4p_t acc[8][2];
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) acc[t][cb] = fx4p_t{0.f, 0.f, 0.f, 0.f};

    const int row16 = lane & 15, rq = lane >> 4;
    const int cq = ((rq & 1) << 1) | (rq >> 1);   // k-chunk of lane row rq after the swap: 0, 2, 1, 3
    int soff[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) soff[h] = row16 * (kBK * 2) + (((4 * h + cq) ^ ((row16 >> 1) & 5)) << 4);

    ExactConsts ec;
    uint32_t w0[4], w1[4];
    float4 r4[2];
    half8_t a00, a01, a10, a11;
    half8_t bP[4], bQ[4];
    bool a_done = false;
    // B fragments of token blocks 4 hb .. 4 hb + 3 of substep j (k-step j >> 1, half j & 1)
    auto read_bh = [&](half8_t (&b)[4], const uint8_t *sb, int j, int hb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            b[i] = *reinterpret_cast<const half8_t *>(sb + (j >> 1) * kPcXSub + soff[j & 1] +
                                                      (4 * hb + i) * 16 * kBK * 2);
    };
    // A fragments of half h for column blocks 0 and 1 from the words of one k-step (as
    // wq_horner16_kernel: dequant_exact of words 2h, 2h + 1 and one v_permlane16_swap per VGPR)
    auto make_a = [&](const uint32_t (&w)[4], int h, half8_t &c0, half8_t &c1) __attribute__((always_inline)) {
        u32x4p_t u0 = __builtin_bit_cast(u32x4p_t, dequant_exact<4>(w, 2 * h, ec));
        u32x4p_t u1 = __builtin_bit_cast(u32x4p_t, dequant_exact<4>(w, 2 * h + 1, ec));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const auto r = __builtin_amdgcn_permlane16_swap(u0[e], u1[e], false, false);
            u0[e] = r[0];
            u1[e] = r[1];
        }
        c0 = __builtin_bit_cast(half8_t, u0);
        c1 = __builtin_bit_cast(half8_t, u1);
    };
    auto mma = [&](int t, int cb, const half8_t &a, const half8_t &b) __attribute__((always_inline)) {
#if DLLM_PC_ABL == 2 || DLLM_PC_ABL == 3
        asm volatile("" ::"v"(a), "v"(b));
        asm volatile("" : "+v"(acc[t][cb]));
#else
        acc[t][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[t][cb], 0, 0, 0);
#endif
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
#if DLLM_PC_BFULL
    half8_t bF0[8], bF1[8];
    auto read_b = [&](half8_t (&b)[8], const uint8_t *sb, int j) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            b[i] = *reinterpret_cast<const half8_t *>(sb + (j >> 1) * kPcXSub + soff[j & 1] + i * 16 * kBK * 2);
    };
    // Substep j: 16 MFMAs (8 token blocks x both column blocks) beside the next substep's B reads and A
    auto full_step = [&](const uint8_t *sb, half8_t (&bc)[8], half8_t (&bn)[8], int j) __attribute__((always_inline)) {
        const half8_t &a0 = (j & 1) ? a10 : a00;
        const half8_t &a1 = (j & 1) ? a11 : a01;
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        if (j < 3) {
            read_b(bn, sb, j + 1);
            if (j == 0) make_a(w0, 1, a10, a11);
            else if (j == 1) make_a(w1, 0, a00, a01);
            else make_a(w1, 1, a10, a11);
        }
        if (j == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                rescale(i);
                mma(i, 0, a0, bc[i]);
                mma(i, 1, a1, bc[i]);
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
                mma(i, 0, a0, bc[i]);
                mma(i, 1, a1, bc[i]);
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
#endif
    // Half hb of substep j: 8 MFMAs (token blocks 4 hb .. + 3, both column blocks) on `bc`, beside
    // the reads of the next half's B fragments into `bn` and (hb = 0) the next substep's A fragments.
    auto half_step = [&](const uint8_t *sb, half8_t (&bc)[4], half8_t (&bn)[4], int j, int hb)
        __attribute__((always_inline)) {
        const half8_t &a0 = (j & 1) ? a10 : a00;
        const half8_t &a1 = (j & 1) ? a11 : a01;
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        if (hb == 0) read_bh(bn, sb, j, 1);
        else if (j < 3) read_bh(bn, sb, j + 1, 0);
        if (hb == 0 && j < 3 && !(DLLM_PC_ABL == 4 && a_done)) {   // the next substep's A fragments (its half is the other one)
            if (j == 0) make_a(w0, 1, a10, a11);
            else if (j == 1) make_a(w1, 0, a00, a01);
            else make_a(w1, 1, a10, a11);
        }
        if (j == 0) {
            // acc <- acc * r_g right before each token block's first MFMA of the group
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                rescale(4 * hb + i);
                mma(4 * hb + i, 0, a0, bc[i]);
                mma(4 * hb + i, 1, a1, bc[i]);
            }
            __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (i + 1 < 4) __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                mma(4 * hb + i, 0, a0, bc[i]);
                mma(4 * hb + i, 1, a1, bc[i]);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
            }
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    // One stage (group) on ring slot `slot`
    auto step = [&](int slot) __attribute__((always_inline)) {
        const uint8_t *sb = smem + slot * kPcStage;
#if DLLM_PC_ABL == 3
        asm volatile("" : "+v"(acc[0][0]));
        __builtin_amdgcn_s_barrier();
        return;
#endif
        {
            const uint4 v0 = *reinterpret_cast<const uint4 *>(sb + kPcXB + wave * 1024 + lane * 16);
            const uint4 v1 = *reinterpret_cast<const uint4 *>(sb + kPcXB + kPcW1 + wave * 1024 + lane * 16);
            w0[0] = v0.x; w0[1] = v0.y; w0[2] = v0.z; w0[3] = v0.w;
            w1[0] = v1.x; w1[1] = v1.y; w1[2] = v1.z; w1[3] = v1.w;
        }
        {
            const uint8_t *gb = sb + kPcXB + kPcWB;
            half2_t nz, sc;
            split_sz(*reinterpret_cast<const uint32_t *>(gb + (wave * 32 + (lane & 31)) * 4), nz, sc);
            ec = exact_consts(nz);
            const float *rl = reinterpret_cast<const float *>(gb + 1024) + wave * 32 + 4 * rq;
            r4[0] = *reinterpret_cast<const float4 *>(rl);
            r4[1] = *reinterpret_cast<const float4 *>(rl + 16);
        }
#if DLLM_PC_BFULL
        read_b(bF0, sb, 0);
        make_a(w0, 0, a00, a01);
        full_step(sb, bF0, bF1, 0);
        full_step(sb, bF1, bF0, 1);
#if DLLM_PC_STAG
        __builtin_amdgcn_s_barrier();   // the half-stage barrier (nothing to wait for: reads only)
        __builtin_amdgcn_sched_barrier(0);
#endif
        full_step(sb, bF0, bF1, 2);
        full_step(sb, bF1, bF0, 3);
#else
        read_bh(bP, sb, 0, 0);
        if (!(DLLM_PC_ABL == 4 && a_done)) make_a(w0, 0, a00, a01);
        half_step(sb, bP, bQ, 0, 0);
        half_step(sb, bQ, bP, 0, 1);
        half_step(sb, bP, bQ, 1, 0);
        half_step(sb, bQ, bP, 1, 1);
#if DLLM_PC_STAG
        __builtin_amdgcn_s_barrier();   // the half-stage barrier (nothing to wait for: reads only)
        __builtin_amdgcn_sched_barrier(0);
#endif
        half_step(sb, bP, bQ, 2, 0);
        half_step(sb, bQ, bP, 2, 1);
        half_step(sb, bP, bQ, 3, 0);
        half_step(sb, bQ, bP, 3, 1);
#endif
        a_done = true;   // (DLLM_PC_ABL 4: A fragments built in the first stage only)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    __builtin_amdgcn_s_barrier();   // stage 0 landed (the producers' prologue wait)
    __builtin_amdgcn_sched_barrier(0);
#if DLLM_PC_STAG
    const bool late = wave >= kPcCons / 2;
    if (late) __builtin_amdgcn_s_barrier();   // enter half a stage behind
#endif
    for (int s = 0; s < ns; s += kPcRing) {
        step(0);
        if (s + 1 < ns) step(1);
        if (s + 2 < ns) step(2);
    }
#if DLLM_PC_STAG
    if (!late) __builtin_amdgcn_s_barrier();  // pairs with the late half's last barrier
#endif

    // acc = sum_g T_g s_g / s_{G-1}: times the last group's scales, then the bias
    const int nc0 = n0 + wave * 32 + 4 * rq;   // + 16 cb: the lane's 4 columns of column block cb
    const float *sl = sf + static_cast<size_t>(ns - 1) * Npad + nc0;
    float4 bv[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
        const float4 s = *reinterpret_cast<const float4 *>(sl + 16 * cb);
        bv[cb] = *reinterpret_cast<const float4 *>(bias + nc0 + 16 * cb);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            acc[t][cb][0] *= s.x;
            acc[t][cb][1] *= s.y;
            acc[t][cb][2] *= s.z;
            acc[t][cb][3] *= s.w;
        }
    }
    if constexpr (EPI == 1) {
        // token block t + 1's x_t values and row coefficients are loaded before block t's stores
        // (psample4_x): each block's loads are in flight during the previous block's noise draw,
        // instead of one serial round trip per 4-column group behind the stores
        float4 xa[2], xn[2];
        float ca[3], cn[3];
        auto load_blk = [&](int t, float4 (&x)[2], float (&c)[3]) __attribute__((always_inline)) {
            const int m = m0 + 16 * t + row16;
            const bool mok = m < M;
            const float *cp = epi.coef + 3 * ((mok ? m : 0) / epi.rps);
            c[0] = cp[0]; c[1] = cp[1]; c[2] = cp[2];
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
                x[cb] = mok && nc0 + 16 * cb < N
                            ? *reinterpret_cast<const float4 *>(epi.x_t + static_cast<size_t>(m) * N + nc0 + 16 * cb)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        };
        load_blk(0, xa, ca);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (t + 1 < 8) load_blk(t + 1, xn, cn);
            const int m = m0 + 16 * t + row16;
            if (m < M) {
#pragma unroll
                for (int cb = 0; cb < 2; ++cb) {
                    if (nc0 + 16 * cb >= N) continue;
                    psample4_x(epi, static_cast<size_t>(m) * N + nc0 + 16 * cb, xa[cb], ca[0], ca[1], ca[2],
                               acc[t][cb][0] + bv[cb].x, acc[t][cb][1] + bv[cb].y, acc[t][cb][2] + bv[cb].z,
                               acc[t][cb][3] + bv[cb].w);
                }
            }
            if (t + 1 < 8) {
                xa[0] = xn[0]; xa[1] = xn[1];
                ca[0] = cn[0]; ca[1] = cn[1]; ca[2] = cn[2];
            }
        }
        return;
    }
    if constexpr (kHalfY) {
        if (full) {
            // the f16 tile through the drained ring: rows of 512 B, 16-B chunks XORed with the row;
            // then all 12 waves store whole rows as 16-B lanes (producers included, above)
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int r = 16 * t + row16;
#pragma unroll
                for (int cb = 0; cb < 2; ++cb) {
                    const int pc = (4 * wave + 2 * cb + (rq >> 1)) ^ (r & 31);
                    union { __half h[4]; uint2 u; } pk;
                    pk.h[0] = __float2half_rn(acc[t][cb][0] + bv[cb].x);
                    pk.h[1] = __float2half_rn(acc[t][cb][1] + bv[cb].y);
                    pk.h[2] = __float2half_rn(acc[t][cb][2] + bv[cb].z);
                    pk.h[3] = __float2half_rn(acc[t][cb][3] + bv[cb].w);
                    *reinterpret_cast<uint2 *>(smem + r * 512 + pc * 16 + (rq & 1) * 8) = pk.u;
                }
            }
            __syncthreads();
            const int c = lane & 31;
            for (int i = wave; i < kPcRows / 2; i += kPcCons + kPcProd) {
                const int t = 2 * i + (lane >> 5);
                const uint4 v = *reinterpret_cast<const uint4 *>(smem + t * 512 + ((c ^ (t & 31)) * 16));
                typedef unsigned int u4nt __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(u4nt{v.x, v.y, v.z, v.w},
                                            reinterpret_cast<u4nt *>(Y + static_cast<size_t>(m0 + t) * N + n0 + 8 * c));
            }
            return;
        }
    }
    const bool vec_ok = (N % 4) == 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const int m = m0 + 16 * t + row16;
        if (m >= M) continue;
        YT *yrow = Y + static_cast<size_t>(m) * N;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
            store_out4<YT>(yrow, bias, nc0 + 16 * cb, N, vec_ok, acc[t][cb][0], acc[t][cb][1], acc[t][cb][2],
                           acc[t][cb][3]);
    }
    }   // MF == 16
}


// ---------------------------------------------------------------------------------------------
// Two-k-group PC kernel: 128-token x 128-column tiles for grids where 128 x 256 tiles leave CUs idle
// and 128 x 128 tiles fill a round (the 4-GPU column shard M = 4096 x N 1024, M = 2048 x N 2048).
// 8 consumers = 4 column waves (32 columns x 128 tokens, the 128 x 256 kernel's wave tile) x 2
// k-groups: k-group kg runs the Horner chain over K-half kg (the second from a zero accumulator, so
// its first ratio is harmless), and the epilogue sums acc0 s_{G/2-1} + acc1 s_{G-1} in that order.
// A stage is one 64-deep k-step of BOTH halves: 2 X sub-tiles (2 x 16 KiB), the 8 consumers' words
// (8 KiB) and, on a group's first k-step, both halves' sz pairs and ratios (4 x 1 KiB: 128 columns,
// lanes 32..63 repeating 0..31); 3 stages in a ring (132 KiB).  Producers: per stage 8 X pieces,
// 2 weight pieces and (group-first stages) 1 group piece each.  STAG (as DLLM_PC_STAG): k-group 1
// (waves 4..7, each SIMD's second consumer) runs half a stage behind k-group 0.
// TB = token blocks of 16 per tile: 8 (128 x 128 tiles), 4 (64 x 128: M = 512 at N = 4096, the
// 8-GPU shard 4096 x 512) or 2 (32 x 128: M = 256).
template <int TB>
struct K2L {
    static_assert(TB == 8 || TB == 4 || TB == 2, "128-, 64- or 32-token tiles");
    static constexpr int kRows = 16 * TB;
    static constexpr int kXSub = kRows * kBK * 2;          // one half's 64-deep X sub-tile
    static constexpr int kXB = 2 * kXSub;                   // X of both halves per stage
    static constexpr int kW = 8 * 1024;                     // 2 halves x 4 column waves x 1 KiB
    static constexpr int kG = 4 * 1024;                     // 2 halves x (sz, ratios) x 1 KiB
    static constexpr int kStage = kXB + kW + kG;            // TB 8: 45056 B (3 stages = 132 KiB)
    static constexpr int kXP = TB / 2;                      // X row blocks per producer per half
    static constexpr int kPieces = 2 * kXP + 2;             // per producer per stage, + 1 on group-first stages
    static constexpr int kXch = TB * 8 * 1024;              // k-group 1's hand-off area, then the f16 image
    static_assert(kXch + kRows * 256 <= kPcRing * kStage, "epilogue fits the drained ring");
};

template <typename YT, int EPI, int TB>
__global__ void __launch_bounds__(kPcThreads, 1)
wq_horner_pc_kg2_kernel(const __half *__restrict__ X, int M, int K, const uint32_t *__restrict__ wdev,
                        const uint32_t *__restrict__ sz, const float *__restrict__ hr, const float *__restrict__ sf,
                        const float *__restrict__ bias, YT *__restrict__ Y, int N, int Npad, int nbm, int nbn,
                        PSampleEpi epi) {
    using L = K2L<TB>;
    __shared__ __attribute__((aligned(16))) uint8_t smem[kPcRing * L::kStage];

    // XCD-aware remap; tiles in groups of 4 row blocks, column-major inside a group (an XCD's 32
    // concurrent tiles: 4 row blocks x 8 column blocks)
    const int nb = nbm * nbn, orig = blockIdx.x;
    const int xcd = orig % kXCDs, q8 = nb / kXCDs, r8 = nb % kXCDs;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / kXCDs;
    constexpr int kGM = 4;
    const int grp = tile / (kGM * nbn), first = grp * kGM, gm = min(kGM, nbm - first);
    const int in_grp = tile - grp * kGM * nbn;
    const int bm = first + in_grp % gm, bn = in_grp / gm;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m0 = bm * L::kRows, n0 = bn * 128;
    const int nk = K / kBK, nk2 = nk / 2;   // k-steps; k-steps per K-half = stages (even: K % 256 == 0)
    const uint32_t sbase = __builtin_amdgcn_readfirstlane(lds_addr(smem));
    const bool full = (m0 + L::kRows <= M) && (n0 + 128 <= N) && (N % 8) == 0;
    constexpr bool kHalfY = std::is_same<YT, __half>::value && EPI == 0;
    float4 *part = reinterpret_cast<float4 *>(smem);   // k-group 1's sums (64 KiB), then the f16 image
    uint8_t *img = smem + L::kXch;

    if (wave >= kPcCons) {
        // ---------------- producer p: X row blocks p + 4 j of both halves; the words of half p >> 1,
        // column waves 2 (p & 1) and 2 (p & 1) + 1; group data: half p >> 1, sz (p even) / ratios
        const int p = wave - kPcCons;
        uint32_t xo[L::kXP];
#pragma unroll
        for (int j = 0; j < L::kXP; ++j) {
            const int row = (p + 4 * j) * 8 + (lane >> 3);
            const int rrow = (m0 + row < M ? m0 + row : M - 1) - m0;
            const int c = (lane & 7) ^ ((row >> 1) & 5);
            xo[j] = static_cast<uint32_t>((rrow * K + c * 8) * 2);
        }
        const __amdgpu_buffer_rsrc_t xr = raw_rsrc(X + static_cast<size_t>(m0) * K);
        const int wkg = p >> 1, nwa = 2 * (p & 1);
        const uint32_t nt0 = static_cast<uint32_t>(n0 + 32 * nwa) >> 5;
        const __amdgpu_buffer_rsrc_t wr0 = raw_rsrc(wdev + static_cast<size_t>(nt0) * nk * 64 * 4);
        const __amdgpu_buffer_rsrc_t wr1 = raw_rsrc(wdev + static_cast<size_t>(nt0 + 1) * nk * 64 * 4);
        const __amdgpu_buffer_rsrc_t gr =
            raw_rsrc((p & 1) == 0 ? static_cast<const void *>(sz + n0) : static_cast<const void *>(hr + n0));
        const uint32_t vo = static_cast<uint32_t>(lane * 16), go = static_cast<uint32_t>((lane & 31) * 16);
        auto stage = [&](int slot, int kt) __attribute__((always_inline)) {
            const uint32_t base = sbase + static_cast<uint32_t>(slot * L::kStage);
#pragma unroll
            for (int kg = 0; kg < 2; ++kg) {
                const uint32_t sx = static_cast<uint32_t>((kg * nk2 + kt) * kBK * 2);
#pragma unroll
                for (int j = 0; j < L::kXP; ++j)
                    blds16_asm(xr, xo[j], sx, base + static_cast<uint32_t>(kg * L::kXSub + (p + 4 * j) * 1024));
            }
            const uint32_t sw = static_cast<uint32_t>((wkg * nk2 + kt) * 1024);
            blds16_asm(wr0, vo, sw, base + static_cast<uint32_t>(L::kXB + wkg * 4096 + nwa * 1024));
            blds16_asm(wr1, vo, sw, base + static_cast<uint32_t>(L::kXB + wkg * 4096 + (nwa + 1) * 1024));
            if ((kt & 1) == 0)   // a group's first k-step: this half's sz pairs or ratios
                blds16_asm(gr, go, static_cast<uint32_t>(((wkg * nk2 + kt) >> 1) * Npad * 4),
                           base + static_cast<uint32_t>(L::kXB + L::kW + wkg * 2048 + (p & 1) * 1024));
        };
        // until only the newest stage (k-step kt2) is in flight
        auto wait_one = [&](int kt2) __attribute__((always_inline)) {
            if ((kt2 & 1) == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L::kPieces + 1) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L::kPieces) : "memory");
        };
        stage(0, 0);
        if (nk2 > 1) {
            stage(1, 1);
            wait_one(1);
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        int slot = 2;
#if DLLM_PC_KG2_STAG
        for (int u = 0; u < nk2; ++u) {
            __builtin_amdgcn_s_barrier();
            if (u + 2 < nk2) {
                stage(slot, u + 2);
                wait_one(u + 2);
                slot = slot == kPcRing - 1 ? 0 : slot + 1;
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_s_barrier();
#else
        for (int s = 0; s < nk2; ++s) {
            if (s + 2 < nk2) {
                stage(slot, s + 2);
                wait_one(s + 2);
                slot = slot == kPcRing - 1 ? 0 : slot + 1;
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();
        }
#endif
        __syncthreads();   // k-group 1's hand-off
        if (!(kHalfY && full)) return;
        __syncthreads();   // the f16 image
        const int c = lane & 15;
        for (int i = wave; i < L::kRows / 4; i += kPcCons + kPcProd) {
            const int t = 4 * i + (lane >> 4);
            const uint4 v = *reinterpret_cast<const uint4 *>(img + t * 256 + ((c ^ (t & 15)) * 16));
            typedef unsigned int u4nt __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(u4nt{v.x, v.y, v.z, v.w},
                                        reinterpret_cast<u4nt *>(Y + static_cast<size_t>(m0 + t) * N + n0 + 8 * c));
        }
        return;
    }

    // ---------------- consumer (kg, nw): columns n0 + 32 nw .. + 32, 128 tokens, K-half kg
    const int kg = wave >> 2, nw = wave & 3;
    constexpr int kHB = TB / 2;   // token blocks per half step
    fx4p_t acc[TB][2];
#pragma unroll
    for (int t = 0; t < TB; ++t)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) acc[t][cb] = fx4p_t{0.f, 0.f, 0.f, 0.f};
    const int row16 = lane & 15, rq = lane >> 4;
    const int cq = ((rq & 1) << 1) | (rq >> 1);
    int soff[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) soff[h] = row16 * (kBK * 2) + (((4 * h + cq) ^ ((row16 >> 1) & 5)) << 4);
    ExactConsts ec;
    uint32_t w[4];
    float4 r4[2];
    half8_t a00, a01, a10, a11;
    half8_t bP[kHB], bQ[kHB];
    auto read_bh = [&](half8_t (&b)[kHB], const uint8_t *sx, int h, int hb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kHB; ++i)
            b[i] = *reinterpret_cast<const half8_t *>(sx + soff[h] + (kHB * hb + i) * 16 * kBK * 2);
    };
    auto make_a = [&](int h, half8_t &c0, half8_t &c1) __attribute__((always_inline)) {
        u32x4p_t u0 = __builtin_bit_cast(u32x4p_t, dequant_exact<4>(w, 2 * h, ec));
        u32x4p_t u1 = __builtin_bit_cast(u32x4p_t, dequant_exact<4>(w, 2 * h + 1, ec));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const auto r = __builtin_amdgcn_permlane16_swap(u0[e], u1[e], false, false);
            u0[e] = r[0];
            u1[e] = r[1];
        }
        c0 = __builtin_bit_cast(half8_t, u0);
        c1 = __builtin_bit_cast(half8_t, u1);
    };
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
    // half hb of substep h (32-deep half h of the k-step): 8 MFMAs on bc beside the next half's reads
    auto half_step = [&](const uint8_t *sx, half8_t (&bc)[kHB], half8_t (&bn)[kHB], int h, int hb, bool gf)
        __attribute__((always_inline)) {
        const half8_t &a0 = h ? a10 : a00;
        const half8_t &a1 = h ? a11 : a01;
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        if (hb == 0) read_bh(bn, sx, h, 1);
        else if (h == 0) read_bh(bn, sx, 1, 0);
        if (hb == 0 && h == 0) make_a(1, a10, a11);
        if (gf && h == 0) {
#pragma unroll
            for (int i = 0; i < kHB; ++i) {
                rescale(kHB * hb + i);
                mma(kHB * hb + i, 0, a0, bc[i]);
                mma(kHB * hb + i, 1, a1, bc[i]);
            }
            __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
#pragma unroll
            for (int i = 0; i < kHB; ++i) {
                if (i + 1 < kHB) __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < kHB; ++i) {
                mma(kHB * hb + i, 0, a0, bc[i]);
                mma(kHB * hb + i, 1, a1, bc[i]);
            }
#pragma unroll
            for (int i = 0; i < kHB; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
            }
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto step = [&](int slot, auto gf_tag) __attribute__((always_inline)) {
        constexpr bool GF = decltype(gf_tag)::value;
        const uint8_t *sb = smem + slot * L::kStage;
        const uint8_t *sx = sb + kg * L::kXSub;
        {
            const uint4 v = *reinterpret_cast<const uint4 *>(sb + L::kXB + kg * 4096 + nw * 1024 + lane * 16);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        }
        if constexpr (GF) {
            const uint8_t *gb = sb + L::kXB + L::kW + kg * 2048;
            half2_t nz, sc;
            split_sz(*reinterpret_cast<const uint32_t *>(gb + (nw * 32 + (lane & 31)) * 4), nz, sc);
            ec = exact_consts(nz);
            const float *rl = reinterpret_cast<const float *>(gb + 1024) + nw * 32 + 4 * rq;
            r4[0] = *reinterpret_cast<const float4 *>(rl);
            r4[1] = *reinterpret_cast<const float4 *>(rl + 16);
        }
        read_bh(bP, sx, 0, 0);
        make_a(0, a00, a01);
        half_step(sx, bP, bQ, 0, 0, GF);
        half_step(sx, bQ, bP, 0, 1, GF);
#if DLLM_PC_KG2_STAG
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
#endif
        half_step(sx, bP, bQ, 1, 0, GF);
        half_step(sx, bQ, bP, 1, 1, GF);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    using GFt = std::integral_constant<bool, true>;
    using GFf = std::integral_constant<bool, false>;
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#if DLLM_PC_KG2_STAG
    const bool late = kg == 1;
    if (late) __builtin_amdgcn_s_barrier();
#endif
    // group = 2 k-steps, ring period 3: unroll 6 so each step's slot and group phase are static
    for (int kt = 0; kt < nk2; kt += 6) {
        step(0, GFt{});
        step(1, GFf{});
        if (kt + 2 < nk2) {
            step(2, GFt{});
            step(0, GFf{});
        }
        if (kt + 4 < nk2) {
            step(1, GFt{});
            step(2, GFf{});
        }
    }
#if DLLM_PC_KG2_STAG
    if (!late) __builtin_amdgcn_s_barrier();
#endif
    // this half's partial: acc times the half's last group scales
    const int nc0 = n0 + nw * 32 + 4 * rq;
    const float *sl = sf + static_cast<size_t>((kg + 1) * (nk2 / 2) - 1) * Npad + nc0;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
        const float4 sv = *reinterpret_cast<const float4 *>(sl + 16 * cb);
#pragma unroll
        for (int t = 0; t < TB; ++t) {
            acc[t][cb][0] *= sv.x;
            acc[t][cb][1] *= sv.y;
            acc[t][cb][2] *= sv.z;
            acc[t][cb][3] *= sv.w;
        }
    }
    // The halves' sums through LDS (the ring is drained): k-group 0 finalizes token blocks
    // [0, TB/2), k-group 1 blocks [TB/2, TB); each hands the other's blocks over and adds the ones
    // it receives (P0 + P1: IEEE addition commutes, so either side's sum is the same bits).
    constexpr int kT0 = TB / 2;
    const int t_own = kg * kT0;   // first own block
    auto hand_off = [&](auto off_tag) __attribute__((always_inline)) {   // the other k-group's blocks
        constexpr int off = decltype(off_tag)::value;
#pragma unroll
        for (int i = 0; i < kT0; ++i)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
                part[((nw * TB + off + i) * 2 + cb) * 64 + lane] =
                    make_float4(acc[off + i][cb][0], acc[off + i][cb][1], acc[off + i][cb][2], acc[off + i][cb][3]);
    };
    if (kg == 0) hand_off(std::integral_constant<int, kT0>{});
    else hand_off(std::integral_constant<int, 0>{});
    __syncthreads();
    float4 bv[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) bv[cb] = *reinterpret_cast<const float4 *>(bias + nc0 + 16 * cb);
    fx4p_t fin[kT0][2];   // the own blocks' sums
    // (each k-group's branch indexes acc with constants: a run-time index would put acc in scratch)
    auto finalize = [&](auto off_tag) __attribute__((always_inline)) {
        constexpr int off = decltype(off_tag)::value;
#pragma unroll
        for (int i = 0; i < kT0; ++i)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                const float4 o = part[((nw * TB + off + i) * 2 + cb) * 64 + lane];
                fin[i][cb] = fx4p_t{acc[off + i][cb][0] + o.x, acc[off + i][cb][1] + o.y, acc[off + i][cb][2] + o.z,
                                    acc[off + i][cb][3] + o.w};
            }
    };
    if (kg == 0) finalize(std::integral_constant<int, 0>{});
    else finalize(std::integral_constant<int, kT0>{});
    if constexpr (EPI == 1) {
        // block i + 1's x_t values and row coefficients are loaded before block i's stores (psample4_x)
        float4 xa[2], xn[2];
        float ca[3], cn[3];
        auto load_blk = [&](int t, float4 (&x)[2], float (&c)[3]) __attribute__((always_inline)) {
            const int m = m0 + 16 * t + row16;
            const bool mok = m < M;
            const float *cp = epi.coef + 3 * ((mok ? m : 0) / epi.rps);
            c[0] = cp[0]; c[1] = cp[1]; c[2] = cp[2];
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
                x[cb] = mok && nc0 + 16 * cb < N
                            ? *reinterpret_cast<const float4 *>(epi.x_t + static_cast<size_t>(m) * N + nc0 + 16 * cb)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        };
        load_blk(t_own, xa, ca);
#pragma unroll
        for (int i = 0; i < kT0; ++i) {
            if (i + 1 < kT0) load_blk(t_own + i + 1, xn, cn);
            const int m = m0 + 16 * (t_own + i) + row16;
            if (m < M) {
#pragma unroll
                for (int cb = 0; cb < 2; ++cb) {
                    if (nc0 + 16 * cb >= N) continue;
                    psample4_x(epi, static_cast<size_t>(m) * N + nc0 + 16 * cb, xa[cb], ca[0], ca[1], ca[2],
                               fin[i][cb][0] + bv[cb].x, fin[i][cb][1] + bv[cb].y, fin[i][cb][2] + bv[cb].z,
                               fin[i][cb][3] + bv[cb].w);
                }
            }
            if (i + 1 < kT0) {
                xa[0] = xn[0]; xa[1] = xn[1];
                ca[0] = cn[0]; ca[1] = cn[1]; ca[2] = cn[2];
            }
        }
        return;
    }
    if constexpr (kHalfY) {
        if (full) {
#pragma unroll
            for (int i = 0; i < kT0; ++i) {
                const int r = 16 * (t_own + i) + row16;
#pragma unroll
                for (int cb = 0; cb < 2; ++cb) {
                    const int pc = (4 * nw + 2 * cb + (rq >> 1)) ^ (r & 15);
                    union { __half h[4]; uint2 u; } pk;
                    pk.h[0] = __float2half_rn(fin[i][cb][0] + bv[cb].x);
                    pk.h[1] = __float2half_rn(fin[i][cb][1] + bv[cb].y);
                    pk.h[2] = __float2half_rn(fin[i][cb][2] + bv[cb].z);
                    pk.h[3] = __float2half_rn(fin[i][cb][3] + bv[cb].w);
                    *reinterpret_cast<uint2 *>(img + r * 256 + pc * 16 + (rq & 1) * 8) = pk.u;
                }
            }
            __syncthreads();
            const int c = lane & 15;
            for (int i = wave; i < L::kRows / 4; i += kPcCons + kPcProd) {
                const int t = 4 * i + (lane >> 4);
                const uint4 v = *reinterpret_cast<const uint4 *>(img + t * 256 + ((c ^ (t & 15)) * 16));
                typedef unsigned int u4nt __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(u4nt{v.x, v.y, v.z, v.w},
                                            reinterpret_cast<u4nt *>(Y + static_cast<size_t>(m0 + t) * N + n0 + 8 * c));
            }
            return;
        }
    }
    const bool vec_ok = (N % 4) == 0;
#pragma unroll
    for (int i = 0; i < kT0; ++i) {
        const int m = m0 + 16 * (t_own + i) + row16;
        if (m >= M) continue;
        YT *yrow = Y + static_cast<size_t>(m) * N;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
            store_out4<YT>(yrow, bias, nc0 + 16 * cb, N, vec_ok, fin[i][cb][0], fin[i][cb][1], fin[i][cb][2],
                           fin[i][cb][3]);
    }
}

}  // namespace

int launch_horner_pc_gemm(const HornerGemmArgs &a, int y_f32, hipStream_t st) {
    if (a.K % 128 != 0 || a.Npad % 256 != 0 || a.M < 1)
        return fail(DLLM_ERR_SHAPE_MISMATCH, "Horner PC GEMM: needs K % 128 == 0 and Npad % 256 == 0");
    const int nbm = (a.M + kPcRows - 1) / kPcRows, nbn = a.Npad / 256;
    const unsigned nb = static_cast<unsigned>(nbm * nbn);
    const PSampleEpi ep = a.epi ? *a.epi : PSampleEpi{};
    if (a.epi)
        wq_horner_pc_kernel<float, 1, DLLM_PC_MF><<<nb, kPcThreads, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                                a.epi->x_prev, a.N, a.Npad, nbm, nbn, ep);
    else if (y_f32)
        wq_horner_pc_kernel<float, 0, DLLM_PC_MF><<<nb, kPcThreads, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                                static_cast<float *>(a.Y), a.N, a.Npad, nbm, nbn, ep);
    else
        wq_horner_pc_kernel<__half, 0, DLLM_PC_MF><<<nb, kPcThreads, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                                 static_cast<__half *>(a.Y), a.N, a.Npad, nbm, nbn, ep);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}


template <int TB>
int launch_pc_kg2_t(const HornerGemmArgs &a, int y_f32, hipStream_t st) {
    const int nbm = (a.M + K2L<TB>::kRows - 1) / K2L<TB>::kRows, nbn = a.Npad / 128;
    const unsigned nb = static_cast<unsigned>(nbm * nbn);
    const PSampleEpi ep = a.epi ? *a.epi : PSampleEpi{};
    if (a.epi)
        wq_horner_pc_kg2_kernel<float, 1, TB><<<nb, kPcThreads, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                                        a.epi->x_prev, a.N, a.Npad, nbm, nbn, ep);
    else if (y_f32)
        wq_horner_pc_kg2_kernel<float, 0, TB><<<nb, kPcThreads, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                                        static_cast<float *>(a.Y), a.N, a.Npad, nbm, nbn, ep);
    else
        wq_horner_pc_kg2_kernel<__half, 0, TB><<<nb, kPcThreads, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.sf, a.bias,
                                                                         static_cast<__half *>(a.Y), a.N, a.Npad, nbm, nbn, ep);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int launch_horner_pc_kg2_gemm(const HornerGemmArgs &a, int rows, int y_f32, hipStream_t st) {
    if (a.K % 256 != 0 || a.Npad % 128 != 0 || a.M < 1)
        return fail(DLLM_ERR_SHAPE_MISMATCH, "Horner PC KG2 GEMM: needs K % 256 == 0 and Npad % 128 == 0");
    switch (rows) {
    case 128: return launch_pc_kg2_t<8>(a, y_f32, st);
    case 64: return launch_pc_kg2_t<4>(a, y_f32, st);
    case 32: return launch_pc_kg2_t<2>(a, y_f32, st);
    default: return fail(DLLM_ERR_UNSUPPORTED, "Horner PC KG2 GEMM: tile rows must be 128, 64 or 32");
    }
}

}  // namespace dllm
