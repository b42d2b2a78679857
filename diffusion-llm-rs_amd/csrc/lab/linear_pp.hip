// linear_pp.hip -- ping-pong 256 x 256 group-quantized GEMM for gfx950 (MI355X).
//
// Same operator as wq_gemm8_kernel<BITS, YT, 8, 8> (linear_wq.hip): Y = X . W^ + b, W^ the int2/4/8
// group-quantized weight of SimpleDiffusionModel::forward (diffuse-llm-rs/src/lib.rs:806-813),
// computed as Y^T = W^^T X^T on the 32x32x16 f16 MFMA, with the same weight layout, the same LDS
// stage layout and the same 3-stage LDS-DMA ring, and therefore the same bits in Y.
//
// What differs is the schedule.  In the ring kernel every wave issues its stage's LDS-DMAs and its
// fragment reads at the head of each k-step, right after the barrier, so the two waves on each
// SIMD are in their load section at the same time and the MFMA pipe idles for it (the loads
// alone took 41 of the kernel's 126 us at M = 4096 and overlapped almost nothing).  Here the
// 8 waves form two groups of 4 -- one wave of each group on every SIMD -- offset by one barrier:
//   group 0: | mem | mfma | mem | mfma | ...
//   group 1: |     | mem  | mfma| mem  | ...
// so that between two consecutive barriers one wave of each SIMD runs MFMAs (at priority 1) while
// its partner reads the next substep's X fragments, dequantizes its weight fragment and issues a
// share of the next-but-one stage's LDS-DMAs.
//
// Phases: a 64-deep k-step is 4/SPP (mem, mfma) phase pairs; a mem phase reads SPP substeps' B
// fragments (8 ds_read_b128 each), dequantizes their A fragments, issues its share of the 6 DMA
// pieces of stage kt+2 (mem phases 1 .. 4/SPP - 1 only) and passes the barrier with its reads in
// flight: they retire (lgkmcnt(0)) at the head of the wave's own mfma phase.
// Synchronisation (barrier b: both groups; group g's mem phase p lies between barriers
// 2p - 1 + g and 2p + g):
//   RAW  stage kt+1 is waited for (counted vmcnt leaving stage kt+2's pieces in flight) at the end
//        of each wave's last mem phase of step kt; group 0 first reads it one barrier after
//        group 1's wait, group 1 one barrier after its own.
//   WAR  stage kt+2 overwrites stage kt-1, whose last reads (group 1's last mem phase of step
//        kt-1) retire at the head of group 1's following mfma phase, i.e. before the barrier that
//        ENDS group 0's first mem phase of step kt: so no DMA is issued in mem phase 0.
#include "linear_common.hpp"

#include <type_traits>

namespace dllm {
namespace {

// LAB (measurement only, 0 in production): 1 no LDS-DMA in the loop, 2 no dequant (raw words as
// the A operand), 8 no barriers in the loop, 16 DMAs issued but never waited for in the loop (stale
// stages), 4 DMAs issued between the MFMAs instead of in the mem phase.
template <int BITS, typename YT, int SPP, int EPI, int LAB = 0>
__global__ void __launch_bounds__(512, 1)
wq_gemm_pp_kernel(const __half *__restrict__ X, int M, int K, const uint32_t *__restrict__ wdev,
                  const uint32_t *__restrict__ sz, const float *__restrict__ bias, YT *__restrict__ Y, int N, int Npad,
                  int group, int nbm, int nbn, PSampleEpi epi) {
    using SL = StageLayout8<BITS, 8, 8, 1>;
    constexpr int MR = 8, kPhases = 4 / SPP, kXR = SL::kXRounds, kPieces = kXR + 2;
    static_assert(kXR == 4 && kPhases >= 2, "256-row tile: 4 X rounds per wave; DMAs need mem phases 1..");
    __shared__ __attribute__((aligned(16))) uint8_t st0[SL::kBytes];
    __shared__ __attribute__((aligned(16))) uint8_t st1[SL::kBytes];
    __shared__ __attribute__((aligned(16))) uint8_t st2[SL::kBytes];

    const int nb = nbm * nbn, orig = blockIdx.x;
    const int xcd = orig % kXCDs, q8 = nb / kXCDs, r8 = nb % kXCDs;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / kXCDs;
    const int bm = wgid / nbn, bn = wgid % nbn;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2;
    const int m0 = bm * 256, n0 = bn * 256;
    const unsigned nk = static_cast<unsigned>(K) / kBK;
    const unsigned kpg = static_cast<unsigned>(group) / kBK;
    const unsigned nt = static_cast<unsigned>(n0 + wave * 32) >> 5;

    const int chunk_st = lane & 7;
    const __half *xsrc[kXR];
#pragma unroll
    for (int i = 0; i < kXR; ++i) {
        const int row = (i * 8 + wave) * 8 + (lane >> 3);
        int grow = m0 + row;
        grow = grow < M ? grow : M - 1;
        const int c = chunk_st ^ ((row >> 1) & 7);
        xsrc[i] = X + static_cast<size_t>(grow) * K + c * 8;
    }
    const uint32_t *wsrc = wdev + (static_cast<size_t>(nt) * nk * 64 + lane) * BITS;
    const uint32_t *szsrc = sz + n0 + 4 * lane;
    const bool has_sz = wave == 0;
    const uint32_t wv = static_cast<uint32_t>(wave);

    // Piece p of stage kt into stage buffer sb: X rounds 0..3, the weight words, the scale dwords.
    auto piece = [&](uint8_t *sb, unsigned kt, int p) {
        const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(sb));
        if (p < kXR) {
            glds16_asm(xsrc[p] + kt * kBK, base + wv * 1024 + p * 8192);
        } else if (p == kXR) {
            const uint32_t *wp = wsrc + static_cast<size_t>(kt) * 64 * BITS;
            const uint32_t wb = base + SL::kX + wv * (64 * BITS * 4);
            if constexpr (BITS == 4) {
                glds16_asm(wp, wb);
            } else if constexpr (BITS == 8) {
                glds16_asm(wp, wb);
                glds16_asm(wp + 4, wb + 64 * 16);
            } else {
                glds4_asm(wp, wb);
                glds4_asm(wp + 1, wb + 256);
            }
        } else if (has_sz) {
            glds16_asm(szsrc + (kt / kpg) * Npad, base + SL::kX + SL::kW);
        }
    };
    auto wait_prev = [&]() {
        if (has_sz) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kXR + SL::kWOps + 1) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kXR + SL::kWOps) : "memory");
    };
    auto barrier = []() {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(LAB & 8)) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    float16_t acc[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[r][e] = 0.0f;

    const int hsel = lane >> 5;
    const int rowx = ((lane & 31) >> 1) & 7;
    const int xoff = (lane & 31) * (kBK * 2);

    auto dequant = [&](half8_t &a, const uint32_t (&w)[BITS], int s, half2_t nz, half2_t sc) {
        if constexpr (LAB & 2) {
            uint32_t raw[4] = {w[0] ^ (uint32_t)s, w[1 % BITS], w[2 % BITS], w[3 % BITS]};
            a = __builtin_bit_cast(half8_t, raw);
        } else {
            a = dequant_frag<BITS>(w, s, nz, sc);
        }
    };
    auto pieces = [&](uint8_t *pf, unsigned kt, int ph) {
#pragma unroll
        for (int p = (ph - 1) * kPieces / (kPhases - 1); p < ph * kPieces / (kPhases - 1); ++p) piece(pf, kt, p);
    };

    auto step = [&](const uint8_t *sb, uint8_t *pf, unsigned kt) {
        const bool issue = !(LAB & 1) && kt + 2 < nk;
        uint32_t w[BITS];
        half2_t nz, sc;
        half8_t a[SPP];
#pragma unroll
        for (int ph = 0; ph < kPhases; ++ph) {
            // ---- mem phase: B fragments of substeps SPP ph .. + SPP (+ the slab's words and the
            // first A fragments at ph 0), this phase's share of the DMA pieces of stage kt+2
            if (ph == 0) {
                lds_words<BITS>(w, sb + SL::kX + wave * (64 * BITS * 4), lane);
                split_sz(*reinterpret_cast<const uint32_t *>(sb + SL::kX + SL::kW + (wave * 32 + (lane & 31)) * 4), nz,
                         sc);
            }
            half8_t b[SPP][MR];
#pragma unroll
            for (int j = 0; j < SPP; ++j) {
                const int off = xoff + ((((2 * (ph * SPP + j) + hsel) ^ rowx)) << 4);
#pragma unroll
                for (int r = 0; r < MR; ++r) b[j][r] = *reinterpret_cast<const half8_t *>(sb + off + r * 32 * kBK * 2);
            }
            if (ph == 0) {
#pragma unroll
                for (int j = 0; j < SPP; ++j) dequant(a[j], w, j, nz, sc);
            }
            if (!(LAB & 4) && issue && ph > 0) pieces(pf, kt + 2, ph);
            if (ph == kPhases - 1 && !(LAB & 16)) {
                if (issue) wait_prev();
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            barrier();
            // ---- mfma phase: the fragment reads retire here, behind the barrier; the next phase's
            // A fragments are dequantized between the MFMAs (the words are already in registers)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_setprio(1);
            half8_t an[SPP];
#pragma unroll
            for (int j = 0; j < SPP; ++j)
#pragma unroll
                for (int r = 0; r < MR; ++r)
                    acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[j], b[j][r], acc[r], 0, 0, 0);
            if (ph + 1 < kPhases) {
#pragma unroll
                for (int j = 0; j < SPP; ++j) dequant(an[j], w, (ph + 1) * SPP + j, nz, sc);
            }
            if ((LAB & 4) && issue && ph > 0) pieces(pf, kt + 2, ph);
#pragma unroll
            for (int i = 0; i < SPP * MR; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            }
            if (ph + 1 < kPhases) {   // pins the dequant inside this phase (IR passes would sink it)
#pragma unroll
                for (int j = 0; j < SPP; ++j) asm volatile("" : "+v"(an[j]));
            }
            __builtin_amdgcn_s_setprio(0);
            barrier();
            if (ph + 1 < kPhases) {
#pragma unroll
                for (int j = 0; j < SPP; ++j) a[j] = an[j];
            }
        }
    };

    // Prologue: stages 0 and 1 in flight, stage 0 retired, then group 1 falls one barrier behind.
#pragma unroll
    for (int p = 0; p < kPieces; ++p) piece(st0, 0, p);
    if (nk > 1) {
#pragma unroll
        for (int p = 0; p < kPieces; ++p) piece(st1, 1, p);
        wait_prev();
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    if (grp == 1) barrier();
    for (unsigned kt = 0; kt < nk; kt += 3) {
        step(st0, st2, kt);
        if (kt + 1 < nk) step(st1, st0, kt + 1);
        if (kt + 2 < nk) step(st2, st1, kt + 2);
    }
    if (grp == 0) barrier();
    if constexpr ((LAB & 16) != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    const int nb0 = n0 + wave * 32 + 4 * hsel;
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
    const bool full = (m0 + 256 <= M) && (n0 + 256 <= N) && (N % 4) == 0;
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

// 16x16x32-MFMA form (sched 3): same tile, waves, groups, LDS stages and DMA pieces; weights in the
// w16 layout of wq_gemm16_kernel (linear_wq.hip), whose fragment maps it uses: wave w owns columns
// n0 + 32 w .. +32 as two 16-column fragments f and all 256 rows as 16 m-reps of 16; a 64-deep
// k-step is two 32-deep phases of 32 MFMAs (2 f x 16 reps, 512 cycles), each B fragment (16 rows x
// 32 k of X) feeding two MFMAs.  Accumulator acc[f][r] reg i: token m0 + 16 r + (lane & 15),
// column n0 + 32 w + 16 f + 4 (lane >> 4) + i.  Bit-identical to wq_gemm16_kernel (same MFMA, same
// k order).  On random data this shape holds a higher clock under DVFS than the 32x32x16 one at
// equal cycles (MI355X_MICROARCH.md, DVFS item 7; measured 2.09 vs 1.80 GHz in the ring kernels).
// DMA placement: LAB & 4 = 0: all six pieces in mem phase 1 (mem phase 0 is ruled out by the WAR
// rule above); LAB & 4: X rounds 0-2 between the MFMAs of phase 0, the rest between those of
// phase 1 (an mfma phase of either group starts after the barrier that retires stage kt-1's
// last reads).
typedef float float4_t16 __attribute__((ext_vector_type(4)));
template <int BITS, typename YT, int EPI, int LAB = 0>
__global__ void __launch_bounds__(512, 1)
wq_gemm_pp16_kernel(const __half *__restrict__ X, int M, int K, const uint32_t *__restrict__ w16,
                    const uint32_t *__restrict__ sz, const float *__restrict__ bias, YT *__restrict__ Y, int N,
                    int Npad, int group, int nbm, int nbn, PSampleEpi epi) {
    using SL = StageLayout8<BITS, 8, 8, 1>;
    constexpr int kRep = 16, kXR = 4, kPieces = kXR + 2;
    constexpr bool kDmaInMfma = (LAB & 4) != 0;
    __shared__ __attribute__((aligned(16))) uint8_t st0[SL::kBytes];
    __shared__ __attribute__((aligned(16))) uint8_t st1[SL::kBytes];
    __shared__ __attribute__((aligned(16))) uint8_t st2[SL::kBytes];

    const int nb = nbm * nbn, orig = blockIdx.x;
    const int xcd = orig % kXCDs, q8 = nb / kXCDs, r8 = nb % kXCDs;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / kXCDs;
    const int bm = wgid / nbn, bn = wgid % nbn;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2;
    const int m0 = bm * 256, n0 = bn * 256;
    const unsigned nk = static_cast<unsigned>(K) / kBK;
    const unsigned kpg = static_cast<unsigned>(group) / kBK;
    const unsigned nt = static_cast<unsigned>(n0 + wave * 32) >> 5;

    const int chunk_st = lane & 7;
    const __half *xsrc[kXR];
#pragma unroll
    for (int i = 0; i < kXR; ++i) {
        const int row = (i * 8 + wave) * 8 + (lane >> 3);
        int grow = m0 + row;
        grow = grow < M ? grow : M - 1;
        const int c = chunk_st ^ ((row >> 1) & 7);
        xsrc[i] = X + static_cast<size_t>(grow) * K + c * 8;
    }
    const uint32_t *wsrc = w16 + (static_cast<size_t>(nt) * nk * 64 + lane) * BITS;
    const uint32_t *szsrc = sz + n0 + 4 * lane;
    const bool has_sz = wave == 0;
    const uint32_t wv = static_cast<uint32_t>(wave);

    auto piece = [&](uint8_t *sb, unsigned kt, int p) {
        const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(sb));
        if (p < kXR) {
            glds16_asm(xsrc[p] + kt * kBK, base + wv * 1024 + p * 8192);
        } else if (p == kXR) {
            const uint32_t *wp = wsrc + static_cast<size_t>(kt) * 64 * BITS;
            const uint32_t wb = base + SL::kX + wv * (64 * BITS * 4);
            if constexpr (BITS == 4) {
                glds16_asm(wp, wb);
            } else if constexpr (BITS == 8) {
                glds16_asm(wp, wb);
                glds16_asm(wp + 4, wb + 64 * 16);
            } else {
                glds4_asm(wp, wb);
                glds4_asm(wp + 1, wb + 256);
            }
        } else if (has_sz) {
            glds16_asm(szsrc + (kt / kpg) * Npad, base + SL::kX + SL::kW);
        }
    };
    // Counted wait at the end of mem phase 1: everything of stage kt+1 retired, this step's
    // stage-(kt+2) pieces issued so far (all six, or X rounds 0-2 under kDmaInMfma) in flight.
    auto wait_prev = [&]() {
        if constexpr (kDmaInMfma) {
            asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        } else {
            if (has_sz) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kXR + SL::kWOps + 1) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kXR + SL::kWOps) : "memory");
        }
    };
    auto barrier = []() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    float4_t16 acc[2][kRep];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int r = 0; r < kRep; ++r) acc[f][r] = float4_t16{0.f, 0.f, 0.f, 0.f};

    const int rl = lane & 15;
    int soff[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) soff[s2] = rl * (kBK * 2) + (((4 * s2 + (lane >> 4)) ^ ((rl >> 1) & 7)) << 4);

    auto dequant = [&](half8_t &a, const uint32_t (&w)[BITS], int s, half2_t nz, half2_t sc) {
        if constexpr (LAB & 2) {
            uint32_t raw[4] = {w[0] ^ (uint32_t)s, w[1 % BITS], w[2 % BITS], w[3 % BITS]};
            a = __builtin_bit_cast(half8_t, raw);
        } else {
            a = dequant_frag<BITS>(w, s, nz, sc);
        }
    };

    auto step = [&](const uint8_t *sb, uint8_t *pf, unsigned kt) {
        const bool issue = !(LAB & 1) && kt + 2 < nk;
        uint32_t w[BITS];
        half2_t nz[2], sc[2];
        half8_t a[2];
#pragma unroll
        for (int ph = 0; ph < 2; ++ph) {
            // ---- mem phase: the 16 B fragments of 32-deep substep ph (+ words, scales, A at ph 0)
            if (ph == 0) {
                lds_words<BITS>(w, sb + SL::kX + wave * (64 * BITS * 4), lane);
#pragma unroll
                for (int f = 0; f < 2; ++f)
                    split_sz(*reinterpret_cast<const uint32_t *>(sb + SL::kX + SL::kW + (wave * 32 + 16 * f + rl) * 4),
                             nz[f], sc[f]);
            }
            half8_t b[kRep];
#pragma unroll
            for (int r = 0; r < kRep; ++r) b[r] = *reinterpret_cast<const half8_t *>(sb + soff[ph] + r * 16 * kBK * 2);
            if (ph == 0) {
#pragma unroll
                for (int f = 0; f < 2; ++f) dequant(a[f], w, 2 * f, nz[f], sc[f]);
            }
            if (!kDmaInMfma && issue && ph == 1) {
#pragma unroll
                for (int p = 0; p < kPieces; ++p) piece(pf, kt + 2, p);
            }
            if (ph == 1) {
                if (issue) wait_prev();
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            barrier();
            // ---- mfma phase
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_setprio(1);
            half8_t an[2];
#pragma unroll
            for (int r = 0; r < kRep; ++r)
#pragma unroll
                for (int f = 0; f < 2; ++f)
                    acc[f][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[f], b[r], acc[f][r], 0, 0, 0);
            if (ph == 0) {
#pragma unroll
                for (int f = 0; f < 2; ++f) dequant(an[f], w, 2 * f + 1, nz[f], sc[f]);
            }
            if (kDmaInMfma && issue) {
#pragma unroll
                for (int p = ph * 3; p < ph * 3 + 3; ++p) piece(pf, kt + 2, p);
            }
#pragma unroll
            for (int i = 0; i < 2 * kRep; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
            }
            if (ph == 0) {
#pragma unroll
                for (int f = 0; f < 2; ++f) asm volatile("" : "+v"(an[f]));
            }
            __builtin_amdgcn_s_setprio(0);
            barrier();
            if (ph == 0) {
                a[0] = an[0];
                a[1] = an[1];
            }
        }
    };

#pragma unroll
    for (int p = 0; p < kPieces; ++p) piece(st0, 0, p);
    if (nk > 1) {
#pragma unroll
        for (int p = 0; p < kPieces; ++p) piece(st1, 1, p);
        if (has_sz) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kXR + SL::kWOps + 1) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kXR + SL::kWOps) : "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    if (grp == 1) barrier();
    for (unsigned kt = 0; kt < nk; kt += 3) {
        step(st0, st2, kt);
        if (kt + 1 < nk) step(st1, st0, kt + 1);
        if (kt + 2 < nk) step(st2, st1, kt + 2);
    }
    if (grp == 0) barrier();

    const bool vec_ok = (N % 4) == 0;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
        const int nb0 = n0 + wave * 32 + 16 * f + 4 * (lane >> 4);
        const float4 bv = *reinterpret_cast<const float4 *>(bias + nb0);
        const bool full = (m0 + 256 <= M) && (nb0 + 4 <= N) && vec_ok;
#pragma unroll
        for (int r = 0; r < kRep; ++r) {
            const int m = m0 + 16 * r + rl;
            if constexpr (EPI == 1) {
                if (m < M && nb0 < N)
                    psample4(epi, m, nb0, N, acc[f][r][0] + bv.x, acc[f][r][1] + bv.y, acc[f][r][2] + bv.z,
                             acc[f][r][3] + bv.w);
            } else if (full) {
                store4<YT>(Y + static_cast<size_t>(m) * N + nb0, acc[f][r][0] + bv.x, acc[f][r][1] + bv.y,
                           acc[f][r][2] + bv.z, acc[f][r][3] + bv.w);
            } else if (m < M) {
                store_out4<YT>(Y + static_cast<size_t>(m) * N, bias, nb0, N, vec_ok, acc[f][r][0], acc[f][r][1],
                               acc[f][r][2], acc[f][r][3]);
            }
        }
    }
}

template <int BITS, typename YT, int EPI>
int launch_pp_t(const __half *X, int M, int K, const uint32_t *wdev, const uint32_t *sz, const float *bias, YT *Y,
                int N, int Npad, int group, int spp, const PSampleEpi &ep, hipStream_t st, int lab) {
    const int nbm = (M + 255) / 256, nbn = Npad / 256;
    const unsigned nb = static_cast<unsigned>(nbm * nbn);
    if constexpr (BITS == 4 && EPI == 0 && std::is_same<YT, __half>::value) {
        if (lab && spp == 3) {   // measurement only
            switch (lab) {
#define DLLM_PP16LAB(L)                                                                                      \
    case L:                                                                                                  \
        wq_gemm_pp16_kernel<4, __half, 0, L><<<nb, 512, 0, st>>>(X, M, K, wdev, sz, bias, Y, N, Npad, group, nbm, \
                                                                 nbn, ep);                                   \
        break;
                DLLM_PP16LAB(1) DLLM_PP16LAB(2) DLLM_PP16LAB(4) DLLM_PP16LAB(5) DLLM_PP16LAB(6)
#undef DLLM_PP16LAB
                default: break;
            }
            DLLM_LAUNCH_CHECK();
            return DLLM_OK;
        }
        if (lab) {   // measurement only
            switch (lab + 64 * (spp == 2)) {
#define DLLM_PPLAB(L)                                                                                           \
    case L:                                                                                                     \
        wq_gemm_pp_kernel<4, __half, 1, 0, L><<<nb, 512, 0, st>>>(X, M, K, wdev, sz, bias, Y, N, Npad, group, nbm, \
                                                                  nbn, ep);                                     \
        break;                                                                                                  \
    case 64 + L:                                                                                                \
        wq_gemm_pp_kernel<4, __half, 2, 0, L><<<nb, 512, 0, st>>>(X, M, K, wdev, sz, bias, Y, N, Npad, group, nbm, \
                                                                  nbn, ep);                                     \
        break;
                DLLM_PPLAB(1) DLLM_PPLAB(2) DLLM_PPLAB(16) DLLM_PPLAB(4)
#undef DLLM_PPLAB
                default: break;
            }
            DLLM_LAUNCH_CHECK();
            return DLLM_OK;
        }
    }
    if (spp == 3)
        wq_gemm_pp16_kernel<BITS, YT, EPI><<<nb, 512, 0, st>>>(X, M, K, wdev, sz, bias, Y, N, Npad, group, nbm, nbn, ep);
    else if (spp == 2)
        wq_gemm_pp_kernel<BITS, YT, 2, EPI><<<nb, 512, 0, st>>>(X, M, K, wdev, sz, bias, Y, N, Npad, group, nbm, nbn, ep);
    else
        wq_gemm_pp_kernel<BITS, YT, 1, EPI><<<nb, 512, 0, st>>>(X, M, K, wdev, sz, bias, Y, N, Npad, group, nbm, nbn, ep);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

template <int BITS>
int launch_pp_bits(int y_f32, const __half *X, int M, int K, const uint32_t *wdev, const uint32_t *sz,
                   const float *bias, void *Y, int N, int Npad, int group, int spp, const PSampleEpi *epi,
                   hipStream_t st, int lab) {
    if (epi)
        return launch_pp_t<BITS, float, 1>(X, M, K, wdev, sz, bias, epi->x_prev, N, Npad, group, spp, *epi, st, 0);
    if (y_f32)
        return launch_pp_t<BITS, float, 0>(X, M, K, wdev, sz, bias, static_cast<float *>(Y), N, Npad, group, spp,
                                           PSampleEpi{}, st, 0);
    return launch_pp_t<BITS, __half, 0>(X, M, K, wdev, sz, bias, static_cast<__half *>(Y), N, Npad, group, spp,
                                        PSampleEpi{}, st, lab);
}

}  // namespace

int launch_pp_gemm(int bits, int y_f32, const __half *X, int M, int K, const uint32_t *wdev, const uint32_t *sz,
                   const float *bias, void *Y, int N, int Npad, int group, int spp, const PSampleEpi *epi,
                   hipStream_t st, int lab) {
    if (Npad % 256 != 0 || M < 1 || K % kBK != 0) return fail(DLLM_ERR_SHAPE_MISMATCH, "ping-pong GEMM: tile shape");
    switch (bits) {
    case 2: return launch_pp_bits<2>(y_f32, X, M, K, wdev, sz, bias, Y, N, Npad, group, spp, epi, st, lab);
    case 4: return launch_pp_bits<4>(y_f32, X, M, K, wdev, sz, bias, Y, N, Npad, group, spp, epi, st, lab);
    case 8: return launch_pp_bits<8>(y_f32, X, M, K, wdev, sz, bias, Y, N, Npad, group, spp, epi, st, lab);
    default: return fail(DLLM_ERR_UNSUPPORTED, "bits");
    }
}

}  // namespace dllm
