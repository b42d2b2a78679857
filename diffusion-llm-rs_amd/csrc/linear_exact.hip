// linear_exact.hip -- the group-quantized GEMM with EXACT dequantized weights (the default
// prefill path of dllm_linear_forward for M > kDecodeMaxM).
//
// The reference layer is Y = X . W^ + b with W^[k][n] = (q - zp) * s[g][n] computed in f32
// (diffuse-llm-rs/src/quantization.rs:81-85 per (column, 128-row group), lib.rs:806-813).  The
// rounded path (wq_gemm8_kernel) feeds the MFMA f16((q - zp) * f16(s)): two f16 roundings of
// every weight, ~2.7e-4 relative error per layer on top of X's own f16 rounding, and 1.17e-3
// after config C5's 12-layer chain.  Here the MFMA A operand is (q - zp) itself -- an integer
// below 2^11, so exact in f16 -- and the per-(group, column) scale is applied in f32 once per
// group:  acc[m][n] += s[g][n] * T_g[m][n],  T_g = sum_{k in g} X[m][k] (q - zp)[k][n]  (MFMA,
// f32 accumulation).  The only rounding left on the operands is X's (f16), ~2.1e-4 per layer.
//
// Tiles: block (32 MR tokens) x (32 NW columns), NW waves side by side in n; wave w owns columns
// n0 + 32 w .. +32 for all 32 MR tokens, accumulators acc[MR] (running sum) and tacc[MR] (the
// current group's T).  Yt = W^t Xt orientation as in linear_wq.hip: the accumulator lane is the
// token, 4 consecutive registers are 4 consecutive columns (16-B f32 / 8-B f16 stores), and a
// lane's 16 registers cover 16 columns whose scales it reads from LDS as 4 float4 per group.
// Global -> LDS is LDS-DMA only (X tile XOR-swizzled, weight slab words, the group's zero-point
// pair and f32 scale words) through a 3-stage ring with counted vmcnt waits and raw s_barrier,
// as wq_gemm8_kernel.  Weight layout: the prefill ("fragment-major") layout of linear_wq.hip.
#include "linear_common.hpp"
#include "stamp.hpp"

#ifndef DLLM_LAB
#define DLLM_LAB 0
#endif
// Policy switches (product defaults; A/B builds flip them, profiles/r02_gemm_ab/):
// DLLM_EXACT_WREG = 1: int4 weight words go global -> VGPR (buffer_load_dwordx4 from inline asm,
//   counted in the same vmcnt waits as the stage's LDS-DMA) instead of through the LDS ring: each
//   wave's slab words are its own (bit-identical; -0.5 %, and 16 KiB less LDS per stage).
// DLLM_EXACT_KG2 = 1: tile-starved grids (column shards) run 128 x 128 or 64 x 128 tiles with two
//   k-groups of 4 waves per block (4096 x 1024: 45.0 -> 40.5 us; 4096 x 512: 32.0 -> 24.4 us).
// DLLM_EXACT_MR2 = 1: grids still short of a round get 64 x 128 tiles (two blocks per CU).
// DLLM_EXACT_PRIO = 0 drops the s_setprio raise around the MFMA sections (measured 1 % slower).
// DLLM_EXACT_RING2 = 1: two groups per stage in a 2-stage ring (one barrier per two groups):
//   spills at 256 VGPRs, not adopted (a build without the per-stage barrier is only 8 % faster).
#ifndef DLLM_EXACT_WREG
#define DLLM_EXACT_WREG 1
#endif
#ifndef DLLM_EXACT_PRIO
#define DLLM_EXACT_PRIO 1
#endif
#ifndef DLLM_EXACT_MR2
#define DLLM_EXACT_MR2 1
#endif
#ifndef DLLM_EXACT_RING2
#define DLLM_EXACT_RING2 0
#endif
// DLLM_EXACT_S16 = 1: the fold kernels on 16x16x32 MFMAs (A/B builds only).  Bit-exact on the policy
// grid, but no faster on the box measured (M 2048 x 4096: 75.7 vs 77.4 us; the 4-GPU shard 4096 x 1024
// 42.7 vs 42.0; 4096 x 512 26.7 vs 24.6; profiles/r04_shard/exact_s16_ab.jsonl), so the product keeps
// the 32x32x16 form here (the Horner kernel's 16x16x32 form wins on 3 of 4 boxes).
#ifndef DLLM_EXACT_S16
#define DLLM_EXACT_S16 0
#endif
// DLLM_EXACT_STAG = 1: the 128 x 256 int4 g128 tiles run their two wave halves half a step apart
// (M 2048 / 3072 x 4096: 76.9 -> 73.9 / 121.6 -> 114.0 us, same bits).  The k-group tiles with
// their k-group halves staggered measured 2-7 % slower (4096 x 1024 / 512, 256 / 512 x 4096) and
// stay unstaggered, and the staggered tiles on 16x16x32 MFMAs measured within +-1.5 % (mixed
// sign) of these (profiles/r05_stag).
#ifndef DLLM_EXACT_STAG
#define DLLM_EXACT_STAG 1
#endif
#ifndef DLLM_EXACT_KG2
#define DLLM_EXACT_KG2 1
#endif
// Horner form on the 128 x 256 tiles (A/B): one accumulator rescaled by s_{g-1}/s_g at each group
// head instead of the transient group sum and its fold (see wq_gemm8_kernel<..., HORNER>).
#ifndef DLLM_EXACT_HORNER
#define DLLM_EXACT_HORNER 0
#endif

// DLLM_EXACT_KG_COAL = 1: on the k-group tiles (KG >= 2) the f16 epilogue is the coalesced LDS-staged
//   one, stored by all KG x NW waves (round 5, profiles/r05_shard/: 4096 x 1024 40.2 -> 38.1 us,
//   2048 x 2048 40.6 -> 38.6 us, rocprof means on one box); 0 = k-group 0's row-per-lane stores.
#ifndef DLLM_EXACT_KG_COAL
#define DLLM_EXACT_KG_COAL 1
#endif

#include <algorithm>
#include <type_traits>
#include <utility>

#ifndef DLLM_EXACT_MF16_ABL
#define DLLM_EXACT_MF16_ABL 0
#endif
#if DLLM_EXACT_MF16_ABL
// A/B build only (results wrong, timing only): each 32x32x16 MFMA replaced by two 16x16x32 MFMAs
// on the same operands -- the MFMA shape's effect on the held clock (as lab ablation 319 did for
// the Horner kernel).
__device__ __forceinline__ float16_t exact_mf16_abl(const half8_t &a, const half8_t &b, float16_t c) {
    typedef float fx4 __attribute__((ext_vector_type(4)));
    typedef float fx8 __attribute__((ext_vector_type(8)));
    fx4 c0 = __builtin_shufflevector(c, c, 0, 1, 2, 3), c1 = __builtin_shufflevector(c, c, 4, 5, 6, 7);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c1, 0, 0, 0);
    const fx8 lo = __builtin_shufflevector(c0, c1, 0, 1, 2, 3, 4, 5, 6, 7);
    const fx8 hi = __builtin_shufflevector(c, c, 8, 9, 10, 11, 12, 13, 14, 15);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
}
#define EXACT_MFMA(a, b, c) exact_mf16_abl((a), (b), (c))
constexpr int kExactMF = 2;
#else
#define EXACT_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_f16((a), (b), (c), 0, 0, 0)
constexpr int kExactMF = 1;
#endif
// DLLM_EXACT_ABL (stamp / timing builds only, results wrong): 1 = no LDS-DMA or weight loads after
// the prologue (the MFMA + VALU + LDS-read skeleton); 2 = no MFMAs (operands kept live: the load +
// VALU skeleton).  Prices the two halves of a k-step in cycles (profiles/r05_shard/).
#ifndef DLLM_EXACT_ABL
#define DLLM_EXACT_ABL 0
#endif
#if DLLM_EXACT_ABL == 2
__device__ __forceinline__ float16_t exact_abl_nomfma(const half8_t &a, const half8_t &b, float16_t c) {
    asm volatile("" ::"v"(a), "v"(b));
    asm volatile("" : "+v"(c));
    return c;
}
#undef EXACT_MFMA
#define EXACT_MFMA(a, b, c) exact_abl_nomfma((a), (b), (c))
#endif

namespace dllm {
namespace {

#if DLLM_STAMP
DLLM_STAMP_BUFFER(g_stamp_exact);   // phase stamps of wq_gemm_exact_kernel (stamp build only)
#endif

// A stage holds SPS consecutive 64-deep slabs (X tile, weight words) plus the group's zero-point
// pairs and f32 scales; SPS = 2 makes a stage one 128-row group (one fold and one barrier per group).
template <int BITS, int NW, int MR, int SPS, bool WREG = false, int GPS = 1>
struct ExactStage {
    static constexpr int kR1 = 4 * MR / NW;                // 1-KiB X pieces per wave per slab
    static constexpr int kXRounds = SPS * kR1;
    static constexpr int kX1 = 32 * MR * kBK * 2;           // one slab's X tile [32 MR][64] f16
    static constexpr int kX = SPS * kX1;
    static constexpr int kW1 = NW * 64 * BITS * 4;          // one slab's weight words
    static constexpr int kW = WREG ? 0 : SPS * kW1;   // WREG: the words live in VGPRs
    static constexpr int kSZ = 1024 * GPS;                  // u32 {-(1024+zp)} pairs, 32 NW columns (+ mirror) per group
    static constexpr int kSF = 1024 * GPS;                  // f32 scales, 32 NW columns (+ mirror) per group
    static constexpr int kBytes = kX + kW + kSZ + kSF;
    static constexpr int kWOps = SPS * (BITS == 4 ? 1 : 2);
    static_assert(kR1 >= 1 && 4 * MR % NW == 0, "X staging must split evenly over the waves");
};

// KPG: stages per group (group = 64 SPS KPG).  Slices of a split K are group-aligned.
// TM (tile-major, 256 x 256 tiles, MR = 8, SPS = 1): each stage runs the token reps one after the
// other -- 4 MFMAs of a rep into a transient accumulator (double-buffered by rep parity), then
// that rep's fold with the group's scales -- so only 2 transient accumulators are live (a 128 + 256
// register budget does not fit at two waves per SIMD).  Folding per 64-deep slab instead of per
// group is the same sum: both slabs of a group carry the same scale.
// GPS > 1 (KPG = 1): a stage holds GPS whole groups (group = 64 SPS / GPS), folded inside the stage.
// RING: LDS stages in the ring (3: stage kt + 2 issued while kt computes; 2: stage kt + 1, one
// barrier per stage -- with GPS = 2 one barrier per two groups).
// KG = 2: two k-groups of NW waves share the block's tile, k-group g taking the g-th half of the
// slice's stages (own LDS stage parts, same barriers); their sums are added in the epilogue,
// k-group 0's first: a tile-starved grid gets two waves per SIMD without a second launch.
typedef float fx4e_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4e_t __attribute__((ext_vector_type(4)));

// S16 accumulator element (t, cb, i) of a lane: token 16 t + (lane & 15), column 32 wave + 16 cb +
// 4 (lane >> 4) + i.  The f16 tile (acc + b) through the drained ring as 16-B row chunks: rows of
// 64 NW bytes, passes of as many whole 16-token blocks as fit.
template <int NW, int MR>
__device__ __forceinline__ void store_tile16x_f16_lds(uint8_t *img, int cap, const fx4e_t (&acc)[2 * MR][2],
                                                      const float4 (&bv)[2], __half *Y, int N, int m0, int n0,
                                                      int wave, int lane) {
    constexpr int kRowB = 64 * NW, kCpr = 4 * NW, kRows = 32 * MR;
    const int row16 = lane & 15, rq = lane >> 4;
    const int per_pass = (cap / kRowB) >= kRows ? kRows : ((cap / kRowB) / 16) * 16;
    for (int p0 = 0; p0 < kRows; p0 += per_pass) {
#pragma unroll
        for (int t = 0; t < 2 * MR; ++t) {
            if (t * 16 < p0 || t * 16 >= p0 + per_pass) continue;
            const int tr = t * 16 - p0 + row16;
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                const int pc = (4 * wave + 2 * cb + (rq >> 1)) ^ (tr & (kCpr - 1));
                union { __half h[4]; uint2 u; } pk;
                pk.h[0] = __float2half_rn(acc[t][cb][0] + bv[cb].x);
                pk.h[1] = __float2half_rn(acc[t][cb][1] + bv[cb].y);
                pk.h[2] = __float2half_rn(acc[t][cb][2] + bv[cb].z);
                pk.h[3] = __float2half_rn(acc[t][cb][3] + bv[cb].w);
                *reinterpret_cast<uint2 *>(img + tr * kRowB + pc * 16 + (rq & 1) * 8) = pk.u;
            }
        }
        __syncthreads();
        constexpr int kRowsPerInst = 1024 / kRowB;
        const int c = lane % kCpr;
        const int nrows = per_pass < kRows - p0 ? per_pass : kRows - p0;
        for (int t0 = wave * kRowsPerInst; t0 < nrows; t0 += NW * kRowsPerInst) {
            const int t = t0 + lane / kCpr;
            const uint4 v = *reinterpret_cast<const uint4 *>(img + t * kRowB + ((c ^ (t & (kCpr - 1))) * 16));
#if DLLM_NT_STORE
            typedef unsigned int u4nt __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(u4nt{v.x, v.y, v.z, v.w},
                                        reinterpret_cast<u4nt *>(Y + static_cast<size_t>(m0 + p0 + t) * N + n0 + 8 * c));
#else
            *reinterpret_cast<uint4 *>(Y + static_cast<size_t>(m0 + p0 + t) * N + n0 + 8 * c) = v;
#endif
        }
        __syncthreads();
    }
}

// Two-k-group f16 epilogue: k-group 0 (which holds the combined sums) writes the f16 tile (acc +
// bias) into `img` as 16-B row chunks XORed with the row, then every wave of the block stores whole
// rows with 16-B lanes -- the coalesced store of store_tile_f16_lds with KG x the storing waves.
template <int NW, int MR, int KG>
__device__ __forceinline__ void store_tile_f16_lds_kg(uint8_t *img, const float16_t (&acc)[MR], const float4 (&bv)[4],
                                                      __half *Y, int N, int m0, int n0, int wave, int kg, int lane) {
    constexpr int kRowB = 64 * NW, kCpr = 4 * NW, kRows = 32 * MR;
    if (kg == 0) {
        const int hsel = lane >> 5, c0 = wave * 4;
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            const int t = r * 32 + (lane & 31);
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                const int pc = (c0 + qd) ^ (t & (kCpr - 1));
                union { __half h[4]; uint2 u; } pk;
                pk.h[0] = __float2half_rn(acc[r][4 * qd + 0] + bv[qd].x);
                pk.h[1] = __float2half_rn(acc[r][4 * qd + 1] + bv[qd].y);
                pk.h[2] = __float2half_rn(acc[r][4 * qd + 2] + bv[qd].z);
                pk.h[3] = __float2half_rn(acc[r][4 * qd + 3] + bv[qd].w);
                *reinterpret_cast<uint2 *>(img + t * kRowB + pc * 16 + hsel * 8) = pk.u;
            }
        }
    }
    __syncthreads();
    constexpr int kRowsPerInst = 1024 / kRowB;
    const int c = lane % kCpr;
    for (int t0 = (kg * NW + wave) * kRowsPerInst; t0 < kRows; t0 += NW * KG * kRowsPerInst) {
        const int t = t0 + lane / kCpr;
        const uint4 v = *reinterpret_cast<const uint4 *>(img + t * kRowB + ((c ^ (t & (kCpr - 1))) * 16));
        typedef unsigned int u4nt __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u4nt{v.x, v.y, v.z, v.w},
                                    reinterpret_cast<u4nt *>(Y + static_cast<size_t>(m0 + t) * N + n0 + 8 * c));
    }
}

// S16: the MFMAs are 16x16x32 (not TM / HORN).  The chip holds a higher clock on that shape at the
// same FLOPs (MI355X_MICROARCH.md, DVFS give-back item 7); per wave the 32 columns x 32 MR tokens are
// 2 column blocks x 2 MR token blocks of 16 x 16 (acc16 / tacc16: the same registers as acc / tacc).
// A substep v (16 deep in the 32x32 form) becomes (32-deep half (v % 4) / 2, token blocks
// MR (v % 2) ..): the same MFMA work, so the group / fold / ring logic is unchanged; the A fragments
// of a half come from the same weight words through dequant_exact + v_permlane16_swap (as
// wq_horner16_kernel), the X tile uses the conflict-free (row >> 1) & 5 chunk swizzle.
template <int BITS, typename YT, int NW, int MR, int SPS, int KPG, bool SPLIT = false, int EPI = 0, bool TM = false,
          int TMB = 1, bool WREG = false, int GPS = 1, int RING = 3, int KG = 1, bool HORN = false, bool S16 = false,
          bool STAG = false>
__global__ void __launch_bounds__(NW * KG * 64, NW * KG >= 8 ? 1 : 2)
wq_gemm_exact_kernel(const __half *__restrict__ X, int M, int K, const uint32_t *__restrict__ wdev,
                     const uint32_t *__restrict__ sz, const float *__restrict__ sf, const float *__restrict__ bias,
                     YT *__restrict__ Y, int N, int Npad, int group, int nbm, int nbn, int nsplit = 1,
                     float *__restrict__ ws = nullptr, PSampleEpi epi = PSampleEpi{},
                     const float *__restrict__ sflast = nullptr) {
    // HORN: `sf` is the Horner ratio array hr (staged where the scales were), `sflast` the scales
    using SL = ExactStage<BITS, NW, MR, SPS, WREG, GPS>;
    static_assert(!HORN || (KPG == 1 && !TM && KG == 1 && !SPLIT && (GPS == 1 || RING == 2)), "Horner form: whole-group stages, whole K");
    static_assert(!WREG || (BITS == 4 && !TM), "register-staged weight words: int4, group-major stages");
    static_assert(GPS == 1 || (KPG == 1 && !TM && (4 * SPS) % GPS == 0 && 2 * GPS <= NW), "whole groups per stage");
    static_assert(RING == 3 || (RING >= 2 && RING <= 8 && !TM), "ring depth");
    static_assert(KG == 1 || (!TM && RING * KG * SL::kBytes >= (KG - 1) * NW * 64 * MR * 16 * 4), "k-group combine fits the ring");
    static_assert(!S16 || (!TM && !HORN), "16x16x32 form: fold kernels");
    static_assert(!STAG || (!TM && !HORN && GPS == 1 && (KG == 1 ? RING >= 4 && NW % 2 == 0 : KG % 2 == 0)),
                  "staggered halves");
    // Stage kt + kDist is issued at the head of step kt.  STAG: one half of the block's waves runs
    // half a step behind the other (one extra barrier at entry; the early half one at exit; a
    // barrier in the middle of every step), so the halves issue their DMA half a step apart instead
    // of together.  KG == 1: the halves are waves 0..NW/2-1 / NW/2.. of the one tile; the slot a
    // step writes was last read by the late half a half step earlier, so the ring keeps one stage
    // fewer in flight (RING - 2).  KG >= 2: the halves are k-groups 0..KG/2-1 / KG/2.., whose
    // stage parts are private, so the ring distance is unchanged.
    constexpr int kDist = (STAG && KG == 1) ? RING - 2 : RING - 1;
    constexpr int kBMt = 32 * MR, kBNt = 32 * NW;
    // RING stages of KG parts each (k-group g's part of stage i at ring + (i KG + g) kBytes)
    __shared__ __attribute__((aligned(16))) uint8_t ring[RING * KG * SL::kBytes];
    auto stp = [&](int i) __attribute__((always_inline)) { return ring + i * KG * SL::kBytes; };   // ring slot i

    // XCD-aware order: consecutive work items land on one XCD (blocks b, b+8 share an XCD under
    // round-robin dispatch); K-slice outermost so an XCD's blocks share the slice's X rows in L2.
    const int nb = nbm * nbn * nsplit, orig = blockIdx.x;
    const int xcd = orig % kXCDs, q8 = nb / kXCDs, r8 = nb % kXCDs;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / kXCDs;
    const int ks = wgid / (nbm * nbn), tile = wgid % (nbm * nbn);
    // Tiles in groups of 4 row-blocks, column-major inside a group: the 32 blocks an XCD runs at
    // once cover 4 row-blocks x 8 column-blocks, so a 64-deep slab costs that XCD's L2 4 X tiles +
    // 8 weight tiles of fetch (row-major order: 2 + 16, 25 % more).
    constexpr int kGM = 4;
    const int grp = tile / (kGM * nbn), first = grp * kGM, gm = min(kGM, nbm - first);
    const int in_grp = tile - grp * kGM * nbn;
    const int bm = first + in_grp % gm, bn = in_grp / gm;

    const int tid = threadIdx.x, lane = tid & 63;
    DLLM_STAMP_RT(g_stamp_exact, stamp::kRtEntry);
    DLLM_STAMP_AT(g_stamp_exact, 0);
    DLLM_STAMP_IDS(g_stamp_exact);
#if DLLM_STAMP
    struct StampEnd {
        __device__ ~StampEnd() {
            DLLM_STAMP_AT(g_stamp_exact, stamp::kEnd);
            DLLM_STAMP_RT(g_stamp_exact, stamp::kRtEnd);
        }
    } stamp_end;
#endif
    const int kg = KG == 1 ? 0 : __builtin_amdgcn_readfirstlane((tid >> 6) / NW);
    const int wave = __builtin_amdgcn_readfirstlane((tid >> 6) - kg * NW);   // wave within the k-group
    const int m0 = bm * kBMt, n0 = bn * kBNt;
    const unsigned nk_all = static_cast<unsigned>(K) / kBK;                 // 64-deep slabs
    const unsigned nk_slice = nk_all / SPS / static_cast<unsigned>(nsplit); // stages of this slice
    const unsigned nk = nk_slice / KG;                                      // stages of this k-group
    const unsigned kt0 = static_cast<unsigned>(ks) * nk_slice + static_cast<unsigned>(kg) * nk;
    const uint32_t kpart = static_cast<uint32_t>(kg) * SL::kBytes;          // this k-group's part of a stage
    const unsigned spg = static_cast<unsigned>(group) / kBK;                // slabs per group
    const unsigned nt = static_cast<unsigned>(n0 + wave * 32) >> 5;

    // DMA sources as buffer descriptors (wave-uniform bases) + fixed per-lane offsets; a stage only
    // moves the scalar offset.  X: the block's first row; rows past M are clamped to M - 1.
    const int chunk_st = lane & 7;
    uint32_t xoff[SL::kR1];
#pragma unroll
    for (int i = 0; i < SL::kR1; ++i) {
        const int row = (i * NW + wave) * 8 + (lane >> 3);
        const int rrow = (m0 + row < M ? m0 + row : M - 1) - m0;
        const int c = chunk_st ^ ((row >> 1) & (S16 ? 5 : 7));
        xoff[i] = static_cast<uint32_t>((rrow * K + c * 8) * 2);
    }
    const __amdgpu_buffer_rsrc_t xrs = raw_rsrc(X + static_cast<size_t>(m0) * K);
    const __amdgpu_buffer_rsrc_t wrs = raw_rsrc(wdev + static_cast<size_t>(nt) * nk_all * 64 * BITS);
    const uint32_t woff = static_cast<uint32_t>(lane * BITS * 4);
    const int ncol = lane & (8 * NW - 1);                    // 4 columns per lane (NW = 4: lanes 32.. mirror)
    // waves 2g / 2g + 1 stage group g's zero-point pairs / f32 scales: the same byte offsets in two arrays
    const int pg = wave >> 1;
    const bool has_sz = wave < 2 * GPS && (wave & 1) == 0, has_sf = wave < 2 * GPS && (wave & 1) == 1;
    const __amdgpu_buffer_rsrc_t prs = raw_rsrc(has_sz ? static_cast<const void *>(sz + n0) : static_cast<const void *>(sf + n0));
    const uint32_t poff = static_cast<uint32_t>(16 * ncol);
    const uint32_t wv = static_cast<uint32_t>(wave);

    // LDS destinations go through readfirstlane: the M0 operand must be an SGPR, and hipcc's
    // divergence analysis does not prove it uniform through the unrolled ring.
    auto u = [](uint32_t v) { return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v))); };
    // WREG: ring slot r's weight words (one 16-B load per lane per 64-deep slab).
    u32x4_t wq[RING][SPS];
    auto stage = [&](uint8_t *sb, unsigned kt, auto slot_tag) __attribute__((always_inline)) {
        constexpr int slot = decltype(slot_tag)::value;
        const uint32_t base = u(lds_addr(sb));
        const unsigned slab0 = (kt + kt0) * SPS;
#pragma unroll
        for (int s = 0; s < SPS; ++s)
#pragma unroll
            for (int i = 0; i < SL::kR1; ++i)
                blds16_asm(xrs, xoff[i], u((slab0 + s) * kBK * 2), u(base + s * SL::kX1 + wv * 1024 + i * NW * 1024));
#pragma unroll
        for (int s = 0; s < SPS; ++s) {
            const uint32_t so = u((slab0 + s) * 64 * BITS * 4);
            const uint32_t wb = u(base + SL::kX + s * SL::kW1 + wv * (64 * BITS * 4));
            if constexpr (WREG) {
                bload16_asm(wq[slot][s], wrs, woff, so);
            } else if constexpr (BITS == 4) {
                blds16_asm(wrs, woff, so, wb);
            } else if constexpr (BITS == 8) {
                blds16_asm(wrs, woff, so, wb);
                blds16_asm(wrs, woff + 16, so, u(wb + 64 * 16));
            } else {
                blds4_asm(wrs, lane * 8, so, wb);
                blds4_asm(wrs, lane * 8 + 4, so, u(wb + 256));
            }
        }
        const uint32_t goff = u((slab0 / spg + pg) * static_cast<uint32_t>(Npad) * 4);
        if (has_sz) blds16_asm(prs, poff, goff, u(base + SL::kX + SL::kW + pg * 1024));
        if (has_sf) blds16_asm(prs, poff, goff, u(base + SL::kX + SL::kW + SL::kSZ + pg * 1024));
    };
    // Counted wait leaving the newest stage's DMAs (this wave's own count) in flight.
    // (kDist > 2: the kDist - 1 newest stages stay in flight.)
    static_assert((kDist - 1) * (SL::kXRounds + SL::kWOps + 1) <= 63, "vmcnt range");
    auto wait_prev = [&]() __attribute__((always_inline)) {
        if constexpr (kDist == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (has_sz || has_sf) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kDist - 1) * (SL::kXRounds + SL::kWOps + 1)) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kDist - 1) * (SL::kXRounds + SL::kWOps)) : "memory");
    };
    const bool late = STAG && (KG == 1 ? wave >= NW / 2 : kg >= KG / 2);   // STAG: the half running behind
    // KG == 1: the late half's share of stage kt + 1 is read by the early half from the mid-step
    // barrier on, so the late half waits for it there; else every wave waits at its own step end.
    const bool wait_mid = STAG && KG == 1 && late;

    float16_t acc[S16 ? 1 : MR], tacc[TM ? TMB : (S16 ? 1 : MR)];
    fx4e_t acc16[S16 ? 2 * MR : 1][2], tacc16[S16 ? 2 * MR : 1][2];
#pragma unroll
    for (int r = 0; r < (S16 ? 1 : MR); ++r)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[r][e] = 0.0f;
#pragma unroll
    for (int t = 0; t < (S16 ? 2 * MR : 1); ++t)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) acc16[t][cb] = fx4e_t{0.f, 0.f, 0.f, 0.f};
    const float16_t zero16 = {};
    const fx4e_t zero4 = {0.f, 0.f, 0.f, 0.f};
    const int row16 = lane & 15, rq = lane >> 4;
    int soff16[2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
        soff16[h] = row16 * (kBK * 2) + (((4 * h + (((rq & 1) << 1) | (rq >> 1))) ^ ((row16 >> 1) & 5)) << 4);

    const int hsel = lane >> 5;
    const int rowx = ((lane & 31) >> 1) & 7;
    int soff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) soff[j] = (lane & 31) * (kBK * 2) + ((((2 * j + hsel) ^ rowx)) << 4);

    // B fragments of substep v (slab v / 4, 16-deep step v % 4) for the MR token reps; S16: of the
    // half (v % 4) / 2 for token blocks MR (v % 2) + r.
    auto read_b = [&](half8_t (&b)[MR], const uint8_t *sb, int v) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            if constexpr (S16)
                b[r] = *reinterpret_cast<const half8_t *>(sb + (v / 4) * SL::kX1 + soff16[(v % 4) / 2] +
                                                          (MR * (v % 2) + r) * 16 * kBK * 2);
            else
                b[r] = *reinterpret_cast<const half8_t *>(sb + (v / 4) * SL::kX1 + soff[v % 4] + r * 32 * kBK * 2);
        }
    };
    // S16: the two 16x16x32 A fragments (column blocks 0, 1) of a 32-deep half from the words of the
    // 32x32 layout (substeps 2h, 2h + 1)
    auto make_a16 = [&](const uint32_t (&wb)[BITS], int h, const ExactConsts &e, half8_t &c0, half8_t &c1)
        __attribute__((always_inline)) {
        u32x4e_t u0 = __builtin_bit_cast(u32x4e_t, dequant_exact<BITS>(wb, 2 * h, e));
        u32x4e_t u1 = __builtin_bit_cast(u32x4e_t, dequant_exact<BITS>(wb, 2 * h + 1, e));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const auto r = __builtin_amdgcn_permlane16_swap(u0[q], u1[q], false, false);
            u0[q] = r[0];
            u1[q] = r[1];
        }
        c0 = __builtin_bit_cast(half8_t, u0);
        c1 = __builtin_bit_cast(half8_t, u1);
    };

    // One stage (SPS slabs) on sb; stage pf receives stage kt + 2.  GF: first stage of a group (the
    // group's first MFMA starts from zero); GL: last (fold the group into acc with its scales).
    auto step = [&](const uint8_t *sb, uint8_t *pf, unsigned kt, auto gf_tag, auto gl_tag, auto cur_tag) __attribute__((always_inline)) {
        constexpr bool GF = decltype(gf_tag)::value, GL = decltype(gl_tag)::value;
        constexpr int cur = decltype(cur_tag)::value;
        constexpr int kSub = 4 * SPS, kSubG = kSub / GPS;
        uint32_t w[SPS][BITS];
        if constexpr (WREG) {
            // This slot's loads landed before the previous step's barrier (counted vmcnt); the empty
            // asm redefines the words after that wait, so no use of them can be scheduled above it.
#pragma unroll
            for (int s = 0; s < SPS; ++s) {
                asm volatile("" : "+v"(wq[cur][s]));
#pragma unroll
                for (int j = 0; j < BITS; ++j) w[s][j] = wq[cur][s][j];
            }
        }
        const bool issue = DLLM_EXACT_ABL != 1 && kt + kDist < nk;
        if (issue) stage(pf, kt + kDist, std::integral_constant<int, (cur + kDist) % RING>{});
        DLLM_STAMP_AT(g_stamp_exact, kt <= stamp::kMaxStep ? 2 + 4 * static_cast<int>(kt) : -1);
        if constexpr (!WREG) {
#pragma unroll
            for (int s = 0; s < SPS; ++s) lds_words<BITS>(w[s], sb + SL::kX + s * SL::kW1 + wave * (64 * BITS * 4), lane);
        }
        ExactConsts ec[GPS];
#pragma unroll
        for (int g = 0; g < GPS; ++g) {
            const half2_t p = __builtin_bit_cast(
                half2_t, *reinterpret_cast<const uint32_t *>(sb + SL::kX + SL::kW + g * 1024 + (wave * 32 + (lane & 31)) * 4));
            ec[g] = exact_consts(half2_t{p[0], p[0]});
        }
        half8_t bA[MR], bB[MR];
        read_b(bA, sb, 0);
        half8_t aA, aB;
        half8_t a16[2][2];   // S16: [half parity][column block]
        if constexpr (S16) make_a16(w[0], 0, ec[0], a16[0][0], a16[0][1]);
        else aA = dequant_exact<BITS>(w[0], 0, ec[0]);
        // Scales of a group (lane half hsel holds columns 4 hsel + 8 qd + (0..3) of the wave's 32): GPS = 1
        // reads them at the head of the stage so the fold never waits on LDS; GPS > 1 at the head of
        // each group's last substep.
        float4 s4[4];
        auto read_s4 = [&](int g) __attribute__((always_inline)) {
            if constexpr (S16) {   // column blocks 0, 1: columns 16 cb + 4 rq + (0..3)
                const float *sfl = reinterpret_cast<const float *>(sb + SL::kX + SL::kW + SL::kSZ + g * 1024) + wave * 32 + 4 * rq;
                s4[0] = *reinterpret_cast<const float4 *>(sfl);
                s4[1] = *reinterpret_cast<const float4 *>(sfl + 16);
            } else {
                const float *sfl = reinterpret_cast<const float *>(sb + SL::kX + SL::kW + SL::kSZ + g * 1024) + wave * 32 + 4 * hsel;
#pragma unroll
                for (int qd = 0; qd < 4; ++qd) s4[qd] = *reinterpret_cast<const float4 *>(sfl + 8 * qd);
            }
        };
        if constexpr (HORN ? GF : (GL && GPS == 1)) read_s4(0);
        // acc[r] += s (.) T_g[r]
        auto fold = [&](int r) __attribute__((always_inline)) {
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                acc[r][4 * qd + 0] = __builtin_fmaf(s4[qd].x, tacc[r][4 * qd + 0], acc[r][4 * qd + 0]);
                acc[r][4 * qd + 1] = __builtin_fmaf(s4[qd].y, tacc[r][4 * qd + 1], acc[r][4 * qd + 1]);
                acc[r][4 * qd + 2] = __builtin_fmaf(s4[qd].z, tacc[r][4 * qd + 2], acc[r][4 * qd + 2]);
                acc[r][4 * qd + 3] = __builtin_fmaf(s4[qd].w, tacc[r][4 * qd + 3], acc[r][4 * qd + 3]);
            }
        };
        // S16: fold token block t of both column blocks
        auto fold16 = [&](int t) __attribute__((always_inline)) {
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                acc16[t][cb][0] = __builtin_fmaf(s4[cb].x, tacc16[t][cb][0], acc16[t][cb][0]);
                acc16[t][cb][1] = __builtin_fmaf(s4[cb].y, tacc16[t][cb][1], acc16[t][cb][1]);
                acc16[t][cb][2] = __builtin_fmaf(s4[cb].z, tacc16[t][cb][2], acc16[t][cb][2]);
                acc16[t][cb][3] = __builtin_fmaf(s4[cb].w, tacc16[t][cb][3], acc16[t][cb][3]);
            }
        };
        // S16 substep v: 2 MR MFMAs (token blocks MR (v % 2) + r, both column blocks) of half (v % 4) / 2;
        // a group's first touch of a token block starts from zero (substeps 0 and 1 of the group), its
        // last (the group's last two substeps) folds it.  The next half's A fragments are built in the
        // substep before it.
        auto sub16 = [&](half8_t (&bc)[MR], half8_t (&bn)[MR], auto v_tag) __attribute__((always_inline)) {
            constexpr int v = decltype(v_tag)::value;
            constexpr int vg = GPS > 1 ? v % kSubG : v;   // substep within the group's stages
            constexpr bool first = GPS > 1 ? vg < 2 : (GF && v < 2);
            constexpr bool last = GPS > 1 ? vg >= kSubG - 2 : (GL && v >= kSub - 2);
            constexpr int hp = (v / 2) % 2, tb0 = MR * (v % 2);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (DLLM_EXACT_PRIO) __builtin_amdgcn_s_setprio(1);
            if constexpr (GPS > 1 && vg == kSubG - 2) read_s4(v / kSubG);
            if constexpr (v + 1 < kSub) read_b(bn, sb, v + 1);
            if constexpr (v % 2 == 1 && v + 1 < kSub)
                make_a16(w[(v + 1) / 4], ((v + 1) % 4) / 2, ec[(v + 1) / kSubG], a16[1 - hp][0], a16[1 - hp][1]);
#pragma unroll
            for (int r = 0; r < MR; ++r) {
                tacc16[tb0 + r][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a16[hp][0], bc[r], first ? zero4 : tacc16[tb0 + r][0], 0, 0, 0);
                tacc16[tb0 + r][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a16[hp][1], bc[r], first ? zero4 : tacc16[tb0 + r][1], 0, 0, 0);
            }
            if constexpr (last) {
#pragma unroll
                for (int r = 0; r < MR; ++r) fold16(tb0 + r);
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // MFMAs of blocks 0, 1
#pragma unroll
                for (int i = 2; i < MR; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);   // fold of block i - 2
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // MFMAs of block i
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
                }
            } else {
#pragma unroll
                for (int i = 0; i < MR; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // MFMAs
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
                    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);   // VALU
                }
            }
            if constexpr (DLLM_EXACT_PRIO) __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
        };
        auto sub = [&](half8_t (&bc)[MR], half8_t (&bn)[MR], const half8_t &ac, half8_t &an, auto v_tag) __attribute__((always_inline)) {
            constexpr int v = decltype(v_tag)::value;
            // first / last substep of a group (GPS > 1: inside the stage; else the stage's tags)
            constexpr bool gfirst = GPS > 1 ? v % kSubG == 0 : (GF && v == 0);
            constexpr bool glast = GPS > 1 ? v % kSubG == kSubG - 1 : (GL && v == kSub - 1);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (DLLM_EXACT_PRIO) __builtin_amdgcn_s_setprio(1);
            if constexpr (!HORN && GPS > 1 && glast) read_s4(v / kSubG);
            if constexpr (HORN && GPS > 1 && gfirst) read_s4(v / kSubG);   // this group's ratios
            if constexpr (!HORN && GPS > 1 && glast && v + 1 < kSub) {
                // A group's last substep with the next group's first in the same stage: prefetch the
                // next fragments and fold this group beside its last MFMAs.
                read_b(bn, sb, v + 1);
                an = dequant_exact<BITS>(w[(v + 1) / 4], (v + 1) % 4, ec[(v + 1) / kSubG]);
#pragma unroll
                for (int r = 0; r < MR; ++r)
                    tacc[r] = EXACT_MFMA(ac, bc[r], gfirst ? zero16 : tacc[r]);
#pragma unroll
                for (int r = 0; r < MR; ++r) fold(r);
#pragma unroll
                for (int i = 0; i < MR; ++i) {
                    if (i >= 2) __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);   // fold of rep i - 2
                    __builtin_amdgcn_sched_group_barrier(0x008, kExactMF, 0);               // MFMA rep i
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);               // DS read
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);               // dequant
                }
            } else if constexpr (HORN && v + 1 < kSub) {
                read_b(bn, sb, v + 1);
                an = dequant_exact<BITS>(w[(v + 1) / 4], (v + 1) % 4, ec[(v + 1) / kSubG]);
                if constexpr (gfirst) {
                    // acc <- acc * r_g before the group's first MFMA of each rep
#pragma unroll
                    for (int r = 0; r < MR; ++r) {
#pragma unroll
                        for (int qd = 0; qd < 4; ++qd) {
                            acc[r][4 * qd + 0] *= s4[qd].x;
                            acc[r][4 * qd + 1] *= s4[qd].y;
                            acc[r][4 * qd + 2] *= s4[qd].z;
                            acc[r][4 * qd + 3] *= s4[qd].w;
                        }
                        acc[r] = EXACT_MFMA(ac, bc[r], acc[r]);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
#pragma unroll
                    for (int i = 0; i < MR; ++i) {
                        if (i + 1 < MR) __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);   // rescale of rep i + 1
                        __builtin_amdgcn_sched_group_barrier(0x008, kExactMF, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < MR; ++r)
                        acc[r] = EXACT_MFMA(ac, bc[r], acc[r]);
#pragma unroll
                    for (int i = 0; i < MR; ++i) {
                        __builtin_amdgcn_sched_group_barrier(0x008, kExactMF, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                    }
                }
            } else if constexpr (HORN) {
#pragma unroll
                for (int r = 0; r < MR; ++r)
                    acc[r] = EXACT_MFMA(ac, bc[r], acc[r]);
            } else if constexpr (v + 1 < kSub) {
                read_b(bn, sb, v + 1);
                an = dequant_exact<BITS>(w[(v + 1) / 4], (v + 1) % 4, ec[(v + 1) / kSubG]);
#pragma unroll
                for (int r = 0; r < MR; ++r)
                    tacc[r] = EXACT_MFMA(ac, bc[r], gfirst ? zero16 : tacc[r]);
#pragma unroll
                for (int i = 0; i < MR; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, kExactMF, 0);   // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // VALU
                }
            } else {
                // Last substep: rep r's fold follows rep r+1's MFMA, so the fold of a group runs
                // beside the group's own last MFMAs instead of after all of them.
#pragma unroll
                for (int r = 0; r < MR; ++r)
                    tacc[r] = EXACT_MFMA(ac, bc[r], gfirst ? zero16 : tacc[r]);
                if constexpr (glast) {
#pragma unroll
                    for (int r = 0; r < MR; ++r) fold(r);
                    __builtin_amdgcn_sched_group_barrier(0x008, 2 * kExactMF, 0);   // MFMA r = 0, 1
#pragma unroll
                    for (int i = 2; i < MR; ++i) {
                        __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);  // fold of rep i - 2
                        __builtin_amdgcn_sched_group_barrier(0x008, kExactMF, 0);   // MFMA rep i
                    }
                }
            }
            if constexpr (DLLM_EXACT_PRIO) __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
        };
        // STAG: the mid-step barrier (the other half's step boundary).  The late half's share of
        // stage kt + 1 must land before it: the early half starts reading kt + 1 right after.
        auto mid = [&]() __attribute__((always_inline)) {
            if constexpr (STAG) {
                if (wait_mid) {
                    if (issue) wait_prev();
                    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        if constexpr (S16) {
            [&]<int... Vs>(std::integer_sequence<int, Vs...>) __attribute__((always_inline)) {
                ((Vs % 2 == 0 ? sub16(bA, bB, std::integral_constant<int, Vs>{})
                              : sub16(bB, bA, std::integral_constant<int, Vs>{}),
                  Vs == kSub / 2 - 1 ? mid() : void()), ...);
            }(std::make_integer_sequence<int, kSub>{});
        } else {
            [&]<int... Vs>(std::integer_sequence<int, Vs...>) __attribute__((always_inline)) {
                ((Vs % 2 == 0 ? sub(bA, bB, aA, aB, std::integral_constant<int, Vs>{})
                              : sub(bB, bA, aB, aA, std::integral_constant<int, Vs>{}),
                  Vs == kSub / 2 - 1 ? mid() : void()), ...);
            }(std::make_integer_sequence<int, kSub>{});
        }
        // Stage kt+1 must have landed; (RING 3) kt+2's DMAs may stay in flight across the barrier.
        DLLM_STAMP_AT(g_stamp_exact, kt <= stamp::kMaxStep ? 3 + 4 * static_cast<int>(kt) : -1);
        if (!wait_mid) {
            if (issue) wait_prev();
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        DLLM_STAMP_AT(g_stamp_exact, kt <= stamp::kMaxStep ? 4 + 4 * static_cast<int>(kt) : -1);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        DLLM_STAMP_AT(g_stamp_exact, kt <= stamp::kMaxStep ? 5 + 4 * static_cast<int>(kt) : -1);
    };
    auto step_tm = [&](const uint8_t *sb, uint8_t *pf, unsigned kt) __attribute__((always_inline)) {
        const bool issue = kt + 2 < nk;
        if (issue) stage(pf, kt + 2, std::integral_constant<int, 0>{});
        uint32_t w[BITS];
        lds_words<BITS>(w, sb + SL::kX + wave * (64 * BITS * 4), lane);
        const half2_t p = __builtin_bit_cast(half2_t,
                                             *reinterpret_cast<const uint32_t *>(sb + SL::kX + SL::kW + (wave * 32 + (lane & 31)) * 4));
        const ExactConsts ec = exact_consts(half2_t{p[0], p[0]});
        const float *sfl = reinterpret_cast<const float *>(sb + SL::kX + SL::kW + SL::kSZ) + wave * 32 + 4 * hsel;
        float4 s4[4];
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) s4[qd] = *reinterpret_cast<const float4 *>(sfl + 8 * qd);
        half8_t a[4], bq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = dequant_exact<BITS>(w, j, ec);
#pragma unroll
        for (int j = 0; j < 4; ++j) bq[j] = *reinterpret_cast<const half8_t *>(sb + soff[j]);
        auto fold = [&](int r) __attribute__((always_inline)) {
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                acc[r][4 * qd + 0] = __builtin_fmaf(s4[qd].x, tacc[r % TMB][4 * qd + 0], acc[r][4 * qd + 0]);
                acc[r][4 * qd + 1] = __builtin_fmaf(s4[qd].y, tacc[r % TMB][4 * qd + 1], acc[r][4 * qd + 1]);
                acc[r][4 * qd + 2] = __builtin_fmaf(s4[qd].z, tacc[r % TMB][4 * qd + 2], acc[r][4 * qd + 2]);
                acc[r][4 * qd + 3] = __builtin_fmaf(s4[qd].w, tacc[r % TMB][4 * qd + 3], acc[r][4 * qd + 3]);
            }
        };
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
            // MFMA j of rep r reads bq[j]; the next rep's fragment j refills it right after.
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                tacc[r % TMB] = EXACT_MFMA(a[j], bq[j], j == 0 ? zero16 : tacc[r % TMB]);
                if (r + 1 < MR) bq[j] = *reinterpret_cast<const half8_t *>(sb + soff[j] + (r + 1) * 32 * kBK * 2);
            }
            if constexpr (TMB == 1) {
                fold(r);
                // Pin the order: the fold of rep r completes before rep r+1's MFMAs (their B
                // fragments pass through this statement), so only one transient accumulator lives.
                asm volatile("" : "+v"(acc[r]), "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]));
            } else if (r > 0) {
                fold(r - 1);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, kExactMF, 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
                __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // VALU (the previous rep's fold)
            }
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (TMB > 1) fold(MR - 1);
        if (issue) wait_prev();
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // The ring rotates with period 3 and the group phase with period KPG: unroll lcm(3, KPG)
    // stages so every stage's buffer and group phase are compile-time (a run-time phase
    // dispatch made hipcc spill ~80 VGPRs).
    auto at = [&](auto i_tag, unsigned kt) __attribute__((always_inline)) {
        constexpr int I = decltype(i_tag)::value;
        constexpr int cur = I % RING, nxt = (I + kDist) % RING;
        uint8_t *sb = stp(cur) + kpart;
        uint8_t *pf = stp(nxt) + kpart;
        if constexpr (TM) step_tm(sb, pf, kt);
        else step(sb, pf, kt, std::integral_constant<bool, I % KPG == 0>{},
                  std::integral_constant<bool, I % KPG == KPG - 1>{}, std::integral_constant<int, cur>{});
    };
    constexpr int kUnroll = RING == 2 ? (KPG == 1 ? 2 : 4)
                          : RING == 3 ? ((KPG == 1 || TM) ? 3 : (KPG == 2 ? 6 : 12))
                                      : (KPG == 1 ? RING : (RING % KPG == 0 ? RING : RING * KPG));

    stage(stp(0) + kpart, 0, std::integral_constant<int, 0>{});
    if constexpr (kDist >= 2) {
        // stages 1 .. kDist - 1 in flight before the loop (stage kt + kDist is issued in step kt)
        [&]<int... Is>(std::integer_sequence<int, Is...>) __attribute__((always_inline)) {
            ((Is + 1 < static_cast<int>(nk) ? (stage(stp(Is + 1) + kpart, Is + 1, std::integral_constant<int, Is + 1>{}), 0) : 0), ...);
        }(std::make_integer_sequence<int, kDist - 1>{});
        if (nk >= static_cast<unsigned>(kDist)) wait_prev();
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (late) __builtin_amdgcn_s_barrier();   // STAG: enter half a step behind
    DLLM_STAMP_AT(g_stamp_exact, 1);
    for (unsigned kt = 0; kt < nk; kt += kUnroll) {
        [&]<int... Is>(std::integer_sequence<int, Is...>) __attribute__((always_inline)) {
            ((kt + Is < nk ? (at(std::integral_constant<int, Is>{}, kt + Is), 0) : 0), ...);
        }(std::make_integer_sequence<int, kUnroll>{});
    }
    if (STAG && !late) __builtin_amdgcn_s_barrier();   // pairs with the late half's last barrier

    if constexpr (HORN) {
        // acc = sum_g T_g s_g / s_{G-1}: times the last group's scales
        const float *sl = sflast + static_cast<size_t>(K / group - 1) * Npad + n0 + wave * 32 + 4 * hsel;
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
            const float4 sv = *reinterpret_cast<const float4 *>(sl + 8 * qd);
#pragma unroll
            for (int r = 0; r < MR; ++r) {
                acc[r][4 * qd + 0] *= sv.x;
                acc[r][4 * qd + 1] *= sv.y;
                acc[r][4 * qd + 2] *= sv.z;
                acc[r][4 * qd + 3] *= sv.w;
            }
        }
    }
    if constexpr (KG >= 2 && S16) {
        constexpr int kXg = NW * MR * 4 * 64;   // float4s per k-group (4 MR per lane, as below)
        float4 *xch = reinterpret_cast<float4 *>(ring) + (wave * MR * 4) * 64 + lane;
        if (kg >= 1) {
#pragma unroll
            for (int t = 0; t < 2 * MR; ++t)
#pragma unroll
                for (int cb = 0; cb < 2; ++cb)
                    xch[(kg - 1) * kXg + (t * 2 + cb) * 64] =
                        make_float4(acc16[t][cb][0], acc16[t][cb][1], acc16[t][cb][2], acc16[t][cb][3]);
        }
        __syncthreads();
        if (kg >= 1) return;
#pragma unroll
        for (int g = 1; g < KG; ++g)
#pragma unroll
            for (int t = 0; t < 2 * MR; ++t)
#pragma unroll
                for (int cb = 0; cb < 2; ++cb) {
                    const float4 o = xch[(g - 1) * kXg + (t * 2 + cb) * 64];
                    acc16[t][cb][0] += o.x; acc16[t][cb][1] += o.y; acc16[t][cb][2] += o.z; acc16[t][cb][3] += o.w;
                }
    } else if constexpr (KG >= 2) {
        // k-groups 1 .. KG-1 hand their sums to k-group 0 through the (drained) ring, 16 B per lane
        // per store; k-group 0 adds them in k-group order.
        constexpr int kXg = NW * MR * 4 * 64;   // float4s per k-group
        float4 *xch = reinterpret_cast<float4 *>(ring) + (wave * MR * 4) * 64 + lane;
        if (kg >= 1) {
#pragma unroll
            for (int r = 0; r < MR; ++r)
#pragma unroll
                for (int qd = 0; qd < 4; ++qd)
                    xch[(kg - 1) * kXg + (r * 4 + qd) * 64] =
                        make_float4(acc[r][4 * qd], acc[r][4 * qd + 1], acc[r][4 * qd + 2], acc[r][4 * qd + 3]);
        }
        __syncthreads();
        // coalesced f16 epilogue by all KG NW waves (the image sits past the hand-off area)
        constexpr bool kCoal = DLLM_EXACT_KG_COAL && std::is_same<YT, __half>::value && !SPLIT && EPI == 0 &&
                               NW * 64 >= 256 && sizeof(ring) >= (KG - 1) * kXg * 16 + 32 * MR * 64 * NW;
        const bool coal = kCoal && (m0 + kBMt <= M) && (n0 + kBNt <= N) && (N % 8) == 0;
        if (kg >= 1 && !coal) return;
        if (kg == 0) {
#pragma unroll
            for (int g = 1; g < KG; ++g)
#pragma unroll
                for (int r = 0; r < MR; ++r)
#pragma unroll
                    for (int qd = 0; qd < 4; ++qd) {
                        const float4 o = xch[(g - 1) * kXg + (r * 4 + qd) * 64];
                        acc[r][4 * qd] += o.x; acc[r][4 * qd + 1] += o.y; acc[r][4 * qd + 2] += o.z; acc[r][4 * qd + 3] += o.w;
                    }
        }
        if constexpr (kCoal) {
            if (coal) {
                const int nb0 = n0 + wave * 32 + 4 * hsel;
                float4 bv[4];
#pragma unroll
                for (int qd = 0; qd < 4; ++qd) bv[qd] = *reinterpret_cast<const float4 *>(bias + nb0 + 8 * qd);
                DLLM_STAMP_AT(g_stamp_exact, stamp::kEpi);
                store_tile_f16_lds_kg<NW, MR, KG>(ring + (KG - 1) * kXg * 16, acc, bv, reinterpret_cast<__half *>(Y), N, m0,
                                                  n0, wave, kg, lane);
                return;
            }
        }
    }
    DLLM_STAMP_AT(g_stamp_exact, stamp::kEpi);
    if constexpr (S16) {
        // element (t, cb, i): m = m0 + 16 t + (lane & 15), n = n0 + 32 wave + 16 cb + 4 rq + i
        const int nc0 = n0 + wave * 32 + 4 * rq;
        if constexpr (SPLIT) {
            float *slab = ws + static_cast<size_t>(ks) * M * Npad;
#pragma unroll
            for (int t = 0; t < 2 * MR; ++t) {
                const int m = m0 + 16 * t + row16;
                if (m >= M) continue;
                float *prow = slab + static_cast<size_t>(m) * Npad + nc0;
#pragma unroll
                for (int cb = 0; cb < 2; ++cb)
                    *reinterpret_cast<float4 *>(prow + 16 * cb) =
                        make_float4(acc16[t][cb][0], acc16[t][cb][1], acc16[t][cb][2], acc16[t][cb][3]);
            }
            return;
        }
        float4 bv16[2];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) bv16[cb] = *reinterpret_cast<const float4 *>(bias + nc0 + 16 * cb);
        if constexpr (EPI == 1) {
#pragma unroll
            for (int t = 0; t < 2 * MR; ++t) {
                const int m = m0 + 16 * t + row16;
                if (m >= M) continue;
#pragma unroll
                for (int cb = 0; cb < 2; ++cb) {
                    if (nc0 + 16 * cb >= N) continue;
                    psample4(epi, m, nc0 + 16 * cb, N, acc16[t][cb][0] + bv16[cb].x, acc16[t][cb][1] + bv16[cb].y,
                             acc16[t][cb][2] + bv16[cb].z, acc16[t][cb][3] + bv16[cb].w);
                }
            }
            return;
        }
        const bool full16 = (m0 + kBMt <= M) && (n0 + kBNt <= N) && (N % 4) == 0;
        if constexpr (std::is_same<YT, __half>::value && KG == 1 && NW * 64 >= 256) {
            if (full16 && (N % 8) == 0) {
                store_tile16x_f16_lds<NW, MR>(ring, static_cast<int>(sizeof(ring)), acc16, bv16, Y, N, m0, n0, wave, lane);
                return;
            }
        }
        const bool vec_ok = (N % 4) == 0;
#pragma unroll
        for (int t = 0; t < 2 * MR; ++t) {
            const int m = m0 + 16 * t + row16;
            if (m >= M) continue;
            YT *yrow = Y + static_cast<size_t>(m) * N;
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                if (full16)
                    store4<YT>(yrow + nc0 + 16 * cb, acc16[t][cb][0] + bv16[cb].x, acc16[t][cb][1] + bv16[cb].y,
                               acc16[t][cb][2] + bv16[cb].z, acc16[t][cb][3] + bv16[cb].w);
                else
                    store_out4<YT>(yrow, bias, nc0 + 16 * cb, N, vec_ok, acc16[t][cb][0], acc16[t][cb][1],
                                   acc16[t][cb][2], acc16[t][cb][3]);
            }
        }
        return;
    } else {
        // Epilogue: acc[r] reg e -> n = n0 + 32 wave + 4 hsel + 8 (e >> 2) + (e & 3), m = m0 + 32 r + (lane & 31).
        const int nb0 = n0 + wave * 32 + 4 * hsel;
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
            // every x_t value and row coefficient of the tile is loaded before the first store (see
            // psample4_x): one memory round trip for the tile instead of two per 4-column group
            float4 xt[MR][4];
            float cf[MR][3];
    #pragma unroll
            for (int r = 0; r < MR; ++r) {
                const int m = m0 + r * 32 + (lane & 31);
                const bool mok = m < M;
                const float *c = epi.coef + 3 * ((mok ? m : 0) / epi.rps);
                cf[r][0] = c[0]; cf[r][1] = c[1]; cf[r][2] = c[2];
    #pragma unroll
                for (int qd = 0; qd < 4; ++qd)
                    xt[r][qd] = mok && nb0 + 8 * qd < N
                                    ? *reinterpret_cast<const float4 *>(epi.x_t + static_cast<size_t>(m) * N + nb0 + 8 * qd)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
            }
    #pragma unroll
            for (int r = 0; r < MR; ++r) {
                const int m = m0 + r * 32 + (lane & 31);
                if (m >= M) continue;
    #pragma unroll
                for (int qd = 0; qd < 4; ++qd) {
                    if (nb0 + 8 * qd >= N) continue;
                    psample4_x(epi, static_cast<size_t>(m) * N + nb0 + 8 * qd, xt[r][qd], cf[r][0], cf[r][1], cf[r][2],
                               acc[r][4 * qd + 0] + bv[qd].x, acc[r][4 * qd + 1] + bv[qd].y,
                               acc[r][4 * qd + 2] + bv[qd].z, acc[r][4 * qd + 3] + bv[qd].w);
                }
            }
            return;
        }
        const bool full = (m0 + kBMt <= M) && (n0 + kBNt <= N) && (N % 4) == 0;
        if constexpr (std::is_same<YT, __half>::value && KG == 1 && NW * 64 >= 256) {
            if (full && (N % 8) == 0) {   // coalesced 16-B row stores (16-B aligned rows) through the drained ring
                store_tile_f16_lds<NW, MR>(ring, static_cast<int>(sizeof(ring)), acc, bv, Y, N, m0, n0, wave, lane);
                return;
            }
        }
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
}

template <int BITS, typename YT, int NW, int MR, int SPS, int KPG, int EPI, bool TM = false, int GPS = 1, int RING = 3,
          int KG = 1, bool WREG = (DLLM_EXACT_WREG != 0 && BITS == 4 && !TM), bool HORN = false,
          bool S16 = (DLLM_EXACT_S16 != 0 && !TM && !HORN), bool STAG = false>
int launch_exact_tile(const ExactGemmArgs &a, int nsplit, hipStream_t st) {
    if constexpr (HORN) {
        const int nbm = (a.M + 32 * MR - 1) / (32 * MR), nbn = a.Npad / (32 * NW);
        const PSampleEpi ep = a.epi ? *a.epi : PSampleEpi{};
        wq_gemm_exact_kernel<BITS, YT, NW, MR, SPS, KPG, false, EPI, false, 1, WREG, GPS, RING, 1, true>
            <<<static_cast<unsigned>(nbm * nbn), NW * 64, 0, st>>>(a.X, a.M, a.K, a.wdev, a.sz, a.hr, a.bias,
                                                                    static_cast<YT *>(a.Y), a.N, a.Npad, a.group, nbm, nbn,
                                                                    1, nullptr, ep, a.sf);
        DLLM_LAUNCH_CHECK();
        return DLLM_OK;
    }
    const int nbm = (a.M + 32 * MR - 1) / (32 * MR), nbn = a.Npad / (32 * NW);
    const unsigned nb = static_cast<unsigned>(nbm * nbn * nsplit);
    const PSampleEpi ep = a.epi ? *a.epi : PSampleEpi{};
    YT *Y = static_cast<YT *>(a.Y);
    if (nsplit == 1) {
        wq_gemm_exact_kernel<BITS, YT, NW, MR, SPS, KPG, false, EPI, TM, 1, WREG, GPS, RING, KG, false, S16, STAG><<<nb, NW * KG * 64, 0, st>>>(
            a.X, a.M, a.K, a.wdev, a.sz, a.sf, a.bias, Y, a.N, a.Npad, a.group, nbm, nbn, 1, nullptr, ep);
        DLLM_LAUNCH_CHECK();
        return DLLM_OK;
    }
    float *ws = device_workspace(st, static_cast<size_t>(nsplit) * a.M * a.Npad * sizeof(float));
    if (!ws) return DLLM_ERR_HIP;
    wq_gemm_exact_kernel<BITS, YT, NW, MR, SPS, KPG, true, 0, TM, 1, WREG, GPS, RING, KG, false, S16, STAG><<<nb, NW * KG * 64, 0, st>>>(
        a.X, a.M, a.K, a.wdev, a.sz, a.sf, a.bias, Y, a.N, a.Npad, a.group, nbm, nbn, nsplit, ws);
    DLLM_LAUNCH_CHECK();
    const size_t q = static_cast<size_t>(a.M) * (a.Npad / 4);
    const unsigned rb = static_cast<unsigned>(std::min<size_t>((q + 255) / 256, 4 * kCUs));
    splitk_reduce_kernel<YT, EPI><<<rb, 256, 0, st>>>(ws, nsplit, a.M, a.N, a.Npad, a.bias, Y, ep);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

// Tile policy (G64 = group / 64):
// 1. 128 x 256 tiles (8 waves, two per SIMD; stages of one 128-row group) when they give >= 256 blocks;
// 2. (int4, group 128, KG2) 128 x 128 tiles with two k-groups per block when those give 256..511
//    blocks, else 64 x 128 tiles with two k-groups when those give >= 256;
// 3. (MR2) 64 x 128 tiles (4 waves) while 128 x 128 tiles give < 512 blocks, K split until >= 512;
// 4. 128 x 128 tiles (4 waves, two blocks per CU, 64-deep stages) with K split over group-aligned
//    slices until the grid has >= ~200 blocks.
// Mid-M 32 x 128 tiles: LDS stages in the ring (10 KiB each; the weight words ride in VGPRs).
// Deeper rings keep more of a block's 512 KiB (X + weight words at K = 4096) in flight but measured
// no gain (M 256 / 384: RING 3 / 4 / 6 / 8 = 20.6 / 20.6 / 20.4 / 20.8 and 24.6 / 24.0 / 24.5 / 26.3
// us, profiles/r03_midm/ring_depth.jsonl): the single wave per SIMD is issue/latency bound, not
// fed short of bytes.
constexpr int kMidRing = 3;
// The mid-M tiles also where their grid is short of a round (DLLM_MIDM_MINFILL tiles and more): one
// 32 x 128 tile per CU takes the same time whether 96 or 256 CUs have one.  N 4096, 40-layer chain:
// M 65 / 96 / 128 / 160 / 192 / 224 = 16.5 / 18.2 / 20.4 / 23.1 / 24.6 / 23.5 -> 15.4 / 17.2 / 17.1 /
// 16.5 / 16.6 / 16.5 us against the K-split 64 x 128 tiles (profiles/r06_tiles/midm_short_grid_ab.jsonl);
// from 48 tiles (narrow N): N 2048 M 128 15.0 -> 13.2, N 1024 M 256 14.9 -> 13.2, N 512 M 384 / 512
// 13.7 / 15.0 -> 13.2 / 13.2 us, nothing slower (profiles/r06_tiles/m48/).
#ifndef DLLM_MIDM_MINFILL
#define DLLM_MIDM_MINFILL 48
#endif

template <int BITS, typename YT, int G64, int EPI>
int launch_exact_bits(const ExactGemmArgs &a, hipStream_t st) {
    const int mb = (a.M + 127) / 128;
#if DLLM_LAB
    if (a.tm && a.Npad % 256 == 0 && ((a.M + 255) / 256) * (a.Npad / 256) >= kCUs)
        return launch_exact_tile<BITS, YT, 8, 8, 1, G64, EPI, true>(a, 1, st);
#endif
    if (a.Npad % 256 == 0 && mb * (a.Npad / 256) >= kCUs) {
        // int8 weights: one-slab stages (two-slab stages exceed the 160 KiB LDS ring)
        if constexpr (G64 == 1 || BITS == 8) return launch_exact_tile<BITS, YT, 8, 4, 1, G64, EPI>(a, 1, st);
#if DLLM_EXACT_RING2
        // two whole 128-row groups per stage, 2-stage ring: one barrier per two groups
        else if constexpr (G64 == 2 && BITS == 4 && DLLM_EXACT_WREG) return launch_exact_tile<BITS, YT, 8, 4, 4, 1, EPI, false, 2, 2>(a, 1, st);
#endif
        else if constexpr (G64 == 2 && BITS == 4 && DLLM_EXACT_HORNER) {
#if DLLM_EXACT_HORNER == 2   // two groups per stage, 2-stage ring: one barrier per two groups
            if (a.hr) return launch_exact_tile<BITS, YT, 8, 4, 4, 1, EPI, false, 2, 2, 1, DLLM_EXACT_WREG != 0, true>(a, 1, st);
#else
            if (a.hr) return launch_exact_tile<BITS, YT, 8, 4, 2, 1, EPI, false, 1, 3, 1, DLLM_EXACT_WREG != 0, true>(a, 1, st);
#endif
            return launch_exact_tile<BITS, YT, 8, 4, 2, 1, EPI>(a, 1, st);
        }
#if DLLM_EXACT_STAG
        // the two wave halves half a step apart (4-slot ring, stage kt + 2 issued in step kt; 136 KiB)
        else if constexpr (G64 == 2 && BITS == 4 && DLLM_EXACT_WREG && !DLLM_EXACT_S16)
            return launch_exact_tile<BITS, YT, 8, 4, 2, 1, EPI, false, 1, 4, 1, true, false, false, true>(a, 1, st);
#endif
        else return launch_exact_tile<BITS, YT, 8, 4, 2, G64 / 2, EPI>(a, 1, st);
    }
    const int tiles = mb * (a.Npad / 128), ngroups = a.K / a.group;
    // Mid M (int4 g128): 32 x 128 tiles of 4 waves streaming the whole K -- no K split, hence no
    // f32 slabs and no combine launch -- where they give a full round but 64 x 128 tiles do not
    // (M 225..448 at N = 4096, where the policy below splits K): M 256 / 384: 25.1 -> 20.4 /
    // 30.0 -> 24.6 us; at M >= 512 the 64 x 128 two-k-group tiles stay faster (23.1 vs 25.8 us)
    // (profiles/r03_midm/policy_ab.json).
    if constexpr (G64 == 2 && BITS == 4 && DLLM_EXACT_WREG) {
        const int t32 = ((a.M + 31) / 32) * (a.Npad / 128), t64 = ((a.M + 63) / 64) * (a.Npad / 128);
        if (a.lab_policy != 1 && tiles < kCUs && t64 < kCUs && t32 >= DLLM_MIDM_MINFILL) {
#if DLLM_LAB
            switch (a.lab_policy) {   // lab A/B: one k-group (RING 3) / two k-groups / four (RING 3)
            case 2: return launch_exact_tile<BITS, YT, 4, 1, 2, 1, EPI, false, 1, kMidRing>(a, 1, st);
            case 3: if (ngroups % 2 == 0) return launch_exact_tile<BITS, YT, 4, 1, 2, 1, EPI, false, 1, 2, 2>(a, 1, st);
                    break;
            case 4: if (ngroups % 4 == 0) return launch_exact_tile<BITS, YT, 4, 1, 2, 1, EPI, false, 1, 3, 4>(a, 1, st);
                    break;
            default: break;
            }
#endif
            // k-groups of 4 waves sharing the tile (k-group g streams the g-th part of K; sums handed
            // to k-group 0 through the ring): four (16 waves, one block per CU) while the grid is
            // one block per CU, else two (8 waves, two blocks per CU fit).  M 256: 20.4 (one
            // k-group) -> 15.5 (two) -> 14.3 us (four); M 384: 24.5 -> 22.1 (two) / 25.1 (four)
            // (profiles/r03_midm/kgroups.jsonl).
            if (t32 <= kCUs && ngroups % 4 == 0)
                return launch_exact_tile<BITS, YT, 4, 1, 2, 1, EPI, false, 1, 2, 4>(a, 1, st);
            if (ngroups % 2 == 0) return launch_exact_tile<BITS, YT, 4, 1, 2, 1, EPI, false, 1, 2, 2>(a, 1, st);
            return launch_exact_tile<BITS, YT, 4, 1, 2, 1, EPI, false, 1, kMidRing>(a, 1, st);
        }
    }
#if DLLM_EXACT_KG2
    // tile-starved grids: 128 x 128 (or 64 x 128) tiles with two k-groups of 4 waves per block
    if constexpr (G64 == 2 && BITS == 4 && DLLM_EXACT_WREG) {
        // (lab A/B policy 5: 64 x 128 tiles, two blocks per CU, where 128 x 128 tiles give one round;
        // 6 / 7: the 128 x 128 tiles with 64-deep stages in a 4- / 3-stage ring instead of 128-deep
        // stages in a 2-stage ring)
#if DLLM_LAB
        if (tiles >= kCUs && tiles < 2 * kCUs && ngroups % 2 == 0 && a.lab_policy == 6)
            return launch_exact_tile<BITS, YT, 4, 4, 1, 2, EPI, false, 1, 4, 2>(a, 1, st);
        if (tiles >= kCUs && tiles < 2 * kCUs && ngroups % 2 == 0 && a.lab_policy == 7)
            return launch_exact_tile<BITS, YT, 4, 4, 1, 2, EPI, false, 1, 3, 2>(a, 1, st);
#endif
        if (tiles >= kCUs && tiles < 2 * kCUs && ngroups % 2 == 0 && a.lab_policy != 5)
            return launch_exact_tile<BITS, YT, 4, 4, 2, 1, EPI, false, 1, 2, 2>(a, 1, st);
        const int t64 = ((a.M + 63) / 64) * (a.Npad / 128);
        if ((tiles < kCUs || a.lab_policy == 5) && t64 >= kCUs && ngroups % 2 == 0)
            return launch_exact_tile<BITS, YT, 4, 2, 2, 1, EPI, false, 1, 2, 2>(a, 1, st);
    }
#endif
#if DLLM_EXACT_MR2
    if (tiles < 2 * kCUs) {
        const int t64 = ((a.M + 63) / 64) * (a.Npad / 128);
        int ns = 1;
        while (t64 * ns < 2 * kCUs && ns < 8 && ngroups % (2 * ns) == 0 && (a.K / kBK) / (2 * ns) >= 4) ns *= 2;
        return launch_exact_tile<BITS, YT, 4, 2, 1, G64, EPI>(a, ns, st);
    }
#endif
    int nsplit = 1;
    while (tiles * nsplit < 200 && nsplit < 8 && ngroups % (2 * nsplit) == 0 && (a.K / kBK) / (2 * nsplit) >= 4)
        nsplit *= 2;
    return launch_exact_tile<BITS, YT, 4, 4, 1, G64, EPI>(a, nsplit, st);
}

template <int KPG, int EPI>
int launch_exact_kpg(const ExactGemmArgs &a, int y_f32, hipStream_t st) {
    switch (a.bits) {
    case 2: return EPI || y_f32 ? launch_exact_bits<2, float, KPG, EPI>(a, st) : launch_exact_bits<2, __half, KPG, 0>(a, st);
    case 4: return EPI || y_f32 ? launch_exact_bits<4, float, KPG, EPI>(a, st) : launch_exact_bits<4, __half, KPG, 0>(a, st);
    case 8: return EPI || y_f32 ? launch_exact_bits<8, float, KPG, EPI>(a, st) : launch_exact_bits<8, __half, KPG, 0>(a, st);
    default: return fail(DLLM_ERR_UNSUPPORTED, "bits");
    }
}

}  // namespace

#if DLLM_STAMP
DLLM_STAMP_READER(dllm_stamp_read_exact, g_stamp_exact)
#endif

bool exact_gemm_supported(int M, int K, int Npad, int group) {
    return M >= 1 && Npad % 128 == 0 && K % group == 0 && (group == 64 || group == 128 || group == 256);
}

int launch_exact_gemm(const ExactGemmArgs &a, int y_f32, hipStream_t st) {
    if (!exact_gemm_supported(a.M, a.K, a.Npad, a.group))
        return fail(DLLM_ERR_SHAPE_MISMATCH, "exact GEMM: needs Npad % 128 == 0, group in {64, 128, 256}, K % group == 0");
    const bool fused = a.epi != nullptr;
    switch (a.group / kBK) {
    case 1: return fused ? launch_exact_kpg<1, 1>(a, 1, st) : launch_exact_kpg<1, 0>(a, y_f32, st);
    case 2: return fused ? launch_exact_kpg<2, 1>(a, 1, st) : launch_exact_kpg<2, 0>(a, y_f32, st);
    default: return fused ? launch_exact_kpg<4, 1>(a, 1, st) : launch_exact_kpg<4, 0>(a, y_f32, st);
    }
}

}  // namespace dllm
