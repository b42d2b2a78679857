// linear_common.hpp -- pieces shared by the group-quantized GEMM kernels (linear_wq.hip,
// linear_pp.hip): operand types, the fused p_sample epilogue, fragment dequant, output stores,
// the LDS stage layout of the 256-row ring kernels.  Weight layouts: see linear_wq.hip.
#pragma once
#include "common.hpp"
#include "diffusion_rng.hpp"

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float float16_t __attribute__((ext_vector_type(16)));

namespace dllm {

// Fused p_sample epilogue (dllm_linear_forward_psample): eps = acc + bias (f32) becomes
// x_prev = (c1 x_t + c2 eps) + std * n, n = stream element offset + m N + n (or 0).
struct PSampleEpi {
    const float *x_t;
    const float *coef;    // [M / rps][3]
    int rps;              // rows per sample
    int add;
    uint64_t seed, offset;
    float *x_prev;
    const float *noise;   // precomputed noise [M][N] (e.g. drawn on a side stream), or null: in-lane
    __half *x_prev_h = nullptr;   // optional f16 copy of x_prev (RNE): the next step's first-layer X
};

namespace {

constexpr int kBM = 256, kBN = 128, kBK = 64, kThreads = 256;

// Four consecutive outputs (element i = m N + n .. + 3) of the fused epilogue with x_t[i..i+3] and
// the row's coefficients already loaded: a caller that hoists every tile load above the tile's
// stores keeps them off the per-group path (x_prev may alias x_t / coef as far as the compiler can
// prove, so loads issued per group wait behind the previous group's stores).  N % 4 == 0,
// offset % 4 == 0.
__device__ __forceinline__ void psample4_x(const PSampleEpi &e, size_t i, float4 x, float c1, float c2, float sd,
                                           float e0, float e1, float e2, float e3) {
    float z[4] = {0.f, 0.f, 0.f, 0.f};
    if (e.add) {
        if (e.noise) {
            const float4 nv = *reinterpret_cast<const float4 *>(e.noise + i);
            z[0] = nv.x; z[1] = nv.y; z[2] = nv.z; z[3] = nv.w;
        } else {
            rng::normal4(e.seed, (e.offset + i) / 4, z);
        }
    }
    float4 o;
    o.x = (c1 * x.x + c2 * e0) + sd * z[0];
    o.y = (c1 * x.y + c2 * e1) + sd * z[1];
    o.z = (c1 * x.z + c2 * e2) + sd * z[2];
    o.w = (c1 * x.w + c2 * e3) + sd * z[3];
    *reinterpret_cast<float4 *>(e.x_prev + i) = o;
    if (e.x_prev_h) {
        union { __half h[4]; uint2 u; } pk;
        pk.h[0] = __float2half_rn(o.x); pk.h[1] = __float2half_rn(o.y);
        pk.h[2] = __float2half_rn(o.z); pk.h[3] = __float2half_rn(o.w);
        *reinterpret_cast<uint2 *>(e.x_prev_h + i) = pk.u;
    }
}

// Four consecutive outputs (m, n..n+3) of the fused epilogue; N % 4 == 0, offset % 4 == 0.
__device__ __forceinline__ void psample4(const PSampleEpi &e, int m, int n, int N, float e0, float e1, float e2,
                                         float e3) {
    const size_t i = static_cast<size_t>(m) * N + n;
    const float *c = e.coef + 3 * (m / e.rps);
    const float c1 = c[0], c2 = c[1], sd = c[2];
    float z[4] = {0.f, 0.f, 0.f, 0.f};
    if (e.add) {
        if (e.noise) {
            const float4 nv = *reinterpret_cast<const float4 *>(e.noise + i);
            z[0] = nv.x; z[1] = nv.y; z[2] = nv.z; z[3] = nv.w;
        } else {
            rng::normal4(e.seed, (e.offset + i) / 4, z);
        }
    }
    const float4 x = *reinterpret_cast<const float4 *>(e.x_t + i);
    float4 o;
    o.x = (c1 * x.x + c2 * e0) + sd * z[0];
    o.y = (c1 * x.y + c2 * e1) + sd * z[1];
    o.z = (c1 * x.z + c2 * e2) + sd * z[2];
    o.w = (c1 * x.w + c2 * e3) + sd * z[3];
    *reinterpret_cast<float4 *>(e.x_prev + i) = o;
    if (e.x_prev_h) {
        union { __half h[4]; uint2 u; } pk;
        pk.h[0] = __float2half_rn(o.x); pk.h[1] = __float2half_rn(o.y);
        pk.h[2] = __float2half_rn(o.z); pk.h[3] = __float2half_rn(o.w);
        *reinterpret_cast<uint2 *>(e.x_prev_h + i) = pk.u;
    }
}

// Dequantizes the A fragment (8 f16) of substep s from a lane's slab words.
template <int BITS>
__device__ __forceinline__ half8_t dequant_frag(const uint32_t (&w)[BITS], int s, half2_t nz, half2_t sc) {
    constexpr int PPW = 16 / BITS;
    constexpr uint32_t mask2 = ((1u << BITS) - 1u) * 0x00010001u;
    half8_t r;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const int P = s * 4 + v;
        const uint32_t word = w[P / PPW];
        const uint32_t t = ((word >> (BITS * (P % PPW))) & mask2) | 0x64006400u;
        half2_t h = __builtin_bit_cast(half2_t, t);
        h = h + nz;        // exact: q - zp
        h = h * sc;        // one f16 rounding of (q - zp) * scale
        r[2 * v] = h[0];
        r[2 * v + 1] = h[1];
    }
    return r;
}

__device__ __forceinline__ void split_sz(uint32_t szv, half2_t &nz, half2_t &sc) {
    half2_t p = __builtin_bit_cast(half2_t, szv);
    nz = half2_t{p[0], p[0]};
    sc = half2_t{p[1], p[1]};
}

__device__ __forceinline__ void glds16(const void *gsrc, void *ldst) {
    __builtin_amdgcn_global_load_lds((gbl_void_ptr)(const_cast<void *>(gsrc)), (lds_void_ptr)(ldst), 16, 0, 0);
}

template <typename YT>
__device__ __forceinline__ void store4(YT *p, float a, float b, float c, float d);
template <>
__device__ __forceinline__ void store4<float>(float *p, float a, float b, float c, float d) {
    *reinterpret_cast<float4 *>(p) = make_float4(a, b, c, d);
}
template <>
__device__ __forceinline__ void store4<__half>(__half *p, float a, float b, float c, float d) {
    union { __half h[4]; uint2 u; } pk;
    pk.h[0] = __float2half_rn(a); pk.h[1] = __float2half_rn(b);
    pk.h[2] = __float2half_rn(c); pk.h[3] = __float2half_rn(d);
    *reinterpret_cast<uint2 *>(p) = pk.u;
}
template <typename YT>
__device__ __forceinline__ void store1(YT *p, float a);
template <>
__device__ __forceinline__ void store1<float>(float *p, float a) { *p = a; }
template <>
__device__ __forceinline__ void store1<__half>(__half *p, float a) { *p = __float2half_rn(a); }

// Stores 4 consecutive outputs y[n..n+3] (+ bias), masking n >= N.
template <typename YT>
__device__ __forceinline__ void store_out4(YT *yrow, const float *__restrict__ bias, int n, int N, bool vec_ok,
                                           float a0, float a1, float a2, float a3) {
    if (n >= N) return;
    const float4 bv = *reinterpret_cast<const float4 *>(bias + n);
    const float y0 = a0 + bv.x, y1 = a1 + bv.y, y2 = a2 + bv.z, y3 = a3 + bv.w;
    if (vec_ok) {
        store4<YT>(yrow + n, y0, y1, y2, y3);
    } else {
        store1<YT>(yrow + n, y0);
        if (n + 1 < N) store1<YT>(yrow + n + 1, y1);
        if (n + 2 < N) store1<YT>(yrow + n + 2, y2);
        if (n + 3 < N) store1<YT>(yrow + n + 3, y3);
    }
}

constexpr int kMReps = kBM / 32;   // 8

// Exact weight codes as f16: a b-bit field at bit position o of a 16-bit half (o + b <= 10) ORed into
// the f16 2^(10-o) (ulp 2^-o) reads mag + q exactly, mag = 2^(10-o): one v_and_or_b32 per pair,
// no shift.  Fields at o >= 8 cross the exponent and are read from the word shifted right by 8.
// Then one exact v_pk_add_f16 of -(mag + zp) gives q - zp.
struct ExactConsts {
    uint32_t magic[5];   // f16 pairs 1024, 256, 64, 16, 4  (index = o / 2)
    half2_t nz[5];       // -(mag + zp) pairs
};

__device__ __forceinline__ ExactConsts exact_consts(half2_t nz1024) {
    ExactConsts c;
    const uint32_t mags[5] = {0x64006400u, 0x5C005C00u, 0x54005400u, 0x4C004C00u, 0x44004400u};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        uint32_t m = mags[i];
        asm("" : "+v"(m));   // a register operand (v_and_or_b32 takes no literal on gfx950); pure: hoisted
        c.magic[i] = m;
        const _Float16 d = static_cast<_Float16>(1024 - (1024 >> (2 * i)));   // 1024 - mag, exact
        c.nz[i] = nz1024 + half2_t{d, d};                                     // -(mag + zp), exact
    }
    return c;
}

// The A fragment (8 f16) of substep s as exact integers (q - zp).
template <int BITS>
__device__ __forceinline__ half8_t dequant_exact(const uint32_t (&w)[BITS], int s, const ExactConsts &c) {
    constexpr int PPW = 16 / BITS;
    constexpr uint32_t mask = ((1u << BITS) - 1u) * 0x00010001u;
    half8_t r;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const int P = s * 4 + v;
        const uint32_t word = w[P / PPW];
        const int pos = BITS * (P % PPW);
        const int o = pos + BITS <= 10 ? pos : pos - 8;
        const uint32_t src = pos + BITS <= 10 ? word : (word >> 8);
        const uint32_t t = (src & (mask << o)) | c.magic[o / 2];
        const half2_t h = __builtin_bit_cast(half2_t, t) + c.nz[o / 2];
        r[2 * v] = h[0];
        r[2 * v + 1] = h[1];
    }
    return r;
}


// Split-K combine: Y[m][n] = sum_s ws[s][m][n] (slice order) + bias[n]; 4 outputs per thread.
template <typename YT, int EPI = 0>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float *__restrict__ ws, int nsplit, int M, int N,
                                                            int Npad, const float *__restrict__ bias,
                                                            YT *__restrict__ Y, PSampleEpi epi = PSampleEpi{}) {
    const int q = Npad / 4;
    const size_t total = static_cast<size_t>(M) * q, slab = static_cast<size_t>(M) * Npad;
    const bool vec_ok = (N % 4) == 0;
    for (size_t i = blockIdx.x * static_cast<size_t>(256) + threadIdx.x; i < total;
         i += static_cast<size_t>(gridDim.x) * 256) {
        const int m = static_cast<int>(i / q), n = static_cast<int>(i % q) * 4;
        if (n >= N) continue;
        const float *p = ws + static_cast<size_t>(m) * Npad + n;
        float4 a = *reinterpret_cast<const float4 *>(p);
        for (int s = 1; s < nsplit; ++s) {
            const float4 b = *reinterpret_cast<const float4 *>(p + s * slab);
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
        if constexpr (EPI == 1) {
            const float4 bv = *reinterpret_cast<const float4 *>(bias + n);
            psample4(epi, m, n, N, a.x + bv.x, a.y + bv.y, a.z + bv.z, a.w + bv.w);
        } else {
            store_out4<YT>(Y + static_cast<size_t>(m) * N, bias, n, N, vec_ok, a.x, a.y, a.z, a.w);
        }
    }
}



template <int BITS>
__device__ __forceinline__ void lds_words(uint32_t (&w)[BITS], const uint8_t *wbase, int lane) {
    if constexpr (BITS == 4) {
        uint4 v = *reinterpret_cast<const uint4 *>(wbase + lane * 16);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else if constexpr (BITS == 8) {
        uint4 a = *reinterpret_cast<const uint4 *>(wbase + lane * 16);
        uint4 b = *reinterpret_cast<const uint4 *>(wbase + 64 * 16 + lane * 16);
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    } else {
        w[0] = *reinterpret_cast<const uint32_t *>(wbase + lane * 4);
        w[1] = *reinterpret_cast<const uint32_t *>(wbase + 256 + lane * 4);
    }
}


// Coalesced f16 store of a block's full output tile through LDS (the drained stage ring `img`,
// `cap` bytes): rows of 32 NW columns (64 NW bytes), `rows` = 32 MR tokens, written in passes of as
// many rows as fit.  acc[r] reg 4 qd + j -> token 32 r + (lane & 31), column 32 wave + 4 hsel +
// 8 qd + j (the 32x32x16 C/D map), each lane's 4 columns one 8-B piece; the 16-B chunk index of a
// row is XORed with the row (conflict-free 16-lane groups for the 8-B writes and the 16-B reads),
// and every wave then stores whole rows with 16-B lanes (64 NW / 16 lanes per row) instead of
// 64 rows x 8 B per instruction.  Ends with the block's waves past a barrier.
template <int NW, int MR>
__device__ __forceinline__ void store_tile_f16_lds(uint8_t *img, int cap, const float16_t (&acc)[MR],
                                                   const float4 (&bv)[4], __half *Y, int N, int m0, int n0,
                                                   int wave, int lane) {
    constexpr int kRowB = 64 * NW, kCpr = 4 * NW;                 // row bytes, 16-B chunks per row
    constexpr int kRows = 32 * MR;
    const int hsel = lane >> 5;
    const int per_pass = (cap / kRowB) >= kRows ? kRows : ((cap / kRowB) / 32) * 32;   // whole reps
    const int c0 = wave * 4;
    for (int p0 = 0; p0 < kRows; p0 += per_pass) {
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            if (r * 32 < p0 || r * 32 >= p0 + per_pass) continue;
            const int t = r * 32 - p0 + (lane & 31);
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
        __syncthreads();
        constexpr int kRowsPerInst = 1024 / kRowB;
        const int c = lane % kCpr;
        const int nrows = per_pass < kRows - p0 ? per_pass : kRows - p0;
        for (int t0 = wave * kRowsPerInst; t0 < nrows; t0 += NW * kRowsPerInst) {
            const int t = t0 + lane / kCpr;
            const uint4 v = *reinterpret_cast<const uint4 *>(img + t * kRowB + ((c ^ (t & (kCpr - 1))) * 16));
#if DLLM_NT_STORE   // non-temporal (streaming) Y stores: 1-2 % on the 4096^3 / 2048 x 4096^2 GEMMs (profiles/r03_nt_store)
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

// LDS-DMA issued from inline asm: invisible to hipcc's waitcnt pass, so the only waits on these
// loads are the counted vmcnt statements placed by hand (guide 5.7, M0 written in the statement).
template <int BITS, int NW = 8, int MR = kMReps, int KG = 1>
struct StageLayout8 {
    static constexpr int kWaves = NW * KG;
    static constexpr int kXRounds = 4 * MR / kWaves;      // 1-KiB wave-instructions per wave for X
    static constexpr int kX = 32 * MR * kBK * 2;
    static constexpr int kW = NW * 64 * BITS * 4;
    static constexpr int kSZ = NW * 64 * 4;
    static constexpr int kBytes = kX + kW + kSZ;
    static constexpr int kWOps = BITS == 4 ? 1 : 2;
    // LDS-DMA instructions per wave per stage.  KG = 1: X rounds + weight words + 1 scale dword.
    // KG = 2: k-group 0 loads the weight words, k-group 1 the scales.
    static constexpr int kOps0 = kXRounds + kWOps + (KG == 1 ? 1 : 0);
    static constexpr int kOps1 = kXRounds + 1;
};


}  // namespace

// Exact-weight GEMM (linear_exact.hip): Y = X . W^ + b with the MFMA A operand the exact integer
// (q - zp) and the f32 scale folded once per group; wdev = prefill layout, sz = per (group, column)
// f16 pair {-(1024+zp), *}, sf = f32 scales [G][Npad].  epi != null: fused p_sample into epi->x_prev.
struct ExactGemmArgs {
    int bits;
    const __half *X;
    int M, K;
    const uint32_t *wdev, *sz;
    const float *sf, *bias;
    void *Y;
    int N, Npad, group;
    const PSampleEpi *epi;
    int tm = 0;   // A/B: 256 x 256 tile-major tiles where they fill the chip
    int lab_policy = 0;   // lab A/B: 1 = the round-2 tile policy (no 32 x 128 mid-M tiles)
    const float *hr = nullptr;   // Horner ratios (DLLM_EXACT_HORNER builds: the 128 x 256 tiles in Horner form)
};
int launch_exact_gemm(const ExactGemmArgs &a, int y_f32, hipStream_t st);

// Exact-weight int4 g128 GEMM in Horner form on 256 x 256 tiles (linear_horner.hip): hr = the
// handle's ratios [G + 1][Npad], sf = its f32 scales (the last group's multiply the result).
// Needs K % 128 == 0 and Npad % 256 == 0.
struct HornerGemmArgs {
    const __half *X;
    int M, K;
    const uint32_t *wdev, *sz;
    const float *hr, *sf, *bias;
    void *Y;
    int N, Npad;
    const PSampleEpi *epi;
    int lab = 0;   // lab build only: 1 = the unstaggered schedule (A/B); 2 / 3 = staggered / not, no stores
    int bits = 4;  // launch_horner_gemm: int4 or int2 codes (the other Horner launchers: int4 only)
};
int launch_horner_gemm(const HornerGemmArgs &a, int y_f32, hipStream_t st);
// The same kernel on 128- or 64-token x 256-column tiles (rows = 128 / 64: grids where larger tiles
// leave CUs idle).
int launch_horner_rows_gemm(const HornerGemmArgs &a, int rows, int y_f32, hipStream_t st);
// The same Horner form on 256 x 128 tiles with two k-groups per tile (linear_horner.hip): needs
// K % 256 == 0 and Npad % 128 == 0.
int launch_horner_kg2_gemm(const HornerGemmArgs &a, int y_f32, hipStream_t st);
// The same Horner form on 128 x 256 tiles with producer / consumer waves (linear_pc.hip): 8 waves
// compute, 4 issue every LDS-DMA of the stage ring.  Needs K % 128 == 0 and Npad % 256 == 0.
int launch_horner_pc_gemm(const HornerGemmArgs &a, int y_f32, hipStream_t st);
// Its two-k-group form on rows x 128 tiles, rows = 128 / 64 / 32 (linear_pc.hip): needs K % 256 == 0
// and Npad % 128 == 0.
int launch_horner_pc_kg2_gemm(const HornerGemmArgs &a, int rows, int y_f32, hipStream_t st);
bool exact_gemm_supported(int M, int K, int Npad, int group);

// Ping-pong 256 x 256 GEMM (linear_pp.hip): Y = X . W^ + b for the 256-column-tile grid, bits in
// {2, 4, 8}, Y f16 (y_f32 = 0) or f32, epi != null: fused p_sample epilogue into epi->x_prev.
// sched: 1 / 2 = 32x32x16 MFMA, 1 or 2 16-deep substeps per phase (wdev = prefill layout);
// 3 = 16x16x32 MFMA (wdev = the w16 layout).  lab: ablation mask (measurement only, 0 in production).
int launch_pp_gemm(int bits, int y_f32, const __half *X, int M, int K, const uint32_t *wdev, const uint32_t *sz,
                   const float *bias, void *Y, int N, int Npad, int group, int sched, const PSampleEpi *epi,
                   hipStream_t st, int lab = 0);

}  // namespace dllm
