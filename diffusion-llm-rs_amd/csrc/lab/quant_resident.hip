// quant_resident.hip -- quantize_tensor (diffuse-llm-rs/src/quantization.rs:38-68) of one or two
// tensors in ONE read of HBM: each CU keeps its slice of the data on chip (VGPRs + LDS) across one
// grid-wide hand-off of the min/max partials, instead of reading the tensor a second time for the
// map (the two-pass path of quant_kernels.hip streams 2 x 4 B per element; both passes already run
// at the fabric rate, ~5.8 TB/s, so only fewer bytes make it faster).
//
// Used for QuantizedKVCacheEntry::new / KVCacheEntry::update's copies (K and V in one launch when
// both fit, quantization.rs:140-157, lib.rs:241-276) and standalone quantize_tensor, whenever the
// tensors fit the chip's on-chip capacity (256 CUs x (23 VGPR slots + 9 LDS slots) x 16 KiB =
// 128 MiB) and the shape is whole octets on 16-B aligned bases.  Outputs are bit-identical to the
// two-pass kernels: the same NaN-ignoring extremes (order-independent), the same params_of and the
// same code_of / div_scale arithmetic.
//
// Layout: block b (one per CU, 1024 threads = 16 waves, 4 per SIMD; its LDS use keeps it alone on
// the CU) owns slots j = 0 .. J_t - 1 of tensor t, slot = 1024 float4 = 4096 values: float4 index
// f = (b J_t + j) 1024 + thread, so every load and every code store of a wave is one contiguous
// piece.  Slots 0 .. 22 of the block live in VGPRs (a static register array), slots 23 .. 31 in
// LDS (LDS-DMA straight from HBM).
//
// Grid hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, the sc1 form -- no whole-cache
// write-back or invalidate), a sense-reversing barrier on library-owned words (no per-launch reset
// launch): thread 0 of every block reads the generation, writes its {max, min} partials with
// agent-scope (sc1) stores, drains them and adds one to the arrival count; the last block to
// arrive resets the count and bumps the generation, the others poll the generation (sc1 loads,
// s_sleep between polls); then every block reads all partials with sc1 loads.  Every block then folds all partials itself (same order-free
// result everywhere), derives the params and quantizes its resident slice.  The grid is exactly
// the CU count and needs every block resident at once; the poll is bounded (about 0.2 s of
// s_memrealtime), after which the block gives up, raises the error word and writes NaN params,
// so a launch that could not become resident ends instead of hanging.
#include "common.hpp"

#include <cstdlib>
#include <type_traits>

#ifndef DLLM_LAB
#define DLLM_LAB 0
#endif

namespace dllm {
namespace {

constexpr int kRT = 1024;                // threads per block (16 waves: 4 per SIMD)
constexpr int kRReg = 23;                // float4 slots per thread in VGPRs (92 of the 128 registers)
constexpr int kRLds = 9;                 // float4 slots per thread in LDS (144 KiB)
constexpr uint64_t kPollTicks = 20000000;   // s_memrealtime runs at 100 MHz: 0.2 s
typedef float f4v __attribute__((ext_vector_type(4)));

struct RTensor {
    const float *x;
    size_t n4;             // float4 count (n / 4; n % 8 == 0)
    uint8_t *out[2];       // packed codes per width
    float *params[2];      // {scale, zp} per width
    int J;                 // slots per block
};
struct RArgs {
    RTensor t[2];
    int nt;                // tensors (1 or 2)
    int bits[2];           // widths (bits[1] == 0: one width)
    float2 *partials;      // [2][nb] {max, min}
    unsigned *sync;        // library-owned, zero at allocation: [0] arrivals (reset by the last block),
                           // [1] generation (bumped by the last block), [2] error word
    unsigned nb;           // blocks = CUs
    int lab;               // lab build only (DLLM_RES_LAB): 1 no hand-off, 2 no code stores, 4 no phase 2,
                           // 8 no phase-1 loads -- timing ablations, results wrong; 0 in the product
};

__device__ __forceinline__ void rs_params(float mx, float mn, int bits, float &scale, float &zp) {
    const float q_max = static_cast<float>(1u << bits) - 1.0f;   // quantization.rs:50
    float s = (mx - mn) / (q_max - 0.0f);                          // :52
    if (s == 0.0f) s = 1.0f;                                       // :53
    const float zpf = 0.0f - mn / s;                               // :55
    zp = static_cast<float>(rs_as_u8(roundf(rs_clamp(zpf, 0.0f, q_max))));   // :56, :67
    scale = s;
}

__device__ __forceinline__ bool markstein_ok_r(float s) { return s >= 0x1p-64f && s <= 0x1p64f; }

template <bool kFast>
__device__ __forceinline__ float div_r(float x, float s, float r) {
    if constexpr (!kFast) {
        return x / s;
    } else {   // Markstein: RN(x / s) in three FMA-pipe ops (quant_kernels.hip, div_scale)
        const float q0 = x * r;
        const float e = __builtin_fmaf(-q0, s, x);
        const float q1 = __builtin_fmaf(e, r, q0);
        return q1 != q1 ? q0 : q1;
    }
}

__device__ __forceinline__ uint32_t code_r(float t, uint32_t hi) {   // quant_kernels.hip, code_of
    const float tr = __builtin_truncf(t);
    const float c = fminf(fmaxf(tr, 0.0f), static_cast<float>(hi));
    const uint32_t u = static_cast<uint32_t>(c) + ((t - tr) >= 0.5f ? 1u : 0u);
    return u > hi ? hi : u;
}

// The 4 codes of float4 index f at width b into the packed stream (bytes f b / 2 ..); ok = f is
// inside the tensor (lanes 2i and 2i + 1 agree: n % 8 == 0).  Width 1 pairs the nibbles of two lanes,
// so every lane takes part in its shuffle.
__device__ __forceinline__ void store_quad_r(uint8_t *__restrict__ out, size_t f, uint32_t w, int b, int lane,
                                             bool ok) {
    if (b == 1) {
        const uint32_t other = static_cast<uint32_t>(__shfl_xor(static_cast<int>(w), 1, 64));
        if (ok && (lane & 1) == 0) out[f >> 1] = static_cast<uint8_t>(w | (other << 4));
        return;
    }
    if (!ok) return;
    if (b == 8) {
        *reinterpret_cast<uint32_t *>(out + f * 4) = w;
    } else if (b == 4) {
        *reinterpret_cast<uint16_t *>(out + f * 2) = static_cast<uint16_t>(w);
    } else {
        out[f] = static_cast<uint8_t>(w);
    }
}

template <int B>
struct WidthC {   // the constants of one width (compile-time width B)
    float s, z, r;
};

template <int B, bool kFast>
__device__ __forceinline__ uint32_t pack4(const float4 &v, const WidthC<B> &c) {
    constexpr uint32_t hi = (1u << B) - 1u;
    const float e[4] = {v.x, v.y, v.z, v.w};
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) w |= code_r(div_r<kFast>(e[i], c.s, c.r) + c.z, hi) << (i * B);   // :61-64
    return w;
}

__device__ __forceinline__ void fold4(const float4 &v, float &mx, float &mn) {
    mx = fmaxf(mx, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    mn = fminf(mn, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
}

// Register slot s (wave-uniform) by a switch: the quantize body below exists once, not once per
// slot (a fully unrolled body over the slots is ~150 KB of code, past the 64 KB instruction cache).
__device__ __forceinline__ float4 pick(const float4 (&r)[kRReg], int s) {
    switch (s) {
    case 0: return r[0];
    case 1: return r[1];
    case 2: return r[2];
    case 3: return r[3];
    case 4: return r[4];
    case 5: return r[5];
    case 6: return r[6];
    case 7: return r[7];
    case 8: return r[8];
    case 9: return r[9];
    case 10: return r[10];
    case 11: return r[11];
    case 12: return r[12];
    case 13: return r[13];
    case 14: return r[14];
    case 15: return r[15];
    case 16: return r[16];
    case 17: return r[17];
    case 18: return r[18];
    case 19: return r[19];
    case 20: return r[20];
    case 21: return r[21];
    case 22: return r[22];
    default: return r[0];
    }
}

template <int BA, int BB>
__global__ void __launch_bounds__(kRT, 1) quantize_resident_kernel(const RArgs A) {
    __shared__ __attribute__((aligned(16))) float4 lds[kRLds * kRT];
    __shared__ float red[2][2][kRT / 64];
    __shared__ float bc[2][2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned b = blockIdx.x;
    const int J0 = A.t[0].J, J1 = A.nt > 1 ? A.t[1].J : 0, S = J0 + J1;
    const int lab = DLLM_LAB ? A.lab : 0;
    // slot s -> (tensor, float4 index); indices past the tensor are clamped to its last float4 for
    // the loads (a duplicate of a value already folded) and skipped by the stores
    auto slot = [&](int s, int &t, size_t &f) __attribute__((always_inline)) {
        t = s < J0 ? 0 : 1;
        const int j = t ? s - J0 : s;
        f = (static_cast<size_t>(b) * A.t[t].J + j) * kRT + tid;
    };

    // ---- phase 1: load the block's slots (VGPRs, then LDS by LDS-DMA) and fold the extremes ----
    float4 r[kRReg];
#pragma unroll
    for (int s = 0; s < kRReg; ++s) {
        if (s < S && (lab & 8) == 0) {
            int t;
            size_t f;
            slot(s, t, f);
            const size_t fc = f < A.t[t].n4 ? f : A.t[t].n4 - 1;
            const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(A.t[t].x) + fc);   // streamed once
            r[s] = make_float4(v.x, v.y, v.z, v.w);
        }
    }
    for (int s = kRReg; s < ((lab & 8) ? kRReg : S); ++s) {
        int t;
        size_t f;
        slot(s, t, f);
        const size_t fc = f < A.t[t].n4 ? f : A.t[t].n4 - 1;
        __builtin_amdgcn_global_load_lds(
            (gbl_void_ptr)(const_cast<float *>(A.t[t].x) + 4 * fc),
            (lds_void_ptr)(&lds[(s - kRReg) * kRT + wave * 64]), 16, 0, 0);
    }
    float mx[2] = {-INFINITY, -INFINITY}, mn[2] = {INFINITY, INFINITY};
    float cmx = -INFINITY, cmn = INFINITY;   // the running tensor's fold (tensor 0's slots come first)
#pragma unroll
    for (int s = 0; s < kRReg; ++s) {
        if (s < S) {
            if (s == J0) { mx[0] = cmx; mn[0] = cmn; cmx = -INFINITY; cmn = INFINITY; }
            fold4(r[s], cmx, cmn);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's LDS-DMA pieces landed
    for (int s = kRReg; s < S; ++s) {
        if (s == J0) { mx[0] = cmx; mn[0] = cmn; cmx = -INFINITY; cmn = INFINITY; }
        fold4(lds[(s - kRReg) * kRT + tid], cmx, cmn);
    }
    if (S <= J0) { mx[0] = cmx; mn[0] = cmn; }   // one tensor: its fold is still running
    else { mx[1] = cmx; mn[1] = cmn; }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        mx[t] = wave_max(mx[t]);
        mn[t] = wave_min(mn[t]);
        if (lane == 0) { red[t][0][wave] = mx[t]; red[t][1][wave] = mn[t]; }
    }
    __syncthreads();

    // ---- grid hand-off of the partials ----
    if (tid == 0 && (lab & 1) == 0) {
        const unsigned gen = __hip_atomic_load(&A.sync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            float a = -INFINITY, c = INFINITY;
            for (int w = 0; w < kRT / 64; ++w) { a = fmaxf(a, red[t][0][w]); c = fminf(c, red[t][1][w]); }
            float *pp = reinterpret_cast<float *>(&A.partials[t * A.nb + b]);
            __hip_atomic_store(pp, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);       // sc1 stores
            __hip_atomic_store(pp + 1, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drained before the arrival is counted
        const unsigned arrived = __hip_atomic_fetch_add(&A.sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == A.nb - 1) {   // the last block: reset the count for the next launch, release all
            __hip_atomic_store(&A.sync[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(&A.sync[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(&A.sync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > kPollTicks) {
                    __hip_atomic_store(&A.sync[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    __syncthreads();

    // ---- every block folds all partials (order-free: identical everywhere) ----
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        float a = -INFINITY, c = INFINITY;
        for (unsigned i = tid; i < A.nb; i += kRT) {   // sc1 loads: the other blocks' partials
            const float *pp = reinterpret_cast<const float *>(&A.partials[t * A.nb + i]);
            a = fmaxf(a, __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            c = fminf(c, __hip_atomic_load(pp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
        a = wave_max(a);
        c = wave_min(c);
        if (lane == 0) { red[t][0][wave] = a; red[t][1][wave] = c; }
    }
    __syncthreads();
    if (tid < 2) {
        float a = -INFINITY, c = INFINITY;
        for (int w = 0; w < kRT / 64; ++w) { a = fmaxf(a, red[tid][0][w]); c = fminf(c, red[tid][1][w]); }
        bc[tid][0] = a;
        bc[tid][1] = c;
    }
    __syncthreads();
    const bool failed = __hip_atomic_load(&A.sync[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    constexpr int BB1 = BB ? BB : BA;
    WidthC<BA> ca[2];
    WidthC<BB1> cb[2];
    bool fast = true;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        float s0, z0, s1 = 1.0f, z1 = 0.0f;
        rs_params(bc[t][0], bc[t][1], BA, s0, z0);
        if (BB) rs_params(bc[t][0], bc[t][1], BB1, s1, z1);
        if (failed) s0 = z0 = s1 = z1 = NAN;
        ca[t] = WidthC<BA>{s0, z0, 1.0f / s0};
        cb[t] = WidthC<BB1>{s1, z1, 1.0f / s1};
        if (t < A.nt) fast = fast && markstein_ok_r(s0) && (BB == 0 || markstein_ok_r(s1));
        if (b == 0 && tid == 0 && t < A.nt) {
            A.t[t].params[0][0] = s0;
            A.t[t].params[0][1] = z0;
            if (BB) { A.t[t].params[1][0] = s1; A.t[t].params[1][1] = z1; }
        }
    }
    if (lab & 4) return;

    // ---- phase 2: quantize the block's slots, one contiguous piece per wave-instruction ----
    auto emit = [&](const float4 &v, int t, size_t f, auto fast_tag) __attribute__((always_inline)) {
        constexpr bool F = decltype(fast_tag)::value;
        const bool ok = f < A.t[t].n4 && (lab & 2) == 0;
        store_quad_r(A.t[t].out[0], f, pack4<BA, F>(v, ca[t]), BA, lane, ok);
        if constexpr (BB != 0) store_quad_r(A.t[t].out[1], f, pack4<BB1, F>(v, cb[t]), BB, lane, ok);
    };
    if (fast) {
        for (int s = 0; s < S; ++s) {   // one copy of the body; the register slot by a uniform switch
            int t;
            size_t f;
            slot(s, t, f);
            const float4 v = s < kRReg ? pick(r, s) : lds[(s - kRReg) * kRT + tid];
            emit(v, t, f, std::integral_constant<bool, true>{});
        }
    } else {
        // scales outside the Markstein range (|s| < 2^-64 or > 2^64): the IEEE division, the
        // slice read back from HBM (rare; kept compact so the fast path keeps the cache)
        for (int s = 0; s < S; ++s) {
            int t;
            size_t f;
            slot(s, t, f);
            const size_t fc = f < A.t[t].n4 ? f : A.t[t].n4 - 1;
            const float4 v = reinterpret_cast<const float4 *>(A.t[t].x)[fc];
            emit(v, t, f, std::integral_constant<bool, false>{});
        }
    }
}

template <int BA>
void launch_res_b(const RArgs &A, int bb, unsigned nb, hipStream_t st) {
    switch (bb) {
    case 0: quantize_resident_kernel<BA, 0><<<nb, kRT, 0, st>>>(A); break;
    case 1: quantize_resident_kernel<BA, 1><<<nb, kRT, 0, st>>>(A); break;
    case 2: quantize_resident_kernel<BA, 2><<<nb, kRT, 0, st>>>(A); break;
    case 4: quantize_resident_kernel<BA, 4><<<nb, kRT, 0, st>>>(A); break;
    default: quantize_resident_kernel<BA, 8><<<nb, kRT, 0, st>>>(A); break;
    }
}

}  // namespace

// Launches the single-pass kernel when the tensors fit on chip; returns 1 (nothing launched) when
// they do not or the shape is outside its preconditions, so the caller runs the two-pass path.
int launch_quantize_resident(const float *const *x, const size_t *n, int nt, const int *bits, uint8_t *const *out,
                             float *const *params, void *ws, size_t ws_bytes, hipStream_t st) {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        hipDeviceProp_t p;
        if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return 1;
        cus = p.multiProcessorCount;
    }
    const unsigned nb = static_cast<unsigned>(cus);
    if (nb == 0 || nb > 1024 || nt < 1 || nt > 2) return 1;
    const auto width_ok = [](int w) { return w == 1 || w == 2 || w == 4 || w == 8; };
    if (!width_ok(bits[0]) || (bits[1] && !width_ok(bits[1]))) return 1;
    RArgs A{};
    A.nt = nt;
    A.bits[0] = bits[0];
    A.bits[1] = bits[1];
    int S = 0;
    for (int t = 0; t < nt; ++t) {
        if (n[t] == 0 || n[t] % 8 || (reinterpret_cast<uintptr_t>(x[t]) & 15)) return 1;
        for (int w = 0; w < (bits[1] ? 2 : 1); ++w)
            if (reinterpret_cast<uintptr_t>(out[2 * t + w]) & 7) return 1;
        const size_t per = static_cast<size_t>(nb) * kRT * 4;   // values per slot over the grid
        const int J = static_cast<int>((n[t] + per - 1) / per);
        A.t[t] = RTensor{x[t], n[t] / 4, {out[2 * t], out[2 * t + 1]}, {params[2 * t], params[2 * t + 1]}, J};
        S += J;
    }
    if (S > kRReg + kRLds) return 1;
    const size_t need = 2 * nb * sizeof(float2);
    if (!ws || ws_bytes < need) return 1;
    A.partials = static_cast<float2 *>(ws);
    A.sync = zeroed_counters(st, 4);
    if (!A.sync) return DLLM_ERR_HIP;
    // sync[2] is the hand-off timeout word: a timed-out launch writes NaN params (so its failure is
    // visible in its own output); clearing it per launch keeps one timeout from poisoning the next
    if (hipMemsetAsync(A.sync + 2, 0, sizeof(unsigned), st) != hipSuccess) return fail(DLLM_ERR_HIP, "hipMemsetAsync");
    A.nb = nb;
#if DLLM_LAB
    if (const char *e = std::getenv("DLLM_RES_LAB")) A.lab = std::atoi(e);
#endif
    switch (bits[0]) {
    case 1: launch_res_b<1>(A, bits[1], nb, st); break;
    case 2: launch_res_b<2>(A, bits[1], nb, st); break;
    case 4: launch_res_b<4>(A, bits[1], nb, st); break;
    default: launch_res_b<8>(A, bits[1], nb, st); break;
    }
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}


}  // namespace dllm
