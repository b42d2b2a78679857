// common.hpp -- shared helpers for the gfx950 HIP kernels and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "dllm_quant.h"

// Streaming (non-temporal) stores for the GEMMs' f16 tile rows (whole 512-B rows per instruction;
// A/B builds: -DDLLM_NT_STORE=0).  Not for the dequantize outputs: there the same hint is 1.1-2.7x
// slower (profiles/r03_nt_store/dequant_ab.jsonl).
#ifndef DLLM_NT_STORE
#define DLLM_NT_STORE 1
#endif

namespace dllm {

// Thread-local error message behind dllm_last_error().
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

#define DLLM_HIP_TRY(expr)                                                                        \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess)                                                                     \
            return ::dllm::fail(DLLM_ERR_HIP, std::string(#expr " -> ") + hipGetErrorString(_e)); \
    } while (0)

#define DLLM_LAUNCH_CHECK()                                                                       \
    do {                                                                                          \
        hipError_t _e = hipGetLastError();                                                        \
        if (_e != hipSuccess)                                                                     \
            return ::dllm::fail(DLLM_ERR_HIP, std::string("kernel launch -> ") + hipGetErrorString(_e)); \
    } while (0)

inline hipStream_t as_stream(dllm_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Grow-only device workspace, one per (device, stream, slot): launches on one stream run in order,
// so every call on that stream can share it.  A growth waits for the stream first (queued kernels
// may still use the old buffer) and is refused while the stream is being captured.  Returns null
// (error set) on failure.
float *device_workspace(hipStream_t st, size_t bytes, int slot = 0);
// Grow-only per-(device, stream) array of u32 words, zeroed when (re)allocated (outside stream
// capture): the grid hand-off words of quant_resident.hip, whose kernels leave them reusable.
unsigned *zeroed_counters(hipStream_t st, size_t n);

typedef __attribute__((address_space(3))) void *lds_void_ptr;
typedef __attribute__((address_space(1))) void *gbl_void_ptr;

// LDS-DMA (global_load_lds) issued from inline asm: invisible to hipcc's waitcnt pass, so the only
// waits on these loads are the counted vmcnt statements placed by hand (M0 written in the statement).
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_ptr)(const_cast<void *>(p))));
}
__device__ __forceinline__ void glds16_asm(const void *gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void glds4_asm(const void *gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

// LDS-DMA through a buffer descriptor: address = base(rs) + voff (per lane, fixed) + soff (wave-
// uniform, advances per stage), so a stage's DMAs need no per-lane address arithmetic.
__device__ __forceinline__ void blds16_asm(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds_dst), "s"(soff) : "memory");
}
__device__ __forceinline__ void blds4_asm(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds_dst), "s"(soff) : "memory");
}
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
// Buffer load of 16 B per lane into VGPRs from inline asm: like the LDS-DMA above, invisible to
// hipcc's waitcnt pass -- the caller's counted vmcnt waits must cover it before d is read.
__device__ __forceinline__ void bload16_asm(u32x4_t &d, __amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(rs), "s"(soff) : "memory");
}
// Raw buffer descriptor over [base, base + 4 GiB) (no range clamp is relied on).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, 0x7FFFFFFF, 0x00020000);
}

constexpr int kWave = 64;      // CDNA wavefront width
constexpr int kCUs = 256;      // MI355X compute units (8 XCDs x 32)
constexpr int kXCDs = 8;

inline unsigned grid_for(size_t work_items, int block, unsigned cap = kCUs * 8) {
    size_t g = (work_items + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return static_cast<unsigned>(g);
}

// ---- Rust f32 semantics on the device (bit-exact with the oracle) -----------------------------
// Built with -ffp-contract=off; x/s below is the IEEE correctly rounded division (hipcc default).

// `f32::clamp`: NaN passes through.  Written as compares + selects so no v_max/v_min (which
// would drop a NaN) can be substituted.
__device__ __forceinline__ float rs_clamp(float x, float lo, float hi) {
    x = (x < lo) ? lo : x;
    x = (x > hi) ? hi : x;
    return x;
}
// `f as u8`: NaN -> 0, saturating, truncating.
__device__ __forceinline__ uint32_t rs_as_u8(float f) {
    if (!(f > 0.0f)) return 0u;          // NaN, <= 0
    if (f >= 255.0f) return 255u;
    return static_cast<uint32_t>(f);     // in (0, 255): truncation
}
// `(round(v) as i32).clamp(0, hi)` fused: NaN -> 0, saturating, then clamp.
__device__ __forceinline__ uint32_t rs_round_i32_clamp(float v, int hi) {
    float r = roundf(v);
    if (!(r > 0.0f)) return 0u;          // NaN -> 0 -> 0, negatives -> 0
    if (r >= static_cast<float>(hi)) return static_cast<uint32_t>(hi);
    return static_cast<uint32_t>(r);
}

// Wave-level reductions (64 lanes, xor-shuffle lowers to DPP/ds_swizzle).
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}

}  // namespace dllm
