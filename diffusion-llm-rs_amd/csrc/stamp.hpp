// stamp.hpp -- in-kernel s_memtime stamps: where a GEMM block's time goes (prologue fill, each
// k-step's MFMA issue and its wait + barrier, epilogue).  Diagnostic builds only:
//     make -C diffusion-llm-rs_amd/csrc variant VNAME=stamp VFLAGS=-DDLLM_STAMP=1
// The product build compiles every hook to nothing (DLLM_STAMP defaults to 0).  Stamps go to a
// buffer of their own that no other code reads (MI355X_MICROARCH.md, DVFS give-back item 6), one
// row of kSlots per (block, wave), written by the wave's lane 0 with a vector store; the TU that
// instruments a kernel exports a reader (dllm_stamp_read_<tu>) in the stamp build only.
#pragma once

#ifndef DLLM_STAMP
#define DLLM_STAMP 0
#endif

#if DLLM_STAMP
#include <hip/hip_runtime.h>
namespace dllm {
namespace stamp {
constexpr int kSlots = 64;    // per (block, wave): 0 entry, 1 prologue done, 2 + 4 kt .. 5 + 4 kt step kt
                              // (its DMA issued / MFMAs issued / vmcnt + lgkmcnt wait passed / past
                              // the step's barrier), kEpi, kEnd, kRtEntry / kRtEnd
                              // (s_memrealtime, 100 MHz, comparable across XCDs), kHwId, kXcc
constexpr int kWaves = 16;
constexpr int kBlocks = 2048;
constexpr int kEpi = 58, kEnd = 59, kRtEntry = 60, kRtEnd = 61, kHwId = 62, kXcc = 63;
constexpr int kPerStep = 4;
constexpr int kMaxStep = (kEpi - 2) / kPerStep - 1;   // steps past this are not stamped
}  // namespace stamp
}  // namespace dllm
#define DLLM_STAMP_BUFFER(name) \
    static __device__ unsigned long long name[dllm::stamp::kBlocks * dllm::stamp::kWaves * dllm::stamp::kSlots]
// Linear block id, so a 2-D grid (the decode kernel's K-split) does not fold rows onto each other.
#define DLLM_STAMP_BLOCK (blockIdx.x + gridDim.x * blockIdx.y)
#define DLLM_STAMP_ROW(buf) \
    (buf + (static_cast<size_t>(DLLM_STAMP_BLOCK) * dllm::stamp::kWaves + (threadIdx.x >> 6)) * dllm::stamp::kSlots)
#define DLLM_STAMP_AT(buf, slot)                                                                            \
    do {                                                                                                    \
        const int _s = (slot);                                                                              \
        if ((threadIdx.x & 63) == 0 && DLLM_STAMP_BLOCK < dllm::stamp::kBlocks && _s >= 0 && _s < dllm::stamp::kSlots) \
            DLLM_STAMP_ROW(buf)[_s] = __builtin_amdgcn_s_memtime();                                         \
    } while (0)
#define DLLM_STAMP_RT(buf, slot)                                                                            \
    do {                                                                                                    \
        if ((threadIdx.x & 63) == 0 && DLLM_STAMP_BLOCK < dllm::stamp::kBlocks)                                   \
            DLLM_STAMP_ROW(buf)[slot] = __builtin_amdgcn_s_memrealtime();                                   \
    } while (0)
#define DLLM_STAMP_IDS(buf)                                                                                 \
    do {                                                                                                    \
        unsigned _hw, _xcc;                                                                                 \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(_hw));                                   \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(_xcc));                                 \
        if ((threadIdx.x & 63) == 0 && DLLM_STAMP_BLOCK < dllm::stamp::kBlocks) {                                 \
            DLLM_STAMP_ROW(buf)[dllm::stamp::kHwId] = _hw;                                                  \
            DLLM_STAMP_ROW(buf)[dllm::stamp::kXcc] = _xcc;                                                  \
        }                                                                                                   \
    } while (0)
// the reader: copies the whole buffer (kBlocks x kWaves x kSlots u64) to host memory
#define DLLM_STAMP_READER(fn, buf)                                                                          \
    extern "C" int fn(void *host, size_t bytes) {                                                           \
        const size_t n = sizeof(buf) < bytes ? sizeof(buf) : bytes;                                         \
        return hipMemcpyFromSymbol(host, HIP_SYMBOL(buf), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 8; \
    }                                                                                                       \
    extern "C" int fn##_zero(void) {                                                                        \
        void *p = nullptr;                                                                                  \
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(buf)) != hipSuccess) return 8;                               \
        return hipMemset(p, 0, sizeof(buf)) == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : 8;  \
    }
#else
#define DLLM_STAMP_AT(buf, slot) ((void)0)
#define DLLM_STAMP_RT(buf, slot) ((void)0)
#define DLLM_STAMP_IDS(buf) ((void)0)
#endif
