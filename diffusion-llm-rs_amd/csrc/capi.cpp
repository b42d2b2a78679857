// capi.cpp -- library-level C-ABI entry points (errors, version, device probe).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>

#include "dllm_quant.h"

namespace dllm {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

float *device_workspace(hipStream_t st, size_t bytes, int slot) {
    static std::mutex mu;
    static std::map<std::tuple<int, hipStream_t, int>, std::pair<float *, size_t>> pool;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    auto &e = pool[{dev, st, slot}];
    if (e.second >= bytes) return e.first;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs != hipStreamCaptureStatusNone) {
        fail(DLLM_ERR_HIP, "device workspace must be sized before stream capture (run the shape once first)");
        return nullptr;
    }
    if (e.first) {
        if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
        (void)hipFree(e.first);
        e = {nullptr, 0};
    }
    float *p = nullptr;
    if (hipMalloc(reinterpret_cast<void **>(&p), bytes) != hipSuccess) {
        fail(DLLM_ERR_HIP, "hipMalloc of a device workspace failed");
        return nullptr;
    }
    e = {p, bytes};
    return p;
}

unsigned *zeroed_counters(hipStream_t st, size_t n) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, std::pair<unsigned *, size_t>> pool;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    auto &e = pool[{dev, st}];
    if (e.second >= n) return e.first;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    if (cs != hipStreamCaptureStatusNone) {
        fail(DLLM_ERR_HIP, "hand-off words must be allocated before stream capture (run the shape once first)");
        return nullptr;
    }
    if (e.first) {
        if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
        (void)hipFree(e.first);
        e = {nullptr, 0};
    }
    unsigned *p = nullptr;
    const size_t cap = std::max<size_t>(n, 64);
    if (hipMalloc(reinterpret_cast<void **>(&p), cap * sizeof(unsigned)) != hipSuccess ||
        hipMemsetAsync(p, 0, cap * sizeof(unsigned), st) != hipSuccess) {
        fail(DLLM_ERR_HIP, "hipMalloc of the hand-off words failed");
        return nullptr;
    }
    e = {p, cap};
    return p;
}

}  // namespace dllm

extern "C" {

const char *dllm_last_error(void) { return dllm::g_last_error.c_str(); }

const char *dllm_version(void) { return "dllm_hip 0.1.0 (gfx950)"; }

int dllm_device_arch(int device, char *buf, size_t len) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return dllm::fail(DLLM_ERR_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= count) return dllm::fail(DLLM_ERR_INVALID_PARAMS, "device index out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return dllm::fail(DLLM_ERR_HIP, "hipGetDeviceProperties");
    if (buf && len) {
        std::strncpy(buf, prop.gcnArchName, len - 1);
        buf[len - 1] = '\0';
    }
    return DLLM_OK;
}

}  // extern "C"
