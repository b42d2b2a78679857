// capi.cpp -- library-level C-ABI entry points (errors, version, device probe).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "dllm_quant.h"

namespace dllm {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

// Grow-only per-(device, stream, slot) workspaces.  A buffer handed out while its stream was being
// captured is referenced by that graph for as long as the graph lives, so once captured it is never
// freed: a later, larger request on the same slot allocates a new buffer and RETIRES the captured one
// (kept until process exit), so replaying an earlier graph after an eager call of a larger shape
// still reads and writes valid memory (its own old buffer, which no eager call uses any more).
// Buffers never seen by a capture are freed on growth as before.
namespace {
struct Workspace {
    void *p = nullptr;
    size_t bytes = 0;
    bool captured = false;
};
std::vector<void *> &retired_workspaces() {
    static std::vector<void *> v;   // captured buffers replaced by larger ones: alive for graph replays
    return v;
}
bool stream_capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cs);
    return cs != hipStreamCaptureStatusNone;
}
// Returns the slot's buffer of at least `bytes` (zeroed when `zero`), or nullptr with the error set.
void *grow_workspace(Workspace &e, hipStream_t st, size_t bytes, bool zero, const char *what) {
    const bool capturing = stream_capturing(st);
    if (e.bytes >= bytes) {
        if (capturing) e.captured = true;
        return e.p;
    }
    if (capturing) {
        fail(DLLM_ERR_HIP, std::string(what) + " must be sized before stream capture (run the shape once first)");
        return nullptr;
    }
    if (e.p) {
        if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
        if (e.captured) retired_workspaces().push_back(e.p);
        else (void)hipFree(e.p);
        e = Workspace{};
    }
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        fail(DLLM_ERR_HIP, std::string("hipMalloc of the ") + what + " failed");
        return nullptr;
    }
    if (zero && hipMemsetAsync(p, 0, bytes, st) != hipSuccess) {
        (void)hipFree(p);
        fail(DLLM_ERR_HIP, std::string("zeroing the ") + what + " failed");
        return nullptr;
    }
    e.p = p;
    e.bytes = bytes;
    return p;
}
std::mutex g_ws_mu;   // guards both pools and the retired list
}  // namespace

float *device_workspace(hipStream_t st, size_t bytes, int slot) {
    static std::map<std::tuple<int, hipStream_t, int>, Workspace> pool;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_ws_mu);
    return static_cast<float *>(grow_workspace(pool[{dev, st, slot}], st, bytes, false, "device workspace"));
}

unsigned *zeroed_counters(hipStream_t st, size_t n) {
    static std::map<std::pair<int, hipStream_t>, Workspace> pool;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_ws_mu);
    const size_t cap = std::max<size_t>(n, 64);
    return static_cast<unsigned *>(grow_workspace(pool[{dev, st}], st, cap * sizeof(unsigned), true, "hand-off words"));
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
