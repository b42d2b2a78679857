// capi_host.cpp -- host-slice entry points (*_host): the literal shapes of the reference's Rust
// signatures (&[f32] in, Vec<u8> / Vec<f32> out).  Each call stages through device memory on its
// own stream, runs the same HIP kernels as the device entry points, and synchronises.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "dllm_quant.h"

namespace dllm {
int fail(int code, const std::string &msg);
}

namespace {

struct Staging {
    std::vector<void *> bufs;
    hipStream_t st = nullptr;
    int err = DLLM_OK;
    Staging() {
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
            st = nullptr;
            err = dllm::fail(DLLM_ERR_HIP, "hipStreamCreate failed (no device?)");
        }
    }
    ~Staging() {
        for (void *p : bufs) (void)hipFree(p);
        if (st) (void)hipStreamDestroy(st);
    }
    template <typename T>
    T *alloc(size_t count) {
        void *p = nullptr;
        if (hipMalloc(&p, count * sizeof(T) + 16) != hipSuccess) {
            err = dllm::fail(DLLM_ERR_HIP, "hipMalloc failed");
            return nullptr;
        }
        bufs.push_back(p);
        return static_cast<T *>(p);
    }
    template <typename T>
    T *upload(const T *h, size_t count) {
        T *d = alloc<T>(count);
        if (d && count && hipMemcpyAsync(d, h, count * sizeof(T), hipMemcpyHostToDevice, st) != hipSuccess)
            err = dllm::fail(DLLM_ERR_HIP, "hipMemcpy H2D failed");
        return d;
    }
    template <typename T>
    int download(T *h, const T *d, size_t count) {
        if (count && hipMemcpyAsync(h, d, count * sizeof(T), hipMemcpyDeviceToHost, st) != hipSuccess)
            return dllm::fail(DLLM_ERR_HIP, "hipMemcpy D2H failed");
        return DLLM_OK;
    }
    int sync() {
        if (hipStreamSynchronize(st) != hipSuccess) return dllm::fail(DLLM_ERR_HIP, "hipStreamSynchronize failed");
        return DLLM_OK;
    }
};

#define STAGE_OK(s) \
    do {            \
        if ((s).err) return (s).err; \
    } while (0)

}  // namespace

extern "C" {

int dllm_quantize_tensor_host(const float *x, size_t n, uint8_t bits, uint8_t *codes, float *scale, float *zp) {
    if (bits < 1 || bits > 8) return dllm::fail(DLLM_ERR_INVALID_PARAMS, "Bits must be between 1 and 8");
    Staging s;
    STAGE_OK(s);
    const float *dx = s.upload(x, n);
    uint8_t *dq = s.alloc<uint8_t>(n);
    float *dp = s.alloc<float>(2);
    const size_t wsb = dllm_quantize_tensor_workspace(n);
    void *ws = s.alloc<uint8_t>(wsb);
    STAGE_OK(s);
    int rc = dllm_quantize_tensor(dx, n, bits, 0, dq, dp, ws, wsb, s.st);
    if (rc) return rc;
    float p[2];
    if ((rc = s.download(codes, dq, n)) || (rc = s.download(p, dp, 2)) || (rc = s.sync())) return rc;
    *scale = p[0];
    *zp = p[1];
    return DLLM_OK;
}

int dllm_dequantize_tensor_host(const uint8_t *codes, size_t n, float scale, float zp, float *out) {
    Staging s;
    STAGE_OK(s);
    const uint8_t *dq = s.upload(codes, n);
    float *dy = s.alloc<float>(n);
    STAGE_OK(s);
    int rc = dllm_dequantize_tensor_scalar(dq, n, 8, 0, scale, zp, dy, DLLM_F32, s.st);
    if (rc || (rc = s.download(out, dy, n)) || (rc = s.sync())) return rc;
    return DLLM_OK;
}

int dllm_default_quantize_host(const float *x, size_t n, int qtype, float scale, int32_t zero_point, uint8_t *out) {
    Staging s;
    STAGE_OK(s);
    const float *dx = s.upload(x, n);
    uint8_t *dq = s.alloc<uint8_t>(n);
    STAGE_OK(s);
    int rc = dllm_default_quantize(dx, n, qtype, scale, zero_point, dq, s.st);
    if (rc || (rc = s.download(out, dq, n)) || (rc = s.sync())) return rc;
    return DLLM_OK;
}

int dllm_default_dequantize_host(const uint8_t *q, size_t n, float scale, int32_t zero_point, float *out) {
    Staging s;
    STAGE_OK(s);
    const uint8_t *dq = s.upload(q, n);
    float *dy = s.alloc<float>(n);
    STAGE_OK(s);
    int rc = dllm_default_dequantize(dq, n, scale, zero_point, dy, s.st);
    if (rc || (rc = s.download(out, dy, n)) || (rc = s.sync())) return rc;
    return DLLM_OK;
}

int dllm_bit_quantize_host(const float *x, size_t n, uint32_t bits, float scale, float zero_point, uint8_t *out) {
    if (bits > 30) return dllm::fail(DLLM_ERR_INVALID_PARAMS, "(1 << bits) - 1 overflows i32");
    Staging s;
    STAGE_OK(s);
    const float *dx = s.upload(x, n);
    uint8_t *dq = s.alloc<uint8_t>(n);
    STAGE_OK(s);
    int rc = dllm_bit_quantize(dx, n, bits, scale, zero_point, dq, s.st);
    if (rc || (rc = s.download(out, dq, n)) || (rc = s.sync())) return rc;
    return DLLM_OK;
}

int dllm_bit_dequantize_host(const uint8_t *q, size_t n, float scale, float zero_point, float *out) {
    Staging s;
    STAGE_OK(s);
    const uint8_t *dq = s.upload(q, n);
    float *dy = s.alloc<float>(n);
    STAGE_OK(s);
    int rc = dllm_bit_dequantize(dq, n, scale, zero_point, dy, DLLM_F32, s.st);
    if (rc || (rc = s.download(out, dy, n)) || (rc = s.sync())) return rc;
    return DLLM_OK;
}

int dllm_compress_vector_host(const float *x, size_t n, uint8_t bits, uint8_t *out, float *scale, float *zp) {
    Staging s;
    STAGE_OK(s);
    const float *dx = s.upload(x, n);
    uint8_t *dq = s.alloc<uint8_t>(n);
    float *dsc = s.alloc<float>(1);
    float *dzp = s.alloc<float>(1);
    STAGE_OK(s);
    int rc = dllm_compress_vectors(dx, 1, n, bits, dq, dsc, dzp, s.st);
    if (rc || (rc = s.download(out, dq, n)) || (rc = s.download(scale, dsc, 1)) || (rc = s.download(zp, dzp, 1)) ||
        (rc = s.sync()))
        return rc;
    return DLLM_OK;
}

int dllm_linear_create_host(const float *W, const float *bias, size_t K, size_t N, uint8_t bits, size_t group,
                            dllm_linear_t *out) {
    Staging s;
    STAGE_OK(s);
    const float *dW = s.upload(W, K * N);
    const float *db = bias ? s.upload(bias, N) : nullptr;
    STAGE_OK(s);
    int rc = dllm_linear_create(dW, db, K, N, bits, group, out, s.st);
    if (rc) return rc;
    return s.sync();
}

int dllm_linear_forward_host(dllm_linear_t h, const float *X, size_t M, float *Y) {
    size_t K = 0, N = 0;
    int rc = dllm_linear_info(h, &K, &N, nullptr, nullptr);
    if (rc) return rc;
    Staging s;
    STAGE_OK(s);
    const float *dX = s.upload(X, M * K);
    float *dY = s.alloc<float>(M * N);
    STAGE_OK(s);
    if ((rc = dllm_linear_forward(h, dX, M, DLLM_F32, dY, DLLM_F32, s.st))) return rc;
    if ((rc = s.download(Y, dY, M * N)) || (rc = s.sync())) return rc;
    return DLLM_OK;
}

}  // extern "C"
