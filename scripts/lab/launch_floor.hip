// Launch-floor calibration (measurement only): rocprofv3 kernel durations of near-empty kernels
// at the decode GEMM's grid shapes, to separate the per-launch floor from the decode kernel's work.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void empty_kernel(float *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) out[0] = 1.0f;
}

// An 8-wave block that does the decode kernel's non-load skeleton: each wave writes a 1 KiB partial
// to LDS, a barrier, wave 0 sums the 8 partials and stores 16 B per lane.
__global__ void __launch_bounds__(512) skeleton_kernel(float *out) {
    __shared__ float red[8 * 64 * 4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float4 v = make_float4(lane, wave, 1.f, 2.f);
    *reinterpret_cast<float4 *>(red + (wave * 64 + lane) * 4) = v;
    __syncthreads();
    if (wave == 0) {
        float4 s = make_float4(0, 0, 0, 0);
        for (int w = 0; w < 8; ++w) {
            float4 t = *reinterpret_cast<const float4 *>(red + (w * 64 + lane) * 4);
            s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
        }
        *reinterpret_cast<float4 *>(out + (blockIdx.x * 64 + lane) * 4) = s;
    }
}

// Streams `bytes` of a buffer once (16 B per lane per load, grid-stride), as the weight stream of
// one decode layer, and keeps a never-true store so the loads stay.
__global__ void __launch_bounds__(512) stream_kernel(const uint4 *in, size_t n16, float *out) {
    uint32_t x = 0;
    for (size_t i = blockIdx.x * 512ull + threadIdx.x; i < n16; i += gridDim.x * 512ull) {
        const uint4 v = in[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9e3779b9u) out[0] = 1.0f;
}

int main() {
    float *out = nullptr;
    uint4 *buf = nullptr;
    const size_t layer = 9u << 20, nl = 48;
    if (hipMalloc(&out, 1 << 22) != hipSuccess || hipMalloc(&buf, layer * nl) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, layer * nl);
    for (int rep = 0; rep < 200; ++rep) {
        empty_kernel<<<256, 512>>>(out);
        empty_kernel<<<256, 256>>>(out);
        empty_kernel<<<256, 64>>>(out);
        empty_kernel<<<1, 64>>>(out);
        skeleton_kernel<<<256, 512>>>(out);
    }
    // 48 distinct 9 MiB "layers" (432 MiB > the 256 MB Infinity Cache), one launch each
    for (int rep = 0; rep < 20; ++rep)
        for (size_t l = 0; l < nl; ++l)
            stream_kernel<<<256, 512>>>(buf + l * (layer / 16), layer / 16, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("done\n");
    return 0;
}
