// diffusion.hip -- the elementwise ops either side of the denoiser in every timestep (SURVEY.md
// 8f rank 1): beta schedules and alpha-bar tables (host scalars, Rust f32 semantics), the
// p_sample posterior step and the add_noise forward step (HBM-bound kernels), and the seeded
// Gaussian noise they draw (Philox4x32-10 + a Box-Muller built only from correctly rounded
// + - * / sqrt, so it is reproducible bit for bit on any IEEE host).
//
// Reference: diffuse-llm-rs/src/lib.rs create_beta_schedule :554-593, p_losses :615-630,
// add_noise :1100-1137, p_sample :1152-1215.
#include "common.hpp"
#include "diffusion_rng.hpp"

#include <cmath>
#include <vector>

namespace dllm {
namespace {

// ---- host scalars (per timestep / per sample) -------------------------------------------------

int alpha_tables(const float *betas, size_t T, int cumprod, std::vector<float> &alphas, std::vector<float> &abar) {
    alphas.resize(T);
    abar.resize(T);
    for (size_t i = 0; i < T; ++i) alphas[i] = 1.0f - betas[i];
    if (cumprod == DLLM_ABAR_INCLUSIVE) {          // p_losses scan, lib.rs:627-630
        float state = 1.0f;
        for (size_t i = 0; i < T; ++i) abar[i] = (state *= alphas[i]);
    } else if (cumprod == DLLM_ABAR_EXCLUSIVE) {   // add_noise / p_sample, lib.rs:1116-1119
        if (T) abar[0] = 1.0f;
        for (size_t i = 1; i < T; ++i) abar[i] = abar[i - 1] * alphas[i - 1];
    } else {
        return fail(DLLM_ERR_INVALID_PARAMS, "cumprod must be DLLM_ABAR_EXCLUSIVE or DLLM_ABAR_INCLUSIVE");
    }
    return DLLM_OK;
}

// ---- device ---------------------------------------------------------------------------------

// x_prev = (c1 x_t + c2 eps) + std * n over rows of D; n = noise[i] (given), the generated stream
// element offset + i (noise == nullptr), or 0 (add == 0).  Four consecutive elements per thread:
// one Philox block when offset % 4 == 0.
__global__ void __launch_bounds__(256) p_sample_kernel(const float *__restrict__ x, const float *__restrict__ eps,
                                                       const float *__restrict__ noise, const float *__restrict__ coef,
                                                       size_t n, size_t D, int add, uint64_t seed, uint64_t offset,
                                                       float *__restrict__ out) {
    const size_t nq = (n + 3) / 4;
    for (size_t q = blockIdx.x * static_cast<size_t>(256) + threadIdx.x; q < nq;
         q += static_cast<size_t>(gridDim.x) * 256) {
        const size_t i0 = q * 4;
        float z[4] = {0.f, 0.f, 0.f, 0.f};
        if (add) {
            if (noise) {
                for (int l = 0; l < 4; ++l)
                    if (i0 + l < n) z[l] = noise[i0 + l];
            } else {
                rng::normal4(seed, (offset + i0) / 4, z);
            }
        }
        if (i0 + 4 <= n && (D % 4) == 0) {
            const float *c = coef + 3 * (i0 / D);
            const float c1 = c[0], c2 = c[1], sd = c[2];
            const float4 xv = *reinterpret_cast<const float4 *>(x + i0);
            const float4 ev = *reinterpret_cast<const float4 *>(eps + i0);
            float4 o;
            o.x = (c1 * xv.x + c2 * ev.x) + sd * z[0];
            o.y = (c1 * xv.y + c2 * ev.y) + sd * z[1];
            o.z = (c1 * xv.z + c2 * ev.z) + sd * z[2];
            o.w = (c1 * xv.w + c2 * ev.w) + sd * z[3];
            *reinterpret_cast<float4 *>(out + i0) = o;
        } else {
            for (int l = 0; l < 4; ++l) {
                const size_t i = i0 + l;
                if (i >= n) break;
                const float *c = coef + 3 * (i / D);
                out[i] = (c[0] * x[i] + c[1] * eps[i]) + c[2] * z[l];
            }
        }
    }
}

// noisy = x0 sqrt(abar) + n sqrt(1 - abar); n given or generated (then optionally written out).
__global__ void __launch_bounds__(256) add_noise_kernel(const float *__restrict__ x0, const float *__restrict__ noise,
                                                        const float *__restrict__ coef, size_t n, size_t D,
                                                        uint64_t seed, uint64_t offset, float *__restrict__ out,
                                                        float *__restrict__ noise_out) {
    const size_t nq = (n + 3) / 4;
    for (size_t q = blockIdx.x * static_cast<size_t>(256) + threadIdx.x; q < nq;
         q += static_cast<size_t>(gridDim.x) * 256) {
        const size_t i0 = q * 4;
        float z[4];
        if (noise) {
            for (int l = 0; l < 4; ++l) z[l] = i0 + l < n ? noise[i0 + l] : 0.f;
        } else {
            rng::normal4(seed, (offset + i0) / 4, z);
        }
        for (int l = 0; l < 4; ++l) {
            const size_t i = i0 + l;
            if (i >= n) break;
            const float *c = coef + 2 * (i / D);
            out[i] = x0[i] * c[0] + z[l] * c[1];
            if (noise_out) noise_out[i] = z[l];
        }
    }
}

__global__ void __launch_bounds__(256) randn_kernel(uint64_t seed, uint64_t offset, size_t n, float *__restrict__ out) {
    const size_t nq = (n + 3) / 4;
    for (size_t q = blockIdx.x * static_cast<size_t>(256) + threadIdx.x; q < nq;
         q += static_cast<size_t>(gridDim.x) * 256) {
        float z[4];
        rng::normal4(seed, offset / 4 + q, z);
        const size_t i0 = q * 4;
        if (i0 + 4 <= n) {
            *reinterpret_cast<float4 *>(out + i0) = make_float4(z[0], z[1], z[2], z[3]);
        } else {
            for (int l = 0; i0 + l < n; ++l) out[i0 + l] = z[l];
        }
    }
}

unsigned elem_grid(size_t n) { return grid_for((n + 3) / 4, 256, kCUs * 16); }

}  // namespace
}  // namespace dllm

using namespace dllm;

extern "C" {

int dllm_beta_schedule(int kind, size_t T, float beta_start, float beta_end, float *betas) {
    if (T && !betas) return fail(DLLM_ERR_INVALID_PARAMS, "betas is NULL");
    const float PI = 3.14159274101257324f;   // std::f32::consts::PI (lib.rs:20)
    for (size_t t = 0; t < T; ++t) {
        float b;
        switch (kind) {
        case DLLM_BETA_LINEAR:       // lib.rs:559-564
            b = beta_start + (beta_end - beta_start) * static_cast<float>(t) / static_cast<float>(T - 1);
            break;
        case DLLM_BETA_QUADRATIC: {  // lib.rs:568-574
            const float tn = static_cast<float>(t) / static_cast<float>(T - 1);
            b = beta_start + (beta_end - beta_start) * tn * tn;
            break;
        }
        case DLLM_BETA_COSINE: {     // lib.rs:578-590
            const float s = 0.008f;
            const float tn = static_cast<float>(t) / static_cast<float>(T);
            float ft = std::cos((tn + s) / (1.0f + s) * PI / 2.0f);
            ft = ft * ft;
            float f0 = std::cos(s / (1.0f + s) * PI / 2.0f);
            f0 = f0 * f0;
            b = std::fmin(1.0f - ft / f0, 0.999f);
            break;
        }
        default:
            return fail(DLLM_ERR_INVALID_PARAMS, "unknown beta schedule kind");
        }
        betas[t] = b;
    }
    return DLLM_OK;
}

int dllm_alpha_bars(const float *betas, size_t T, int cumprod, float *alphas, float *alpha_bars) {
    if (T && (!betas || !alphas || !alpha_bars)) return fail(DLLM_ERR_INVALID_PARAMS, "NULL table");
    std::vector<float> a, ab;
    const int rc = alpha_tables(betas, T, cumprod, a, ab);
    if (rc) return rc;
    for (size_t i = 0; i < T; ++i) {
        alphas[i] = a[i];
        alpha_bars[i] = ab[i];
    }
    return DLLM_OK;
}

int dllm_p_sample_coeffs(const float *betas, size_t T, int cumprod, int alpha_mode, const size_t *t, size_t B,
                         float *coef, int *add_noise) {
    if (T == 0) return fail(DLLM_ERR_INVALID_PARAMS, "empty schedule (betas.len() - 1 underflows, lib.rs:1169)");
    if (!betas || (B && (!t || !coef))) return fail(DLLM_ERR_INVALID_PARAMS, "NULL argument");
    if (alpha_mode != DLLM_ALPHA_PER_SAMPLE && alpha_mode != DLLM_ALPHA_LITERAL)
        return fail(DLLM_ERR_INVALID_PARAMS, "alpha_mode must be DLLM_ALPHA_PER_SAMPLE or DLLM_ALPHA_LITERAL");
    if (alpha_mode == DLLM_ALPHA_LITERAL && B != T)
        return fail(DLLM_ERR_INVALID_PARAMS, "literal alphas broadcast only when batch == num_timesteps (lib.rs:1191)");
    std::vector<float> a, ab;
    const int rc = alpha_tables(betas, T, cumprod, a, ab);
    if (rc) return rc;
    for (size_t i = 0; i < B; ++i) {
        const size_t ti = std::min(t[i], T - 1);
        const float abar_t = ab[ti], beta_t = betas[ti];
        const float alpha = alpha_mode == DLLM_ALPHA_LITERAL ? a[i] : a[ti];
        const float prev = ti > 0 ? ab[ti - 1] : 1.0f;
        coef[3 * i + 0] = (std::sqrt(prev) * beta_t) / (1.0f - abar_t);
        coef[3 * i + 1] = (std::sqrt(alpha) * (1.0f - prev)) / (1.0f - abar_t);
        coef[3 * i + 2] = std::sqrt(((1.0f - prev) / (1.0f - abar_t)) * beta_t);
    }
    if (add_noise) *add_noise = B > 0 && t[0] > 0;   // lib.rs:1198: decided by t[0] alone
    return DLLM_OK;
}

int dllm_add_noise_coeffs(const float *betas, size_t T, int cumprod, const size_t *t, size_t B, float *coef) {
    if (T == 0) return fail(DLLM_ERR_INVALID_PARAMS, "empty schedule (alpha_bars.len() - 1 underflows)");
    if (!betas || (B && (!t || !coef))) return fail(DLLM_ERR_INVALID_PARAMS, "NULL argument");
    std::vector<float> a, ab;
    const int rc = alpha_tables(betas, T, cumprod, a, ab);
    if (rc) return rc;
    for (size_t i = 0; i < B; ++i) {
        const size_t ti = std::min(t[i], T - 1);
        coef[2 * i + 0] = std::sqrt(ab[ti]);
        coef[2 * i + 1] = std::sqrt(1.0f - ab[ti]);
    }
    return DLLM_OK;
}

int dllm_randn(uint64_t seed, uint64_t offset, float *out, size_t n, dllm_stream_t stream) {
    if (n == 0) return DLLM_OK;
    if (!out) return fail(DLLM_ERR_INVALID_PARAMS, "out is NULL");
    if (offset % 4) return fail(DLLM_ERR_INVALID_PARAMS, "offset must be a multiple of 4");
    randn_kernel<<<elem_grid(n), 256, 0, as_stream(stream)>>>(seed, offset, n, out);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_p_sample(const float *x_t, const float *eps, const float *noise, const float *coef, size_t B, size_t D,
                  int add_noise, uint64_t seed, uint64_t offset, float *x_prev, dllm_stream_t stream) {
    const size_t n = B * D;
    if (n == 0) return DLLM_OK;
    if (!x_t || !eps || !coef || !x_prev) return fail(DLLM_ERR_INVALID_PARAMS, "NULL argument");
    if (!noise && offset % 4) return fail(DLLM_ERR_INVALID_PARAMS, "offset must be a multiple of 4");
    if ((reinterpret_cast<uintptr_t>(x_t) | reinterpret_cast<uintptr_t>(eps) | reinterpret_cast<uintptr_t>(x_prev)) % 16)
        return fail(DLLM_ERR_INVALID_PARAMS, "x_t, eps and x_prev must be 16-byte aligned");
    p_sample_kernel<<<elem_grid(n), 256, 0, as_stream(stream)>>>(x_t, eps, noise, coef, n, D, add_noise ? 1 : 0,
                                                                 seed, offset, x_prev);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

int dllm_add_noise(const float *x0, const float *noise, const float *coef, size_t B, size_t D, uint64_t seed,
                   uint64_t offset, float *noisy, float *noise_out, dllm_stream_t stream) {
    const size_t n = B * D;
    if (n == 0) return DLLM_OK;
    if (!x0 || !coef || !noisy) return fail(DLLM_ERR_INVALID_PARAMS, "NULL argument");
    if (!noise && offset % 4) return fail(DLLM_ERR_INVALID_PARAMS, "offset must be a multiple of 4");
    add_noise_kernel<<<elem_grid(n), 256, 0, as_stream(stream)>>>(x0, noise, coef, n, D, seed, offset, noisy,
                                                                  noise_out);
    DLLM_LAUNCH_CHECK();
    return DLLM_OK;
}

}  // extern "C"
