/*
 * dllm_oracle_diffusion.c -- CPU restatement of the reference's diffusion-step elementwise ops
 * (SURVEY.md section 8f rank 1): beta schedules, alpha-bar cumulative products, the p_sample
 * posterior step and the add_noise forward step, plus the build's seeded Gaussian noise.
 *
 * TEST INFRASTRUCTURE ONLY (see dllm_oracle.h).  Rust f32 semantics throughout (-ffp-contract=off).
 *
 * Reference: diffuse-llm-rs/src/lib.rs
 *   create_beta_schedule          :554-593   (PI = std::f32::consts::PI, :20)
 *   p_losses inclusive cumprod    :623-630   (alphas.iter().scan(1.0, |s, &a| {*s *= a; Some(*s)}))
 *   add_noise                     :1100-1137 (exclusive cumprod :1116-1119)
 *   p_sample                      :1152-1215 (exclusive cumprod :1162-1165; full-length `alphas`
 *                                             in mean_coeff2 :1191, an elementwise op only when
 *                                             batch == num_timesteps)
 * The reference draws its noise from rand::thread_rng (unseeded, lib.rs:1108-1110, :1198-1201);
 * the build replaces it by a counter-based generator whose every floating-point step is a
 * correctly rounded IEEE operation (+ - * / sqrt), so this oracle reproduces the device noise
 * bit for bit.
 */
#include "dllm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---- schedules ------------------------------------------------------------------------------ */

int orc_beta_schedule(int kind, size_t T, float beta_start, float beta_end, float *betas) {
    const float PI = 3.14159274101257324f;   /* std::f32::consts::PI */
    for (size_t t = 0; t < T; ++t) {
        float b;
        if (kind == ORC_BETA_LINEAR) {                       /* lib.rs:559-564 */
            b = beta_start + (beta_end - beta_start) * (float)t / (float)(T - 1);
        } else if (kind == ORC_BETA_QUADRATIC) {             /* lib.rs:568-574 */
            const float tn = (float)t / (float)(T - 1);
            b = beta_start + (beta_end - beta_start) * tn * tn;
        } else if (kind == ORC_BETA_COSINE) {                /* lib.rs:578-590 */
            const float s = 0.008f;
            const float tn = (float)t / (float)T;
            float ft = cosf((tn + s) / (1.0f + s) * PI / 2.0f);
            ft = ft * ft;                                    /* powi(2) */
            float f0 = cosf(s / (1.0f + s) * PI / 2.0f);
            f0 = f0 * f0;
            b = fminf(1.0f - ft / f0, 0.999f);               /* f32::min: NaN-ignoring */
        } else {
            return ORC_INVALID_PARAMS;
        }
        betas[t] = b;
    }
    return ORC_OK;
}

int orc_alpha_bars(const float *betas, size_t T, int inclusive, float *alphas, float *alpha_bars) {
    for (size_t i = 0; i < T; ++i) alphas[i] = 1.0f - betas[i];
    if (inclusive) {                                         /* lib.rs:627-630 */
        float state = 1.0f;
        for (size_t i = 0; i < T; ++i) {
            state *= alphas[i];
            alpha_bars[i] = state;
        }
    } else {                                                 /* lib.rs:1116-1119, 1162-1165 */
        if (T > 0) alpha_bars[0] = 1.0f;
        for (size_t i = 1; i < T; ++i) alpha_bars[i] = alpha_bars[i - 1] * alphas[i - 1];
    }
    return ORC_OK;
}

/* lib.rs:1167-1195: per-sample scalars of the posterior step.  coef[i] = {c1, c2, std}. */
int orc_p_sample_coeffs(const float *betas, size_t T, int inclusive, int literal_alphas, const size_t *t, size_t B,
                        float *coef) {
    if (T == 0) return ORC_INVALID_PARAMS;                   /* betas.len() - 1 underflows */
    if (literal_alphas && B != T) return ORC_INVALID_PARAMS; /* ndarray broadcast panics */
    float *alphas = (float *)malloc(T * sizeof(float)), *abar = (float *)malloc(T * sizeof(float));
    if (!alphas || !abar) { free(alphas); free(abar); return ORC_INVALID_PARAMS; }
    orc_alpha_bars(betas, T, inclusive, alphas, abar);
    for (size_t i = 0; i < B; ++i) {
        const size_t ti = t[i] < T - 1 ? t[i] : T - 1;
        const float abar_t = abar[ti], beta_t = betas[ti];
        const float alpha_sel = literal_alphas ? alphas[i] : alphas[ti];
        const float abar_prev = ti > 0 ? abar[ti - 1] : 1.0f;
        const float c1 = (sqrtf(abar_prev) * beta_t) / (1.0f - abar_t);
        const float c2 = (sqrtf(alpha_sel) * (1.0f - abar_prev)) / (1.0f - abar_t);
        const float var = ((1.0f - abar_prev) / (1.0f - abar_t)) * beta_t;
        coef[3 * i + 0] = c1;
        coef[3 * i + 1] = c2;
        coef[3 * i + 2] = sqrtf(var);
    }
    free(alphas);
    free(abar);
    return ORC_OK;
}

/* lib.rs:1112-1133: coef[i] = {sqrt(alpha_bar_t), sqrt(1 - alpha_bar_t)}. */
int orc_add_noise_coeffs(const float *betas, size_t T, int inclusive, const size_t *t, size_t B, float *coef) {
    if (T == 0) return ORC_INVALID_PARAMS;
    float *alphas = (float *)malloc(T * sizeof(float)), *abar = (float *)malloc(T * sizeof(float));
    if (!alphas || !abar) { free(alphas); free(abar); return ORC_INVALID_PARAMS; }
    orc_alpha_bars(betas, T, inclusive, alphas, abar);
    for (size_t i = 0; i < B; ++i) {
        const size_t ti = t[i] < T - 1 ? t[i] : T - 1;
        coef[2 * i + 0] = sqrtf(abar[ti]);
        coef[2 * i + 1] = sqrtf(1.0f - abar[ti]);
    }
    free(alphas);
    free(abar);
    return ORC_OK;
}

/* ---- seeded Gaussian noise (build-defined) -------------------------------------------------
 * Element e of stream (seed, offset): Philox4x32-10 with key (seed lo, seed hi) on counter
 * ((offset + e) / 4 as 64 bits, 0, 0) gives r0..r3; Box-Muller on (r0, r1) -> z0, z1 and on
 * (r2, r3) -> z2, z3; element e takes z_{(offset+e) % 4}.
 *   u1 = ((ra >> 8) + 1) * 2^-24 in (0, 1],  u2 = (rb >> 8) * 2^-24 in [0, 1)
 *   rad = sqrt(-2 ln u1), ln by exponent split + atanh series; angle 2 pi u2 by quadrant and a
 *   Taylor sin/cos on [0, pi/2).  Only + - * / sqrt, each correctly rounded. */
static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

static float ln_exact_ops(float u) {   /* u in (0, 1] */
    uint32_t bits;
    memcpy(&bits, &u, 4);
    int e = (int)((bits >> 23) & 0xff) - 127;
    uint32_t mb = (bits & 0x007fffffu) | 0x3f800000u;
    float m;
    memcpy(&m, &mb, 4);                       /* m in [1, 2) */
    if (m > 0x1.6a09e6p+0f) { m = m * 0.5f; e += 1; }
    const float s = (m - 1.0f) / (m + 1.0f);
    const float s2 = s * s;
    float p = 0x1.3b13b2p-4f;                 /* 1/13 */
    p = 0x1.745d18p-4f + s2 * p;              /* 1/11 */
    p = 0x1.c71c72p-4f + s2 * p;              /* 1/9 */
    p = 0x1.24924ap-3f + s2 * p;              /* 1/7 */
    p = 0x1.99999ap-3f + s2 * p;              /* 1/5 */
    p = 0x1.555556p-2f + s2 * p;              /* 1/3 */
    p = 1.0f + s2 * p;
    const float lnm = (2.0f * s) * p;
    return (float)e * 0x1.62e430p-1f + lnm;   /* e ln 2 + ln m */
}

static void sincos_quarter(float phi, float *sn, float *cs) {   /* phi in [0, pi/2) */
    const float x2 = phi * phi;
    float sp = 1.0f - x2 * 0x1.a41a42p-8f;    /* 1/156 */
    sp = 1.0f - x2 * 0x1.29e412p-7f * sp;     /* 1/110 */
    sp = 1.0f - x2 * 0x1.c71c72p-7f * sp;     /* 1/72 */
    sp = 1.0f - x2 * 0x1.861862p-6f * sp;     /* 1/42 */
    sp = 1.0f - x2 * 0x1.99999ap-5f * sp;     /* 1/20 */
    sp = 1.0f - x2 * 0x1.555556p-3f * sp;     /* 1/6 */
    *sn = phi * sp;
    float cp = 1.0f - x2 * 0x1.f07c20p-8f;    /* 1/132 */
    cp = 1.0f - x2 * 0x1.6c16c2p-7f * cp;     /* 1/90 */
    cp = 1.0f - x2 * 0x1.24924ap-6f * cp;     /* 1/56 */
    cp = 1.0f - x2 * 0x1.111112p-5f * cp;     /* 1/30 */
    cp = 1.0f - x2 * 0x1.555556p-4f * cp;     /* 1/12 */
    cp = 1.0f - x2 * 0.5f * cp;               /* 1/2 */
    *cs = cp;
}

static void box_muller(uint32_t ra, uint32_t rb, float *z0, float *z1) {
    const float u1 = (float)((ra >> 8) + 1u) * 0x1p-24f;
    const float u2 = (float)(rb >> 8) * 0x1p-24f;
    const float rad = sqrtf(-2.0f * ln_exact_ops(u1));
    const float v = u2 * 4.0f;
    const int q = (int)v;
    const float phi = (v - (float)q) * 0x1.921fb6p+0f;   /* pi/2 */
    float sn, cs;
    sincos_quarter(phi, &sn, &cs);
    float c, s;
    switch (q) {
    case 0: c = cs; s = sn; break;
    case 1: c = -sn; s = cs; break;
    case 2: c = -cs; s = -sn; break;
    default: c = sn; s = -cs; break;
    }
    *z0 = rad * c;
    *z1 = rad * s;
}

void orc_randn(uint64_t seed, uint64_t offset, size_t n, float *out) {
    size_t i = 0;
    while (i < n) {
        const uint64_t e = offset + i, blk = e / 4;
        uint32_t c[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0u};
        philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        float z[4];
        box_muller(c[0], c[1], &z[0], &z[1]);
        box_muller(c[2], c[3], &z[2], &z[3]);
        for (unsigned l = (unsigned)(e % 4); l < 4 && i < n; ++l, ++i) out[i] = z[l];
    }
}

/* ---- elementwise steps ----------------------------------------------------------------------- */

/* lib.rs:1188-1212: x_prev = (c1 x_t + c2 eps) + std * noise, per-row scalars, noise = 0 when
 * add_noise == 0 (the reference's t[0] == 0 branch, lib.rs:1198-1204). */
void orc_p_sample(const float *x_t, const float *eps, const float *noise, const float *coef, size_t B, size_t D,
                  int add_noise, float *x_prev) {
    for (size_t r = 0; r < B; ++r) {
        const float c1 = coef[3 * r], c2 = coef[3 * r + 1], sd = coef[3 * r + 2];
        for (size_t j = 0; j < D; ++j) {
            const size_t i = r * D + j;
            const float mean = c1 * x_t[i] + c2 * eps[i];
            const float nz = add_noise ? noise[i] : 0.0f;
            x_prev[i] = mean + sd * nz;
        }
    }
}

/* lib.rs:1130-1135: noisy = x0 * sqrt(abar_t) + noise * sqrt(1 - abar_t). */
void orc_add_noise(const float *x0, const float *noise, const float *coef, size_t B, size_t D, float *noisy) {
    for (size_t r = 0; r < B; ++r) {
        const float sa = coef[2 * r], sb = coef[2 * r + 1];
        for (size_t j = 0; j < D; ++j) {
            const size_t i = r * D + j;
            noisy[i] = x0[i] * sa + noise[i] * sb;
        }
    }
}
