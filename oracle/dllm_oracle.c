/*
 * dllm_oracle.c -- CPU restatement of the reference's quantized hot path (see dllm_oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline); never linked by the product.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math -fopenmp).
 * Every function cites the reference file:line it restates.
 */
#include "dllm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---- Rust f32 semantics helpers ------------------------------------------------------- */

/* `f as i32` (Rust >= 1.45): saturating, NaN -> 0. */
static inline int32_t rs_as_i32(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT32_MAX;
    if (f <= -2147483648.0f) return INT32_MIN;
    return (int32_t)f;
}
/* `f as u8`: saturating, truncation toward zero, NaN -> 0. */
static inline uint8_t rs_as_u8(float f) {
    if (f != f) return 0;
    if (f <= 0.0f) return 0;
    if (f >= 255.0f) return 255;
    return (uint8_t)f;
}
/* `f as usize` (64-bit). */
static inline size_t rs_as_usize(float f) {
    if (f != f || f <= 0.0f) return 0;
    if (f >= 18446744073709551616.0f) return SIZE_MAX;
    return (size_t)f;
}
/* `f32::clamp(lo, hi)`: NaN passes through (core::f32::clamp). */
static inline float rs_clamp(float x, float lo, float hi) {
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}
/* `i32::clamp`. */
static inline int32_t rs_clamp_i32(int32_t x, int32_t lo, int32_t hi) {
    return x < lo ? lo : (x > hi ? hi : x);
}

/* ---- a1 / a2 / a3: diffuse-llm-rs/src/quantization.rs ---------------------------------- */

/* quantization.rs:38-68 */
int orc_quantize_tensor(const float *x, size_t n, uint8_t bits, uint8_t *codes, float *scale_out, float *zp_out) {
    if (bits < 1 || bits > 8) return ORC_INVALID_PARAMS; /* :39 assert! -> panic */
    float max_val = -INFINITY, min_val = INFINITY;     /* :41-46 folds, NaN-ignoring */
    for (size_t i = 0; i < n; ++i) max_val = fmaxf(max_val, x[i]);
    for (size_t i = 0; i < n; ++i) min_val = fminf(min_val, x[i]);
    const float q_min = 0.0f;                            /* :49 */
    const float q_max = (float)(1u << bits) - 1.0f;      /* :50 */
    float scale = (max_val - min_val) / (q_max - q_min); /* :52 */
    if (scale == 0.0f) scale = 1.0f;                     /* :53 */
    float zpf = q_min - min_val / scale;                 /* :55 */
    uint8_t zp = rs_as_u8(roundf(rs_clamp(zpf, q_min, q_max))); /* :56 clamp, then round */
    const int32_t hi = (int32_t)((1u << bits) - 1u);
    const float zpf32 = (float)zp;
    for (size_t i = 0; i < n; ++i) {                     /* :59-65 */
        float v = x[i] / scale;
        v = v + zpf32;
        codes[i] = (uint8_t)rs_clamp_i32(rs_as_i32(roundf(v)), 0, hi);
    }
    *scale_out = scale;
    *zp_out = zpf32;                                     /* :67 zero_point as f32 */
    return ORC_OK;
}

/* quantization.rs:81-85 */
void orc_dequantize_tensor(const uint8_t *codes, size_t n, float scale, float zp, float *out) {
    for (size_t i = 0; i < n; ++i) {
        float d = (float)codes[i] - zp;
        out[i] = d * scale;
    }
}

/* quantization.rs:120-124 */
float orc_compression_ratio(size_t numel, size_t len, uint8_t bits) {
    size_t original = numel * 4;
    size_t compressed = (len * (size_t)bits + 7) / 8;
    return (float)original / (float)compressed;
}

/* ---- a6: build-defined packing (size contract quantization.rs:122, lib.rs:284-285) -------- */

size_t orc_packed_bytes(size_t n, uint8_t bits) { return (n * (size_t)bits + 7) / 8; }

int orc_pack_bits(const uint8_t *codes, size_t n, uint8_t bits, uint8_t *packed) {
    if (bits < 1 || bits > 8) return ORC_INVALID_PARAMS;
    size_t nb = orc_packed_bytes(n, bits);
    memset(packed, 0, nb);
    const unsigned mask = (1u << bits) - 1u;
    for (size_t i = 0; i < n; ++i) {
        size_t bit = i * bits;
        unsigned v = (unsigned)(codes[i] & mask) << (bit & 7);
        packed[bit >> 3] |= (uint8_t)(v & 0xFF);
        if ((bit & 7) + bits > 8) packed[(bit >> 3) + 1] |= (uint8_t)(v >> 8);
    }
    return ORC_OK;
}

int orc_unpack_bits(const uint8_t *packed, size_t n, uint8_t bits, uint8_t *codes) {
    if (bits < 1 || bits > 8) return ORC_INVALID_PARAMS;
    const unsigned mask = (1u << bits) - 1u;
    for (size_t i = 0; i < n; ++i) {
        size_t bit = i * bits;
        unsigned v = packed[bit >> 3];
        if ((bit & 7) + bits > 8) v |= (unsigned)packed[(bit >> 3) + 1] << 8;
        codes[i] = (uint8_t)((v >> (bit & 7)) & mask);
    }
    return ORC_OK;
}

/* ---- a4: quantization/src/quantize.rs DefaultQuantizer --------------------------------- */

/* quantize.rs:69-78 */
int orc_qtype_bits(int qtype) {
    switch (qtype) {
    case 0: return 8; case 1: return 4; case 2: return 1; case 3: return 8;
    default: return -1;
    }
}

/* quantize.rs:127-154 with quantize_value :111-124 (T = f32; result stored `q as u8`, :150). */
int orc_default_quantize(const float *x, size_t n, int qtype, float scale, int32_t zero_point, uint8_t *out) {
    float lo, hi;
    switch (qtype) { /* :139-144 */
    case 0: lo = -128.0f; hi = 127.0f; break;
    case 1: lo = -8.0f; hi = 7.0f; break;
    case 2: lo = 0.0f; hi = 1.0f; break;
    case 3: lo = -127.0f; hi = 127.0f; break;
    default: return ORC_UNSUPPORTED;
    }
    const float zp = (float)zero_point; /* :136 */
    for (size_t i = 0; i < n; ++i) {
        float v = x[i] / scale;
        v = v + zp;
        v = fminf(fmaxf(v, lo), hi); /* .max(min).min(max): NaN -> min */
        out[i] = rs_as_u8(roundf(v));
    }
    return ORC_OK;
}

/* quantize.rs:172-184 (also types.rs:71-81) */
void orc_default_dequantize(const uint8_t *q, size_t n, float scale, int32_t zero_point, float *out) {
    const float zp = (float)zero_point;
    for (size_t i = 0; i < n; ++i) {
        float d = (float)q[i] - zp;
        out[i] = d * scale;
    }
}

/* ---- a8-ii: prefill-kvquant-rs/lib.rs BitQuantizer ------------------------------------- */

/* lib.rs:40-46.  `(1 << bits) - 1` is i32 arithmetic; bits > 30 overflows (panic in debug). */
int orc_bit_quantize(const float *x, size_t n, uint32_t bits, float scale, float zero_point, uint8_t *out) {
    if (bits > 30) return ORC_INVALID_PARAMS;
    const float max_val = (float)((1 << bits) - 1);
    for (size_t i = 0; i < n; ++i) {
        float s = (x[i] - zero_point) / scale;
        out[i] = rs_as_u8(rs_clamp(s, 0.0f, max_val));
    }
    return ORC_OK;
}

/* lib.rs:48-52 */
void orc_bit_dequantize(const uint8_t *q, size_t n, float scale, float zero_point, float *out) {
    for (size_t i = 0; i < n; ++i) {
        float p = (float)q[i] * scale;
        out[i] = p + zero_point;
    }
}

/* lib.rs:104-108: scale = 1.0 / ((1 << bits) - 1) as f32 */
int orc_prefill_scale(uint32_t cfg_bits, float *scale) {
    if (cfg_bits > 30) return ORC_INVALID_PARAMS;
    *scale = 1.0f / (float)((1 << cfg_bits) - 1);
    return ORC_OK;
}

/* lib.rs:127-146 */
int orc_quantize_vectors(const float *x, size_t rows, size_t dim, const uint8_t *cfg_bits, size_t ncfg,
                         const uint8_t *req_bits, size_t nreq, uint8_t *out, uint8_t *out_bits) {
    if (nreq == 0) return ORC_OK; /* zip with cycle() of an empty slice yields nothing */
    for (size_t r = 0; r < rows; ++r) {
        uint8_t b = req_bits[r % nreq];             /* :132 bits.iter().cycle() */
        size_t qi = (size_t)b / 2;                   /* :133 quantizers[bits / 2] */
        if (qi >= ncfg) return ORC_INVALID_PARAMS;   /* out-of-bounds index -> panic */
        float scale;
        if (orc_prefill_scale(cfg_bits[qi], &scale)) return ORC_INVALID_PARAMS;
        if (orc_bit_quantize(x + r * dim, dim, b, scale, 0.0f, out + r * dim)) return ORC_INVALID_PARAMS;
        out_bits[r] = b;                             /* :140 bits: bit_precision */
    }
    return ORC_OK;
}

/* ---- a8-iii: diffusion_prefill/src/prefill_kv.rs compress_vector ----------------------- */

/* prefill_kv.rs:104-121 (quantizer :53-60 uses u32 max) */
int orc_compress_vector(const float *x, size_t n, uint8_t bits, uint8_t *out, float *scale_out, float *zp_out) {
    if (bits > 31) return ORC_INVALID_PARAMS;
    float min_val = INFINITY, max_val = -INFINITY;
    for (size_t i = 0; i < n; ++i) min_val = fminf(min_val, x[i]);
    for (size_t i = 0; i < n; ++i) max_val = fmaxf(max_val, x[i]);
    const float levels = (float)((1u << bits) - 1u);
    const float scale = (max_val - min_val) / levels;
    const float zp = min_val;
    for (size_t i = 0; i < n; ++i) {
        float s = (x[i] - zp) / scale;
        out[i] = rs_as_u8(rs_clamp(s, 0.0f, levels));
    }
    *scale_out = scale;
    *zp_out = zp;
    return ORC_OK;
}

/* ---- a10: quantization/src/calibrate.rs ----------------------------------------------- */

/* calibrate.rs:30-39 */
void orc_calib_init(orc_calib_t *c, size_t num_bins, uint64_t *hist) {
    c->min = 3.40282347e+38f;   /* f32::MAX */
    c->max = -3.40282347e+38f;  /* f32::MIN */
    c->num_bins = num_bins;
    c->total_samples = 0;
    c->histogram = hist;
    if (hist) memset(hist, 0, num_bins * sizeof(uint64_t));
}

/* calibrate.rs:42-69 (per-channel stats are host bookkeeping, not restated) */
void orc_calib_update(orc_calib_t *c, const float *x, size_t n) {
    float mn = 3.40282347e+38f, mx = -3.40282347e+38f;
    for (size_t i = 0; i < n; ++i) { mn = fminf(mn, x[i]); mx = fmaxf(mx, x[i]); }
    c->min = fminf(c->min, mn);
    c->max = fmaxf(c->max, mx);
    c->total_samples += n;
    if (c->max > c->min && c->num_bins > 0) {
        const float bin_width = (c->max - c->min) / (float)c->num_bins;
        for (size_t i = 0; i < n; ++i) {
            float v = x[i];
            if (v >= c->min && v <= c->max) {
                size_t bin = rs_as_usize(floorf((v - c->min) / bin_width));
                if (bin > c->num_bins - 1) bin = c->num_bins - 1;
                c->histogram[bin] += 1;
            }
        }
    }
}

/* calibrate.rs:72-110 */
int orc_calib_compute_params(const orc_calib_t *c, uint8_t bits, int symmetric, float *scale, int32_t *zero_point) {
    if (c->total_samples == 0) return ORC_CALIBRATION_REQUIRED;
    if (bits > 31) return ORC_INVALID_PARAMS; /* 2u32.pow(32) overflows -> panic */
    const float num_levels = (float)(1u << bits);
    const float range = c->max - c->min;
    if (range <= 1.1920929e-07f) { *scale = 1.0f; *zero_point = 0; return ORC_OK; }
    float s;
    if (symmetric) {
        float max_abs = fmaxf(fabsf(c->max), fabsf(c->min));
        s = max_abs * 2.0f;
        s = s / (num_levels - 1.0f);
        *zero_point = rs_as_i32(num_levels / 2.0f - 1.0f);
    } else {
        s = range / (num_levels - 1.0f);
        float m = -c->min;
        *zero_point = rs_as_i32(roundf(m / s));
    }
    *scale = s;
    return ORC_OK;
}

/* ---- 8f rank 4: AdaptiveQuantizer (diffuse-llm-rs/src/quantization.rs:178-235) ----------- */
/* The statistics are a quantiles-0.7 CKMS<f32>(0.01) (third-party, absent) queried only at
 * q = 0.0 and q = 1.0 (:209-210).  Restated as the exact extremes of the inserted samples: rank
 * error 0, inside CKMS's eps*n guarantee; NaN samples are skipped.  Parity unpinned beyond the
 * reference's property test (:267-277). */
void orc_adaptive_update(float *minmax, const float *x, size_t n) {
    for (size_t i = 0; i < n; ++i) { minmax[0] = fminf(minmax[0], x[i]); minmax[1] = fmaxf(minmax[1], x[i]); }
}

/* :206-217 compute_params: query(..).unwrap_or(0.0 / 1.0) when no sample was inserted;
 * scale = (max - min) / q_max (no zero guard); zp = round(-min / scale).clamp(0, q_max)
 * (round, THEN clamp; NaN passes). */
int orc_adaptive_params(const float *minmax, int has_samples, uint32_t bits, float *scale, float *zero_point) {
    if (bits > 31) return ORC_INVALID_PARAMS;          /* 1u32 << bits overflows -> panic */
    const float mn = has_samples ? minmax[0] : 0.0f;
    const float mx = has_samples ? minmax[1] : 1.0f;
    const float q_max = (float)(1u << bits) - 1.0f;     /* :212 */
    const float s = (mx - mn) / q_max;                  /* :213 */
    const float m = -mn;
    *scale = s;
    *zero_point = rs_clamp(roundf(m / s), 0.0f, q_max); /* :214 */
    return ORC_OK;
}

/* :220-234 quantize: ((x / scale) + zp).round() as i32, .clamp(0, q_max as i32) as u8 -- the
 * `as u8` of an i32 keeps the low byte, which matters only for bits > 8. */
int orc_adaptive_quantize(const float *x, size_t n, uint32_t bits, float scale, float zero_point, uint8_t *out) {
    if (bits > 31) return ORC_INVALID_PARAMS;
    const int32_t hi = rs_as_i32((float)(1u << bits) - 1.0f);
    for (size_t i = 0; i < n; ++i) {
        const float t = x[i] / scale;
        const float u = t + zero_point;
        out[i] = (uint8_t)(rs_clamp_i32(rs_as_i32(roundf(u)), 0, hi) & 0xff);
    }
    return ORC_OK;
}

/* ---- a5: group-wise composition + linear layer ----------------------------------------- */

int orc_quantize_weights(const float *W, size_t K, size_t N, uint8_t bits, size_t group,
                         uint8_t *codes, float *scales, uint8_t *zps) {
    if (bits < 1 || bits > 8 || group == 0) return ORC_INVALID_PARAMS;
    const size_t G = (K + group - 1) / group;
    float *col = (float *)malloc(group * sizeof(float));
    uint8_t *cq = (uint8_t *)malloc(group);
    if (!col || !cq) { free(col); free(cq); return ORC_INVALID_PARAMS; }
    for (size_t g = 0; g < G; ++g) {
        size_t k0 = g * group, len = (K - k0 < group) ? K - k0 : group;
        for (size_t n = 0; n < N; ++n) {
            for (size_t k = 0; k < len; ++k) col[k] = W[(k0 + k) * N + n];
            float s, z;
            orc_quantize_tensor(col, len, bits, cq, &s, &z);
            for (size_t k = 0; k < len; ++k) codes[(k0 + k) * N + n] = cq[k];
            scales[g * N + n] = s;
            zps[g * N + n] = (uint8_t)z;
        }
    }
    free(col);
    free(cq);
    return ORC_OK;
}

void orc_dequantize_weights(const uint8_t *codes, const float *scales, const uint8_t *zps,
                            size_t K, size_t N, size_t group, float *What) {
    for (size_t k = 0; k < K; ++k) {
        size_t g = k / group;
        for (size_t n = 0; n < N; ++n) {
            float d = (float)codes[k * N + n] - (float)zps[g * N + n];
            What[k * N + n] = d * scales[g * N + n];
        }
    }
}

/* diffuse-llm-rs/src/lib.rs:806-813: x.dot(&self.weights) + &self.bias.
 * i-k-j order with a K-blocked inner panel so the N-row of W stays in cache. */
void orc_linear_forward(const float *X, size_t M, size_t K, const float *W, size_t N, const float *bias,
                        float *Y, int nthreads) {
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (size_t m = 0; m < M; ++m) {
        float *y = Y + m * N;
        for (size_t n = 0; n < N; ++n) y[n] = 0.0f;
        const float *x = X + m * K;
        for (size_t k = 0; k < K; ++k) {
            const float a = x[k];
            const float *w = W + k * N;
            for (size_t n = 0; n < N; ++n) y[n] += a * w[n];
        }
        if (bias)
            for (size_t n = 0; n < N; ++n) y[n] += bias[n];
    }
}

/* ---- a9: build-defined attention consumer (lib.rs:910-915 hands K,V to the model) ------ */

void orc_attention(const float *Q, const float *K, const float *V, size_t S, size_t H, size_t D, float *O,
                   size_t q_rows, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (q_rows > S) q_rows = S;
    const double inv = 1.0 / sqrt((double)D);
#pragma omp parallel num_threads(nthreads)
    {
        double *p = (double *)malloc(S * sizeof(double));
        double *acc = (double *)malloc(D * sizeof(double));
#pragma omp for collapse(2) schedule(static)
        for (size_t h = 0; h < H; ++h) {
            for (size_t i = 0; i < q_rows; ++i) {
                const float *q = Q + (i * H + h) * D;
                double mx = -INFINITY;
                for (size_t j = 0; j < S; ++j) {
                    const float *k = K + (j * H + h) * D;
                    double s = 0.0;
                    for (size_t d = 0; d < D; ++d) s += (double)q[d] * (double)k[d];
                    p[j] = s * inv;
                    if (p[j] > mx) mx = p[j];
                }
                double l = 0.0;
                for (size_t j = 0; j < S; ++j) { p[j] = exp(p[j] - mx); l += p[j]; }
                for (size_t d = 0; d < D; ++d) acc[d] = 0.0;
                for (size_t j = 0; j < S; ++j) {
                    const float *v = V + (j * H + h) * D;
                    for (size_t d = 0; d < D; ++d) acc[d] += p[j] * (double)v[d];
                }
                float *o = O + (i * H + h) * D;
                for (size_t d = 0; d < D; ++d) o[d] = (float)(acc[d] / l);
            }
        }
        free(p);
        free(acc);
    }
}
