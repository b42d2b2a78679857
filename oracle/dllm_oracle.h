/*
 * dllm_oracle.h -- CPU restatement of zetareticula/diffusion-llm-rs's quantized hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker, never the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product path
 * (diffusion-llm-rs_amd/, libdllm_hip.so) never links or calls anything in this directory.
 *
 * Semantics: every function restates the Rust code it cites with Rust f32 semantics:
 * IEEE binary32, each operation separately rounded (built with -ffp-contract=off), Rust
 * `round` = C roundf (half away from zero), `f32::max/min` = fmaxf/fminf (NaN-ignoring),
 * `f32::clamp` passes NaN through, `f as u8` / `f as i32` saturate with NaN -> 0.
 *
 * Pinning: the reference is Rust and cannot be built here (no cargo/rustc; it also does not
 * compile as shipped), so there is no reference binary to run.  This
 * oracle is pinned by (1) every known-answer assertion in the reference's own #[test]s for
 * this path, replayed in tests/test_oracle_golden.py, and (2) bit-exact agreement with an
 * independent numpy restatement (oracle/oracle_np.py) on the committed golden vectors in
 * tests/golden/.  Beyond those known answers, full-vector parity with the Rust binary is
 * unpinned (documented in DESIGN.md).
 *
 * Error codes mirror quantization/src/error.rs:18-40 discriminant order + 1 (0 = Ok).
 */
#ifndef DLLM_ORACLE_H
#define DLLM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORC_OK = 0,
    ORC_INVALID_PARAMS = 1,        /* QuantizationError::InvalidParams; also reference panics */
    ORC_UNSUPPORTED = 2,
    ORC_SHAPE_MISMATCH = 3,
    ORC_CALIBRATION_REQUIRED = 4,
};

/* a1: diffuse-llm-rs/src/quantization.rs:38-68 quantize_tensor -> (codes, scale, zp as f32). */
int orc_quantize_tensor(const float *x, size_t n, uint8_t bits, uint8_t *codes, float *scale, float *zp);
/* a2: diffuse-llm-rs/src/quantization.rs:81-85 dequantize_tensor. */
void orc_dequantize_tensor(const uint8_t *codes, size_t n, float scale, float zp, float *out);
/* a3: diffuse-llm-rs/src/quantization.rs:120-124 QuantizedTensor::compression_ratio. */
float orc_compression_ratio(size_t numel, size_t len, uint8_t bits);

/* a6 (build-defined): LSB-first bitstream, element i at bit i*bits; ceil(n*bits/8) bytes. */
size_t orc_packed_bytes(size_t n, uint8_t bits);
int orc_pack_bits(const uint8_t *codes, size_t n, uint8_t bits, uint8_t *packed);
int orc_unpack_bits(const uint8_t *packed, size_t n, uint8_t bits, uint8_t *codes);

/* a4: quantization/src/quantize.rs:60-78 QuantizationType, :111-154 DefaultQuantizer quantize,
 *     :172-184 dequantize.  qtype: 0 Int8, 1 Int4, 2 Binary, 3 Float8. */
int orc_qtype_bits(int qtype);
int orc_default_quantize(const float *x, size_t n, int qtype, float scale, int32_t zero_point, uint8_t *out);
void orc_default_dequantize(const uint8_t *q, size_t n, float scale, int32_t zero_point, float *out);

/* a8-ii: prefill-kvquant-rs/lib.rs:39-53 BitQuantizer (truncating). */
int orc_bit_quantize(const float *x, size_t n, uint32_t bits, float scale, float zero_point, uint8_t *out);
void orc_bit_dequantize(const uint8_t *q, size_t n, float scale, float zero_point, float *out);
/* prefill-kvquant-rs/lib.rs:101-110: per configured width, scale = 1/((1<<b)-1), zp = 0. */
int orc_prefill_scale(uint32_t cfg_bits, float *scale);
/* prefill-kvquant-rs/lib.rs:127-146 quantize_vectors over `rows` vectors of `dim` values.
 * cfg_bits[ncfg] = SystemConfig::quantization_bits, req_bits[nreq] cycled per vector.
 * out is rows*dim bytes; out_bits[rows] receives the width recorded in CompressedVector. */
int orc_quantize_vectors(const float *x, size_t rows, size_t dim, const uint8_t *cfg_bits, size_t ncfg,
                         const uint8_t *req_bits, size_t nreq, uint8_t *out, uint8_t *out_bits);

/* a8-iii: diffusion_prefill/src/prefill_kv.rs:104-121 compress_vector / :124-132 decompress. */
int orc_compress_vector(const float *x, size_t n, uint8_t bits, uint8_t *out, float *scale, float *zero_point);

/* a10: quantization/src/calibrate.rs:28-110 CalibrationData. */
typedef struct {
    float min, max;
    size_t num_bins, total_samples;
    uint64_t *histogram; /* caller-owned, num_bins entries */
} orc_calib_t;
void orc_calib_init(orc_calib_t *c, size_t num_bins, uint64_t *hist_storage);
void orc_calib_update(orc_calib_t *c, const float *x, size_t n);
int orc_calib_compute_params(const orc_calib_t *c, uint8_t bits, int symmetric, float *scale, int32_t *zero_point);

/* 8f rank 4: diffuse-llm-rs/src/quantization.rs:178-235 AdaptiveQuantizer (CKMS q = 0 / 1 as
 * exact extremes; minmax = {min, max}, start {+inf, -inf}). */
void orc_adaptive_update(float *minmax, const float *x, size_t n);
int orc_adaptive_params(const float *minmax, int has_samples, uint32_t bits, float *scale, float *zero_point);
int orc_adaptive_quantize(const float *x, size_t n, uint32_t bits, float scale, float zero_point, uint8_t *out);

/* a5 (build-defined composition): per (column n, K-group g) a1 with `bits`, then a2.
 *   W [K][N] f32 row-major (reference layout, diffuse-llm-rs/src/lib.rs:776-777).
 *   codes [K][N] u8, scales [G][N] f32, zps [G][N] u8, G = ceil(K/group). */
int orc_quantize_weights(const float *W, size_t K, size_t N, uint8_t bits, size_t group,
                         uint8_t *codes, float *scales, uint8_t *zps);
void orc_dequantize_weights(const uint8_t *codes, const float *scales, const uint8_t *zps,
                            size_t K, size_t N, size_t group, float *What);
/* diffuse-llm-rs/src/lib.rs:806-813 forward: Y[M][N] = X[M][K] . W[K][N] + b[N] (f32 sgemm).
 * nthreads <= 1: single-threaded (faithful: ndarray dot is single-threaded). */
void orc_linear_forward(const float *X, size_t M, size_t K, const float *W, size_t N, const float *bias,
                        float *Y, int nthreads);

/* a9 (build-defined): per-head bidirectional SDPA, O = softmax(Q K^T / sqrt(D)) V.
 * Q,K,V,O laid out [S][H][D]; computed with f64 accumulation. */
void orc_attention(const float *Q, const float *K, const float *V, size_t S, size_t H, size_t D, float *O,
                   size_t q_rows, int nthreads);

/* ---- 8f rank 1: diffusion-step elementwise ops (dllm_oracle_diffusion.c) ---------------- */
enum { ORC_BETA_LINEAR = 0, ORC_BETA_QUADRATIC = 1, ORC_BETA_COSINE = 2 };
/* DiffusionConfig::create_beta_schedule, diffuse-llm-rs/src/lib.rs:554-593 (T = 0: nothing). */
int orc_beta_schedule(int kind, size_t T, float beta_start, float beta_end, float *betas);
/* alphas = 1 - betas; alpha_bars: inclusive = p_losses scan (lib.rs:627-630), exclusive =
 * add_noise / p_sample loop (lib.rs:1116-1119, 1162-1165). */
int orc_alpha_bars(const float *betas, size_t T, int inclusive, float *alphas, float *alpha_bars);
/* p_sample per-sample scalars (lib.rs:1167-1195), coef[B][3] = {c1, c2, std}; literal_alphas = 1
 * takes the reference's full-length `alphas` row-wise (valid only when B == T). */
int orc_p_sample_coeffs(const float *betas, size_t T, int inclusive, int literal_alphas, const size_t *t, size_t B,
                        float *coef);
/* add_noise per-sample scalars (lib.rs:1121-1133), coef[B][2] = {sqrt(abar_t), sqrt(1 - abar_t)}. */
int orc_add_noise_coeffs(const float *betas, size_t T, int inclusive, const size_t *t, size_t B, float *coef);
/* Build-defined seeded N(0,1) stream (Philox4x32-10 + exact-op Box-Muller), elements
 * offset .. offset + n - 1. */
void orc_randn(uint64_t seed, uint64_t offset, size_t n, float *out);
/* x_prev = (c1 x_t + c2 eps) + std * (add_noise ? noise : 0), rows of D (lib.rs:1188-1212). */
void orc_p_sample(const float *x_t, const float *eps, const float *noise, const float *coef, size_t B, size_t D,
                  int add_noise, float *x_prev);
/* noisy = x0 sqrt(abar) + noise sqrt(1 - abar), rows of D (lib.rs:1130-1135). */
void orc_add_noise(const float *x0, const float *noise, const float *coef, size_t B, size_t D, float *noisy);

#ifdef __cplusplus
}
#endif
#endif
