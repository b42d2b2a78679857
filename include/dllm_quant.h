/*
 * dllm_quant.h -- C-ABI drop-in boundary for diffusion-llm-rs's quantized inference hot path,
 * implemented by hand-written HIP kernels for MI355X (gfx950) in libdllm_hip.so.
 *
 * The reference (zetareticula/diffusion-llm-rs, Rust, CPU-only) has no FFI: its operator surface
 * is three in-process Rust APIs.  Each entry point below names the Rust
 * item it replaces (paths relative to the reference root).  Conventions:
 *   - return int status: 0 = Ok; 1..7 = quantization::QuantizationError discriminant order + 1
 *     (quantization/src/error.rs:18-40); reference panics (assert!, out-of-bounds index) map to
 *     DLLM_ERR_INVALID_PARAMS; 16+ = HIP / runtime errors.  dllm_last_error() gives a message.
 *   - plain pointers and sizes only.  Unless a name ends in _host, every data pointer is DEVICE
 *     memory and the call is asynchronous on `stream` (a hipStream_t; NULL = default stream);
 *     nothing is synchronised inside and, after a first call of the same shape, nothing is
 *     allocated (graph-capturable; see dllm_linear_forward).  The *_host variants take
 *     host pointers, stage through device memory and synchronise (parity/test convenience).
 *   - quantized codes are either one code per byte ("unpacked", the reference's storage,
 *     diffuse-llm-rs/src/quantization.rs:59-65) or the packed LSB-first bitstream below.
 *   - handles (dllm_linear_t) own device memory, are immutable after create and may be used
 *     from several threads on distinct
 *     streams (the reference's Send + Sync model bound).
 *
 * Packed layout (build-defined; the reference only assumes its size, quantization.rs:122):
 *   element i of an n-element, b-bit tensor occupies bits [i*b, (i+1)*b) of a little-endian
 *   bitstream, i.e. byte (i*b)/8 from bit (i*b)%8 upward (spilling into the next byte when
 *   b does not divide 8); total ceil(n*b/8) bytes; unused high bits of the last byte are 0.
 */
#ifndef DLLM_QUANT_H
#define DLLM_QUANT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *dllm_stream_t; /* hipStream_t */

enum dllm_status {
    DLLM_OK = 0,
    DLLM_ERR_INVALID_PARAMS = 1,        /* QuantizationError::InvalidParams + reference panics */
    DLLM_ERR_UNSUPPORTED = 2,           /* QuantizationError::UnsupportedOperation */
    DLLM_ERR_SHAPE_MISMATCH = 3,        /* QuantizationError::ShapeMismatch */
    DLLM_ERR_CALIBRATION_REQUIRED = 4,  /* QuantizationError::CalibrationRequired */
    DLLM_ERR_IO = 5,                    /* QuantizationError::Io */
    DLLM_ERR_SERIALIZATION = 6,         /* QuantizationError::Serialization */
    DLLM_ERR_INVALID_DATA_FORMAT = 7,   /* QuantizationError::InvalidDataFormat */
    DLLM_ERR_HIP = 16,                  /* a HIP runtime call failed */
    DLLM_ERR_NO_DEVICE = 17,            /* no gfx950 device visible */
};

enum dllm_dtype { DLLM_F32 = 0, DLLM_F16 = 1 };

/* quantization/src/quantize.rs:62-67 QuantizationType */
enum dllm_qtype { DLLM_QT_INT8 = 0, DLLM_QT_INT4 = 1, DLLM_QT_BINARY = 2, DLLM_QT_FLOAT8 = 3 };

/* ---- library ---------------------------------------------------------------------------- */
const char *dllm_last_error(void);  /* thread-local message of the last failing call */
const char *dllm_version(void);
int dllm_device_arch(int device, char *buf, size_t len); /* gcnArchName, e.g. "gfx950:sramecc+:xnack-" */

/* ---- a1 / a2: diffuse-llm-rs/src/quantization.rs --------------------------------------- */

/* Bytes of device workspace dllm_quantize_tensor needs for n elements. */
size_t dllm_quantize_tensor_workspace(size_t n);

/* quantize_tensor(data: &[f32], bits: u8) -> (Vec<u8>, f32, f32)   (quantization.rs:38-68)
 * Per-tensor asymmetric quantization: global min/max, scale = (max-min)/(2^bits-1) (1.0 if 0),
 * zp = round(clamp(0 - min/scale, 0, 2^bits-1)) as u8, q = clamp(round(x/scale + zp), 0, 2^bits-1).
 * x[n] f32; out: n bytes (packed=0) or ceil(n*bits/8) bytes (packed=1);
 * params_out[2] = {scale, zero_point as f32} written on the device (no host sync).
 * bits outside 1..=8 -> DLLM_ERR_INVALID_PARAMS (the reference's assert!, quantization.rs:39). */
int dllm_quantize_tensor(const float *x, size_t n, uint8_t bits, int packed, uint8_t *out, float *params_out,
                         void *workspace, size_t workspace_bytes, dllm_stream_t stream);

/* quantize_tensor of the SAME data at two widths, as KVCacheEntry::update does for its prefill and
 * decode copies (diffuse-llm-rs/src/lib.rs:241-276, QuantizedKVCacheEntry::new at each width,
 * quantization.rs:140-157): one min/max pass (the extremes do not depend on the width) and one read
 * of x that writes both code sets.  Outputs are bit-identical to two dllm_quantize_tensor calls.
 * Workspace: dllm_quantize_tensor_workspace(n).  bits_a, bits_b in 1..=8. */
int dllm_quantize_tensor_pair(const float *x, size_t n, uint8_t bits_a, uint8_t bits_b, int packed, uint8_t *out_a,
                              float *params_a, uint8_t *out_b, float *params_b, void *workspace,
                              size_t workspace_bytes, dllm_stream_t stream);

/* quantize_tensor split at its one reduction, for a tensor sharded over ranks (the KV
 * cache sharded by head needs the per-tensor scale of quantization.rs:41-56 over ALL shards).
 * The extremes fold (:41-46, NaN-ignoring) is order-independent, so each rank folds its shard into
 * stats[2] = {min, max} (device, seeded {+inf, -inf} by the caller), the ranks combine them with one
 * all-reduce (max over {-min, max}), and each rank then writes the params (:49-56) and codes
 * (:59-65) that dllm_quantize_tensor of the whole tensor writes for its elements, bit for bit.
 * Workspace: dllm_quantize_tensor_workspace(n).  bits outside 1..=8 -> INVALID_PARAMS. */
int dllm_tensor_extremes(const float *x, size_t n, float *stats, void *workspace, size_t workspace_bytes,
                         dllm_stream_t stream);
int dllm_quantize_params_from_extremes(const float *stats, uint8_t bits, float *params, dllm_stream_t stream);
int dllm_quantize_tensor_with_params(const float *x, size_t n, uint8_t bits, int packed, const float *params,
                                     uint8_t *out, dllm_stream_t stream);
/* The same at two widths in one read of x (KVCacheEntry::update's prefill and decode copies of a
 * head shard, diffuse-llm-rs/src/lib.rs:246-276); == two dllm_quantize_tensor_with_params calls. */
int dllm_quantize_tensor_pair_with_params(const float *x, size_t n, uint8_t bits_a, uint8_t bits_b, int packed,
                                          const float *params_a, const float *params_b, uint8_t *out_a,
                                          uint8_t *out_b, dllm_stream_t stream);

/* ---- a3 / a8-i: both tensors of one KV-cache quantization ----------------------------------
 * QuantizedKVCacheEntry::new(keys, values, bits) (quantization.rs:140-157: K and V each quantized
 * per tensor by quantize_tensor) and, with bits_b != 0, KVCacheEntry::update's prefill and decode
 * copies of the same K/V (diffuse-llm-rs/src/lib.rs:241-276): outputs bit-identical to
 * dllm_quantize_tensor[_pair] of k and of v (each tensor: one min/max pass, one map pass that
 * writes both widths).  bits_b = 0: one width (the *_b pointers unused).  Workspace:
 * dllm_quantize_kv_workspace(n_k, n_v). */
size_t dllm_quantize_kv_workspace(size_t n_k, size_t n_v);
int dllm_quantize_kv(const float *k, size_t n_k, const float *v, size_t n_v, uint8_t bits_a, uint8_t bits_b,
                     int packed, uint8_t *k_a, float *kp_a, uint8_t *v_a, float *vp_a, uint8_t *k_b, float *kp_b,
                     uint8_t *v_b, float *vp_b, void *workspace, size_t workspace_bytes, dllm_stream_t stream);
/* The same split at its reduction for a head-sharded cache: red[4] = {-min_K, max_K,
 * -min_V, max_V} of this rank's shards (NaN-ignoring, quantization.rs:41-46; one launch over both
 * tensors plus a fold), to be combined over the ranks by one all_reduce(MAX); then both tensors'
 * params (:49-56) and codes (:59-65) at one or two widths in one launch.  Workspace as above. */
int dllm_kv_extremes(const float *k, size_t n_k, const float *v, size_t n_v, float *red, void *workspace,
                     size_t workspace_bytes, dllm_stream_t stream);
int dllm_quantize_kv_with_extremes(const float *k, size_t n_k, const float *v, size_t n_v, const float *red,
                                   uint8_t bits_a, uint8_t bits_b, int packed, uint8_t *k_a, float *kp_a,
                                   uint8_t *v_a, float *vp_a, uint8_t *k_b, float *kp_b, uint8_t *v_b, float *vp_b,
                                   dllm_stream_t stream);

/* dequantize_tensor(data: &[u8], scale: f32, zero_point: f32) -> Vec<f32> (quantization.rs:81-85)
 * and QuantizedTensor::dequantize (:115-117):  y = ((q as f32) - zp) * scale.
 * params[2] = {scale, zp} in DEVICE memory (as written by dllm_quantize_tensor).
 * out_dtype DLLM_F32 gives the reference's f32 bits exactly; DLLM_F16 = that f32 rounded (RNE). */
int dllm_dequantize_tensor(const uint8_t *q, size_t n, uint8_t bits, int packed, const float *params,
                           void *out, int out_dtype, dllm_stream_t stream);
/* Same with host scalars (dequantize_tensor's literal signature). */
int dllm_dequantize_tensor_scalar(const uint8_t *q, size_t n, uint8_t bits, int packed, float scale, float zp,
                                  void *out, int out_dtype, dllm_stream_t stream);

/* QuantizedTensor::compression_ratio (quantization.rs:120-124); host-only arithmetic. */
float dllm_compression_ratio(size_t numel, size_t len, uint8_t bits);

/* ---- a6: pack / unpack (build-defined layout above) -------------------------------------- */
size_t dllm_packed_bytes(size_t n, uint8_t bits);
int dllm_pack(const uint8_t *codes, size_t n, uint8_t bits, uint8_t *packed, dllm_stream_t stream);
int dllm_unpack(const uint8_t *packed, size_t n, uint8_t bits, uint8_t *codes, dllm_stream_t stream);

/* ---- a4: quantization crate DefaultQuantizer ---------------------------------------------
 * trait Quantizer::quantize / dequantize (quantization/src/quantize.rs:81-90) as implemented by
 * DefaultQuantizer (:98-184) and quant_utils::{quantize, dequantize} (:191-215):
 *   q = (round(min(max(x/scale + zp, lo), hi)) as u8), (lo,hi) by qtype (:139-144);
 *   y = (q as f32 - zp) * scale.  One code per byte (the reference's QuantizedTensor::data). */
int dllm_default_quantize(const float *x, size_t n, int qtype, float scale, int32_t zero_point, uint8_t *out,
                          dllm_stream_t stream);
int dllm_default_dequantize(const uint8_t *q, size_t n, float scale, int32_t zero_point, float *out,
                            dllm_stream_t stream);

/* ---- a10: calibration (quantization/src/calibrate.rs:42-110) ------------------------------
 * Device-side CalibrationData::update reduction: stats[2] = {min, max} folded into the running
 * values (initialise to {f32::MAX, f32::MIN}), histogram[num_bins] (u64) accumulated for the
 * updated range exactly as calibrate.rs:58-68.  compute_params is host arithmetic. */
int dllm_calib_update(const float *x, size_t n, float *stats, uint64_t *histogram, size_t num_bins,
                      void *workspace, size_t workspace_bytes, dllm_stream_t stream);
int dllm_calib_compute_params(float min, float max, size_t total_samples, uint8_t bits, int symmetric,
                              float *scale, int32_t *zero_point);

/* ---- 8f rank 4: AdaptiveQuantizer (diffuse-llm-rs/src/quantization.rs:178-235) -------------
 * Replaces AdaptiveQuantizer::{update_stats, compute_params, quantize} (:198-234).
 * stats[2] DEVICE {min, max}, initialised by the caller to {+inf, -inf}.  The reference's
 * statistics are a quantiles-0.7 CKMS<f32>(0.01) queried only at q = 0.0 and q = 1.0 (:209-210);
 * update folds x into the exact extremes instead (rank error 0, inside CKMS's eps*n bound; NaN
 * skipped; parity unpinned: the crate is absent).  Workspace: dllm_quantize_tensor_workspace(n).
 * compute_params writes params[2] = {scale, zero_point} on the device:
 *   min, max = stats, or the unwrap_or defaults 0.0 / 1.0 when has_samples == 0;
 *   scale = (max - min) / (2^bits - 1) (no zero guard); zp = round(-min / scale).clamp(0, q_max).
 * quantize: q = (round(x / scale + zp) as i32).clamp(0, q_max as i32) as u8 (the low byte when
 * bits > 8).  packed = 1 needs 1 <= bits <= 8; unpacked accepts 0..=31; bits > 31 -> INVALID_PARAMS
 * (1u32 << bits overflows). */
int dllm_adaptive_update(const float *x, size_t n, float *stats, void *workspace, size_t workspace_bytes,
                         dllm_stream_t stream);
int dllm_adaptive_compute_params(const float *stats, int has_samples, uint32_t bits, float *params,
                                 dllm_stream_t stream);
int dllm_adaptive_quantize(const float *x, size_t n, uint32_t bits, const float *params, int packed, uint8_t *out,
                           dllm_stream_t stream);

/* ---- a8-ii: prefill-kvquant-rs kvquant::BitQuantizer (prefill-kvquant-rs/lib.rs:29-53) ------
 * quantize: q = ((x - zp) / scale).clamp(0, (1<<bits)-1) as u8  (truncation, no rounding);
 * dequantize: y = q as f32 * scale + zp.  bits > 30 -> INVALID_PARAMS (i32 shift overflow). */
int dllm_bit_quantize(const float *x, size_t n, uint32_t bits, float scale, float zero_point, uint8_t *out,
                      dllm_stream_t stream);
int dllm_bit_dequantize(const uint8_t *q, size_t n, float scale, float zero_point, void *out, int out_dtype,
                        dllm_stream_t stream);

/* PrefillKVQuant::quantize_vectors (prefill-kvquant-rs/lib.rs:127-146) over `rows` token vectors of
 * `dim` values: row r uses bits req_bits[r % nreq] and quantizers[bits/2] built by
 * PrefillKVQuant::new from cfg_bits (:101-110).  cfg_bits/req_bits are HOST arrays (the config);
 * x/out DEVICE.  out_bits[rows] (host) receives CompressedVector::bits.  bits/2 >= ncfg -> the
 * reference panics -> INVALID_PARAMS, nothing launched. */
int dllm_quantize_vectors(const float *x, size_t rows, size_t dim, const uint8_t *cfg_bits, size_t ncfg,
                          const uint8_t *req_bits, size_t nreq, uint8_t *out, uint8_t *out_bits,
                          dllm_stream_t stream);

/* ---- a8-iii: diffusion_prefill KVCache::compress_vector / decompress_vector -----------------
 * (diffusion_prefill/src/prefill_kv.rs:104-132), batched over rows: per row min/max,
 * scale = (max-min)/(2^bits-1), zp = min, BitQuantizer.  scales/zps [rows] device. */
int dllm_compress_vectors(const float *x, size_t rows, size_t dim, uint8_t bits, uint8_t *out, float *scales,
                          float *zps, dllm_stream_t stream);
int dllm_decompress_vectors(const uint8_t *q, size_t rows, size_t dim, const float *scales, const float *zps,
                            float *out, dllm_stream_t stream);

/* ---- a5: group-quantized linear layer ---------------------------------------------------
 * Replaces SimpleDiffusionModel::forward = x.dot(W) + b (diffuse-llm-rs/src/lib.rs:806-813),
 * W [K, N] ("[input_dim, output_dim]", :776-777), with W quantized per (output column n, K-group g
 * of `group` rows) by quantize_tensor (a1, bits in {2,4,8}) and dequantized by a2 inside the
 * GEMM.  group = QuantizationConfig::default().group_size = 128 (quantization/src/types.rs:124-127).
 * Device compute: X in f16, f16 MFMA with f32 accumulation, bias in f32; the dequantized weight
 * (q - zp) * scale of a2 reaches the MFMA in one of two precisions:
 *   DLLM_PRECISION_EXACT (default): the MFMA operand is the exact integer (q - zp) and the f32
 *     scale multiplies each group's f32 partial sum, so the weight is the reference's f32 a2 value;
 *     the only operand rounding is X's (f16).  Needs group in {64, 128, 256} and K % group == 0
 *     (other shapes use the F16W arithmetic).
 *   DLLM_PRECISION_F16W: the weight is rounded to f16 (f16((q - zp) * f16(scale))) before the MFMA;
 *     ~2.7e-4 more relative error per layer (and no faster: EXACT's Horner kernel is the faster one
 *     at M >= 4096).
 * Requirements: K % 64 == 0, group % 64 == 0; any M >= 0, any N >= 1. */
typedef struct dllm_linear *dllm_linear_t;
enum dllm_precision { DLLM_PRECISION_EXACT = 0, DLLM_PRECISION_F16W = 1 };
/* Flag OR'ed into the `precision` argument of the *_create_ex calls: a prefill-only handle builds no
 * decode layout (the 16x16x32 code image the M <= 64 kernels read): 9.02 MiB instead of 17.02 MiB at
 * 4096 x 4096 int4 g128, the canonical codes' footprint.  Its M <= 64 calls run the prefill kernels
 * (same precision and bound, slower at those M). */
enum dllm_linear_flags { DLLM_LINEAR_PREFILL_ONLY = 0x100 };

/* W (device, f32 [K][N] row-major), bias (device f32 [N] or NULL = zeros, the reference's
 * Array1::zeros, lib.rs:798).  Quantization runs on the GPU (bit-exact with a1).  Precision
 * DLLM_PRECISION_EXACT.  Create builds everything a forward reads -- the prefill and (unless
 * DLLM_LINEAR_PREFILL_ONLY) decode code layouts, the per-(group, column) parameters and, for int4
 * g128 EXACT handles with N % 256 == 0, the Horner-form ratios s_{g-1}/s_g with the check that the
 * scales allow that form -- in temporaries of its own, and synchronises `stream` once before it
 * returns (it is not capturable).  The handle is immutable afterwards and its forwards keep their
 * scratch per (device, stream): one handle may serve several threads on distinct streams. */
int dllm_linear_create(const float *W, const float *bias, size_t K, size_t N, uint8_t bits, size_t group,
                       dllm_linear_t *out, dllm_stream_t stream);
int dllm_linear_create_ex(const float *W, const float *bias, size_t K, size_t N, uint8_t bits, size_t group,
                          int precision, dllm_linear_t *out, dllm_stream_t stream);
/* Import already-quantized weights: codes packed in the canonical bitstream of the [K][N]
 * row-major code matrix, scales f32 [G][N], zps u8 [G][N] (G = ceil(K/group)); all device. */
int dllm_linear_create_quantized(const uint8_t *packed_codes, const float *scales, const uint8_t *zps,
                                 const float *bias, size_t K, size_t N, uint8_t bits, size_t group,
                                 dllm_linear_t *out, dllm_stream_t stream);
int dllm_linear_create_quantized_ex(const uint8_t *packed_codes, const float *scales, const uint8_t *zps,
                                    const float *bias, size_t K, size_t N, uint8_t bits, size_t group,
                                    int precision, dllm_linear_t *out, dllm_stream_t stream);
/* Y[M][N] = X[M][K] . W^ + b.  x_dtype/y_dtype in {DLLM_F32, DLLM_F16}; an f32 X is cast to f16
 * through a per-(device, stream) staging workspace.  Shapes with too few output tiles to fill the GPU
 * (M roughly 65..1000 at N = 4096) split K into slices whose f32 partials are combined in slice
 * order (deterministic) through a per-(device, stream) workspace.  Both workspaces only grow and
 * are allocated on the first call that needs them, which therefore must precede stream capture.
 * A workspace a capture has used is never freed: when a later, larger call on the same stream grows
 * it, the captured buffer is retired (kept for the process lifetime), so an earlier graph still
 * replays on valid memory.  Otherwise the call only launches kernels on `stream`: it never synchronises, and the kernel a
 * shape runs (hence its result bits) does not depend on call history or on capture.
 * DLLM_PRECISION_EXACT, int4 g128, on grids of >= 256 tiles of 256 x 256 (M >= 4096 at N = 4096)
 * runs the Horner-form kernel when the handle's create accepted its ratios, else the fold form
 * (same bound, different f32 summation order). */
int dllm_linear_forward(dllm_linear_t h, const void *X, size_t M, int x_dtype, void *Y, int y_dtype,
                        dllm_stream_t stream);
/* The epilogue of a row-parallel layer after its partial sums are reduced over the ranks
 * (parallel.RowParallelLinear): out[m][n] = y[m][n] + bias[n] in f32 -- the
 * reference's `x.dot(&self.weights) + &self.bias` (diffuse-llm-rs/src/lib.rs:812), the bias added
 * once after the reduction -- stored as f32 (out may equal y) or RNE f16.  bias NULL = zeros.
 * y, out [M][N] device; asynchronous on `stream`. */
int dllm_bias_cast(const float *y, size_t M, size_t N, const float *bias, void *out, int out_dtype,
                   dllm_stream_t stream);
/* Export the quantized weights in canonical form (packed bitstream [K][N], scales [G][N], zps);
 * the codes are rebuilt from the device layout (the handle keeps no canonical copy). */
int dllm_linear_export(dllm_linear_t h, uint8_t *packed_codes, float *scales, uint8_t *zps,
                       dllm_stream_t stream);
int dllm_linear_info(dllm_linear_t h, size_t *K, size_t *N, uint8_t *bits, size_t *group);
int dllm_linear_precision(dllm_linear_t h);   /* DLLM_PRECISION_*, -1 on a null handle */
/* HBM bytes the forward's GEMM kernel reads for the weights (packed codes + scales/zps). */
size_t dllm_linear_weight_bytes(dllm_linear_t h);
/* Device memory the handle owns: the prefill and decode code layouts and the per-(group, column)
 * parameters (f16 zero-point/scale pairs + f32 scales) -- 17.02 MiB at 4096 x 4096 int4 g128, 9.02
 * MiB prefill-only -- plus the Horner ratios where kept (+0.52 MiB there). */
size_t dllm_linear_device_bytes(dllm_linear_t h);
int dllm_linear_destroy(dllm_linear_t h);

/* ---- f3: wire formats (host buffers; no device work) --------------------------------------
 * The serde derives of QuantizationParams / QuantizedTensor (quantization/src/types.rs:19-47) and
 * CompressedVector (diffusion_prefill/src/prefill_kv.rs:25-33) in the two encodings the reference's
 * crates use (bincode 1.3 legacy, quantization/src/error.rs:44-47; serde_json, :48-53):
 * bincode = little-endian fixed-width, usize as u64, Vec/String = u64 length + items, bool 1 byte,
 * Option = 1-byte tag (+ value); json = compact serde_json, f32 as ryu's shortest digits, non-finite
 * as null.  Encoders write into out[cap] and always set *len to the size needed (out = NULL: size
 * query; cap too small: DLLM_ERR_SERIALIZATION).  Decoders: strict = 0 ignores trailing bytes like
 * bincode::deserialize, strict = 1 rejects them; output arrays may be NULL to query their counts;
 * malformed input -> DLLM_ERR_SERIALIZATION (QuantizationError::Serialization). */
typedef struct dllm_qparams {
    uint8_t bits;
    float scale;
    int32_t zero_point;
    uint8_t symmetric;
    uint8_t has_axis;   /* Option<usize> axis */
    uint64_t axis;
} dllm_qparams;
int dllm_format_f32(float x, char *out, size_t cap, size_t *len);   /* serde_json's f32 text */
int dllm_qparams_to_bincode(const dllm_qparams *p, uint8_t *out, size_t cap, size_t *len);
int dllm_qparams_from_bincode(const uint8_t *buf, size_t len, int strict, dllm_qparams *p, size_t *consumed);
int dllm_qparams_to_json(const dllm_qparams *p, char *out, size_t cap, size_t *len);
int dllm_qparams_from_json(const char *s, size_t len, dllm_qparams *p);
int dllm_qtensor_to_bincode(const uint8_t *codes, size_t n, const uint64_t *shape, size_t ndim, const dllm_qparams *p,
                            uint8_t *out, size_t cap, size_t *len);
int dllm_qtensor_from_bincode(const uint8_t *buf, size_t len, int strict, uint8_t *codes, size_t codes_cap, size_t *n,
                              uint64_t *shape, size_t shape_cap, size_t *ndim, dllm_qparams *p);
int dllm_qtensor_to_json(const uint8_t *codes, size_t n, const uint64_t *shape, size_t ndim, const dllm_qparams *p,
                         char *out, size_t cap, size_t *len);
int dllm_qtensor_from_json(const char *s, size_t len, uint8_t *codes, size_t codes_cap, size_t *n, uint64_t *shape,
                           size_t shape_cap, size_t *ndim, dllm_qparams *p);
int dllm_compressed_vector_to_bincode(const char *id, size_t id_len, const uint8_t *data, size_t n, uint8_t bits,
                                      const uint64_t *shape, size_t ndim, float scale, float zero_point,
                                      uint8_t *out, size_t cap, size_t *len);
int dllm_compressed_vector_from_bincode(const uint8_t *buf, size_t len, int strict, char *id, size_t id_cap,
                                        size_t *id_len, uint8_t *data, size_t data_cap, size_t *n, uint8_t *bits,
                                        uint64_t *shape, size_t shape_cap, size_t *ndim, float *scale,
                                        float *zero_point);
int dllm_compressed_vector_to_json(const char *id, size_t id_len, const uint8_t *data, size_t n, uint8_t bits,
                                   const uint64_t *shape, size_t ndim, float scale, float zero_point, char *out,
                                   size_t cap, size_t *len);
int dllm_compressed_vector_from_json(const char *s, size_t len, char *id, size_t id_cap, size_t *id_len,
                                     uint8_t *data, size_t data_cap, size_t *n, uint8_t *bits, uint64_t *shape,
                                     size_t shape_cap, size_t *ndim, float *scale, float *zero_point);

/* ---- a9: int-quantized KV dequant-attention (consumer of QuantizedKVCacheEntry) -------------
 * The reference dequantizes K/V (QuantizedKVCacheEntry::dequantize_keys/values,
 * diffuse-llm-rs/src/quantization.rs:160-175) and hands them to DiffusionModel::forward_with_cache
 * (diffuse-llm-rs/src/lib.rs:910-915).  Build-defined consumer: per head, bidirectional SDPA
 * O = softmax(Q K^T / sqrt(D)) V, with K,V given as per-tensor quantized codes (a1 layout,
 * packed, `bits` in {4, 8}) + device params {scale, zp} (a2 dequant fused into the kernel).
 * Q f16 [S][H][D], O f16 [S][H][D], D == 128; Q, O and the codes 16-byte aligned (O is written as
 * 16-byte row pieces).  K/V are unpacked once per call into a grow-only
 * per-stream workspace (H * ceil(S/64) * 35 KiB), allocated on the first call of a shape. */
int dllm_kv_attention(const void *Q, const uint8_t *Kq, const float *k_params, const uint8_t *Vq,
                      const float *v_params, uint8_t bits, size_t S, size_t H, size_t D, void *O,
                      dllm_stream_t stream);

/* ---- 8f rank 1: diffusion-step ops either side of the denoiser --------------------------------
 * DiffuseLLM's schedule and sampling step (diffuse-llm-rs/src/lib.rs).  Host functions compute the
 * per-timestep / per-sample scalars with Rust f32 semantics (host arrays); the elementwise steps
 * run on the GPU.  Reference conventions exposed as flags ("pin the chosen form"):
 *   cumprod   DLLM_ABAR_EXCLUSIVE: alpha_bar[0] = 1, alpha_bar[i] = alpha_bar[i-1] alpha[i-1]
 *             (add_noise :1116-1119 and p_sample :1162-1165; gives 1 - alpha_bar = 0 at t = 0, so the
 *             reference's last p_sample step divides by zero); DLLM_ABAR_INCLUSIVE: the p_losses
 *             scan alpha_bar[i] = prod_{j<=i} alpha[j] (:627-630).
 *   alpha     DLLM_ALPHA_PER_SAMPLE: mean_coeff2 uses alpha[t_i] (the intended posterior);
 *             DLLM_ALPHA_LITERAL: the reference's full-length `alphas` row-wise (:1191), which is
 *             an elementwise op only when batch == num_timesteps (otherwise ndarray panics).
 * Noise: the reference draws rand::thread_rng normals (unseeded); the build uses a seeded
 * counter-based stream: element e of (seed) = Philox4x32-10(key seed, counter e/4) + a Box-Muller
 * of correctly rounded + - * / sqrt only (bit-reproducible on any IEEE host; see
 * csrc/diffusion_rng.hpp).  Stream offsets must be multiples of 4. */
enum dllm_beta_kind { DLLM_BETA_LINEAR = 0, DLLM_BETA_QUADRATIC = 1, DLLM_BETA_COSINE = 2 };
enum dllm_cumprod { DLLM_ABAR_EXCLUSIVE = 0, DLLM_ABAR_INCLUSIVE = 1 };
enum dllm_alpha_mode { DLLM_ALPHA_PER_SAMPLE = 0, DLLM_ALPHA_LITERAL = 1 };
/* DiffusionConfig::create_beta_schedule (lib.rs:554-593); host betas[T]. */
int dllm_beta_schedule(int kind, size_t T, float beta_start, float beta_end, float *betas);
/* alphas = 1 - betas and the alpha_bar table of the given cumprod convention (host arrays). */
int dllm_alpha_bars(const float *betas, size_t T, int cumprod, float *alphas, float *alpha_bars);
/* p_sample scalars (lib.rs:1167-1195) for timesteps t[B] (clamped to T-1 as :1175):
 * coef[B][3] = {c1 = sqrt(abar_prev) beta / (1 - abar), c2 = sqrt(alpha) (1 - abar_prev) / (1 - abar),
 * std = sqrt((1 - abar_prev) / (1 - abar) beta)}; *add_noise = (t[0] > 0) (:1198). Host arrays. */
int dllm_p_sample_coeffs(const float *betas, size_t T, int cumprod, int alpha_mode, const size_t *t, size_t B,
                         float *coef, int *add_noise);
/* add_noise scalars (lib.rs:1121-1133): coef[B][2] = {sqrt(abar_t), sqrt(1 - abar_t)}. Host arrays. */
int dllm_add_noise_coeffs(const float *betas, size_t T, int cumprod, const size_t *t, size_t B, float *coef);
/* out[i] = element offset + i of the seeded N(0,1) stream (device). */
int dllm_randn(uint64_t seed, uint64_t offset, float *out, size_t n, dllm_stream_t stream);
/* p_sample elementwise step (lib.rs:1197-1212) on B rows of D (device f32; coef device [B][3]):
 * x_prev = (c1 x_t + c2 eps) + std * n, n = noise[i] if noise != NULL, else stream element
 * offset + i of `seed`; n = 0 when add_noise == 0.  x_t, eps, x_prev 16-byte aligned. */
int dllm_p_sample(const float *x_t, const float *eps, const float *noise, const float *coef, size_t B, size_t D,
                  int add_noise, uint64_t seed, uint64_t offset, float *x_prev, dllm_stream_t stream);
/* add_noise forward step (lib.rs:1130-1135): noisy = x0 sqrt(abar) + n sqrt(1 - abar) on B rows
 * of D; n = noise (device) or the stream (noise == NULL; then written to noise_out if non-NULL,
 * the reference's returned noise). */
int dllm_add_noise(const float *x0, const float *noise, const float *coef, size_t B, size_t D, uint64_t seed,
                   uint64_t offset, float *noisy, float *noise_out, dllm_stream_t stream);
/* Denoiser output layer fused with p_sample: eps = X . W^ + b (f32, as dllm_linear_forward with
 * y_dtype DLLM_F32) feeds x_prev = (c1 x_t + c2 eps) + std * n in the GEMM epilogue, with x_t and
 * x_prev f32 [M][N] (device, may alias), coef device [M / rows_per_sample][3] (row m uses
 * sample m / rows_per_sample) and n = noise[m][n] when noise != NULL (f32 [M][N], e.g. drawn by
 * dllm_randn on a side stream while the earlier layers run), else stream element offset + m N + n
 * generated in the epilogue.  Bit-identical to dllm_linear_forward(..., DLLM_F32) followed by
 * dllm_p_sample with the same noise.  N % 4 == 0. */
int dllm_linear_forward_psample(dllm_linear_t h, const void *X, size_t M, int x_dtype, const float *x_t,
                                const float *coef, size_t rows_per_sample, int add_noise, uint64_t seed,
                                uint64_t offset, const float *noise, float *x_prev, dllm_stream_t stream);
/* The same, also writing x_prev rounded to f16 (RNE, the cast dllm_linear_forward applies to an f32
 * X) into x_prev_f16 (device [M][N], 16-byte aligned; NULL = none) from the same epilogue: the next
 * denoise step's first layer takes it as its f16 input instead of casting x_prev again
 * (DiffuseLLM::sample's x = x_prev hand-off, lib.rs:917-920). */
int dllm_linear_forward_psample_ex(dllm_linear_t h, const void *X, size_t M, int x_dtype, const float *x_t,
                                   const float *coef, size_t rows_per_sample, int add_noise, uint64_t seed,
                                   uint64_t offset, const float *noise, float *x_prev, void *x_prev_f16,
                                   dllm_stream_t stream);

/* ---- host-slice variants (synchronous; stage through device memory; not graph-capturable) ----
 * The literal shapes of the reference's Rust signatures, for callers holding host slices. */
/* quantize_tensor(&[f32], u8) -> (Vec<u8>, f32, f32): codes one per byte (quantization.rs:38-68). */
int dllm_quantize_tensor_host(const float *x, size_t n, uint8_t bits, uint8_t *codes, float *scale, float *zp);
/* dequantize_tensor(&[u8], f32, f32) -> Vec<f32> (quantization.rs:81-85). */
int dllm_dequantize_tensor_host(const uint8_t *codes, size_t n, float scale, float zp, float *out);
/* DefaultQuantizer quantize / dequantize (quantization/src/quantize.rs:111-184). */
int dllm_default_quantize_host(const float *x, size_t n, int qtype, float scale, int32_t zero_point, uint8_t *out);
int dllm_default_dequantize_host(const uint8_t *q, size_t n, float scale, int32_t zero_point, float *out);
/* kvquant::BitQuantizer::{quantize, dequantize} (prefill-kvquant-rs/lib.rs:39-53). */
int dllm_bit_quantize_host(const float *x, size_t n, uint32_t bits, float scale, float zero_point, uint8_t *out);
int dllm_bit_dequantize_host(const uint8_t *q, size_t n, float scale, float zero_point, float *out);
/* diffusion_prefill KVCache::compress_vector (diffusion_prefill/src/prefill_kv.rs:104-121). */
int dllm_compress_vector_host(const float *x, size_t n, uint8_t bits, uint8_t *out, float *scale, float *zp);
/* SimpleDiffusionModel::new + forward (diffuse-llm-rs/src/lib.rs:791-813) with quantized W. */
int dllm_linear_create_host(const float *W, const float *bias, size_t K, size_t N, uint8_t bits, size_t group,
                            dllm_linear_t *out);
int dllm_linear_forward_host(dllm_linear_t h, const float *X, size_t M, float *Y);

#ifdef __cplusplus
}
#endif
#endif /* DLLM_QUANT_H */
