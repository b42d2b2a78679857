// dllm_quant.hpp -- C++ host-side mirror of diffusion-llm-rs's quantized-path operator surface,
// implemented over the C-ABI of dllm_quant.h (HIP kernels in libdllm_hip.so).
//
// Same names, argument meaning and error behaviour as the Rust items (cited per item; paths
// relative to the reference root).  Rust `Result` errors and panics become dllm::QuantizationError
// exceptions carrying the C-ABI status (1..7 = QuantizationError variants, reference panics ->
// InvalidParams).  Everything here takes and returns host containers, like the Rust APIs.
#pragma once

#include <cmath>
#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "dllm_quant.h"

namespace dllm {

// quantization/src/error.rs:18-40
class QuantizationError : public std::runtime_error {
  public:
    QuantizationError(int code, const std::string &msg) : std::runtime_error(msg), code_(code) {}
    int code() const { return code_; }

  private:
    int code_;
};

namespace detail {
inline void check(int rc) {
    if (rc != DLLM_OK) throw QuantizationError(rc, std::string("[") + std::to_string(rc) + "] " + dllm_last_error());
}
inline size_t product(const std::vector<size_t> &shape) {
    size_t n = 1;
    for (size_t s : shape) n *= s;
    return n;
}
}  // namespace detail

// ===================================================================================================
// diffuse_llm_rs::quantization (diffuse-llm-rs/src/quantization.rs)
// ===================================================================================================
namespace diffuse_llm_rs {
namespace quantization {

// :38-68
inline std::tuple<std::vector<uint8_t>, float, float> quantize_tensor(const std::vector<float> &data, uint8_t bits) {
    std::vector<uint8_t> q(data.size());
    float scale = 0.f, zp = 0.f;
    detail::check(dllm_quantize_tensor_host(data.data(), data.size(), bits, q.data(), &scale, &zp));
    return {std::move(q), scale, zp};
}

// :81-85
inline std::vector<float> dequantize_tensor(const std::vector<uint8_t> &data, float scale, float zero_point) {
    std::vector<float> out(data.size());
    detail::check(dllm_dequantize_tensor_host(data.data(), data.size(), scale, zero_point, out.data()));
    return out;
}

// :88-125
class QuantizedTensor {
  public:
    QuantizedTensor(std::vector<uint8_t> data, std::vector<size_t> shape, float scale, float zero_point, uint8_t bits)
        : data(std::move(data)), shape(std::move(shape)), scale(scale), zero_point(zero_point), bits(bits) {}
    static QuantizedTensor new_(std::vector<uint8_t> data, std::vector<size_t> shape, float scale, float zero_point,
                                uint8_t bits) {
        return QuantizedTensor(std::move(data), std::move(shape), scale, zero_point, bits);
    }
    std::vector<float> dequantize() const { return dequantize_tensor(data, scale, zero_point); }   // :115-117
    float compression_ratio() const {                                                             // :120-124
        return dllm_compression_ratio(detail::product(shape), data.size(), bits);
    }

    std::vector<uint8_t> data;
    std::vector<size_t> shape;
    float scale;
    float zero_point;
    uint8_t bits;
};

// :128-176 (Array3 passed as flat row-major data + shape [num_layers, seq, hidden])
class QuantizedKVCacheEntry {
  public:
    static QuantizedKVCacheEntry new_(const std::vector<float> &keys, const std::vector<float> &values,
                                      const std::vector<size_t> &shape, uint8_t bits) {
        if (shape.size() != 3 || detail::product(shape) != keys.size() || keys.size() != values.size())
            throw QuantizationError(DLLM_ERR_SHAPE_MISMATCH, "keys/values must match a 3-d shape");
        auto [kq, ks, kz] = quantize_tensor(keys, bits);
        auto [vq, vs, vz] = quantize_tensor(values, bits);
        return QuantizedKVCacheEntry{QuantizedTensor(std::move(kq), shape, ks, kz, bits),
                                     QuantizedTensor(std::move(vq), shape, vs, vz, bits), shape[1]};
    }
    std::vector<float> dequantize_keys() const { return keys.dequantize(); }      // :160-166
    std::vector<float> dequantize_values() const { return values.dequantize(); }  // :169-175

    QuantizedTensor keys;
    QuantizedTensor values;
    size_t seq_len;
};

}  // namespace quantization

namespace diffuse_llm {

// SimpleDiffusionModel (diffuse-llm-rs/src/lib.rs:775-836) with its [input_dim, output_dim]
// weight group-quantized (QuantizationConfig::default(): 4 bits, group 128) and the forward
// x.dot(W) + b (:806-813) run as the dequant + MFMA GEMM.  Not copyable (owns device memory).
class SimpleDiffusionModel {
  public:
    SimpleDiffusionModel(const std::vector<float> &weights, const std::vector<float> &bias, size_t input_dim,
                         size_t output_dim, uint8_t bits = 4, size_t group = 128)
        : in_(input_dim), out_(output_dim) {
        if (weights.size() != input_dim * output_dim || (!bias.empty() && bias.size() != output_dim))
            throw QuantizationError(DLLM_ERR_SHAPE_MISMATCH, "weights must be [input_dim, output_dim]");
        detail::check(dllm_linear_create_host(weights.data(), bias.empty() ? nullptr : bias.data(), input_dim,
                                              output_dim, bits, group, &h_));
    }
    SimpleDiffusionModel(const SimpleDiffusionModel &) = delete;
    SimpleDiffusionModel &operator=(const SimpleDiffusionModel &) = delete;
    SimpleDiffusionModel(SimpleDiffusionModel &&o) noexcept : h_(o.h_), in_(o.in_), out_(o.out_) { o.h_ = nullptr; }
    ~SimpleDiffusionModel() {
        if (h_) dllm_linear_destroy(h_);
    }
    // forward(x: &Array2<f32> [batch, input_dim], _t) -> Array2<f32> [batch, output_dim]
    std::vector<float> forward(const std::vector<float> &x, size_t batch) const {
        if (x.size() != batch * in_) throw QuantizationError(DLLM_ERR_SHAPE_MISMATCH, "x must be [batch, input_dim]");
        std::vector<float> y(batch * out_);
        detail::check(dllm_linear_forward_host(h_, x.data(), batch, y.data()));
        return y;
    }
    size_t input_dim() const { return in_; }
    size_t output_dim() const { return out_; }

  private:
    dllm_linear_t h_ = nullptr;
    size_t in_, out_;
};

}  // namespace diffuse_llm
}  // namespace diffuse_llm_rs

// ===================================================================================================
// quantization crate (quantization/src/*.rs)
// ===================================================================================================
namespace quantization {

// quantize.rs:62-78
enum class QuantizationType { Int8 = DLLM_QT_INT8, Int4 = DLLM_QT_INT4, Binary = DLLM_QT_BINARY, Float8 = DLLM_QT_FLOAT8 };
inline uint8_t bits(QuantizationType t) {
    switch (t) {
    case QuantizationType::Int8: return 8;
    case QuantizationType::Int4: return 4;
    case QuantizationType::Binary: return 1;
    default: return 8;
    }
}

// types.rs:20-40
struct QuantizationParams {
    uint8_t bits = 8;
    float scale = 1.0f;
    int32_t zero_point = 0;
    bool symmetric = true;
    std::optional<size_t> axis;
};

// types.rs:42-82
struct QuantizedTensor {
    std::vector<uint8_t> data;
    std::vector<size_t> shape;
    QuantizationParams params;
    size_t len() const { return detail::product(shape); }
    bool is_empty() const { return data.empty(); }
    std::vector<float> dequantize() const {
        std::vector<float> out(len());
        detail::check(dllm_default_dequantize_host(data.data(), data.size(), params.scale, params.zero_point,
                                                   out.data()));
        return out;
    }
};

// quantize.rs:81-90
class Quantizer {
  public:
    virtual ~Quantizer() = default;
    virtual QuantizedTensor quantize(const std::vector<float> &data, const std::vector<size_t> &shape,
                                     QuantizationType qtype) const = 0;
    virtual std::vector<float> dequantize(const QuantizedTensor &tensor) const = 0;
    virtual const QuantizationParams &get_params() const = 0;
};

// quantize.rs:93-189: new(bits, symmetric, axis) fixes scale 1.0, zero_point 0.
class DefaultQuantizer : public Quantizer {
  public:
    DefaultQuantizer(uint8_t bits, bool symmetric, std::optional<size_t> axis) {
        params_.bits = bits;
        params_.symmetric = symmetric;
        params_.axis = axis;
    }
    static DefaultQuantizer new_(uint8_t bits, bool symmetric, std::optional<size_t> axis) {
        return DefaultQuantizer(bits, symmetric, axis);
    }
    QuantizedTensor quantize(const std::vector<float> &data, const std::vector<size_t> &shape,
                             QuantizationType qtype) const override {
        if (detail::product(shape) != data.size())
            throw QuantizationError(DLLM_ERR_SHAPE_MISMATCH, "data length does not match shape");
        QuantizedTensor t{std::vector<uint8_t>(data.size()), shape, params_};
        detail::check(dllm_default_quantize_host(data.data(), data.size(), static_cast<int>(qtype), params_.scale,
                                                 params_.zero_point, t.data.data()));
        return t;
    }
    std::vector<float> dequantize(const QuantizedTensor &tensor) const override { return tensor.dequantize(); }
    const QuantizationParams &get_params() const override { return params_; }

  private:
    QuantizationParams params_;
};

// quantize.rs:191-215
namespace quant_utils {
inline QuantizedTensor quantize(const std::vector<float> &data, const std::vector<size_t> &shape,
                                QuantizationType qtype, bool symmetric, std::optional<size_t> axis = std::nullopt) {
    return DefaultQuantizer(bits(qtype), symmetric, axis).quantize(data, shape, qtype);
}
inline std::vector<float> dequantize(const QuantizedTensor &t) {
    return DefaultQuantizer(t.params.bits, t.params.symmetric, t.params.axis).dequantize(t);
}
}  // namespace quant_utils

// calibrate.rs:72-110 (compute_params from accumulated min/max; the device-side update reduction
// is exposed by dllm_calib_update and the Python mirror).
inline QuantizationParams calibration_compute_params(float min, float max, size_t total_samples, uint8_t nbits,
                                                     bool symmetric) {
    QuantizationParams p;
    p.bits = nbits;
    p.symmetric = symmetric;
    detail::check(dllm_calib_compute_params(min, max, total_samples, nbits, symmetric ? 1 : 0, &p.scale, &p.zero_point));
    return p;
}

}  // namespace quantization

// ===================================================================================================
// prefill_kvquant_rs::kvquant (prefill-kvquant-rs/lib.rs)
// ===================================================================================================
namespace prefill_kvquant_rs {
namespace kvquant {

// :29-32 (Send + Sync: implementations hold only immutable scalars)
class Quantizer {
  public:
    virtual ~Quantizer() = default;
    virtual std::vector<uint8_t> quantize(const std::vector<float> &input, uint8_t bits) const = 0;
    virtual std::vector<float> dequantize(const std::vector<uint8_t> &input, uint8_t bits) const = 0;
};

// :34-53
class BitQuantizer : public Quantizer {
  public:
    BitQuantizer(float scale, float zero_point) : scale(scale), zero_point(zero_point) {}
    std::vector<uint8_t> quantize(const std::vector<float> &input, uint8_t nbits) const override {
        std::vector<uint8_t> out(input.size());
        detail::check(dllm_bit_quantize_host(input.data(), input.size(), nbits, scale, zero_point, out.data()));
        return out;
    }
    std::vector<float> dequantize(const std::vector<uint8_t> &input, uint8_t) const override {
        std::vector<float> out(input.size());
        detail::check(dllm_bit_dequantize_host(input.data(), input.size(), scale, zero_point, out.data()));
        return out;
    }
    float scale;
    float zero_point;
};

// :61-67
struct CompressedVector {
    std::string id;
    std::vector<uint8_t> data;
    uint8_t bits;
    std::vector<size_t> original_shape;
};

// :76-91
struct SystemConfig {
    size_t num_quantizers = 4;
    size_t cache_size = 1024;
    std::vector<uint8_t> quantization_bits{4, 6, 8, 16};
};

// :93-97 (embeddings: rows x cols, row-major)
struct TokenizedVector {
    std::string id;
    std::vector<uint32_t> tokens;
    size_t rows = 0, cols = 0;
    std::vector<float> embeddings;
};

// :23-147
class PrefillKVQuant {
  public:
    static PrefillKVQuant new_(const SystemConfig &config) { return PrefillKVQuant(config); }
    explicit PrefillKVQuant(const SystemConfig &config) : cfg_(config) {
        for (uint8_t b : config.quantization_bits) {   // :102-110
            if (b > 30) throw QuantizationError(DLLM_ERR_INVALID_PARAMS, "(1 << bits) - 1 overflows");
            quantizers_.emplace_back(1.0f / static_cast<float>((1 << b) - 1), 0.0f);
        }
    }
    // :127-146: bits cycled over the token vectors; quantizer index bits / 2 (panics -> throws).
    std::vector<CompressedVector> quantize_vectors(const std::vector<TokenizedVector> &tokens,
                                                   const std::vector<uint8_t> &nbits) const {
        std::vector<CompressedVector> out;
        if (nbits.empty()) return out;
        for (size_t i = 0; i < tokens.size(); ++i) {
            const uint8_t b = nbits[i % nbits.size()];
            const size_t qi = b / 2;
            if (qi >= quantizers_.size())
                throw QuantizationError(DLLM_ERR_INVALID_PARAMS, "index out of bounds: quantizers[bits / 2]");
            out.push_back(CompressedVector{tokens[i].id, quantizers_[qi].quantize(tokens[i].embeddings, b), b,
                                           {tokens[i].rows, tokens[i].cols}});
        }
        return out;
    }
    const std::vector<BitQuantizer> &quantizers() const { return quantizers_; }

  private:
    SystemConfig cfg_;
    std::vector<BitQuantizer> quantizers_;
};

}  // namespace kvquant
}  // namespace prefill_kvquant_rs

// diffusion_prefill::prefill_kv::KVCache::compress_vector (diffusion_prefill/src/prefill_kv.rs:104-121)
namespace diffusion_prefill {
struct CompressedVector {
    std::string id;
    std::vector<uint8_t> data;
    uint8_t bits;
    std::vector<size_t> original_shape;
    float quant_scale;
    float quant_zero_point;
};
inline CompressedVector compress_vector(const std::string &id, const std::vector<float> &vector, uint8_t bits) {
    CompressedVector cv{id, std::vector<uint8_t>(vector.size()), bits, {vector.size()}, 0.f, 0.f};
    detail::check(dllm_compress_vector_host(vector.data(), vector.size(), bits, cv.data.data(), &cv.quant_scale,
                                            &cv.quant_zero_point));
    return cv;
}
// :124-132
inline std::vector<float> decompress_vector(const CompressedVector &v) {
    return prefill_kvquant_rs::kvquant::BitQuantizer(v.quant_scale, v.quant_zero_point).dequantize(v.data, v.bits);
}
}  // namespace diffusion_prefill

}  // namespace dllm
