// The reference's own #[test]s for the quantized path, replayed through the C++ mirror
// (include/dllm_quant.hpp -> C-ABI -> HIP kernels).  Where a reference test contradicts the
// reference's code, the assertion here pins the CODE's behaviour and says so.
// Build: g++ -std=c++17 -I include tests/cpp/test_reference_mirror.cpp -L <lib> -ldllm_hip
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#include "dllm_quant.hpp"

static int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                                  \
    do {                                                                             \
        if (!(cond)) {                                                               \
            std::printf("  CHECK FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);    \
            throw std::runtime_error("check");                                       \
        }                                                                            \
    } while (0)

static void run(const char *name, const std::function<void()> &f) {
    try {
        f();
        ++g_pass;
        std::printf("ok   %s\n", name);
    } catch (const std::exception &e) {
        ++g_fail;
        std::printf("FAIL %s (%s)\n", name, e.what());
    }
}

using namespace dllm;

int main() {
    // diffuse-llm-rs/src/quantization.rs:242-252 test_quantization.  The test asserts a 0.1
    // round-trip error; under the code zp clamps to 0 and q = [4,7,11,15,15] (max error 1.0).
    run("quantization.rs::test_quantization (literal semantics)", [] {
        std::vector<float> data{1, 2, 3, 4, 5};
        auto [q, scale, zp] = diffuse_llm_rs::quantization::quantize_tensor(data, 4);
        CHECK((q == std::vector<uint8_t>{4, 7, 11, 15, 15}));
        uint32_t sbits;
        std::memcpy(&sbits, &scale, 4);
        CHECK(sbits == 0x3E888889u && zp == 0.0f);
        auto deq = diffuse_llm_rs::quantization::dequantize_tensor(q, scale, zp);
        float maxerr = 0;
        for (size_t i = 0; i < data.size(); ++i) maxerr = std::fmax(maxerr, std::fabs(data[i] - deq[i]));
        CHECK(std::fabs(maxerr - 1.0f) < 1e-6f);
    });
    // quantization.rs:254-265 test_quantized_tensor (passes as written)
    run("quantization.rs::test_quantized_tensor", [] {
        std::vector<float> data{1, 2, 3, 4};
        auto [q, scale, zp] = diffuse_llm_rs::quantization::quantize_tensor(data, 4);
        auto qt = diffuse_llm_rs::quantization::QuantizedTensor::new_(q, {2, 2}, scale, zp, 4);
        CHECK(qt.dequantize().size() == 4);
        CHECK(qt.compression_ratio() > 4.0f);
    });
    // quantization.rs:39 assert! -> InvalidParams
    run("quantize_tensor bits out of range -> InvalidParams", [] {
        bool threw = false;
        try {
            diffuse_llm_rs::quantization::quantize_tensor({1.f}, 9);
        } catch (const QuantizationError &e) {
            threw = e.code() == DLLM_ERR_INVALID_PARAMS;
        }
        CHECK(threw);
    });
    // quantization.rs:140-175 QuantizedKVCacheEntry
    run("QuantizedKVCacheEntry::new / dequantize", [] {
        std::vector<float> k(2 * 8 * 16), v(k.size());
        for (size_t i = 0; i < k.size(); ++i) { k[i] = std::sin(0.1f * i); v[i] = std::cos(0.07f * i) * 3; }
        auto e = diffuse_llm_rs::quantization::QuantizedKVCacheEntry::new_(k, v, {2, 8, 16}, 4);
        CHECK(e.seq_len == 8);
        auto dk = e.dequantize_keys();
        auto [q, s, z] = diffuse_llm_rs::quantization::quantize_tensor(k, 4);
        CHECK(dk == diffuse_llm_rs::quantization::dequantize_tensor(q, s, z));
    });
    // quantization/src/lib.rs:61-79 test_quantization_roundtrip: -1.0 -> u8 0 (saturating cast)
    run("quantization::test_quantization_roundtrip (literal semantics)", [] {
        std::vector<float> data{-1, 0, 1, 2, 3, 4};
        ::dllm::quantization::DefaultQuantizer qz(8, false, std::nullopt);
        auto t = qz.quantize(data, {2, 3}, ::dllm::quantization::QuantizationType::Int8);
        CHECK((t.shape == std::vector<size_t>{2, 3}));
        CHECK((t.data == std::vector<uint8_t>{0, 0, 1, 2, 3, 4}));
        auto d = qz.dequantize(t);
        CHECK((d == std::vector<float>{0, 0, 1, 2, 3, 4}));
    });
    // quantize.rs:222-233 test_quantize_int8 (shape preserved)
    run("quantize.rs::test_quantize_int8", [] {
        auto t = ::dllm::quantization::quant_utils::quantize({-1, 0, 1, 2, 3, 4}, {2, 3},
                                                             ::dllm::quantization::QuantizationType::Int8, false);
        CHECK((t.shape == std::vector<size_t>{2, 3}) && t.dequantize().size() == 6);
    });
    // calibrate.rs:123-132 asserts scale ~0.0235, zp -43; the code gives 5/255 and -51.
    run("calibrate.rs::test_calibration (literal semantics)", [] {
        auto p = ::dllm::quantization::calibration_compute_params(1.0f, 6.0f, 6, 8, false);
        CHECK(p.scale == 5.0f / 255.0f && p.zero_point == -51);
    });
    // diffusion_prefill/src/prefill_kv.rs:147-160 test_quantization (passes as written)
    run("prefill_kv.rs::test_quantization", [] {
        std::vector<float> v{0.1f, 0.5f, 1.0f, 0.0f};
        auto c = diffusion_prefill::compress_vector("test", v, 4);
        CHECK((c.data == std::vector<uint8_t>{1, 7, 14, 0}));
        auto d = diffusion_prefill::decompress_vector(c);
        for (size_t i = 0; i < v.size(); ++i) CHECK(std::fabs(v[i] - d[i]) < 0.1f);
    });
    // prefill-kvquant-rs/lib.rs:101-146 PrefillKVQuant (4-bit request -> quantizers[2] = 8-bit scale)
    run("PrefillKVQuant::quantize_vectors", [] {
        using namespace prefill_kvquant_rs::kvquant;
        auto pk = PrefillKVQuant::new_(SystemConfig{});
        std::vector<TokenizedVector> toks(3);
        for (int i = 0; i < 3; ++i) toks[i] = TokenizedVector{"t" + std::to_string(i), {}, 2, 2, {0.5f, 1.0f, -1.f, 0.01f}};
        auto cv = pk.quantize_vectors(toks, {4, 2});
        CHECK(cv.size() == 3 && cv[0].bits == 4 && cv[1].bits == 2 && cv[2].bits == 4);
        CHECK((cv[0].data == std::vector<uint8_t>{15, 15, 0, 2}));   // 0.5*255 = 127.5 -> clamp 15
        bool threw = false;
        try { pk.quantize_vectors(toks, {8}); } catch (const QuantizationError &e) { threw = e.code() == DLLM_ERR_INVALID_PARAMS; }
        CHECK(threw);
    });
    // SimpleDiffusionModel forward (lib.rs:806-813) with the quantized weight
    run("SimpleDiffusionModel::forward (int4 g128)", [] {
        const size_t in = 256, out = 64, batch = 3;
        std::vector<float> w(in * out), b(out, 0.5f), x(batch * in);
        for (size_t i = 0; i < w.size(); ++i) w[i] = 0.02f * std::sin(0.37f * i);
        for (size_t i = 0; i < x.size(); ++i) x[i] = std::cos(0.11f * i);
        diffuse_llm_rs::diffuse_llm::SimpleDiffusionModel m(w, b, in, out);
        auto y = m.forward(x, batch);
        CHECK(y.size() == batch * out);
        // reference: per (column, 128-group) quantize_tensor -> dequantize -> f64 dot
        double num = 0, den = 0;
        for (size_t r = 0; r < batch; ++r)
            for (size_t n = 0; n < out; ++n) {
                double acc = b[n];
                for (size_t g = 0; g < in / 128; ++g) {
                    std::vector<float> col(128);
                    for (size_t k = 0; k < 128; ++k) col[k] = w[(g * 128 + k) * out + n];
                    auto [q, s, z] = diffuse_llm_rs::quantization::quantize_tensor(col, 4);
                    auto d = diffuse_llm_rs::quantization::dequantize_tensor(q, s, z);
                    for (size_t k = 0; k < 128; ++k) acc += double(x[r * in + g * 128 + k]) * d[k];
                }
                num += (y[r * out + n] - acc) * (y[r * out + n] - acc);
                den += acc * acc;
            }
        CHECK(std::sqrt(num / den) <= 1e-3);
    });
    std::printf("%d passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
