// attention.hip -- quantized-KV dequant-attention (a9).  Placeholder until the kernel lands.
#include "common.hpp"

using namespace dllm;

extern "C" int dllm_kv_attention(const void *Q, const uint8_t *Kq, const float *k_params, const uint8_t *Vq,
                                 const float *v_params, uint8_t bits, size_t S, size_t H, size_t D, void *O,
                                 dllm_stream_t stream) {
    return fail(DLLM_ERR_UNSUPPORTED, "dllm_kv_attention: not built yet");
}
