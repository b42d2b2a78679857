"""diffusion-llm-rs_amd: MI355X-native (gfx950) quantized inference hot path of
zetareticula/diffusion-llm-rs.

Compute runs in hand-written HIP kernels (lib/libdllm_hip.so, C-ABI in include/dllm_quant.h);
this package is the host-side mirror of the reference's Rust operator surface:

* ``quantization`` -- ``diffuse_llm_rs::quantization`` (quantize_tensor, dequantize_tensor,
  QuantizedTensor, QuantizedKVCacheEntry) + packing.
* ``quant``        -- the ``quantization`` crate (Quantizer, DefaultQuantizer, QuantizationType,
  quant_utils, CalibrationData).
* ``kvquant``      -- ``prefill_kvquant_rs::kvquant`` (BitQuantizer, PrefillKVQuant, SystemConfig)
  and ``diffusion_prefill``'s compress/decompress_vector.
* ``linear``       -- the int2/int4/int8 group-quantized linear layer (dequant + MFMA GEMM).
* ``serde``        -- bincode / serde_json wire formats of QuantizationParams, QuantizedTensor and
  the diffusion_prefill CompressedVector hand-off record.
* ``diffusion``    -- ``diffuse_llm``'s schedules, add_noise / p_sample (seeded device noise), the
  phase-aware KVCacheEntry and the denoise loop (last layer fused with p_sample).
"""
from . import _lib
from ._lib import (CalibrationRequired, HipError, InvalidParams, QuantizationError, SerializationError,
                   ShapeMismatch, UnsupportedOperation)
from . import quantization, quant, kvquant, linear, parallel, diffusion, serde
from .quantization import (AdaptiveQuantizer, QuantizedKVCacheEntry, QuantizedTensor, compression_ratio, dequantize_tensor, kv_attention,
                           pack, quantize_tensor, quantize_tensor_pair, unpack)
from .quant import CalibrationData, DefaultQuantizer, QuantizationParams, QuantizationType, quant_utils
from .kvquant import BitQuantizer, PrefillKVQuant, SystemConfig, compress_vectors, decompress_vectors
from .linear import MixedPrecisionStack, QuantLinear
from .diffusion import (AlphaMode, BetaSchedule, Cumprod, DenoiseLoop, DiffusionConfig, KVCacheEntry, KVCacheStore,
                        add_noise,
                        p_sample, randn)

__all__ = [
    "quantize_tensor", "quantize_tensor_pair", "dequantize_tensor", "pack", "unpack", "compression_ratio", "QuantizedTensor",
    "QuantizedKVCacheEntry", "kv_attention", "QuantizationType", "QuantizationParams", "DefaultQuantizer", "quant_utils",
    "CalibrationData", "BitQuantizer", "PrefillKVQuant", "SystemConfig", "compress_vectors", "decompress_vectors",
    "QuantLinear", "MixedPrecisionStack", "QuantizationError", "InvalidParams", "UnsupportedOperation",
    "ShapeMismatch", "CalibrationRequired", "HipError", "BetaSchedule", "Cumprod", "AlphaMode", "DiffusionConfig",
    "KVCacheEntry", "KVCacheStore", "DenoiseLoop", "add_noise", "p_sample", "randn", "AdaptiveQuantizer",
]


def load_library():
    """Loads the HIP library now (raises ImportError if it was not built)."""
    return _lib.load()
