"""ctypes binding of libdllm_hip.so (the C-ABI in include/dllm_quant.h).

The product path: every compute call goes to the HIP kernels in lib/libdllm_hip.so.  There is no
CPU fallback; if the library is missing or no GPU is visible, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "lib" / "libdllm_hip.so"
HEADER = PKG_DIR.parent / "include" / "dllm_quant.h"

# Status codes (include/dllm_quant.h, mirroring quantization/src/error.rs:18-40).
OK = 0
ERR_INVALID_PARAMS = 1
ERR_UNSUPPORTED = 2
ERR_SHAPE_MISMATCH = 3
ERR_CALIBRATION_REQUIRED = 4
ERR_IO = 5
ERR_SERIALIZATION = 6
ERR_INVALID_DATA_FORMAT = 7
ERR_HIP = 16
ERR_NO_DEVICE = 17

F32, F16 = 0, 1


class QuantizationError(RuntimeError):
    """Mirror of quantization::QuantizationError (quantization/src/error.rs:18-40)."""

    code = -1

    def __init__(self, msg: str, code: int | None = None):
        super().__init__(msg)
        if code is not None:
            self.code = code


class InvalidParams(QuantizationError, ValueError):
    code = ERR_INVALID_PARAMS


class UnsupportedOperation(QuantizationError):
    code = ERR_UNSUPPORTED


class ShapeMismatch(QuantizationError, ValueError):
    code = ERR_SHAPE_MISMATCH


class CalibrationRequired(QuantizationError):
    code = ERR_CALIBRATION_REQUIRED


class HipError(QuantizationError):
    code = ERR_HIP


class SerializationError(QuantizationError, ValueError):
    """QuantizationError::Serialization (quantization/src/error.rs:29-30, from bincode / serde_json)."""
    code = ERR_SERIALIZATION


_ERRORS = {ERR_INVALID_PARAMS: InvalidParams, ERR_UNSUPPORTED: UnsupportedOperation,
           ERR_SHAPE_MISMATCH: ShapeMismatch, ERR_CALIBRATION_REQUIRED: CalibrationRequired,
           ERR_SERIALIZATION: SerializationError, ERR_HIP: HipError, ERR_NO_DEVICE: HipError}

P, S, U8, I32, U32, FL, INT = (C.c_void_p, C.c_size_t, C.c_uint8, C.c_int32, C.c_uint32, C.c_float, C.c_int)
U64 = C.c_uint64

# name -> (restype, argtypes); the authoritative list of exported entry points.
SIGNATURES = {
    "dllm_last_error": (C.c_char_p, []),
    "dllm_version": (C.c_char_p, []),
    "dllm_device_arch": (INT, [INT, C.c_char_p, S]),
    "dllm_quantize_tensor_workspace": (S, [S]),
    "dllm_quantize_tensor": (INT, [P, S, U8, INT, P, P, P, S, P]),
    "dllm_quantize_tensor_pair": (INT, [P, S, U8, U8, INT, P, P, P, P, P, S, P]),
    "dllm_dequantize_tensor": (INT, [P, S, U8, INT, P, P, INT, P]),
    "dllm_dequantize_tensor_scalar": (INT, [P, S, U8, INT, FL, FL, P, INT, P]),
    "dllm_compression_ratio": (FL, [S, S, U8]),
    "dllm_packed_bytes": (S, [S, U8]),
    "dllm_pack": (INT, [P, S, U8, P, P]),
    "dllm_unpack": (INT, [P, S, U8, P, P]),
    "dllm_default_quantize": (INT, [P, S, INT, FL, I32, P, P]),
    "dllm_default_dequantize": (INT, [P, S, FL, I32, P, P]),
    "dllm_calib_update": (INT, [P, S, P, P, S, P, S, P]),
    "dllm_calib_compute_params": (INT, [FL, FL, S, U8, INT, P, P]),
    "dllm_tensor_extremes": (INT, [P, S, P, P, S, P]),
    "dllm_quantize_params_from_extremes": (INT, [P, U8, P, P]),
    "dllm_quantize_tensor_with_params": (INT, [P, S, U8, INT, P, P, P]),
    "dllm_quantize_tensor_pair_with_params": (INT, [P, S, U8, U8, INT, P, P, P, P, P]),
    "dllm_quantize_kv_workspace": (S, [S, S]),
    "dllm_quantize_kv": (INT, [P, S, P, S, U8, U8, INT, P, P, P, P, P, P, P, P, P, S, P]),
    "dllm_kv_extremes": (INT, [P, S, P, S, P, P, S, P]),
    "dllm_quantize_kv_with_extremes": (INT, [P, S, P, S, P, U8, U8, INT, P, P, P, P, P, P, P, P, P]),
    "dllm_bias_cast": (INT, [P, S, S, P, P, INT, P]),
    "dllm_adaptive_update": (INT, [P, S, P, P, S, P]),
    "dllm_adaptive_compute_params": (INT, [P, INT, U32, P, P]),
    "dllm_adaptive_quantize": (INT, [P, S, U32, P, INT, P, P]),
    "dllm_bit_quantize": (INT, [P, S, U32, FL, FL, P, P]),
    "dllm_bit_dequantize": (INT, [P, S, FL, FL, P, INT, P]),
    "dllm_quantize_vectors": (INT, [P, S, S, P, S, P, S, P, P, P]),
    "dllm_compress_vectors": (INT, [P, S, S, U8, P, P, P, P]),
    "dllm_decompress_vectors": (INT, [P, S, S, P, P, P, P]),
    "dllm_linear_create": (INT, [P, P, S, S, U8, S, P, P]),
    "dllm_linear_create_quantized": (INT, [P, P, P, P, S, S, U8, S, P, P]),
    "dllm_linear_forward": (INT, [P, P, S, INT, P, INT, P]),
    "dllm_linear_export": (INT, [P, P, P, P, P]),
    "dllm_linear_info": (INT, [P, P, P, P, P]),
    "dllm_linear_weight_bytes": (S, [P]),
    "dllm_linear_device_bytes": (S, [P]),
    "dllm_linear_create_ex": (INT, [P, P, S, S, U8, S, INT, P, P]),
    "dllm_linear_create_quantized_ex": (INT, [P, P, P, P, S, S, U8, S, INT, P, P]),
    "dllm_linear_precision": (INT, [P]),
    "dllm_linear_destroy": (INT, [P]),
    "dllm_kv_attention": (INT, [P, P, P, P, P, U8, S, S, S, P, P]),
    "dllm_beta_schedule": (INT, [INT, S, FL, FL, P]),
    "dllm_alpha_bars": (INT, [P, S, INT, P, P]),
    "dllm_p_sample_coeffs": (INT, [P, S, INT, INT, P, S, P, P]),
    "dllm_add_noise_coeffs": (INT, [P, S, INT, P, S, P]),
    "dllm_randn": (INT, [U64, U64, P, S, P]),
    "dllm_p_sample": (INT, [P, P, P, P, S, S, INT, U64, U64, P, P]),
    "dllm_add_noise": (INT, [P, P, P, S, S, U64, U64, P, P, P]),
    "dllm_linear_forward_psample": (INT, [P, P, S, INT, P, P, S, INT, U64, U64, P, P, P]),
    "dllm_linear_forward_psample_ex": (INT, [P, P, S, INT, P, P, S, INT, U64, U64, P, P, P, P]),
    "dllm_quantize_tensor_host": (INT, [P, S, U8, P, P, P]),
    "dllm_dequantize_tensor_host": (INT, [P, S, FL, FL, P]),
    "dllm_default_quantize_host": (INT, [P, S, INT, FL, I32, P]),
    "dllm_default_dequantize_host": (INT, [P, S, FL, I32, P]),
    "dllm_bit_quantize_host": (INT, [P, S, U32, FL, FL, P]),
    "dllm_bit_dequantize_host": (INT, [P, S, FL, FL, P]),
    "dllm_compress_vector_host": (INT, [P, S, U8, P, P, P]),
    "dllm_linear_create_host": (INT, [P, P, S, S, U8, S, P]),
    "dllm_format_f32": (INT, [FL, P, S, P]),
    "dllm_qparams_to_bincode": (INT, [P, P, S, P]),
    "dllm_qparams_from_bincode": (INT, [P, S, INT, P, P]),
    "dllm_qparams_to_json": (INT, [P, P, S, P]),
    "dllm_qparams_from_json": (INT, [P, S, P]),
    "dllm_qtensor_to_bincode": (INT, [P, S, P, S, P, P, S, P]),
    "dllm_qtensor_from_bincode": (INT, [P, S, INT, P, S, P, P, S, P, P]),
    "dllm_qtensor_to_json": (INT, [P, S, P, S, P, P, S, P]),
    "dllm_qtensor_from_json": (INT, [P, S, P, S, P, P, S, P, P]),
    "dllm_compressed_vector_to_bincode": (INT, [P, S, P, S, U8, P, S, FL, FL, P, S, P]),
    "dllm_compressed_vector_from_bincode": (INT, [P, S, INT, P, S, P, P, S, P, P, P, S, P, P, P]),
    "dllm_compressed_vector_to_json": (INT, [P, S, P, S, U8, P, S, FL, FL, P, S, P]),
    "dllm_compressed_vector_from_json": (INT, [P, S, P, S, P, P, S, P, P, P, S, P, P, P]),
    "dllm_linear_forward_host": (INT, [P, P, S, P]),
}

# Exported only by the lab build (lib/libdllm_hip_lab.so, `make -C diffusion-llm-rs_amd/csrc lab`):
# schedule variants and ablation masks for A/B measurement scripts.
LAB_SIGNATURES = {
    "dllm_linear_set_kernel_variant": (INT, [P, INT]),
}
LAB_LIB_PATH = PKG_DIR / "lib" / "libdllm_hip_lab.so"

_lib = None


def load(path: str | os.PathLike | None = None):
    """Loads libdllm_hip.so (raises if absent: there is no CPU fallback).  No environment variable
    is read: the product library is the one in lib/.  ``path`` loads another build of the same ABI
    and returns it without installing it (``use`` installs one: measurement scripts only)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise ImportError(f"{p} not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
                          f"(or make -C diffusion-llm-rs_amd/csrc)")
    lib = C.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    for name, (res, args) in LAB_SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    if path is None:
        _lib = lib
    return lib


def use(path: str | os.PathLike):
    """Installs another build of the same ABI (the lab build, an A/B variant) as the library every
    call of this process goes to.  Measurement scripts and the lab tests call it explicitly."""
    global _lib
    _lib = load(path)
    return _lib


def check(rc: int):
    if rc != OK:
        msg = load().dllm_last_error().decode(errors="replace")
        raise _ERRORS.get(rc, QuantizationError)(f"[{rc}] {msg}", rc)
    return rc
