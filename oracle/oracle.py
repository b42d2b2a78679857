"""ctypes binding of the C oracle (oracle/_build/liborc.so).

TEST INFRASTRUCTURE ONLY: the parity checker and the CPU baseline.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liborc.so"

_lib = None


def build(force: bool = False) -> Path:
    srcs = [HERE / "dllm_oracle.c", HERE / "dllm_oracle_diffusion.c", HERE / "dllm_oracle.h", HERE / "dllm_sgemm.c"]
    newest = max(p.stat().st_mtime for p in srcs)
    if force or not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < newest:
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(LIB_PATH))
        P, S, F, U8, I32 = C.c_void_p, C.c_size_t, C.c_float, C.c_uint8, C.c_int32
        sig = {
            "orc_quantize_tensor": (C.c_int, [P, S, U8, P, P, P]),
            "orc_dequantize_tensor": (None, [P, S, F, F, P]),
            "orc_compression_ratio": (F, [S, S, U8]),
            "orc_packed_bytes": (S, [S, U8]),
            "orc_pack_bits": (C.c_int, [P, S, U8, P]),
            "orc_unpack_bits": (C.c_int, [P, S, U8, P]),
            "orc_default_quantize": (C.c_int, [P, S, C.c_int, F, I32, P]),
            "orc_default_dequantize": (None, [P, S, F, I32, P]),
            "orc_bit_quantize": (C.c_int, [P, S, C.c_uint32, F, F, P]),
            "orc_bit_dequantize": (None, [P, S, F, F, P]),
            "orc_prefill_scale": (C.c_int, [C.c_uint32, P]),
            "orc_quantize_vectors": (C.c_int, [P, S, S, P, S, P, S, P, P]),
            "orc_compress_vector": (C.c_int, [P, S, U8, P, P, P]),
            "orc_quantize_weights": (C.c_int, [P, S, S, U8, S, P, P, P]),
            "orc_dequantize_weights": (None, [P, P, P, S, S, S, P]),
            "orc_linear_forward": (None, [P, S, S, P, S, P, P, C.c_int]),
            "orc_sgemm_blocked": (C.c_int, [P, S, S, P, S, P, P, C.c_int]),
            "orc_attention": (None, [P, P, P, S, S, S, P, S, C.c_int]),
            "orc_beta_schedule": (C.c_int, [C.c_int, S, F, F, P]),
            "orc_alpha_bars": (C.c_int, [P, S, C.c_int, P, P]),
            "orc_p_sample_coeffs": (C.c_int, [P, S, C.c_int, C.c_int, P, S, P]),
            "orc_add_noise_coeffs": (C.c_int, [P, S, C.c_int, P, S, P]),
            "orc_randn": (None, [C.c_uint64, C.c_uint64, S, P]),
            "orc_p_sample": (None, [P, P, P, P, S, S, C.c_int, P]),
            "orc_add_noise": (None, [P, P, P, S, S, P]),
            "orc_adaptive_update": (None, [P, P, S]),
            "orc_adaptive_params": (C.c_int, [P, C.c_int, C.c_uint32, P, P]),
            "orc_adaptive_quantize": (C.c_int, [P, S, C.c_uint32, F, F, P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class OracleError(RuntimeError):
    pass


def _check(rc):
    if rc != 0:
        raise OracleError(f"oracle returned {rc}")


def quantize_tensor(x: np.ndarray, bits: int):
    x = np.ascontiguousarray(x, np.float32).ravel()
    q = np.zeros(x.size, np.uint8)
    s, z = C.c_float(), C.c_float()
    _check(lib().orc_quantize_tensor(_p(x), x.size, bits, _p(q), C.byref(s), C.byref(z)))
    return q, np.float32(s.value), np.float32(z.value)


def dequantize_tensor(q, scale, zp):
    q = np.ascontiguousarray(q, np.uint8).ravel()
    out = np.zeros(q.size, np.float32)
    lib().orc_dequantize_tensor(_p(q), q.size, float(scale), float(zp), _p(out))
    return out


def pack_bits(codes, bits):
    codes = np.ascontiguousarray(codes, np.uint8).ravel()
    out = np.zeros(lib().orc_packed_bytes(codes.size, bits), np.uint8)
    _check(lib().orc_pack_bits(_p(codes), codes.size, bits, _p(out)))
    return out


def unpack_bits(packed, n, bits):
    packed = np.ascontiguousarray(packed, np.uint8).ravel()
    out = np.zeros(n, np.uint8)
    _check(lib().orc_unpack_bits(_p(packed), n, bits, _p(out)))
    return out


def default_quantize(x, qtype, scale=1.0, zero_point=0):
    x = np.ascontiguousarray(x, np.float32).ravel()
    out = np.zeros(x.size, np.uint8)
    _check(lib().orc_default_quantize(_p(x), x.size, qtype, scale, zero_point, _p(out)))
    return out


def default_dequantize(q, scale=1.0, zero_point=0):
    q = np.ascontiguousarray(q, np.uint8).ravel()
    out = np.zeros(q.size, np.float32)
    lib().orc_default_dequantize(_p(q), q.size, scale, zero_point, _p(out))
    return out


def bit_quantize(x, bits, scale, zero_point):
    x = np.ascontiguousarray(x, np.float32).ravel()
    out = np.zeros(x.size, np.uint8)
    _check(lib().orc_bit_quantize(_p(x), x.size, bits, scale, zero_point, _p(out)))
    return out


def bit_dequantize(q, scale, zero_point):
    q = np.ascontiguousarray(q, np.uint8).ravel()
    out = np.zeros(q.size, np.float32)
    lib().orc_bit_dequantize(_p(q), q.size, scale, zero_point, _p(out))
    return out


def prefill_scale(bits):
    s = C.c_float()
    _check(lib().orc_prefill_scale(bits, C.byref(s)))
    return np.float32(s.value)


def quantize_vectors(x, cfg_bits, req_bits):
    x = np.ascontiguousarray(x, np.float32)
    rows, dim = x.shape
    cfg = np.ascontiguousarray(cfg_bits, np.uint8)
    req = np.ascontiguousarray(req_bits, np.uint8)
    out = np.zeros((rows, dim), np.uint8)
    widths = np.zeros(rows, np.uint8)
    _check(lib().orc_quantize_vectors(_p(x), rows, dim, _p(cfg), cfg.size, _p(req), req.size, _p(out),
                                      _p(widths)))
    return out, widths


def compress_vector(x, bits):
    x = np.ascontiguousarray(x, np.float32).ravel()
    out = np.zeros(x.size, np.uint8)
    s, z = C.c_float(), C.c_float()
    _check(lib().orc_compress_vector(_p(x), x.size, bits, _p(out), C.byref(s), C.byref(z)))
    return out, np.float32(s.value), np.float32(z.value)


def quantize_weights(W, bits=4, group=128):
    W = np.ascontiguousarray(W, np.float32)
    K, N = W.shape
    G = (K + group - 1) // group
    codes = np.zeros((K, N), np.uint8)
    scales = np.zeros((G, N), np.float32)
    zps = np.zeros((G, N), np.uint8)
    _check(lib().orc_quantize_weights(_p(W), K, N, bits, group, _p(codes), _p(scales), _p(zps)))
    return codes, scales, zps


def dequantize_weights(codes, scales, zps, group=128):
    codes = np.ascontiguousarray(codes, np.uint8)
    K, N = codes.shape
    out = np.zeros((K, N), np.float32)
    lib().orc_dequantize_weights(_p(codes), _p(np.ascontiguousarray(scales, np.float32)),
                                 _p(np.ascontiguousarray(zps, np.uint8)), K, N, group, _p(out))
    return out


def linear_forward(X, W, bias=None, nthreads=1):
    X = np.ascontiguousarray(X, np.float32)
    W = np.ascontiguousarray(W, np.float32)
    M, K = X.shape
    N = W.shape[1]
    Y = np.zeros((M, N), np.float32)
    b = None if bias is None else np.ascontiguousarray(bias, np.float32)
    lib().orc_linear_forward(_p(X), M, K, _p(W), N, None if b is None else _p(b), _p(Y), nthreads)
    return Y


def sgemm_blocked(X, W, bias=None, nthreads=1):
    """Y = X . W + bias by the blocked AVX2/FMA GEMM (dllm_sgemm.c): the CPU baseline's GEMM, of
    the class ndarray's dot runs (matrixmultiply).  Not a parity restatement (FMA, blocked order)."""
    X = np.ascontiguousarray(X, np.float32)
    W = np.ascontiguousarray(W, np.float32)
    M, K = X.shape
    N = W.shape[1]
    Y = np.empty((M, N), np.float32)
    b = None if bias is None else np.ascontiguousarray(bias, np.float32)
    if lib().orc_sgemm_blocked(_p(X), M, K, _p(W), N, None if b is None else _p(b), _p(Y), nthreads) != 0:
        raise RuntimeError("orc_sgemm_blocked: no AVX2/FMA on this host or allocation failed")
    return Y


def attention_rows(Qsel, K, V):
    """f64 SDPA softmax(q K^T / sqrt(D)) V (bidirectional, the a9 consumer's definition) for a
    selection of query rows Qsel [R, H, D] against all keys K, V [S, H, D]: the same math as
    orc_attention, for rows sampled across a long sequence."""
    Qs = np.asarray(Qsel, np.float64)
    R, H, D = Qs.shape
    out = np.empty((R, H, D), np.float64)
    inv = 1.0 / np.sqrt(D)
    for h in range(H):
        s = (Qs[:, h, :] @ np.asarray(K[:, h, :], np.float64).T) * inv
        s -= s.max(axis=1, keepdims=True)
        p = np.exp(s)
        out[:, h, :] = (p @ np.asarray(V[:, h, :], np.float64)) / p.sum(axis=1, keepdims=True)
    return out


def attention(Q, K, V, q_rows=None, nthreads=None):
    Q, K, V = (np.ascontiguousarray(a, np.float32) for a in (Q, K, V))
    S, H, D = Q.shape
    q_rows = S if q_rows is None else q_rows
    O = np.zeros((q_rows, H, D), np.float32)
    nthreads = nthreads or (os.cpu_count() or 1)
    lib().orc_attention(_p(Q), _p(K), _p(V), S, H, D, _p(O), q_rows, nthreads)
    return O


# ---- 8f rank 1: diffusion-step ops -------------------------------------------------------------
BETA_LINEAR, BETA_QUADRATIC, BETA_COSINE = 0, 1, 2


def beta_schedule(kind, T, beta_start=0.0001, beta_end=0.02):
    out = np.zeros(T, np.float32)
    _check(lib().orc_beta_schedule(kind, T, beta_start, beta_end, _p(out)))
    return out


def alpha_bars(betas, inclusive):
    betas = np.ascontiguousarray(betas, np.float32)
    a = np.zeros(betas.size, np.float32)
    ab = np.zeros(betas.size, np.float32)
    _check(lib().orc_alpha_bars(_p(betas), betas.size, int(inclusive), _p(a), _p(ab)))
    return a, ab


def p_sample_coeffs(betas, t, inclusive=False, literal_alphas=False):
    betas = np.ascontiguousarray(betas, np.float32)
    t = np.ascontiguousarray(t, np.uint64)
    coef = np.zeros((t.size, 3), np.float32)
    _check(lib().orc_p_sample_coeffs(_p(betas), betas.size, int(inclusive), int(literal_alphas), _p(t), t.size,
                                     _p(coef)))
    return coef


def add_noise_coeffs(betas, t, inclusive=False):
    betas = np.ascontiguousarray(betas, np.float32)
    t = np.ascontiguousarray(t, np.uint64)
    coef = np.zeros((t.size, 2), np.float32)
    _check(lib().orc_add_noise_coeffs(_p(betas), betas.size, int(inclusive), _p(t), t.size, _p(coef)))
    return coef


def randn(seed, offset, n):
    out = np.zeros(n, np.float32)
    lib().orc_randn(seed, offset, n, _p(out))
    return out


def p_sample(x_t, eps, noise, coef, add_noise=True):
    x_t = np.ascontiguousarray(x_t, np.float32)
    B, D = x_t.shape
    eps = np.ascontiguousarray(eps, np.float32)
    noise = np.zeros_like(x_t) if noise is None else np.ascontiguousarray(noise, np.float32)
    out = np.zeros_like(x_t)
    lib().orc_p_sample(_p(x_t), _p(eps), _p(noise), _p(np.ascontiguousarray(coef, np.float32)), B, D,
                       int(add_noise), _p(out))
    return out


def add_noise(x0, noise, coef):
    x0 = np.ascontiguousarray(x0, np.float32)
    B, D = x0.shape
    out = np.zeros_like(x0)
    lib().orc_add_noise(_p(x0), _p(np.ascontiguousarray(noise, np.float32)),
                        _p(np.ascontiguousarray(coef, np.float32)), B, D, _p(out))
    return out


# ---- 8f rank 4: AdaptiveQuantizer (diffuse-llm-rs/src/quantization.rs:178-235) ---------------

class AdaptiveQuantizer:
    """Oracle mirror of the reference's AdaptiveQuantizer (CKMS q = 0 / 1 as exact extremes)."""

    def __init__(self, bits: int, target_ratio: float = 4.0):
        self.bits, self.target_ratio = bits, target_ratio
        self.minmax = np.array([np.inf, -np.inf], np.float32)
        self.count = 0

    def update_stats(self, data):
        x = np.ascontiguousarray(data, np.float32).ravel()
        lib().orc_adaptive_update(_p(self.minmax), _p(x), x.size)
        self.count += x.size

    def compute_params(self):
        s, z = C.c_float(), C.c_float()
        _check(lib().orc_adaptive_params(_p(self.minmax), int(self.count > 0), self.bits, C.byref(s), C.byref(z)))
        return np.float32(s.value), np.float32(z.value)

    def quantize(self, data):
        x = np.ascontiguousarray(data, np.float32).ravel()
        s, z = self.compute_params()
        out = np.zeros(x.size, np.uint8)
        _check(lib().orc_adaptive_quantize(_p(x), x.size, self.bits, float(s), float(z), _p(out)))
        return out, s, z


# ---- 8f rank 2: phase-aware KV cache + progressive precision (diffuse-llm-rs/src/lib.rs) --------

def progressive_bits(decode_bits: int, min_decode_bits: int, num_steps: int, t: int) -> int:
    """lib.rs:890-897: progress = (num_steps - t) as f32 / (num_steps / 2) as f32;
    target = (decode * (1 - progress) + min * progress) as u8 -- f32 ops, each rounded, and the
    saturating `as u8` (negative -> 0, NaN -> 0, truncation toward zero)."""
    f = np.float32
    progress = f(f(num_steps - t) / f(num_steps // 2))
    v = f(f(f(decode_bits) * f(f(1.0) - progress)) + f(f(min_decode_bits) * progress))
    if not np.isfinite(v):
        return 0 if np.isnan(v) else (255 if v > 0 else 0)
    return int(min(max(int(np.trunc(v)), 0), 255))


class KVCacheEntryRef:
    """Oracle restatement of KVCacheEntry (lib.rs:121-313) over host f32 K/V and the C oracle's
    quantize_tensor / dequantize_tensor (QuantizedKVCacheEntry::new quantizes K and V per tensor,
    quantization.rs:140-157): an Option<(codes, scale, zp)> per tensor and phase."""

    def __init__(self, keys, values, prefill_bits, decode_bits):
        self.keys = np.ascontiguousarray(keys, np.float32)
        self.values = np.ascontiguousarray(values, np.float32)
        self.prefill_quant_bits, self.decode_quant_bits = int(prefill_bits), int(decode_bits)
        self.prefill_quantized = self._q(prefill_bits) if prefill_bits > 0 else None    # :145-153
        self.decode_quantized = self._q(decode_bits) if decode_bits > 0 else None       # :155-163
        self.is_prefill_phase = True

    def _q(self, bits):
        return (quantize_tensor(self.keys, bits), quantize_tensor(self.values, bits))

    def _get(self, which):                                                              # :178-208
        q = self.prefill_quantized if self.is_prefill_phase else self.decode_quantized
        src = self.keys if which == 0 else self.values
        if q is None:
            return src.copy()
        return dequantize_tensor(*q[which]).reshape(src.shape)

    def get_keys(self):
        return self._get(0)

    def get_values(self):
        return self._get(1)

    def set_phase(self, is_prefill):                                                    # :221-239
        if self.is_prefill_phase == is_prefill:
            return
        self.is_prefill_phase = is_prefill
        if not is_prefill and self.decode_quant_bits > 0 and self.decode_quantized is None:
            self.decode_quantized = self._q(self.decode_quant_bits)

    def update(self, keys, values):                                                     # :246-276
        self.keys = np.ascontiguousarray(keys, np.float32)
        self.values = np.ascontiguousarray(values, np.float32)
        if self.prefill_quant_bits > 0:
            self.prefill_quantized = self._q(self.prefill_quant_bits)
        if self.decode_quant_bits > 0:
            self.decode_quantized = self._q(self.decode_quant_bits)


def sample_kv_step(entry: KVCacheEntryRef, t: int, num_steps: int, decode_bits: int, min_decode_bits: int,
                   progressive: bool = True, phase_aware: bool = True):
    """The cache half of one DiffuseLLM::sample iteration (lib.rs:884-918) with the simple model's
    pass-through update_kv_cache (:826-835): phase switch, progressive decode bits, the K/V that
    forward_with_cache receives, then the re-quantizing update.  Returns (keys, values) given."""
    is_prefill = t > num_steps // 2                                                     # :886
    entry.set_phase(is_prefill)
    if phase_aware and progressive and not is_prefill:                                   # :890-903
        tb = progressive_bits(decode_bits, min_decode_bits, num_steps, t)
        if tb != entry.decode_quant_bits:
            entry.decode_quant_bits = tb
            entry.decode_quantized = None
    new_k, new_v = entry.keys, entry.values                                             # :907
    k, v = entry.get_keys(), entry.get_values()                                         # :913-914
    entry.update(new_k, new_v)                                                          # :918
    return k, v
