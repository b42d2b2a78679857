"""Mirror of ``diffuse_llm_rs::quantization`` (diffuse-llm-rs/src/quantization.rs) on the GPU.

Same names, argument meaning and error behaviour as the Rust module; data lives in HBM as torch
tensors and every computation is a HIP kernel behind the C-ABI (include/dllm_quant.h).
Differences forced by the device boundary are documented per item (e.g. scale/zero_point stay
on the device as a 2-float tensor until read, so nothing synchronises the stream).
"""
from __future__ import annotations

import math
import threading
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import check


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


def _dev(t: torch.Tensor, dtype=None) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(np.asarray(t))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if not t.is_cuda:
        t = t.cuda()
    return t.contiguous()


def packed_bytes(n: int, bits: int) -> int:
    return (n * bits + 7) // 8


def quantize_tensor(data: torch.Tensor, bits: int, packed: bool = False):
    """quantization.rs:38-68 ``quantize_tensor(data, bits) -> (Vec<u8>, f32, f32)``.

    Returns ``(codes, params)``: codes u8 (one per element, or the packed bitstream when
    ``packed``), params = device f32[2] {scale, zero_point}.  ``bits`` outside 1..=8 raises
    InvalidParams (the reference's ``assert!``, :39).
    """
    if not 1 <= int(bits) <= 8:
        raise _lib.InvalidParams("Bits must be between 1 and 8")
    x = _dev(data, torch.float32).reshape(-1)
    n = x.numel()
    out = torch.empty(packed_bytes(n, bits) if packed else n, dtype=torch.uint8, device=x.device)
    params = torch.empty(2, dtype=torch.float32, device=x.device)
    L = _lib.load()
    ws_bytes = L.dllm_quantize_tensor_workspace(n)
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=x.device)
    check(L.dllm_quantize_tensor(_ptr(x) if n else None, n, bits, int(packed), _ptr(out) if out.numel() else None,
                                 _ptr(params), _ptr(ws), ws.numel(), _stream()))
    return out, params


def quantize_tensor_pair(data: torch.Tensor, bits_a: int, bits_b: int, packed: bool = False):
    """:func:`quantize_tensor` of the same data at two widths in one min/max pass and one read
    (KVCacheEntry::update's prefill and decode copies, diffuse-llm-rs/src/lib.rs:241-276).
    Returns ``((codes_a, params_a), (codes_b, params_b))``, bit-identical to two calls."""
    for b in (bits_a, bits_b):
        if not 1 <= int(b) <= 8:
            raise _lib.InvalidParams("Bits must be between 1 and 8")
    x = _dev(data, torch.float32).reshape(-1)
    n = x.numel()
    outs = [torch.empty(packed_bytes(n, b) if packed else n, dtype=torch.uint8, device=x.device)
            for b in (bits_a, bits_b)]
    params = [torch.empty(2, dtype=torch.float32, device=x.device) for _ in range(2)]
    L = _lib.load()
    ws = torch.empty(max(L.dllm_quantize_tensor_workspace(n), 16), dtype=torch.uint8, device=x.device)
    ptr = lambda t: _ptr(t) if t.numel() else None  # noqa: E731
    check(L.dllm_quantize_tensor_pair(_ptr(x) if n else None, n, bits_a, bits_b, int(packed), ptr(outs[0]),
                                      _ptr(params[0]), ptr(outs[1]), _ptr(params[1]), _ptr(ws), ws.numel(),
                                      _stream()))
    return (outs[0], params[0]), (outs[1], params[1])


def _kv_outs(nk: int, nv: int, bits, packed: bool, device):
    mk = lambda n, b: torch.empty(packed_bytes(n, b) if packed else n, dtype=torch.uint8, device=device)  # noqa: E731
    return [(mk(nk, b), torch.empty(2, dtype=torch.float32, device=device),
             mk(nv, b), torch.empty(2, dtype=torch.float32, device=device)) for b in bits]


def _kv_args(outs):
    ptr = lambda t: _ptr(t) if t.numel() else None  # noqa: E731
    (ka, kpa, va, vpa) = outs[0]
    b = outs[1] if len(outs) > 1 else (None, None, None, None)
    pb = [None if t is None else (ptr(t) if t.dtype == torch.uint8 else _ptr(t)) for t in b]
    return [ptr(ka), _ptr(kpa), ptr(va), _ptr(vpa), pb[0], pb[1], pb[2], pb[3]]


def quantize_kv(keys: torch.Tensor, values: torch.Tensor, bits_a: int, bits_b: int = 0, packed: bool = True):
    """QuantizedKVCacheEntry::new (quantization.rs:140-157) -- K and V each quantized per tensor --
    at one width, or (``bits_b``) at two widths of the same K/V (KVCacheEntry::update's copies,
    lib.rs:241-276), through dllm_quantize_kv: min/max K | map K + min/max V | map V.  Returns one
    ``(k_codes, k_params, v_codes, v_params)`` per width, bit-identical to quantize_tensor[_pair]."""
    bits = [int(bits_a)] + ([int(bits_b)] if bits_b else [])
    for b in bits:
        if not 1 <= b <= 8:
            raise _lib.InvalidParams("Bits must be between 1 and 8")
    k = _dev(keys, torch.float32).reshape(-1)
    v = _dev(values, torch.float32).reshape(-1)
    nk, nv = k.numel(), v.numel()
    outs = _kv_outs(nk, nv, bits, packed, k.device)
    L = _lib.load()
    ws = torch.empty(max(L.dllm_quantize_kv_workspace(nk, nv), 16), dtype=torch.uint8, device=k.device)
    check(L.dllm_quantize_kv(_ptr(k) if nk else None, nk, _ptr(v) if nv else None, nv, bits[0],
                             bits[1] if len(bits) > 1 else 0, int(packed), *_kv_args(outs), _ptr(ws), ws.numel(),
                             _stream()))
    return outs


def kv_extremes(keys: torch.Tensor, values: torch.Tensor) -> torch.Tensor:
    """dllm_kv_extremes: device f32[4] {-min_K, max_K, -min_V, max_V} (NaN-ignoring fold of
    quantization.rs:41-46) -- the operand of a head-sharded cache's one all_reduce(MAX)."""
    k = _dev(keys, torch.float32).reshape(-1)
    v = _dev(values, torch.float32).reshape(-1)
    nk, nv = k.numel(), v.numel()
    red = torch.empty(4, dtype=torch.float32, device=k.device)
    L = _lib.load()
    ws = torch.empty(max(L.dllm_quantize_kv_workspace(nk, nv), 16), dtype=torch.uint8, device=k.device)
    check(L.dllm_kv_extremes(_ptr(k) if nk else None, nk, _ptr(v) if nv else None, nv, _ptr(red), _ptr(ws),
                             ws.numel(), _stream()))
    return red


def quantize_kv_with_extremes(keys: torch.Tensor, values: torch.Tensor, red: torch.Tensor, bits_a: int,
                              bits_b: int = 0, packed: bool = True):
    """The codes and params :func:`quantize_kv` writes, with the extremes given as ``red`` =
    {-min_K, max_K, -min_V, max_V} (already reduced over the ranks); one launch for K and V."""
    bits = [int(bits_a)] + ([int(bits_b)] if bits_b else [])
    for b in bits:
        if not 1 <= b <= 8:
            raise _lib.InvalidParams("Bits must be between 1 and 8")
    k = _dev(keys, torch.float32).reshape(-1)
    v = _dev(values, torch.float32).reshape(-1)
    nk, nv = k.numel(), v.numel()
    outs = _kv_outs(nk, nv, bits, packed, k.device)
    check(_lib.load().dllm_quantize_kv_with_extremes(_ptr(k) if nk else None, nk, _ptr(v) if nv else None, nv,
                                                     _ptr(_dev(red, torch.float32)), bits[0],
                                                     bits[1] if len(bits) > 1 else 0, int(packed), *_kv_args(outs),
                                                     _stream()))
    return outs


def bias_cast(y: torch.Tensor, bias: torch.Tensor | None, out_dtype=torch.float16, out: torch.Tensor | None = None):
    """dllm_bias_cast: ``y + bias`` (f32) stored as ``out_dtype`` -- a row-parallel layer's epilogue
    after its partial sums are reduced (diffuse-llm-rs/src/lib.rs:812).  ``y`` must be a contiguous
    2-D f32 device tensor and the output f16 or f32 (the kernel's two store types); anything else
    raises ``UnsupportedOperation`` / ``ShapeMismatch`` rather than storing the wrong element size."""
    if y.dim() != 2 or y.dtype != torch.float32 or not y.is_cuda or not y.is_contiguous():
        raise _lib.UnsupportedOperation("bias_cast: y must be a contiguous 2-D float32 device tensor")
    M, N = y.shape
    dtype = out.dtype if out is not None else out_dtype
    if dtype not in (torch.float16, torch.float32):
        raise _lib.UnsupportedOperation(f"bias_cast: output dtype {dtype} (only float16 / float32)")
    if out is None:
        out = torch.empty(M, N, dtype=dtype, device=y.device)
    elif tuple(out.shape) != (M, N) or not out.is_contiguous() or out.device != y.device:
        raise _lib.ShapeMismatch(f"bias_cast: out must be a contiguous [{M}, {N}] tensor on {y.device}")
    dt = _lib.F16 if dtype == torch.float16 else _lib.F32
    b = None if bias is None else _dev(bias, torch.float32)
    if b is not None and b.numel() != N:
        raise _lib.ShapeMismatch(f"bias_cast: bias has {b.numel()} elements, y has {N} columns")
    check(_lib.load().dllm_bias_cast(_ptr(y), M, N, None if b is None else _ptr(b), _ptr(out), dt, _stream()))
    return out


def tensor_extremes(data: torch.Tensor, stats: torch.Tensor | None = None) -> torch.Tensor:
    """The extremes fold of quantization.rs:41-46 (NaN-ignoring) as a device f32[2] {min, max},
    folded into ``stats`` when given (seed {+inf, -inf}).  First half of :func:`quantize_tensor`
    split at its reduction, for tensors sharded over ranks (``parallel.HeadParallelKVCache``)."""
    x = _dev(data, torch.float32).reshape(-1)
    if stats is None:
        stats = torch.tensor([math.inf, -math.inf], dtype=torch.float32, device=x.device)
    n = x.numel()
    if n:
        L = _lib.load()
        ws = torch.empty(max(L.dllm_quantize_tensor_workspace(n), 16), dtype=torch.uint8, device=x.device)
        check(L.dllm_tensor_extremes(_ptr(x), n, _ptr(stats), _ptr(ws), ws.numel(), _stream()))
    return stats


def quantize_params_from_extremes(stats: torch.Tensor, bits: int) -> torch.Tensor:
    """quantization.rs:49-56: device params {scale, zero_point} from device extremes {min, max}."""
    if not 1 <= int(bits) <= 8:
        raise _lib.InvalidParams("Bits must be between 1 and 8")
    st = _dev(stats, torch.float32)
    params = torch.empty(2, dtype=torch.float32, device=st.device)
    check(_lib.load().dllm_quantize_params_from_extremes(_ptr(st), bits, _ptr(params), _stream()))
    return params


def quantize_tensor_with_params(data: torch.Tensor, bits: int, params: torch.Tensor, packed: bool = False):
    """quantization.rs:59-65 with given device params: the codes :func:`quantize_tensor` writes once
    the params are known.  Returns the codes (one per byte, or the packed bitstream)."""
    if not 1 <= int(bits) <= 8:
        raise _lib.InvalidParams("Bits must be between 1 and 8")
    x = _dev(data, torch.float32).reshape(-1)
    n = x.numel()
    pr = _dev(params, torch.float32)
    out = torch.empty(packed_bytes(n, bits) if packed else n, dtype=torch.uint8, device=x.device)
    check(_lib.load().dllm_quantize_tensor_with_params(_ptr(x) if n else None, n, bits, int(packed), _ptr(pr),
                                                       _ptr(out) if out.numel() else None, _stream()))
    return out


def quantize_tensor_pair_with_params(data: torch.Tensor, bits_a: int, bits_b: int, params_a: torch.Tensor,
                                     params_b: torch.Tensor, packed: bool = False):
    """:func:`quantize_tensor_with_params` at two widths in one read of ``data`` (the prefill and
    decode copies of a head-sharded KVCacheEntry::update, diffuse-llm-rs/src/lib.rs:246-276).
    Returns ``(codes_a, codes_b)``, bit-identical to two single-width calls."""
    for b in (bits_a, bits_b):
        if not 1 <= int(b) <= 8:
            raise _lib.InvalidParams("Bits must be between 1 and 8")
    x = _dev(data, torch.float32).reshape(-1)
    n = x.numel()
    pa, pb = _dev(params_a, torch.float32), _dev(params_b, torch.float32)
    outs = [torch.empty(packed_bytes(n, b) if packed else n, dtype=torch.uint8, device=x.device) for b in (bits_a, bits_b)]
    ptr = lambda t: _ptr(t) if t.numel() else None  # noqa: E731
    check(_lib.load().dllm_quantize_tensor_pair_with_params(_ptr(x) if n else None, n, bits_a, bits_b, int(packed),
                                                            _ptr(pa), _ptr(pb), ptr(outs[0]), ptr(outs[1]),
                                                            _stream()))
    return outs[0], outs[1]


def dequantize_tensor(codes: torch.Tensor, scale, zero_point=None, *, bits: int = 8, packed: bool = False,
                      n: int | None = None, out_dtype=torch.float32) -> torch.Tensor:
    """quantization.rs:81-85 ``dequantize_tensor(data, scale, zero_point)``.

    ``scale`` may be the device params tensor returned by :func:`quantize_tensor` (then
    ``zero_point`` is None) or a host float (the literal Rust signature).
    """
    q = _dev(codes, torch.uint8).reshape(-1)
    if n is None:
        if packed:
            raise _lib.InvalidParams("n is required for packed codes")
        n = q.numel()
    out = torch.empty(n, dtype=out_dtype, device=q.device)
    dt = _lib.F32 if out_dtype == torch.float32 else _lib.F16
    L = _lib.load()
    if isinstance(scale, torch.Tensor) and zero_point is None:
        params = _dev(scale, torch.float32)
        check(L.dllm_dequantize_tensor(_ptr(q), n, bits, int(packed), _ptr(params), _ptr(out), dt, _stream()))
    else:
        check(L.dllm_dequantize_tensor_scalar(_ptr(q), n, bits, int(packed), float(scale), float(zero_point),
                                              _ptr(out), dt, _stream()))
    return out


def pack(codes: torch.Tensor, bits: int) -> torch.Tensor:
    """LSB-first bitstream packing (build-defined; size contract quantization.rs:122)."""
    c = _dev(codes, torch.uint8).reshape(-1)
    out = torch.empty(packed_bytes(c.numel(), bits), dtype=torch.uint8, device=c.device)
    check(_lib.load().dllm_pack(_ptr(c), c.numel(), bits, _ptr(out), _stream()))
    return out


def unpack(packed_codes: torch.Tensor, n: int, bits: int) -> torch.Tensor:
    p = _dev(packed_codes, torch.uint8).reshape(-1)
    out = torch.empty(n, dtype=torch.uint8, device=p.device)
    check(_lib.load().dllm_unpack(_ptr(p), n, bits, _ptr(out), _stream()))
    return out


def compression_ratio(numel: int, length: int, bits: int) -> float:
    """quantization.rs:120-124."""
    return float(_lib.load().dllm_compression_ratio(numel, length, bits))


@dataclass
class QuantizedTensor:
    """quantization.rs:88-125 ``QuantizedTensor {data, shape, scale, zero_point, bits}``.

    ``data`` holds the codes in the packed bitstream (``packed=True``, the size the reference's
    accounting assumes) or one code per byte; ``params`` = device {scale, zero_point}.
    """

    data: torch.Tensor
    shape: tuple
    params: torch.Tensor
    bits: int
    packed: bool = True

    @classmethod
    def new(cls, data, shape, scale, zero_point, bits, packed=False):
        """quantization.rs:104-112 (host scale / zero_point)."""
        d = _dev(data, torch.uint8)
        params = torch.tensor([float(scale), float(zero_point)], dtype=torch.float32, device=d.device)
        return cls(d, tuple(shape), params, int(bits), packed)

    @classmethod
    def quantize(cls, t: torch.Tensor, bits: int, packed: bool = True):
        codes, params = quantize_tensor(t, bits, packed=packed)
        return cls(codes, tuple(t.shape), params, int(bits), packed)

    def numel(self) -> int:
        return math.prod(self.shape)

    @property
    def scale(self) -> float:
        return float(self.params[0].item())

    @property
    def zero_point(self) -> float:
        return float(self.params[1].item())

    def dequantize(self, out_dtype=torch.float32) -> torch.Tensor:
        """quantization.rs:115-117."""
        return dequantize_tensor(self.data, self.params, bits=self.bits, packed=self.packed, n=self.numel(),
                                 out_dtype=out_dtype)

    def codes(self) -> torch.Tensor:
        """One code per byte (the reference's ``data`` field)."""
        return unpack(self.data, self.numel(), self.bits) if self.packed else self.data

    def compression_ratio(self) -> float:
        """quantization.rs:120-124: ``(prod(shape) * 4) / ceil(len * bits / 8)``."""
        return compression_ratio(self.numel(), self.numel(), self.bits)

    def clone(self) -> "QuantizedTensor":
        return QuantizedTensor(self.data.clone(), self.shape, self.params.clone(), self.bits, self.packed)


@dataclass
class QuantizedKVCacheEntry:
    """quantization.rs:128-176: K and V each quantized per tensor (own scale / zero point)."""

    keys: QuantizedTensor
    values: QuantizedTensor
    seq_len: int = field(default=0)

    @classmethod
    def new(cls, keys: torch.Tensor, values: torch.Tensor, bits: int, packed: bool = True):
        """quantization.rs:140-157 (keys/values are [num_layers, seq, hidden])."""
        (kc, kp, vc, vp), = quantize_kv(keys, values, bits, 0, packed)
        ks, vs = tuple(keys.shape), tuple(values.shape)
        return cls(QuantizedTensor(kc, ks, kp, int(bits), packed), QuantizedTensor(vc, vs, vp, int(bits), packed),
                   int(keys.shape[1]) if keys.dim() > 1 else 0)

    @classmethod
    def new_pair(cls, keys: torch.Tensor, values: torch.Tensor, bits_a: int, bits_b: int, packed: bool = True):
        """``new(keys, values, bits_a)`` and ``new(keys, values, bits_b)`` in one pass per tensor
        (:func:`quantize_tensor_pair`); bit-identical to the two separate calls."""
        seq = int(keys.shape[1]) if keys.dim() > 1 else 0
        (ka, pka, va, pva), (kb, pkb, vb, pvb) = quantize_kv(keys, values, bits_a, bits_b, packed)
        ks, vs = tuple(keys.shape), tuple(values.shape)
        return (cls(QuantizedTensor(ka, ks, pka, int(bits_a), packed), QuantizedTensor(va, vs, pva, int(bits_a), packed), seq),
                cls(QuantizedTensor(kb, ks, pkb, int(bits_b), packed), QuantizedTensor(vb, vs, pvb, int(bits_b), packed), seq))

    def dequantize_keys(self, out_dtype=torch.float32) -> torch.Tensor:
        """quantization.rs:160-166."""
        return self.keys.dequantize(out_dtype).reshape(self.keys.shape)

    def dequantize_values(self, out_dtype=torch.float32) -> torch.Tensor:
        """quantization.rs:169-175."""
        return self.values.dequantize(out_dtype).reshape(self.values.shape)

    def clone(self) -> "QuantizedKVCacheEntry":
        return QuantizedKVCacheEntry(self.keys.clone(), self.values.clone(), self.seq_len)

    def memory_usage(self) -> int:
        """Packed bytes of K and V (the accounting of diffuse-llm-rs/src/lib.rs:279-302)."""
        return sum(packed_bytes(t.numel(), t.bits) for t in (self.keys, self.values))


def kv_attention(q: torch.Tensor, keys: QuantizedTensor, values: QuantizedTensor) -> torch.Tensor:
    """Quantized-KV dequant-attention (a9): O = softmax(Q K^T / sqrt(D)) V per head with K, V the
    per-tensor quantized cache tensors of ``QuantizedKVCacheEntry`` (packed, 4 or 8 bits),
    dequantized inside the kernel.  q: f16 [S, H, 128] -> O f16 [S, H, 128]."""
    if q.dim() != 3:
        raise _lib.ShapeMismatch("q must be [S, H, D]")
    S, H, D = q.shape
    for t in (keys, values):
        if not t.packed or t.numel() != S * H * D:
            raise _lib.ShapeMismatch("keys/values must be packed [S, H, D] QuantizedTensors")
    if keys.bits != values.bits:
        raise _lib.InvalidParams("keys and values must share the bit width")
    qd = _dev(q, torch.float16)
    out = torch.empty(S, H, D, dtype=torch.float16, device=qd.device)
    check(_lib.load().dllm_kv_attention(_ptr(qd), _ptr(keys.data), _ptr(keys.params), _ptr(values.data),
                                        _ptr(values.params), keys.bits, S, H, D, _ptr(out), _stream()))
    return out


class AdaptiveQuantizer:
    """``AdaptiveQuantizer`` (quantization.rs:178-235): bits, target_ratio, and running statistics
    behind a lock (the reference's ``Arc<Mutex<CKMS<f32>>>``).

    The statistics stay on the device as {min, max} (dllm_adaptive_update).  The reference queries
    its CKMS(0.01) summary only at q = 0.0 and q = 1.0 (:209-210); the exact extremes answer those
    queries with rank error 0, inside CKMS's eps*n bound.  NaN samples are skipped.  Parity is
    unpinned: the quantiles crate is absent.  ``target_ratio`` is stored and unused, as in the
    reference."""

    def __init__(self, bits: int, target_ratio: float, device="cuda"):
        self.bits, self.target_ratio = int(bits), float(target_ratio)
        self._lock = threading.Lock()
        self._stats = torch.tensor([math.inf, -math.inf], dtype=torch.float32, device=device)
        self._count = 0

    def update_stats(self, data) -> None:
        """:198-203 -- every element inserted into the summary."""
        x = _dev(data, torch.float32).reshape(-1)
        n = x.numel()
        if n == 0:
            return
        L = _lib.load()
        ws = torch.empty(max(L.dllm_quantize_tensor_workspace(n), 16), dtype=torch.uint8, device=x.device)
        with self._lock:
            check(L.dllm_adaptive_update(_ptr(x), n, _ptr(self._stats), _ptr(ws), ws.numel(), _stream()))
            self._count += n

    def compute_params_device(self) -> torch.Tensor:
        """:206-217 as a device f32[2] {scale, zero_point}; nothing synchronises the stream."""
        params = torch.empty(2, dtype=torch.float32, device=self._stats.device)
        with self._lock:
            check(_lib.load().dllm_adaptive_compute_params(_ptr(self._stats), int(self._count > 0), self.bits,
                                                           _ptr(params), _stream()))
        return params

    def compute_params(self) -> tuple[float, float]:
        """:206-217 ``-> (f32, f32)`` (reads the two floats back)."""
        s, z = self.compute_params_device().cpu().tolist()
        return s, z

    def quantize(self, data, packed: bool = False):
        """:220-234 ``-> (Vec<u8>, f32, f32)``: codes u8 (one per element, or the packed stream for
        1 <= bits <= 8) and the device params {scale, zero_point} used."""
        x = _dev(data, torch.float32).reshape(-1)
        n = x.numel()
        params = self.compute_params_device()
        out = torch.empty(packed_bytes(n, self.bits) if packed else n, dtype=torch.uint8, device=x.device)
        check(_lib.load().dllm_adaptive_quantize(_ptr(x) if n else None, n, self.bits, _ptr(params), int(packed),
                                                 _ptr(out) if out.numel() else None, _stream()))
        return out, params
