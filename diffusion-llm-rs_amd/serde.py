"""Wire formats of the quantized objects: what the reference's serde derives
produce for the checkpoint / hand-off structs, in both encodings its crates use.

* ``QuantizationParams``, ``QuantizedTensor`` -- quantization/src/types.rs:19-47 (#[derive(Serialize,
  Deserialize)]); the crate converts both bincode and serde_json errors (quantization/src/error.rs:44-53).
* ``PrefillCompressedVector`` -- diffusion_prefill/src/prefill_kv.rs:25-33 (the KV hand-off record
  with its per-vector quant_scale / quant_zero_point), built from ``kvquant.compress_vectors``.

Every encoder and decoder here is the library's C-ABI (csrc/serde.cpp, include/dllm_quant.h
section f3: bincode 1.3 legacy layout, serde_json compact form with ryu's f32 digits); this module
only moves host buffers across it.  Device tensors are copied to / from the host around it.  The
independent restatement that checks these bytes is ``oracle/serde_ref.py`` (tests only).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from . import _lib
from ._lib import check
from .quant import QuantizationParams, QuantizedTensor


class _QP(C.Structure):
    """``dllm_qparams``."""
    _fields_ = [("bits", C.c_uint8), ("scale", C.c_float), ("zero_point", C.c_int32), ("symmetric", C.c_uint8),
                ("has_axis", C.c_uint8), ("axis", C.c_uint64)]


def _qp(p: QuantizationParams) -> _QP:
    return _QP(int(p.bits), float(p.scale), int(p.zero_point), int(bool(p.symmetric)), 0 if p.axis is None else 1,
               0 if p.axis is None else int(p.axis))


def _params(q: _QP) -> QuantizationParams:
    return QuantizationParams(bits=int(q.bits), scale=float(np.float32(q.scale)), zero_point=int(q.zero_point),
                              symmetric=bool(q.symmetric), axis=int(q.axis) if q.has_axis else None)


def _emit(fn, *args) -> bytes:
    """An encoder call: size query, then the write."""
    n = C.c_size_t()
    check(fn(*args, None, 0, C.byref(n)))
    buf = C.create_string_buffer(max(1, n.value))
    check(fn(*args, buf, n.value, C.byref(n)))
    return buf.raw[: n.value]


def _u8(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, np.uint8).ravel())


def _shape(shape):
    return (C.c_uint64 * max(1, len(shape)))(*[int(s) for s in shape])


def ryu_f32(x) -> str:
    """serde_json's text of a finite f32 (ryu's shortest round-trip digits; dllm_format_f32)."""
    if not np.isfinite(np.float32(x)):
        raise ValueError("non-finite")
    return _emit(_lib.load().dllm_format_f32, C.c_float(float(x))).decode()


# ---- QuantizationParams ------------------------------------------------------------------------------

def params_to_bincode(p: QuantizationParams) -> bytes:
    q = _qp(p)
    return _emit(_lib.load().dllm_qparams_to_bincode, C.byref(q))


def params_from_bincode(b: bytes, strict: bool = False) -> QuantizationParams:
    """``bincode::deserialize`` (trailing bytes allowed, bincode 1.3 legacy options) or, with
    ``strict``, the DefaultOptions reader that rejects them."""
    q = _QP()
    check(_lib.load().dllm_qparams_from_bincode(bytes(b), len(b), int(strict), C.byref(q), None))
    return _params(q)


def params_to_json(p: QuantizationParams) -> str:
    q = _qp(p)
    return _emit(_lib.load().dllm_qparams_to_json, C.byref(q)).decode()


def params_from_json(s: str) -> QuantizationParams:
    b = s.encode()
    q = _QP()
    check(_lib.load().dllm_qparams_from_json(b, len(b), C.byref(q)))
    return _params(q)


# ---- QuantizedTensor (quantization crate) -------------------------------------------------------------

def _host_codes(t: QuantizedTensor) -> np.ndarray:
    d = t.data
    return _u8(d.detach().to("cpu").numpy() if isinstance(d, torch.Tensor) else d)


def qtensor_to_bincode(t: QuantizedTensor) -> bytes:
    codes, q = _host_codes(t), _qp(t.params)
    return _emit(_lib.load().dllm_qtensor_to_bincode, codes.ctypes.data, codes.size, _shape(t.shape), len(t.shape),
                 C.byref(q))


def qtensor_to_json(t: QuantizedTensor) -> str:
    codes, q = _host_codes(t), _qp(t.params)
    return _emit(_lib.load().dllm_qtensor_to_json, codes.ctypes.data, codes.size, _shape(t.shape), len(t.shape),
                 C.byref(q)).decode()


def _decode_tensor(fn, buf, extra, device) -> QuantizedTensor:
    n, nd, q = C.c_size_t(), C.c_size_t(), _QP()
    check(fn(buf, len(buf), *extra, None, 0, C.byref(n), None, 0, C.byref(nd), C.byref(q)))   # counts
    codes = np.zeros(max(1, n.value), np.uint8)
    shape = (C.c_uint64 * max(1, nd.value))()
    check(fn(buf, len(buf), *extra, codes.ctypes.data, codes.size, C.byref(n), shape, len(shape), C.byref(nd),
             C.byref(q)))
    return QuantizedTensor(torch.from_numpy(codes[: n.value].copy()).to(device), tuple(int(v) for v in shape[: nd.value]),
                           _params(q))


def qtensor_from_bincode(b: bytes, device="cuda", strict: bool = False) -> QuantizedTensor:
    return _decode_tensor(_lib.load().dllm_qtensor_from_bincode, bytes(b), (int(strict),), device)


def qtensor_from_json(s: str, device="cuda") -> QuantizedTensor:
    return _decode_tensor(_lib.load().dllm_qtensor_from_json, s.encode(), (), device)


# ---- diffusion_prefill CompressedVector ------------------------------------------------------------------

@dataclass
class PrefillCompressedVector:
    """diffusion_prefill/src/prefill_kv.rs:25-33 (codes one per byte, host array)."""
    id: str
    data: np.ndarray
    bits: int
    original_shape: List[int]
    quant_scale: float
    quant_zero_point: float

    def _args(self):
        idb, d = self.id.encode("utf-8"), _u8(self.data)
        return (idb, len(idb), d.ctypes.data, d.size, int(self.bits), _shape(self.original_shape),
                len(self.original_shape), C.c_float(self.quant_scale), C.c_float(self.quant_zero_point)), d

    def to_bincode(self) -> bytes:
        args, _keep = self._args()
        return _emit(_lib.load().dllm_compressed_vector_to_bincode, *args)

    def to_json(self) -> str:
        args, _keep = self._args()
        return _emit(_lib.load().dllm_compressed_vector_to_json, *args).decode()

    @classmethod
    def _decode(cls, fn, buf: bytes, extra) -> "PrefillCompressedVector":
        il, n, nb, nd, sc, zp = C.c_size_t(), C.c_size_t(), C.c_uint8(), C.c_size_t(), C.c_float(), C.c_float()
        tail = (C.byref(nb),)
        check(fn(buf, len(buf), *extra, None, 0, C.byref(il), None, 0, C.byref(n), *tail, None, 0, C.byref(nd),
                 C.byref(sc), C.byref(zp)))
        ib = C.create_string_buffer(max(1, il.value))
        data = np.zeros(max(1, n.value), np.uint8)
        shape = (C.c_uint64 * max(1, nd.value))()
        check(fn(buf, len(buf), *extra, ib, len(ib), C.byref(il), data.ctypes.data, data.size, C.byref(n), *tail,
                 shape, len(shape), C.byref(nd), C.byref(sc), C.byref(zp)))
        return cls(ib.raw[: il.value].decode("utf-8"), data[: n.value].copy(), int(nb.value),
                   [int(v) for v in shape[: nd.value]], float(np.float32(sc.value)), float(np.float32(zp.value)))

    @classmethod
    def from_bincode(cls, b: bytes, strict: bool = False) -> "PrefillCompressedVector":
        return cls._decode(_lib.load().dllm_compressed_vector_from_bincode, bytes(b), (int(strict),))

    @classmethod
    def from_json(cls, s) -> "PrefillCompressedVector":
        """``s``: the JSON text (str) or its bytes (serde_json::from_slice: not valid UTF-8 ->
        SerializationError)."""
        b = s if isinstance(s, (bytes, bytearray)) else s.encode("utf-8")
        return cls._decode(_lib.load().dllm_compressed_vector_from_json, bytes(b), ())


def compressed_vector_records(x: torch.Tensor, bits: int, ids: Optional[List[str]] = None) -> List[PrefillCompressedVector]:
    """KVCache::compress_vector over the rows of x (diffusion_prefill/src/prefill_kv.rs:104-121, on the
    GPU via kvquant.compress_vectors) as serialisable records."""
    from .kvquant import compress_vectors
    codes, scales, zps = compress_vectors(x, bits)
    codes, scales, zps = codes.cpu().numpy(), scales.cpu().numpy(), zps.cpu().numpy()
    rows = codes.shape[0]
    shape = [int(codes.shape[1])]       # vec![vector.len()] (prefill_kv.rs:117): the row's length
    ids = ids or [str(i) for i in range(rows)]
    return [PrefillCompressedVector(ids[i], codes[i].copy(), int(bits), shape, float(scales[i]), float(zps[i]))
            for i in range(rows)]
