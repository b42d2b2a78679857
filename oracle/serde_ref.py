"""TEST INFRASTRUCTURE (oracle): an independent pure-Python restatement of the wire formats the
reference's serde derives produce, the checker of the product's C-ABI
encoders/decoders (csrc/serde.cpp, include/dllm_quant.h section f3).  Only tests import it; it
imports nothing from the product package.

* ``QuantizationParams``, ``QuantizedTensor`` -- quantization/src/types.rs:19-47 (#[derive(Serialize,
  Deserialize)]); the crate converts both bincode and serde_json errors (quantization/src/error.rs:44-53).
* ``PrefillCompressedVector`` -- diffusion_prefill/src/prefill_kv.rs:25-33 (the KV hand-off record
  with its per-vector quant_scale / quant_zero_point), built from ``kvquant.compress_vectors``.

Encodings (third-party, absent from the container; restated from their published specifications):
* bincode 1.3 ``bincode::serialize`` (legacy config): little-endian, fixed-width integers, usize as
  u64, Vec / String = u64 length + elements, bool = 1 byte, Option = 1-byte tag (+ value).
* serde_json ``to_string``: compact, struct fields in declaration order, Vec<u8> as an array of
  integers, None as null, f32 via ryu's shortest round-trip digits in ryu's layout (non-finite
  f32 serialises as null).  Deserialising parses the number as f64 and rounds to f32 (serde's
  f32 visitor), which ``float`` + ``np.float32`` reproduces.
The byte layout is pinned by these specifications only (the reference ships no serialized
fixture): parity unpinned beyond the spec-derived tests in tests/test_serde.py.
Objects are plain host values: ``Params`` mirrors QuantizationParams, a tensor record is
(codes u8 array, shape, Params).
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

F32 = np.float32


class SerializationError(ValueError):
    """QuantizationError::Serialization (quantization/src/error.rs:33-34)."""


@dataclass
class Params:
    """quantization/src/types.rs:20-40 (Default: 8 bits, scale 1.0, zp 0, symmetric, no axis)."""
    bits: int = 8
    scale: float = 1.0
    zero_point: int = 0
    symmetric: bool = True
    axis: Optional[int] = None


@dataclass
class TensorRecord:
    """quantization/src/types.rs:42-47: data (one code per byte), shape, params."""
    data: np.ndarray
    shape: tuple
    params: Params


# ---- ryu f32 formatting (serde_json's float writer) ----------------------------------------------

def ryu_f32(x) -> str:
    """Rust ``ryu::Buffer::format_finite(f32)`` (ryu/src/pretty/mod.rs format32)."""
    x = F32(x)
    if not np.isfinite(x):
        raise ValueError("non-finite")
    bits = int(np.asarray(x).view(np.uint32))
    sign = "-" if bits >> 31 else ""
    if bits & 0x7FFFFFFF == 0:
        return sign + "0.0"
    sci = np.format_float_scientific(abs(x), unique=True, trim="-", exp_digits=1)
    mant, exp = sci.split("e")
    digits = mant.replace(".", "")
    digits = digits.rstrip("0") or "0"
    length = len(digits)
    e10 = int(exp)                 # value = d.ddd * 10^e10
    k = e10 - (length - 1)         # value = digits * 10^k
    kk = length + k                # 10^(kk-1) <= value < 10^kk
    if 0 <= k and kk <= 13:
        out = digits + "0" * (kk - length) + ".0"
    elif 0 < kk <= 13:
        out = digits[:kk] + "." + digits[kk:]
    elif -6 < kk <= 0:
        out = "0." + "0" * (-kk) + digits
    elif length == 1:
        out = digits + "e" + str(kk - 1)
    else:
        out = digits[0] + "." + digits[1:] + "e" + str(kk - 1)
    return sign + out


def _json_f32(x):
    x = F32(x)
    return "null" if not np.isfinite(x) else ryu_f32(x)


def _json_u8_array(a: np.ndarray) -> str:
    return "[" + ",".join(str(int(v)) for v in a) + "]"


# ---- bincode primitives ----------------------------------------------------------------------------

class _Reader:
    def __init__(self, b: bytes, strict: bool = False):
        self.b, self.i, self.strict = memoryview(b), 0, strict

    def take(self, n):
        if self.i + n > len(self.b):
            raise SerializationError("bincode: unexpected end of input")
        v = self.b[self.i:self.i + n]
        self.i += n
        return bytes(v)

    def u8(self):
        return self.take(1)[0]

    def u64(self):
        return struct.unpack("<Q", self.take(8))[0]

    def i32(self):
        return struct.unpack("<i", self.take(4))[0]

    def f32(self):
        return F32(struct.unpack("<f", self.take(4))[0])

    def bool(self):
        v = self.u8()
        if v > 1:
            raise SerializationError(f"bincode: invalid bool {v}")
        return bool(v)

    def bytes_vec(self):
        return np.frombuffer(self.take(self.u64()), dtype=np.uint8).copy()

    def usize_vec(self):
        n = self.u64()
        return [self.u64() for _ in range(n)]

    def string(self):
        return self.take(self.u64()).decode("utf-8")

    def done(self):
        """bincode 1.3's ``bincode::deserialize`` (the legacy free function the reference's
        ``bincode`` error conversion serves, quantization/src/error.rs:44-47) is
        ``DefaultOptions::new().with_fixint_encoding().allow_trailing_bytes()``: bytes after the
        value are ignored, not an error.  ``strict=True`` readers reject them (the
        ``DefaultOptions`` default)."""
        if self.strict and self.i != len(self.b):
            raise SerializationError("bincode: trailing bytes")


def _b_params(p: Params) -> bytes:
    out = struct.pack("<Bfi?", int(p.bits), float(F32(p.scale)), int(p.zero_point), bool(p.symmetric))
    out += b"\x00" if p.axis is None else b"\x01" + struct.pack("<Q", int(p.axis))
    return out


def _r_params(r: _Reader) -> Params:
    bits, scale, zp, sym = r.u8(), r.f32(), r.i32(), r.bool()
    tag = r.u8()
    if tag > 1:
        raise SerializationError(f"bincode: invalid Option tag {tag}")
    axis = None if tag == 0 else r.u64()
    return Params(bits=bits, scale=float(scale), zero_point=zp, symmetric=sym, axis=axis)


def _b_usize_vec(v) -> bytes:
    return struct.pack("<Q", len(v)) + b"".join(struct.pack("<Q", int(x)) for x in v)


def _b_bytes(a: np.ndarray) -> bytes:
    a = np.ascontiguousarray(a, np.uint8).ravel()
    return struct.pack("<Q", a.size) + a.tobytes()


# ---- QuantizationParams ------------------------------------------------------------------------------

def params_to_bincode(p: Params) -> bytes:
    return _b_params(p)


def params_from_bincode(b: bytes, strict: bool = False) -> Params:
    r = _Reader(b, strict)
    p = _r_params(r)
    r.done()
    return p


def _params_json(p: Params) -> str:
    axis = "null" if p.axis is None else str(int(p.axis))
    return (f'{{"bits":{int(p.bits)},"scale":{_json_f32(p.scale)},"zero_point":{int(p.zero_point)},'
            f'"symmetric":{"true" if p.symmetric else "false"},"axis":{axis}}}')


def params_to_json(p: Params) -> str:
    return _params_json(p)


def _no_duplicates(pairs):
    """serde's derived Deserialize: a field given twice is an error ("duplicate field"); unknown
    fields are ignored (no deny_unknown_fields on the reference's structs)."""
    keys = [k for k, _ in pairs]
    if len(keys) != len(set(keys)):
        raise SerializationError("json: duplicate field")
    return dict(pairs)


def _loads(s: str):
    return json.loads(s, object_pairs_hook=_no_duplicates)


def _params_from_obj(o) -> Params:
    scale = F32(float("nan") if o["scale"] is None else float(o["scale"]))
    return Params(bits=int(o["bits"]), scale=float(scale), zero_point=int(o["zero_point"]),
                              symmetric=bool(o["symmetric"]), axis=None if o["axis"] is None else int(o["axis"]))


def params_from_json(s: str) -> Params:
    return _params_from_obj(_loads(s))


# ---- QuantizedTensor (quantization crate) -------------------------------------------------------------

def _host_codes(t: TensorRecord) -> np.ndarray:
    return np.asarray(t.data, np.uint8).ravel()


def qtensor_to_bincode(t: TensorRecord) -> bytes:
    return _b_bytes(_host_codes(t)) + _b_usize_vec(t.shape) + _b_params(t.params)


def qtensor_from_bincode(b: bytes, strict: bool = False) -> TensorRecord:
    r = _Reader(b, strict)
    data, shape = r.bytes_vec(), r.usize_vec()
    params = _r_params(r)
    r.done()
    return TensorRecord(data, tuple(shape), params)


def qtensor_to_json(t: TensorRecord) -> str:
    shape = "[" + ",".join(str(int(s)) for s in t.shape) + "]"
    return f'{{"data":{_json_u8_array(_host_codes(t))},"shape":{shape},"params":{_params_json(t.params)}}}'


def _u8_array(v) -> np.ndarray:
    """serde's Vec<u8> visitor: every element an integer in 0..=255, else a data error."""
    if not isinstance(v, list) or not all(type(e) is int and 0 <= e <= 255 for e in v):
        raise SerializationError("json: data must be an array of integers in 0..=255")
    return np.asarray(v, dtype=np.uint8)


def qtensor_from_json(s: str) -> TensorRecord:
    o = _loads(s)
    return TensorRecord(_u8_array(o["data"]), tuple(int(v) for v in o["shape"]), _params_from_obj(o["params"]))


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

    def to_bincode(self) -> bytes:
        idb = self.id.encode("utf-8")
        return (struct.pack("<Q", len(idb)) + idb + _b_bytes(self.data) + struct.pack("<B", int(self.bits)) +
                _b_usize_vec(self.original_shape) + struct.pack("<ff", float(F32(self.quant_scale)),
                                                                float(F32(self.quant_zero_point))))

    @classmethod
    def from_bincode(cls, b: bytes, strict: bool = False) -> "PrefillCompressedVector":
        r = _Reader(b, strict)
        v = cls(r.string(), r.bytes_vec(), r.u8(), r.usize_vec(), float(r.f32()), float(r.f32()))
        r.done()
        return v

    def to_json(self) -> str:
        shape = "[" + ",".join(str(int(s)) for s in self.original_shape) + "]"
        return (f'{{"id":{json.dumps(self.id, ensure_ascii=False)},"data":{_json_u8_array(self.data)},'
                f'"bits":{int(self.bits)},"original_shape":{shape},"quant_scale":{_json_f32(self.quant_scale)},'
                f'"quant_zero_point":{_json_f32(self.quant_zero_point)}}}')

    @classmethod
    def from_json(cls, s: str) -> "PrefillCompressedVector":
        o = _loads(s)
        f = (lambda v: float(F32(float("nan") if v is None else float(v))))
        bits = int(o["bits"])
        if not 0 <= bits <= 255:
            raise SerializationError("json: bits out of u8 range")
        return cls(o["id"], _u8_array(o["data"]), bits, [int(v) for v in o["original_shape"]],
                   f(o["quant_scale"]), f(o["quant_zero_point"]))
