"""Mirror of the ``quantization`` crate's operator surface (quantization/src/*.rs) on the GPU.

``Quantizer`` trait, ``DefaultQuantizer``, ``QuantizationType``, ``QuantizationParams``,
``QuantizedTensor``, ``quant_utils`` and ``CalibrationData``, with the same argument meaning and
``Result``-style errors (raised as ``QuantizationError`` subclasses).
"""
from __future__ import annotations

import abc
import enum
from dataclasses import dataclass, field
from typing import Optional

import torch

from . import _lib
from ._lib import check
from .quantization import _dev, _ptr, _stream


class QuantizationType(enum.IntEnum):
    """quantization/src/quantize.rs:62-67."""

    Int8 = 0
    Int4 = 1
    Binary = 2
    Float8 = 3

    def bits(self) -> int:
        """quantize.rs:69-78."""
        return {0: 8, 1: 4, 2: 1, 3: 8}[int(self)]


@dataclass
class QuantizationParams:
    """quantization/src/types.rs:20-40 (Default: 8 bits, scale 1.0, zp 0, symmetric, no axis)."""

    bits: int = 8
    scale: float = 1.0
    zero_point: int = 0
    symmetric: bool = True
    axis: Optional[int] = None


@dataclass
class QuantizedTensor:
    """quantization/src/types.rs:42-82: one code per byte + params."""

    data: torch.Tensor
    shape: tuple
    params: QuantizationParams

    def __len__(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n

    def is_empty(self) -> bool:
        return self.data.numel() == 0

    def dequantize(self) -> torch.Tensor:
        """types.rs:71-81."""
        n = len(self)
        out = torch.empty(n, dtype=torch.float32, device=self.data.device)
        check(_lib.load().dllm_default_dequantize(_ptr(self.data), n, float(self.params.scale),
                                                  int(self.params.zero_point), _ptr(out), _stream()))
        return out.reshape(self.shape)


class Quantizer(abc.ABC):
    """quantize.rs:81-90 ``trait Quantizer``."""

    @abc.abstractmethod
    def quantize(self, data: torch.Tensor, qtype: QuantizationType) -> QuantizedTensor: ...

    @abc.abstractmethod
    def dequantize(self, tensor: QuantizedTensor) -> torch.Tensor: ...

    @abc.abstractmethod
    def get_params(self) -> QuantizationParams: ...


class DefaultQuantizer(Quantizer):
    """quantize.rs:93-189.  ``new(bits, symmetric, axis)`` fixes scale = 1.0, zero_point = 0
    (:98-108); ``symmetric``/``axis`` are stored but do not enter the arithmetic.

    Element order is the flat row-major order (the reference's ``output[i]`` on an ``ArrayD``
    indexes axis 0 only for >= 2-D shapes; see SURVEY.md 8a-a4 and DESIGN.md)."""

    def __init__(self, bits: int, symmetric: bool, axis: Optional[int] = None, *, scale: float = 1.0,
                 zero_point: int = 0):
        self.params = QuantizationParams(bits, float(scale), int(zero_point), bool(symmetric), axis)

    @classmethod
    def new(cls, bits: int, symmetric: bool, axis: Optional[int] = None):
        return cls(bits, symmetric, axis)

    def quantize(self, data: torch.Tensor, qtype: QuantizationType) -> QuantizedTensor:
        x = _dev(data, torch.float32)
        n = x.numel()
        out = torch.empty(n, dtype=torch.uint8, device=x.device)
        check(_lib.load().dllm_default_quantize(_ptr(x), n, int(qtype), float(self.params.scale),
                                                int(self.params.zero_point), _ptr(out), _stream()))
        p = QuantizationParams(**vars(self.params))
        return QuantizedTensor(out, tuple(x.shape), p)

    def dequantize(self, tensor: QuantizedTensor) -> torch.Tensor:
        """quantize.rs:172-184 (uses the tensor's own params)."""
        return tensor.dequantize()

    def get_params(self) -> QuantizationParams:
        return self.params


class quant_utils:  # noqa: N801 - mirrors `pub mod utils` re-exported as quant_utils
    """quantize.rs:191-215."""

    @staticmethod
    def quantize(data: torch.Tensor, qtype: QuantizationType, symmetric: bool, axis: Optional[int] = None):
        return DefaultQuantizer(QuantizationType(qtype).bits(), symmetric, axis).quantize(data, qtype)

    @staticmethod
    def dequantize(tensor: QuantizedTensor) -> torch.Tensor:
        p = tensor.params
        return DefaultQuantizer(p.bits, p.symmetric, p.axis).dequantize(tensor)


@dataclass
class CalibrationData:
    """quantization/src/calibrate.rs:19-116 with the reduction on the GPU."""

    num_bins: int
    per_channel: bool = False
    total_samples: int = 0
    per_channel_stats: dict = field(default_factory=dict)

    def __post_init__(self):
        dev = torch.device("cuda")
        self._stats = torch.tensor([3.40282347e38, -3.40282347e38], dtype=torch.float32, device=dev)
        self._hist = torch.zeros(max(self.num_bins, 1), dtype=torch.int64, device=dev)

    @classmethod
    def new(cls, num_bins: int, per_channel: bool):
        return cls(num_bins, per_channel)

    @property
    def min(self) -> float:
        return float(self._stats[0].item())

    @property
    def max(self) -> float:
        return float(self._stats[1].item())

    @property
    def histogram(self) -> torch.Tensor:
        return self._hist[: self.num_bins]

    def update(self, data: torch.Tensor, channel: Optional[int] = None):
        """calibrate.rs:42-69."""
        x = _dev(data, torch.float32).reshape(-1)
        n = x.numel()
        L = _lib.load()
        ws_bytes = L.dllm_quantize_tensor_workspace(n)
        ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=x.device)
        if self.per_channel and channel is not None and n:
            # calibrate.rs:52-56: per-channel running (min, max), folded on the device.
            ch = self.per_channel_stats.get(channel)
            if ch is None:
                ch = torch.tensor([3.40282347e38, -3.40282347e38], dtype=torch.float32, device=x.device)
                self.per_channel_stats[channel] = ch
            check(L.dllm_calib_update(_ptr(x), n, _ptr(ch), None, 0, _ptr(ws), ws.numel(), _stream()))
        check(L.dllm_calib_update(_ptr(x) if n else None, n, _ptr(self._stats), _ptr(self._hist), self.num_bins,
                                  _ptr(ws), ws.numel(), _stream()))
        self.total_samples += n

    def compute_params(self, bits: int, symmetric: bool) -> QuantizationParams:
        """calibrate.rs:72-110."""
        import ctypes as C
        s, z = C.c_float(), C.c_int32()
        st = self._stats.cpu()
        check(_lib.load().dllm_calib_compute_params(float(st[0]), float(st[1]), self.total_samples, bits,
                                                    int(symmetric), C.byref(s), C.byref(z)))
        return QuantizationParams(bits, s.value, z.value, symmetric, None)
