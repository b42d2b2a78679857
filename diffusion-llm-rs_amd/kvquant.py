"""Mirror of ``prefill_kvquant_rs::kvquant`` (prefill-kvquant-rs/lib.rs) and of
``diffusion_prefill::prefill_kv``'s per-vector compressor (diffusion_prefill/src/prefill_kv.rs),
backed by HIP kernels.  Vectors are batched as rows of a [rows, dim] device tensor instead of a
``Vec`` of owned structs; ``CompressedVector`` views index into the batch.
"""
from __future__ import annotations

import abc
from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check
from .quantization import _dev, _ptr, _stream


class Quantizer(abc.ABC):
    """prefill-kvquant-rs/lib.rs:29-32 ``trait Quantizer: Send + Sync`` (infallible in Rust;
    misuse that panics there raises InvalidParams here)."""

    @abc.abstractmethod
    def quantize(self, input: torch.Tensor, bits: int) -> torch.Tensor: ...

    @abc.abstractmethod
    def dequantize(self, input: torch.Tensor, bits: int) -> torch.Tensor: ...


@dataclass
class BitQuantizer(Quantizer):
    """prefill-kvquant-rs/lib.rs:34-53: fixed (scale, zero_point), truncating quantizer."""

    scale: float
    zero_point: float

    def quantize(self, input: torch.Tensor, bits: int) -> torch.Tensor:
        x = _dev(input, torch.float32).reshape(-1)
        out = torch.empty(x.numel(), dtype=torch.uint8, device=x.device)
        check(_lib.load().dllm_bit_quantize(_ptr(x), x.numel(), int(bits), float(self.scale),
                                            float(self.zero_point), _ptr(out), _stream()))
        return out

    def dequantize(self, input: torch.Tensor, bits: int = 0, out_dtype=torch.float32) -> torch.Tensor:
        q = _dev(input, torch.uint8).reshape(-1)
        out = torch.empty(q.numel(), dtype=out_dtype, device=q.device)
        dt = _lib.F32 if out_dtype == torch.float32 else _lib.F16
        check(_lib.load().dllm_bit_dequantize(_ptr(q), q.numel(), float(self.scale), float(self.zero_point),
                                              _ptr(out), dt, _stream()))
        return out


@dataclass
class SystemConfig:
    """prefill-kvquant-rs/lib.rs:76-91."""

    num_quantizers: int = 4
    cache_size: int = 1024
    quantization_bits: List[int] = field(default_factory=lambda: [4, 6, 8, 16])


@dataclass
class CompressedVector:
    """prefill-kvquant-rs/lib.rs:61-67 (``data`` is a device view)."""

    id: str
    data: torch.Tensor
    bits: int
    original_shape: tuple


@dataclass
class TokenizedVectors:
    """Batched ``TokenizedVector`` (lib.rs:93-97): ids + embeddings [rows, r, c] or [rows, dim]."""

    ids: Sequence[str]
    embeddings: torch.Tensor


class PrefillKVQuant:
    """prefill-kvquant-rs/lib.rs:23-147."""

    def __init__(self, config: SystemConfig | None = None):
        cfg = config or SystemConfig()
        self.config = cfg
        # lib.rs:102-110: one BitQuantizer per configured width, scale = 1/((1<<b)-1), zp = 0.
        self.quantizers = []
        for b in cfg.quantization_bits:
            if b > 30:
                raise _lib.InvalidParams("(1 << bits) - 1 overflows")
            self.quantizers.append(BitQuantizer(float(np.float32(1.0) / np.float32((1 << b) - 1)), 0.0))
        self.compression_ratio = 1.0

    @classmethod
    def new(cls, config: SystemConfig):
        return cls(config)

    def quantize_vectors_batched(self, embeddings: torch.Tensor, bits: Sequence[int]):
        """lib.rs:127-146 on a [rows, ...] batch -> (codes [rows, dim] u8, widths [rows] u8)."""
        x = _dev(embeddings, torch.float32)
        rows = x.shape[0] if x.dim() else 0
        x2 = x.reshape(rows, -1) if rows else x.reshape(0, 0)
        dim = x2.shape[1] if rows else 0
        req = np.ascontiguousarray(np.asarray(list(bits), dtype=np.uint8))
        cfg = np.ascontiguousarray(np.asarray(self.config.quantization_bits, dtype=np.uint8))
        if req.size == 0:
            return torch.empty(0, dim, dtype=torch.uint8, device=x.device), np.zeros(0, np.uint8)
        out = torch.empty(rows, dim, dtype=torch.uint8, device=x.device)
        widths = np.zeros(rows, np.uint8)
        check(_lib.load().dllm_quantize_vectors(_ptr(x2), rows, dim, cfg.ctypes.data, cfg.size, req.ctypes.data,
                                                req.size, _ptr(out), widths.ctypes.data, _stream()))
        return out, widths

    def quantize_vectors(self, tokens: TokenizedVectors, bits: Sequence[int]) -> List[CompressedVector]:
        emb = tokens.embeddings
        codes, widths = self.quantize_vectors_batched(emb, bits)
        shape = tuple(emb.shape[1:]) if emb.dim() > 2 else (1, emb.shape[1])
        return [CompressedVector(tokens.ids[i], codes[i], int(widths[i]), shape) for i in range(codes.shape[0])]


def compress_vectors(x: torch.Tensor, bits: int):
    """diffusion_prefill/src/prefill_kv.rs:104-121 over rows -> (codes, scales, zero_points)."""
    x = _dev(x, torch.float32)
    rows = x.shape[0]
    x2 = x.reshape(rows, -1)
    dim = x2.shape[1]
    out = torch.empty(rows, dim, dtype=torch.uint8, device=x.device)
    scales = torch.empty(rows, dtype=torch.float32, device=x.device)
    zps = torch.empty(rows, dtype=torch.float32, device=x.device)
    check(_lib.load().dllm_compress_vectors(_ptr(x2), rows, dim, int(bits), _ptr(out), _ptr(scales), _ptr(zps),
                                            _stream()))
    return out, scales, zps


def decompress_vectors(codes: torch.Tensor, scales: torch.Tensor, zero_points: torch.Tensor) -> torch.Tensor:
    """diffusion_prefill/src/prefill_kv.rs:124-132 over rows."""
    q = _dev(codes, torch.uint8)
    rows = q.shape[0]
    dim = q.numel() // max(rows, 1)
    out = torch.empty(rows, dim, dtype=torch.float32, device=q.device)
    check(_lib.load().dllm_decompress_vectors(_ptr(q), rows, dim, _ptr(_dev(scales, torch.float32)),
                                              _ptr(_dev(zero_points, torch.float32)), _ptr(out), _stream()))
    return out
