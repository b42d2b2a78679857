"""Group-quantized linear layer: the GPU replacement of ``SimpleDiffusionModel``'s forward
(diffuse-llm-rs/src/lib.rs:775-836), W [in, out] quantized per (column, 128-row K-group) with
``quantize_tensor`` and dequantized inside the MFMA GEMM (C-ABI ``dllm_linear_*``)."""
from __future__ import annotations

import ctypes as C

from typing import Optional

import torch

from . import _lib
from ._lib import check
from .quantization import _dev, _ptr, _stream


EXACT, F16W = 0, 1   # DLLM_PRECISION_EXACT (default), DLLM_PRECISION_F16W
PREFILL_ONLY = 0x100  # DLLM_LINEAR_PREFILL_ONLY: no decode layout (M <= 64 calls run the prefill kernels)


class QuantLinear:
    """Owns a ``dllm_linear_t`` handle (device weights uploaded once; immutable; Send + Sync).

    ``precision``: EXACT (default) feeds the MFMA the exact integer (q - zp) and applies the f32
    scale per group, so the weight is the reference's f32 a2 value; F16W rounds the dequantized
    weight to f16 first (~2.7e-4 more relative error per layer, and no faster).  ``prefill_only``
    skips the decode layout (half the device memory of an int4 layer) for layers that never see
    M <= 64, such as every layer of the denoise loop."""

    def __init__(self, handle, K: int, N: int, bits: int, group: int, precision: int = EXACT):
        self._h = handle
        self.K, self.N, self.bits, self.group, self.precision = K, N, bits, group, precision

    @classmethod
    def from_weight(cls, W: torch.Tensor, bias: torch.Tensor | None = None, bits: int = 4, group: int = 128,
                    precision: int = EXACT, prefill_only: bool = False):
        """W f32 [K, N] (the reference's ``weights: Array2<f32>`` of shape [input_dim, output_dim])."""
        W = _dev(W, torch.float32)
        K, N = W.shape
        b = None if bias is None else _dev(bias, torch.float32)
        h = C.c_void_p()
        flags = int(precision) | (PREFILL_ONLY if prefill_only else 0)
        check(_lib.load().dllm_linear_create_ex(_ptr(W), _ptr(b), K, N, bits, group, flags, C.byref(h), _stream()))
        return cls(h, K, N, bits, group, precision)

    @classmethod
    def from_quantized(cls, packed_codes: torch.Tensor, scales: torch.Tensor, zps: torch.Tensor, K: int, N: int,
                       bits: int = 4, group: int = 128, bias: torch.Tensor | None = None, precision: int = EXACT,
                       prefill_only: bool = False):
        h = C.c_void_p()
        b = None if bias is None else _dev(bias, torch.float32)
        check(_lib.load().dllm_linear_create_quantized_ex(
            _ptr(_dev(packed_codes, torch.uint8)), _ptr(_dev(scales, torch.float32)), _ptr(_dev(zps, torch.uint8)),
            _ptr(b), K, N, bits, group, int(precision) | (PREFILL_ONLY if prefill_only else 0), C.byref(h), _stream()))
        return cls(h, K, N, bits, group, precision)

    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None, out_dtype=torch.float16) -> torch.Tensor:
        """``forward(x) = x . W^ + b`` for x [M, K] (f16 or f32) -> [M, N]."""
        if x.dim() != 2 or x.shape[1] != self.K:
            raise _lib.ShapeMismatch(f"x must be [M, {self.K}], got {tuple(x.shape)}")
        if not x.is_cuda or not x.is_contiguous():
            x = _dev(x)
        if x.dtype not in (torch.float16, torch.float32):
            x = x.to(torch.float16)
        M = x.shape[0]
        if out is None:
            out = torch.empty(M, self.N, dtype=out_dtype, device=x.device)
        xdt = _lib.F16 if x.dtype == torch.float16 else _lib.F32
        ydt = _lib.F16 if out.dtype == torch.float16 else _lib.F32
        check(_lib.load().dllm_linear_forward(self._h, _ptr(x), M, xdt, _ptr(out), ydt, _stream()))
        return out

    __call__ = forward

    def forward_psample(self, x: torch.Tensor, x_t: torch.Tensor, coef: torch.Tensor, rows_per_sample: int,
                        add_noise: bool, seed: int, offset: int, out: Optional[torch.Tensor] = None,
                        noise: Optional[torch.Tensor] = None, out16: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Output layer of the denoiser fused with p_sample (diffuse-llm-rs/src/lib.rs:1188-1212):
        eps = x . W^ + b (f32) and x_prev = (c1 x_t + c2 eps) + std * noise in the GEMM epilogue.
        x [M, K] f16/f32, x_t / out f32 [M, N], coef f32 [M / rows_per_sample, 3] (device); noise
        f32 [M, N] precomputed, or None to draw stream elements offset + m N + n in the epilogue.
        ``out16`` (f16 [M, N], optional): also receives x_prev rounded to f16 from the same epilogue
        (dllm_linear_forward_psample_ex), the next step's first-layer input."""
        if x.dim() != 2 or x.shape[1] != self.K:
            raise _lib.ShapeMismatch(f"x must be [M, {self.K}], got {tuple(x.shape)}")
        x = _dev(x) if (not x.is_cuda or not x.is_contiguous()) else x
        if x.dtype not in (torch.float16, torch.float32):
            x = x.to(torch.float16)
        M = x.shape[0]
        if tuple(x_t.shape) != (M, self.N) or x_t.dtype != torch.float32:
            raise _lib.ShapeMismatch(f"x_t must be f32 [{M}, {self.N}]")
        out = torch.empty_like(x_t) if out is None else out
        xdt = _lib.F16 if x.dtype == torch.float16 else _lib.F32
        if out16 is not None and (tuple(out16.shape) != (M, self.N) or out16.dtype != torch.float16):
            raise _lib.ShapeMismatch(f"out16 must be f16 [{M}, {self.N}]")
        check(_lib.load().dllm_linear_forward_psample_ex(self._h, _ptr(x), M, xdt, _ptr(x_t), _ptr(coef),
                                                         int(rows_per_sample), int(bool(add_noise)), int(seed),
                                                         int(offset), None if noise is None else _ptr(noise),
                                                         _ptr(out), None if out16 is None else _ptr(out16),
                                                         _stream()))
        return out

    @staticmethod
    def bias_cast(y: torch.Tensor, bias: torch.Tensor | None, out_dtype=torch.float16,
                  out: torch.Tensor | None = None) -> torch.Tensor:
        """``y + bias`` (f32) cast to ``out_dtype`` on the device (dllm_bias_cast): the epilogue of a
        row-parallel shard after its partial sums are reduced (parallel.RowParallelLinear)."""
        from .quantization import bias_cast
        return bias_cast(y, bias, out_dtype, out)

    def export(self):
        """-> (packed codes of the [K][N] code matrix, scales [G][N] f32, zero points [G][N] u8)."""
        G = (self.K + self.group - 1) // self.group
        dev = torch.device("cuda")
        codes = torch.empty((self.K * self.N * self.bits + 7) // 8, dtype=torch.uint8, device=dev)
        scales = torch.empty(G, self.N, dtype=torch.float32, device=dev)
        zps = torch.empty(G, self.N, dtype=torch.uint8, device=dev)
        check(_lib.load().dllm_linear_export(self._h, _ptr(codes), _ptr(scales), _ptr(zps), _stream()))
        return codes, scales, zps

    def device_bytes(self) -> int:
        """Device memory the handle owns (dllm_linear_device_bytes)."""
        return int(_lib.load().dllm_linear_device_bytes(self._h))

    def set_kernel_variant(self, variant: int):
        """Schedule variant / ablation mask: lab build only (installed by `_lib.use`, measurement scripts)."""
        lib = _lib.load()
        if not hasattr(lib, "dllm_linear_set_kernel_variant"):
            raise _lib.UnsupportedOperation("schedule variants exist only in the lab build (_lib.use(LAB_LIB_PATH))", 2)
        check(lib.dllm_linear_set_kernel_variant(self._h, int(variant)))

    def weight_bytes(self) -> int:
        return int(_lib.load().dllm_linear_weight_bytes(self._h))

    def close(self):
        if self._h is not None and self._h.value:
            torch.cuda.current_stream().synchronize()
            _lib.load().dllm_linear_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MixedPrecisionStack:
    """Config 3: L linear layers, layer l quantized at ``bits[l % len(bits)]`` (the reference's
    ``bits.iter().cycle()`` idiom, prefill-kvquant-rs/lib.rs:132); X_{l+1} = Y_l."""

    def __init__(self, weights, biases=None, bits=(2, 4), group: int = 128):
        self.layers = []
        for i, W in enumerate(weights):
            b = None if biases is None else biases[i]
            self.layers.append(QuantLinear.from_weight(W, b, bits[i % len(bits)], group))

    def forward(self, x: torch.Tensor, out_dtype=torch.float16) -> torch.Tensor:
        for i, layer in enumerate(self.layers):
            x = layer(x, out_dtype=out_dtype if i == len(self.layers) - 1 else torch.float16)
        return x

    __call__ = forward
