"""The diffusion-step ops either side of the denoiser and the denoise loop (SURVEY.md 8f rank 1-2,
config C5), mirroring ``diffuse_llm_rs::diffuse_llm`` (diffuse-llm-rs/src/lib.rs):

* ``DiffusionConfig.create_beta_schedule``  -- lib.rs:554-593 (host scalars, Rust f32 semantics)
* ``add_noise``                             -- DiffuseLLM::add_noise, lib.rs:1100-1137
* ``p_sample``                              -- DiffuseLLM::p_sample, lib.rs:1152-1215
* ``KVCacheEntry``                          -- phase-aware dual-precision KV cache, lib.rs:121-313
* ``DenoiseLoop``                           -- DiffuseLLM::sample, lib.rs:853-955, with an
  L-layer quantized denoiser whose last layer runs p_sample in its GEMM epilogue.

Reference conventions that the code gets wrong or leaves open are explicit arguments (see
include/dllm_quant.h): ``cumprod`` (exclusive alpha-bar of add_noise/p_sample, whose t = 0
step divides by zero, vs the inclusive p_losses scan) and ``alpha_mode`` (per-sample alpha_t vs
the reference's full-length ``alphas`` broadcast).  Noise is the build's seeded stream
(``randn``), not thread_rng.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from enum import IntEnum
from typing import Callable, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check
from .quantization import QuantizedKVCacheEntry


class BetaSchedule(IntEnum):
    """lib.rs:111-118."""
    Linear = 0
    Quadratic = 1
    Cosine = 2


class Cumprod(IntEnum):
    EXCLUSIVE = 0   # add_noise / p_sample (lib.rs:1116-1119, 1162-1165)
    INCLUSIVE = 1   # p_losses (lib.rs:627-630)


class AlphaMode(IntEnum):
    PER_SAMPLE = 0  # alpha[t_i] (the posterior the code intends)
    LITERAL = 1     # full-length `alphas` row-wise (lib.rs:1191; batch == num_timesteps only)


def _ptr(t):
    return C.c_void_p(t.data_ptr() if isinstance(t, torch.Tensor) else t.ctypes.data)


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


@dataclass
class DiffusionConfig:
    """lib.rs:456-488 (DiffusionConfig::default) plus the phase-aware KV fields DiffuseLLM::sample
    reads (lib.rs:880-903)."""
    num_timesteps: int = 1000
    hidden_size: int = 768
    num_layers: int = 12
    num_attention_heads: int = 12
    vocab_size: int = 50257
    max_sequence_length: int = 1024
    beta_start: float = 0.0001
    beta_end: float = 0.02
    beta_schedule: BetaSchedule = BetaSchedule.Linear
    use_kv_cache: bool = True
    kv_quant_bits: int = 4
    max_cache_size: int = 2 * 1024 * 1024 * 1024
    use_phase_aware_quant: bool = True
    prefill_bits: int = 8
    decode_bits: int = 4
    min_decode_bits: int = 2
    progressive_precision: bool = True      # QuantizationConfig::default() (lib.rs:96-104)

    def create_beta_schedule(self) -> np.ndarray:
        """lib.rs:554-593 -> f32 [num_timesteps] (host)."""
        out = np.zeros(self.num_timesteps, np.float32)
        check(_lib.load().dllm_beta_schedule(int(self.beta_schedule), self.num_timesteps, float(self.beta_start),
                                             float(self.beta_end), _ptr(out)))
        return out

    def alpha_bars(self, cumprod: Cumprod = Cumprod.EXCLUSIVE):
        betas = self.create_beta_schedule()
        a = np.zeros_like(betas)
        ab = np.zeros_like(betas)
        check(_lib.load().dllm_alpha_bars(_ptr(betas), betas.size, int(cumprod), _ptr(a), _ptr(ab)))
        return a, ab


def randn(n: int, seed: int, offset: int = 0, device="cuda") -> torch.Tensor:
    """Elements offset .. offset + n - 1 of the seeded N(0, 1) stream (f32, device)."""
    out = torch.empty(n, dtype=torch.float32, device=device)
    check(_lib.load().dllm_randn(seed, offset, _ptr(out), n, _stream()))
    return out


def _timesteps(t, B):
    t = np.asarray([t] * B if np.isscalar(t) else t, dtype=np.uint64)
    if t.size != B:
        raise _lib.ShapeMismatch("Timesteps must match batch size")   # lib.rs:624
    return t


def p_sample_coeffs(config: DiffusionConfig, t, B: int, cumprod=Cumprod.EXCLUSIVE, alpha_mode=AlphaMode.PER_SAMPLE):
    """Per-sample {c1, c2, std} (host f32 [B, 3]) and the reference's noise flag (t[0] > 0)."""
    betas = config.create_beta_schedule()
    tt = _timesteps(t, B)
    coef = np.zeros((B, 3), np.float32)
    flag = C.c_int(0)
    check(_lib.load().dllm_p_sample_coeffs(_ptr(betas), betas.size, int(cumprod), int(alpha_mode), _ptr(tt), B,
                                           _ptr(coef), C.byref(flag)))
    return coef, bool(flag.value)


def add_noise_coeffs(config: DiffusionConfig, t, B: int, cumprod=Cumprod.EXCLUSIVE):
    betas = config.create_beta_schedule()
    tt = _timesteps(t, B)
    coef = np.zeros((B, 2), np.float32)
    check(_lib.load().dllm_add_noise_coeffs(_ptr(betas), betas.size, int(cumprod), _ptr(tt), B, _ptr(coef)))
    return coef


def _dev32(x):
    return x.to(device="cuda", dtype=torch.float32).contiguous()


def add_noise(config: DiffusionConfig, x_start: torch.Tensor, t, noise: Optional[torch.Tensor] = None, seed: int = 0,
              offset: int = 0, cumprod: Cumprod = Cumprod.EXCLUSIVE):
    """DiffuseLLM::add_noise (lib.rs:1100-1137): (noisy, noise) for x_start [B, D]."""
    x0 = _dev32(x_start)
    B, D = x0.shape
    coef = torch.from_numpy(add_noise_coeffs(config, t, B, cumprod)).to(x0.device)
    noisy = torch.empty_like(x0)
    if noise is None:
        nz = torch.empty_like(x0)
        check(_lib.load().dllm_add_noise(_ptr(x0), None, _ptr(coef), B, D, seed, offset, _ptr(noisy), _ptr(nz),
                                         _stream()))
    else:
        nz = _dev32(noise)
        if nz.shape != x0.shape:
            raise _lib.ShapeMismatch("Noise shape must match input shape")   # lib.rs:623
        check(_lib.load().dllm_add_noise(_ptr(x0), _ptr(nz), _ptr(coef), B, D, 0, 0, _ptr(noisy), None, _stream()))
    return noisy, nz


def p_sample(config: DiffusionConfig, x_t: torch.Tensor, t, noise_pred: torch.Tensor, seed: int = 0,
             offset: int = 0, noise: Optional[torch.Tensor] = None, cumprod: Cumprod = Cumprod.EXCLUSIVE,
             alpha_mode: AlphaMode = AlphaMode.PER_SAMPLE, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """DiffuseLLM::p_sample (lib.rs:1152-1215) for x_t, noise_pred [B, D]."""
    x = _dev32(x_t)
    eps = _dev32(noise_pred)
    B, D = x.shape
    coef_np, flag = p_sample_coeffs(config, t, B, cumprod, alpha_mode)
    coef = torch.from_numpy(coef_np).to(x.device)
    out = torch.empty_like(x) if out is None else out
    nz = None if noise is None else _dev32(noise)
    check(_lib.load().dllm_p_sample(_ptr(x), _ptr(eps), None if nz is None else _ptr(nz), _ptr(coef), B, D, int(flag),
                                    seed, offset, _ptr(out), _stream()))
    return out


class KVCacheEntry:
    """Phase-aware dual-precision KV cache (lib.rs:121-313): f32 K/V [layers, seq, hidden] on
    the device plus a prefill-width and a decode-width QuantizedKVCacheEntry (per-tensor a1
    codes, packed).  ``update`` re-quantizes both copies on the GPU (the reference's up-to-4
    quantize_tensor calls per timestep); ``get_keys``/``get_values`` dequantize the copy of the
    current phase."""

    def __init__(self, keys: torch.Tensor, values: torch.Tensor, prefill_bits: int, decode_bits: int):
        self.keys, self.values = keys, values
        self.prefill_quant_bits, self.decode_quant_bits = prefill_bits, decode_bits
        self.prefill_quantized = self._quantize(keys, values, prefill_bits) if prefill_bits > 0 else None
        self.decode_quantized = self._quantize(keys, values, decode_bits) if decode_bits > 0 else None
        self.is_prefill_phase = True
        self.seq_len = int(keys.shape[1])

    # The quantization steps (QuantizedKVCacheEntry::new at one width, or at two widths in one pass);
    # parallel.HeadParallelKVCacheEntry overrides them with the head-sharded form.
    def _quantize(self, keys, values, bits):
        return QuantizedKVCacheEntry.new(keys, values, bits)

    def _quantize_pair(self, keys, values, bits_a, bits_b):
        return QuantizedKVCacheEntry.new_pair(keys, values, bits_a, bits_b)

    @classmethod
    def new(cls, keys, values, prefill_bits, decode_bits):
        return cls(keys, values, prefill_bits, decode_bits)

    def _current(self):
        return self.prefill_quantized if self.is_prefill_phase else self.decode_quantized

    def get_keys(self) -> torch.Tensor:
        q = self._current()
        return self.keys.clone() if q is None else self._dequantize(q.keys)

    def get_values(self) -> torch.Tensor:
        q = self._current()
        return self.values.clone() if q is None else self._dequantize(q.values)

    def _dequantize(self, t):
        """QuantizedKVCacheEntry::dequantize_keys/values (quantization.rs:160-175)."""
        return t.dequantize().reshape(t.shape)

    def get_current_quant_bits(self) -> int:
        return self.prefill_quant_bits if self.is_prefill_phase else self.decode_quant_bits

    def set_phase(self, is_prefill: bool):
        self.transition_phase(is_prefill)

    def transition_phase(self, is_prefill: bool):
        """lib.rs:221-239."""
        if self.is_prefill_phase == is_prefill:
            return
        self.is_prefill_phase = is_prefill
        if not is_prefill and self.decode_quant_bits > 0 and self.decode_quantized is None:
            self.decode_quantized = self._quantize(self.keys, self.values, self.decode_quant_bits)

    def update(self, new_keys: torch.Tensor, new_values: torch.Tensor):
        """lib.rs:241-276 (the missing QuantizedKVCacheEntry::update is a re-quantization)."""
        self.keys, self.values = new_keys, new_values
        self.seq_len = int(new_keys.shape[1])
        if self.prefill_quant_bits > 0 and self.decode_quant_bits > 0:
            # both widths from one min/max pass and one read per tensor (bit-identical)
            self.prefill_quantized, self.decode_quantized = self._quantize_pair(
                new_keys, new_values, self.prefill_quant_bits, self.decode_quant_bits)
            return
        if self.prefill_quant_bits > 0:
            self.prefill_quantized = self._quantize(new_keys, new_values, self.prefill_quant_bits)
        if self.decode_quant_bits > 0:
            self.decode_quantized = self._quantize(new_keys, new_values, self.decode_quant_bits)

    def clone(self) -> "KVCacheEntry":
        """``#[derive(Clone)]``: an independent copy (device tensors duplicated)."""
        c = object.__new__(type(self))
        c.__dict__.update(self.__dict__)
        c.keys, c.values = self.keys.clone(), self.values.clone()
        c.prefill_quantized = None if self.prefill_quantized is None else self.prefill_quantized.clone()
        c.decode_quantized = None if self.decode_quantized is None else self.decode_quantized.clone()
        return c

    def memory_usage(self) -> int:
        """lib.rs:279-302: packed bytes of the quantized copies, else f32 bytes."""
        total = sum(q.memory_usage() for q in (self.prefill_quantized, self.decode_quantized) if q is not None)
        return total if total else (self.keys.numel() + self.values.numel()) * 4

    def __len__(self):
        return self.seq_len

    def is_empty(self) -> bool:
        return self.seq_len == 0


_USIZE = 1 << 64


class KVCacheStore:
    """DiffuseLLM's KV-cache registry: ``kv_cache: DashMap<String, KVCacheEntry>`` and
    ``cache_memory_usage: AtomicUsize`` (lib.rs:338-345) with
    ``init_kv_cache`` (:958-980), ``get_or_init_cache`` (:983-991), ``update_kv_cache`` (:994-1043),
    ``evict_oldest_entries`` (:1046-1073), ``clear_kv_cache`` (:1076-1079) and
    ``kv_cache_memory_usage`` (:1082-1084).

    The accounting is the reference's, quirks included:
    - The eviction check prices an update at ``keys.len() * 4 * 2`` bytes, f32 K + V.
    - A new entry adds its packed ``memory_usage()``.
    - An update of an existing entry adds ``new_size.saturating_sub(old_size)``.
    - Eviction removes the LARGEST entries first, despite its name, until the freed bytes reach the
      request. It then subtracts them with the wrapping ``fetch_sub`` of an AtomicUsize.
    - ``get_or_init_cache`` inserts a fresh entry without accounting, and hands out a clone.
    Ties in the size order keep insertion order; the DashMap's iteration order is unspecified.
    The entries' K/V and quantized copies live on the device; evicting an entry frees them. The
    reference's update path calls ``KVCacheEntry::new`` with one width (:1028-1032), so a new entry
    there uses ``kv_quant_bits`` for both phases."""

    def __init__(self, config: DiffusionConfig, entry_factory: Optional[Callable] = None, device="cuda"):
        self.config = config
        self.entry_factory = entry_factory or KVCacheEntry.new
        self.device = device
        self.kv_cache: dict = {}
        self.cache_memory_usage = 0
        self._lock = __import__("threading").RLock()

    def _phase_bits(self):
        c = self.config
        return (c.prefill_bits, c.decode_bits) if c.use_phase_aware_quant else (c.kv_quant_bits, c.kv_quant_bits)

    def init_kv_cache(self, batch_size: int):
        """:958-980 -- empty [num_layers, 0, heads * head_dim] K/V at the phase widths."""
        c = self.config
        hd = (c.hidden_size // c.num_attention_heads) * c.num_attention_heads
        z = torch.zeros((c.num_layers, 0, hd), dtype=torch.float32, device=self.device)
        pb, db = self._phase_bits()
        return self.entry_factory(z, z.clone(), pb, db)

    def get_or_init_cache(self, cache_id: str, batch_size: int):
        """:983-991 -- a clone of the stored entry; a missing one is created and inserted."""
        with self._lock:
            e = self.kv_cache.get(cache_id)
            if e is None:
                e = self.init_kv_cache(batch_size)
                self.kv_cache[cache_id] = e
            return e.clone()

    def update_kv_cache(self, cache_id: str, keys: torch.Tensor, values: torch.Tensor) -> None:
        """:994-1043."""
        c = self.config
        if not c.use_kv_cache:
            return
        with self._lock:
            entry_size = keys.numel() * 4 * 2
            new_usage = self.cache_memory_usage + entry_size
            if new_usage > c.max_cache_size:
                self.evict_oldest_entries(new_usage - c.max_cache_size)
            e = self.kv_cache.get(cache_id)
            if e is not None:
                old_size = e.memory_usage()
                new_size = keys.numel() * 4 * 2
                e.update(keys, values)
                self.cache_memory_usage = (self.cache_memory_usage + max(new_size - old_size, 0)) % _USIZE
            else:
                e = self.entry_factory(keys, values, c.kv_quant_bits, c.kv_quant_bits)
                self.kv_cache[cache_id] = e
                self.cache_memory_usage = (self.cache_memory_usage + e.memory_usage()) % _USIZE

    def evict_oldest_entries(self, bytes_to_free: int) -> None:
        """:1046-1073 -- largest entries first until ``bytes_to_free`` is reached."""
        with self._lock:
            entries = sorted(((k, v.memory_usage()) for k, v in self.kv_cache.items()), key=lambda kv: -kv[1])
            freed = 0
            for key, size in entries:
                if freed >= bytes_to_free:
                    break
                if self.kv_cache.pop(key, None) is not None:
                    freed += size
            self.cache_memory_usage = (self.cache_memory_usage - freed) % _USIZE

    def clear_kv_cache(self) -> None:
        with self._lock:
            self.kv_cache.clear()
            self.cache_memory_usage = 0

    def kv_cache_memory_usage(self) -> int:
        return self.cache_memory_usage

    def __contains__(self, cache_id):
        return cache_id in self.kv_cache

    def __len__(self):
        return len(self.kv_cache)


def progressive_bits(config: DiffusionConfig, num_steps: int, t: int) -> int:
    """lib.rs:890-897: decode bits interpolated towards min_decode_bits over the decode half:
    ``((decode * (1 - p) + min * p) as u8`` with p = (num_steps - t) / (num_steps / 2), every op a
    rounded f32 op and the saturating ``as u8`` (negative and NaN -> 0, +inf -> 255).

    Past the middle of the decode half the target falls below 1 (with 50 steps: 2 at t = 25,
    1 for t = 24..13, 0 for t <= 12).  Bits 0 is a defined state in the reference, not its
    ``assert!`` (quantization.rs:39): ``transition_phase`` and ``update`` only quantize when
    ``decode_quant_bits > 0`` (lib.rs:230, :262), so the decode copy stays ``None`` and
    ``get_keys``/``get_values`` hand out the f32 K/V (lib.rs:190-197).  KVCacheEntry does the
    same; quantize_tensor itself still rejects bits outside 1..=8 (InvalidParams)."""
    f = np.float32
    progress = f(f(num_steps - t) / f(num_steps // 2)) if num_steps // 2 else f(np.inf if num_steps > t else np.nan)
    v = f(f(f(config.decode_bits) * f(f(1.0) - progress)) + f(f(config.min_decode_bits) * progress))
    if np.isnan(v):
        return 0
    return int(min(max(np.trunc(v), 0), 255))


class DeviceLoopOps:
    """The loop's elementwise steps as HIP kernels behind the C-ABI (the product path)."""

    @staticmethod
    def p_sample(x, eps, noise, coef, flag, seed, offset, out):
        """lib.rs:1152-1215 over x as one sample of x.numel() elements (coef = device f32 [1, 3])."""
        check(_lib.load().dllm_p_sample(_ptr(x), _ptr(eps), None if noise is None else _ptr(noise), _ptr(coef), 1,
                                        x.numel(), int(flag), seed, offset, _ptr(out), _stream()))

    @staticmethod
    def randn(out, seed, offset):
        check(_lib.load().dllm_randn(seed, offset, _ptr(out), out.numel(), _stream()))


class DenoiseLoop:
    """DiffuseLLM::sample (lib.rs:853-955) over an L-layer quantized denoiser (config C5).

    Per timestep t = num_steps-1 .. 0: the KV phase switch and re-quantization (KVCacheEntry),
    the denoiser (layers 0..L-2 chained in f16, f32 x in / f32 eps out), and p_sample.  With local
    QuantLinear layers the last layer runs p_sample inside its GEMM epilogue
    (dllm_linear_forward_psample); a layer callable without that entry point (e.g. a
    tensor-parallel pair whose output is all-reduced) is followed by the p_sample kernel.
    x is [M, d] f32 for one sample of M = seq tokens (the reference's [batch, hidden*seq] row
    laid out token-major); the noise of step i is stream elements [i M d, (i+1) M d).

    overlap=True runs the work of a step that does not depend on x -- the KV-cache update (the
    simple model's update_kv_cache passes K/V through, lib.rs:826-835, and forward_with_cache
    ignores them, :815-824) -- on a side stream while the layers run.  The step's noise is drawn
    inside the last layer's fused p_sample epilogue (noise="epilogue", the default when the last
    layer has forward_psample), or on the side stream into one of two buffers (noise="side"; the
    last layer then waits for it).  Every form is bit-identical to overlap=False.  Measured at
    config C5 (scripts/c5_ab.py): epilogue 0.922, side 0.953, serial 0.963 ms per step -- the
    side-stream draw costs the GEMMs more CU time than the in-epilogue draw costs the last layer.

    The layers may be tensor-parallel (parallel.TensorParallelPair: one reduction per pair, x
    replicated on every rank) and the cache head-sharded (parallel.HeadParallelKVCacheEntry): every
    rank then runs this same loop on its shards, with the same phase, width and noise sequence.
    Token-parallel (``noise_rows=(row0, rows_total)``, parallel.token_rows): every rank runs its
    rows of x through replicated layers -- the linear layers and p_sample are per token, so no
    collective -- with its rows of K/V in a sharded cache (one 4-float all_reduce(MAX) per
    quantization) and the noise its rows get in the unsharded loop.
    ``ops`` holds the elementwise steps (p_sample, noise) and ``device`` where x lives: the HIP
    kernels on the GPU (``DeviceLoopOps``); the CPU multi-process tests pass the oracle's
    restatement and device "cpu" (serial schedule only)."""

    f16_handoff = True   # overlapped loop: x_prev's f16 copy from the fused epilogue feeds the next step

    def __init__(self, layers: Sequence, config: DiffusionConfig, cumprod: Cumprod = Cumprod.INCLUSIVE,
                 alpha_mode: AlphaMode = AlphaMode.PER_SAMPLE, seed: int = 0,
                 kv_cache: Optional[KVCacheEntry] = None, overlap: bool = True, noise: str = "epilogue",
                 ops=DeviceLoopOps, device="cuda", noise_rows: Optional[tuple] = None):
        if noise not in ("side", "epilogue"):
            raise ValueError("noise must be 'side' or 'epilogue'")
        # noise_rows = (row0, rows_total): x holds rows row0.. of a rows_total-token sample (a token
        # shard); step i then draws stream elements [i rows_total d + row0 d, ...), the same noise
        # those rows get in the unsharded loop
        if noise_rows is not None and not (0 <= int(noise_rows[0]) < int(noise_rows[1])):
            raise ValueError("noise_rows must be (row0, rows_total) with 0 <= row0 < rows_total")
        self.noise_rows = None if noise_rows is None else (int(noise_rows[0]), int(noise_rows[1]))
        self.ops, self.device = ops, torch.device(device)
        if self.device.type != "cuda":
            overlap = False
        self.layers = list(layers)
        self.noise_mode = noise if self.layers and hasattr(self.layers[-1], "forward_psample") else "side"
        self.config = config
        self.cumprod, self.alpha_mode, self.seed = cumprod, alpha_mode, seed
        self.kv_cache = kv_cache
        self.overlap = overlap
        self._betas = config.create_beta_schedule()
        self._coef_cache = {}
        self._side = None
        # kv_spread: the side stream's KV step i waits for the main stream to reach step i, so the
        # 50 KV steps run beside their own steps instead of back to back from the start (config C5:
        # 0.861 -> 0.841 ms per step, median of 6 rounds, and a tighter spread; bit-identical;
        # profiles/r05_spread/).  False: the round-4 free-running side stream.
        self.kv_spread = True
        self._noise = None

    def _coef(self, t: int) -> tuple[torch.Tensor, bool]:
        if t not in self._coef_cache:
            coef = np.zeros((1, 3), np.float32)
            flag = C.c_int(0)
            tt = np.asarray([t], np.uint64)
            check(_lib.load().dllm_p_sample_coeffs(_ptr(self._betas), self._betas.size, int(self.cumprod),
                                                   int(self.alpha_mode), _ptr(tt), 1, _ptr(coef), C.byref(flag)))
            self._coef_cache[t] = (torch.from_numpy(coef).to(self.device), bool(flag.value))
        return self._coef_cache[t]

    def _noise_offset(self, step_index: int, M: int, d: int) -> int:
        """First noise-stream element of step ``step_index`` for this x (its rows of the sample)."""
        if self.noise_rows is None:
            return step_index * M * d
        row0, total = self.noise_rows
        if row0 + M > total:
            raise ValueError(f"x has {M} rows from row {row0}: past the sample's {total}")
        return step_index * total * d + row0 * d

    def step(self, x: torch.Tensor, t: int, step_index: int, out: Optional[torch.Tensor] = None,
             noise: Optional[torch.Tensor] = None, noise_ready: Optional[torch.cuda.Event] = None,
             x16: Optional[torch.Tensor] = None, out16: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One timestep.  ``x16``: x already rounded to f16 (the first layer's input; the layer would
        otherwise round x itself, to the same bits); ``out16``: receives x_prev rounded to f16 from
        the fused last layer's epilogue (the next step's ``x16``), when the last layer is fused."""
        M, d = x.shape
        coef, flag = self._coef(t)
        offset = self._noise_offset(step_index, M, d)
        h = x if x16 is None else x16
        for layer in self.layers[:-1]:
            h = layer(h, out_dtype=torch.float16)
        last = self.layers[-1]
        out = torch.empty_like(x) if out is None else out
        if noise_ready is not None:
            torch.cuda.current_stream().wait_event(noise_ready)
        if hasattr(last, "forward_psample"):
            last.forward_psample(h, x, coef, M, flag, self.seed, offset, out, noise=noise, out16=out16)
        else:
            eps = last(h, out_dtype=torch.float32)
            self.ops.p_sample(x, eps, noise, coef, flag, self.seed, offset, out)
        return out

    def kv_step(self, t: int, num_steps: int):
        """lib.rs:880-916: phase switch, progressive decode bits, update (re-quantize), dequant."""
        c = self.kv_cache
        if c is None:
            return None
        is_prefill = t > num_steps // 2
        c.set_phase(is_prefill)
        if self.config.use_phase_aware_quant and self.config.progressive_precision and not is_prefill:
            tb = progressive_bits(self.config, num_steps, t)
            if tb != c.decode_quant_bits:
                c.decode_quant_bits = tb
                c.decode_quantized = None
        keys, values = c.keys, c.values          # SimpleDiffusionModel::update_kv_cache (:826-835)
        k, v = c.get_keys(), c.get_values()      # what forward_with_cache receives (:910-915)
        c.update(keys, values)
        return k, v

    def sample(self, x: torch.Tensor, num_steps: Optional[int] = None, store: Optional[KVCacheStore] = None,
               cache_id: Optional[str] = None) -> torch.Tensor:
        """The loop of lib.rs:880-931.  With a ``store`` and ``cache_id`` (and use_kv_cache) the
        cache is the reference's: a clone of the stored entry (get_or_init_cache, prefill phase,
        :864-872), saved back at the end as its dequantized K/V (update_kv_cache, :936-943)."""
        if store is not None and cache_id is not None and self.config.use_kv_cache:
            kv = store.get_or_init_cache(cache_id, 1)
            kv.set_phase(True)
            saved, self.kv_cache = self.kv_cache, kv
            try:
                x = self._sample(x, num_steps)
            finally:
                self.kv_cache = saved
            store.update_kv_cache(cache_id, kv.get_keys(), kv.get_values())
            return x
        return self._sample(x, num_steps)

    def _sample(self, x: torch.Tensor, num_steps: Optional[int] = None) -> torch.Tensor:
        num_steps = num_steps or self.config.num_timesteps
        x = x.to(device=self.device, dtype=torch.float32).contiguous()
        buf = torch.empty_like(x)
        M, d = x.shape
        if not self.overlap:
            for i, t in enumerate(range(num_steps - 1, -1, -1)):
                self.kv_step(t, num_steps)
                buf = self.step(x, t, i, out=buf)
                x, buf = buf, x
            return x
        main = torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream()
        if self._noise is None or self._noise[0].shape != x.shape:
            self._noise = [torch.empty_like(x), torch.empty_like(x)]
        side = self._side
        freed = [None, None]        # main-stream events: noise buffer j no longer read
        side.wait_stream(main)
        # the fused last layer also writes x_prev in f16: the next step's first layer reads it
        # instead of casting x again (same bits; one 32 MiB read + 16 MiB write less per step)
        f16 = [torch.empty(x.shape, dtype=torch.float16, device=x.device) for _ in range(2)] \
            if self.f16_handoff and hasattr(self.layers[-1], "forward_psample") else None
        for i, t in enumerate(range(num_steps - 1, -1, -1)):
            x16 = None if f16 is None or i == 0 else f16[i % 2]
            out16 = None if f16 is None else f16[(i + 1) % 2]
            if self.noise_mode == "epilogue":      # noise drawn in the last layer's epilogue
                with torch.cuda.stream(side):
                    if self.kv_spread:             # KV step i starts with step i (see __init__)
                        side.wait_stream(main)
                    self.kv_step(t, num_steps)
                buf = self.step(x, t, i, out=buf, x16=x16, out16=out16)
                x, buf = buf, x
                continue
            j = i % 2
            nz = self._noise[j]
            with torch.cuda.stream(side):
                if freed[j] is not None:
                    side.wait_event(freed[j])
                self.ops.randn(nz, self.seed, self._noise_offset(i, M, d))
                ready = torch.cuda.Event()
                ready.record(side)
                self.kv_step(t, num_steps)
            buf = self.step(x, t, i, out=buf, noise=nz, noise_ready=ready, x16=x16, out16=out16)
            freed[j] = torch.cuda.Event()
            freed[j].record(main)
            x, buf = buf, x
        main.wait_stream(side)
        return x
