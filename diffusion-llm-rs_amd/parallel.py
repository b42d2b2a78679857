"""Multi-GPU partitioning of the quantized linear layer.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on ROCm).  The layer is
``SimpleDiffusionModel::forward = x.dot(W) + b`` (diffuse-llm-rs/src/lib.rs:806-813); its hidden
dimension shards cleanly because the quantization groups (128 rows of one column, a5) never
straddle a column boundary and K/G is a whole number of groups for G <= 32.  Modes:

* column-parallel (``ColumnParallelLinear``): rank r owns output columns [n0, n1) -- the
  per-(column, group) quantization of a shard is bit-identical to the same columns of the
  unsharded layer -- and returns its Y slice; ``gather=True`` all-gathers the full Y.  No
  collective on the data path otherwise (the bench's strong-scaling mode).
* row-parallel (``RowParallelLinear``): rank r owns K-groups [g0, g1) (shards aligned to the
  quantization group, so again bit-identical codes/scales) and computes a partial Y in f32.  The
  partials are combined either by one ``all_reduce(sum)`` of f32 (``reduce="allreduce"``) or by a
  ``reduce_scatter(sum)`` of f32 over token rows, the bias and the output cast on the local rows,
  and an ``all_gather`` of the cast rows (``reduce="rs_ag"``: with f16 output that moves
  (G-1)/G * (4 + 2) B per element instead of the all-reduce's (G-1)/G * 2 * 4 B, and the sum is
  still f32).  The bias is added once, after the reduction.
* Megatron pairing (column then row, ``TensorParallelPair``): one reduction per layer pair.
* token-parallel (``TokenParallelLinear``, ``token_rows``): the full 8 MiB int4 weight on every
  rank, rank r runs its token rows with no collective.  For config C5 (DenoiseLoop with
  ``noise_rows``) each rank also holds its rows of K/V in a ``HeadParallelKVCacheEntry`` (one
  4-float all_reduce(MAX) per quantization): the bench's ``denoise_loop_dp``.

``shard=(world, rank)`` builds the shard rank ``rank`` of a ``world``-way split in a process that
is not part of such a group and disables the collectives (``partial`` gives the un-reduced
output; a row shard's ``forward`` refuses, since its output would lack the other ranks' sums and
carry the whole bias): the one-process emulation the GPU parity tests use to compose the HIP GEMM
with the partition logic (their helpers, which put all G shards behind the unsharded interface,
live in tests/tp_emulation.py).  The local layer is pluggable (``local_factory``): on the GPU it is
``QuantLinear`` (HIP kernels: the GEMM and the row-parallel epilogue ``bias_cast``); the CPU
multi-process tests pass the oracle's restatement so the partition and collective logic is checked
under gloo without a GPU.  A local layer is built as ``local_factory(W_shard, bias_shard, bits,
group)`` and called as ``local(x, out_dtype=..., out=...)``; it may provide
``bias_cast(y, bias, out_dtype)`` for the row-parallel epilogue (QuantLinear's is the library
kernel), otherwise that epilogue is ``(y + bias).to(out_dtype)``.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

from .diffusion import KVCacheEntry
from .quantization import QuantizedKVCacheEntry, QuantizedTensor


def _world(pg=None, shard=None):
    if shard is not None:
        world, rank = int(shard[0]), int(shard[1])
        if not 0 <= rank < world:
            raise ValueError(f"shard rank {rank} outside world {world}")
        return world, rank
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(pg), dist.get_rank(pg)


def column_range(N: int, world: int, rank: int, align: int = 32):
    """Contiguous output-column shard [n0, n1); boundaries on multiples of ``align`` (the MFMA
    n-tile) except the last."""
    units = (N + align - 1) // align
    per, rem = divmod(units, world)
    u0 = rank * per + min(rank, rem)
    u1 = u0 + per + (1 if rank < rem else 0)
    return min(u0 * align, N), min(u1 * align, N)


def row_range(K: int, world: int, rank: int, group: int = 128):
    """K shard [k0, k1) made of whole quantization groups (so shard quantization == unsharded)."""
    G = (K + group - 1) // group
    per, rem = divmod(G, world)
    g0 = rank * per + min(rank, rem)
    g1 = g0 + per + (1 if rank < rem else 0)
    return min(g0 * group, K), min(g1 * group, K)


def token_rows(M: int, world: int, rank: int):
    """Contiguous token-row shard [r0, r1) of an M-token batch or sample (token parallelism: the
    linear layers and p_sample are per token, so rank r runs rows r0..r1 through replicated layers
    with no collective; in the denoise loop its K/V rows go to a sharded cache,
    HeadParallelKVCacheEntry).  Every rank gets at least one row: ``world <= M`` is required (an
    empty shard would still have to join the KV step's all_reduce, and DenoiseLoop refuses a zero-row
    x), so a larger world raises instead of handing some ranks nothing."""
    if not 1 <= world <= M or not 0 <= rank < world:
        raise ValueError(f"token_rows: need 1 <= world <= M and 0 <= rank < world (M={M}, world={world}, rank={rank})")
    per, rem = divmod(M, world)
    r0 = rank * per + min(rank, rem)
    return r0, r0 + per + (1 if rank < rem else 0)


def _default_factory(W, bias, bits, group):
    """The shards serve the denoise loop's layers (M = the tokens of a sequence): prefill-only
    handles, without the decode layout (an M <= 64 call still runs, on the prefill kernels)."""
    from .linear import QuantLinear
    return QuantLinear.from_weight(W, bias, bits, group, prefill_only=True)


class ColumnParallelLinear:
    def __init__(self, W: torch.Tensor, bias: Optional[torch.Tensor], bits: int = 4, group: int = 128, pg=None,
                 gather: bool = False, local_factory: Callable = _default_factory, n_range=None, shard=None):
        self.pg, self.gather = pg, gather
        self.world, self.rank = _world(pg, shard)
        self.collective = shard is None and self.world > 1
        K, N = W.shape
        self.K, self.N = K, N
        self.n0, self.n1 = n_range if n_range is not None else column_range(N, self.world, self.rank)
        b = None if bias is None else bias[self.n0:self.n1].contiguous()
        self.local = local_factory(W[:, self.n0:self.n1].contiguous(), b, bits, group)

    def forward(self, x: torch.Tensor, out_dtype=torch.float16) -> torch.Tensor:
        y = self.local(x, out_dtype=out_dtype)
        if not self.gather or not self.collective:
            return y
        return self.all_gather(y)

    def _widths(self):
        return [n1 - n0 for n0, n1 in (column_range(self.N, self.world, r) for r in range(self.world))]

    def all_gather(self, y: torch.Tensor, out: Optional[torch.Tensor] = None, async_op: bool = False):
        """The full [M, N] Y (row-major, into ``out`` when given) from every rank's column slice: ONE
        all_gather_into_tensor of the [M, w] slices into a rank-major [world * M, w] buffer, then the
        slices are laid side by side into Y's rows (unequal slices -- N not a multiple of 32 x world
        -- travel padded to the widest).  ``async_op``: returns ``(finish, out)`` -- the exchange is
        in flight on the collective's stream, and ``finish()`` makes the current stream wait for it
        and writes ``out``."""
        M = y.shape[0]
        if out is None:
            out = torch.empty(M, self.N, dtype=y.dtype, device=y.device)
        widths = self._widths()
        wmax = max(widths)
        if y.shape[1] == wmax:
            y = y.contiguous()
        else:
            yp = torch.zeros(M, wmax, dtype=y.dtype, device=y.device)
            yp[:, :y.shape[1]] = y
            y = yp
        buf = torch.empty(self.world * M, wmax, dtype=y.dtype, device=y.device)   # rank-major slices
        work = dist.all_gather_into_tensor(buf, y, group=self.pg, async_op=async_op)

        def finish():
            if work is not None:
                work.wait()
            parts = buf.view(self.world, M, wmax)
            if len(set(widths)) == 1:
                out.view(M, self.world, wmax).copy_(parts.transpose(0, 1))
            else:
                for r, (n0, n1) in enumerate(column_range(self.N, self.world, q) for q in range(self.world)):
                    out[:, n0:n1] = parts[r, :, :n1 - n0]
            return out

        if async_op:
            return finish, out
        return finish()

    def forward_gathered(self, x: torch.Tensor, out: Optional[torch.Tensor] = None, out_dtype=torch.float16,
                         chunks: int = 1, stage: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The whole layer on every rank: Y = x.dot(W) + b as the full [M, N] (lib.rs:806-813) from
        the column shards -- each rank's slice GEMM, then the all-gather of the slices.  ``chunks`` > 1
        splits the tokens: chunk i's all-gather (asynchronous, on the collective's stream) runs while
        chunk i+1's GEMM computes.  Rows are independent, so every chunking gives the same Y.
        ``stage``: an optional [M, n1 - n0] buffer for the local slices."""
        M = x.shape[0]
        if out is None:
            out = torch.empty(M, self.N, dtype=out_dtype, device=x.device)
        if stage is None:
            stage = torch.empty(M, self.n1 - self.n0, dtype=out.dtype, device=x.device)
        if not self.collective:
            if self.world > 1:
                raise ValueError("forward_gathered needs the ranks' collective (shard emulation has none)")
            return self.local(x, out_dtype=out.dtype, out=out)
        pending, r0 = [], 0
        for xc in (torch.tensor_split(x, min(chunks, M), dim=0) if chunks > 1 and M > 1 else (x,)):
            r1 = r0 + xc.shape[0]
            yc = self.local(xc, out_dtype=out.dtype, out=stage[r0:r1])
            pending.append(self.all_gather(yc, out=out[r0:r1], async_op=True)[0])
            r0 = r1
        for finish in pending:
            finish()
        return out

    __call__ = forward


class RowParallelLinear:
    REDUCE_MODES = ("allreduce", "rs_ag")

    def __init__(self, W: torch.Tensor, bias: Optional[torch.Tensor], bits: int = 4, group: int = 128, pg=None,
                 local_factory: Callable = _default_factory, shard=None, reduce: str = "allreduce"):
        if reduce not in self.REDUCE_MODES:
            raise ValueError(f"reduce must be one of {self.REDUCE_MODES}")
        self.pg, self.reduce = pg, reduce
        self.world, self.rank = _world(pg, shard)
        self.collective = shard is None and self.world > 1
        K, N = W.shape
        self.K, self.N = K, N
        self.k0, self.k1 = row_range(K, self.world, self.rank, group)
        self.bias = bias
        self.local = local_factory(W[self.k0:self.k1].contiguous(), None, bits, group)

    def partial(self, x: torch.Tensor, x_is_shard: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """This rank's un-reduced f32 partial X[:, k0:k1] . W^[k0:k1, :] (no bias), into ``out`` when given."""
        xs = x if x_is_shard else x[:, self.k0:self.k1].contiguous()
        if out is None:
            return self.local(xs, out_dtype=torch.float32)
        return self.local(xs, out=out, out_dtype=torch.float32)

    def _finish(self, y: torch.Tensor, out_dtype) -> torch.Tensor:
        """The bias, once, after the reduction, and the output cast: the local layer's epilogue
        (``QuantLinear.bias_cast`` = dllm_bias_cast, lib.rs:812)."""
        bias = None if self.bias is None else self.bias.to(y.device, torch.float32)
        cast = getattr(self.local, "bias_cast", None)
        if cast is None or out_dtype not in (torch.float16, torch.float32):
            # a local layer without the library epilogue (a custom local_factory), or an output type
            # the kernel does not store: the same sum in f32, then the cast
            yb = y if bias is None else y + bias
            return yb.to(out_dtype)
        return cast(y, bias, out_dtype)

    @staticmethod
    def _padded(M: int, Mp: int, N: int, device) -> torch.Tensor:
        """A fresh [Mp, N] f32 buffer whose rows M.. (the padding) are zero; the GEMM writes rows
        ..M.  Allocated per call from the stream-ordered caching allocator, so nothing is shared
        between concurrent forwards and nothing accumulates per sequence length."""
        y = torch.empty(Mp, N, dtype=torch.float32, device=device)
        y[M:].zero_()
        return y

    def forward(self, x: torch.Tensor, out_dtype=torch.float16, x_is_shard: bool = False,
                chunks: int = 1) -> torch.Tensor:
        """``chunks`` > 1 splits the tokens: the all-reduce of chunk i (asynchronous, on the
        collective's own stream) runs while the GEMM of chunk i+1 computes (the
        hidden-dim-sharded loop is communication-bound, so the exchange must hide under compute).
        Rows are independent, so every chunking gives the same per-row partial sums."""
        xs = x if x_is_shard else x[:, self.k0:self.k1].contiguous()
        if not self.collective:
            if self.world > 1:   # shard emulation: the reduction belongs to the caller
                raise ValueError("a row shard's forward needs the reduction over its ranks: use partial() "
                                 "(or EmulatedTensorParallel) under shard=(world, rank)")
            return self._finish(self.partial(xs, True), out_dtype)
        if self.reduce == "rs_ag":
            return self._forward_rs_ag(xs, out_dtype, chunks)
        if chunks <= 1 or xs.shape[0] < 2:
            y = self.partial(xs, True)   # partial sums stay f32 until reduced
            dist.all_reduce(y, op=dist.ReduceOp.SUM, group=self.pg)
        else:
            # each chunk's partial goes straight into its rows of y (row blocks are contiguous views)
            y = torch.empty(xs.shape[0], self.N, dtype=torch.float32, device=xs.device)
            works, r0 = [], 0
            for xc in torch.tensor_split(xs, min(chunks, xs.shape[0]), dim=0):
                yc = y[r0:r0 + xc.shape[0]]
                self.partial(xc, True, out=yc)
                works.append(dist.all_reduce(yc, op=dist.ReduceOp.SUM, group=self.pg, async_op=True))
                r0 += xc.shape[0]
            for w in works:
                w.wait()
        return self._finish(y, out_dtype)

    def _forward_rs_ag(self, xs: torch.Tensor, out_dtype, chunks: int) -> torch.Tensor:
        """Per token chunk: reduce_scatter(sum) of the f32 partial rows (padded to a multiple of
        the world; asynchronous, so chunk i's exchange overlaps chunk i+1's GEMM), then bias +
        cast on this rank's rows and an all_gather of the cast rows."""
        split = (torch.tensor_split(xs, min(chunks, xs.shape[0]), dim=0) if chunks > 1 and xs.shape[0] > 1
                 else (xs,))
        scattered = []
        for c, xc in enumerate(split):
            M = xc.shape[0]
            Mp = -(-M // self.world) * self.world
            if Mp == M:
                y = self.partial(xc, True)
            else:   # the chunk's rows padded to a multiple of the world with zero rows
                y = self._padded(M, Mp, self.N, xc.device)
                self.partial(xc, True, out=y[:M])
            mine = torch.empty(Mp // self.world, y.shape[1], dtype=torch.float32, device=y.device)
            work = dist.reduce_scatter_tensor(mine, y, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            scattered.append((work, mine, y, M))
        gathered = []
        for work, mine, y, M in scattered:
            work.wait()
            rows = self._finish(mine, out_dtype).contiguous()
            full = torch.empty(y.shape[0], y.shape[1], dtype=out_dtype, device=y.device)
            gathered.append((dist.all_gather_into_tensor(full, rows, group=self.pg, async_op=True), full, M))
        outs = []
        for work, full, M in gathered:
            work.wait()
            outs.append(full[:M])
        return outs[0] if len(outs) == 1 else torch.cat(outs, dim=0)

    __call__ = forward


class TensorParallelPair:
    """Megatron pairing: column-parallel A (K -> H, no gather) then row-parallel B (H -> N) whose
    K-shard is exactly A's column shard, so the only collective is B's reduction."""

    def __init__(self, WA, bA, WB, bB, bits: int = 4, group: int = 128, pg=None,
                 local_factory: Callable = _default_factory, shard=None, reduce: str = "allreduce"):
        world, rank = _world(pg, shard)
        H = WA.shape[1]
        if H % (group * world) != 0:
            raise ValueError("hidden size must split into whole groups per rank")
        # A's column shard must equal B's row shard: group-aligned column ranges.
        self.a = ColumnParallelLinear(WA, bA, bits, group, pg, gather=False, local_factory=local_factory,
                                      n_range=row_range(H, world, rank, group), shard=shard)
        self.b = RowParallelLinear(WB, bB, bits, group, pg, local_factory=local_factory, shard=shard, reduce=reduce)
        assert (self.b.k0, self.b.k1) == (self.a.n0, self.a.n1)

    chunks = 1   # default token chunking of the reduction overlap (callers such as DenoiseLoop pass none)

    def partial(self, x: torch.Tensor) -> torch.Tensor:
        """This rank's un-reduced f32 partial of B(f16(A_shard(x))) (emulation / tests)."""
        return self.b.partial(self.a(x, out_dtype=torch.float16), x_is_shard=True)

    def forward(self, x: torch.Tensor, out_dtype=torch.float16, chunks: Optional[int] = None) -> torch.Tensor:
        h = self.a(x, out_dtype=torch.float16)
        return self.b(h, out_dtype=out_dtype, x_is_shard=True, chunks=self.chunks if chunks is None else chunks)

    def close(self):
        for part in (self.a.local, self.b.local):
            if hasattr(part, "close"):
                part.close()

    __call__ = forward


class TokenParallelLinear:
    """Replicas: rank r processes tokens [m0, m1) of a global batch with the full weight."""

    def __init__(self, W, bias, bits: int = 4, group: int = 128, pg=None, local_factory: Callable = _default_factory,
                 shard=None):
        self.pg = pg
        self.world, self.rank = _world(pg, shard)
        self.local = local_factory(W, bias, bits, group)

    def token_range(self, M: int):
        return token_rows(M, self.world, self.rank)

    def forward(self, x_local: torch.Tensor, out_dtype=torch.float16) -> torch.Tensor:
        return self.local(x_local, out_dtype=out_dtype)

    __call__ = forward


def head_range(H: int, world: int, rank: int):
    """Contiguous head shard [h0, h1) (heads are independent in attention)."""
    per, rem = divmod(H, world)
    h0 = rank * per + min(rank, rem)
    return h0, h0 + per + (1 if rank < rem else 0)


class DeviceKVOps:
    """The per-shard device steps of :class:`HeadParallelKVCache` (HIP kernels behind the C-ABI)."""

    @staticmethod
    def extremes(x):
        from .quantization import tensor_extremes
        return tensor_extremes(x)

    @staticmethod
    def params(stats, bits):
        from .quantization import quantize_params_from_extremes
        return quantize_params_from_extremes(stats, bits)

    @staticmethod
    def quantize(x, bits, params):
        from .quantization import quantize_tensor_with_params
        return quantize_tensor_with_params(x, bits, params, packed=True)

    @staticmethod
    def dequantize(t):
        return t.dequantize().reshape(t.shape)

    @staticmethod
    def quantize_pair(x, bits_a, bits_b, params_a, params_b):
        from .quantization import quantize_tensor_pair_with_params
        return quantize_tensor_pair_with_params(x, bits_a, bits_b, params_a, params_b, packed=True)

    @staticmethod
    def attention(q, k, v):
        from .quantization import kv_attention
        return kv_attention(q, k, v)

    @staticmethod
    def kv_extremes(k, v):
        """{-min_K, max_K, -min_V, max_V} of the local shards in one launch (dllm_kv_extremes)."""
        from .quantization import kv_extremes
        return kv_extremes(k, v)

    @staticmethod
    def quantize_kv(k, v, red, bits_a, bits_b):
        """Both tensors' params and codes from the reduced extremes (dllm_quantize_kv_with_extremes)."""
        from .quantization import quantize_kv_with_extremes
        return quantize_kv_with_extremes(k, v, red, bits_a, bits_b, packed=True)


class HeadParallelKVCache:
    """``QuantizedKVCacheEntry`` (diffuse-llm-rs/src/quantization.rs:140-175) with K and V sharded
    by head over the ranks: rank r holds heads [h0, h1) of K, V, Q ``[S, H, D]`` as
    its own contiguous ``[S, h1-h0, D]`` tensors.

    The reference quantizes K and V per WHOLE tensor (one scale / zero point each, :142-150), so
    the shards need the global extremes: each rank folds its shard (NaN-ignoring min/max, the
    order-independent reduction of :41-46), one ``all_reduce(MAX)`` of 4 floats {-min_K, max_K,
    -min_V, max_V} combines K and V, and every rank writes the params and codes the unsharded
    ``quantize_tensor`` writes for its elements -- bit for bit.  Attention is per head, so it runs
    on the local heads with no exchange.  ``ops`` is pluggable (``DeviceKVOps`` on the GPU; the CPU
    gloo tests pass the oracle's restatement)."""

    def __init__(self, H: int, bits: int = 4, pg=None, ops=DeviceKVOps):
        self.pg, self.bits, self.ops = pg, int(bits), ops
        self.world, self.rank = _world(pg)
        self.H = H
        self.h0, self.h1 = head_range(H, self.world, self.rank)

    def local_extremes(self, keys_local: torch.Tensor, values_local: torch.Tensor) -> torch.Tensor:
        """This rank's {-min_K, max_K, -min_V, max_V} (the all-reduce operand; NaN skipped)."""
        return _local_extremes_of(keys_local, values_local, self.ops)

    def quantize_with_extremes(self, keys_local: torch.Tensor, values_local: torch.Tensor, red: torch.Tensor):
        """Params and local codes from the all-reduced extremes ``red``."""
        kp = self.ops.params(torch.stack([-red[0], red[1]]), self.bits)
        vp = self.ops.params(torch.stack([-red[2], red[3]]), self.bits)
        return (self.ops.quantize(keys_local, self.bits, kp), kp, self.ops.quantize(values_local, self.bits, vp), vp)

    def quantize(self, keys_local: torch.Tensor, values_local: torch.Tensor):
        """QuantizedKVCacheEntry::new(keys, values, bits) on the local heads (global per-tensor params).
        Returns ``(k_codes, k_params, v_codes, v_params)``: packed local codes, device params."""
        red = self.local_extremes(keys_local, values_local)
        if self.world > 1:
            dist.all_reduce(red, op=dist.ReduceOp.MAX, group=self.pg)
        return self.quantize_with_extremes(keys_local, values_local, red)

    def entry(self, keys_local: torch.Tensor, values_local: torch.Tensor, red: Optional[torch.Tensor] = None):
        """The local shard as a ``QuantizedKVCacheEntry``; ``red`` = already all-reduced extremes."""
        from .quantization import QuantizedKVCacheEntry, QuantizedTensor
        kc, kp, vc, vp = (self.quantize(keys_local, values_local) if red is None
                          else self.quantize_with_extremes(keys_local, values_local, red))
        ks, vs = tuple(keys_local.shape), tuple(values_local.shape)
        seq = int(keys_local.shape[0]) if keys_local.dim() == 3 else 0
        return QuantizedKVCacheEntry(QuantizedTensor(kc, ks, kp, self.bits, True),
                                     QuantizedTensor(vc, vs, vp, self.bits, True), seq)

    def attention(self, q_local: torch.Tensor, entry) -> torch.Tensor:
        """Dequant-attention of the local heads: O[:, h0:h1, :] of the unsharded call."""
        return self.ops.attention(q_local, entry.keys, entry.values)


# ---- config C5 sharded as a whole loop: the phase-aware KV cache by head, emulation helpers ----------

def head_columns(hidden: int, num_heads: int, world: int, rank: int):
    """Hidden-column shard [c0, c1) of rank ``rank``: its heads [h0, h1) (head_range) times head_dim
    (hidden = num_heads * head_dim, the K/V layout [layers, seq, heads * head_dim] of
    init_kv_cache, diffuse-llm-rs/src/lib.rs:958-980)."""
    if hidden % num_heads:
        raise ValueError("hidden size must be a whole number of heads")
    hd = hidden // num_heads
    h0, h1 = head_range(num_heads, world, rank)
    return h0 * hd, h1 * hd


class HeadParallelKVCacheEntry(KVCacheEntry):
    """``KVCacheEntry`` (diffuse-llm-rs/src/lib.rs:121-313: f32 K/V plus a prefill-width and a
    decode-width per-tensor quantized copy, phase switch, progressive decode widths, re-quantizing
    ``update``) with K and V sharded by head over the ranks: rank r holds the hidden
    columns of its heads (``head_columns``) of K, V ``[layers, seq, hidden]`` as contiguous local
    tensors -- or its token rows (``token_rows``, the token-parallel denoise loop): the quantization
    below needs only the shard's elements and the global extremes, so any disjoint split works.  The
    phase logic and the accounting (lib.rs:279-302, per shard) are KVCacheEntry's.

    The reference quantizes K and V per WHOLE tensor (quantization.rs:142-150), so a shard's
    params need the global extremes: each quantization folds the local K and V (NaN-ignoring,
    order-independent, :41-46), combines {-min_K, max_K, -min_V, max_V} over the ranks with ONE
    ``all_reduce(MAX)`` of 4 floats, and derives the params of every width it writes from that one
    result (:49-56) -- an update's prefill and decode copies come from the same reduction, both
    widths written in one read of the shard (dllm_quantize_tensor_pair_with_params).  Codes and
    params are bit-identical to the unsharded entry's for the shard's elements.
    ``transition_phase`` re-quantizes the same K/V the last quantization reduced, so it reuses that
    reduction (no collective; bit-identical).  ``red``: extremes already reduced over the ranks
    (the one-process emulation supplies them); ``ops``: the per-shard device steps
    (``DeviceKVOps``; the CPU gloo tests pass the oracle's)."""

    def __init__(self, keys_local, values_local, prefill_bits, decode_bits, pg=None, ops=DeviceKVOps,
                 red=None):
        self.pg, self.ops = pg, ops
        self.world, self.rank = _world(pg)
        self._red_next = red       # the emulation's pre-reduced extremes for the next quantization
        self._red_of = None        # (keys, values, reduced extremes) of the last quantization
        self._reuse = True         # the constructor's two widths share one reduction
        super().__init__(keys_local, values_local, prefill_bits, decode_bits)
        self._reuse = False

    def transition_phase(self, is_prefill: bool):
        """lib.rs:221-239; a decode copy made here quantizes the K/V of the last reduction."""
        self._reuse = True
        try:
            super().transition_phase(is_prefill)
        finally:
            self._reuse = False

    def update(self, new_keys, new_values):
        """lib.rs:241-276: one fresh reduction of the new K/V for both widths."""
        self._red_of = None
        super().update(new_keys, new_values)

    def local_extremes(self, keys, values):
        """This shard's {-min_K, max_K, -min_V, max_V} (the all-reduce operand; NaN skipped)."""
        return _local_extremes_of(keys, values, self.ops)

    def _reduced(self, keys, values):
        last = self._red_of
        if self._reuse and last is not None and last[0] is keys and last[1] is values:
            return last[2]
        if self._red_next is not None:
            red, self._red_next = self._red_next, None
        else:
            red = self.local_extremes(keys, values)
            if self.world > 1:
                dist.all_reduce(red, op=dist.ReduceOp.MAX, group=self.pg)
        self._red_of = (keys, values, red)
        return red

    def _dequantize(self, t):
        return self.ops.dequantize(t)

    def _params(self, red, bits):
        return (self.ops.params(torch.stack([-red[0], red[1]]), bits),
                self.ops.params(torch.stack([-red[2], red[3]]), bits))

    def _entry(self, keys, values, kc, kp, vc, vp, bits):
        seq = int(keys.shape[1]) if keys.dim() > 1 else 0
        return QuantizedKVCacheEntry(QuantizedTensor(kc, tuple(keys.shape), kp, int(bits), True),
                                     QuantizedTensor(vc, tuple(values.shape), vp, int(bits), True), seq)

    def _quantize(self, keys, values, bits):
        red = self._reduced(keys, values)
        if hasattr(self.ops, "quantize_kv"):   # both tensors' params and codes in one launch
            (kc, kp, vc, vp), = self.ops.quantize_kv(keys, values, red, bits, 0)
            return self._entry(keys, values, kc, kp, vc, vp, bits)
        kp, vp = self._params(red, bits)
        return self._entry(keys, values, self.ops.quantize(keys, bits, kp), kp, self.ops.quantize(values, bits, vp),
                           vp, bits)

    def _quantize_pair(self, keys, values, bits_a, bits_b):
        red = self._reduced(keys, values)
        if hasattr(self.ops, "quantize_kv"):   # both tensors at both widths in one launch
            (kca, kpa, vca, vpa), (kcb, kpb, vcb, vpb) = self.ops.quantize_kv(keys, values, red, bits_a, bits_b)
            return (self._entry(keys, values, kca, kpa, vca, vpa, bits_a),
                    self._entry(keys, values, kcb, kpb, vcb, vpb, bits_b))
        (kpa, vpa), (kpb, vpb) = self._params(red, bits_a), self._params(red, bits_b)
        kca, kcb = self.ops.quantize_pair(keys, bits_a, bits_b, kpa, kpb)
        vca, vcb = self.ops.quantize_pair(values, bits_a, bits_b, vpa, vpb)
        return (self._entry(keys, values, kca, kpa, vca, vpa, bits_a),
                self._entry(keys, values, kcb, kpb, vcb, vpb, bits_b))


def _local_extremes_of(keys, values, ops=DeviceKVOps):
    if hasattr(ops, "kv_extremes"):
        return ops.kv_extremes(keys, values)
    sk, sv = ops.extremes(keys), ops.extremes(values)
    return torch.stack([-sk[0], sk[1], -sv[0], sv[1]]).contiguous()
