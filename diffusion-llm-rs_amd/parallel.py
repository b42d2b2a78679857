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
* token-parallel replicas (``TokenParallelLinear``): the full 8 MiB int4 weight per rank.

``shard=(world, rank)`` builds the shard rank ``rank`` of a ``world``-way split in a process that
is not part of such a group and disables the collectives (``partial`` gives the un-reduced
output): the one-process emulation the GPU parity tests use to compose the HIP GEMM with the
partition logic.  The local GEMM is pluggable (``local_factory``): on the GPU it is ``QuantLinear``
(HIP kernels); the CPU multi-process tests pass the oracle's restatement so the partition and
collective logic is checked under gloo without a GPU.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


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


def _default_factory(W, bias, bits, group):
    from .linear import QuantLinear
    return QuantLinear.from_weight(W, bias, bits, group)


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

    def all_gather(self, y: torch.Tensor) -> torch.Tensor:
        """The full [M, N] Y from every rank's column slice (one all_gather over the ranks)."""
        parts = [torch.empty(y.shape[0], n1 - n0, dtype=y.dtype, device=y.device)
                 for n0, n1 in (column_range(self.N, self.world, r) for r in range(self.world))]
        dist.all_gather(parts, y.contiguous(), group=self.pg)
        return torch.cat(parts, dim=1)

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

    def partial(self, x: torch.Tensor, x_is_shard: bool = False) -> torch.Tensor:
        """This rank's un-reduced f32 partial X[:, k0:k1] . W^[k0:k1, :] (no bias)."""
        xs = x if x_is_shard else x[:, self.k0:self.k1].contiguous()
        return self.local(xs, out_dtype=torch.float32)

    def _finish(self, y: torch.Tensor, out_dtype) -> torch.Tensor:
        if self.bias is not None:
            y = y + self.bias.to(y.device, torch.float32)[None, :]
        return y.to(out_dtype)

    def forward(self, x: torch.Tensor, out_dtype=torch.float16, x_is_shard: bool = False,
                chunks: int = 1) -> torch.Tensor:
        """``chunks`` > 1 splits the tokens: the all-reduce of chunk i (asynchronous, on the
        collective's own stream) runs while the GEMM of chunk i+1 computes (the
        hidden-dim-sharded loop is communication-bound, so the exchange must hide under compute).
        Rows are independent, so every chunking gives the same per-row partial sums."""
        xs = x if x_is_shard else x[:, self.k0:self.k1].contiguous()
        if not self.collective:
            return self._finish(self.partial(xs, True), out_dtype)
        if self.reduce == "rs_ag":
            return self._forward_rs_ag(xs, out_dtype, chunks)
        if chunks <= 1 or xs.shape[0] < 2:
            y = self.partial(xs, True)   # partial sums stay f32 until reduced
            dist.all_reduce(y, op=dist.ReduceOp.SUM, group=self.pg)
        else:
            parts, works = [], []
            for xc in torch.tensor_split(xs, min(chunks, xs.shape[0]), dim=0):
                yc = self.partial(xc.contiguous(), True)
                works.append(dist.all_reduce(yc, op=dist.ReduceOp.SUM, group=self.pg, async_op=True))
                parts.append(yc)
            for w in works:
                w.wait()
            y = torch.cat(parts, dim=0)
        return self._finish(y, out_dtype)

    def _forward_rs_ag(self, xs: torch.Tensor, out_dtype, chunks: int) -> torch.Tensor:
        """Per token chunk: reduce_scatter(sum) of the f32 partial rows (padded to a multiple of
        the world; asynchronous, so chunk i's exchange overlaps chunk i+1's GEMM), then bias +
        cast on this rank's rows and an all_gather of the cast rows."""
        split = (torch.tensor_split(xs, min(chunks, xs.shape[0]), dim=0) if chunks > 1 and xs.shape[0] > 1
                 else (xs,))
        scattered = []
        for xc in split:
            y = self.partial(xc.contiguous(), True)
            M = y.shape[0]
            Mp = -(-M // self.world) * self.world
            if Mp != M:
                y = torch.cat([y, y.new_zeros(Mp - M, y.shape[1])], dim=0)
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
        per, rem = divmod(M, self.world)
        m0 = self.rank * per + min(self.rank, rem)
        return m0, m0 + per + (1 if self.rank < rem else 0)

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
    def attention(q, k, v):
        from .quantization import kv_attention
        return kv_attention(q, k, v)


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
        sk, sv = self.ops.extremes(keys_local), self.ops.extremes(values_local)
        return torch.stack([-sk[0], sk[1], -sv[0], sv[1]]).contiguous()

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
