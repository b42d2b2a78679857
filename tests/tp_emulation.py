"""One-process emulation of the tensor-parallel layers and the head-sharded KV cache (test
infrastructure: the GPU parity tests and measurement scripts, never the product path).

``EmulatedTensorParallel`` and ``EmulatedHeadParallelKV`` put all G shards of a layer / of the KV
cache (built with ``shard=(G, r)`` / per-rank head columns) behind the unsharded interface,
replacing each collective by its definition -- the f32 sum of the partials in rank order for the
pair's all_reduce(SUM), the max of the shards' extremes for the cache's all_reduce(MAX) -- so that a
whole ``DenoiseLoop`` runs sharded in one process (diffuse-llm-rs/src/lib.rs:853-955).
"""
from __future__ import annotations

import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
import __graft_entry__ as _g  # noqa: E402

_par = _g.load_package().parallel
head_columns = _par.head_columns
HeadParallelKVCacheEntry = _par.HeadParallelKVCacheEntry
TensorParallelPair = _par.TensorParallelPair
DeviceKVOps = _par.DeviceKVOps
_local_extremes_of = _par._local_extremes_of


class EmulatedHeadParallelKV:
    """All G head shards of one KV cache entry in one process behind KVCacheEntry's interface (what
    ``DenoiseLoop.kv_step`` calls): each quantization folds every shard's extremes, takes their max
    (the all_reduce(MAX) by definition) and hands it to every shard.  ``keys``/``values`` are the
    lists of shard tensors; ``get_keys``/``get_values`` concatenate the shards' hand-outs along the
    hidden dimension (the unsharded entry's tensor, for comparison)."""

    def __init__(self, keys, values, prefill_bits, decode_bits, num_heads, world, ops=DeviceKVOps, split="heads"):
        """``split="rows"``: the shards are token rows (``parallel.token_rows`` of the seq axis, the
        token-parallel loop) instead of head columns; ``cols`` then holds the row ranges."""
        if split not in ("heads", "rows"):
            raise ValueError("split must be 'heads' or 'rows'")
        self.split = split
        hidden = keys.shape[-1]
        self.world, self.num_heads = world, num_heads
        if split == "heads":
            self.cols = [head_columns(hidden, num_heads, world, r) for r in range(world)]
        else:
            self.cols = [_par.token_rows(keys.shape[1], world, r) for r in range(world)]
        ks = [self._part(keys, c) for c in self.cols]
        vs = [self._part(values, c) for c in self.cols]
        red = torch.stack([_local_extremes_of(k, v, ops) for k, v in zip(ks, vs)]).amax(0)
        self.shards = [HeadParallelKVCacheEntry(k, v, prefill_bits, decode_bits, ops=ops, red=red) for k, v in zip(ks, vs)]

    def _part(self, t, c):
        c0, c1 = c
        return (t[..., c0:c1] if self.split == "heads" else t[:, c0:c1]).contiguous()

    def _reduce_for(self, keys, values):
        red = torch.stack([s.local_extremes(k, v) for s, k, v in zip(self.shards, keys, values)]).amax(0)
        for s in self.shards:
            s._red_next = red

    # -- KVCacheEntry's interface ------------------------------------------------------------------
    keys = property(lambda self: [s.keys for s in self.shards])
    values = property(lambda self: [s.values for s in self.shards])
    is_prefill_phase = property(lambda self: self.shards[0].is_prefill_phase)
    prefill_quant_bits = property(lambda self: self.shards[0].prefill_quant_bits)

    @property
    def decode_quant_bits(self):
        return self.shards[0].decode_quant_bits

    @decode_quant_bits.setter
    def decode_quant_bits(self, b):
        for s in self.shards:
            s.decode_quant_bits = b

    @property
    def decode_quantized(self):
        return [s.decode_quantized for s in self.shards] if self.shards[0].decode_quantized is not None else None

    @decode_quantized.setter
    def decode_quantized(self, v):
        if v is not None:
            raise ValueError("only None (drop the decode copy, lib.rs:900-903) can be assigned")
        for s in self.shards:
            s.decode_quantized = None

    @property
    def prefill_quantized(self):
        return [s.prefill_quantized for s in self.shards] if self.shards[0].prefill_quantized is not None else None

    def set_phase(self, is_prefill: bool):
        for s in self.shards:
            s.set_phase(is_prefill)

    transition_phase = set_phase

    def get_current_quant_bits(self) -> int:
        return self.shards[0].get_current_quant_bits()

    def get_keys(self):
        return torch.cat([s.get_keys() for s in self.shards], dim=-1 if self.split == "heads" else 1)

    def get_values(self):
        return torch.cat([s.get_values() for s in self.shards], dim=-1 if self.split == "heads" else 1)

    def update(self, new_keys, new_values):
        """KVCacheEntry::update of every shard; ``new_keys``/``new_values`` are the shard lists (as
        ``keys``/``values`` hand them out) or full tensors, which are split by head here."""
        if isinstance(new_keys, torch.Tensor):
            new_keys = [self._part(new_keys, c) for c in self.cols]
            new_values = [self._part(new_values, c) for c in self.cols]
        self._reduce_for(new_keys, new_values)
        for s, k, v in zip(self.shards, new_keys, new_values):
            s.update(k, v)

    def memory_usage(self) -> int:
        return sum(s.memory_usage() for s in self.shards)

    def __len__(self):
        return len(self.shards[0])




class EmulatedTensorParallel:
    """All G shards of a tensor-parallel layer (``TensorParallelPair`` or ``RowParallelLinear``
    built with ``shard=(G, r)``) in one process behind the unsharded layer's call: the f32 partials
    summed in rank order (the all-reduce by definition), then the bias once and the output cast --
    what every rank holds after the pair's reduction."""

    def __init__(self, shards):
        self.shards = list(shards)
        last = self.shards[0]
        self.bias = (last.b if isinstance(last, TensorParallelPair) else last).bias

    def __call__(self, x, out_dtype=torch.float16):
        tot = None
        for s in self.shards:
            p = s.partial(x)
            tot = p if tot is None else tot.add_(p)
        row = self.shards[0].b if isinstance(self.shards[0], TensorParallelPair) else self.shards[0]
        return row._finish(tot, out_dtype)   # the real path's epilogue: bias once, then the cast

    forward = __call__

    def close(self):
        for s in self.shards:
            if hasattr(s, "close"):
                s.close()
