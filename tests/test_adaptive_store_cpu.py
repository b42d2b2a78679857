"""AdaptiveQuantizer (diffuse-llm-rs/src/quantization.rs:178-235) and the
DiffuseLLM KV-cache registry (8f rank 2; lib.rs:958-1084) on the CPU.

- The two oracle restatements of AdaptiveQuantizer agree bit for bit.
- They reproduce the reference's own property test (:267-277).
- The product's argument checks fire before any launch.
- KVCacheStore's accounting and eviction policy (host logic) match the reference's arithmetic,
  driven by a stand-in entry whose memory_usage() is set by the test.

CKMS parity is unpinned: the quantiles crate is absent, and the q = 0 / 1 queries are restated as
the exact extremes."""
import math

import numpy as np
import pytest


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


DATA = {
    "ramp": np.arange(1000, dtype=np.float32) / 1000,
    "normal": np.random.default_rng(5).standard_normal(5003).astype(np.float32) * 7,
    "const": np.full(9, 3.0, np.float32),
    "empty": np.zeros(0, np.float32),
    "nan": np.array([-5, np.nan, 2, np.inf], np.float32),
    "neg": -np.abs(np.random.default_rng(6).standard_normal(300).astype(np.float32)) - 1,
}


@pytest.mark.parametrize("nbits", [0, 1, 2, 4, 8, 9, 12, 16, 24, 25, 31])
@pytest.mark.parametrize("name", sorted(DATA))
def test_adaptive_oracles_agree(orc, onp, nbits, name):
    x = DATA[name]
    a, b = orc.AdaptiveQuantizer(nbits), onp.AdaptiveQuantizer(nbits)
    for chunk in np.array_split(x, 3):   # streaming updates
        a.update_stats(chunk)
        b.update_stats(chunk)
    qa, sa, za = a.quantize(x)
    qb, sb, zb = b.quantize(x)
    assert np.array_equal(qa, qb)
    same = (bits([sa, za]) == bits([sb, zb])) | (np.isnan([sa, za]) & np.isnan([sb, zb]))
    assert same.all()


def test_adaptive_reference_property_test(orc):
    """quantization.rs:267-277: 0..1000 / 1000 at 4 bits -> scale > 0, zero_point >= 0."""
    q = orc.AdaptiveQuantizer(4, 4.0)
    q.update_stats(np.arange(1000, dtype=np.float32) / 1000.0)
    s, z = q.compute_params()
    assert s > 0 and z >= 0
    # the literal values: max 0.999, min 0 -> scale = 0.999 / 15, zp = round(-0 / s) = -0.0
    assert bits(s) == bits(np.float32(np.float32(0.999) / np.float32(15.0)))
    assert bits(z) == bits(np.float32(-0.0))


def test_adaptive_defaults_without_samples(orc):
    """query(..) is None on an empty summary -> unwrap_or(0.0) / unwrap_or(1.0) (:209-210)."""
    s, z = orc.AdaptiveQuantizer(8).compute_params()
    assert s == np.float32(1.0) / np.float32(255.0) and z == 0.0


def test_adaptive_quantize_rounds_then_clamps(orc):
    """zp = round(-min / scale).clamp(0, q_max): a positive minimum gives a negative round that
    clamps to 0; the map then clamps codes to [0, q_max]."""
    q = orc.AdaptiveQuantizer(2)
    q.update_stats(np.array([10.0, 13.0], np.float32))
    codes, s, z = q.quantize(np.array([9.0, 10.0, 11.5, 13.0, 100.0], np.float32))
    assert s == np.float32(1.0) and z == 0.0
    assert codes.tolist() == [3, 3, 3, 3, 3]   # x / 1 + 0 >= 9 -> clamped to q_max = 3


def test_adaptive_capi_argument_checks(dllm):
    L = dllm._lib.load()
    E = dllm._lib.ERR_INVALID_PARAMS
    assert L.dllm_adaptive_compute_params(None, 0, 32, None, None) == E
    assert L.dllm_adaptive_quantize(None, 4, 9, None, 1, None, None) == E    # packed needs 1..8
    assert L.dllm_adaptive_quantize(None, 4, 0, None, 1, None, None) == E
    assert L.dllm_adaptive_quantize(None, 4, 40, None, 0, None, None) == E
    assert L.dllm_adaptive_update(None, 0, None, None, 0, None) == E           # null stats


# ---- KVCacheStore: lib.rs:958-1084 accounting and eviction --------------------------------------

class FakeEntry:
    """Stands in for KVCacheEntry: memory_usage() = the packed size of both phases."""

    def __init__(self, keys, values, pb, db):
        self.keys, self.values, self.bits = keys, values, (pb, db)
        self.updates = 0

    def _packed(self, b):
        return 2 * ((self.keys.numel() * b + 7) // 8) if b else 0

    def memory_usage(self):
        t = self._packed(self.bits[0]) + self._packed(self.bits[1])
        return t if t else (self.keys.numel() + self.values.numel()) * 4

    def update(self, k, v):
        self.keys, self.values = k, v
        self.updates += 1

    def clone(self):
        c = FakeEntry(self.keys.clone(), self.values.clone(), *self.bits)
        c.updates = self.updates
        return c


def _store(dllm, **kw):
    cfg = dllm.DiffusionConfig(**kw)
    return dllm.KVCacheStore(cfg, entry_factory=FakeEntry, device="cpu")


def _kv(n):
    import torch
    return torch.zeros(1, n, 1), torch.zeros(1, n, 1)


def test_store_insert_update_accounting(dllm):
    s = _store(dllm, kv_quant_bits=4)
    s.update_kv_cache("a", *_kv(1000))
    # new entry: its packed size, both phases at kv_quant_bits (lib.rs:1028-1040)
    assert s.kv_cache_memory_usage() == 2 * 2 * 500
    # update: + (keys.len()*8).saturating_sub(old packed size) (lib.rs:1013-1024)
    s.update_kv_cache("a", *_kv(1000))
    assert s.kv_cache_memory_usage() == 2000 + (8000 - 2000)
    s.update_kv_cache("a", *_kv(10))   # 80 - 2000 saturates at 0
    assert s.kv_cache_memory_usage() == 8000 and s.kv_cache["a"].updates == 2


def test_store_evicts_largest_first_and_wraps(dllm):
    s = _store(dllm, kv_quant_bits=8, max_cache_size=30_000)
    for name, n in (("small", 100), ("big", 2000), ("mid", 500)):
        s.update_kv_cache(name, *_kv(n))
    # packed sizes 400, 8000, 2000; each check prices the incoming f32 K+V (800, 16000, 4000)
    assert s.kv_cache_memory_usage() == 400 + 8000 + 2000
    # 2500 incoming elements: 10400 + 20000 > 30000 -> free 400 bytes, the largest entry first
    s.update_kv_cache("new", *_kv(2500))
    assert "big" not in s and {"small", "mid", "new"} == set(s.kv_cache)
    assert s.kv_cache_memory_usage() == 10400 - 8000 + 4 * 2500
    # the check can evict everything: a 10 KB store, then a 16 KB incoming price
    t = _store(dllm, kv_quant_bits=8, max_cache_size=10_000)
    t.update_kv_cache("small", *_kv(100))
    t.update_kv_cache("big", *_kv(2000))
    assert set(t.kv_cache) == {"big"} and t.kv_cache_memory_usage() == 8000
    # fetch_sub wraps: drive the counter below the freed bytes
    s.cache_memory_usage = 10
    s.evict_oldest_entries(1)
    assert "new" not in s and s.kv_cache_memory_usage() == (10 - 10000) % (1 << 64)
    s.clear_kv_cache()
    assert s.kv_cache_memory_usage() == 0 and len(s) == 0


def test_store_get_or_init_clone_and_phase_bits(dllm):
    s = _store(dllm, num_layers=3, hidden_size=64, num_attention_heads=4, prefill_bits=8, decode_bits=4)
    e = s.get_or_init_cache("x", 1)
    assert tuple(e.keys.shape) == (3, 0, 64) and e.bits == (8, 4)
    assert s.kv_cache_memory_usage() == 0          # get_or_init does not account (lib.rs:983-991)
    assert s.kv_cache["x"] is not e                # a clone
    s2 = _store(dllm, use_phase_aware_quant=False, kv_quant_bits=2)
    assert s2.get_or_init_cache("y", 1).bits == (2, 2)
    s3 = _store(dllm, use_kv_cache=False)
    s3.update_kv_cache("z", *_kv(10))
    assert len(s3) == 0
