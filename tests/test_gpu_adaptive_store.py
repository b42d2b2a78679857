"""GPU parity of the AdaptiveQuantizer kernels against the C oracle, and
the KV-cache registry with device entries (8f rank 2; lib.rs:958-1084) inside the denoise loop."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return ((bits(a) == bits(b)) | (np.isnan(a) & np.isnan(b))).all()


@pytest.mark.parametrize("nbits,packed", [(1, 1), (2, 1), (4, 1), (8, 1), (4, 0), (8, 0), (0, 0), (12, 0), (16, 0),
                                          (25, 0), (31, 0)])
def test_adaptive_stream_bit_exact(dllm, cuda, orc, nbits, packed):
    import torch
    rng = np.random.default_rng(nbits * 2 + packed)
    chunks = [rng.standard_normal(n).astype(np.float32) * s for n, s in ((4099, 3.0), (1, 50.0), (1 << 20, 1.0), (77, 0.1))]
    chunks[3][5] = np.nan
    q, ref = dllm.AdaptiveQuantizer(nbits, 4.0), orc.AdaptiveQuantizer(nbits, 4.0)
    for c in chunks:
        t = torch.from_numpy(c).cuda()
        q.update_stats(t[1:] if c.size > 1 else t)   # unaligned device pointer for the larger chunks
        ref.update_stats(c[1:] if c.size > 1 else c)
    s, z = q.compute_params()
    rs, rz = ref.compute_params()
    assert same([s, z], [rs, rz])
    x = np.concatenate(chunks[:2] + [np.array([-1e30, 1e30, 0.0, -0.0], np.float32)])
    codes, params = q.quantize(torch.from_numpy(x).cuda(), packed=bool(packed))
    rc, _, _ = ref.quantize(x)
    got = codes.cpu().numpy()
    if packed:
        got = orc.unpack_bits(got, x.size, nbits)
    assert np.array_equal(got, rc)
    assert same(params.cpu().numpy(), [rs, rz])


def test_adaptive_reference_test_and_defaults(dllm, cuda, orc):
    """quantization.rs:267-277 on the device; an empty summary's unwrap_or defaults."""
    import torch
    q = dllm.AdaptiveQuantizer(4, 4.0)
    assert same(q.compute_params(), orc.AdaptiveQuantizer(4).compute_params())
    q.update_stats(torch.arange(1000, dtype=torch.float32) / 1000.0)
    s, z = q.compute_params()
    assert s > 0 and z >= 0
    ref = orc.AdaptiveQuantizer(4)
    ref.update_stats(np.arange(1000, dtype=np.float32) / np.float32(1000.0))
    assert same([s, z], ref.compute_params())


def test_store_with_device_entries(dllm, cuda, orc):
    import torch
    cfg = dllm.DiffusionConfig(kv_quant_bits=4, max_cache_size=200_000)
    store = dllm.KVCacheStore(cfg)
    g = torch.Generator(device="cuda").manual_seed(1)
    K = torch.randn(1, 64, 256, device="cuda", generator=g)
    store.update_kv_cache("a", K, K * 2)
    e = store.kv_cache["a"]
    q, s, z = orc.quantize_tensor(K.cpu().numpy(), 4)
    assert np.array_equal(bits(e.get_keys().cpu().numpy().ravel()), bits(orc.dequantize_tensor(q, s, z)))
    assert store.kv_cache_memory_usage() == e.memory_usage() == 4 * ((K.numel() * 4 + 7) // 8)
    # entries of 32768 packed bytes, each update priced at 131072: the fourth evicts the first
    for name in "bcd":
        store.update_kv_cache(name, K + 1, K)
    assert set(store.kv_cache) == {"b", "c", "d"} and store.kv_cache_memory_usage() == 3 * 32768


def test_denoise_loop_saves_to_store(dllm, cuda, orc):
    """lib.rs:864-872 / 936-943: the loop runs on a clone of the stored entry and saves its final
    dequantized K/V back; the stored entry then holds 4-bit codes of those values."""
    import torch
    d, M = 256, 64
    g = torch.Generator(device="cuda").manual_seed(2)
    layers = [dllm.QuantLinear.from_weight(0.04 * torch.randn(d, d, device="cuda", generator=g), None, 4, 128)]
    cfg = dllm.DiffusionConfig(num_timesteps=4, beta_start=0.01, beta_end=0.2, num_layers=2, hidden_size=256,
                               num_attention_heads=4)
    store = dllm.KVCacheStore(cfg)
    K = torch.randn(2, 16, 256, device="cuda", generator=g)
    store.update_kv_cache("s", K, K * 3)
    before = store.kv_cache["s"].get_keys().clone()
    x0 = torch.randn(M, d, device="cuda", generator=g)
    loop = dllm.DenoiseLoop(layers, cfg, cumprod=dllm.Cumprod.INCLUSIVE, seed=3)
    out = loop.sample(x0.clone(), 4, store=store, cache_id="s")
    ref = dllm.DenoiseLoop(layers, cfg, cumprod=dllm.Cumprod.INCLUSIVE, seed=3).sample(x0.clone(), 4)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)                 # the simple model ignores K/V (lib.rs:815-824)
    # saved back: the stored entry re-quantizes the loop's final dequantized keys (4 bits both phases)
    q, s, z = orc.quantize_tensor(K.cpu().numpy(), 4)
    once = orc.dequantize_tensor(q, s, z)
    q2, s2, z2 = orc.quantize_tensor(once, 4)
    after = store.kv_cache["s"].get_keys().cpu().numpy().ravel()
    assert np.array_equal(bits(after), bits(orc.dequantize_tensor(q2, s2, z2)))
    assert np.array_equal(bits(before.cpu().numpy().ravel()), bits(once))
    # a new id starts from the empty [layers, 0, hidden] entry
    loop.sample(x0.clone(), 2, store=store, cache_id="fresh")
    assert tuple(store.kv_cache["fresh"].keys.shape) == (2, 0, 256)
