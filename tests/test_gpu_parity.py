"""GPU parity: every HIP kernel through the C-ABI vs the oracle / golden vectors.

Bar: bit-exact for codes, packed bytes and the f32 outputs of a1/a2/a4/a8/a10; the GEMM within
``REL_TOL`` relative Frobenius error of the f32 CPU restatement (north_star: 1e-3).
"""
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).resolve().parent / "golden" / "golden_v1.npz"
REL_TOL = 1e-3  # north_star: "outputs within 1e-3 rel-err of the CPU reference"
EXACT_TOL = 2e-5   # exact-weight path vs f32 on the same f16 X (summation order only)


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def torch(cuda):
    import torch as t
    return t


def dev(torch, a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return t if dtype is None else t.to(dtype)


def host(t):
    return t.detach().cpu().numpy()


def same_bits(a, b):
    return np.ascontiguousarray(a).view(np.uint8).tobytes() == np.ascontiguousarray(b).view(np.uint8).tobytes()


def rel_err(y, ref):
    ref = np.asarray(ref, np.float64)
    return float(np.linalg.norm(np.asarray(y, np.float64) - ref) / np.linalg.norm(ref))


# ---- a1 / a2 / a6 ------------------------------------------------------------------------------

def test_quantize_tensor_golden(dllm, torch, gold):
    names = sorted({k.split("/")[1] for k in gold if k.startswith("a1/")})
    for name in names:
        x = gold[f"a1/{name}/x"]
        for bits in range(1, 9):
            for packed in (False, True):
                q, params = dllm.quantize_tensor(dev(torch, x), bits, packed=packed)
                exp = gold[f"a1/{name}/b{bits}/packed" if packed else f"a1/{name}/b{bits}/q"]
                assert np.array_equal(host(q), exp), (name, bits, packed)
                assert same_bits(host(params), gold[f"a1/{name}/b{bits}/params"]), (name, bits)
                y = dllm.dequantize_tensor(q, params, bits=bits, packed=packed, n=x.size)
                assert same_bits(host(y), gold[f"a1/{name}/b{bits}/deq"]), (name, bits, packed)


def test_quantize_tensor_random_sizes(dllm, torch, orc):
    """Ragged sizes (odd tails, every octet remainder) and unaligned base pointers."""
    rng = np.random.default_rng(7)
    for n in [1, 7, 8, 9, 63, 64, 65, 1000, 4097, 100_003, 1 << 20]:
        x = (rng.standard_normal(n + 3) * rng.uniform(0.1, 10)).astype(np.float32)
        xd = dev(torch, x)
        for off in (0, 1, 3):
            xs = x[off:off + n]
            for bits in (1, 2, 3, 4, 5, 8):
                q, params = dllm.quantize_tensor(xd[off:off + n], bits, packed=True)
                rq, rs, rz = orc.quantize_tensor(xs, bits)
                assert np.array_equal(host(q), orc.pack_bits(rq, bits)), (n, off, bits)
                assert same_bits(host(params), np.array([rs, rz], np.float32))
                for dt in (torch.float32, torch.float16):
                    y = dllm.dequantize_tensor(q, params, bits=bits, packed=True, n=n, out_dtype=dt)
                    ref = orc.dequantize_tensor(rq, rs, rz)
                    if dt == torch.float32:
                        assert same_bits(host(y), ref)
                    else:
                        assert same_bits(host(y), ref.astype(np.float16))


@pytest.mark.parametrize("n", [1, 7, 8, 1000, 65537, 1 << 21])
def test_quantize_tensor_pair_matches_two_calls(dllm, torch, orc, n):
    """dllm_quantize_tensor_pair (one min/max pass, one read, two widths) == two quantize_tensor
    calls bit for bit (codes, packed bytes and params), at ragged n and an unaligned base."""
    rng = np.random.default_rng(n)
    x = (rng.standard_normal(n + 1) * 3 + 0.5).astype(np.float32)
    xd = dev(torch, x)[1:]                       # 4-byte but not 16-byte aligned base
    for packed in (True, False):
        for ba, bb in ((8, 4), (4, 2), (3, 5), (1, 8)):
            (ca, pa), (cb, pb) = dllm.quantize_tensor_pair(xd, ba, bb, packed=packed)
            ra, qa = dllm.quantize_tensor(xd, ba, packed=packed)
            rb, qb = dllm.quantize_tensor(xd, bb, packed=packed)
            assert torch.equal(ca, ra) and torch.equal(cb, rb), (n, packed, ba, bb)
            assert same_bits(host(pa), host(qa)) and same_bits(host(pb), host(qb)), (n, packed, ba, bb)
    q, s, z = orc.quantize_tensor(x[1:], 4)
    (c4, p4), _ = dllm.quantize_tensor_pair(xd, 4, 2, packed=True)
    assert np.array_equal(host(c4), orc.pack_bits(q, 4))
    assert same_bits(host(p4), np.array([s, z], np.float32))


def _scaled_tensors(rng):
    """Inputs whose per-tensor scale falls on either side of the fused kernel's exact-division
    guard [2^-64, 2^64] (inside it the corrected reciprocal product runs, outside the IEEE division),
    plus quotients on rounding ties, inf/NaN elements and an all-positive tensor."""
    base = rng.standard_normal(4099).astype(np.float32)
    out = {}
    for e in (-90, -66, -64, -63, -10, 0, 10, 62, 63, 64, 66, 90):
        out[f"range2^{e}"] = (base * np.float32(2.0 ** e)).astype(np.float32)
    ties = np.arange(31, dtype=np.float32) * np.float32(2.0 ** -4)   # 4-bit: s = 1/8, x/s = k/2
    out["ties"] = np.tile(ties, 37)
    special = base.copy()
    special[[5, 77, 1000]] = [np.inf, -np.inf, np.nan]
    out["inf_nan"] = special
    out["positive"] = (np.abs(base) + np.float32(1000.0)).astype(np.float32)
    return out


def test_quantize_fused_path_scale_guard(dllm, torch, orc):
    """The fused quantize kernel (params folded into the prologue, Markstein division) is the
    default for packed 1/2/4/8-bit codes from a 16-B aligned x; it must give the oracle's codes and
    params bit for bit on both sides of its division guard, alone and as a pair of widths, and the
    same bytes as the generic two-kernel path (which runs for the same data at a base that is not
    16-byte aligned)."""
    rng = np.random.default_rng(2024)
    for name, x in _scaled_tensors(rng).items():
        xd = dev(torch, x)
        assert xd.data_ptr() % 16 == 0
        for bits in (1, 2, 4, 8):
            q, params = dllm.quantize_tensor(xd, bits, packed=True)
            rq, rs, rz = orc.quantize_tensor(x, bits)
            assert np.array_equal(host(q), orc.pack_bits(rq, bits)), (name, bits)
            assert same_bits(host(params), np.array([rs, rz], np.float32)), (name, bits)
        for ba, bb in ((4, 2), (8, 4), (2, 1)):
            (ca, pa), (cb, pb) = dllm.quantize_tensor_pair(xd, ba, bb, packed=True)
            for c, pr, b in ((ca, pa, ba), (cb, pb, bb)):
                rq, rs, rz = orc.quantize_tensor(x, b)
                assert np.array_equal(host(c), orc.pack_bits(rq, b)), (name, ba, bb, b)
                assert same_bits(host(pr), np.array([rs, rz], np.float32)), (name, ba, bb, b)
            xu = dev(torch, np.concatenate([np.zeros(1, np.float32), x]))[1:]   # 4-B aligned: generic path
            assert xu.data_ptr() % 16 != 0
            (ga, _), (gb, _) = dllm.quantize_tensor_pair(xu, ba, bb, packed=True)
            assert torch.equal(ga, ca) and torch.equal(gb, cb), (name, ba, bb)


def test_dequantize_scalar_signature(dllm, torch, orc):
    rng = np.random.default_rng(1)
    q = rng.integers(0, 16, 777).astype(np.uint8)
    y = dllm.dequantize_tensor(dev(torch, q), 0.123, 7.0)
    assert same_bits(host(y), orc.dequantize_tensor(q, np.float32(0.123), np.float32(7.0)))


def test_pack_unpack_golden(dllm, torch, gold):
    for bits in range(1, 9):
        c = gold[f"a6/b{bits}/codes"]
        p = dllm.pack(dev(torch, c), bits)
        assert np.array_equal(host(p), gold[f"a6/b{bits}/packed"])
        assert np.array_equal(host(dllm.unpack(p, c.size, bits)), c)


def test_quantized_kv_cache_entry(dllm, torch, orc):
    """quantization.rs:128-176 on a [layers, seq, hidden] cache: per-tensor K and V params."""
    rng = np.random.default_rng(11)
    K = rng.standard_normal((2, 96, 256)).astype(np.float32)
    V = (rng.standard_normal((2, 96, 256)) * 3 + 1).astype(np.float32)
    e = dllm.QuantizedKVCacheEntry.new(dev(torch, K), dev(torch, V), 4)
    assert e.seq_len == 96
    for t, ref in ((e.dequantize_keys(), K), (e.dequantize_values(), V)):
        rq, rs, rz = orc.quantize_tensor(ref, 4)
        assert same_bits(host(t).ravel(), orc.dequantize_tensor(rq, rs, rz))
    assert e.keys.compression_ratio() == pytest.approx(8.0)
    assert e.memory_usage() == 2 * ((K.size * 4 + 7) // 8)


# ---- a4 -----------------------------------------------------------------------------------------

def test_default_quantizer_golden(dllm, torch, gold):
    x = dev(torch, gold["a4/x"])
    for qt in range(4):
        for tag, (s, z) in {"p0": (1.0, 0), "p1": (0.37, 3)}.items():
            qz = dllm.DefaultQuantizer(8, True, None, scale=s, zero_point=z)
            t = qz.quantize(x, dllm.QuantizationType(qt))
            assert np.array_equal(host(t.data), gold[f"a4/qt{qt}/{tag}/q"].ravel()), (qt, tag)
            assert same_bits(host(qz.dequantize(t)).ravel(), gold[f"a4/qt{qt}/{tag}/deq"])
            assert tuple(t.shape) == (64, 64)


def test_quant_utils_int8_1024sq(dllm, torch, orc):
    """Config 1: int8 symmetric quantize -> dequantize round trip on 1024x1024 N(0,1) (bit-exact)."""
    x = np.random.default_rng(0).standard_normal((1024, 1024)).astype(np.float32)
    t = dllm.quant_utils.quantize(dev(torch, x), dllm.QuantizationType.Int8, True, None)
    y = dllm.quant_utils.dequantize(t)
    q = orc.default_quantize(x, 0, 1.0, 0)
    assert np.array_equal(host(t.data), q)
    assert same_bits(host(y).ravel(), orc.default_dequantize(q, 1.0, 0))


# ---- a8 -----------------------------------------------------------------------------------------

def test_bit_quantizer_golden(dllm, torch, gold):
    x = dev(torch, gold["a8/x"])
    for bits in (2, 4, 8, 16):
        for tag in ("pref", "aff"):
            s, z = gold[f"a8/b{bits}/{tag}/params"]
            bq = dllm.BitQuantizer(float(s), float(z))
            q = bq.quantize(x, bits)
            assert np.array_equal(host(q), gold[f"a8/b{bits}/{tag}/q"]), (bits, tag)
            assert same_bits(host(bq.dequantize(q, bits)), gold[f"a8/b{bits}/{tag}/deq"])


def test_compress_vectors_golden(dllm, torch, gold):
    for bits in (2, 4, 8, 16):
        q, s, z = dllm.compress_vectors(dev(torch, gold[f"a8iii/b{bits}/x"]), bits)
        assert np.array_equal(host(q), gold[f"a8iii/b{bits}/q"])
        assert same_bits(host(s), gold[f"a8iii/b{bits}/scale"]) and same_bits(host(z), gold[f"a8iii/b{bits}/zp"])
        y = dllm.decompress_vectors(q, s, z)
        exp = np.stack([np.asarray((gold[f"a8iii/b{bits}/q"][i].astype(np.float32) * gold[f"a8iii/b{bits}/scale"][i])
                                   .astype(np.float32) + gold[f"a8iii/b{bits}/zp"][i], np.float32)
                        for i in range(q.shape[0])])
        assert same_bits(host(y), exp)


def test_prefill_kvquant_quantize_vectors(dllm, torch, gold, orc):
    pk = dllm.PrefillKVQuant(dllm.SystemConfig())
    q, w = pk.quantize_vectors_batched(dev(torch, gold["qv/x"]), [2, 4])
    assert np.array_equal(host(q), gold["qv/q"]) and np.array_equal(w, gold["qv/widths"])
    # long cycle (> 64 slots) and many rows
    rng = np.random.default_rng(5)
    x = rng.uniform(-0.5, 1.5, (300, 40)).astype(np.float32)
    req = rng.choice([0, 1, 2, 3, 4, 5, 6, 7], 70).astype(np.uint8)
    q, w = pk.quantize_vectors_batched(dev(torch, x), req)
    rq, rw = orc.quantize_vectors(x, [4, 6, 8, 16], req)
    assert np.array_equal(host(q), rq) and np.array_equal(w, rw)
    with pytest.raises(dllm.InvalidParams):
        pk.quantize_vectors_batched(dev(torch, x), [8])


# ---- a10 ----------------------------------------------------------------------------------------

def test_calibration_golden(dllm, torch, gold):
    cal = dllm.CalibrationData.new(64, False)
    for i in range(3):
        cal.update(dev(torch, gold[f"a10/rand/x{i}"]))
    assert same_bits(np.array([cal.min, cal.max], np.float32), gold["a10/rand/minmax"])
    assert np.array_equal(host(cal.histogram), gold["a10/rand/hist"])
    for bits in (4, 8):
        for sym in (0, 1):
            p = cal.compute_params(bits, bool(sym))
            exp = gold[f"a10/rand/params_b{bits}_s{sym}"]
            assert np.float32(p.scale) == exp[0] and p.zero_point == int(exp[1])
    ref = dllm.CalibrationData.new(10, False)
    ref.update(dev(torch, np.array([[1, 2, 3], [4, 5, 6]], np.float32)))
    assert np.array_equal(host(ref.histogram), gold["a10/ref/hist"])
    with pytest.raises(dllm.CalibrationRequired):
        dllm.CalibrationData.new(4, False).compute_params(8, False)


# ---- a5: group-quantized linear -----------------------------------------------------------------

def _linear_case(dllm, torch, orc, M, K, N, bits, ydt, seed=0, bias=True, precision=0):
    rng = np.random.default_rng(seed)
    W = (0.02 * rng.standard_normal((K, N))).astype(np.float32)
    X = rng.standard_normal((M, K)).astype(np.float32)
    b = (0.1 * rng.standard_normal(N)).astype(np.float32) if bias else None
    lin = dllm.QuantLinear.from_weight(dev(torch, W), None if b is None else dev(torch, b), bits, 128, precision)
    codes, scales, zps = orc.quantize_weights(W, bits, 128)
    pc, ps, pz = lin.export()
    assert np.array_equal(host(pc), orc.pack_bits(codes.ravel(), bits)), "weight codes differ"
    assert same_bits(host(ps), scales) and np.array_equal(host(pz), zps), "weight scales/zps differ"
    Y = lin(dev(torch, X).half(), out_dtype=ydt)
    Yr = orc.linear_forward(X, orc.dequantize_weights(codes, scales, zps, 128), b, nthreads=8)
    return host(Y.float()), Yr, lin, X


@pytest.mark.parametrize("M,K,N", [(16, 256, 96), (64, 512, 256), (256, 1024, 512), (300, 640, 200),
                                   (1, 128, 128), (513, 256, 384), (40, 576, 200), (17, 4096, 1024),
                                   (64, 4096, 4096), (65, 512, 128), (8, 256, 130)])
@pytest.mark.parametrize("precision", [0, 1])   # DLLM_PRECISION_EXACT, DLLM_PRECISION_F16W
def test_linear_int4_shapes(dllm, torch, orc, M, K, N, precision):
    for ydt in (torch.float32, torch.float16):
        Y, Yr, _, _ = _linear_case(dllm, torch, orc, M, K, N, 4, ydt, precision=precision)
        assert rel_err(Y, Yr) <= REL_TOL, (M, K, N, ydt, rel_err(Y, Yr))


@pytest.mark.parametrize("bits,group,K,N,misalign", [
    (4, 128, 640, 256, False), (2, 128, 576, 200, False), (8, 64, 320, 132, False),   # register kernel
    (4, 128, 448, 96, False),                                                         # ragged last group
    (4, 192, 640, 256, False), (4, 128, 512, 130, False), (2, 128, 256, 256, True)])  # atomicOr fallback
def test_weight_quantization_bit_exact(dllm, torch, orc, bits, group, K, N, misalign):
    """a5 weight quantization (a1 per column-group, quantization.rs:38-68) on both device kernels
    (quantize_weights4_kernel: N % 4 == 0, group <= 128, 16-B aligned W; otherwise the atomicOr
    kernel) vs the oracle, bit for bit, with NaN, +-inf, +-0 and constant column-groups."""
    rng = np.random.default_rng(bits * 1000 + group + K + N)
    W = (0.02 * rng.standard_normal((K, N))).astype(np.float32)
    W[3, 5], W[7, 1], W[K - 1, N - 1] = np.nan, np.inf, -np.inf
    W[:group, 2] = 0.25                        # constant group: scale 1.0 (quantization.rs:53)
    W[:, 3] = -0.0
    W[group - 1, 4] = np.nan                   # NaN on the last row of a group
    codes, scales, zps = orc.quantize_weights(W, bits, group)
    if misalign:
        buf = torch.empty(K * N + 1, dtype=torch.float32, device="cuda")
        buf[1:].copy_(torch.from_numpy(W.ravel()).cuda())
        Wd = buf[1:].view(K, N)
        assert Wd.data_ptr() % 16 != 0
    else:
        Wd = dev(torch, W)
    lin = dllm.QuantLinear.from_weight(Wd, None, bits, group)
    pc, ps, pz = lin.export()
    assert np.array_equal(host(pc), orc.pack_bits(codes.ravel(), bits)), "weight codes differ"
    assert same_bits(host(ps), scales), "weight scales differ"
    assert np.array_equal(host(pz), zps), "weight zero points differ"
    lin.close()


@pytest.mark.parametrize("bits", [2, 8])
@pytest.mark.parametrize("precision", [0, 1])
def test_linear_other_widths(dllm, torch, orc, bits, precision):
    Y, Yr, _, _ = _linear_case(dllm, torch, orc, 128, 512, 256, bits, torch.float32, seed=bits, precision=precision)
    assert rel_err(Y, Yr) <= REL_TOL, rel_err(Y, Yr)


def test_linear_exact_integer_layout(dllm, torch, orc):
    """Asymmetric exact-integer data: catches any row/col swap in the MFMA fragment maps.
    W columns use 16 distinct levels exactly (scale 1, zp 0 per group), X small integers, so
    the f16 GEMM is exact and must equal the f64 product bit for bit."""
    K, N, M = 256, 128, 64
    rng = np.random.default_rng(9)
    W = rng.integers(0, 16, (K, N)).astype(np.float32)
    W[0, :], W[1, :] = 0.0, 15.0  # pin min/max of group 0 -> scale 1, zp 0
    W[128, :], W[129, :] = 0.0, 15.0
    X = rng.integers(-3, 4, (M, K)).astype(np.float32)
    lin = dllm.QuantLinear.from_weight(dev(torch, W), None, 4, 128)
    Y = host(lin(dev(torch, X).half(), out_dtype=torch.float32))
    assert np.array_equal(Y, (X.astype(np.float64) @ W.astype(np.float64)).astype(np.float32))


def test_linear_from_quantized_roundtrip(dllm, torch, orc):
    rng = np.random.default_rng(4)
    K, N = 512, 256
    W = (0.02 * rng.standard_normal((K, N))).astype(np.float32)
    codes, scales, zps = orc.quantize_weights(W, 4, 128)
    lin = dllm.QuantLinear.from_quantized(dev(torch, orc.pack_bits(codes.ravel(), 4)), dev(torch, scales),
                                          dev(torch, zps), K, N, 4, 128)
    X = rng.standard_normal((32, K)).astype(np.float32)
    Y = host(lin(dev(torch, X), out_dtype=torch.float32))  # f32 X path (cast kernel)
    Yr = orc.linear_forward(X, orc.dequantize_weights(codes, scales, zps, 128))
    assert rel_err(Y, Yr) <= REL_TOL
    lin2 = dllm.QuantLinear.from_weight(dev(torch, W), None, 4, 128)
    Y2 = host(lin2(dev(torch, X), out_dtype=torch.float32))
    assert np.array_equal(Y, Y2), "import path and quantize path disagree"


def test_linear_full_size_vs_torch_fp32(dllm, torch, orc):
    """Config 2 / metric shape (M=4096, K=N=4096): the f32 reference product of the oracle's
    dequantized weights, computed by torch fp32 on the GPU (no TF32 on gfx950)."""
    M = K = N = 4096
    g = torch.Generator(device="cuda").manual_seed(2)
    W = 0.02 * torch.randn(K, N, device="cuda", generator=g)
    X = torch.randn(M, K, device="cuda", generator=g).half()
    lin = dllm.QuantLinear.from_weight(W, None, 4, 128)
    Y = lin(X, out_dtype=torch.float16).float()
    codes, scales, zps = orc.quantize_weights(host(W), 4, 128)
    pc, ps, pz = lin.export()
    assert np.array_equal(host(pc), orc.pack_bits(codes.ravel(), 4)) and same_bits(host(ps), scales)
    Wh = dev(torch, orc.dequantize_weights(codes, scales, zps, 128))
    Yr = X.float() @ Wh
    rel = (torch.linalg.norm(Y - Yr) / torch.linalg.norm(Yr)).item()
    assert rel <= REL_TOL, rel
    # exact weights: against the f32 product of the f16-rounded X, only f32 summation order remains
    Y32 = lin(X, out_dtype=torch.float32)
    rel = (torch.linalg.norm(Y32 - Yr) / torch.linalg.norm(Yr)).item()
    assert rel <= EXACT_TOL, ("exact", rel)
    lin16 = dllm.QuantLinear.from_weight(W, None, 4, 128, dllm.linear.F16W)
    Y16 = lin16(X, out_dtype=torch.float16).float()
    rel = (torch.linalg.norm(Y16 - Yr) / torch.linalg.norm(Yr)).item()
    assert rel <= REL_TOL, ("f16 weights", rel)
    lin16.close()


@pytest.mark.parametrize("M", [65, 256, 512, 1024, 1500, 2048])
def test_linear_mid_m_paths_vs_torch_fp32(dllm, torch, orc, M):
    """Mid-M dispatch at K=N=4096: 128-row tiles with K split into 8 slices (M = 65, slab partials +
    ordered combine), 32 x 128 tiles with four k-groups (256), 64 x 128 tiles with two k-groups
    (512), 128-row tiles (1024, 1500), and the 128 x 256 tile (2048), each
    within tolerance of the f32 product of the exported weights, for f16 and f32 outputs with
    bias; the other schedules (variants 3, 5, 6) agree too."""
    K = N = 4096
    g = torch.Generator(device="cuda").manual_seed(M)
    W = 0.02 * torch.randn(K, N, device="cuda", generator=g)
    b = 0.1 * torch.randn(N, device="cuda", generator=g)
    X = torch.randn(M, K, device="cuda", generator=g).half()
    lin = dllm.QuantLinear.from_weight(W, b, 4, 128)
    codes, scales, zps = lin.export()
    Wh = dev(torch, orc.dequantize_weights(orc.unpack_bits(host(codes), K * N, 4).reshape(K, N), host(scales),
                                           host(zps), 128))
    Yr = X.float() @ Wh + b
    for ydt in (torch.float16, torch.float32):
        Y = lin(X, out_dtype=ydt).float()
        rel = (torch.linalg.norm(Y - Yr) / torch.linalg.norm(Yr)).item()
        assert rel <= REL_TOL, (M, ydt, rel)
        if ydt == torch.float32:
            assert rel <= EXACT_TOL, (M, "exact weights", rel)
    lin16 = dllm.QuantLinear.from_quantized(codes, scales, zps, K, N, 4, 128, b, dllm.linear.F16W)
    Yv = lin16(X, out_dtype=torch.float32)
    rel = (torch.linalg.norm(Yv - Yr) / torch.linalg.norm(Yr)).item()
    assert rel <= REL_TOL, (M, "f16 weights", rel)
    lin16.close()
    lin.close()


@pytest.mark.parametrize("M,K,N", [(256, 4096, 4096), (384, 4096, 4096), (240, 1024, 4096), (300, 768, 4096)])
def test_linear_mid_m_kgroups_exact_integers(dllm, torch, orc, M, K, N):
    """The mid-M 32 x 128 tiles on exact-integer data: four k-groups (M 256 / 240: one block per CU),
    two (M 384 / 300; K = 768 has 6 groups), k-groups 1.. handing their sums to k-group 0 through
    the ring.  Every partial sum is an exact integer below 2^24, so the result equals the f64
    product bit for bit."""
    rng = np.random.default_rng(M + K)
    W = rng.integers(0, 16, (K, N)).astype(np.float32)
    for g0 in range(0, K, 128):
        W[g0, :], W[g0 + 1, :] = 0.0, 15.0
    X = rng.integers(-2, 3, (M, K)).astype(np.float32)
    lin = dllm.QuantLinear.from_weight(dev(torch, W), None, 4, 128)
    Y = host(lin(dev(torch, X).half(), out_dtype=torch.float32))
    assert np.array_equal(Y, (X.astype(np.float64) @ W.astype(np.float64)).astype(np.float32))
    Yh = host(lin(dev(torch, X).half(), out_dtype=torch.float16).float())
    assert np.array_equal(Yh, Y.astype(np.float16).astype(np.float32))
    lin.close()


def test_linear_split_k_exact_integers(dllm, torch, orc):
    """Exact-integer data through the split-K path (M=256, K=1024, N=512 -> 4 slices): every
    partial and the combine are exact, so the result equals the f64 product bit for bit."""
    K, N, M = 1024, 512, 256
    rng = np.random.default_rng(21)
    W = rng.integers(0, 16, (K, N)).astype(np.float32)
    for g0 in range(0, K, 128):
        W[g0, :], W[g0 + 1, :] = 0.0, 15.0
    X = rng.integers(-2, 3, (M, K)).astype(np.float32)
    lin = dllm.QuantLinear.from_weight(dev(torch, W), None, 4, 128)
    Y = host(lin(dev(torch, X).half(), out_dtype=torch.float32))
    assert np.array_equal(Y, (X.astype(np.float64) @ W.astype(np.float64)).astype(np.float32))


@pytest.mark.parametrize("precision", [0, 1])
@pytest.mark.parametrize("bits", [2, 4, 8])
@pytest.mark.parametrize("M,N", [(4096, 4096), (2048, 4096), (1800, 4096), (4096, 1024), (4096, 512), (512, 1024),
                                 (300, 256), (64, 200), (33, 200), (17, 200), (1, 200), (4096, 4092), (2048, 4092),
                                 (128, 4096), (200, 4096)])
def test_linear_policy_exact_integers(dllm, torch, orc, precision, bits, M, N):
    """Every tile of both precision policies on exact-integer data (each group spans [0, 2^b - 1]:
    scale 1, zp 0; K = 768 = 6 groups, so every product and partial sum is an exact integer):
    exact weights -- the Horner kernel (int4, M 4096 at N 4096), the producer/consumer 128 x 256
    tiles (int4, M 2048; other widths: the 128 x 256 fold-form tiles), the KG2 Horner tiles (int4,
    M 1800), the two-k-group producer/consumer 128 x 128 tiles (int4, N 1024 at M 4096),
    128 x 128 + group-aligned split-K
    (N 1024 / 512, M 512, 300), the exact decode kernel (M <= 64, one or 4 column tiles, K split) --
    and rounded weights (256 x 256, 256 x 128 two k-groups, 128 x 128 split-K, decode), with bias,
    ragged M and a padded last column group: bit-equal to the f64 product, f32 and f16 outputs.
    N = 4092 (N % 8 == 4: every other output row starts 8-B aligned) takes the Horner grid (M 4096)
    and the 128 x 256 exact tiles (M 2048) on their 8-B row-store path, not the 16-B coalesced one."""
    K = 768
    rng = np.random.default_rng(100 * bits + M + N + precision)
    q = (1 << bits) - 1
    W = rng.integers(0, q + 1, (K, N)).astype(np.float32)
    for g0 in range(0, K, 128):
        W[g0, :], W[g0 + 1, :] = 0.0, float(q)
    X = rng.integers(-2, 3, (M, K)).astype(np.float32)
    b = rng.integers(-4, 5, N).astype(np.float32)
    lin = dllm.QuantLinear.from_weight(dev(torch, W), dev(torch, b), bits, 128, precision)
    assert lin.precision == precision and dllm._lib.load().dllm_linear_precision(lin._h) == precision
    ref = (X.astype(np.float64) @ W.astype(np.float64) + b).astype(np.float32)
    Xd = dev(torch, X).half()
    assert np.array_equal(host(lin(Xd, out_dtype=torch.float32)), ref)
    assert np.array_equal(host(lin(Xd, out_dtype=torch.float16).float()), ref.astype(np.float16).astype(np.float32))
    lin.close()


@pytest.mark.parametrize("M,N,group", [(4096, 4096, 128), (2048, 4096, 128), (2048, 4096, 64), (2048, 4096, 256),
                                       (4096, 2048, 128), (3001, 4096, 128), (4096, 1024, 128), (4096, 512, 128), (256, 4096, 128), (65, 4096, 256),
                                       (64, 4096, 128), (40, 1024, 64), (16, 4096, 128), (1, 4096, 256),
                                       (128, 4096, 128), (200, 4096, 128)])
def test_linear_exact_weights_tight(dllm, torch, orc, M, N, group):
    """DLLM_PRECISION_EXACT: the MFMA consumes the exact integer (q - zp) and the f32 scale is
    applied per group, so against the f32 product of the same f16-rounded X with the reference's
    f32 a2 weights (quantization.rs:81-85) only f32 summation order differs: relative Frobenius
    error <= EXACT_TOL (measured ~1e-6), where rounding the weight to f16 alone costs ~2.5e-4."""
    K = 4096
    g = torch.Generator(device="cuda").manual_seed(M + N + group)
    W = 0.02 * torch.randn(K, N, device="cuda", generator=g)
    b = 0.1 * torch.randn(N, device="cuda", generator=g)
    X = torch.randn(M, K, device="cuda", generator=g).half()
    lin = dllm.QuantLinear.from_weight(W, b, 4, group)
    codes, scales, zps = lin.export()
    Wh = dev(torch, orc.dequantize_weights(orc.unpack_bits(host(codes), K * N, 4).reshape(K, N), host(scales),
                                           host(zps), group))
    Yr = X.float() @ Wh + b
    Y = lin(X, out_dtype=torch.float32)
    rel = (torch.linalg.norm(Y - Yr) / torch.linalg.norm(Yr)).item()
    assert rel <= EXACT_TOL, (M, N, group, rel)
    lin.close()


@pytest.mark.parametrize("spread,M,K", [(8, 4096, 4096), (8, 8000, 1024), (8, 4300, 1024), (30, 4096, 2048), (45, 4096, 1024),
                                         (8, 1800, 4096), (30, 1850, 2048), (45, 1800, 1024),
                                         (8, 2048, 4096), (30, 3000, 2048), (45, 2048, 1024),
                                         (8, 1024, 4096), (30, 1000, 2048), (45, 1024, 1024),
                                         (8, 448, 4096), (30, 400, 2048), (8, 700, 4096)])
def test_linear_horner_scale_spread(dllm, torch, orc, spread, M, K):
    """The 256 x 256-tile exact kernel (int4 g128, >= 256 tiles) keeps one accumulator in Horner form:
    acc <- acc * (s_{g-1} / s_g) + T_g, times s_{G-1} at the end; at M = 2048 / 3000 the same form
    runs on the producer/consumer 128 x 256 tiles, at M = 1024 / 1000 on the two-k-group 128 x 128
    producer/consumer tiles (one chain per K-half), at M = 448 / 400 on their 64 x 128 form; at M =
    1800 / 1850 (120 such tiles,
    240 of the fold form's 128 x 256) the 256 x 128-tile KG2 kernel runs one chain per K-half (the
    second starting from a zero accumulator) and sums the two halves' partials times their last
    scales.  Per-(group, column) weight
    magnitudes spread by 2^U(-spread, spread): every column is checked on its own against f32 on the
    same f16 X with the reference's a2 weights (quantization.rs:81-85), so a group rescaled wrongly
    shows even where other groups dominate the column.  spread 45 gives columns whose scales span
    more than 2^64: create must reject the ratios (none kept) and the handle run the fold-form
    kernel (same bound); otherwise it keeps the (G + 1) x N f32 ratios."""
    N = 4096
    g = torch.Generator(device="cuda").manual_seed(spread + M + K)
    G = K // 128
    mult = torch.exp2((torch.rand(G, N, device="cuda", generator=g) * 2 - 1) * spread)
    W = 0.02 * torch.randn(K, N, device="cuda", generator=g) * mult.repeat_interleave(128, 0)
    X = torch.randn(M, K, device="cuda", generator=g).half()
    lin = dllm.QuantLinear.from_weight(W, None, 4, 128)
    base = 2 * K * N // 2 + G * N * 8 + N * 4        # code layouts, sz + sf, bias
    assert lin.device_bytes() == base + (0 if spread == 45 else (G + 1) * N * 4), (spread, lin.device_bytes())
    codes, scales, zps = lin.export()
    Wh = dev(torch, orc.dequantize_weights(orc.unpack_bits(host(codes), K * N, 4).reshape(K, N), host(scales),
                                           host(zps), 128))
    Yr = X.double() @ Wh.double()
    for rep in range(2):   # the kernel is fixed at create: both calls run it
        Y = lin(X, out_dtype=torch.float32).double()
        assert torch.isfinite(Y).all()
        col = torch.linalg.norm(Y - Yr, dim=0) / torch.linalg.norm(Yr, dim=0)
        assert col.max().item() <= EXACT_TOL, (spread, rep, col.max().item())
    lin.close()


@pytest.mark.parametrize("spread,M,K", [(8, 4096, 4096), (30, 4096, 2048), (45, 4096, 1024), (8, 8000, 1024),
                                         (8, 4300, 1024)])
def test_linear_horner_int2_scale_spread(dllm, torch, orc, spread, M, K):
    """int2 g128 (config C3's int2 layers) on the 256 x 256-tile Horner kernel (wq_horner16_kernel
    with BITS = 2: each stage moves its k-step pair's 1-KiB piece of weight words and reads its half),
    the same per-column bound as the int4 case above against the f64 product of the same f16 X with
    the reference's a2 weights; spread 45 rejects the ratios (fold-form kernel); M = 4300 takes the
    fold form (its 256 x 256 grid needs too many rounds)."""
    N, bits = 4096, 2
    g = torch.Generator(device="cuda").manual_seed(7 * spread + M + K)
    G = K // 128
    mult = torch.exp2((torch.rand(G, N, device="cuda", generator=g) * 2 - 1) * spread)
    W = 0.02 * torch.randn(K, N, device="cuda", generator=g) * mult.repeat_interleave(128, 0)
    X = torch.randn(M, K, device="cuda", generator=g).half()
    lin = dllm.QuantLinear.from_weight(W, None, bits, 128)
    base = 2 * K * N * bits // 8 + G * N * 8 + N * 4   # code layouts (prefill, decode), sz + sf, bias
    assert lin.device_bytes() == base + (0 if spread == 45 else (G + 1) * N * 4), (spread, lin.device_bytes())
    codes, scales, zps = lin.export()
    Wh = dev(torch, orc.dequantize_weights(orc.unpack_bits(host(codes), K * N, bits).reshape(K, N), host(scales),
                                           host(zps), 128))
    Yr = X.double() @ Wh.double()
    for rep in range(2):
        Y = lin(X, out_dtype=torch.float32).double()
        assert torch.isfinite(Y).all()
        col = torch.linalg.norm(Y - Yr, dim=0) / torch.linalg.norm(Yr, dim=0)
        assert col.max().item() <= EXACT_TOL, (spread, rep, col.max().item())
    Y16 = lin(X, out_dtype=torch.float16).double()
    assert torch.equal(Y16, lin(X, out_dtype=torch.float32).half().double())
    lin.close()


@pytest.mark.parametrize("M,N,group", [(4096, 1024, 128), (4096, 512, 128), (1024, 4096, 128), (256, 4096, 256),
                                       (65, 4096, 128), (300, 1280, 64), (129, 384, 128)])
def test_linear_split_k_combine_repeatable(dllm, torch, orc, M, N, group):
    """Shapes whose exact GEMM splits K (f32 slice slabs summed in slice order by the combine
    kernel): back-to-back calls into a NaN-filled output, with the f32 and the f16 outputs, must be
    bit-identical to each other and within the exact-weights bound of the f32 product -- a stale or
    partially written slab would break the equality or the bound."""
    K = 4096 if N <= 1280 else 2048
    g = torch.Generator(device="cuda").manual_seed(M + N)
    W = 0.02 * torch.randn(K, N, device="cuda", generator=g)
    b = 0.1 * torch.randn(N, device="cuda", generator=g)
    X = torch.randn(M, K, device="cuda", generator=g).half()
    lin = dllm.QuantLinear.from_weight(W, b, 4, group)
    codes, scales, zps = lin.export()
    outs = []
    for rep in range(3):
        Y = torch.full((M, N), float("nan"), device="cuda")
        lin(X, out=Y)
        outs.append(Y.clone())
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    Wh = dev(torch, orc.dequantize_weights(orc.unpack_bits(host(codes), K * N, 4).reshape(K, N),
                                           host(scales), host(zps), group))
    Yr = X.float() @ Wh + b
    rel = (torch.linalg.norm(outs[0] - Yr) / torch.linalg.norm(Yr)).item()
    assert rel <= EXACT_TOL, rel
    Y16 = torch.full((M, N), float("nan"), device="cuda", dtype=torch.float16)
    lin(X, out=Y16)
    assert torch.equal(Y16, outs[0].half())
    lin.close()


def test_linear_device_memory(dllm, torch):
    """Create builds everything a forward reads: the prefill and decode code layouts (8 MiB each at
    4096^2 int4), the per-(group, column) parameters (sz pairs + f32 scales, 1 MiB) and the Horner
    ratios (f32 [G + 1][N], 0.52 MiB) -- no canonical, scale/zp or A/B copies; forward calls on
    either path add nothing (f16 X: no X workspace) and repeat bit for bit."""
    W = 0.02 * torch.randn(4096, 4096, device="cuda")
    lin = dllm.QuantLinear.from_weight(W, None, 4, 128)
    mib = lin.device_bytes() / 2**20
    assert 17.5 <= mib <= 17.55, mib
    X = torch.randn(8, 4096, device="cuda").half()
    y = lin(X)
    Xp = torch.randn(4096, 4096, device="cuda").half()
    y4 = lin(Xp)
    assert lin.device_bytes() / 2**20 == mib
    assert torch.equal(lin(X), y) and torch.equal(lin(Xp), y4)
    lin.close()
    # a shape outside the Horner form holds no ratios
    lin = dllm.QuantLinear.from_weight(W[:, :384].contiguous(), None, 4, 128)
    assert lin.device_bytes() == 2 * 4096 * 384 // 2 + 32 * 384 * 8 + 384 * 4
    lin.close()


def test_linear_decode_first_call_in_capture(dllm, torch):
    """The decode layout is built by create, so a handle's very first M <= 64 call may be captured:
    the replay matches an eager call of a fresh handle bit for bit."""
    W = 0.02 * torch.randn(1024, 512, device="cuda")
    lin = dllm.QuantLinear.from_weight(W, None, 4, 128)
    X = torch.randn(4, 1024, device="cuda").half()
    Y = torch.empty(4, 512, device="cuda", dtype=torch.float16)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            lin(X, out=Y)
    g.replay()
    torch.cuda.synchronize()
    ref = dllm.QuantLinear.from_weight(W, None, 4, 128)
    assert torch.equal(ref(X), Y)
    lin.close()
    ref.close()


@pytest.mark.parametrize("M", [4096, 1800])
def test_linear_horner_first_call_in_capture(dllm, torch, orc, M):
    """The forward contract: a handle's first call on a Horner grid (K = N = 4096, int4 g128; M 4096:
    256 x 256 tiles, M 1800: the KG2 256 x 128 tiles) made inside stream capture runs the same
    kernel as every later eager call -- the Horner ratios were decided at create, nothing is
    allocated or synchronised by the call -- so the graph replay and two eager calls are
    bit-identical, within the exact-weights bound of f32 on the same f16 X."""
    K = N = 4096
    g = torch.Generator(device="cuda").manual_seed(4242)
    W = 0.02 * torch.randn(K, N, device="cuda", generator=g)
    X = torch.randn(M, K, device="cuda", generator=g).half()
    lin = dllm.QuantLinear.from_weight(W, None, 4, 128)
    before = lin.device_bytes()
    codes, scales, zps = lin.export()
    Wh = dev(torch, orc.dequantize_weights(orc.unpack_bits(host(codes), K * N, 4).reshape(K, N), host(scales),
                                           host(zps), 128))
    Yr = X.float() @ Wh
    Yg = torch.empty(M, N, device="cuda")
    s = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            lin(X, out=Yg)
    graph.replay()
    torch.cuda.synchronize()
    Ye = lin(X, out_dtype=torch.float32)
    Ye2 = lin(X, out_dtype=torch.float32)
    assert lin.device_bytes() == before
    assert torch.equal(Yg, Ye) and torch.equal(Ye, Ye2)
    rel = (torch.linalg.norm(Ye - Yr) / torch.linalg.norm(Yr)).item()
    assert rel <= EXACT_TOL, rel
    lin.close()


@pytest.mark.lab
@pytest.mark.parametrize("variant", [4, 8, 9, 10, 11, 14, 15])
@pytest.mark.parametrize("bits", [2, 4, 8])
def test_linear_big_tile_exact_integers(dllm, torch, orc, variant, bits):
    """256x256-tile kernels (variant 4: 32x32x16 MFMA, w-layout; variant 8: 16x16x32 MFMA, w16
    layout; 9/10: the ping-pong schedule, 1 or 2 substeps per phase; 11: ping-pong on 16x16x32) on
    exact-integer data at M = N = 4096 (K = 256, so the f16 products and f32 sums are
    exact): the result must equal the f64 product bit for bit, catching any fragment-map error."""
    K, N, M = 256, 4096, 4096
    rng = np.random.default_rng(31 + bits)
    q = (1 << bits) - 1
    W = rng.integers(0, q + 1, (K, N)).astype(np.float32)
    for g0 in range(0, K, 128):
        W[g0, :], W[g0 + 1, :] = 0.0, float(q)
    X = rng.integers(-2, 3, (M, K)).astype(np.float32)
    lin = dllm.QuantLinear.from_weight(dev(torch, W), None, bits, 128)
    lin.set_kernel_variant(variant)
    Y = host(lin(dev(torch, X).half(), out_dtype=torch.float32))
    assert np.array_equal(Y, (X.astype(np.float64) @ W.astype(np.float64)).astype(np.float32))
    lin.close()


@pytest.mark.lab
def test_linear_split_big_tile_exact_integers(dllm, torch, orc):
    """Variant 13 (A/B only: 256x256 tiles with a 2-way K split + slab reduce, profiles/r01_splitk_ab)
    at M = 2048, on exact-integer data with bias: bit-equal to the f64 product."""
    K, N, M = 512, 4096, 2048
    rng = np.random.default_rng(77)
    W = rng.integers(0, 16, (K, N)).astype(np.float32)
    for g0 in range(0, K, 128):     # every group spans [0, 15]: scale 1, zp 0, exact dequant
        W[g0, :], W[g0 + 1, :] = 0.0, 15.0
    X = rng.integers(-2, 3, (M, K)).astype(np.float32)
    b = rng.integers(-4, 5, N).astype(np.float32)
    lin = dllm.QuantLinear.from_weight(dev(torch, W), dev(torch, b), 4, 128)
    lin.set_kernel_variant(13)
    Y = host(lin(dev(torch, X).half(), out_dtype=torch.float32))
    assert np.array_equal(Y, (X.astype(np.float64) @ W.astype(np.float64) + b).astype(np.float32))
    lin.close()


def test_mixed_precision_stack(dllm, torch, orc):
    """Config 3 shape family: layers cycle bits [2, 4]; each layer within tolerance of the f32
    restatement applied to the same f16 input."""
    rng = np.random.default_rng(12)
    d, M, L = 512, 96, 4
    Ws = [(0.05 * rng.standard_normal((d, d))).astype(np.float32) for _ in range(L)]
    stack = dllm.MixedPrecisionStack([dev(torch, w) for w in Ws], bits=(2, 4))
    x = dev(torch, rng.standard_normal((M, d)).astype(np.float32)).half()
    h = x
    for i, layer in enumerate(stack.layers):
        assert layer.bits == (2, 4)[i % 2]
        y = layer(h, out_dtype=torch.float16)
        c, s, z = orc.quantize_weights(Ws[i], layer.bits, 128)
        yr = orc.linear_forward(host(h.float()), orc.dequantize_weights(c, s, z, 128))
        assert rel_err(host(y.float()), yr) <= REL_TOL, (i, rel_err(host(y.float()), yr))
        h = y
    assert torch.equal(stack(x), h)


def test_mixed_precision_stack_config3_full_size(dllm, torch, orc):
    """Config C3 at its full size: 12 layers d = 4096 cycling int2 / int4 on seq 4096.  Each
    layer's output is within REL_TOL of torch fp32 applied to the same f16 input with the weights
    the oracle dequantizes from the layer's exported codes; the stack's own forward equals the
    layer-by-layer chain bit for bit."""
    d, M, L = 4096, 4096, 12
    g = torch.Generator(device="cuda").manual_seed(3)
    stack = dllm.MixedPrecisionStack([0.02 * torch.randn(d, d, device="cuda", generator=g) for _ in range(L)],
                                     bits=(2, 4))
    x = torch.randn(M, d, device="cuda", generator=g).half()
    h = x
    for i, layer in enumerate(stack.layers):
        assert layer.bits == (2, 4)[i % 2]
        y = layer(h, out_dtype=torch.float16)
        codes, scales, zps = layer.export()
        Wh = dev(torch, orc.dequantize_weights(orc.unpack_bits(host(codes), d * d, layer.bits).reshape(d, d),
                                               host(scales), host(zps), 128))
        yr = h.float() @ Wh
        rel = (torch.linalg.norm(y.float() - yr) / torch.linalg.norm(yr)).item()
        assert rel <= REL_TOL, (i, layer.bits, rel)
        h = y
    assert torch.equal(stack(x), h)


# ---- a9: quantized-KV dequant-attention ---------------------------------------------------------

@pytest.mark.parametrize("S,H,bits", [(256, 2, 4), (200, 3, 4), (96, 1, 8), (512, 4, 4), (33, 2, 4)])
def test_kv_attention_vs_oracle(dllm, torch, orc, S, H, bits):
    """O = softmax(Q K^T/sqrt(128)) V with K, V per-tensor quantized (a1) and dequantized (a2) in
    the kernel; oracle: f64 SDPA on the oracle-dequantized K, V and the same f16-rounded Q."""
    rng = np.random.default_rng(S * 10 + H)
    D = 128
    Q = rng.standard_normal((S, H, D)).astype(np.float32).astype(np.float16)
    K = rng.standard_normal((S, H, D)).astype(np.float32)
    V = (rng.standard_normal((S, H, D)) * 2 + 0.5).astype(np.float32)
    kq = dllm.QuantizedTensor.quantize(dev(torch, K), bits, packed=True)
    vq = dllm.QuantizedTensor.quantize(dev(torch, V), bits, packed=True)
    O = host(dllm.kv_attention(dev(torch, Q), kq, vq).float())
    Kh = orc.dequantize_tensor(*orc.quantize_tensor(K, bits)).reshape(S, H, D)
    Vh = orc.dequantize_tensor(*orc.quantize_tensor(V, bits)).reshape(S, H, D)
    Oref = orc.attention(Q.astype(np.float32), Kh, Vh)
    assert rel_err(O, Oref) <= REL_TOL, rel_err(O, Oref)


def test_kv_attention_peaked_softmax(dllm, torch, orc):
    """A key that dominates one query forces the online-softmax rescale branch at a chosen block
    (rule: a rare data-dependent branch needs its own test)."""
    S, H, D = 256, 1, 128
    rng = np.random.default_rng(3)
    Q = (rng.standard_normal((S, H, D)) * 0.1).astype(np.float16)
    K = (rng.standard_normal((S, H, D)) * 0.1).astype(np.float32)
    V = rng.standard_normal((S, H, D)).astype(np.float32)
    K[200, 0, :] = 8.0 * np.sign(Q[5, 0, :].astype(np.float32))   # key 200 (7th block) spikes query 5
    kq = dllm.QuantizedTensor.quantize(dev(torch, K), 8, packed=True)
    vq = dllm.QuantizedTensor.quantize(dev(torch, V), 8, packed=True)
    O = host(dllm.kv_attention(dev(torch, Q), kq, vq).float())
    Kh = orc.dequantize_tensor(*orc.quantize_tensor(K, 8)).reshape(S, H, D)
    Vh = orc.dequantize_tensor(*orc.quantize_tensor(V, 8)).reshape(S, H, D)
    Oref = orc.attention(Q.astype(np.float32), Kh, Vh)
    assert rel_err(O, Oref) <= REL_TOL
    assert rel_err(O[5], Oref[5]) <= REL_TOL


def _tile_rows(S, tile=256, extra=(), stride=37):
    """Query rows that touch every ``tile``-query workgroup of the attention kernel: each tile's
    first and last row and one pseudo-random interior row, plus ``extra``."""
    rows = set(r for r in extra if 0 <= r < S)
    for t0 in range(0, S, tile):
        t1 = min(S, t0 + tile)
        rows.update({t0, t1 - 1, t0 + (t0 // tile * stride) % (t1 - t0)})
    return np.array(sorted(rows))


def test_kv_quantize_attention_config4_full_size(dllm, torch, orc):
    """Config C4 at its full size (K, V, Q [8192, 32, 128]): the int4 per-tensor KV quantization
    is bit-exact against the C oracle on all 33.5 M elements of each tensor (packed codes and
    params), and the dequant-attention is within REL_TOL of the oracle's f64 SDPA on the
    oracle-dequantized K and V, on query rows from EVERY 256-query tile of every head (first,
    last and one interior row of each of the 32 tiles, plus rows 0, 255, 256, 4095, 4096, 8191),
    against all 8192 keys."""
    S, H, D = 8192, 32, 128
    rng = np.random.default_rng(84)
    K = rng.standard_normal((S, H, D), dtype=np.float32)
    V = rng.standard_normal((S, H, D), dtype=np.float32)
    Q = rng.standard_normal((S, H, D), dtype=np.float32).astype(np.float16)
    e = dllm.QuantizedKVCacheEntry.new(dev(torch, K), dev(torch, V), 4)
    deq = []
    for t, ref in ((e.keys, K), (e.values, V)):
        rq, rs, rz = orc.quantize_tensor(ref.ravel(), 4)
        assert np.array_equal(host(t.data), orc.pack_bits(rq, 4))
        assert same_bits(host(t.params), np.array([rs, rz], np.float32))
        deq.append(orc.dequantize_tensor(rq, rs, rz).reshape(S, H, D))
    rows = _tile_rows(S, extra=(0, 255, 256, 4095, 4096, 8191))
    assert len(set(rows // 256)) == S // 256
    O = host(dllm.kv_attention(dev(torch, Q), e.keys, e.values).float())[rows]
    Oref = orc.attention_rows(Q.astype(np.float32)[rows], deq[0], deq[1])
    for h in range(H):
        assert rel_err(O[:, h], Oref[:, h]) <= REL_TOL, (h, rel_err(O[:, h], Oref[:, h]))
    for i in range(len(rows)):   # every sampled row of every tile, all heads
        assert rel_err(O[i], Oref[i]) <= REL_TOL, (rows[i], rel_err(O[i], Oref[i]))


@pytest.mark.parametrize("S,H,bits", [(8003, 4, 4), (4160, 3, 8), (65, 2, 4)])
def test_kv_attention_ragged_full_tiles(dllm, torch, orc, S, H, bits):
    """Ragged S: a partial last 256-query tile AND a partial last 64-key block (8003 = 31*256 + 67
    = 125*64 + 3; 4160 = 16*256 + 64 with whole key blocks; 65 = one tile, two key blocks); rows
    from every query tile, including every row of the partial last tile, vs the f64 oracle."""
    rng = np.random.default_rng(S + H)
    D = 128
    K = rng.standard_normal((S, H, D), dtype=np.float32)
    V = (rng.standard_normal((S, H, D), dtype=np.float32) * 1.5 - 0.25).astype(np.float32)
    Q = rng.standard_normal((S, H, D), dtype=np.float32).astype(np.float16)
    kq = dllm.QuantizedTensor.quantize(dev(torch, K), bits, packed=True)
    vq = dllm.QuantizedTensor.quantize(dev(torch, V), bits, packed=True)
    Kh = orc.dequantize_tensor(*orc.quantize_tensor(K.ravel(), bits)).reshape(S, H, D)
    Vh = orc.dequantize_tensor(*orc.quantize_tensor(V.ravel(), bits)).reshape(S, H, D)
    last = (S - 1) // 256 * 256
    rows = np.union1d(_tile_rows(S), np.arange(last, S))
    O = host(dllm.kv_attention(dev(torch, Q), kq, vq).float())[rows]
    Oref = orc.attention_rows(Q.astype(np.float32)[rows], Kh, Vh)
    assert np.isfinite(O).all()
    for i in range(len(rows)):
        assert rel_err(O[i], Oref[i]) <= REL_TOL, (rows[i], rel_err(O[i], Oref[i]))


@pytest.mark.lab
@pytest.mark.parametrize("S,H,bits", [(512, 2, 4), (333, 3, 8), (8192, 2, 4)])
def test_kv_attention_schedules_bit_identical(dllm, torch, orc, S, H, bits, monkeypatch):
    """The v5 (DLLM_ATTN_LAB=0) and v6 (4 waves x 64 queries: 200) schedules share the block
    order and every per-query operation, so their outputs must agree bit for bit, including a
    ragged last key block and query tile; v4 (100) sums the row in a different order (a chain,
    not a tree), so it agrees within rounding."""
    g = torch.Generator(device="cuda").manual_seed(S + H)
    K = torch.randn(S, H, 128, device="cuda", generator=g)
    V = torch.randn(S, H, 128, device="cuda", generator=g)
    Q = torch.randn(S, H, 128, device="cuda", generator=g).half()
    kq = dllm.QuantizedTensor.quantize(K, bits, packed=True)
    vq = dllm.QuantizedTensor.quantize(V, bits, packed=True)
    outs = {}
    for lab in (0, 100, 200):
        monkeypatch.setenv("DLLM_ATTN_LAB", str(lab))
        outs[lab] = dllm.kv_attention(Q, kq, vq)
    monkeypatch.delenv("DLLM_ATTN_LAB")
    assert torch.equal(outs[0], outs[200])
    d4 = (outs[0].float() - outs[100].float()).norm() / outs[100].float().norm()
    assert d4.item() <= 1e-3, d4.item()


# ---- host-slice entry points (the literal Rust signatures) ---------------------------------------

def test_host_entry_points(dllm, orc):
    import ctypes as C
    L = dllm._lib.load()
    rng = np.random.default_rng(21)
    x = (rng.standard_normal(1001) * 2).astype(np.float32)
    q = np.zeros(x.size, np.uint8)
    s, z = C.c_float(), C.c_float()
    assert L.dllm_quantize_tensor_host(x.ctypes.data, x.size, 4, q.ctypes.data, C.byref(s), C.byref(z)) == 0
    rq, rs, rz = orc.quantize_tensor(x, 4)
    assert np.array_equal(q, rq) and np.float32(s.value) == rs and np.float32(z.value) == rz
    y = np.zeros(x.size, np.float32)
    assert L.dllm_dequantize_tensor_host(q.ctypes.data, q.size, s.value, z.value, y.ctypes.data) == 0
    assert same_bits(y, orc.dequantize_tensor(rq, rs, rz))
    assert L.dllm_bit_quantize_host(x.ctypes.data, x.size, 4, 0.25, -1.0, q.ctypes.data) == 0
    assert np.array_equal(q, orc.bit_quantize(x, 4, 0.25, -1.0))
    assert L.dllm_default_quantize_host(x.ctypes.data, x.size, 0, 0.5, 3, q.ctypes.data) == 0
    assert np.array_equal(q, orc.default_quantize(x, 0, 0.5, 3))


@pytest.mark.lab
def test_gemm_variants_bit_identical(dllm, torch):
    """All prefill schedules (0..3: 256x128 tile; 4: 256x256 tile, 3-stage LDS ring, 1x8 waves;
    7: the same tile with 2x4 waves; 9/10: ping-pong wave groups) accumulate every output in the
    same k order, so they must agree bit for bit -- including a ragged M tail -- for f32 and f16
    outputs."""
    K, N, M = 1024, 4096, 4352
    g = torch.Generator(device="cuda").manual_seed(8)
    W = 0.02 * torch.randn(K, N, device="cuda", generator=g)
    X = torch.randn(M, K, device="cuda", generator=g).half()
    lin = dllm.QuantLinear.from_weight(W, 0.1 * torch.randn(N, device="cuda", generator=g), 4, 128)
    outs, outs16 = {}, {}
    for v in (0, 3, 4, 7, 9, 10):
        lin.set_kernel_variant(v)
        outs[v] = lin(X, out_dtype=torch.float32)
        outs16[v] = lin(X, out_dtype=torch.float16)
    for v in (3, 4, 7, 9, 10):
        assert torch.equal(outs[0], outs[v]), v
        assert torch.equal(outs16[0], outs16[v]), v
    # the 16x16x32 kernels sum 32-deep MFMA chunks: equal to each other, not to the 32x32x16 ones
    for v in (8, 11):
        lin.set_kernel_variant(v)
        outs[v] = lin(X, out_dtype=torch.float32)
        outs16[v] = lin(X, out_dtype=torch.float16)
    assert torch.equal(outs[8], outs[11]) and torch.equal(outs16[8], outs16[11])


@pytest.mark.parametrize("K", [128, 256, 384, 1152])
def test_linear_staggered_tiles_exact_integers(dllm, torch, K):
    """The 128 x 256 exact tiles, product policy, on exact-integer data: every partial is exact, so
    each output equals the f64 product bit for bit.  int4 g128 with valid Horner ratios runs the
    producer/consumer kernel (linear_pc.hip: 8 consumer waves, 4 producer waves issuing every DMA
    piece, consumer halves half a stage apart, one 12-wave barrier per half stage, 3-slot ring).
    M 2048 / 2100 x N 4096 take those tiles (>= 256 of them; 2100 leaves a ragged last row block);
    K 128 / 256 / 384 run fewer stages than the ring keeps in flight (1 / 2 / 3), K 1152 a ring
    period that does not divide the stage count."""
    N = 4096
    rng = np.random.default_rng(K)
    W = rng.integers(0, 16, (K, N)).astype(np.float32)
    for g0 in range(0, K, 128):
        W[g0, :], W[g0 + 1, :] = 0.0, 15.0
    b = rng.integers(-4, 5, N).astype(np.float32)
    lin = dllm.QuantLinear.from_weight(dev(torch, W), dev(torch, b), 4, 128, prefill_only=True)
    for M in (2048, 2100):
        X = rng.integers(-2, 3, (M, K)).astype(np.float32)
        ref = (X.astype(np.float64) @ W.astype(np.float64) + b).astype(np.float32)
        Xd = dev(torch, X).half()
        assert np.array_equal(host(lin(Xd, out_dtype=torch.float32)), ref), (K, M)
        Y16 = host(lin(Xd, out_dtype=torch.float16).float())
        assert np.array_equal(Y16, ref.astype(np.float16).astype(np.float32)), (K, M, "f16")
    lin.close()


@pytest.mark.parametrize("K", [256, 512, 768, 2304])
@pytest.mark.parametrize("M,N", [(4096, 1024), (2048, 2048), (1024, 4096), (1000, 4096), (4096, 1020),
                                 (512, 4096), (4096, 512), (500, 4096), (256, 4096), (300, 4096),
                                 (384, 4096), (420, 4096), (448, 4096), (576, 4096), (700, 4096)])
def test_linear_pc_kg2_tiles_exact_integers(dllm, torch, K, M, N):
    """The two-k-group producer/consumer kernel (linear_pc.hip) on exact-integer data, bit-equal to
    the f64 product for f32 and f16 outputs: K-half kg's Horner chain in k-group kg, the halves'
    partials summed through LDS (each k-group finalizes half the token blocks).  Tiles of 128 x 128
    (the 4-GPU column shard 4096 x 1024, 2048 x 2048, 1024 x 4096) and 64 x 128 (M 512 / 500 at N
    4096, the 8-GPU shard 4096 x 512, and M 384 / 420 / 448: grids of 3/4 of a round and more; M 576 /
    700 take 128-row tiles short of a round rather than 64-row tiles in more than one); M
    256 / 300 take the 4-k-group fold tiles of mid M (the 32 x 128 PC tiles are an A/B build only).
    K 256 .. 2304 = 1 .. 9 groups
    per half (a ring period of 3 stages that does not divide the 2 .. 18 k-steps of a half); M
    1000 / 500 / 300 leave a ragged last row block, N 1020 a padded last column block (the 8-B
    row-store path)."""
    rng = np.random.default_rng(K + M + N)
    W = rng.integers(0, 16, (K, N)).astype(np.float32)
    for g0 in range(0, K, 128):
        W[g0, :], W[g0 + 1, :] = 0.0, 15.0
    b = rng.integers(-4, 5, N).astype(np.float32)
    X = rng.integers(-2, 3, (M, K)).astype(np.float32)
    lin = dllm.QuantLinear.from_weight(dev(torch, W), dev(torch, b), 4, 128, prefill_only=True)
    ref = (X.astype(np.float64) @ W.astype(np.float64) + b).astype(np.float32)
    Xd = dev(torch, X).half()
    assert np.array_equal(host(lin(Xd, out_dtype=torch.float32)), ref), (K, M, N)
    assert np.array_equal(host(lin(Xd, out_dtype=torch.float16).float()), ref.astype(np.float16).astype(np.float32))
    lin.close()


@pytest.mark.parametrize("bits", [2, 4, 8])
def test_linear_decode_lds_staged_exact_integers(dllm, torch, bits):
    """The decode path for M 9..16 (linear_wq.hip, XL: the block's X rows, a zero row and its
    columns' zero-point pairs / scales staged in LDS) on exact-integer data, product policy: every
    partial is exact, so each output equals the f64 product bit for bit.  Shapes: K 1536 (12 slabs
    over 8 waves: clamped duplicate slabs read the zero row), K 6144 (two rounds of slabs), group
    256, a padded last column group (N 200 / 136), and M 8 / 17 on either side of the XL range."""
    for K, N, group, Ms in ((1024, 200, 128, (8, 9, 16, 17)), (1536, 136, 128, (12,)),
                            (6144, 64, 128, (9,)), (4096, 256, 256, (16,))):
        rng = np.random.default_rng(7 * bits + K)
        q = (1 << bits) - 1
        W = rng.integers(0, q + 1, (K, N)).astype(np.float32)
        for g0 in range(0, K, group):
            W[g0, :], W[g0 + 1, :] = 0.0, float(q)
        b = rng.integers(-4, 5, N).astype(np.float32)
        lin = dllm.QuantLinear.from_weight(dev(torch, W), dev(torch, b), bits, group)
        for M in Ms:
            X = rng.integers(-2, 3, (M, K)).astype(np.float32)
            ref = (X.astype(np.float64) @ W.astype(np.float64) + b).astype(np.float32)
            Xd = dev(torch, X).half()
            assert np.array_equal(host(lin(Xd, out_dtype=torch.float32)), ref), (bits, K, N, group, M)
            if np.abs(ref).max() < 60000:
                Y16 = host(lin(Xd, out_dtype=torch.float16).float())
                assert np.array_equal(Y16, ref.astype(np.float16).astype(np.float32)), (bits, K, M, "f16")
        lin.close()


@pytest.mark.lab
@pytest.mark.parametrize("bits", [2, 4, 8])
def test_linear_decode_tiles_exact_integers(dllm, torch, orc, bits):
    """Decode kernel (M <= 64) under every (NT column tiles, K-split) configuration on
    exact-integer data (K = 576: a half 128-deep slab at the end; N = 200: a padded last column
    group; integer bias): every partial and the ordered slab combine are exact, so each output
    equals the f64 product bit for bit, for f32 and f16 outputs, at ragged M."""
    K, N = 576, 200
    rng = np.random.default_rng(41 + bits)
    q = (1 << bits) - 1
    W = rng.integers(0, q + 1, (K, N)).astype(np.float32)
    for g0 in range(0, K, 128):
        W[g0, :], W[g0 + 1, :] = 0.0, float(q)
    b = rng.integers(-4, 5, N).astype(np.float32)
    lin = dllm.QuantLinear.from_weight(dev(torch, W), dev(torch, b), bits, 128)
    for M in (1, 5, 16, 17, 33, 64):
        X = rng.integers(-2, 3, (M, K)).astype(np.float32)
        ref = (X.astype(np.float64) @ W.astype(np.float64) + b).astype(np.float32)
        Xd = dev(torch, X).half()
        for nt_log in (0, 1, 2):
            for split_log in (0, 1, 2, 3):
                lin.set_kernel_variant(200 + 16 * nt_log + split_log)
                Y = host(lin(Xd, out_dtype=torch.float32))
                assert np.array_equal(Y, ref), (bits, M, 1 << nt_log, 1 << split_log)
                Y16 = host(lin(Xd, out_dtype=torch.float16).float())
                assert np.array_equal(Y16, ref.astype(np.float16).astype(np.float32)), (bits, M, nt_log, split_log)
        lin.set_kernel_variant(-1)
        assert np.array_equal(host(lin(Xd, out_dtype=torch.float32)), ref), (bits, M, "policy")
    lin.close()


@pytest.mark.parametrize("S,H,G,bits", [(1024, 8, 4, 4), (333, 5, 2, 8), (8192, 32, 8, 4)])
def test_head_parallel_kv_cache_bitexact(dllm, torch, orc, S, H, G, bits):
    """K/V sharded by head over G ranks, emulated in one process with the HIP ops of
    parallel.HeadParallelKVCache (the all_reduce(MAX) of the per-rank extremes is a torch max here).
    Each shard's params equal the unsharded per-tensor params bit for bit, its packed codes equal
    the unsharded codes of its heads, and its attention equals the unsharded call's heads."""
    par = dllm.parallel
    rng = np.random.default_rng(S + H + G)
    K = rng.standard_normal((S, H, 128), dtype=np.float32)
    V = (rng.standard_normal((S, H, 128), dtype=np.float32) * 2 + 0.5).astype(np.float32)
    Q = rng.standard_normal((S, H, 128), dtype=np.float32).astype(np.float16)
    Kd, Vd, Qd = dev(torch, K), dev(torch, V), dev(torch, Q)
    full = dllm.QuantizedKVCacheEntry.new(Kd, Vd, bits)
    O_full = dllm.kv_attention(Qd, full.keys, full.values)
    ranks = []
    for r in range(G):
        kv = par.HeadParallelKVCache(H, bits)
        kv.world, kv.rank = G, r
        kv.h0, kv.h1 = par.head_range(H, G, r)
        loc = [t[:, kv.h0:kv.h1].contiguous() for t in (Qd, Kd, Vd)]
        ranks.append((kv, loc, kv.local_extremes(loc[1], loc[2])))
    red = torch.stack([x[2] for x in ranks]).amax(dim=0)
    codes_full = [dllm.unpack(t.data, S * H * 128, bits).reshape(S, H, 128) for t in (full.keys, full.values)]
    for kv, loc, _ in ranks:
        kc, kp, vc, vp = kv.quantize_with_extremes(loc[1], loc[2], red)
        n = S * (kv.h1 - kv.h0) * 128
        for c, p, ref_t, ref_c in ((kc, kp, full.keys, codes_full[0]), (vc, vp, full.values, codes_full[1])):
            assert same_bits(host(p), host(ref_t.params))
            assert torch.equal(dllm.unpack(c, n, bits).reshape(S, -1, 128), ref_c[:, kv.h0:kv.h1])
        e = kv.entry(loc[1], loc[2], red)
        O = kv.attention(loc[0], e)
        assert torch.equal(O, O_full[:, kv.h0:kv.h1]), "per-head attention must not depend on the shard"


def test_linear_prefill_only_handle(dllm, torch, orc):
    """DLLM_LINEAR_PREFILL_ONLY: no decode layout -- 8 MiB of codes + 1 MiB of sz/sf parameters +
    the bias (9.02 MiB, the canonical footprint) plus the 0.52 MiB of Horner ratios at 4096^2 int4
    g128, against 17.54 MiB for the full handle -- and its M <= 64 calls run the prefill kernels:
    within the exact-weight bound of the f32 product on the same f16 X, like the decode kernels of
    the full handle; M > 64 calls are the same kernels as the full handle's, bit for bit."""
    K = N = 4096
    W = 0.02 * torch.randn(K, N, device="cuda")
    full = dllm.QuantLinear.from_weight(W, None, 4, 128)
    pre = dllm.QuantLinear.from_weight(W, None, 4, 128, prefill_only=True)
    assert full.device_bytes() - pre.device_bytes() == K * N // 2          # exactly the decode layout
    assert pre.device_bytes() == K * N // 2 + 32 * N * 8 + N * 4 + 33 * N * 4, pre.device_bytes()
    codes, scales, zps = full.export()
    c2, s2, z2 = pre.export()
    assert torch.equal(codes, c2) and torch.equal(scales, s2) and torch.equal(zps, z2)
    cw, cs, cz = (host(t) for t in (codes, scales, zps))
    Wh = orc.dequantize_weights(orc.unpack_bits(cw, K * N, 4).reshape(K, N), cs, cz, 128)
    Wt = torch.from_numpy(Wh).cuda()
    for M in (1, 17, 64, 65, 300, 2048):
        X = torch.randn(M, K, device="cuda").half()
        ref = X.float() @ Wt
        y = pre(X, out_dtype=torch.float32)
        rel = float((y - ref).norm() / ref.norm())
        assert rel <= 2e-5, (M, rel)
        if M > 64:
            assert torch.equal(y, full(X, out_dtype=torch.float32)), M
    full.close()
    pre.close()


def test_bias_cast(dllm, torch):
    """dllm_bias_cast (the row-parallel epilogue): y + bias in f32, then RNE f16 or f32; vector and
    scalar paths (N % 4), no bias, f32 in place."""
    for M, N in ((2048, 4096), (33, 1027), (5, 3)):
        y = torch.randn(M, N, device="cuda")
        b = torch.randn(N, device="cuda")
        ref = y + b[None, :]
        assert torch.equal(dllm.quantization.bias_cast(y, b, torch.float16), ref.half())
        assert torch.equal(dllm.quantization.bias_cast(y, b, torch.float32), ref)
        assert torch.equal(dllm.quantization.bias_cast(y, None, torch.float16), y.half())
        yy = y.clone()
        dllm.quantization.bias_cast(yy, b, torch.float32, out=yy)
        assert torch.equal(yy, ref)


def test_bias_cast_refuses_other_dtypes(dllm, torch):
    """The kernel stores f16 or f32 only: a bf16 / f64 output, a non-f32 or non-contiguous y and a
    wrong-size bias are refused before any launch (a bf16 output used to get f32 stores
    past the end of its 2-byte buffer)."""
    y = torch.randn(64, 128, device="cuda")
    b = torch.randn(128, device="cuda")
    for dt in (torch.bfloat16, torch.float64):
        with pytest.raises(dllm.UnsupportedOperation):
            dllm.quantization.bias_cast(y, b, dt)
        with pytest.raises(dllm.UnsupportedOperation):
            dllm.quantization.bias_cast(y, b, out=torch.empty(64, 128, dtype=dt, device="cuda"))
    with pytest.raises(dllm.UnsupportedOperation):
        dllm.quantization.bias_cast(y.half(), b, torch.float16)
    with pytest.raises(dllm.UnsupportedOperation):
        dllm.quantization.bias_cast(y.t(), b, torch.float16)
    with pytest.raises(dllm.ShapeMismatch):
        dllm.quantization.bias_cast(y, b[:100], torch.float16)
    with pytest.raises(dllm.ShapeMismatch):
        dllm.quantization.bias_cast(y, b, out=torch.empty(64, 127, device="cuda"))


def test_graph_replay_after_workspace_growth(dllm, torch, orc):
    """A graph captured with an f32-X forward (the f32 -> f16 staging workspace of the stream) stays
    valid after a LARGER eager f32 forward on the same stream grew that workspace: the captured
    buffer is retired, not freed, so the replay reproduces its first result bit for bit."""
    K, N = 512, 256
    g = torch.Generator(device="cuda").manual_seed(77)
    lin = dllm.QuantLinear.from_weight(0.02 * torch.randn(K, N, device="cuda", generator=g), None, 4, 128)
    s = torch.cuda.Stream()
    Xs = torch.randn(96, K, device="cuda", generator=g)            # f32 X: staged to f16 in the workspace
    Xl = torch.randn(4096, K, device="cuda", generator=g)
    Ys = torch.empty(96, N, device="cuda")
    with torch.cuda.stream(s):
        lin(Xs, out=Ys)                                             # sizes the workspace for the small shape
        torch.cuda.current_stream().synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            lin(Xs, out=Ys)
        graph.replay()
        s.synchronize()
        first = Ys.clone()
        Ys.zero_()
        big = lin(Xl, out_dtype=torch.float32)                      # grows the same stream's workspace
        graph.replay()
        s.synchronize()
    assert torch.equal(Ys, first)
    assert bool(torch.isfinite(big).all())
    lin.close()


def _two_pass_ref(q, x, bits):
    """Codes and params by an independent device path: the min/max kernels (tensor_extremes), the
    params of :49-56, then the map alone (quantize_tensor_with_params)."""
    p = q.quantize_params_from_extremes(q.tensor_extremes(x), bits)
    return q.quantize_tensor_with_params(x, bits, p, packed=True), p


@pytest.mark.parametrize("nk,nv", [(1, 1), (7, 9), (2047, 2048), (2048, 2049), (100003, 77777), (1 << 21, 1 << 21),
                                   ((1 << 22) + 8, (1 << 22) + 2056), (2048 * 4096, 2048 * 4096),
                                   (8192 * 32 * 128, 8192 * 32 * 128), (40 << 20, 1 << 22)])
@pytest.mark.parametrize("bits_a,bits_b", [(4, 0), (8, 4), (2, 1), (1, 8)])
def test_quantize_kv_matches_per_tensor(dllm, torch, orc, nk, nv, bits_a, bits_b):
    """dllm_quantize_kv -- the single-pass resident kernel where the tensors fit on chip (K and V
    together: C5's 2 x 2048 x 4096; each alone: C4's 2 x 8192 x 32 x 128; ragged last slots), else
    the multi-pass kernels (a 40 Mi-value K) -- and dllm_quantize_tensor[_pair] on the same data,
    against an independent device path (min/max kernels + params + the map alone): codes and params
    bit-identical at one and two widths, NaN and +-inf included; the split form (dllm_kv_extremes +
    dllm_quantize_kv_with_extremes) likewise; the small sizes also against the oracle."""
    if nk > (1 << 21) and (bits_a, bits_b) not in ((4, 0), (8, 4)):
        pytest.skip("large sizes at the KV cache's widths only")
    q = dllm.quantization
    g = torch.Generator(device="cuda").manual_seed(nk + 3 * nv + bits_a)
    k = torch.randn(nk, device="cuda", generator=g) * 2 + 0.25
    v = torch.randn(nv, device="cuda", generator=g) * 0.5 - 1
    if nk > 64:
        k[nk // 3] = float("nan")
        v[nv // 5] = float("inf") if bits_a == 4 else float("nan")
    outs = q.quantize_kv(k, v, bits_a, bits_b)
    for w, bits in enumerate([bits_a] + ([bits_b] if bits_b else [])):
        kc, kp, vc, vp = outs[w]
        for x, c, pr in ((k, kc, kp), (v, vc, vp)):
            rc, rp = _two_pass_ref(q, x, bits)
            assert torch.equal(c, rc) and same_bits(host(pr), host(rp)), (w, bits)
            tc, tp = q.quantize_tensor(x, bits, packed=True)
            assert torch.equal(tc, rc) and same_bits(host(tp), host(rp)), (w, bits)
    if bits_b:
        (ka, pka), (kb, pkb) = q.quantize_tensor_pair(k, bits_a, bits_b, packed=True)
        assert torch.equal(ka, outs[0][0]) and torch.equal(kb, outs[1][0])
        assert same_bits(host(pka), host(outs[0][1])) and same_bits(host(pkb), host(outs[1][1]))
    red = q.kv_extremes(k, v)
    ek, ev = q.tensor_extremes(k), q.tensor_extremes(v)
    assert same_bits(host(red), host(torch.stack([-ek[0], ek[1], -ev[0], ev[1]])))
    outs2 = q.quantize_kv_with_extremes(k, v, red, bits_a, bits_b)
    for a, b in zip(outs, outs2):
        for ta, tb in zip(a, b):
            assert torch.equal(ta, tb)
    if nk <= 100003:
        rq, rs, rz = orc.quantize_tensor(host(k), bits_a)
        assert np.array_equal(host(outs[0][0]), orc.pack_bits(rq, bits_a))
        assert host(outs[0][1]).tobytes() == np.array([rs, rz], np.float32).tobytes()


def test_quantize_resident_vs_oracle_full_size(dllm, torch, orc):
    """The single-pass kernel at config C4's tensor size (8192 x 32 x 128 values, every slot of all
    256 blocks, 45 in VGPRs and 19 in LDS) against the C oracle: codes, packed bytes and params."""
    x = torch.randn(8192 * 32 * 128, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5)) * 3
    c, p = dllm.quantize_tensor(x, 4, packed=True)
    rq, rs, rz = orc.quantize_tensor(host(x), 4)
    assert np.array_equal(host(c), orc.pack_bits(rq, 4))
    assert host(p).tobytes() == np.array([rs, rz], np.float32).tobytes()


def test_quantize_kv_unaligned_and_empty(dllm, torch):
    """The generic fallbacks of dllm_quantize_kv: a K/V base not 16-B aligned, unpacked codes and an
    empty tensor give what quantize_tensor gives."""
    q = dllm.quantization
    base = torch.randn(70001, device="cuda")
    k, v = base[1:50001], base[50001:]
    for packed in (True, False):
        (kc, kp, vc, vp), = q.quantize_kv(k, v, 4, 0, packed)
        rk, rkp = q.quantize_tensor(k, 4, packed=packed)
        rv, rvp = q.quantize_tensor(v, 4, packed=packed)
        assert torch.equal(kc, rk) and torch.equal(vc, rv) and same_bits(host(kp), host(rkp)) and same_bits(host(vp), host(rvp))
    e = torch.empty(0, device="cuda")
    (kc, kp, vc, vp), = q.quantize_kv(e, v, 4, 0)
    rk, rkp = q.quantize_tensor(e, 4, packed=True)
    assert kc.numel() == 0 and same_bits(host(kp), host(rkp))
