"""CPU suite: pins the oracle.

1. The reference's own #[test] assertions for this path, replayed against the C oracle (the
   reference is Rust and cannot run here).  Three of them contradict the reference's code; the
   oracle follows the CODE and those asserts are recorded as expected failures.
2. The C oracle agrees bit-for-bit with the committed golden vectors, which were produced by the
   independent numpy restatement (tests/golden/make_golden.py).
"""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden" / "golden_v1.npz"


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def bits_of(a):
    return np.ascontiguousarray(a).view(np.uint8).tobytes()


# ---- 1. reference known-answer tests -------------------------------------------------------

def test_ref_quantized_tensor_ratio(orc):
    """diffuse-llm-rs/src/quantization.rs:254-265: len 4, compression_ratio() > 4 (== 8.0)."""
    q, s, z = orc.quantize_tensor(np.array([1, 2, 3, 4], np.float32), 4)
    assert orc.dequantize_tensor(q, s, z).size == 4
    assert orc.lib().orc_compression_ratio(4, 4, 4) == pytest.approx(8.0)


def test_ref_quantization_roundtrip_literal(orc):
    """quantization.rs:242-252 asserts |x - deq| < 0.1 for 4-bit [1..5]; under the code's literal
    semantics zp clamps to 0 and the max error is 1.0, so the oracle pins the
    code's output instead: q = [4, 7, 11, 15, 15], scale = 0x3E888889, zp = 0."""
    q, s, z = orc.quantize_tensor(np.arange(1, 6, dtype=np.float32), 4)
    assert q.tolist() == [4, 7, 11, 15, 15]
    assert np.float32(s).view(np.uint32) == 0x3E888889 and z == 0.0
    deq = orc.dequantize_tensor(q, s, z)
    assert np.max(np.abs(deq - np.arange(1, 6))) == pytest.approx(1.0, abs=1e-6)


@pytest.mark.xfail(strict=True, reason="reference test contradicts reference code (quantization.rs:242-252)")
def test_ref_quantization_roundtrip_as_written(orc):
    x = np.arange(1, 6, dtype=np.float32)
    q, s, z = orc.quantize_tensor(x, 4)
    assert np.all(np.abs(x - orc.dequantize_tensor(q, s, z)) < 0.1)


def test_ref_compress_vector(orc):
    """diffusion_prefill/src/prefill_kv.rs:147-160 (passes under the code): within 0.1."""
    x = np.array([0.1, 0.5, 1.0, 0.0], np.float32)
    q, s, z = orc.compress_vector(x, 4)
    assert q.tolist() == [1, 7, 14, 0]
    assert np.all(np.abs(orc.bit_dequantize(q, s, z) - x) < 0.1)


def test_ref_calibration_literal(onp):
    """quantization/src/calibrate.rs:123-132 expects scale 0.0235 / zp -43; the code gives
    scale = 5/255 = 0.019607844, zp = round(-1 / scale) = -51."""
    cal = onp.Calibration(10)
    cal.update(np.array([[1, 2, 3], [4, 5, 6]], np.float32))
    s, z = cal.compute_params(8, False)
    assert np.float32(s) == np.float32(5.0) / np.float32(255.0) and z == -51


@pytest.mark.xfail(strict=True, reason="reference test contradicts reference code (calibrate.rs:123-132)")
def test_ref_calibration_as_written(onp):
    cal = onp.Calibration(10)
    cal.update(np.array([[1, 2, 3], [4, 5, 6]], np.float32))
    s, z = cal.compute_params(8, False)
    assert abs(s - 0.0235) < 1e-3 and z == -43


def test_ref_default_int8_roundtrip_literal(orc):
    """quantization/src/lib.rs:61-79: Int8 round trip of [[-1,0,1],[2,3,4]]; the saturating
    `q as u8` maps -1 -> 0, so the code dequantizes -1.0 to 0.0."""
    x = np.array([[-1, 0, 1], [2, 3, 4]], np.float32)
    q = orc.default_quantize(x, 0, 1.0, 0)
    assert q.tolist() == [0, 0, 1, 2, 3, 4]
    assert orc.default_dequantize(q, 1.0, 0).tolist() == [0, 0, 1, 2, 3, 4]


@pytest.mark.xfail(strict=True, reason="reference test contradicts reference code (quantization/src/lib.rs:61-79)")
def test_ref_default_int8_roundtrip_as_written(orc):
    x = np.array([-1, 0, 1, 2, 3, 4], np.float32)
    d = orc.default_dequantize(orc.default_quantize(x, 0, 1.0, 0), 1.0, 0)
    assert np.all(np.abs(x - d) < 0.1)


def test_ref_quantize_int8_shape(orc):
    """quantization/src/quantize.rs:222-233: shape [2,3] preserved (6 codes, 6 values)."""
    x = np.array([[-1, 0, 1], [2, 3, 4]], np.float32)
    assert orc.default_quantize(x, 0).size == 6


def test_ref_prefill_quantizer_index_panics(orc):
    """prefill-kvquant-rs/lib.rs:133: quantizers[bits/2] with the default [4,6,8,16] config panics
    for an 8-bit request (index 4 of 4)."""
    x = np.zeros((2, 8), np.float32)
    with pytest.raises(orc.OracleError):
        orc.quantize_vectors(x, [4, 6, 8, 16], [8])
    q, w = orc.quantize_vectors(x + 0.5, [4, 6, 8, 16], [4])  # 4-bit request uses the 8-bit scale 1/255
    assert w.tolist() == [4, 4] and np.all(q == 15)


# ---- 2. C oracle == numpy restatement (golden vectors) ------------------------------------

def test_golden_a1_a2(orc, gold):
    names = sorted({k.split("/")[1] for k in gold if k.startswith("a1/")})
    for name in names:
        x = gold[f"a1/{name}/x"]
        for bits in range(1, 9):
            q, s, z = orc.quantize_tensor(x, bits)
            assert np.array_equal(q, gold[f"a1/{name}/b{bits}/q"]), (name, bits)
            assert bits_of(np.array([s, z], np.float32)) == bits_of(gold[f"a1/{name}/b{bits}/params"]), (name, bits)
            assert bits_of(orc.dequantize_tensor(q, s, z)) == bits_of(gold[f"a1/{name}/b{bits}/deq"]), (name, bits)
            assert np.array_equal(orc.pack_bits(q, bits), gold[f"a1/{name}/b{bits}/packed"])


def test_golden_a6(orc, gold):
    for bits in range(1, 9):
        c = gold[f"a6/b{bits}/codes"]
        p = orc.pack_bits(c, bits)
        assert np.array_equal(p, gold[f"a6/b{bits}/packed"])
        assert np.array_equal(orc.unpack_bits(p, c.size, bits), c)


def test_golden_a4(orc, gold):
    x = gold["a4/x"]
    for qt in range(4):
        for tag, (s, z) in {"p0": (1.0, 0), "p1": (0.37, 3)}.items():
            q = orc.default_quantize(x, qt, s, z)
            assert np.array_equal(q, gold[f"a4/qt{qt}/{tag}/q"]), (qt, tag)
            assert bits_of(orc.default_dequantize(q, s, z)) == bits_of(gold[f"a4/qt{qt}/{tag}/deq"])
    assert np.array_equal(orc.default_quantize(gold["a4/basic_example/x"], 0), gold["a4/basic_example/q"])


def test_golden_a8(orc, gold):
    x = gold["a8/x"]
    for bits in (2, 4, 8, 16):
        for tag in ("pref", "aff"):
            s, z = gold[f"a8/b{bits}/{tag}/params"]
            q = orc.bit_quantize(x, bits, s, z)
            assert np.array_equal(q, gold[f"a8/b{bits}/{tag}/q"]), (bits, tag)
            assert bits_of(orc.bit_dequantize(q, s, z)) == bits_of(gold[f"a8/b{bits}/{tag}/deq"])
        for i, row in enumerate(gold[f"a8iii/b{bits}/x"]):
            q, s, z = orc.compress_vector(row, bits)
            assert np.array_equal(q, gold[f"a8iii/b{bits}/q"][i])
            assert s == gold[f"a8iii/b{bits}/scale"][i] and z == gold[f"a8iii/b{bits}/zp"][i]
    q, w = orc.quantize_vectors(gold["qv/x"], [4, 6, 8, 16], [2, 4])
    assert np.array_equal(q, gold["qv/q"]) and np.array_equal(w, gold["qv/widths"])


def test_golden_a5(orc, gold):
    W = gold["a5/W"]
    codes, scales, zps = orc.quantize_weights(W, 4, 128)
    assert np.array_equal(codes, gold["a5/codes"])
    assert bits_of(scales) == bits_of(gold["a5/scales"]) and np.array_equal(zps, gold["a5/zps"])
    assert np.array_equal(orc.pack_bits(codes.ravel(), 4), gold["a5/packed"])
    Y = orc.linear_forward(gold["a5/X"], orc.dequantize_weights(codes, scales, zps, 128))
    ref = gold["a5/Y"]
    assert np.linalg.norm(Y - ref) / np.linalg.norm(ref) < 1e-6
    for bits in (2, 8):
        c2, s2, z2 = orc.quantize_weights(W, bits, 128)
        assert np.array_equal(c2, gold[f"a5/b{bits}/codes"]) and bits_of(s2) == bits_of(gold[f"a5/b{bits}/scales"])
        assert np.array_equal(z2, gold[f"a5/b{bits}/zps"])


def test_golden_a10_numpy_vs_c(orc, onp, gold):
    """The C oracle's calibration (orc_calib_*) against the golden stream."""
    L = orc.lib()

    class Calib(C.Structure):
        _fields_ = [("min", C.c_float), ("max", C.c_float), ("num_bins", C.c_size_t),
                    ("total_samples", C.c_size_t), ("histogram", C.c_void_p)]

    L.orc_calib_init.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
    L.orc_calib_update.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.orc_calib_compute_params.argtypes = [C.c_void_p, C.c_uint8, C.c_int, C.c_void_p, C.c_void_p]
    hist = np.zeros(64, np.uint64)
    cb = Calib()
    L.orc_calib_init(C.byref(cb), 64, hist.ctypes.data)
    for i in range(3):
        x = np.ascontiguousarray(gold[f"a10/rand/x{i}"])
        L.orc_calib_update(C.byref(cb), x.ctypes.data, x.size)
    assert np.array([cb.min, cb.max], np.float32).tobytes() == gold["a10/rand/minmax"].tobytes()
    assert np.array_equal(hist.astype(np.int64), gold["a10/rand/hist"])
    for bits in (4, 8):
        for sym in (0, 1):
            s, z = C.c_float(), C.c_int32()
            assert L.orc_calib_compute_params(C.byref(cb), bits, sym, C.byref(s), C.byref(z)) == 0
            exp = gold[f"a10/rand/params_b{bits}_s{sym}"]
            assert np.float32(s.value) == exp[0] and z.value == int(exp[1])


def test_oracle_attention_softmax_identity(orc):
    """a9 oracle sanity: with V = one-hot of the key index and identical keys, O is uniform."""
    S, H, D = 8, 2, 16
    Q = np.ones((S, H, D), np.float32)
    K = np.ones((S, H, D), np.float32)
    V = np.zeros((S, H, D), np.float32)
    for j in range(S):
        V[j, :, j] = 1.0
    O = orc.attention(Q, K, V, nthreads=1)
    assert np.allclose(O[:, :, :S], 1.0 / S) and np.allclose(O[:, :, S:], 0.0)


def test_attention_rows_matches_c_oracle(orc):
    """The row-sampled f64 SDPA checker (oracle.attention_rows) agrees with the C oracle's
    orc_attention on the same rows."""
    rng = np.random.default_rng(9)
    S, H, D = 200, 3, 128
    Q, K, V = (rng.standard_normal((S, H, D)).astype(np.float32) for _ in range(3))
    full = orc.attention(Q, K, V)
    rows = np.array([0, 7, 63, 64, 199])
    np.testing.assert_allclose(orc.attention_rows(Q[rows], K, V), full[rows], rtol=0, atol=1e-6)
