"""CPU suite: the C-ABI wire formats (include/dllm_quant.h section f3, csrc/serde.cpp) against the
independent Python restatement in the oracle (oracle/serde_ref.py, test infrastructure) of the same
published layouts
(bincode 1.3 legacy, serde_json + ryu) for QuantizationParams / QuantizedTensor
(quantization/src/types.rs:19-47) and CompressedVector (diffusion_prefill/src/prefill_kv.rs:25-33):
byte-identical encodings, decoders that invert them, the bincode trailing-byte rule and
malformed-input errors.  Parity with the Rust crates themselves is unpinned (none ship a fixture)."""
import ctypes as C
import math

import numpy as np
import pytest


class QP(C.Structure):
    _fields_ = [("bits", C.c_uint8), ("scale", C.c_float), ("zero_point", C.c_int32), ("symmetric", C.c_uint8),
                ("has_axis", C.c_uint8), ("axis", C.c_uint64)]


def qp(p):
    return QP(p.bits, p.scale, p.zero_point, int(p.symmetric), 0 if p.axis is None else 1,
              0 if p.axis is None else p.axis)


def out_buf(fn, *args):
    n = C.c_size_t()
    assert fn(*args, None, 0, C.byref(n)) == 0
    buf = C.create_string_buffer(max(1, n.value))
    assert fn(*args, buf, n.value, C.byref(n)) == 0
    return buf.raw[: n.value]


FLOATS = [0.1, 1.0, -2.5, 1e-7, 1.5e-5, 9.99e-6, 1e13, 1.234e12, 3.4028235e38, 1.4e-45, 1.17549435e-38,
          -0.0, 0.0, 0.26666668, 123456.79, 1e-3, float("nan"), float("inf"), -float("inf")]


@pytest.fixture(scope="module")
def lib(dllm):
    return dllm._lib.load()


@pytest.fixture(scope="module")
def ref():
    from oracle import serde_ref
    return serde_ref


def params_cases(ref):
    rng = np.random.default_rng(5)
    out = []
    for i, f in enumerate(FLOATS):
        out.append(ref.Params(bits=int(rng.integers(0, 256)), scale=f,
                                           zero_point=int(rng.integers(-2**31, 2**31)), symmetric=bool(i % 2),
                                           axis=None if i % 3 == 0 else int(rng.integers(0, 2**40))))
    return out


def test_format_f32_matches_ryu_layout(dllm, lib, ref):
    rng = np.random.default_rng(0)
    vals = FLOATS[:-3] + list(rng.standard_normal(200).astype(np.float32)) + \
        list((10.0 ** rng.uniform(-40, 38, 300)).astype(np.float32))
    for v in vals:
        got = out_buf(lib.dllm_format_f32, C.c_float(v)).decode()
        assert got == ref.ryu_f32(v), v
        assert np.float32(float(got)) == np.float32(v) or (v == 0 and got.endswith("0.0"))
    assert out_buf(lib.dllm_format_f32, C.c_float(float("nan"))) == b"null"


def test_params_bincode_json(dllm, lib, ref):
    S = ref
    for p in params_cases(ref):
        c = qp(p)
        b = out_buf(lib.dllm_qparams_to_bincode, C.byref(c))
        assert b == S.params_to_bincode(p)
        j = out_buf(lib.dllm_qparams_to_json, C.byref(c)).decode()
        assert j == S.params_to_json(p)
        # decode both encodings back (bincode keeps the f32 bits; json: null -> NaN like serde's f32 visitor)
        r, used = QP(), C.c_size_t()
        assert lib.dllm_qparams_from_bincode(b + b"\x07\x07", len(b) + 2, 0, C.byref(r), C.byref(used)) == 0
        assert used.value == len(b)
        assert bytes(r)[:1] == bytes(c)[:1] and r.zero_point == c.zero_point and r.axis == c.axis
        assert np.float32(r.scale).tobytes() == np.float32(c.scale).tobytes()
        assert lib.dllm_qparams_from_bincode(b + b"\x00", len(b) + 1, 1, C.byref(r), None) == dllm._lib.ERR_SERIALIZATION
        r2 = QP()
        assert lib.dllm_qparams_from_json(j.encode(), len(j), C.byref(r2)) == 0
        py = S.params_from_json(j)
        assert (r2.bits, r2.zero_point, bool(r2.symmetric)) == (py.bits, py.zero_point, py.symmetric)
        assert (None if not r2.has_axis else r2.axis) == py.axis
        assert (math.isnan(r2.scale) and math.isnan(py.scale)) or np.float32(r2.scale) == np.float32(py.scale)


def test_params_malformed(dllm, lib):
    r = QP()
    bad_tag = bytes([4]) + np.float32(1).tobytes() + (3).to_bytes(4, "little") + b"\x01\x02"
    assert lib.dllm_qparams_from_bincode(bad_tag, len(bad_tag), 0, C.byref(r), None) == dllm._lib.ERR_SERIALIZATION
    assert lib.dllm_qparams_from_bincode(bad_tag[:5], 5, 0, C.byref(r), None) == dllm._lib.ERR_SERIALIZATION
    for s in (b'{"bits":4,"scale":1.0,"zero_point":0,"symmetric":true}',          # missing field
              b'{"bits":256,"scale":1.0,"zero_point":0,"symmetric":true,"axis":null}',   # u8 range
              b'{"bits":4,"scale":1.0,"zero_point":0,"symmetric":1,"axis":null}',       # bool type
              b'{"bits":4,"scale":1.0,"zero_point":0,"symmetric":true,"axis":null} x'):  # trailing
        assert lib.dllm_qparams_from_json(s, len(s), C.byref(r)) == dllm._lib.ERR_SERIALIZATION, s


@pytest.mark.parametrize("n,shape", [(0, []), (5, [5]), (4096, [1, 64, 64]), (300, [3, 100])])
def test_qtensor_bincode_json(dllm, lib, ref, n, shape):
    S = ref
    rng = np.random.default_rng(n)
    codes = rng.integers(0, 256, n).astype(np.uint8)
    p = ref.Params(bits=4, scale=0.0123, zero_point=7, symmetric=False, axis=None if n % 2 else 1)
    t = ref.TensorRecord(codes, tuple(shape), p)
    shp = (C.c_uint64 * max(1, len(shape)))(*shape)
    c = qp(p)
    b = out_buf(lib.dllm_qtensor_to_bincode, codes.ctypes.data, n, shp, len(shape), C.byref(c))
    assert b == S.qtensor_to_bincode(t)
    j = out_buf(lib.dllm_qtensor_to_json, codes.ctypes.data, n, shp, len(shape), C.byref(c)).decode()
    assert j == S.qtensor_to_json(t)
    # decode: size query, then fill
    cn, cd, r = C.c_size_t(), C.c_size_t(), QP()
    assert lib.dllm_qtensor_from_bincode(b, len(b), 1, None, 0, C.byref(cn), None, 0, C.byref(cd), C.byref(r)) == 0
    assert (cn.value, cd.value) == (n, len(shape))
    oc = np.zeros(max(1, n), np.uint8)
    os_ = (C.c_uint64 * max(1, len(shape)))()
    assert lib.dllm_qtensor_from_bincode(b, len(b), 1, oc.ctypes.data, oc.size, C.byref(cn), os_, len(os_),
                                         C.byref(cd), C.byref(r)) == 0
    assert np.array_equal(oc[:n], codes) and list(os_)[: len(shape)] == shape and r.zero_point == 7
    oc[:] = 0
    assert lib.dllm_qtensor_from_json(j.encode(), len(j), oc.ctypes.data, oc.size, C.byref(cn), os_, len(os_),
                                      C.byref(cd), C.byref(r)) == 0
    assert np.array_equal(oc[:n], codes) and list(os_)[: len(shape)] == shape
    assert np.float32(r.scale) == np.float32(0.0123)
    # truncated input and out-of-range json data are errors
    assert lib.dllm_qtensor_from_bincode(b[:-1], len(b) - 1, 0, None, 0, C.byref(cn), None, 0, C.byref(cd),
                                         C.byref(r)) == dllm._lib.ERR_SERIALIZATION
    bad = j.replace('"data":[', '"data":[256,', 1).encode()
    assert lib.dllm_qtensor_from_json(bad, len(bad), None, 0, C.byref(cn), None, 0, C.byref(cd),
                                      C.byref(r)) == dllm._lib.ERR_SERIALIZATION


@pytest.mark.parametrize("ident", ["0", "row-17", 'quote"back\\slash', "tab\tnl\nctl\x01", "ünï-κωδ"])
def test_compressed_vector(dllm, lib, ref, ident):
    S = ref
    rng = np.random.default_rng(len(ident))
    data = rng.integers(0, 16, 40).astype(np.uint8)
    rec = S.PrefillCompressedVector(ident, data, 4, [40], float(np.float32(0.071)), float(np.float32(-1.25)))
    idb = ident.encode()
    shp = (C.c_uint64 * 1)(40)
    args = (idb, len(idb), data.ctypes.data, data.size, 4, shp, 1, C.c_float(rec.quant_scale),
            C.c_float(rec.quant_zero_point))
    b = out_buf(lib.dllm_compressed_vector_to_bincode, *args)
    assert b == rec.to_bincode()
    j = out_buf(lib.dllm_compressed_vector_to_json, *args).decode()
    assert j == rec.to_json()
    idl, n, nb, nd = C.c_size_t(), C.c_size_t(), C.c_uint8(), C.c_size_t()
    sc, zp = C.c_float(), C.c_float()
    ib = C.create_string_buffer(64)
    ob = np.zeros(64, np.uint8)
    os_ = (C.c_uint64 * 4)()
    assert lib.dllm_compressed_vector_from_bincode(b, len(b), 1, ib, 64, C.byref(idl), ob.ctypes.data, 64, C.byref(n),
                                                   C.byref(nb), os_, 4, C.byref(nd), C.byref(sc), C.byref(zp)) == 0
    assert ib.raw[: idl.value] == idb and np.array_equal(ob[: n.value], data) and nb.value == 4
    assert list(os_)[: nd.value] == [40] and np.float32(sc.value) == np.float32(0.071) and zp.value == -1.25
    bad = bytearray(b)
    bad[8] = 0xFF      # first byte of the id: not valid UTF-8
    assert lib.dllm_compressed_vector_from_bincode(bytes(bad), len(bad), 0, ib, 64, C.byref(idl), None, 0, C.byref(n),
                                                   C.byref(nb), None, 0, C.byref(nd), C.byref(sc),
                                                   C.byref(zp)) == dllm._lib.ERR_SERIALIZATION


@pytest.mark.parametrize("ident", ["0", 'quote"back\\slash', "tab\tnl\nctl\x01\x1f", "ünï-κωδ-😀"])
def test_compressed_vector_json_decode(dllm, ref, ident):
    """dllm_compressed_vector_from_json (through the product's PrefillCompressedVector.from_json)
    inverts the C-ABI encoder and agrees with the oracle's decoder field for field, escapes and
    non-BMP characters included; \\u escapes (surrogate pairs too) decode as serde_json does, and
    raw control characters, lone surrogates, out-of-range codes and trailing text are
    SerializationError."""
    S = dllm.serde
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, 33).astype(np.uint8)
    rec = S.PrefillCompressedVector(ident, data, 8, [33], float(np.float32(0.3)), float(np.float32(-2.0)))
    j = rec.to_json()
    assert j == ref.PrefillCompressedVector(ident, data, 8, [33], rec.quant_scale, rec.quant_zero_point).to_json()
    back = S.PrefillCompressedVector.from_json(j)
    oref = ref.PrefillCompressedVector.from_json(j)
    for r in (back, oref):
        assert r.id == ident and np.array_equal(r.data, data) and r.bits == 8 and r.original_shape == [33]
        assert np.float32(r.quant_scale) == np.float32(0.3) and r.quant_zero_point == -2.0
    esc = '{"id":"a\\u00e9\\ud83d\\ude00\\/","data":[],"bits":2,"original_shape":[],"quant_scale":null,' \
          '"quant_zero_point":1e-3}'
    r = S.PrefillCompressedVector.from_json(esc)
    assert r.id == "aé😀/" and r.data.size == 0 and np.isnan(r.quant_scale)
    assert np.float32(r.quant_zero_point) == np.float32(1e-3)
    good = '{"id":"a","data":[1],"bits":4,"original_shape":[1],"quant_scale":0.5,"quant_zero_point":0.0}'
    for bad in (good.replace('"a"', '"a\x01"'), good.replace('"a"', '"\\udc00"'), good.replace('[1]', '[256]', 1),
                good + " x", good.replace(',"bits":4', '')):
        with pytest.raises(dllm.SerializationError):
            S.PrefillCompressedVector.from_json(bad)


def test_json_unknown_and_duplicate_fields(dllm, lib, ref):
    """serde's derived Deserialize on QuantizationParams / QuantizedTensor / CompressedVector (no
    deny_unknown_fields): an unknown field -- any JSON value, nested ones included -- is skipped, a
    field given twice is an error, and a String that is not valid UTF-8 is a data error; the C
    reader and the oracle's restatement agree."""
    S = dllm.serde
    pj = '{"bits":4,"extra":{"a":[1,{"b":null}],"c":"x"},"scale":0.5,"zero_point":3,"symmetric":false,"axis":null}'
    r = QP()
    assert lib.dllm_qparams_from_json(pj.encode(), len(pj), C.byref(r)) == 0
    assert r.bits == 4 and r.zero_point == 3 and ref.params_from_json(pj).zero_point == 3
    dup = '{"bits":4,"scale":0.5,"zero_point":3,"zero_point":4,"symmetric":false,"axis":null}'
    assert lib.dllm_qparams_from_json(dup.encode(), len(dup), C.byref(r)) == dllm._lib.ERR_SERIALIZATION
    with pytest.raises(ref.SerializationError):
        ref.params_from_json(dup)
    good = '{"id":"a","data":[1],"bits":4,"original_shape":[1],"quant_scale":0.5,"quant_zero_point":0.0}'
    extra = good.replace('"bits":4', '"bits":4,"note":[true,false,-1.5e3,"s"]')
    v = S.PrefillCompressedVector.from_json(extra)
    assert v.bits == 4 and list(v.data) == [1] and ref.PrefillCompressedVector.from_json(extra).bits == 4
    for bad in (good.replace('"data":[1]', '"data":[1],"data":[2]'),
                good.replace('"original_shape":[1]', '"original_shape":[1],"original_shape":[1]')):
        with pytest.raises(dllm.SerializationError):
            S.PrefillCompressedVector.from_json(bad)
        with pytest.raises(ref.SerializationError):
            ref.PrefillCompressedVector.from_json(bad)
    raw = good.encode().replace(b'"a"', b'"a\xff"')
    with pytest.raises(dllm.SerializationError):
        S.PrefillCompressedVector.from_json(raw)
    tj = '{"shape":[2],"skip":{},"data":[7,8],"params":' + pj + '}'
    t = S.qtensor_from_json(tj, device="cpu")
    assert list(t.shape) == [2] and ref.qtensor_from_json(tj).shape == (2,)
