"""Wire formats: bincode 1.3 legacy layout and serde_json compact form of
QuantizationParams / QuantizedTensor (quantization/src/types.rs:19-47) and the diffusion_prefill
CompressedVector (prefill_kv.rs:25-33).  The reference ships no serialized fixture, so the expected
bytes/strings below are derived by hand from the encoders' published specifications (parity
unpinned beyond them).  CPU only: the records are host objects."""
import json
import struct

import numpy as np
import pytest


@pytest.fixture(scope="module")
def sd():
    import __graft_entry__ as g
    return g.load_package()


@pytest.mark.parametrize("x,s", [
    (1.0, "1.0"), (0.1, "0.1"), (-2.5, "-2.5"), (0.0, "0.0"), (-0.0, "-0.0"), (100.0, "100.0"),
    (0.26666668, "0.26666668"), (1e-7, "1e-7"), (1.5e-6, "0.0000015"), (1e-6, "0.000001"),
    (123456789.0, "123456790.0"), (1e10, "10000000000.0"), (1e13, "1e13"), (1.25e13, "1.25e13"),
    (3.4028235e38, "3.4028235e38"), (1.4e-45, "1e-45"), (12.34, "12.34"), (0.001234, "0.001234"),
])
def test_ryu_f32_layout(sd, x, s):
    assert sd.serde.ryu_f32(x) == s
    assert np.float32(float(s)) == np.float32(x)   # round trip through serde's f64 -> f32 parse


def test_ryu_shortest_roundtrip_random(sd):
    rng = np.random.default_rng(0)
    vals = rng.standard_normal(2000).astype(np.float32) * np.float32(10.0) ** rng.integers(-12, 12, 2000)
    for v in vals.astype(np.float32):
        s = sd.serde.ryu_f32(v)
        assert np.float32(float(s)) == v, (v, s)


def test_params_bincode_layout(sd):
    P = sd.QuantizationParams
    p = P(bits=4, scale=0.5, zero_point=-3, symmetric=False, axis=None)
    b = sd.serde.params_to_bincode(p)
    assert b == bytes([4]) + struct.pack("<f", 0.5) + struct.pack("<i", -3) + b"\x00" + b"\x00"
    q = P(bits=8, scale=1.0, zero_point=0, symmetric=True, axis=2)
    b2 = sd.serde.params_to_bincode(q)
    assert b2 == bytes([8]) + struct.pack("<f", 1.0) + b"\x00\x00\x00\x00" + b"\x01" + b"\x01" + struct.pack("<Q", 2)
    assert sd.serde.params_from_bincode(b) == p and sd.serde.params_from_bincode(b2) == q
    with pytest.raises(sd.SerializationError):
        sd.serde.params_from_bincode(b2[:-1])
    # bincode 1.3's deserialize (legacy options) allows trailing bytes; strict readers reject them
    assert sd.serde.params_from_bincode(b + b"\x00\x07") == p
    with pytest.raises(sd.SerializationError):
        sd.serde.params_from_bincode(b + b"\x00", strict=True)


def test_params_json(sd):
    P = sd.QuantizationParams
    assert sd.serde.params_to_json(P()) == '{"bits":8,"scale":1.0,"zero_point":0,"symmetric":true,"axis":null}'
    p = P(bits=4, scale=0.26666668, zero_point=7, symmetric=False, axis=1)
    s = sd.serde.params_to_json(p)
    assert s == '{"bits":4,"scale":0.26666668,"zero_point":7,"symmetric":false,"axis":1}'
    assert sd.serde.params_from_json(s) == P(bits=4, scale=float(np.float32(0.26666668)), zero_point=7,
                                             symmetric=False, axis=1)
    assert '"scale":null' in sd.serde.params_to_json(P(scale=float("nan")))   # serde_json: non-finite -> null


def test_qtensor_bincode_and_json_roundtrip(sd):
    import torch
    codes = np.arange(10, dtype=np.uint8)
    t = sd.quant.QuantizedTensor(torch.from_numpy(codes), (2, 5), sd.QuantizationParams(bits=4, scale=0.25))
    b = sd.serde.qtensor_to_bincode(t)
    head = struct.pack("<Q", 10) + codes.tobytes() + struct.pack("<Q", 2) + struct.pack("<QQ", 2, 5)
    assert b.startswith(head) and len(b) == len(head) + 1 + 4 + 4 + 1 + 1
    t2 = sd.serde.qtensor_from_bincode(b, device="cpu")
    assert np.array_equal(t2.data.numpy(), codes) and t2.shape == (2, 5) and t2.params == t.params
    s = sd.serde.qtensor_to_json(t)
    assert s == ('{"data":[0,1,2,3,4,5,6,7,8,9],"shape":[2,5],'
                 '"params":{"bits":4,"scale":0.25,"zero_point":0,"symmetric":true,"axis":null}}')
    assert json.loads(s)["shape"] == [2, 5]
    t3 = sd.serde.qtensor_from_json(s, device="cpu")
    assert np.array_equal(t3.data.numpy(), codes) and t3.params == t.params
    with pytest.raises(sd.SerializationError):
        sd.serde.qtensor_from_json(s.replace("[0,1,", "[300,1,"), device="cpu")


def test_compressed_vector_record(sd):
    rec = sd.serde.PrefillCompressedVector("k0", np.array([1, 7, 14, 0], np.uint8), 4, [4], 0.0666666701, -0.5)
    b = rec.to_bincode()
    exp = (struct.pack("<Q", 2) + b"k0" + struct.pack("<Q", 4) + bytes([1, 7, 14, 0]) + bytes([4]) +
           struct.pack("<QQ", 1, 4) + struct.pack("<ff", np.float32(0.0666666701), -0.5))
    assert b == exp
    r2 = sd.serde.PrefillCompressedVector.from_bincode(b)
    assert r2.id == "k0" and np.array_equal(r2.data, rec.data) and r2.original_shape == [4]
    assert np.float32(r2.quant_scale) == np.float32(0.0666666701) and r2.quant_zero_point == -0.5
    s = rec.to_json()
    assert s == ('{"id":"k0","data":[1,7,14,0],"bits":4,"original_shape":[4],'
                 '"quant_scale":0.06666667,"quant_zero_point":-0.5}')
    r3 = sd.serde.PrefillCompressedVector.from_json(s)
    assert np.float32(r3.quant_scale) == np.float32(0.0666666701)


def test_compressed_vector_json_u8_range_and_shape(sd):
    """from_json rejects codes outside u8 (serde's Vec<u8> visitor) with SerializationError, not an
    OverflowError or a silent wrap; a 3-D input row's record has original_shape = [row length]
    (vec![vector.len()], prefill_kv.rs:117)."""
    good = ('{"id":"a","data":[1,255],"bits":4,"original_shape":[2],"quant_scale":0.5,"quant_zero_point":0.0}')
    assert list(sd.serde.PrefillCompressedVector.from_json(good).data) == [1, 255]
    for bad in ('[1,256]', '[-1,2]', '[1.5,2]', '[[1],[2]]'):
        with pytest.raises(sd.SerializationError):
            sd.serde.PrefillCompressedVector.from_json(good.replace('[1,255]', bad))
