"""Generates the committed golden vectors in tests/golden/*.npz (no pickles: plain arrays).

The expected outputs come from the independent numpy restatement (oracle/oracle_np.py); the C
oracle and the HIP kernels are both checked against these files.  Inputs are seeded; regenerate
with ``python tests/golden/make_golden.py`` (the reference itself cannot be run here: it is Rust,
no toolchain, and does not compile as shipped -- SURVEY.md section 4.3).
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))
from oracle import oracle_np as N  # noqa: E402


def edge_inputs(rng):
    return {
        "randn4096": rng.standard_normal(4096).astype(np.float32),
        "const": np.full(100, 3.5, np.float32),
        "allpos": (np.abs(rng.standard_normal(333)) + 1).astype(np.float32),
        "allneg": (-np.abs(rng.standard_normal(333)) - 1).astype(np.float32),
        "specials": np.array([0.0, -0.0, np.nan, 1.0, 2.5, -2.0, 7.0], np.float32),
        "inf": np.array([1.0, np.inf, -3.0, 2.0], np.float32),
        "ref_test": np.arange(1, 6, dtype=np.float32),  # quantization.rs:244
        "empty": np.zeros(0, np.float32),
        "odd13": rng.uniform(-5, 5, 13).astype(np.float32),
    }


def main():
    rng = np.random.default_rng(20251010)
    out = {}
    # a1 / a2 (quantization.rs:38-85) for bits 1..8 on every edge input.
    for name, x in edge_inputs(rng).items():
        out[f"a1/{name}/x"] = x
        for bits in range(1, 9):
            q, s, z = N.quantize_tensor(x, bits)
            out[f"a1/{name}/b{bits}/q"] = q
            out[f"a1/{name}/b{bits}/packed"] = N.pack_bits(q, bits)
            out[f"a1/{name}/b{bits}/params"] = np.array([s, z], np.float32)
            out[f"a1/{name}/b{bits}/deq"] = N.dequantize_tensor(q, s, z)
    # a6 pack/unpack for every width.
    for bits in range(1, 9):
        c = rng.integers(0, 1 << bits, 1003).astype(np.uint8)
        out[f"a6/b{bits}/codes"] = c
        out[f"a6/b{bits}/packed"] = N.pack_bits(c, bits)
    # a4 DefaultQuantizer on a 64x64 tile, all four types, default + non-default params.
    x = (rng.standard_normal((64, 64)) * 4).astype(np.float32)
    x.ravel()[:3] = [np.nan, np.inf, -np.inf]
    out["a4/x"] = x
    for qt in range(4):
        for tag, (s, z) in {"p0": (1.0, 0), "p1": (0.37, 3)}.items():
            q = N.default_quantize(x, qt, s, z)
            out[f"a4/qt{qt}/{tag}/q"] = q
            out[f"a4/qt{qt}/{tag}/deq"] = N.default_dequantize(q, s, z)
    out["a4/basic_example/x"] = np.array([[-1.5, -0.5, 0.5, 1.5], [2.0, 3.0, 4.0, 5.0]], np.float32)
    out["a4/basic_example/q"] = N.default_quantize(out["a4/basic_example/x"], 0, 1.0, 0)
    # a8-ii BitQuantizer for bits {2,4,8,16}, a8-iii compress_vector.
    kv = (rng.standard_normal(2048) * 0.7).astype(np.float32)
    kv[:3] = [np.nan, 5.0, -5.0]
    out["a8/x"] = kv
    for bits in (2, 4, 8, 16):
        for tag, (s, z) in {"pref": (float(N.prefill_scale(bits if bits < 16 else 16)), 0.0),
                            "aff": (0.05, -1.0)}.items():
            q = N.bit_quantize(kv, bits, s, z)
            out[f"a8/b{bits}/{tag}/q"] = q
            out[f"a8/b{bits}/{tag}/params"] = np.array([s, z], np.float32)
            out[f"a8/b{bits}/{tag}/deq"] = N.bit_dequantize(q, s, z)
        rows = kv[3:3 + 16 * 64].reshape(16, 64)
        qs, ss, zs = zip(*(N.compress_vector(r, bits) for r in rows))
        out[f"a8iii/b{bits}/x"] = rows
        out[f"a8iii/b{bits}/q"] = np.stack(qs)
        out[f"a8iii/b{bits}/scale"] = np.array(ss, np.float32)
        out[f"a8iii/b{bits}/zp"] = np.array(zs, np.float32)
    # quantize_vectors (lib.rs:127-146): default config [4,6,8,16], request widths cycled [2, 4].
    tv = rng.uniform(-0.2, 1.2, (10, 48)).astype(np.float32)
    qv, wv = N.quantize_vectors(tv, [4, 6, 8, 16], [2, 4])
    out["qv/x"], out["qv/q"], out["qv/widths"] = tv, qv, wv
    # a5: group-128 weight quantization of a 256x96 block + linear on M=16.
    W = (0.02 * rng.standard_normal((256, 96))).astype(np.float32)
    X = rng.standard_normal((16, 256)).astype(np.float32)
    codes, scales, zps = N.quantize_weights(W, 4, 128)
    out["a5/W"], out["a5/X"] = W, X
    out["a5/codes"], out["a5/scales"], out["a5/zps"] = codes, scales, zps
    out["a5/packed"] = N.pack_bits(codes.ravel(), 4)
    out["a5/Y"] = N.linear_forward(X, N.dequantize_weights(codes, scales, zps, 128))
    for bits in (2, 8):
        c2, s2, z2 = N.quantize_weights(W, bits, 128)
        out[f"a5/b{bits}/codes"], out[f"a5/b{bits}/scales"], out[f"a5/b{bits}/zps"] = c2, s2, z2
    # a10 calibration (calibrate.rs): reference test data + a random stream.
    cal = N.Calibration(10)
    cal.update(np.array([[1, 2, 3], [4, 5, 6]], np.float32))
    s, z = cal.compute_params(8, False)
    out["a10/ref/hist"] = cal.histogram.astype(np.int64)
    out["a10/ref/params_asym8"] = np.array([s, np.float32(z)], np.float32)
    cal2 = N.Calibration(64)
    c_in = [rng.standard_normal(5000).astype(np.float32) * (i + 1) for i in range(3)]
    for i, c in enumerate(c_in):
        out[f"a10/rand/x{i}"] = c
        cal2.update(c)
    out["a10/rand/minmax"] = np.array([cal2.min, cal2.max], np.float32)
    out["a10/rand/hist"] = cal2.histogram.astype(np.int64)
    for bits in (4, 8):
        for sym in (0, 1):
            s, z = cal2.compute_params(bits, bool(sym))
            out[f"a10/rand/params_b{bits}_s{sym}"] = np.array([s, np.float32(z)], np.float32)
    np.savez_compressed(HERE / "golden_v1.npz", **out)
    print(f"wrote {len(out)} arrays to {HERE / 'golden_v1.npz'}")


if __name__ == "__main__":
    main()
