"""CPU suite: the C-ABI library loads, exports every symbol include/dllm_quant.h declares, and its
host-side argument checks and host arithmetic behave like the reference (no GPU work here)."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "dllm_quant.h"
LAB_HEADER = ROOT / "include" / "dllm_quant_lab.h"   # the lab build's extra entry points only


def declared_symbols(lab=False):
    """Symbols of the product header; ``lab``: plus those of the lab-only header."""
    text = "".join(re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
                   for h in ((HEADER, LAB_HEADER) if lab else (HEADER,)))
    return sorted(set(re.findall(r"\b(dllm_\w+)\s*\(", text)))


def test_product_header_declares_no_lab_entry_point():
    """The product header is the product ABI only: no lab section, no lab entry point."""
    text = HEADER.read_text()
    assert "DLLM_LAB" not in text and "set_kernel_variant" not in text
    assert declared_symbols(lab=True) != declared_symbols()


def test_header_symbols_exported(dllm):
    lib = dllm._lib.load()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in dllm_quant.h but not exported"
    assert set(syms) == set(dllm._lib.SIGNATURES), "ctypes signature table out of sync with the header"
    lab_only = set(declared_symbols(lab=True)) - set(syms)
    assert lab_only == set(dllm._lib.LAB_SIGNATURES)
    for s in lab_only:   # the product library carries no A/B knobs
        assert not hasattr(lib, s), f"{s} is lab-only but the product library exports it"


def test_product_library_has_no_lab_switches(dllm):
    """The product library reads no environment on its compute paths: the A/B schedules and ablation
    masks (DLLM_ATTN_LAB, DLLM_LAB_HORNER128, ...) exist only in the lab build."""
    so = dllm._lib.LIB_PATH.read_bytes()
    for knob in (b"DLLM_ATTN_LAB", b"DLLM_LAB_HORNER128", b"DLLM_QUANT_GENERIC"):
        assert knob not in so, knob
    import subprocess
    undef = subprocess.run(["nm", "-D", "--undefined-only", str(dllm._lib.LIB_PATH)], capture_output=True,
                           text=True).stdout.split()
    assert "getenv" not in undef and "getenv@GLIBC_2.2.5" not in undef, "the product library calls getenv"


def test_library_is_gfx950(dllm):
    so = dllm._lib.LIB_PATH.read_bytes()
    assert b"gfx950" in so, "libdllm_hip.so carries no gfx950 code object"


def test_version(dllm):
    assert b"gfx950" in dllm._lib.load().dllm_version()


def test_invalid_bits_is_invalid_params(dllm):
    """quantization.rs:39 assert!((1..=8).contains(&bits)) -> InvalidParams, checked before any launch."""
    L = dllm._lib.load()
    for bits in (0, 9, 16):
        assert L.dllm_quantize_tensor(None, 0, bits, 0, None, None, None, 0, None) == dllm._lib.ERR_INVALID_PARAMS
        assert b"between 1 and 8" in L.dllm_last_error()
    assert L.dllm_pack(None, 4, 0, None, None) == dllm._lib.ERR_INVALID_PARAMS
    assert L.dllm_bit_quantize(None, 4, 31, 1.0, 0.0, None, None) == dllm._lib.ERR_INVALID_PARAMS
    assert L.dllm_default_quantize(None, 4, 7, 1.0, 0, None, None) == dllm._lib.ERR_UNSUPPORTED


def test_quantize_vectors_index_panic(dllm):
    """prefill-kvquant-rs/lib.rs:133: quantizers[bits/2] out of bounds -> InvalidParams, no launch."""
    L = dllm._lib.load()
    cfg = np.array([4, 6, 8, 16], np.uint8)
    req = np.array([8], np.uint8)
    out_bits = np.zeros(2, np.uint8)
    rc = L.dllm_quantize_vectors(None, 2, 8, cfg.ctypes.data, 4, req.ctypes.data, 1, None, out_bits.ctypes.data,
                                 None)
    assert rc == dllm._lib.ERR_INVALID_PARAMS and b"out of bounds" in L.dllm_last_error()
    # empty request list: zip with an empty cycle yields nothing (lib.rs:132)
    assert L.dllm_quantize_vectors(None, 2, 8, cfg.ctypes.data, 4, None, 0, None, None, None) == 0


def test_linear_shape_checks(dllm):
    L = dllm._lib.load()
    h = C.c_void_p()
    dummy = C.c_void_p(16)
    assert L.dllm_linear_create(dummy, None, 100, 64, 4, 128, C.byref(h), None) == dllm._lib.ERR_SHAPE_MISMATCH
    assert L.dllm_linear_create(dummy, None, 128, 64, 3, 128, C.byref(h), None) == dllm._lib.ERR_UNSUPPORTED
    assert L.dllm_linear_create(dummy, None, 128, 64, 4, 100, C.byref(h), None) == dllm._lib.ERR_INVALID_PARAMS


def test_compression_ratio_matches_oracle(dllm, orc):
    L = dllm._lib.load()
    for numel, ln, bits in [(4, 4, 4), (1024, 1024, 8), (33, 33, 3), (7, 7, 1), (8192 * 4096, 8192 * 4096, 4)]:
        assert L.dllm_compression_ratio(numel, ln, bits) == orc.lib().orc_compression_ratio(numel, ln, bits)
        assert L.dllm_packed_bytes(ln, bits) == orc.lib().orc_packed_bytes(ln, bits)


def test_calib_compute_params_matches_oracle(dllm, onp):
    """calibrate.rs:72-110 host arithmetic, bit-exact with the numpy restatement."""
    L = dllm._lib.load()
    rng = np.random.default_rng(3)
    for _ in range(200):
        mn, mx = np.sort(rng.standard_normal(2).astype(np.float32) * 10)
        for bits in (2, 4, 8):
            for sym in (0, 1):
                cal = onp.Calibration(4)
                cal.min, cal.max, cal.total_samples = np.float32(mn), np.float32(mx), 1
                es, ez = cal.compute_params(bits, bool(sym))
                s, z = C.c_float(), C.c_int32()
                assert L.dllm_calib_compute_params(float(mn), float(mx), 1, bits, sym, C.byref(s), C.byref(z)) == 0
                assert np.float32(s.value) == np.float32(es) and z.value == ez
    s, z = C.c_float(), C.c_int32()
    assert L.dllm_calib_compute_params(0.0, 1.0, 0, 8, 0, C.byref(s), C.byref(z)) == dllm._lib.ERR_CALIBRATION_REQUIRED
