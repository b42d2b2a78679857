"""Diffusion-step ops on the CPU: the C oracle against the numpy
restatement, the committed golden vectors and the reference's own doc-test assertion; the
product's host-side schedule / coefficient entry points (libdllm_hip.so, no GPU needed for
these) against the oracle bit for bit; error behaviour of the reference's panics."""
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden" / "diffusion_v1.npz"


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def test_reference_doctest_linear_schedule(orc):
    """diffuse-llm-rs/src/lib.rs:509-529 doc example: len 1000, betas[0] >= 1e-4, betas[999] <= 0.02."""
    b = orc.beta_schedule(orc.BETA_LINEAR, 1000, 0.0001, 0.02)
    assert b.size == 1000 and b[0] >= np.float32(0.0001) and b[999] <= np.float32(0.02)


@pytest.mark.parametrize("T", [1, 2, 7, 1000])
def test_schedules_oracle_vs_numpy(orc, onp, T):
    for k in (0, 1):   # linear / quadratic: bit-exact (NaN at T = 1 is 0/0 in both)
        a, b = orc.beta_schedule(k, T), onp.beta_schedule(k, T)
        assert np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(bits(a)[~np.isnan(a)], bits(b)[~np.isnan(b)])
    # cosine: the oracle calls glibc cosf (what Rust's f32::cos calls on Linux); numpy's is a
    # correctly rounded cos, so single-ulp cos differences are amplified by 1 - f_t / f_0.
    a, b = orc.beta_schedule(2, T), onp.beta_schedule(2, T)
    assert np.allclose(a, b, rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("inclusive", [0, 1])
def test_alpha_bars_and_coeffs_oracle_vs_numpy(orc, onp, inclusive):
    b = orc.beta_schedule(0, 1000)
    a1, ab1 = orc.alpha_bars(b, inclusive)
    a2, ab2 = onp.alpha_bars(b, inclusive)
    assert np.array_equal(bits(a1), bits(a2)) and np.array_equal(bits(ab1), bits(ab2))
    t = np.array([999, 998, 500, 3, 2, 1, 0, 5000])   # 5000: clamped to T-1 (lib.rs:1175)
    c1, c2 = orc.p_sample_coeffs(b, t, inclusive), onp.p_sample_coeffs(b, t, inclusive)
    same = (bits(c1) == bits(c2)) | (np.isnan(c1) & np.isnan(c2))
    assert same.all()
    assert np.array_equal(bits(orc.add_noise_coeffs(b, t, inclusive)), bits(onp.add_noise_coeffs(b, t, inclusive)))


def test_exclusive_cumprod_last_step_divides_by_zero(orc):
    """The reference's p_sample at t = 0 (exclusive alpha-bar: 1 - alpha_bar[0] = 0): c1 = inf,
    c2 = std = NaN -- reproduced, not repaired; the inclusive (p_losses) form is finite."""
    b = orc.beta_schedule(0, 1000)
    c = orc.p_sample_coeffs(b, [0], inclusive=False)[0]
    assert np.isinf(c[0]) and np.isnan(c[1]) and np.isnan(c[2])
    assert np.isfinite(orc.p_sample_coeffs(b, [0], inclusive=True)).all()


def test_literal_alphas_mode(orc, onp):
    """lib.rs:1191 full-length `alphas` broadcast row-wise when batch == num_timesteps."""
    b = orc.beta_schedule(0, 8, 0.01, 0.2)
    t = np.array([7, 6, 5, 4, 3, 2, 1, 1])
    lit = orc.p_sample_coeffs(b, t, inclusive=True, literal_alphas=True)
    assert np.array_equal(bits(lit), bits(onp.p_sample_coeffs(b, t, True, True)))
    per = orc.p_sample_coeffs(b, t, inclusive=True)
    assert np.array_equal(bits(lit[:, 0]), bits(per[:, 0])) and not np.array_equal(lit[:, 1], per[:, 1])
    with pytest.raises(orc.OracleError):
        orc.p_sample_coeffs(b, t[:5], inclusive=True, literal_alphas=True)


@pytest.mark.parametrize("seed,offset,n", [(0, 0, 1000), (1234, 4, 4099), (2**63 + 7, 1 << 40, 77)])
def test_randn_oracle_vs_numpy(orc, onp, seed, offset, n):
    a, b = orc.randn(seed, offset, n), onp.randn(seed, offset, n)
    assert np.array_equal(bits(a), bits(b))
    # stream property: a window is a slice of a longer draw
    assert np.array_equal(bits(orc.randn(seed, offset + 8, n - 8)), bits(a[8:]))


def test_randn_distribution(orc):
    z = orc.randn(42, 0, 1 << 20)
    assert abs(z.mean()) < 5e-3 and abs(z.var() - 1.0) < 5e-3
    # Kolmogorov-Smirnov against N(0, 1)
    from scipy import stats
    assert stats.kstest(z[:200000], "norm").pvalue > 1e-3
    assert np.isfinite(z).all() and np.abs(z).max() < 7.0


def test_golden_vectors(orc, onp):
    g = np.load(GOLD)
    for k, name in ((0, "linear"), (1, "quadratic"), (2, "cosine")):
        assert np.array_equal(bits(orc.beta_schedule(k, 1000)), bits(g[f"betas_{name}"])), name
    t = g["timesteps"]
    for tag, inc in (("excl", 0), ("incl", 1)):
        c = orc.p_sample_coeffs(g["betas_linear"], t, inc)
        ref = g[f"psample_coef_{tag}"]
        assert ((bits(c) == bits(ref)) | (np.isnan(c) & np.isnan(ref))).all()
        assert np.array_equal(bits(orc.add_noise_coeffs(g["betas_linear"], t, inc)), bits(g[f"addnoise_coef_{tag}"]))
    assert np.array_equal(bits(orc.randn(1234, 0, 4099)), bits(g["randn_seed1234"]))
    nz = orc.randn(99, 0, 6 * 64).reshape(6, 64)
    assert np.array_equal(bits(onp.p_sample(g["ps_x"], g["ps_eps"], nz, g["psample_coef_incl"])), bits(g["ps_out_incl"]))
    assert np.array_equal(bits(onp.add_noise(g["ps_x"], nz, g["addnoise_coef_incl"])), bits(g["an_out_incl"]))


# ---- product host entry points (no GPU touched) -------------------------------------------------

@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    return g.load_package()._lib.load()


def _ptr(a):
    import ctypes as C
    return C.c_void_p(a.ctypes.data)


@pytest.mark.parametrize("kind", [0, 1, 2])
@pytest.mark.parametrize("T", [1, 50, 1000])
def test_product_schedule_matches_oracle(lib, orc, kind, T):
    out = np.zeros(T, np.float32)
    assert lib.dllm_beta_schedule(kind, T, 0.0001, 0.02, _ptr(out)) == 0
    ref = orc.beta_schedule(kind, T)
    assert ((bits(out) == bits(ref)) | (np.isnan(out) & np.isnan(ref))).all()


@pytest.mark.parametrize("cumprod", [0, 1])
def test_product_coeffs_match_oracle(lib, orc, cumprod):
    import ctypes as C
    b = orc.beta_schedule(0, 1000)
    a, ab = np.zeros_like(b), np.zeros_like(b)
    assert lib.dllm_alpha_bars(_ptr(b), b.size, cumprod, _ptr(a), _ptr(ab)) == 0
    ra, rab = orc.alpha_bars(b, cumprod)
    assert np.array_equal(bits(a), bits(ra)) and np.array_equal(bits(ab), bits(rab))
    t = np.array([999, 500, 1, 0, 4000], np.uint64)
    coef = np.zeros((t.size, 3), np.float32)
    flag = C.c_int(-1)
    assert lib.dllm_p_sample_coeffs(_ptr(b), b.size, cumprod, 0, _ptr(t), t.size, _ptr(coef), C.byref(flag)) == 0
    ref = orc.p_sample_coeffs(b, t, cumprod)
    assert ((bits(coef) == bits(ref)) | (np.isnan(coef) & np.isnan(ref))).all() and flag.value == 1
    an = np.zeros((t.size, 2), np.float32)
    assert lib.dllm_add_noise_coeffs(_ptr(b), b.size, cumprod, _ptr(t), t.size, _ptr(an)) == 0
    assert np.array_equal(bits(an), bits(orc.add_noise_coeffs(b, t, cumprod)))


def test_product_coeff_errors(lib):
    import ctypes as C
    b = np.zeros(4, np.float32)
    t = np.zeros(2, np.uint64)
    coef = np.zeros((2, 3), np.float32)
    flag = C.c_int(0)
    assert lib.dllm_p_sample_coeffs(_ptr(b), 0, 0, 0, _ptr(t), 2, _ptr(coef), C.byref(flag)) == 1   # T == 0
    assert lib.dllm_p_sample_coeffs(_ptr(b), 4, 0, 1, _ptr(t), 2, _ptr(coef), C.byref(flag)) == 1   # literal, B != T
    assert lib.dllm_p_sample_coeffs(_ptr(b), 4, 7, 0, _ptr(t), 2, _ptr(coef), C.byref(flag)) == 1   # bad cumprod
    assert lib.dllm_beta_schedule(9, 4, 0.1, 0.2, _ptr(b)) == 1
    assert lib.dllm_p_sample_coeffs(_ptr(b), 4, 0, 0, _ptr(t), 2, _ptr(coef), C.byref(flag)) == 0 and flag.value == 0


def test_progressive_bits_sequence(orc):
    """Progressive decode precision (lib.rs:890-903, on by default: QuantizationConfig::default,
    lib.rs:96-104) for the C5 schedule of 50 steps: prefill while t > 25, then the target width is
    2 at t = 25, 1 for t = 24..13 and 0 for t <= 12 (the saturating `as u8` of a negative f32)."""
    seq = [orc.progressive_bits(4, 2, 50, t) for t in range(25, -1, -1)]
    assert seq == [2] + [1] * 12 + [0] * 13


def test_progressive_bits_product_matches_oracle(dllm, orc):
    """The product's host-side target-width arithmetic equals the oracle's restatement for every
    (num_steps, t) up to 80 steps and several (decode, min) widths, including num_steps = 1
    (progress = 1/0 = inf, so the f32 expression is NaN -> 0)."""
    for ns in range(1, 81):
        for t in range(ns):
            for db, mb in ((4, 2), (8, 1), (3, 3), (2, 4), (8, 0)):
                cfg = dllm.DiffusionConfig(decode_bits=db, min_decode_bits=mb)
                assert dllm.diffusion.progressive_bits(cfg, ns, t) == orc.progressive_bits(db, mb, ns, t), (ns, t, db, mb)
    assert dllm.DiffusionConfig().progressive_precision is True


def test_kv_cache_ref_zero_bits_hands_out_f32(orc):
    """The oracle's KVCacheEntry restatement: once progressive precision drives decode bits to 0
    the decode copy is None and get_keys returns the f32 keys (lib.rs:190-197); no
    quantize_tensor(.., 0) is ever made (the `> 0` guards of lib.rs:230, :262)."""
    rng = np.random.default_rng(2)
    K = rng.standard_normal((1, 16, 32)).astype(np.float32)
    e = orc.KVCacheEntryRef(K, 2 * K, 8, 4)
    widths = []
    for t in range(9, -1, -1):
        k, v = orc.sample_kv_step(e, t, 10, 4, 2)
        widths.append(e.decode_quant_bits if not e.is_prefill_phase else e.prefill_quant_bits)
        if not e.is_prefill_phase and e.decode_quant_bits == 0:
            assert np.array_equal(k, K) and np.array_equal(v, 2 * K)
    assert widths == [8, 8, 8, 8, 2, 1, 1, 0, 0, 0]
