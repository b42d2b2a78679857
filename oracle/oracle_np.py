"""Independent numpy restatement of the reference's quantized hot path.

TEST INFRASTRUCTURE ONLY.  Written separately from ``dllm_oracle.c`` so the two restatements can
cross-check each other bit for bit.  Used by ``tests/golden/make_golden.py``
to produce the committed golden vectors and by the CPU test-suite; never imported by the product.

All arithmetic is float32 with one rounding per operation (numpy never fuses), matching Rust f32.
Each function cites the Rust code it restates (paths relative to the reference root).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def rs_round(x: np.ndarray) -> np.ndarray:
    """Rust ``f32::round``: half away from zero (numpy's ``round`` is half-to-even)."""
    x = np.asarray(x, dtype=F32)
    t = np.trunc(x)
    with np.errstate(invalid="ignore"):
        frac = np.abs(x - t)
        up = frac >= F32(0.5)
    return np.where(up, t + np.sign(x).astype(F32), t).astype(F32)


def rs_as_u8(x: np.ndarray) -> np.ndarray:
    """Rust ``f as u8``: saturating, truncating, NaN -> 0."""
    x = np.asarray(x, dtype=F32)
    with np.errstate(invalid="ignore"):
        out = np.where(np.isnan(x) | (x <= 0), F32(0), np.where(x >= 255, F32(255), np.trunc(x)))
    return out.astype(np.uint8)


def rs_as_i32(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.float64)  # exact widening
    with np.errstate(invalid="ignore"):
        out = np.where(np.isnan(x), 0.0, np.clip(np.trunc(x), -2147483648.0, 2147483647.0))
    return out.astype(np.int64)


def rs_clamp(x: np.ndarray, lo: float, hi: float) -> np.ndarray:
    """Rust ``f32::clamp``: NaN passes through."""
    x = np.asarray(x, dtype=F32)
    with np.errstate(invalid="ignore"):
        x = np.where(x < F32(lo), F32(lo), x)
        x = np.where(x > F32(hi), F32(hi), x)
    return x.astype(F32)


def fold_max(x: np.ndarray) -> F32:
    return F32(np.fmax.reduce(np.asarray(x, F32).ravel(), initial=-np.inf))


def fold_min(x: np.ndarray) -> F32:
    return F32(np.fmin.reduce(np.asarray(x, F32).ravel(), initial=np.inf))


# ---- a1 / a2: diffuse-llm-rs/src/quantization.rs -------------------------------------------

def params_from_extremes(mx, mn, bits: int):
    """quantization.rs:49-56 -> (scale f32, zero_point f32) from the folds of :41-46."""
    q_min, q_max = F32(0.0), F32(float(1 << bits) - 1.0)
    with np.errstate(all="ignore"):
        scale = F32((F32(mx) - F32(mn)) / (q_max - q_min))
        if scale == F32(0.0):
            scale = F32(1.0)
        zpf = F32(q_min - F32(F32(mn) / scale))
        zp = rs_as_u8(rs_round(rs_clamp(np.array([zpf], F32), q_min, q_max)))[0]
    return F32(scale), F32(zp)


def quantize_with_params(data: np.ndarray, bits: int, scale, zp) -> np.ndarray:
    """quantization.rs:59-65: the code map once (scale, zero_point) are known."""
    x = np.asarray(data, dtype=F32).ravel()
    with np.errstate(all="ignore"):
        v = (x / F32(scale)).astype(F32)
        v = (v + F32(zp)).astype(F32)
        return np.clip(rs_as_i32(rs_round(v)), 0, (1 << bits) - 1).astype(np.uint8)


def quantize_tensor(data: np.ndarray, bits: int):
    """quantization.rs:38-68 -> (codes u8, scale f32, zero_point f32)."""
    if not 1 <= bits <= 8:
        raise ValueError("Bits must be between 1 and 8")  # :39 assert!
    x = np.asarray(data, dtype=F32).ravel()
    scale, zp = params_from_extremes(fold_max(x), fold_min(x), bits)
    return quantize_with_params(x, bits, scale, zp), scale, zp


def dequantize_tensor(q: np.ndarray, scale, zero_point) -> np.ndarray:
    """quantization.rs:81-85."""
    d = (np.asarray(q).astype(F32) - F32(zero_point)).astype(F32)
    return (d * F32(scale)).astype(F32)


def compression_ratio(numel: int, length: int, bits: int) -> float:
    """quantization.rs:120-124."""
    return float(F32(numel * 4) / F32((length * bits + 7) // 8))


# ---- a6: build-defined LSB-first packing ----------------------------------------------------

def pack_bits(codes: np.ndarray, bits: int) -> np.ndarray:
    codes = np.asarray(codes, np.uint8).ravel().astype(np.uint64) & ((1 << bits) - 1)
    n = codes.size
    nbytes = (n * bits + 7) // 8
    bitpos = np.arange(n, dtype=np.uint64) * bits
    out = np.zeros(nbytes + 1, dtype=np.uint64)
    lo = (codes << (bitpos & 7)) & 0xFF
    hi = (codes << (bitpos & 7)) >> 8
    np.bitwise_or.at(out, (bitpos >> 3).astype(np.int64), lo)
    np.bitwise_or.at(out, ((bitpos >> 3) + 1).astype(np.int64), hi)
    return out[:nbytes].astype(np.uint8)


def unpack_bits(packed: np.ndarray, n: int, bits: int) -> np.ndarray:
    p = np.concatenate([np.asarray(packed, np.uint8).ravel(), np.zeros(1, np.uint8)]).astype(np.uint64)
    bitpos = np.arange(n, dtype=np.uint64) * bits
    idx = (bitpos >> 3).astype(np.int64)
    v = p[idx] | (p[idx + 1] << 8)
    return ((v >> (bitpos & 7)) & ((1 << bits) - 1)).astype(np.uint8)


# ---- a4: quantization/src/quantize.rs DefaultQuantizer -------------------------------------

QTYPE_RANGE = {0: (-128.0, 127.0), 1: (-8.0, 7.0), 2: (0.0, 1.0), 3: (-127.0, 127.0)}  # :139-144
QTYPE_BITS = {0: 8, 1: 4, 2: 1, 3: 8}  # :69-78


def default_quantize(x: np.ndarray, qtype: int, scale=1.0, zero_point=0) -> np.ndarray:
    """quantize.rs:111-154 (quantize_value then ``q as u8``)."""
    lo, hi = QTYPE_RANGE[qtype]
    x = np.asarray(x, F32).ravel()
    with np.errstate(all="ignore"):
        v = (x / F32(scale)).astype(F32)
        v = (v + F32(zero_point)).astype(F32)
        v = np.fmin(np.fmax(v, F32(lo)), F32(hi)).astype(F32)
    return rs_as_u8(rs_round(v))


def default_dequantize(q: np.ndarray, scale=1.0, zero_point=0) -> np.ndarray:
    """quantize.rs:172-184."""
    return dequantize_tensor(q, F32(scale), F32(zero_point))


# ---- a8-ii: prefill-kvquant-rs/lib.rs BitQuantizer ----------------------------------------

def bit_quantize(x: np.ndarray, bits: int, scale, zero_point) -> np.ndarray:
    """lib.rs:40-46 (truncation, no rounding)."""
    max_val = F32((1 << bits) - 1)
    with np.errstate(all="ignore"):
        s = ((np.asarray(x, F32).ravel() - F32(zero_point)).astype(F32) / F32(scale)).astype(F32)
    return rs_as_u8(rs_clamp(s, F32(0.0), max_val))


def bit_dequantize(q: np.ndarray, scale, zero_point) -> np.ndarray:
    """lib.rs:48-52."""
    p = (np.asarray(q).astype(F32) * F32(scale)).astype(F32)
    return (p + F32(zero_point)).astype(F32)


def prefill_scale(cfg_bits: int) -> F32:
    """lib.rs:104-108."""
    return F32(F32(1.0) / F32((1 << cfg_bits) - 1))


def quantize_vectors(x: np.ndarray, cfg_bits, req_bits):
    """lib.rs:127-146 over rows of x [rows, dim]."""
    out, widths = [], []
    if len(req_bits) == 0:
        return np.zeros((0, x.shape[1]), np.uint8), np.zeros(0, np.uint8)
    for r in range(x.shape[0]):
        b = int(req_bits[r % len(req_bits)])
        qi = b // 2
        if qi >= len(cfg_bits):
            raise IndexError("quantizers[bits / 2] out of bounds")
        out.append(bit_quantize(x[r], b, prefill_scale(int(cfg_bits[qi])), 0.0))
        widths.append(b)
    return np.stack(out), np.array(widths, np.uint8)


# ---- a8-iii: diffusion_prefill/src/prefill_kv.rs compress_vector ---------------------------

def compress_vector(x: np.ndarray, bits: int):
    """prefill_kv.rs:104-121."""
    x = np.asarray(x, F32).ravel()
    mn, mx = fold_min(x), fold_max(x)
    levels = F32((1 << bits) - 1)
    with np.errstate(all="ignore"):
        scale = F32((mx - mn) / levels)
        s = ((x - mn).astype(F32) / scale).astype(F32)
    return rs_as_u8(rs_clamp(s, F32(0.0), levels)), scale, F32(mn)


# ---- a10: quantization/src/calibrate.rs ------------------------------------------------------

class Calibration:
    """calibrate.rs:19-110."""

    F32_MAX = F32(3.40282347e38)

    def __init__(self, num_bins: int):
        self.min, self.max = self.F32_MAX, -self.F32_MAX
        self.num_bins = num_bins
        self.histogram = np.zeros(num_bins, np.uint64)
        self.total_samples = 0

    def update(self, data: np.ndarray):
        x = np.asarray(data, F32).ravel()
        mn = F32(np.fmin.reduce(x, initial=self.F32_MAX))
        mx = F32(np.fmax.reduce(x, initial=-self.F32_MAX))
        self.min, self.max = F32(np.fmin(self.min, mn)), F32(np.fmax(self.max, mx))
        self.total_samples += x.size
        if self.max > self.min:
            bw = F32((self.max - self.min) / F32(self.num_bins))
            sel = x[(x >= self.min) & (x <= self.max)]
            b = np.floor(((sel - self.min).astype(F32) / bw).astype(F32))
            b = np.minimum(np.where(b <= 0, 0, b).astype(np.int64), self.num_bins - 1)
            np.add.at(self.histogram, b, 1)

    def compute_params(self, bits: int, symmetric: bool):
        if self.total_samples == 0:
            raise RuntimeError("CalibrationRequired")
        nl = F32(2 ** bits)
        rng = F32(self.max - self.min)
        if rng <= F32(1.1920929e-07):
            return F32(1.0), 0
        if symmetric:
            ma = F32(max(abs(self.max), abs(self.min)))
            scale = F32(F32(ma * F32(2.0)) / F32(nl - F32(1.0)))
            zp = int(rs_as_i32(np.array([F32(nl / F32(2.0)) - F32(1.0)], F32))[0])
        else:
            scale = F32(rng / F32(nl - F32(1.0)))
            zp = int(rs_as_i32(rs_round(np.array([F32(-self.min) / scale], F32)))[0])
        return scale, zp


# ---- 8f rank 4: AdaptiveQuantizer (diffuse-llm-rs/src/quantization.rs:178-235) --------------

class AdaptiveQuantizer:
    """quantization.rs:178-235; the CKMS q = 0.0 / 1.0 queries (:209-210) as exact extremes."""

    def __init__(self, bits: int, target_ratio: float = 4.0):
        self.bits, self.target_ratio = bits, target_ratio
        self.min, self.max, self.count = F32(np.inf), F32(-np.inf), 0

    def update_stats(self, data):
        x = np.asarray(data, F32).ravel()
        self.min = F32(np.fmin(self.min, fold_min(x)))
        self.max = F32(np.fmax(self.max, fold_max(x)))
        self.count += x.size

    def compute_params(self):
        mn, mx = (self.min, self.max) if self.count else (F32(0.0), F32(1.0))
        q_max = F32(F32(2.0 ** self.bits) - F32(1.0))
        with np.errstate(divide="ignore", invalid="ignore"):
            scale = F32(F32(mx - mn) / q_max)
            zp = rs_clamp(rs_round(np.array([F32(-mn) / scale], F32)), 0.0, q_max)[0]
        return scale, F32(zp)

    def quantize(self, data):
        x = np.asarray(data, F32).ravel()
        scale, zp = self.compute_params()
        hi = int(rs_as_i32(np.array([F32(2.0 ** self.bits) - F32(1.0)], F32))[0])
        with np.errstate(divide="ignore", invalid="ignore"):
            t = ((x / scale).astype(F32) + zp).astype(F32)
        q = np.clip(rs_as_i32(rs_round(t)), 0, hi)
        return (q & 0xFF).astype(np.uint8), scale, zp


# ---- a5: group-wise weight quantization + linear layer --------------------------------------

def quantize_weights(W: np.ndarray, bits: int = 4, group: int = 128):
    """Per (column, K-group) quantize_tensor -> codes [K,N], scales [G,N], zps [G,N]."""
    K, N = W.shape
    G = (K + group - 1) // group
    codes = np.zeros((K, N), np.uint8)
    scales = np.zeros((G, N), F32)
    zps = np.zeros((G, N), np.uint8)
    for g in range(G):
        blk = np.asarray(W[g * group:(g + 1) * group], F32)
        mx = np.fmax.reduce(blk, axis=0, initial=-np.inf).astype(F32)
        mn = np.fmin.reduce(blk, axis=0, initial=np.inf).astype(F32)
        q_max = F32(float(1 << bits) - 1.0)
        with np.errstate(all="ignore"):
            s = ((mx - mn).astype(F32) / q_max).astype(F32)
            s = np.where(s == 0, F32(1.0), s).astype(F32)
            zpf = (F32(0.0) - (mn / s).astype(F32)).astype(F32)
            z = rs_as_u8(rs_round(rs_clamp(zpf, 0.0, q_max)))
            v = (blk / s[None, :]).astype(F32)
            v = (v + z.astype(F32)[None, :]).astype(F32)
        codes[g * group:(g + 1) * group] = np.clip(rs_as_i32(rs_round(v)), 0, (1 << bits) - 1)
        scales[g], zps[g] = s, z
    return codes, scales, zps


def dequantize_weights(codes, scales, zps, group: int = 128) -> np.ndarray:
    K = codes.shape[0]
    g = np.arange(K) // group
    d = (codes.astype(F32) - zps[g].astype(F32)).astype(F32)
    return (d * scales[g]).astype(F32)


def linear_forward(X: np.ndarray, W: np.ndarray, bias=None) -> np.ndarray:
    """diffuse-llm-rs/src/lib.rs:806-813 (accumulated in f64, returned f32)."""
    Y = np.asarray(X, np.float64) @ np.asarray(W, np.float64)
    if bias is not None:
        Y = Y + np.asarray(bias, np.float64)[None, :]
    return Y.astype(F32)


# ---- 8f rank 1: diffusion-step ops (independent numpy restatement of dllm_oracle_diffusion.c) --
# Every intermediate is forced to float32 so each step is one correctly rounded binary32 op.

def beta_schedule(kind: int, T: int, beta_start=0.0001, beta_end=0.02) -> np.ndarray:
    """DiffusionConfig::create_beta_schedule (diffuse-llm-rs/src/lib.rs:554-593).  Cosine uses
    cos in f64 rounded to f32 (a correctly rounded cosf; glibc's cosf may differ by 1 ulp)."""
    bs, be = F32(beta_start), F32(beta_end)
    t = np.arange(T, dtype=F32)
    with np.errstate(all="ignore"):
        if kind == 0:
            return (bs + ((be - bs) * t).astype(F32) / F32(T - 1)).astype(F32)
        if kind == 1:
            tn = (t / F32(T - 1)).astype(F32)
            return (bs + (((be - bs) * tn).astype(F32) * tn).astype(F32)).astype(F32)
        s, pi = F32(0.008), F32(np.pi)
        tn = (t / F32(T)).astype(F32)
        arg = (((((tn + s).astype(F32) / (F32(1.0) + s)).astype(F32) * pi).astype(F32)) / F32(2.0)).astype(F32)
        ft = np.cos(arg.astype(np.float64)).astype(F32)
        ft = (ft * ft).astype(F32)
        a0 = (((s / (F32(1.0) + s)).astype(F32) * pi).astype(F32) / F32(2.0)).astype(F32)
        f0 = F32(np.cos(np.float64(a0)))
        f0 = F32(f0 * f0)
        return np.fmin((F32(1.0) - (ft / f0).astype(F32)).astype(F32), F32(0.999)).astype(F32)


def alpha_bars(betas: np.ndarray, inclusive: bool):
    a = (F32(1.0) - np.asarray(betas, F32)).astype(F32)
    ab = np.empty_like(a)
    state = F32(1.0)
    for i in range(a.size):
        if inclusive:
            state = F32(state * a[i])
            ab[i] = state
        else:
            ab[i] = F32(1.0) if i == 0 else F32(ab[i - 1] * a[i - 1])
    return a, ab


def p_sample_coeffs(betas, t, inclusive=False, literal_alphas=False) -> np.ndarray:
    a, ab = alpha_bars(betas, inclusive)
    T = a.size
    out = np.zeros((len(t), 3), F32)
    with np.errstate(all="ignore"):
        for i, ti in enumerate(t):
            ti = min(int(ti), T - 1)
            abar_t, beta_t = ab[ti], F32(betas[ti])
            alpha = a[i] if literal_alphas else a[ti]
            prev = ab[ti - 1] if ti > 0 else F32(1.0)
            den = F32(F32(1.0) - abar_t)
            out[i, 0] = F32(F32(np.sqrt(prev) * beta_t) / den)
            out[i, 1] = F32(F32(np.sqrt(alpha) * F32(F32(1.0) - prev)) / den)
            out[i, 2] = np.sqrt(F32(F32(F32(F32(1.0) - prev) / den) * beta_t))
    return out


def add_noise_coeffs(betas, t, inclusive=False) -> np.ndarray:
    _, ab = alpha_bars(betas, inclusive)
    T = ab.size
    out = np.zeros((len(t), 2), F32)
    for i, ti in enumerate(t):
        ti = min(int(ti), T - 1)
        out[i] = np.sqrt(ab[ti]), np.sqrt(F32(F32(1.0) - ab[ti]))
    return out


def _philox(ctr_lo, ctr_hi, seed):
    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
    c0 = ctr_lo.astype(np.uint32)
    c1 = ctr_hi.astype(np.uint32)
    c2 = np.zeros_like(c0)
    c3 = np.zeros_like(c0)
    k0, k1 = np.uint32(seed & 0xFFFFFFFF), np.uint32(seed >> 32)
    for _ in range(10):
        p0 = M0 * c0.astype(np.uint64)
        p1 = M1 * c2.astype(np.uint64)
        hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), p0.astype(np.uint32)
        hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), p1.astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def _ln01(u):
    bits = u.view(np.uint32)
    e = ((bits >> np.uint32(23)) & np.uint32(0xFF)).astype(np.int32) - 127
    m = ((bits & np.uint32(0x007FFFFF)) | np.uint32(0x3F800000)).view(F32)
    big = m > F32(float.fromhex("0x1.6a09e6p+0"))
    m = np.where(big, (m * F32(0.5)).astype(F32), m)
    e = e + big.astype(np.int32)
    s = ((m - F32(1.0)).astype(F32) / (m + F32(1.0)).astype(F32)).astype(F32)
    s2 = (s * s).astype(F32)
    p = np.full_like(s, F32(float.fromhex("0x1.3b13b2p-4")))
    for c in ("0x1.745d18p-4", "0x1.c71c72p-4", "0x1.24924ap-3", "0x1.99999ap-3", "0x1.555556p-2"):
        p = (F32(float.fromhex(c)) + (s2 * p).astype(F32)).astype(F32)
    p = (F32(1.0) + (s2 * p).astype(F32)).astype(F32)
    lnm = ((F32(2.0) * s).astype(F32) * p).astype(F32)
    return ((e.astype(F32) * F32(float.fromhex("0x1.62e430p-1"))).astype(F32) + lnm).astype(F32)


def _box_muller(ra, rb):
    u1 = (((ra >> np.uint32(8)) + np.uint32(1)).astype(F32) * F32(2.0 ** -24)).astype(F32)
    u2 = ((rb >> np.uint32(8)).astype(F32) * F32(2.0 ** -24)).astype(F32)
    rad = np.sqrt((F32(-2.0) * _ln01(u1)).astype(F32)).astype(F32)
    v = (u2 * F32(4.0)).astype(F32)
    q = v.astype(np.int32)
    phi = ((v - q.astype(F32)).astype(F32) * F32(float.fromhex("0x1.921fb6p+0"))).astype(F32)
    x2 = (phi * phi).astype(F32)
    sp = (F32(1.0) - (x2 * F32(float.fromhex("0x1.a41a42p-8"))).astype(F32)).astype(F32)
    for c in ("0x1.29e412p-7", "0x1.c71c72p-7", "0x1.861862p-6", "0x1.99999ap-5", "0x1.555556p-3"):
        sp = (F32(1.0) - ((x2 * F32(float.fromhex(c))).astype(F32) * sp).astype(F32)).astype(F32)
    sn = (phi * sp).astype(F32)
    cp = (F32(1.0) - (x2 * F32(float.fromhex("0x1.f07c20p-8"))).astype(F32)).astype(F32)
    for c in ("0x1.6c16c2p-7", "0x1.24924ap-6", "0x1.111112p-5", "0x1.555556p-4", "0x1.0p-1"):
        cp = (F32(1.0) - ((x2 * F32(float.fromhex(c))).astype(F32) * cp).astype(F32)).astype(F32)
    c = np.select([q == 0, q == 1, q == 2], [cp, -sn, -cp], sn).astype(F32)
    s = np.select([q == 0, q == 1, q == 2], [sn, cp, -sn], -cp).astype(F32)
    return (rad * c).astype(F32), (rad * s).astype(F32)


def randn(seed: int, offset: int, n: int) -> np.ndarray:
    e = np.arange(offset, offset + n, dtype=np.uint64)
    blk = e // np.uint64(4)
    c0, c1, c2, c3 = _philox(blk & np.uint64(0xFFFFFFFF), blk >> np.uint64(32), seed)
    z0, z1 = _box_muller(c0, c1)
    z2, z3 = _box_muller(c2, c3)
    lane = (e % np.uint64(4)).astype(np.int64)
    return np.choose(lane, [z0, z1, z2, z3]).astype(F32)


def p_sample(x_t, eps, noise, coef, add_noise=True) -> np.ndarray:
    coef = np.asarray(coef, F32)
    c1, c2, sd = coef[:, 0:1], coef[:, 1:2], coef[:, 2:3]
    with np.errstate(all="ignore"):
        mean = ((c1 * x_t).astype(F32) + (c2 * eps).astype(F32)).astype(F32)
        nz = noise if add_noise else np.zeros_like(x_t)
        return (mean + (sd * nz).astype(F32)).astype(F32)


def add_noise(x0, noise, coef) -> np.ndarray:
    coef = np.asarray(coef, F32)
    return ((x0 * coef[:, 0:1]).astype(F32) + (noise * coef[:, 1:2]).astype(F32)).astype(F32)
