"""Regenerates tests/golden/diffusion_v1.npz from the C oracle (oracle/dllm_oracle_diffusion.c),
after checking it against the independent numpy restatement (oracle/oracle_np.py).  The arrays
are data (inputs and expected outputs), not reference source.

    python tests/golden/make_golden_diffusion.py
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle as o, oracle_np as n  # noqa: E402


def main():
    g = {}
    for k, name in ((0, "linear"), (1, "quadratic"), (2, "cosine")):
        b = o.beta_schedule(k, 1000)
        if k < 2:
            assert np.array_equal(b.view(np.uint32), n.beta_schedule(k, 1000).view(np.uint32))
        g[f"betas_{name}"] = b
    b = g["betas_linear"]
    t = np.array([999, 700, 500, 2, 1, 0], np.uint64)
    for inc in (0, 1):
        c = o.p_sample_coeffs(b, t, inclusive=inc)
        assert np.array_equal(c.view(np.uint32), n.p_sample_coeffs(b, t, inc).view(np.uint32))
        g[f"psample_coef_{'incl' if inc else 'excl'}"] = c
        g[f"addnoise_coef_{'incl' if inc else 'excl'}"] = o.add_noise_coeffs(b, t, inclusive=inc)
    g["timesteps"] = t
    z = o.randn(1234, 0, 4099)
    assert np.array_equal(z.view(np.uint32), n.randn(1234, 0, 4099).view(np.uint32))
    g["randn_seed1234"] = z
    rng = np.random.default_rng(5)
    x = rng.standard_normal((6, 64)).astype(np.float32)
    eps = rng.standard_normal((6, 64)).astype(np.float32)
    nz = o.randn(99, 0, 6 * 64).reshape(6, 64)
    g["ps_x"], g["ps_eps"] = x, eps
    g["ps_out_incl"] = o.p_sample(x, eps, nz, g["psample_coef_incl"])
    g["an_out_incl"] = o.add_noise(x, nz, g["addnoise_coef_incl"])
    np.savez_compressed(Path(__file__).with_name("diffusion_v1.npz"), **g)
    print("wrote", len(g), "arrays")


if __name__ == "__main__":
    main()
