"""The exact-division identity of the fused quantize kernel (div_scale in
diffusion-llm-rs_amd/csrc/quant_kernels.hip), checked exhaustively on the host: for every
significand of x over two binades and a sample of divisor significands, Markstein's corrected
quotient equals the IEEE quotient Rust computes (quantization.rs:61) bit for bit.  The GPU's
v_fma_f32 / v_mul_f32 are IEEE round-to-nearest like the host's, so the identity carries over;
the a1 parity tests check the device codes against the oracle as well."""
import shutil
import subprocess
from pathlib import Path

import pytest

SRC = Path(__file__).parent / "cpp" / "markstein_check.c"


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_markstein_division_exhaustive(tmp_path):
    exe = tmp_path / "markstein_check"
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", str(SRC), "-o", str(exe), "-lm"],
                   check=True)
    out = subprocess.run([str(exe), "96", "12345"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip() == f"checked {96 << 24} mismatches 0"
