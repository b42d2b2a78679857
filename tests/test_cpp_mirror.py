"""The C++ host-side mirror (include/dllm_quant.hpp) replays the reference's own #[test]s through
the C-ABI.  CPU: the headers compile as C and C++; GPU: the compiled test program passes."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "cpp" / "test_reference_mirror.cpp"
LIBDIR = ROOT / "diffusion-llm-rs_amd" / "lib"


def test_headers_compile(tmp_path):
    c = tmp_path / "t.c"
    c.write_text('#include "dllm_quant.h"\nint main(void){return dllm_packed_bytes(3, 4) == 2 ? 0 : 1;}\n')
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-fsyntax-only", f"-I{ROOT / 'include'}", str(c)],
                   check=True)
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", f"-I{ROOT / 'include'}", str(SRC)],
                   check=True)


@pytest.mark.gpu
def test_reference_tests_through_cpp_mirror(tmp_path, dllm):
    exe = tmp_path / "mirror"
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{ROOT / 'include'}", str(SRC), f"-L{LIBDIR}", "-ldllm_hip",
                    f"-Wl,-rpath,{LIBDIR}", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout
