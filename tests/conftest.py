import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "lab: A/B schedules of the lab build (DLLM_LIB=lab); skipped otherwise")


def pytest_collection_modifyitems(config, items):
    import os
    if os.environ.get("DLLM_LIB") == "lab":
        return
    skip = pytest.mark.skip(reason="lab-build schedule (set DLLM_LIB=lab with lib/libdllm_hip_lab.so built)")
    for it in items:
        if "lab" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def orc():
    """The C oracle (parity checker)."""
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def onp():
    from oracle import oracle_np
    return oracle_np


@pytest.fixture(scope="session")
def dllm():
    """The product package (HIP path).  Fails loudly if the library is missing."""
    import __graft_entry__ as g
    mod = g.load_package()
    from scripts import _lab   # DLLM_LIB=lab: the lab tests install the lab build explicitly
    _lab.select(mod)
    mod.load_library()
    return mod


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("-m gpu test run without a visible GPU")
    return torch.device("cuda")
