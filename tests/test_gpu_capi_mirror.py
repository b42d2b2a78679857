"""The C-ABI export check (tests/test_capi.py) and the f3 wire-format parity (tests/test_serde_capi.py)
again under ``-m gpu``, so the round-end suite on the GPU box -- which runs only ``-m gpu`` -- covers
them too.  Each test here is the CPU suite's test function itself, wrapped with the gpu marker; the
CPU suite keeps running the originals."""
import functools

import pytest

from tests import test_capi as _capi
from tests import test_serde_capi as _serde
from tests.test_serde_capi import lib, ref  # noqa: F401  (the module's fixtures)


def _mirror(fn):
    @functools.wraps(fn)
    def wrapped(*args, **kwargs):
        return fn(*args, **kwargs)
    wrapped.pytestmark = list(getattr(fn, "pytestmark", [])) + [pytest.mark.gpu]
    return wrapped


for _mod, _tag in ((_capi, "capi"), (_serde, "serde")):
    for _name in dir(_mod):
        if _name.startswith("test_") and callable(getattr(_mod, _name)):
            globals()[f"test_gpu_{_tag}_{_name[5:]}"] = _mirror(getattr(_mod, _name))
