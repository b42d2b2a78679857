"""Measurement-only library selection for the scripts and the lab tests: DLLM_LIB=lab installs the
lab build (lib/libdllm_hip_lab.so), DLLM_LIB=<file> another build of the same ABI.  The product
loader (`_lib.load`) reads no environment variable; this is the one place that does."""
import os


def select(d):
    """d = the imported package (``__graft_entry__.load_package()``); returns it."""
    p = os.environ.get("DLLM_LIB")
    if p:
        d._lib.use(d._lib.LAB_LIB_PATH if p == "lab" else p)
    return d
