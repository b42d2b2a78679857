"""A/B of library builds of the same ABI on the int4-g128 GEMM (default EXACT precision): each build
in its own subprocess (DLLM_LIB=<file>), rounds interleaved, HIP events around 20 launches, median
over rounds; a bit-level hash of Y shows whether two builds compute the same bits.
Usage: LIBS=a.so,b.so [SHAPES=4096:4096,2048:4096] [AB_BITS=4|2] python scripts/gemm_ab.py   (measurement only)."""
import json, os, subprocess, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
CODE = r"""
import sys, json, torch
sys.path.insert(0, %r)
import __graft_entry__ as g
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
K = 4096
out = {}
for sh in %r.split(","):
    M, N = (int(v) for v in sh.split(":"))
    torch.manual_seed(0)
    W = 0.02 * torch.randn(K, N, device="cuda")
    lin = d.QuantLinear.from_weight(W, None, int(__import__("os").environ.get("AB_BITS", "4")), 128)
    X = torch.randn(M, K, device="cuda").half()
    Y = torch.empty(M, N, dtype=torch.float16, device="cuda")
    for _ in range(30): lin(X, out=Y)
    torch.cuda.synchronize()
    import time as _t
    t0 = _t.perf_counter()
    while _t.perf_counter() - t0 < %r:   # PREWARM_MS: the clocks' steady state before timing
        for _ in range(20): lin(X, out=Y)
        torch.cuda.synchronize()
    ts = []
    for r in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20): lin(X, out=Y)
        b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 20 * 1e3)
    ts.sort()
    h = int(Y.view(torch.int16).to(torch.int64).mul(torch.arange(Y.numel(), device="cuda").view(M, N) %% 65521 + 1).sum())
    out[sh] = {"us": round(ts[2], 2), "us_min": round(ts[0], 2), "tflops": round(2 * M * N * K / ts[2] / 1e6, 1), "yhash": h}
    lin.close()
print(json.dumps(out))
"""
libs = os.environ["LIBS"].split(",")
shapes = os.environ.get("SHAPES", "4096:4096,2048:4096,4096:1024,4096:512")
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for lib in libs:
        env = dict(os.environ, DLLM_LIB=str((ROOT / lib).resolve()))
        res = subprocess.run([sys.executable, "-c", CODE % (str(ROOT), shapes, float(os.environ.get("PREWARM_MS", "0")) / 1e3)], env=env, capture_output=True, text=True,
                             timeout=300)
        line = [l for l in res.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"lib": lib, "round": rnd, **(json.loads(line[-1]) if line else {"error": res.stderr[-400:]})}),
              flush=True)
