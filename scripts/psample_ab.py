"""A/B of library builds on C5's fused last layer (dllm_linear_forward_psample: int4 g128 GEMM
2048 x 4096 x 4096 + the p_sample epilogue drawing its noise in-lane) and the plain layer of the same
shape: each build in its own subprocess (DLLM_LIB=<file>), rounds interleaved, 300 ms pre-warm, HIP
events over 20 calls.  x_prev must be bit-identical across builds.
Usage: LIBS=a.so,b.so [ROUNDS=3 M=2048] python scripts/psample_ab.py   (measurement only)."""
import json, os, subprocess, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
CODE = r"""
import sys, json, time, torch
sys.path.insert(0, %r)
import __graft_entry__ as g
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
M, dm = %d, 4096
gen = torch.Generator(device="cuda").manual_seed(7)
lin = d.QuantLinear.from_weight((0.5 / 64.0) * torch.randn(dm, dm, device="cuda", generator=gen), None, 4, 128,
                                prefill_only=True)
h = torch.randn(M, dm, device="cuda", generator=gen).half()
x = torch.randn(M, dm, device="cuda", generator=gen)
coef = torch.tensor([[0.9, 0.05, 0.1]], device="cuda")
out = torch.empty_like(x)
y = torch.empty(M, dm, dtype=torch.float16, device="cuda")
res = {}
for name, fn in (("fused", lambda: lin.forward_psample(h, x, coef, M, True, 1, 0, out)), ("plain", lambda: lin(h, out=y))):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(10): fn()
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20): fn()
    b.record(); torch.cuda.synchronize()
    res[name] = round(a.elapsed_time(b) / 20 * 1e3, 2)
res["hash"] = int(out.view(torch.int32).to(torch.int64).sum())
print(json.dumps(res))
"""
libs = os.environ["LIBS"].split(",")
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for lib in libs:
        env = dict(os.environ, DLLM_LIB=str((ROOT / lib).resolve()))
        r = subprocess.run([sys.executable, "-c", CODE % (str(ROOT), int(os.environ.get("M", "2048")))], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"lib": lib, "round": rnd, **(json.loads(line[-1]) if line else {"error": r.stderr[-400:]})}),
              flush=True)
