"""A/B of library builds on dequantize_tensor (a2) at the C2' size: 8192 x 4096 int4 packed codes ->
f16 and -> f32, and the 4096^3 GEMM as a control; each build in its own subprocess (DLLM_LIB=<file>),
rounds interleaved, 0.2 s warm-up per op, HIP events.  Usage: LIBS=a.so,b.so python scripts/dequant_ab.py"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CODE = r"""
import sys, json, time, torch
sys.path.insert(0, %r)
import __graft_entry__ as g
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
n = 8192 * 4096
x = torch.randn(n, device="cuda")
q, params = d.quantize_tensor(x, 4, packed=True)
def timed(fn, reps=20):
    t0 = time.time()
    while time.time() - t0 < 0.2:
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3
o16 = torch.empty(n, dtype=torch.float16, device="cuda")
o32 = torch.empty(n, dtype=torch.float32, device="cuda")
out = {}
out["deq_f16_us"] = round(timed(lambda: d.dequantize_tensor(q, params, bits=4, packed=True, n=n, out_dtype=torch.float16)), 2)
out["deq_f32_us"] = round(timed(lambda: d.dequantize_tensor(q, params, bits=4, packed=True, n=n, out_dtype=torch.float32)), 2)
y = d.dequantize_tensor(q, params, bits=4, packed=True, n=n, out_dtype=torch.float32)
out["hash"] = int(y.view(torch.int32).to(torch.int64).sum().item()) %% 1000003
print(json.dumps(out))
""" % str(ROOT)
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for lib in os.environ["LIBS"].split(","):
        env = dict(os.environ, DLLM_LIB=str((ROOT / lib).resolve()))
        r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"lib": lib, "round": rnd, **(json.loads(line[-1]) if line else {"error": r.stderr[-400:]})}),
              flush=True)
