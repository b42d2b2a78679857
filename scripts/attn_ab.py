"""A/B of library builds on config C4's dequant-attention (S 8192, 32 heads x 128, int4 KV): each
build in its own subprocess (DLLM_LIB=<file>), rounds interleaved, HIP events, ms per call.
Usage: LIBS=a.so,b.so python scripts/attn_ab.py   (measurement only)."""
import json, os, subprocess, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
CODE = r"""
import sys, json, torch
sys.path.insert(0, %r)
import __graft_entry__ as g
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
S, H, D = 8192, 32, 128
torch.manual_seed(0)
K = torch.randn(S, H, D, device='cuda'); V = torch.randn(S, H, D, device='cuda'); Q = torch.randn(S, H, D, device='cuda').half()
e = d.QuantizedKVCacheEntry.new(K, V, 4)
import time
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    for _ in range(3): O = d.kv_attention(Q, e.keys, e.values)
    torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10): d.kv_attention(Q, e.keys, e.values)
b.record(); torch.cuda.synchronize()
print(json.dumps({"ms": round(a.elapsed_time(b) / 10, 3), "checksum": float(O.float().abs().sum())}))
""" % str(ROOT)
libs = os.environ["LIBS"].split(",")
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for lib in libs:
        env = dict(os.environ, DLLM_LIB=str((ROOT / lib).resolve()))
        out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"lib": lib, "round": rnd, **(json.loads(line[-1]) if line else {"error": out.stderr[-300:]})}), flush=True)
