"""Attention ablation timings: runs C4 (S 8192, 32 heads x 128, int4 KV) under each DLLM_ATTN_LAB
mask in a fresh subprocess (the mask is read once per process).  Measurement only."""
import json, os, subprocess, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
CODE = r"""
import sys, json, torch
sys.path.insert(0, %r)
import __graft_entry__ as g
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
S, H, D = 8192, 32, 128
K = torch.randn(S, H, D, device='cuda'); V = torch.randn(S, H, D, device='cuda'); Q = torch.randn(S, H, D, device='cuda').half()
e = d.QuantizedKVCacheEntry.new(K, V, 4)
for _ in range(3): d.kv_attention(Q, e.keys, e.values)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10): d.kv_attention(Q, e.keys, e.values)
b.record(); torch.cuda.synchronize()
print(json.dumps({"ms": round(a.elapsed_time(b) / 10, 3)}))
""" % str(ROOT)
for lab in [int(x) for x in os.environ.get("LABS", "0,1,2,4,8,3,12,15").split(",")]:
    env = dict(os.environ, DLLM_ATTN_LAB=str(lab))
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    print(json.dumps({"lab": lab, **(json.loads(line[-1]) if line else {"error": out.stderr[-300:]})}), flush=True)
