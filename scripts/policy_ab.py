"""A/B of the product tile policy against a lab variant over an M-sweep (K = N = 4096 int4 g128,
f16 Y; lab build, one process, interleaved rounds, HIP events; outputs compared bit for bit).
Usage: policy_ab.py <variant> [M ...]"""
import json
import os
import sys
import time
from pathlib import Path
os.environ.setdefault("DLLM_LIB", "lab")
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
var = int(sys.argv[1])
Ms = [int(m) for m in (sys.argv[2:] or ["256", "512", "1024"])]
K = N = 4096
W = 0.02 * torch.randn(K, N, device="cuda")
lp = d.QuantLinear.from_weight(W, None, 4, 128)
lv = d.QuantLinear.from_weight(W, None, 4, 128)
lv.set_kernel_variant(var)
out = []
for M in Ms:
    X = torch.randn(M, K, device="cuda").half()
    Y = torch.empty(M, N, device="cuda", dtype=torch.float16)
    yp, yv = lp(X, out_dtype=torch.float32), lv(X, out_dtype=torch.float32)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for lin in (lp, lv):
            for _ in range(10):
                lin(X, out=Y)
        torch.cuda.synchronize()
    ts = {"product": [], str(var): []}
    for _ in range(5):
        for name, lin in (("product", lp), (str(var), lv)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                lin(X, out=Y)
            e1.record()
            torch.cuda.synchronize()
            ts[name].append(e0.elapsed_time(e1) / 20 * 1e3)
    r = {"M": M, "rel_diff_f32": ((yp - yv).norm() / yv.norm()).item()}
    for k, v in ts.items():
        r[k + "_us"] = round(sorted(v)[2], 2)
    r["product_frac"] = round(2 * M * N * K / (r["product_us"] * 1e-6) / 2.5e15, 4)
    out.append(r)
    print(json.dumps(r), flush=True)
