"""Per-K timing of the default (Horner, 256 x 256) exact GEMM at M = N = 4096: the slope is the main
loop's cost per 64-deep k-step, the intercept the fixed cost (launch, prologue, epilogue store).
HIP events, 300 ms clock pre-warm per shape, median of 5 rounds of 20 launches."""
import json
import sys
import time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
M = N = 4096
res = []
for K in [int(a) for a in (sys.argv[1:] or ["128", "256", "512", "1024", "2048", "4096"])]:
    W = 0.02 * torch.randn(K, N, device="cuda")
    X = torch.randn(M, K, device="cuda").half()
    Y = torch.empty(M, N, device="cuda", dtype=torch.float16)
    lin = d.QuantLinear.from_weight(W, None, 4, 128)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(20):
            lin(X, out=Y)
        torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            lin(X, out=Y)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    ts.sort()
    res.append({"K": K, "us_median": round(ts[2], 2), "us_min": round(ts[0], 2)})
    print(json.dumps(res[-1]), flush=True)
    lin.close()
ks = [r["K"] / 64 for r in res]
us = [r["us_median"] for r in res]
n = len(ks)
mx, my = sum(ks) / n, sum(us) / n
slope = sum((a - mx) * (b - my) for a, b in zip(ks, us)) / sum((a - mx) ** 2 for a in ks)
print(json.dumps({"slope_us_per_kstep": round(slope, 4), "intercept_us": round(my - slope * mx, 2)}))
