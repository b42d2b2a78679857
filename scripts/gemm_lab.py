"""A/B the prefill GEMM schedule variants in ONE process (interleaved rounds), checking that
every variant is bit-identical to variant 0.  Usage: python scripts/gemm_lab.py [M ...]"""
import json, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
Ms = [int(a) for a in sys.argv[1:]] or [2048, 4096]
VARS = [int(v) for v in __import__("os").environ.get("VARS", "0,1,2,3").split(",")]
K = N = 4096
torch.manual_seed(0)
W = 0.02 * torch.randn(K, N, device="cuda")
lin = d.QuantLinear.from_weight(W, None, 4, 128)
for M in Ms:
    X = torch.randn(M, K, device="cuda").half()
    Y = {v: torch.empty(M, N, dtype=torch.float16, device="cuda") for v in VARS}
    times = {v: [] for v in VARS}
    for v in VARS:
        lin.set_kernel_variant(v)
        for _ in range(3):
            lin(X, out=Y[v])
    torch.cuda.synchronize()
    for rnd in range(5):
        for v in VARS:
            lin.set_kernel_variant(v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                lin(X, out=Y[v])
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 10)
    for v in VARS:
        t = sorted(times[v])
        same = torch.equal(Y[v], Y[VARS[0]])
        print(json.dumps({"M": M, "variant": v, "us_med": round(t[len(t)//2]*1e3, 1), "us_min": round(t[0]*1e3, 1),
                          "tflops_med": round(2*M*N*K/(t[len(t)//2]*1e-3)/1e12, 1), "bitwise_same_as_v0": same}), flush=True)
