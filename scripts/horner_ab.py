"""A/B of the int4 g128 Horner-form GEMM schedules at M = K = N = 4096 (lab build, one process,
interleaved rounds, HIP events): -1 = the product kernel (linear_horner.hip, staggered half
k-steps), 25 = the same without the stagger, 24 = round 2's wq_gemm8_kernel<..., HORNER>.
All three run the same arithmetic in the same order, so their outputs must be bit-identical."""
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
M = N = K = int(os.environ.get("AB_K", "4096"))
N = int(os.environ.get("AB_N", str(N)))
M = int(os.environ.get("AB_M", str(M)))
W = 0.02 * torch.randn(K, N, device="cuda")
X = torch.randn(M, K, device="cuda").half()
variants = [int(v) for v in (sys.argv[1:] or ["-1", "25", "24"])]
lins = {}
for v in variants:
    lin = d.QuantLinear.from_weight(W, None, 4, 128)
    lin.set_kernel_variant(v)
    lins[v] = lin
outs = {v: lins[v](X, out_dtype=torch.float32) for v in variants}
ident = {v: bool(torch.equal(outs[v], outs[variants[0]])) for v in variants}
Y = torch.empty(M, N, device="cuda", dtype=torch.float16)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    for v in variants:
        for _ in range(10):
            lins[v](X, out=Y)
    torch.cuda.synchronize()
res = {v: [] for v in variants}
for rnd in range(7):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            lins[v](X, out=Y)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 20 * 1e3)
summ = {str(v): {"median_us": round(sorted(t)[3], 2), "min_us": round(min(t), 2),
                 "frac": round(2 * M * N * K / (sorted(t)[3] * 1e-6) / 2.5e15, 4)} for v, t in res.items()}
print(json.dumps({"M": M, "K": K, "N": N, "bit_identical_to_first": ident, "us": summ}))
