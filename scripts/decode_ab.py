"""A/B of decode-kernel variants (lab build) in the bench's setting: a chain of 40 distinct int4 g128
layers of K = N = 4096 (weights from HBM, past the MALL), captured in one HIP graph per variant and
replayed (HIP events).  Usage: decode_ab.py <variant> [M ...]; prints per M the product's and the
variant's us per layer and the relative difference of one layer's f32 output."""
import json
import os
import sys
from pathlib import Path
os.environ.setdefault("DLLM_LIB", "lab")
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
var = int(sys.argv[1])
Ms = [int(m) for m in (sys.argv[2:] or ["1", "16", "32", "64"])]
K = N = 4096
L = 40
gen = torch.Generator(device="cuda").manual_seed(5)
chain = []
for _ in range(L):
    chain.append(d.QuantLinear.from_weight(0.02 * torch.randn(K, N, device="cuda", generator=gen), None, 4, 128))


def timed(seq, xs, ys, cs):
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=cs):
        for lyr in seq:
            lyr(xs, out=ys)
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * len(seq)) * 1e3


for M in Ms:
    xs = torch.randn(M, K, device="cuda").half()
    ys = torch.empty(M, N, device="cuda", dtype=torch.float16)
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    res = {"M": M}
    for lyr in chain:
        lyr.set_kernel_variant(-1)
    y0 = chain[0](xs, out_dtype=torch.float32)
    with torch.cuda.stream(cs):
        for lyr in chain:
            lyr(xs, out=ys)
    torch.cuda.synchronize()
    t_prod = [timed(chain, xs, ys, cs)]
    for lyr in chain:
        lyr.set_kernel_variant(var)
    y1 = chain[0](xs, out_dtype=torch.float32)
    with torch.cuda.stream(cs):
        for lyr in chain:
            lyr(xs, out=ys)
    torch.cuda.synchronize()
    t_var = [timed(chain, xs, ys, cs)]
    for rnd in range(2):   # interleave once more
        for lyr in chain:
            lyr.set_kernel_variant(-1)
        t_prod.append(timed(chain, xs, ys, cs))
        for lyr in chain:
            lyr.set_kernel_variant(var)
        t_var.append(timed(chain, xs, ys, cs))
    res["product_us"] = round(sorted(t_prod)[1], 2)
    res[f"{var}_us"] = round(sorted(t_var)[1], 2)
    res["rel_diff_f32"] = ((y1 - y0).norm() / y0.norm()).item()
    print(json.dumps(res), flush=True)
