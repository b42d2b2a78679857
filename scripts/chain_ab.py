"""Per-layer time of a chain of 40 distinct 4096 x 4096 int4 g128 layers (40 x 9 MiB of weights:
past the Infinity Cache) captured in one HIP graph and replayed, at the given M (JSON line).  The
library build is chosen by DLLM_LIB (scripts/_lab.py), so two builds or lab switches A/B on the
same shapes.  Usage: [DLLM_LIB=...] MS=33,48,64 python scripts/chain_ab.py   (measurement only)."""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
dev = torch.device("cuda")
K = N = 4096
gen = torch.Generator(device=dev).manual_seed(99)
chain = [d.QuantLinear.from_weight(0.02 * torch.randn(K, N, device=dev, generator=gen), None, 4, 128) for _ in range(40)]
out = {"env": {k: v for k, v in os.environ.items() if k.startswith("DLLM_")}}
for m in [int(v) for v in os.environ.get("MS", "1,16,33,48,64,256").split(",")]:
    xs = torch.randn(m, K, device=dev).half()
    ys = torch.empty(m, N, dtype=torch.float16, device=dev)
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        for lyr in chain:
            lyr(xs, out=ys)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=cs):
        for lyr in chain:
            lyr(xs, out=ys)
    gr.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / len(chain) * 1e3)
    ts.sort()
    out[str(m)] = round(ts[2], 2)
print(json.dumps(out), flush=True)
