"""Eager chain of 40 distinct 4096 x 4096 int4 g128 layers at one M (MS env), run 3 times, for PMC
passes (rocprofv3 --pmc ... -- python scripts/pmc_chain.py): the same launches the M-sweep replays
in a HIP graph, without the graph (counters are collected per dispatch)."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
dev = torch.device("cuda")
gen = torch.Generator(device=dev).manual_seed(99)
chain = [d.QuantLinear.from_weight(0.02 * torch.randn(4096, 4096, device=dev, generator=gen), None, 4, 128)
         for _ in range(40)]
m = int(os.environ.get("MS", "64"))
xs = torch.randn(m, 4096, device=dev).half()
ys = torch.empty(m, 4096, dtype=torch.float16, device=dev)
for _ in range(3):
    for lyr in chain:
        lyr(xs, out=ys)
torch.cuda.synchronize()
