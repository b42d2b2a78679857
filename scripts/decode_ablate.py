"""Decode-kernel ablation (measurement only): time the M<=16 decode GEMM with parts of its load
phase replaced by constants (1: X, 2: scales, 4: weights), 48 distinct layers > Infinity Cache."""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
dev = torch.device("cuda")
K = N = int(os.environ.get("DIM", "4096"))
L = 48
layers = [d.QuantLinear.from_weight(0.02 * torch.randn(K, N, device=dev), None, 4, 128) for _ in range(L)]
for M in (1, 16):
    X = torch.randn(M, K, device=dev).half()
    Y = torch.empty(M, N, dtype=torch.float16, device=dev)
    for lab in range(8):
        for lin in layers:
            lin.set_kernel_variant(16 + lab)
        for _ in range(3):
            for lin in layers:
                lin(X, out=Y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            for lin in layers:
                lin(X, out=Y)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / (10 * L) * 1e3
        print(json.dumps({"M": M, "lab": lab, "skip": [n for b, n in ((1, "X"), (2, "sz"), (4, "W")) if lab & b],
                          "us_per_layer": round(us, 2)}), flush=True)
