"""Vendor reference for the shard shapes: torch.matmul (hipBLASLt) f16 X [M, K] @ f16 W [K, N] with
f32 accumulation, HIP events around 20 back-to-back calls after a 300 ms pre-warm, median of 5
rounds.  Prints one JSON line {"M:N": {"us", "tflops"}}.  Measurement only: tells how much of a
shard's per-column slowdown a plain f16 GEMM of the same shape shows too."""
import json
import os
import time

import torch

K = 4096
shapes = os.environ.get("SHAPES", "4096:4096,4096:2048,4096:1024,4096:512,2048:4096,2048:2048,2048:1024,2048:512")
out = {}
for sh in shapes.split(","):
    M, N = (int(v) for v in sh.split(":"))
    torch.manual_seed(0)
    X = torch.randn(M, K, device="cuda").half()
    W = (0.02 * torch.randn(K, N, device="cuda")).half()
    Y = torch.empty(M, N, dtype=torch.float16, device="cuda")
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        torch.matmul(X, W, out=Y)
        torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            torch.matmul(X, W, out=Y)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 20 * 1e3)
    ts.sort()
    out[sh] = {"us": round(ts[2], 2), "tflops": round(2 * M * N * K / ts[2] / 1e6, 1)}
print(json.dumps(out), flush=True)
