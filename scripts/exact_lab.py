"""A/B the two precision modes of the product library -- DLLM_PRECISION_F16W (rounded weights) and
DLLM_PRECISION_EXACT -- in ONE process (interleaved rounds): kernel time (HIP events) and the
relative Frobenius error of each against torch f32 on the f32-dequantized weights (reference a2:
(q - zp) * s in f32).  With DLLM_LIB=lab, VARS=... selects lab schedule variants instead.
Usage: python scripts/exact_lab.py [M:N ...]   (default 2048:4096 4096:4096 4096:2048 4096:1024 4096:512)"""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
shapes = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or [(2048, 4096), (4096, 4096), (4096, 2048),
                                                                         (4096, 1024), (4096, 512), (1024, 4096),
                                                                         (256, 4096)]
LAB = "VARS" in os.environ
VARS = [int(v) for v in os.environ["VARS"].split(",")] if LAB else ["f16w", "exact"]
K = 4096
torch.manual_seed(0)


def dequant_f32(lin, K, N, group=128):
    codes, s, z = lin.export()
    b = codes.view(torch.uint8).to(torch.int32)
    q = torch.stack([b & 15, b >> 4], dim=1).reshape(-1)[: K * N].reshape(K, N).float()
    G = K // group
    zf = z.reshape(G, N).float().repeat_interleave(group, 0)
    sf = s.reshape(G, N).repeat_interleave(group, 0)
    return (q - zf) * sf


for M, N in shapes:
    W = 0.02 * torch.randn(K, N, device="cuda")
    if LAB:
        lin = d.QuantLinear.from_weight(W, None, 4, 128)
        lins = {v: lin for v in VARS}
    else:
        lins = {"f16w": d.QuantLinear.from_weight(W, None, 4, 128, d.linear.F16W),
                "exact": d.QuantLinear.from_weight(W, None, 4, 128, d.linear.EXACT)}
        lin = lins["exact"]
    X = torch.randn(M, K, device="cuda").half()
    ref = X.float() @ dequant_f32(lin, K, N)
    Y = {v: torch.empty(M, N, dtype=torch.float32, device="cuda") for v in VARS}
    times = {v: [] for v in VARS}
    def use(v):
        if LAB:
            lin.set_kernel_variant(v)
        return lins[v]
    for v in VARS:
        for _ in range(3):
            use(v)(X, out=Y[v])
    torch.cuda.synchronize()
    for rnd in range(7):
        for v in VARS:
            L = use(v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                L(X, out=Y[v])
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 20)
    for v in VARS:
        t = sorted(times[v])
        rel = (torch.linalg.norm(Y[v] - ref) / torch.linalg.norm(ref)).item()
        print(json.dumps({"M": M, "N": N, "variant": v, "us_med": round(t[len(t) // 2] * 1e3, 1),
                          "us_min": round(t[0] * 1e3, 1),
                          "tflops_med": round(2 * M * N * K / (t[len(t) // 2] * 1e-3) / 1e12, 1),
                          "rel_err_vs_f32_xf16": rel}), flush=True)
    for L in set(lins.values()):
        L.close()
