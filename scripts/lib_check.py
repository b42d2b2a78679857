"""Correctness screen of one library build (DLLM_LIB=<file> via scripts/_lab) on int4 g128 GEMM shapes
(measurement-script check, the -m gpu suite is the record): exact-integer data (K 768, scale 1, zp 0)
must match the f64 product bit for bit (f32 and f16 outputs); random data within 2e-5 of f32 on the
same f16 X with the exported a2 weights.  Usage: DLLM_LIB=<so> python scripts/lib_check.py M:N[,M:N...]"""
import json, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import __graft_entry__ as g
d = g.load_package()
import scripts._lab as _lab
_lab.select(d)
from oracle import oracle as orc
out = {}
for sh in sys.argv[1].split(","):
    M, N = (int(v) for v in sh.split(":"))
    rng = np.random.default_rng(M + N)
    K = 768
    W = rng.integers(0, 16, (K, N)).astype(np.float32)
    for g0 in range(0, K, 128):
        W[g0, :], W[g0 + 1, :] = 0.0, 15.0
    X = rng.integers(-2, 3, (M, K)).astype(np.float32)
    b = rng.integers(-4, 5, N).astype(np.float32)
    lin = d.QuantLinear.from_weight(torch.from_numpy(W).cuda(), torch.from_numpy(b).cuda(), 4, 128)
    ref = (X.astype(np.float64) @ W.astype(np.float64) + b).astype(np.float32)
    Xd = torch.from_numpy(X).cuda().half()
    y32 = lin(Xd, out_dtype=torch.float32).cpu().numpy()
    y16 = lin(Xd, out_dtype=torch.float16).float().cpu().numpy()
    exact = bool(np.array_equal(y32, ref)) and bool(np.array_equal(y16, ref.astype(np.float16).astype(np.float32)))
    lin.close()
    K = 4096
    gen = torch.Generator(device="cuda").manual_seed(M + N)
    Wr = 0.02 * torch.randn(K, N, device="cuda", generator=gen)
    br = 0.1 * torch.randn(N, device="cuda", generator=gen)
    Xr = torch.randn(M, K, device="cuda", generator=gen).half()
    lin = d.QuantLinear.from_weight(Wr, br, 4, 128)
    codes, scales, zps = lin.export()
    Wh = torch.from_numpy(orc.dequantize_weights(orc.unpack_bits(codes.cpu().numpy(), K * N, 4).reshape(K, N),
                                                 scales.cpu().numpy(), zps.cpu().numpy(), 128)).cuda()
    Yr = Xr.float() @ Wh + br
    Y = lin(Xr, out_dtype=torch.float32)
    rel = (torch.linalg.norm(Y - Yr) / torch.linalg.norm(Yr)).item()
    lin.close()
    out[sh] = {"exact_integers": exact, "rel_vs_f32": rel, "ok": exact and rel <= 2e-5}
print(json.dumps(out))
