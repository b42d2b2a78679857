"""A/B of the dequant-attention schedules on config C4 (S 8192, 32 heads x 128, int4 KV), lab build,
one process (DLLM_ATTN_LAB is read per call), interleaved rounds, HIP events: 0 = the product
(v5 with s_setprio 1 over region 2), 302 = v5 without that priority, 198 = v5 with waves 4-7
staggered by half a key block, 4196 = v5 with the round-2 epilogue (64 two-byte O stores per
lane).  The outputs must be bit-identical.
Also checks ragged S (partial key blocks / query tiles).  Measurement only."""
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
labs = [int(v) for v in (sys.argv[1:] or ["0", "302", "198"])]


def run(lab, Q, e):
    os.environ["DLLM_ATTN_LAB"] = str(lab)
    return d.kv_attention(Q, e.keys, e.values)


ident = {}
for S in (65, 200, 4160, 8003):
    torch.manual_seed(S)
    K = torch.randn(S, 4, 128, device="cuda"); V = torch.randn(S, 4, 128, device="cuda")
    Q = torch.randn(S, 4, 128, device="cuda").half()
    e = d.QuantizedKVCacheEntry.new(K, V, 4)
    outs = [run(l, Q, e) for l in labs]
    ident[S] = all(torch.equal(outs[0], o) for o in outs[1:])
S, H, D = int(os.environ.get("AB_S", "8192")), 32, 128   # AB_S: timed sequence length
torch.manual_seed(0)
K = torch.randn(S, H, D, device="cuda"); V = torch.randn(S, H, D, device="cuda")
Q = torch.randn(S, H, D, device="cuda").half()
e = d.QuantizedKVCacheEntry.new(K, V, 4)
outs = [run(l, Q, e) for l in labs]
ident[S] = all(torch.equal(outs[0], o) for o in outs[1:])
for _ in range(3):
    for l in labs:
        run(l, Q, e)
torch.cuda.synchronize()
res = {l: [] for l in labs}
for rnd in range(5):
    for l in labs:
        os.environ["DLLM_ATTN_LAB"] = str(l)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            d.kv_attention(Q, e.keys, e.values)
        b.record()
        torch.cuda.synchronize()
        res[l].append(a.elapsed_time(b) / 10)
flops = 4.0 * S * S * H * D
print(json.dumps({"bit_identical": ident,
                  "ms": {str(l): round(sorted(t)[2], 4) for l, t in res.items()},
                  "frac": {str(l): round(flops / (sorted(t)[2] * 1e-3) / 2.5e15, 4) for l, t in res.items()}}))
