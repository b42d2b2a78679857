"""C4 dequant-attention (S 8192, 32 heads x 128, int4 K/V per tensor): 3 warm + 20 timed calls."""
import json, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
S, H, D = [int(a) for a in sys.argv[1:4]] if len(sys.argv) > 3 else (8192, 32, 128)
K = torch.randn(S, H, D, device="cuda"); V = torch.randn(S, H, D, device="cuda")
Q = torch.randn(S, H, D, device="cuda").half()
e = d.QuantizedKVCacheEntry.new(K, V, 4)
for _ in range(3):
    d.kv_attention(Q, e.keys, e.values)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    d.kv_attention(Q, e.keys, e.values)
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / 20
print(json.dumps({"S": S, "H": H, "ms": round(ms, 4), "tflops": round(4 * S * S * H * D / ms / 1e9, 1)}))
