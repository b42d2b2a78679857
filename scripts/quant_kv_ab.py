"""Per-tensor quantize and the KV-cache quantization step, timed in one process (HIP events around
back-to-back calls after a clock pre-warm; median of rounds).  Measurement only.
  qt      quantize_tensor of an 8192 x 4096 f32 tensor -> packed int4 (min/max + map)
  c4_old  config C4's QuantizedKVCacheEntry::new as two quantize_tensor calls (K, V: 8192 x 32 x 128)
  c4_kv   the same through dllm_quantize_kv (min/max K | map K + min/max V | map V)
  c5_old  the C5 KV update (K, V [1, 2048, 4096], widths 8 and 4) as two quantize_tensor_pair calls
  c5_kv   the same through dllm_quantize_kv
  c5_ext  the head-sharded form at one rank = the whole tensors: dllm_kv_extremes + _with_extremes
Usage: [DLLM_LIB=<file>] python scripts/quant_kv_ab.py"""
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
q = d.quantization
dev = torch.device("cuda")


def timed(fn, reps=20, rounds=5):
    t0 = time.time()
    while time.time() - t0 < 0.3:
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    return round(statistics.median(ts), 2)


x = torch.randn(8192 * 4096, device=dev)
K4 = torch.randn(8192 * 32 * 128, device=dev)
V4 = torch.randn(8192 * 32 * 128, device=dev) * 0.5
K5 = torch.randn(2048 * 4096, device=dev)
V5 = torch.randn(2048 * 4096, device=dev) * 0.5
res = {
    "qt": timed(lambda: q.quantize_tensor(x, 4, packed=True)),
    "c4_old": timed(lambda: (q.quantize_tensor(K4, 4, packed=True), q.quantize_tensor(V4, 4, packed=True))),
    "c4_kv": timed(lambda: q.quantize_kv(K4, V4, 4, 0)),
    "c5_old": timed(lambda: (q.quantize_tensor_pair(K5, 8, 4, packed=True), q.quantize_tensor_pair(V5, 8, 4, packed=True))),
    "c5_kv": timed(lambda: q.quantize_kv(K5, V5, 8, 4)),
}
red = q.kv_extremes(K5, V5)
res["c5_ext"] = timed(lambda: q.quantize_kv_with_extremes(K5, V5, q.kv_extremes(K5, V5), 8, 4))
# algorithmic bytes: f32 in once + packed codes out
res["qt_TBps"] = round((x.numel() * 4 + x.numel() // 2) / res["qt"] / 1e6, 2)
res["c4_kv_TBps"] = round(2 * (K4.numel() * 4 + K4.numel() // 2) / res["c4_kv"] / 1e6, 2)
res["c5_kv_TBps"] = round(2 * (K5.numel() * 4 + K5.numel() * 12 // 8) / res["c5_kv"] / 1e6, 2)
print(json.dumps(res), flush=True)
