"""Does quantize_tensor's second pass (the quantize map, a second read of x) hit the 256 MB Infinity
Cache after the min/max pass?  8192 x 4096 f32 (128 MiB) -> int4 packed, HIP events:
  extremes  -- the min/max pass alone (x cold: a 512 MiB sweep first)
  map_cold  -- quantize_tensor_with_params alone, x cold
  map_warm  -- quantize_tensor_with_params right after a read of x (the min/max pass)
  fused     -- dllm_quantize_tensor (both passes), x cold
Prints one JSON line.  Measurement only."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import __graft_entry__ as g  # noqa: E402

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
from dllm_amd import quantization as dq  # noqa: E402
n = 8192 * 4096
x = torch.randn(n, device="cuda")
flush = torch.empty(128 * 2**20, device="cuda")   # 512 MiB
params = dq.quantize_params_from_extremes(dq.tensor_extremes(x), 4)


def cold():
    flush.add_(1.0)   # reads and writes 512 MiB: evicts x from L2 and the MALL


def timed(fn, pre, reps=20):
    ts = []
    for _ in range(reps):
        pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


for _ in range(3):
    d.quantize_tensor(x, 4, packed=True)
res = {
    "extremes_cold_us": timed(lambda: dq.tensor_extremes(x), cold),
    "map_cold_us": timed(lambda: dq.quantize_tensor_with_params(x, 4, params, packed=True), cold),
    "map_warm_us": timed(lambda: dq.quantize_tensor_with_params(x, 4, params, packed=True),
                         lambda: (cold(), dq.tensor_extremes(x))),
    "fused_cold_us": timed(lambda: d.quantize_tensor(x, 4, packed=True), cold),
    "fused_warm_us": timed(lambda: d.quantize_tensor(x, 4, packed=True), lambda: dq.tensor_extremes(x)),
}
res["bytes_read_once"] = n * 4
print(json.dumps(res))
