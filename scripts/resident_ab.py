"""A/B of quantize_tensor at the C4 / C5 KV shape (8192 x 4096 f32 -> int4, and the 8 + 4 bit pair of
KVCacheEntry::update): the resident single-read kernel vs the two-kernel path (DLLM_QUANT_TWO_PASS=1),
HIP events over 20 calls each, interleaved; algorithmic bytes = 4n read once + the packed codes."""
import json, os, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
n = 8192 * 4096
x = torch.randn(n, device="cuda")
cases = {"int4": lambda: d.quantize_tensor(x, 4, packed=True),
         "pair8+4": lambda: d.quantize_tensor_pair(x, 8, 4, packed=True)}
wbytes = {"int4": n // 2, "pair8+4": n + n // 2}
for name, fn in cases.items():
    res = {}
    for rnd in range(3):
        for mode in ("resident", "two_pass"):
            os.environ["DLLM_QUANT_TWO_PASS"] = "1" if mode == "two_pass" else "0"
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / 20 * 1e3)
    for mode, ts in res.items():
        us = sorted(ts)[len(ts) // 2]
        b = 4 * n + wbytes[name]
        print(json.dumps({"case": name, "mode": mode, "us": round(us, 2), "alg_TBps": round(b / us / 1e6, 3),
                          "hbm_frac": round(b / us / 1e6 / 8.0, 4)}), flush=True)
