"""Where config C5's step goes (bench.py denoise_loop workload: 12 int4 g128 layers d 4096, seq 2048):
per-step ms of the product loop (KV update on the side stream, noise in the last layer's epilogue),
of the serial loop, and of the loop without a KV cache (the denoiser + p_sample alone).  Measurement
only: python scripts/c5_breakdown.py [steps] [modes, comma-separated]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
dev = torch.device("cuda")
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
want = sys.argv[2].split(",") if len(sys.argv) > 2 else ["product", "product_cast", "serial", "nokv"]
dm, M, L = 4096, 2048, 12
gen = torch.Generator(device=dev).manual_seed(99)
layers = [d.QuantLinear.from_weight((0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=gen), None, 4, 128)
          for _ in range(L)]
cfg = d.DiffusionConfig(num_timesteps=steps, hidden_size=dm, num_layers=L)
K0 = torch.randn(1, M, dm, device=dev, generator=gen)
V0 = torch.randn(1, M, dm, device=dev, generator=gen)
x = torch.randn(M, dm, device=dev, generator=gen)
modes = {"product": dict(overlap=True), "serial": dict(overlap=False), "nokv": dict(overlap=True),
         "product_cast": dict(overlap=True), "spread": dict(overlap=True)}   # product_cast: without the f16 x_prev hand-off
res = {}
for rnd in range(int(__import__("os").environ.get("ROUNDS", "2"))):
    for name in want:
        kv = None if name == "nokv" else d.KVCacheEntry.new(K0.clone(), V0.clone(), cfg.prefill_bits, cfg.decode_bits)
        loop = d.DenoiseLoop(layers, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=1, kv_cache=kv, **modes[name])
        loop.f16_handoff = name != "product_cast"
        loop.kv_spread = name != "product"     # "product": the round-4 free-running side stream
        loop.sample(x, 3)
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        out = loop.sample(x, steps)
        e1.record(st)
        torch.cuda.synchronize()
        res.setdefault(name, []).append(round(e0.elapsed_time(e1) / steps, 4))
        res[name + "_out"] = out
ref = res.get("serial_out")
for name in want:
    o = res[name + "_out"]
    print(json.dumps({"mode": name, "ms_per_step": res[name], "finite": bool(torch.isfinite(o).all()),
                      "bit_identical_to_serial": None if ref is None or name == "nokv" else bool(torch.equal(o, ref))}),
          flush=True)
