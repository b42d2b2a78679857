"""A/B of config C5's step (bench.py denoise_loop workload: 12 int4 g128 layers d 4096, seq 2048,
KV update): noise drawn on the side stream (default) vs inside the last layer's fused p_sample
epilogue, vs everything serial.  Same seeds, so the final states must be bit-identical.
Measurement only: python scripts/c5_ab.py [steps]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
dev = torch.device("cuda")
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dm, M, L = 4096, 2048, 12
gen = torch.Generator(device=dev).manual_seed(99)
layers = [d.QuantLinear.from_weight((0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=gen), None, 4, 128)
          for _ in range(L)]
cfg = d.DiffusionConfig(num_timesteps=steps, hidden_size=dm, num_layers=L)
K0 = torch.randn(1, M, dm, device=dev, generator=gen)
V0 = torch.randn(1, M, dm, device=dev, generator=gen)
x = torch.randn(M, dm, device=dev, generator=gen)
modes = {"side": dict(overlap=True, noise="side"), "epilogue": dict(overlap=True, noise="epilogue"),
         "serial": dict(overlap=False)}
outs, times = {}, {k: [] for k in modes}
for rnd in range(3):
    for name, kw in modes.items():
        kv = d.KVCacheEntry.new(K0.clone(), V0.clone(), cfg.prefill_bits, cfg.decode_bits)
        loop = d.DenoiseLoop(layers, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=1, kv_cache=kv, **kw)
        loop.sample(x, 3)
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        out = loop.sample(x, steps)
        e1.record(st)
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / steps)
        outs[name] = out
ref = outs["serial"]
for name in modes:
    t = sorted(times[name])
    print(json.dumps({"mode": name, "ms_per_step_med": round(t[1], 4), "ms_per_step_min": round(t[0], 4),
                      "bit_identical_to_serial": bool(torch.equal(outs[name], ref)),
                      "finite": bool(torch.isfinite(outs[name]).all())}), flush=True)
