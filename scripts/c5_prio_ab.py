"""C5 step (bench.py denoise_loop workload) with the loop's main stream at high priority against the
product (caller's default-priority stream), rounds interleaved; final states must be bit-identical.
Measurement only: python scripts/c5_prio_ab.py"""
import json, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import __graft_entry__ as g
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
dev = torch.device("cuda")
steps, dm, M, L = 50, 4096, 2048, 12
gen = torch.Generator(device=dev).manual_seed(99)
layers = [d.QuantLinear.from_weight((0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=gen), None, 4, 128,
                                    prefill_only=True) for _ in range(L)]
cfg = d.DiffusionConfig(num_timesteps=steps, hidden_size=dm, num_layers=L)
K0 = torch.randn(1, M, dm, device=dev, generator=gen)
V0 = torch.randn(1, M, dm, device=dev, generator=gen)
x = torch.randn(M, dm, device=dev, generator=gen)
lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
print(json.dumps({"priority_range": [lo, hi]}), flush=True)
hp = torch.cuda.Stream(priority=hi)
def run(mode):
    kv = d.KVCacheEntry.new(K0.clone(), V0.clone(), cfg.prefill_bits, cfg.decode_bits)
    loop = d.DenoiseLoop(layers, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=1, kv_cache=kv, overlap=True)
    st = hp if mode == "main_high" else torch.cuda.current_stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        if mode == "side_low":
            loop._side = torch.cuda.Stream(priority=lo)
        loop.sample(x, 3)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        out = loop.sample(x, steps)
        e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps, out
run("product")
res, outs = {}, {}
for rnd in range(3):
    for mode in ("product", "main_high"):
        t, o = run(mode)
        res.setdefault(mode, []).append(round(t, 4))
        outs[mode] = o
for mode, t in res.items():
    print(json.dumps({"mode": mode, "ms_per_step": t, "bit_identical": bool(torch.equal(outs[mode], outs["product"]))}))
