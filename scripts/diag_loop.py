"""Diagnostic: one C5 step, sharded (G = 2 emulated) vs unsharded, layer by layer."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
import __graft_entry__ as g
from tests import tp_emulation as emu

dllm = g.load_package(); import scripts._lab as _lab; _lab.select(dllm)
par = dllm.parallel
d, M, L, steps, seed, G = 4096, 2048, 12, 50, 7, 2
gen = torch.Generator(device="cuda").manual_seed(7)
Ws = [(1.0 / 64.0) * torch.randn(d, d, device="cuda", generator=gen) for _ in range(L)]
x = torch.randn(M, d, device="cuda", generator=gen)
unsh = [dllm.QuantLinear.from_weight(W, None, 4, 128) for W in Ws]
pairs = [emu.EmulatedTensorParallel([par.TensorParallelPair(Ws[2 * p], None, Ws[2 * p + 1], None, 4, 128,
                                                            shard=(G, r)) for r in range(G)]) for p in range(L // 2)]
rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()
hu, hs = x, x
for p in range(L // 2):
    hu = unsh[2 * p](hu, out_dtype=torch.float16)
    hu = unsh[2 * p + 1](hu, out_dtype=torch.float16 if p < L // 2 - 1 else torch.float32)
    hs = pairs[p](hs, out_dtype=torch.float16 if p < L // 2 - 1 else torch.float32)
    print(f"pair {p}: rel {rel(hs.float(), hu.float()):.3e}", flush=True)
cfg = dllm.DiffusionConfig(num_timesteps=steps, hidden_size=d, num_layers=L)
lu = dllm.DenoiseLoop(unsh, cfg, cumprod=dllm.Cumprod.INCLUSIVE, seed=seed, overlap=False)
ls = dllm.DenoiseLoop(pairs, cfg, cumprod=dllm.Cumprod.INCLUSIVE, seed=seed, overlap=False)
xu = lu.step(x, steps - 1, 0)
xs = ls.step(x, steps - 1, 0)
print("step rel", rel(xs, xu))
# unfused last layer for the unsharded loop
coef, flag = lu._coef(steps - 1)
eps_u = hu
out = torch.empty_like(x)
dllm.diffusion.DeviceLoopOps.p_sample(x, eps_u, None, coef, flag, seed, 0, out)
print("unsharded fused vs unfused:", rel(xu, out))
print("sharded vs unsharded unfused:", rel(xs, out))
print("eps rel", rel(hs, hu))
