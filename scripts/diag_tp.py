"""Diagnostic: where do the sharded and unsharded C5 steps part?  One Megatron pair at the C5 shape,
G = 2 emulated, against the unsharded pair and an f64 chain with the f16 rounding points."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
import __graft_entry__ as g
from tests import tp_emulation as emu
from oracle import oracle as orc

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
par = d.parallel
D, M, G = 4096, 2048, 2
gen = torch.Generator(device="cuda").manual_seed(7)
WA = (1 / 64) * torch.randn(D, D, device="cuda", generator=gen)
WB = (1 / 64) * torch.randn(D, D, device="cuda", generator=gen)
x = torch.randn(M, D, device="cuda", generator=gen)
A = d.QuantLinear.from_weight(WA, None, 4, 128)
B = d.QuantLinear.from_weight(WB, None, 4, 128)


def deq(lin):
    c, s, z = lin.export()
    cd = orc.unpack_bits(c.cpu().numpy(), lin.K * lin.N, 4).reshape(lin.K, lin.N)
    return torch.from_numpy(orc.dequantize_weights(cd, s.cpu().numpy(), z.cpu().numpy(), 128)).cuda()


WAh, WBh = deq(A).double(), deq(B).double()
rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()
h_u = A(x, out_dtype=torch.float16)
h_64 = x.half().double() @ WAh
print("A unsharded f16 out vs f64(f16 x):", rel(h_u.float(), h_64))
hA32 = A(x, out_dtype=torch.float32)
print("A unsharded f32 out vs f64(f16 x):", rel(hA32, h_64))
y_u = B(h_u, out_dtype=torch.float32)
y_64 = h_u.double() @ WBh
print("B unsharded f32 vs f64(same f16 h):", rel(y_u, y_64))
pairs = [par.TensorParallelPair(WA, None, WB, None, 4, 128, shard=(G, r)) for r in range(G)]
hs = torch.cat([p.a(x, out_dtype=torch.float16) for p in pairs], dim=1)
print("A column shards f16 == unsharded:", torch.equal(hs, h_u), "rel", rel(hs.float(), h_u.float()),
      "differing elems", (hs != h_u).sum().item())
em = emu.EmulatedTensorParallel(pairs)
y_s = em(x, out_dtype=torch.float32)
print("pair sharded vs unsharded f32:", rel(y_s, y_u))
print("pair sharded vs f64:", rel(y_s, y_64))
parts = [p.partial(x) for p in pairs]
for r, p in enumerate(pairs):
    k0, k1 = p.b.k0, p.b.k1
    ref = h_u[:, k0:k1].double() @ WBh[k0:k1]
    print(f"partial {r} vs f64:", rel(parts[r], ref))
print("x f32 -> torch matmul f32 vs f64:", rel(x @ WAh.float(), x.double() @ WAh))
