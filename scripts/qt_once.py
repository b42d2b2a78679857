import sys, torch
sys.path.insert(0, "/root/repo")
import __graft_entry__ as g
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
q = d.quantization
x = torch.randn(8192 * 4096, device="cuda")
K5 = torch.randn(2048 * 4096, device="cuda"); V5 = torch.randn(2048 * 4096, device="cuda")
for _ in range(30): q.quantize_tensor(x, 4, packed=True)
for _ in range(30): q.quantize_kv(K5, V5, 8, 4)
torch.cuda.synchronize()
