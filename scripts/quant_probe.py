"""Per-kernel probe of quantize_tensor (a1) at the C2'/C4 size: run under
rocprofv3 --kernel-trace --stats to split the min/max pass from the quantize map."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import __graft_entry__ as g  # noqa: E402

dllm = g.load_package(); import scripts._lab as _lab; _lab.select(dllm)
n_iter = int(sys.argv[1]) if len(sys.argv) > 1 else 20
x = torch.randn(8192 * 4096, device="cuda")
k = torch.randn(8192 * 4096, device="cuda")
for _ in range(n_iter):
    dllm.quantize_tensor(x, 4, packed=True)
    dllm.quantize_tensor_pair(k, 4, 2, packed=True)
w = 0.02 * torch.randn(4096, 4096, device="cuda")
for _ in range(5):
    dllm.QuantLinear.from_weight(w, None, 4, 128)     # a5 weight quantization (quantize_weights4_kernel)
torch.cuda.synchronize()
print("done")
