"""Per-kernel probe of quantize_tensor (a1) at the C2'/C4 size: run under
rocprofv3 --kernel-trace --stats to split the min/max pass from the quantize map."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import __graft_entry__ as g  # noqa: E402

dllm = g.load_package()
n_iter = int(sys.argv[1]) if len(sys.argv) > 1 else 20
x = torch.randn(8192 * 4096, device="cuda")
k = torch.randn(8192 * 4096, device="cuda")
for _ in range(n_iter):
    dllm.quantize_tensor(x, 4, packed=True)
    dllm.quantize_tensor_pair(k, 4, 2, packed=True)
torch.cuda.synchronize()
print("done")
