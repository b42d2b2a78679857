"""FETCH_SIZE calibration: a streaming read of a known byte count on the same box and
counter as the GEMM passes.  minmax_partial_kernel (dllm_tensor_extremes) reads a 1 GiB f32 tensor
once with 16-B coalesced loads per lane (4 in flight per thread) and writes one float2 per block.
Run under `rocprofv3 --pmc FETCH_SIZE --kernel-include-regex minmax_partial`; compare the per-dispatch
FETCH_SIZE (KiB) with 1 GiB = 1048576 KiB."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
x = torch.randn(1 << 28, device="cuda")          # 1 GiB, larger than the 256 MiB Infinity Cache
flush = torch.empty(1 << 28, device="cuda")
for _ in range(5):
    flush.fill_(1.0)                             # evict x from the Infinity Cache between reads
    d.quantization.tensor_extremes(x)
torch.cuda.synchronize()
print("read bytes per dispatch:", x.numel() * 4)
