"""One decode chain for a kernel trace: L distinct 4096x4096 int4 g128 layers at M tokens (argv),
captured in a HIP graph and replayed 20 times.  Measurement only:
rocprofv3 --kernel-trace --stats -- python3 scripts/decode_chain_once.py 64"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import __graft_entry__ as g  # noqa: E402

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 64
K = N = 4096
L = 40
gen = torch.Generator(device="cuda").manual_seed(7)
layers = [d.QuantLinear.from_weight((0.5 / 64) * torch.randn(K, N, device="cuda", generator=gen), None, 4, 128)
          for _ in range(L)]
X = torch.randn(M, K, device="cuda", generator=gen).half()
bufs = [X] + [torch.empty(M, N, dtype=torch.float16, device="cuda") for _ in range(L)]
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    for i, lin in enumerate(layers):
        lin(bufs[i], out=bufs[i + 1])
    torch.cuda.synchronize()
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph, stream=st):
        for i, lin in enumerate(layers):
            lin(bufs[i], out=bufs[i + 1])
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(5):
    gph.replay()
torch.cuda.synchronize()
e0.record()
for _ in range(20):
    gph.replay()
e1.record()
torch.cuda.synchronize()
print(f"M={M} us_per_layer={e0.elapsed_time(e1) / 20 / L * 1e3:.3f}")
