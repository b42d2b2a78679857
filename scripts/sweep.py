"""M-sweep of the quantized linear layer (K=N=4096 int4 g128).  Prints per-M event timings; run
under `rocprofv3 --kernel-trace` and pass the trace to scripts/sweep_trace.py for pure kernel
durations (no launch gaps).  Every M issues exactly WARM + REPS wq_* launches, in order.
VARIANTS=4,5 (env) repeats the sweep per kernel variant for A/B runs."""
import json, os, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import __graft_entry__ as g

WARM, REPS = 5, 20
Ms = [int(a) for a in sys.argv[1:]] or [1, 4, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192]
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
K = N = 4096
torch.manual_seed(0)
W = 0.02 * torch.randn(K, N, device="cuda")
lin = d.QuantLinear.from_weight(W, None, 4, 128)
torch.cuda.synchronize()
VARS = [int(v) for v in os.environ.get("VARIANTS", "4").split(",")]
# Clock pre-warm (~0.3 s of the largest shape) so the first entries are not measured cold.
Xw = torch.randn(max(Ms), K, device="cuda").half()
Yw = torch.empty(max(Ms), N, dtype=torch.float16, device="cuda")
import time
t0 = time.time()
while time.time() - t0 < 0.3:
    for _ in range(10):
        lin(Xw, out=Yw)
    torch.cuda.synchronize()
del Xw, Yw
for M in Ms:
  for var in VARS:
    lin.set_kernel_variant(var)
    X = torch.randn(M, K, device="cuda").half()
    Y = torch.empty(M, N, dtype=torch.float16, device="cuda")
    torch.cuda.synchronize()
    for _ in range(WARM):
        lin(X, out=Y)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        lin(X, out=Y)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / REPS
    print(json.dumps({"M": M, "variant": var, "event_us": round(ms * 1e3, 2),
                      "tflops": round(2 * M * N * K / ms / 1e9, 1)}), flush=True)
