"""Runs the int4-g128 GEMM of one library build on one shape, for `rocprofv3 --kernel-trace --stats`:
a 0.3 s warm-up, then 200 launches.  Usage (measurement only):
  rocprofv3 --kernel-trace --stats -d OUT -o NAME -- python3 scripts/kernel_times.py LIB M:N"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    import __graft_entry__ as g
    d = g.load_package()
    d._lib.use(str((ROOT / sys.argv[1]).resolve()))
    K = 4096
    M, N = (int(v) for v in sys.argv[2].split(":"))
    torch.manual_seed(0)
    lin = d.QuantLinear.from_weight(0.02 * torch.randn(K, N, device="cuda"), None, 4, 128, prefill_only=True)
    X = torch.randn(M, K, device="cuda").half()
    Y = torch.empty(M, N, dtype=torch.float16, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(20):
            lin(X, out=Y)
        torch.cuda.synchronize()
    for _ in range(200):
        lin(X, out=Y)
    torch.cuda.synchronize()
    lin.close()


if __name__ == "__main__":
    main()
