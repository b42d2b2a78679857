"""Per-rank compute of config C5's sharded forms at G = 1/2/4/8, measured in one process (VERDICT r04
item 6: DESIGN section 6's C5-sharded cost table).  HIP events around 50 launches after a 0.2 s warm
per shape; weights 0.5/64 N(0,1) as the bench's denoise loop, prefill-only handles as the shards.

* hidden-dim (Megatron pair, parallel.TensorParallelPair): the column shard [2048, 4096] x [4096, 4096/G]
  (f16 out) and the row shard [2048, 4096/G] x [4096/G, 4096] (f32 partial out), the pair's epilogue
  (dllm_bias_cast of the reduced [2048, 4096] f32 to f16), and the f32 partial's bytes;
* token-parallel replicas: one full layer on 2048/G tokens (no reduction for the linear layers).
Output: one JSON object (stdout / --out)."""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def timed(fn, torch, reps=50, warm_s=0.2):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) / reps * 1e3)
    best.sort()
    return round(best[1], 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--lib", default=None)
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    d = g.load_package()
    if args.lib:
        d._lib.use(args.lib)
    M, dm = 2048, 4096
    gen = torch.Generator(device="cuda").manual_seed(7)
    X = torch.randn(M, dm, device="cuda", generator=gen).half()
    res = {"note": "per-rank device time (us, HIP events, median of 3 x 50 launches), one process", "G": {}}
    for G in (1, 2, 4, 8):
        n = dm // G
        r = {}
        Wc = (0.5 / 64) * torch.randn(dm, n, device="cuda", generator=gen)
        col = d.QuantLinear.from_weight(Wc, None, 4, 128, prefill_only=True)
        Yc = torch.empty(M, n, dtype=torch.float16, device="cuda")
        r["column_gemm_us"] = timed(lambda: col(X, out=Yc), torch)
        Wr = (0.5 / 64) * torch.randn(n, dm, device="cuda", generator=gen)
        row = d.QuantLinear.from_weight(Wr, None, 4, 128, prefill_only=True)
        Xr = X[:, :n].contiguous()
        Yr = torch.empty(M, dm, dtype=torch.float32, device="cuda")
        r["row_gemm_f32_us"] = timed(lambda: row(Xr, out=Yr), torch)
        b = torch.zeros(dm, device="cuda")
        Yh = torch.empty(M, dm, dtype=torch.float16, device="cuda")
        r["bias_cast_us"] = timed(lambda: d.quantization.bias_cast(Yr, b, torch.float16, out=Yh), torch)
        r["partial_bytes"] = M * dm * 4
        Mt = M // G
        Wt = (0.5 / 64) * torch.randn(dm, dm, device="cuda", generator=gen)
        tok = d.QuantLinear.from_weight(Wt, None, 4, 128, prefill_only=True)
        Xt = X[:Mt].contiguous()
        Yt = torch.empty(Mt, dm, dtype=torch.float16, device="cuda")
        r["token_parallel_layer_us"] = timed(lambda: tok(Xt, out=Yt), torch)
        r["pair_compute_us"] = round(r["column_gemm_us"] + r["row_gemm_f32_us"] + r["bias_cast_us"], 2)
        res["G"][G] = r
        print(json.dumps({"G": G, **r}), flush=True)
        for h in (col, row, tok):
            h.close()
        del Wc, Wr, Wt
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
