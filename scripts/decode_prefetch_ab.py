"""Decode chain A/B: per-layer time of a chain of L distinct 4096x4096 int4 g128 layers (L x 17.6 MiB
of layouts, past the 256 MiB MALL) captured in one HIP graph, each layer launched with
dllm_linear_forward (plain) or dllm_linear_forward_prefetch(next = the following layer, the last
one prefetching layer 0 for the next replay).  Also checks that both forms give the same bits.
Prints JSON lines."""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

import __graft_entry__ as g

d = g.load_package()
dev = torch.device("cuda")
K = N = int(os.environ.get("DIM", "4096"))
L = int(os.environ.get("LAYERS", "40"))
Ms = [int(m) for m in os.environ.get("MS", "1,8,16,32,48,64").split(",")]
REPS = int(os.environ.get("REPS", "5"))


def graph_time(fn, stream):
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(gph, stream=stream):
            fn()
    torch.cuda.synchronize()
    gph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        gph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / REPS / L * 1e3   # us per layer


def main():
    gen = torch.Generator(device=dev).manual_seed(7)
    layers = [d.QuantLinear.from_weight(0.02 * torch.randn(K, N, device=dev, generator=gen), None, 4, 128)
              for _ in range(L)]
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    for M in Ms:
        X = torch.randn(M, K, device=dev, generator=gen).half()
        bufs = [X] + [torch.empty(M, N, dtype=torch.float16, device=dev) for _ in range(L)]

        def plain():
            for i, lin in enumerate(layers):
                lin(bufs[i], out=bufs[i + 1])

        def pref():
            for i, lin in enumerate(layers):
                lin(bufs[i], out=bufs[i + 1], prefetch=layers[(i + 1) % L])

        with torch.cuda.stream(st):
            plain()
        torch.cuda.synchronize()
        ref = [b.clone() for b in bufs[1:]]
        with torch.cuda.stream(st):
            pref()
        torch.cuda.synchronize()
        same = all(torch.equal(a, b) for a, b in zip(ref, bufs[1:]))
        rows = {}
        for tag, fn in (("plain", plain), ("prefetch", pref), ("plain2", plain), ("prefetch2", pref)):
            rows[tag] = round(graph_time(fn, st), 3)
        wb = K * N // 2 + (K // 128) * N * 5 + 2 * M * K + 2 * M * N
        best = min(rows["prefetch"], rows["prefetch2"])
        print(json.dumps({"M": M, "layers": L, "bit_identical": same, **{k + "_us": v for k, v in rows.items()},
                          "prefetch_hbm_frac": round(wb / (best * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
