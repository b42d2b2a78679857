"""Small-M (decode) dequant+GEMM lab: per-launch time of one 4096x4096 int4 layer, and a chain of
L distinct layers (L*9 MiB > the 256 MB Infinity Cache, so the weights really stream from HBM)
run eagerly and as one captured HIP graph.  Prints JSON lines."""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

import __graft_entry__ as g

d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
dev = torch.device("cuda")
K = N = int(os.environ.get("DIM", "4096"))
L = int(os.environ.get("LAYERS", "48"))
BITS = int(os.environ.get("BITS", "4"))
Ms = [int(m) for m in os.environ.get("MS", "1,4,16,32,64").split(",")]


def ev_time(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    big = torch.empty(1 << 28, dtype=torch.uint8, device=dev)
    big2 = torch.empty_like(big)
    s = ev_time(lambda: big2.copy_(big), 20)
    print(json.dumps({"probe": "d2d copy 256 MiB", "GBs": round(2 * big.numel() / s / 1e9, 1)}), flush=True)
    small = big[: 9 << 20]
    small2 = big2[: 9 << 20]
    s = ev_time(lambda: small2.copy_(small), 200)
    print(json.dumps({"probe": "d2d copy 9 MiB (back-to-back)", "us": round(s * 1e6, 2)}), flush=True)
    del big, big2

    layers = [d.QuantLinear.from_weight(0.02 * torch.randn(K, N, device=dev), None, BITS, 128) for _ in range(L)]
    wbytes = K * N * BITS // 8 + (K // 128) * N * 4
    for M in Ms:
        X = torch.randn(M, K, device=dev).half()
        Y = torch.empty(M, N, dtype=torch.float16, device=dev)
        s1 = ev_time(lambda: layers[0](X, out=Y), 200)
        bufs = [X] + [torch.empty(M, N, dtype=torch.float16, device=dev) for _ in range(L)]

        def chain():
            for i, lin in enumerate(layers):
                lin(bufs[i], out=bufs[i + 1])
        chain()
        se = ev_time(chain, 10)
        gph = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            chain()
            torch.cuda.synchronize()
            with torch.cuda.graph(gph, stream=st):
                chain()
        torch.cuda.synchronize()
        sg = ev_time(gph.replay, 20)
        per_b = wbytes + 2 * M * K + 2 * M * N
        print(json.dumps({"M": M, "single_us": round(s1 * 1e6, 2),
                          "chain_eager_us_per_layer": round(se / L * 1e6, 2),
                          "chain_graph_us_per_layer": round(sg / L * 1e6, 2),
                          "graph_GBs": round(per_b * L / sg / 1e9, 1),
                          "graph_hbm_frac": round(per_b * L / sg / 8e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
