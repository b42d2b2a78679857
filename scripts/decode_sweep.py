"""Decode (M <= 64) tile sweep: for each M and each (NT column tiles, K-split) configuration
(dllm_linear_set_kernel_variant 200 + 16 log2 NT + log2 nsplit; 0 = the built-in policy), the
per-layer time of a chain of L distinct 4096x4096 int4 layers (L * 9 MiB > the 256 MB Infinity
Cache, so weights stream from HBM) replayed as one HIP graph, and of one layer launched back to
back.  Prints JSON lines."""
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
Ms = [int(m) for m in os.environ.get("MS", "1,8,16,32,64").split(",")]
CFGS = [None] + [(nt, sp) for nt in (0, 1, 2) for sp in (0, 1, 2, 3)]


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
    layers = [d.QuantLinear.from_weight(0.02 * torch.randn(K, N, device=dev), None, BITS, 128) for _ in range(L)]
    wbytes = K * N * BITS // 8 + (K // 128) * N * 4
    for M in Ms:
        X = torch.randn(M, K, device=dev).half()
        bufs = [X] + [torch.empty(M, N, dtype=torch.float16, device=dev) for _ in range(L)]
        for cfg in CFGS:
            var = 4 if cfg is None else 200 + 16 * cfg[0] + cfg[1]
            for lin in layers:
                lin.set_kernel_variant(var)

            def chain():
                for i, lin in enumerate(layers):
                    lin(bufs[i], out=bufs[i + 1])
            chain()
            s1 = ev_time(lambda: layers[0](X, out=bufs[1]), 200)
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
            print(json.dumps({"M": M, "nt": "policy" if cfg is None else 1 << cfg[0], "nsplit": "policy" if cfg is None else 1 << cfg[1],
                              "single_us": round(s1 * 1e6, 2), "graph_us_per_layer": round(sg / L * 1e6, 2),
                              "graph_GBs": round(per_b * L / sg / 1e9, 1)}), flush=True)
            del gph


if __name__ == "__main__":
    main()
