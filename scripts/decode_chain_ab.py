"""A/B of library builds on the decode / mid-M chain (bench.py m_sweep's method): a chain of 40
distinct int4 g128 K x N layers (weights from HBM) captured in one HIP graph per M and replayed;
each build in its own subprocess (DLLM_LIB=<file>), rounds interleaved; a bit hash of the last
layer's Y shows whether builds agree.  Usage: LIBS=a.so,b.so [MS=1,4,16] [POS=0,1] python scripts/decode_chain_ab.py  (POS=1: the same
layers as prefill-only handles, so every M runs the exact prefill kernels)"""
import json, os, subprocess, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
CODE = r"""
import sys, json, time, torch
sys.path.insert(0, %r)
import __graft_entry__ as g
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
gen = torch.Generator(device="cuda").manual_seed(99)
import os
K = 4096; N = int(os.environ.get("AB_N", "4096"))
po = os.environ.get("PO") == "1"   # prefill-only handles: M <= 64 runs the exact prefill kernels
chain = [d.QuantLinear.from_weight(0.02 * torch.randn(K, N, device="cuda", generator=gen), None, 4, 128, prefill_only=po) for _ in range(40)]
out = {}
for m in (int(v) for v in %r.split(",")):
    xs = torch.randn(m, K, device="cuda", generator=gen).half()
    ys = torch.empty(m, N, dtype=torch.float16, device="cuda")
    cs = torch.cuda.Stream(); cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        for l in chain: l(xs, out=ys)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=cs):
        for l in chain: l(xs, out=ys)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2: gr.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); gr.replay(); gr.replay(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 80 * 1e3)
    ts.sort()
    h = int(ys.view(torch.int16).to(torch.int64).mul(torch.arange(ys.numel(), device="cuda").view(m, N) %% 65521 + 1).sum())
    out[str(m)] = {"us": round(ts[3], 3), "us_min": round(ts[0], 3), "yhash": h}
    del gr
for l in chain: l.close()
print(json.dumps(out))
"""
libs = os.environ["LIBS"].split(",")
ms = os.environ.get("MS", "1,2,4,8,16,17,32,64")
pos = os.environ.get("POS", "0").split(",")
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for lib, po in ((l, p) for l in libs for p in pos):
        env = dict(os.environ, DLLM_LIB=str((ROOT / lib).resolve()), PO=po)
        res = subprocess.run([sys.executable, "-c", CODE % (str(ROOT), ms)], env=env, capture_output=True, text=True,
                             timeout=300)
        line = [l for l in res.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"lib": lib + ("+prefill_only" if po == "1" else ""), "round": rnd, **(json.loads(line[-1]) if line else {"error": res.stderr[-600:]})}),
              flush=True)
