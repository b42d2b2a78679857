"""A/B of library builds on the decode chain: per-layer time of L distinct 4096x4096 int4 g128 layers
(past the MALL) captured in one HIP graph, at several M <= 64; each build in its own subprocess
(DLLM_LIB=<file>), rounds interleaved; a bit-level hash of the chain's output shows whether the builds
compute the same bits.  Usage: LIBS=a.so,b.so [MS=1,16,32,64] python scripts/decode_lib_ab.py"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CODE = r"""
import sys, json, time, torch
sys.path.insert(0, %r)
import __graft_entry__ as g
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
K = N = 4096
L = 40
gen = torch.Generator(device="cuda").manual_seed(7)
layers = [d.QuantLinear.from_weight((0.5 / 64) * torch.randn(K, N, device="cuda", generator=gen), None, 4, 128)
          for _ in range(L)]
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
out = {}
for M in [int(m) for m in %r.split(",")]:
    X = torch.randn(M, K, device="cuda", generator=gen).half()
    bufs = [X] + [torch.empty(M, N, dtype=torch.float16, device="cuda") for _ in range(L)]
    def chain():
        for i, lin in enumerate(layers):
            lin(bufs[i], out=bufs[i + 1])
    with torch.cuda.stream(st):
        chain()
        torch.cuda.synchronize()
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph, stream=st):
            chain()
    torch.cuda.synchronize()
    t0 = time.time()
    while time.time() - t0 < 0.2:
        gph.replay()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        gph.replay()
    e1.record()
    torch.cuda.synchronize()
    h = int(bufs[-1].view(torch.int16).to(torch.int64).sum().item())
    out[M] = {"us": round(e0.elapsed_time(e1) / 10 / L * 1e3, 3), "yhash": h}
print(json.dumps(out))
"""
libs = os.environ["LIBS"].split(",")
ms = os.environ.get("MS", "1,16,32,64")
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for lib in libs:
        env = dict(os.environ, DLLM_LIB=str((ROOT / lib).resolve()))
        r = subprocess.run([sys.executable, "-c", CODE % (str(ROOT), ms)], env=env, capture_output=True, text=True,
                           timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"lib": lib, "round": rnd, **(json.loads(line[-1]) if line else {"error": r.stderr[-400:]})}),
              flush=True)
