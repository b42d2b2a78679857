"""A/B of library builds on config C5's step (bench.py's denoise_loop: 12 int4 g128 layers d 4096,
seq 2048, 50 steps, KV update + fused p_sample): each build in its own subprocess (DLLM_LIB=<file>),
rounds interleaved, REPS loops per process after a clock pre-warm of the same loop.
Usage: LIBS=a.so,b.so [ROUNDS=3 REPS=2] python scripts/c5_lib_ab.py   (measurement only)."""
import json, os, subprocess, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
CODE = r"""
import sys, json, torch
sys.path.insert(0, %r)
import __graft_entry__ as g
d = g.load_package(); import scripts._lab as _lab; _lab.select(d)
import bench
dev = torch.device("cuda")
bench.denoise_loop(d, torch, dev, steps=10)   # pre-warm (clocks, workspaces)
res = [bench.denoise_loop(d, torch, dev) for _ in range(%d)]
print(json.dumps({"ms": [r["ms_per_step"] for r in res], "finite": all(r["finite"] for r in res)}))
"""
libs = os.environ["LIBS"].split(",")
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for lib in libs:
        env = dict(os.environ, DLLM_LIB=str((ROOT / lib).resolve()))
        r = subprocess.run([sys.executable, "-c", CODE % (str(ROOT), int(os.environ.get("REPS", "2")))], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"lib": lib, "round": rnd, **(json.loads(line[-1]) if line else {"error": r.stderr[-400:]})}),
              flush=True)
