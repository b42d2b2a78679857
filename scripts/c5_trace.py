"""Kernel timeline of config C5's denoise loop (bench.denoise_loop, 10 steps after a pre-warm) for
rocprofv3 --kernel-trace: the gaps between consecutive kernels show the launch overhead per step.
Usage: rocprofv3 --kernel-trace -d DIR -o c5 --output-format csv -- python3 scripts/c5_trace.py [nokv]"""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import __graft_entry__ as g
import bench

d = g.load_package()
dev = torch.device("cuda")
print(bench.denoise_loop(d, torch, dev, steps=10), flush=True)
