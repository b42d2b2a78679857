"""Kernel trace of the hidden-dim-sharded C5 step (bench.py's denoise_loop_tp, allreduce mode) on
one card: run under ``rocprofv3 --kernel-trace`` via ``torch.distributed.run --nproc-per-node 2``
with DLLM_BENCH_BACKEND=gloo.  Two marker launches (dllm_bias_cast on a 3-element row: one 256-thread block, a grid
no other bias_cast of the step uses) bracket ``TP_STEPS`` timesteps after a warm-up, so ``--analyze <kernel_trace.csv>``
lists exactly the kernels the step issues.  Measurement only."""
import json
import os
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def analyze(path):
    import collections
    import csv
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    by_thread = collections.defaultdict(list)
    for r in rows:
        by_thread[r["Thread_Id"]].append(r)
    out = {}
    for tid, rs in by_thread.items():
        marks = [i for i, r in enumerate(rs) if "bias_cast_kernel" in r["Kernel_Name"] and r["Grid_Size_X"] == "256"]
        if len(marks) < 2:
            continue
        inside = rs[marks[0] + 1:marks[-1]]
        names = collections.Counter(
            re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))
            for r in inside)
        out[tid] = {"kernels": sum(names.values()), "at_native": sum(v for k, v in names.items() if "at::native" in k),
                    "by_name": dict(names.most_common())}
    print(json.dumps(out, indent=1))


def main():
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as g
    d = g.load_package()
    par = d.parallel
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group(os.environ.get("DLLM_BENCH_BACKEND", "nccl"))
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dm, M, L, heads, steps = 4096, 2048, 12, 32, int(os.environ.get("TP_STEPS", "2"))
    c0, c1 = par.head_columns(dm, heads, world, rank)
    gen = torch.Generator(device=dev).manual_seed(99)
    pairs = []
    for _ in range(L // 2):
        WA = (0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=gen)
        WB = (0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=gen)
        pairs.append(par.TensorParallelPair(WA, None, WB, None, 4, 128, reduce=os.environ.get("MODE", "allreduce")))
        del WA, WB
    cfg = d.DiffusionConfig(num_timesteps=steps + 2, hidden_size=dm, num_layers=L, num_attention_heads=heads)
    gk = torch.Generator(device=dev).manual_seed(98)
    K = torch.randn(1, M, dm, device=dev, generator=gk)
    V = torch.randn(1, M, dm, device=dev, generator=gk)
    kv = par.HeadParallelKVCacheEntry(K[..., c0:c1].contiguous(), V[..., c0:c1].contiguous(), cfg.prefill_bits,
                                      cfg.decode_bits)
    del K, V
    x = torch.randn(M, dm, device=dev, generator=gen)
    loop = d.DenoiseLoop(pairs, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=1, kv_cache=kv, overlap=False)
    loop.sample(x, 2)
    marker = torch.zeros(1, 3, device=dev)
    torch.cuda.synchronize()
    dist.barrier()
    d.QuantLinear.bias_cast(marker, None, torch.float16)
    out = loop.sample(x, steps)
    d.QuantLinear.bias_cast(marker, None, torch.float16)
    torch.cuda.synchronize()
    dist.barrier()
    if rank == 0:
        print(json.dumps({"steps": steps, "finite": bool(torch.isfinite(out).all())}), flush=True)
    for p in pairs:
        p.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        main()
