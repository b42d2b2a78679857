"""Benchmark: int4 group-128 dequant+GEMM (the linear layer of every denoise step) on MI355X.

Workload (BASELINE.json metric, north_star shape): one step = Y[M][N] = X[M][K] . W^[K][N] + b with
M = 4096 tokens, K = N = 4096, W int4 group-128 (per-column, per-group asymmetric quantize_tensor),
X/Y f16 resident in HBM, f16 MFMA with f32 accumulation.  Synthetic data: X ~ N(0,1),
W ~ 0.02 N(0,1), b = 0 (SimpleDiffusionModel::new, diffuse-llm-rs/src/lib.rs:791-801).

Multi-GPU (--gpus N, launched by torch.distributed.run): token-parallel replicas -- every rank owns
its own M = 4096 tokens and a replica of the 8 MiB int4 weight (linear layers are per-token, so no
data-path collective exists); value = total tokens over all ranks / max-over-ranks time
("scaling": "weak").  The hidden-dim (tensor-parallel) variant with RCCL lives in
diffusion-llm-rs_amd/parallel.py (see DESIGN.md section Multi-GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_F16_TFLOPS = 2500.0   # MI355X dense f16/bf16 MFMA (MI355X_MICROARCH.md chip table)
PEAK_HBM_GBS = 8000.0      # HBM3E spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--M", type=int, default=4096)
    p.add_argument("--K", type=int, default=4096)
    p.add_argument("--N", type=int, default=4096)
    p.add_argument("--bits", type=int, default=4)
    p.add_argument("--group", type=int, default=128)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--sweep", action="store_true", help="also print an M-sweep to stderr")
    p.add_argument("--tp-steps", type=int, default=10,
                   help="N > 1: steps of the hidden-dim-sharded C5 loop reported as 'denoise_loop_tp' (0 skips)")
    p.add_argument("--no-denoise", action="store_true",
                   help="skip the config-C5 denoise-loop side measurement (reported as 'denoise_loop')")
    p.add_argument("--prewarm-ms", type=float, default=300.0,
                   help="untimed launches of the same step before the W warmup steps, so the clocks "
                        "have ramped before timing (outside the timed region)")
    return p.parse_args()


def algorithmic_bytes(M, K, N, bits, group):
    G = (K + group - 1) // group
    return K * N * bits // 8 + G * N * 5 + M * K * 2 + M * N * 2 + N * 4


def cpu_baseline(K, N, bits, group, M, budget_s):
    """The oracle's restatement of the reference path (a2 dequant of the group-quantized weight,
    then f32 x.dot(W) + b, diffuse-llm-rs/src/lib.rs:806-813), single-threaded as the reference's
    ndarray dot is; timed on a bounded row sample and extrapolated to the M-token step."""
    from oracle import oracle as orc
    rng = np.random.default_rng(0)
    W = (0.02 * rng.standard_normal((K, N))).astype(np.float32)
    codes, scales, zps = orc.quantize_weights(W, bits, group)
    t0 = time.perf_counter()
    What = orc.dequantize_weights(codes, scales, zps, group)
    t_deq = time.perf_counter() - t0
    b = np.zeros(N, np.float32)
    rows, t_rows = 4, 0.0
    X = rng.standard_normal((4, K)).astype(np.float32)
    t0 = time.perf_counter()
    orc.linear_forward(X, What, b, nthreads=1)
    t_rows = time.perf_counter() - t0
    per_row = t_rows / rows
    rows = int(max(4, min(M, (budget_s - t_deq) / max(per_row, 1e-9))))
    X = rng.standard_normal((rows, K)).astype(np.float32)
    t0 = time.perf_counter()
    orc.linear_forward(X, What, b, nthreads=1)
    t_rows = time.perf_counter() - t0
    t_step = t_deq + t_rows / rows * M
    # the same restatement on the host cores of this job's share (the GPU box
    # gives one GPU 16 CPUs; os.cpu_count() there shows the whole machine), rows split by thread.
    threads = max(1, min(16, os.cpu_count() or 1))
    rows_mt = int(max(threads, min(M, rows * threads)))
    Xm = rng.standard_normal((rows_mt, K)).astype(np.float32)
    t0 = time.perf_counter()
    orc.linear_forward(Xm, What, b, nthreads=threads)
    t_mt = time.perf_counter() - t0
    t_step_mt = t_deq + t_mt / rows_mt * M
    all_cores = {"value": M / t_step_mt, "unit": "tok/s", "cores": threads,
                 "sample": f"same restatement, {threads} threads: {rows_mt} of {M} rows ({t_mt:.2f}s), "
                           f"step extrapolated to {M} rows = {t_step_mt:.2f}s"}
    return {"value": M / t_step, "unit": "tok/s", "cores": 1, "kind": "port",
            "sample": f"C restatement (oracle/dllm_oracle.c), 1 thread: a2 dequant of the {K}x{N} int{bits} "
                      f"g{group} weight ({t_deq:.3f}s) + f32 sgemm+bias on {rows} of {M} rows "
                      f"({t_rows:.2f}s), step time extrapolated to {M} rows = {t_step:.2f}s",
            "host_cpu": _cpu_model(), "nproc": os.cpu_count(), "all_cores": all_cores}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_pmc_traffic():
    """Per-launch HBM bytes of the GEMM kernel from the committed rocprofv3 PMC summary
    (profiles/*_pmc_gemm.json, FETCH_SIZE doubled per the gfx950 note + WRITE_SIZE)."""
    files = sorted((ROOT / "profiles").glob("*_pmc_gemm.json"))
    if not files:
        return None
    try:
        d = json.loads(files[-1].read_text())
        return float(d["hbm_bytes_per_launch"])
    except Exception:
        return None


def denoise_loop(d, torch, dev, steps=50):
    """Config C5 on this rank's GPU: DiffuseLLM::sample (diffuse-llm-rs/src/lib.rs:853-955)
    over 12 int4 g128 layers of d 4096 at seq 2048, 50 steps, KV-cache update + noise on the side stream,
    p_sample fused into the last layer.  Weights 0.5/sqrt(d) N(0,1) keep the 50-step recursion finite
    (the reference's 0.02 N(0,1) overflows f32 in a 12-layer stack; the kernels do the same work).
    A side figure next to `value`, timed with HIP events on the loop's stream."""
    dm, M, L = 4096, 2048, 12
    g = torch.Generator(device=dev).manual_seed(99)
    layers = [d.QuantLinear.from_weight((0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=g), None, 4, 128)
              for _ in range(L)]
    cfg = d.DiffusionConfig(num_timesteps=steps, hidden_size=dm, num_layers=L)
    kv = d.KVCacheEntry.new(torch.randn(1, M, dm, device=dev, generator=g),
                            torch.randn(1, M, dm, device=dev, generator=g), cfg.prefill_bits, cfg.decode_bits)
    loop = d.DenoiseLoop(layers, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=1, kv_cache=kv, overlap=True)
    x = torch.randn(M, dm, device=dev, generator=g)
    loop.sample(x, 3)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    out = loop.sample(x, steps)
    e1.record(st)
    torch.cuda.synchronize()
    s = e0.elapsed_time(e1) * 1e-3
    res = {"workload": f"C5: {L} x int4-g128 d{dm} layers, seq {M}, {steps} steps, KV update + fused p_sample, 1 GPU",
           "ms_per_step": round(s / steps * 1e3, 4), "tok_per_s_per_step": round(M / (s / steps), 1),
           "gemm_tflops": round(steps * L * 2 * M * dm * dm / s / 1e12, 1),
           "finite": bool(torch.isfinite(out).all())}
    for lyr in layers:
        lyr.close()
    return res


def denoise_loop_tp(d, torch, dist, dev, world, steps):
    """Config C5 hidden-dim sharded over the job's ranks: 12 int4 layers as 6
    Megatron pairs (parallel.TensorParallelPair: column shard, row shard, one all-reduce(sum) of the
    f32 partial [2048, 4096] per pair over RCCL), p_sample after the last pair, no KV cache.
    Every rank builds the same full weights (seeded) and keeps its shard.  Timed with a barrier and
    synchronize on both sides, max over ranks."""
    par = d.parallel
    dm, M, L = 4096, 2048, 12
    g = torch.Generator(device=dev).manual_seed(99)
    pairs = []
    for _ in range(L // 2):
        WA = (0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=g)
        WB = (0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=g)
        pairs.append(par.TensorParallelPair(WA, None, WB, None, 4, 128))
        del WA, WB
    cfg = d.DiffusionConfig(num_timesteps=steps, hidden_size=dm, num_layers=L)
    loop = d.DenoiseLoop(pairs, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=1, kv_cache=None, overlap=False)
    x = torch.randn(M, dm, device=dev, generator=g)
    res = {"workload": f"C5 hidden-dim sharded: {L // 2} TensorParallelPair of int4-g128 d{dm}, seq {M}, "
                       f"{steps} steps, one all-reduce (f32 [{M}, {dm}]) per pair, p_sample, no KV cache",
           "n_ranks": world}
    for chunks in (1, 4):   # 4: each pair's all-reduce issued per token chunk, overlapping the next GEMM
        for p in pairs:
            p.chunks = chunks
        loop.sample(x, 2)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        out = loop.sample(x, steps)
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        s = float(t.item())
        key = "" if chunks == 1 else f"_chunks{chunks}"
        res["ms_per_step" + key] = round(s / steps * 1e3, 4)
        res["tok_per_s_per_step" + key] = round(M / (s / steps), 1)
        res["finite" + key] = bool(torch.isfinite(out).all())
    for p in pairs:
        p.a.local.close()
        p.b.local.close()
    return res


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DLLM_BENCH_BACKEND=gloo + device = local % device_count: a rehearsal of the N > 1 path with
    # several ranks on one GPU (the driver's multi-GPU runs use RCCL, one GPU per rank).
    backend = os.environ.get("DLLM_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    import __graft_entry__ as g
    d = g.load_package()
    d.load_library()

    M, K, N = args.M, args.K, args.N
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    W = 0.02 * torch.randn(K, N, device=dev, generator=gen)
    X = torch.randn(M, K, device=dev, generator=gen).half()
    lin = d.QuantLinear.from_weight(W, None, args.bits, args.group)
    del W
    Y = torch.empty(M, N, dtype=torch.float16, device=dev)
    stream = torch.cuda.current_stream()

    t_pre = time.perf_counter()
    while (time.perf_counter() - t_pre) * 1e3 < args.prewarm_ms:
        for _ in range(20):
            lin(X, out=Y)
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        lin(X, out=Y)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        lin(X, out=Y)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps   # HIP events on the launch stream

    t = torch.tensor([t_wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t.item())
    ms_per_step = t_max / args.steps * 1e3
    tokens = M * world * args.steps
    value = tokens / t_max

    flops = 2.0 * M * N * K
    abytes = algorithmic_bytes(M, K, N, args.bits, args.group)
    achieved_tflops = flops / (kernel_ms * 1e-3) / 1e12
    out = {
        "metric": "int4 dequant+GEMM GiB/s & tok/s per denoise step, 4096×4096, 1/2/4/8 GPU",
        "value": round(value, 1), "unit": "tok/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f16 (int4 weights)", "data": "synthetic",
        "config": {"workload": f"int{args.bits}-g{args.group} dequant+GEMM, M={M} tokens x K={K} x N={N} "
                               f"per rank (token-parallel replicas)",
                   "M": M, "K": K, "N": N, "bits": args.bits, "group": args.group,
                   "global_batch_tokens": M * world, "parallelism": f"token-replica x{world}"},
        "gib_per_s": round(abytes / (ms_per_step * 1e-3) / 2**30, 1),
        "tflops": round(flops / (ms_per_step * 1e-3) / 1e12, 1),
        "roofline": {"bound": "mfma", "achieved": round(achieved_tflops, 1), "peak": PEAK_F16_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved_tflops / PEAK_F16_TFLOPS, 4),
                     "traffic": load_pmc_traffic(), "algorithmic_bytes": abytes,
                     "kernel_ms": round(kernel_ms, 5)},
    }
    if not args.no_denoise:
        out["denoise_loop"] = denoise_loop(d, torch, dev)
        if world > 1 and args.tp_steps > 0:
            out["denoise_loop_tp"] = denoise_loop_tp(d, torch, dist, dev, world, args.tp_steps)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(K, N, args.bits, args.group, M, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if args.sweep and rank == 0:
        for m in (1, 16, 64, 256, 1024, 2048, 4096, 8192):
            xs = torch.randn(m, K, device=dev).half()
            ys = torch.empty(m, N, dtype=torch.float16, device=dev)
            for _ in range(5):
                lin(xs, out=ys)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                lin(xs, out=ys)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            b = algorithmic_bytes(m, K, N, args.bits, args.group)
            print(json.dumps({"sweep_M": m, "us": round(ms * 1e3, 2), "tflops": round(2 * m * N * K / ms / 1e9, 1),
                              "gbs": round(b / ms / 1e6, 1)}), file=sys.stderr, flush=True)
    lin.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
