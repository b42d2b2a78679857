"""Benchmark: int4 group-128 dequant+GEMM (the linear layer of every denoise step) on MI355X.

Workload (BASELINE.json metric, north_star shape): one step = Y[M][N] = X[M][K] . W^[K][N] + b with
M = 4096 tokens, K = N = 4096, W int4 group-128 (per-column, per-group asymmetric quantize_tensor),
X/Y f16 resident in HBM, f16 MFMA with f32 accumulation, the library's default precision
(DLLM_PRECISION_EXACT: the MFMA consumes the exact integer q - zp, the f32 group scale is applied
to each group's partial sum).  The rounded-weight mode (DLLM_PRECISION_F16W) is timed beside it
as ``f16_weights``.  Synthetic data: X ~ N(0,1), W ~ 0.02 N(0,1), b = 0 (SimpleDiffusionModel::new,
diffuse-llm-rs/src/lib.rs:791-801).

Multi-GPU (--gpus N, one process per GPU: launched by torch.distributed.run, or -- when WORLD_SIZE
is unset -- by bench.py itself, which starts N fresh rank processes before anything touches the
GPU; a WORLD_SIZE that differs from --gpus is an error): the SAME fixed
4096-token step is split over the ranks by hidden (output) dimension -- column-parallel, rank r
owns the group-aligned columns [n0, n1) of W (parallel.ColumnParallelLinear), X replicated -- and
the step ends with the full [M, N] Y on every rank, as x.dot(W) + b returns it (lib.rs:812): the
rank's slice GEMM + one RCCL all-gather of the f16 slices (``forward_gathered``).  ``value`` =
4096 tokens per step / max-over-ranks time of that whole step ("scaling": "strong", ``value_from``
says so); the slice GEMM alone is the side key ``kernel_only``.  Token-parallel replicas (each
rank its own 4096 tokens) are a side key (``replicas``, weak scaling), config C5 hidden-dim
sharded over RCCL is ``denoise_loop_tp`` and C5 token-parallel (each rank its 2048 / N tokens of
the sample, replicated weights) ``denoise_loop_dp``.
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
# Revision tag of the default prefill GEMM kernel; a PMC record's traffic is quoted only when its
# config carries the same tag (r04-horner16b: wq_horner16_kernel of linear_horner.hip, the 256 x 256
# Horner-form exact kernel on 16x16x32 MFMAs, conflict-free X swizzle, half 1's A fragments built
# behind substep 1, stage DMA pieces spread between MFMA pairs, the LDS-staged coalesced f16 store
# written with non-temporal 16-B stores).
GEMM_REV = "r04-horner16b"


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
    p.add_argument("--sweep", action="store_true", help="rank 0 at N = 1: add the local layer's M-sweep (m_sweep) to the JSON line")
    p.add_argument("--tp-steps", type=int, default=10,
                   help="N > 1: steps of the hidden-dim-sharded C5 loop reported as 'denoise_loop_tp' (0 skips)")
    p.add_argument("--dp-steps", type=int, default=50,
                   help="N > 1: steps of the token-parallel C5 loop reported as 'denoise_loop_dp' (0 skips)")
    p.add_argument("--gather-chunks", type=int, default=2,
                   help="N > 1: token chunks of the headline step's all-gather (chunk i's gather overlaps "
                        "chunk i+1's GEMM; 2 by default: priced in DESIGN.md section 6)")
    p.add_argument("--no-denoise", action="store_true",
                   help="skip the config-C5 denoise-loop side measurement (reported as 'denoise_loop')")
    p.add_argument("--prewarm-ms", type=float, default=300.0,
                   help="untimed launches of the same step before the W warmup steps, so the clocks "
                        "have ramped before timing (outside the timed region)")
    a = p.parse_args()
    for name in ("tp_steps", "dp_steps"):
        if getattr(a, name) == 1:
            # a 1-step schedule is the reference's degenerate linear schedule (0/0 in the beta ramp,
            # lib.rs:554-593): its output is NaN by construction, so it measures nothing useful
            p.error(f"--{name.replace('_', '-')} must be 0 (skip) or >= 2")
    return a


def algorithmic_bytes(M, K, N, bits, group):
    G = (K + group - 1) // group
    return K * N * bits // 8 + G * N * 5 + M * K * 2 + M * N * 2 + N * 4


def cpu_baseline(K, N, bits, group, M, budget_s):
    """The reference path on the host: a2 dequant of the group-quantized weight (the oracle's C
    restatement), then the f32 ``x.dot(W) + b`` of diffuse-llm-rs/src/lib.rs:806-813 by a blocked
    AVX2/FMA sgemm (oracle/dllm_sgemm.c) -- the class of kernel ndarray's ``dot`` runs
    (matrixmultiply) -- on 1 thread (the reference is single-threaded) over as many of the M rows
    as the budget allows, and on the job's host-core share over all M rows."""
    from oracle import oracle as orc
    rng = np.random.default_rng(0)
    W = (0.02 * rng.standard_normal((K, N))).astype(np.float32)
    codes, scales, zps = orc.quantize_weights(W, bits, group)
    t0 = time.perf_counter()
    What = orc.dequantize_weights(codes, scales, zps, group)
    t_deq = time.perf_counter() - t0
    b = np.zeros(N, np.float32)
    X = rng.standard_normal((M, K)).astype(np.float32)
    orc.sgemm_blocked(X[:64], What, b, nthreads=1)                  # page-in / warm
    t0 = time.perf_counter()
    orc.sgemm_blocked(X[:256], What, b, nthreads=1)
    per_row = (time.perf_counter() - t0) / 256
    rows = int(max(256, min(M, (budget_s - t_deq) / max(per_row, 1e-9))))
    t0 = time.perf_counter()
    orc.sgemm_blocked(X[:rows], What, b, nthreads=1)
    t_rows = time.perf_counter() - t0
    t_step = t_deq + t_rows / rows * M
    extrap = "" if rows == M else f", extrapolated from {rows} rows"
    # the same on the host cores this process may run on (its affinity mask;
    # os.cpu_count() on the GPU box shows the whole machine), capped at the job's 16-CPU share.
    threads = host_threads()
    orc.sgemm_blocked(X[:256], What, b, nthreads=threads)
    t0 = time.perf_counter()
    orc.sgemm_blocked(X, What, b, nthreads=threads)
    t_mt = t_deq + time.perf_counter() - t0
    gf = 2.0 * M * K * N / 1e9
    all_cores = {"value": M / t_mt, "unit": "tok/s", "cores": threads,
                 "sample": f"same path on {threads} threads (affinity mask {len(os.sched_getaffinity(0))} CPUs, "
                           f"capped at the job's 16), all {M} rows: {t_mt:.3f}s per step "
                           f"({gf / (t_mt - t_deq):.0f} GFLOP/s sgemm)"}
    return {"value": M / t_step, "unit": "tok/s", "cores": 1, "kind": "port",
            "sample": f"1 thread: a2 dequant of the {K}x{N} int{bits} g{group} weight ({t_deq:.3f}s, C restatement) "
                      f"+ blocked AVX2/FMA sgemm (6x16 micro-tile, KC 256, MC 72; matrixmultiply's class) + bias on "
                      f"{rows} of {M} rows ({t_rows:.2f}s, {2.0 * rows * K * N / t_rows / 1e9:.0f} GFLOP/s){extrap}; "
                      f"step {t_step:.3f}s",
            "host_cpu": _cpu_model(), "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "multi_thread": all_cores}


def cpu_denoise_step(dm=4096, M=2048, L=12, bits=4, group=128):
    """SURVEY.md 8d's C5 CPU plan: one denoise step of the reference path on the host = L layers of
    (a2 dequant + f32 sgemm of M tokens x dm^2 + b) + p_sample; one layer is timed on 1 thread and on
    the job's host-core share and multiplied by L (the elementwise p_sample is < 0.1 % of a layer and
    not timed): labelled an extrapolation."""
    from oracle import oracle as orc
    rng = np.random.default_rng(1)
    W = (0.02 * rng.standard_normal((dm, dm))).astype(np.float32)
    codes, scales, zps = orc.quantize_weights(W, bits, group)
    t0 = time.perf_counter()
    What = orc.dequantize_weights(codes, scales, zps, group)
    t_deq = time.perf_counter() - t0
    b = np.zeros(dm, np.float32)
    X = rng.standard_normal((M, dm)).astype(np.float32)
    res = {}
    for threads in (1, host_threads()):
        orc.sgemm_blocked(X[:64], What, b, nthreads=threads)
        t0 = time.perf_counter()
        orc.sgemm_blocked(X, What, b, nthreads=threads)
        t_layer = t_deq + time.perf_counter() - t0
        res[f"{threads}_threads"] = {"ms_per_step": round(1e3 * L * t_layer, 1),
                                     "tok_per_s_per_step": M / (L * t_layer)}
    res["sample"] = (f"one layer (a2 dequant + blocked AVX2 sgemm {M}x{dm}x{dm} + b) timed per thread count, "
                     f"x {L} layers = one denoise step (extrapolated; p_sample not timed)")
    return res


def host_threads():
    """Threads for the multi-threaded CPU baseline: the CPUs of this process's affinity mask
    (os.sched_getaffinity), at most the 16 a one-GPU job is given."""
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_pmc_traffic(cfg):
    """Per-launch HBM bytes of the bench GEMM from a committed rocprofv3 PMC record whose recorded
    config (M, K, N_local, bits, group) equals this run's (profiles/**/pmc_gemm.json written by
    scripts/pmc_to_json.py: FETCH_SIZE doubled per the gfx950 calibration + WRITE_SIZE).  None when
    no record matches: the figure is never carried over to another shape."""
    best = None
    for f in sorted((ROOT / "profiles").glob("**/pmc_gemm.json")):
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        if d.get("config") == cfg and "hbm_bytes_per_launch" in d:
            best = (float(d["hbm_bytes_per_launch"]), str(f.relative_to(ROOT)))
    return best


def denoise_loop(d, torch, dev, steps=50):
    """Config C5 on this rank's GPU: DiffuseLLM::sample (diffuse-llm-rs/src/lib.rs:853-955)
    over 12 int4 g128 layers of d 4096 at seq 2048, 50 steps, KV-cache update + noise on the side stream,
    p_sample fused into the last layer.  Weights 0.5/sqrt(d) N(0,1) keep the 50-step recursion finite
    (the reference's 0.02 N(0,1) overflows f32 in a 12-layer stack; the kernels do the same work).
    A side figure next to `value`, timed with HIP events on the loop's stream."""
    dm, M, L = 4096, 2048, 12
    g = torch.Generator(device=dev).manual_seed(99)
    layers = [d.QuantLinear.from_weight((0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=g), None, 4, 128,
                                        prefill_only=True)   # M = 2048 only: no decode layout
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


class _ComputeOnlyPair:
    """A TensorParallelPair's two local GEMMs without its reduction: times the sharded loop's compute
    alone (report compute-only and end-to-end scaling separately; the values are the
    rank's un-reduced partials, so only the timing means anything)."""

    def __init__(self, pair):
        self.pair = pair

    def __call__(self, x, out_dtype=None):
        y = self.pair.partial(x)
        return y if out_dtype is None or y.dtype == out_dtype else y.to(out_dtype)


def denoise_loop_tp(d, torch, dist, dev, world, steps):
    """Config C5 hidden-dim sharded over the job's ranks, the same work per step as
    ``denoise_loop``: 12 int4 layers as 6 Megatron pairs (parallel.TensorParallelPair: column shard,
    row shard, one reduction of the f32 partial [2048, 4096] per pair over RCCL), p_sample after the
    last pair, and the KV step of every timestep on the head-sharded phase-aware cache
    (parallel.HeadParallelKVCacheEntry: the rank's 32/N heads of K, V [1, 2048, 4096]; phase switch,
    progressive decode widths, one all_reduce(MAX) of 4 floats per update, both widths from it).
    Every rank builds the same full weights and K/V (seeded) and keeps its shard.  Each reduction
    mode is timed with a barrier and synchronize on both sides, max over ranks: "allreduce" (f32
    all_reduce, then bias + f16 cast) and "rs_ag" (f32 reduce_scatter over token rows, cast on the
    local rows, f16 all_gather: 3/4 of the bytes), each unchunked and with the reduction split into 4
    token chunks that overlap the next chunk's GEMM.  "compute_only": the same loop with each pair's
    reduction left out (the GEMMs, casts, KV step and p_sample only).  Serial schedule (the KV step
    and its 4-float all-reduce in stream order before the layers)."""
    par = d.parallel
    dm, M, L, heads = 4096, 2048, 12, 32
    rank = dist.get_rank()
    c0, c1 = par.head_columns(dm, heads, world, rank)
    res = {"workload": f"C5 hidden-dim sharded: {L // 2} TensorParallelPair of int4-g128 d{dm}, seq {M}, "
                       f"{steps} steps, one reduction of the f32 [{M}, {dm}] partial per pair, p_sample, KV step on "
                       f"the head-sharded phase-aware cache ({heads // world} of {heads} heads per rank)",
           "n_ranks": world, "schedule": "serial (KV step and its all-reduce in stream order, overlap=False)"}

    def kv_cache(cfg):
        gk = torch.Generator(device=dev).manual_seed(98)
        K = torch.randn(1, M, dm, device=dev, generator=gk)
        V = torch.randn(1, M, dm, device=dev, generator=gk)
        kv = par.HeadParallelKVCacheEntry(K[..., c0:c1].contiguous(), V[..., c0:c1].contiguous(), cfg.prefill_bits,
                                          cfg.decode_bits)
        del K, V
        return kv

    for mode in ("allreduce", "rs_ag"):
        g = torch.Generator(device=dev).manual_seed(99)
        pairs = []
        for _ in range(L // 2):
            WA = (0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=g)
            WB = (0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=g)
            pairs.append(par.TensorParallelPair(WA, None, WB, None, 4, 128, reduce=mode))
            del WA, WB
        cfg = d.DiffusionConfig(num_timesteps=steps, hidden_size=dm, num_layers=L, num_attention_heads=heads)
        x = torch.randn(M, dm, device=dev, generator=g)
        for chunks in (1, 4):   # 4: each pair's reduction issued per token chunk, overlapping the next GEMM
            for p in pairs:
                p.chunks = chunks
            loop = d.DenoiseLoop(pairs, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=1, kv_cache=kv_cache(cfg),
                                 overlap=False)
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
            key = f"{mode}_chunks{chunks}"
            res[key] = {"ms_per_step": round(s / steps * 1e3, 4), "tok_per_s_per_step": round(M / (s / steps), 1),
                        "finite": bool(torch.isfinite(out).all())}
        if mode == "allreduce":
            loop_c = d.DenoiseLoop([_ComputeOnlyPair(p) for p in pairs], cfg, cumprod=d.Cumprod.INCLUSIVE, seed=1,
                                   kv_cache=kv_cache(cfg), overlap=False)
            loop_c.sample(x, 2)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            loop_c.sample(x, steps)
            torch.cuda.synchronize()
            dist.barrier()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            s = float(t.item())
            res["compute_only"] = {"ms_per_step": round(s / steps * 1e3, 4),
                                   "tok_per_s_per_step": round(M / (s / steps), 1),
                                   "note": "the pairs' local GEMMs + casts + KV step + p_sample, no pair reduction "
                                           "(timing only)"}
        for p in pairs:
            p.close()
    return res


def denoise_loop_dp(d, torch, dist, dev, world, steps):
    """Config C5 token-parallel over the job's ranks (SURVEY.md 8e's exchange-free form): rank r runs
    its 2048 / N token rows (parallel.token_rows) of the same sample through the same 12 int4 layers
    (replicated weights: the linear layers and p_sample are per token), drawing the noise those rows
    get in the unsharded loop (DenoiseLoop noise_rows), with its token rows of K, V [1, 2048, 4096]
    in the sharded phase-aware cache (parallel.HeadParallelKVCacheEntry: one all_reduce(MAX) of 4
    floats per quantization, both widths from it).  The same work per step as ``denoise_loop``;
    timed between barriers, max over ranks.  Serial schedule (the KV step and its 4-float
    all-reduce in stream order before the layers)."""
    par = d.parallel
    dm, M, L = 4096, 2048, 12
    rank = dist.get_rank()
    r0, r1 = par.token_rows(M, world, rank)
    g = torch.Generator(device=dev).manual_seed(99)
    layers = [d.QuantLinear.from_weight((0.5 / 64.0) * torch.randn(dm, dm, device=dev, generator=g), None, 4, 128,
                                        prefill_only=True) for _ in range(L)]
    cfg = d.DiffusionConfig(num_timesteps=steps, hidden_size=dm, num_layers=L)
    K = torch.randn(1, M, dm, device=dev, generator=g)
    V = torch.randn(1, M, dm, device=dev, generator=g)
    x = torch.randn(M, dm, device=dev, generator=g)[r0:r1].contiguous()
    kv = par.HeadParallelKVCacheEntry(K[:, r0:r1].contiguous(), V[:, r0:r1].contiguous(), cfg.prefill_bits,
                                      cfg.decode_bits)
    del K, V
    loop = d.DenoiseLoop(layers, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=1, kv_cache=kv, overlap=False,
                         noise_rows=(r0, M))
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
    res = {"workload": f"C5 token-parallel: {L} x int4-g128 d{dm} layers replicated, {M // world} of {M} tokens "
                       f"per rank, {steps} steps, KV step on the rank's token rows (one 4-float all_reduce(MAX) per "
                       f"quantization), p_sample fused in the last layer",
           "n_ranks": world, "ms_per_step": round(s / steps * 1e3, 4), "tok_per_s_per_step": round(M / (s / steps), 1),
           "finite": bool(torch.isfinite(out).all()),
           "schedule": "serial (KV step and its all-reduce in stream order, overlap=False); denoise_loop (1 GPU) "
                       "overlaps the KV step on a side stream, so the two are not like-for-like"}
    for lyr in layers:
        lyr.close()
    return res


def headline(world, M, steps, t_slice, t_full=None, chunks=1):
    """``value`` / ``ms_per_step`` of the JSON line and where they come from.  N = 1: the GEMM step
    (t_slice).  N > 1: the WHOLE step on every rank -- the column-slice GEMM plus the all-gather of
    the slices into the full [M, N] Y (t_full; lib.rs:812 returns the full Y) -- with the slice GEMM
    alone kept as the side key ``kernel_only`` (no rank holds the full Y there)."""
    if world == 1:
        return {"value": M * steps / t_slice, "ms_per_step": t_slice / steps * 1e3, "value_from": "gemm"}
    if t_full is None:
        raise ValueError("N > 1: the headline needs the gathered step's time")
    return {"value": M * steps / t_full, "ms_per_step": t_full / steps * 1e3,
            "value_from": f"gemm+allgather (chunks={chunks})",
            "kernel_only": {"value": round(M * steps / t_slice, 1), "ms_per_step": round(t_slice / steps * 1e3, 5),
                            "note": "the rank's column-slice GEMM alone (kernel only: the full Y exists on no "
                                    "rank; not the headline)"}}


def _timed(fn, steps, stream, torch, dist, world, dev):
    """``steps`` calls of ``fn`` bracketed by barrier + synchronize; returns (max-over-ranks wall
    seconds, this rank's HIP-event ms per call on ``stream``)."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        fn()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_wall = time.perf_counter() - t0
    t = torch.tensor([t_wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), ev0.elapsed_time(ev1) / steps


def m_sweep(lin, K, N, bits, group, torch, dev, stream, n_layers=40):
    """Per-M kernel time over a chain of ``n_layers`` DISTINCT int{bits}-g{group} layers of the same
    shape, launched back to back -- 40 x (9.1 MiB prefill + 8.5 MiB decode layout) is well past the
    256 MiB MALL, so every launch reads its weights from HBM, as a model's layer stack does.  The
    chain is captured once in a HIP graph and replayed (one warm replay, two timed: HIP events), so
    the host's per-call cost is not in the figure.  ``hot_us`` is 20 graph-captured launches on ONE
    layer (weights L2/MALL-resident: an upper bound, not a layer time)."""
    gen = torch.Generator(device=dev).manual_seed(99)
    chain = []
    for _ in range(n_layers):
        Wl = 0.02 * torch.randn(K, N, device=dev, generator=gen)
        chain.append(type(lin).from_weight(Wl, None, bits, group))
        del Wl
    rows = []
    for m in (1, 16, 64, 256, 384, 512, 1024, 2048, 4096, 8192):
        xs = torch.randn(m, K, device=dev).half()
        ys = torch.empty(m, N, dtype=torch.float16, device=dev)
        cs = torch.cuda.Stream()   # split-K workspaces are per stream: size them on the capture stream
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            for lyr in chain + [lin]:
                lyr(xs, out=ys)
        torch.cuda.synchronize()
        per = {}
        for tag, seq in (("chain", chain), ("hot", [lin] * 20)):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cs):
                for lyr in seq:
                    lyr(xs, out=ys)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            per[tag] = e0.elapsed_time(e1) / (2 * len(seq))
            del g
        ms = per["chain"]
        b = algorithmic_bytes(m, K, N, bits, group)
        rows.append({"M": m, "us": round(ms * 1e3, 2), "tflops": round(2 * m * N * K / ms / 1e9, 1),
                     "gbs": round(b / ms / 1e6, 1), "hbm_frac": round(b / ms / 1e6 / PEAK_HBM_GBS, 4),
                     "hot_us": round(per["hot"] * 1e3, 2)})
    for lyr in chain:
        lyr.close()
    return {"layers": n_layers, "timing": "HIP graph replay, HIP events", "rows": rows}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, script=None):
    """``bench.py --gpus N`` run without a launcher: start N fresh rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their env, rendezvous on 127.0.0.1) and return the
    first non-zero exit code (else 0).  Called before anything imports torch or touches the GPU, and
    the children are new processes, never an exec of this one; rank 0 prints the JSON line."""
    import signal
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, str(script or Path(__file__).resolve()), *argv], env=env))

    def stop_all():
        for q in procs:
            if q.poll() is None:
                q.send_signal(signal.SIGTERM)

    rc = 0
    try:
        # Poll every child: whichever rank fails first stops the others at once (a rank blocked in
        # a collective on a dead peer would otherwise hang until the collective's timeout).
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c is not None and c != 0]
            if bad and rc == 0:
                rc = bad[0]
                stop_all()
            if all(c is not None for c in codes):
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        stop_all()
        raise
    return rc if rc >= 0 else 128 - rc


def check_world(gpus, env):
    """The job's world size must be the --gpus it was asked for: returns (world, error or None).
    WORLD_SIZE unset means a single process, i.e. --gpus 1 (--gpus > 1 is spawned by main)."""
    world = int(env.get("WORLD_SIZE", "1"))
    if world != gpus:
        return world, (f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: the launcher started a different number "
                       f"of ranks than asked for")
    return world, None


def main():
    args = parse()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world, err = check_world(args.gpus, os.environ)
    if err:
        sys.exit(err)
    import torch
    import torch.distributed as dist

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
    gen = torch.Generator(device=dev).manual_seed(1234)       # the same W and X on every rank
    W = 0.02 * torch.randn(K, N, device=dev, generator=gen)
    X = torch.randn(M, K, device=dev, generator=gen).half()
    col = d.parallel.ColumnParallelLinear(W, None, args.bits, args.group, gather=False)
    lin = col.local
    n_local = col.n1 - col.n0
    Y = torch.empty(M, n_local, dtype=torch.float16, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        lin(X, out=Y)

    t_pre = time.perf_counter()
    while (time.perf_counter() - t_pre) * 1e3 < args.prewarm_ms:
        for _ in range(20):
            step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    # the rank's slice GEMM alone: the roofline kernel (HIP events on its stream); at N = 1 this IS
    # the step
    t_slice, kernel_ms = _timed(step, args.steps, stream, torch, dist, world, dev)
    t_full = None
    if world > 1:
        # the whole step on every rank: Y = x.dot(W) + b as the full [M, N] (lib.rs:806-813) = the
        # rank's column-slice GEMM + the RCCL all-gather of the f16 slices into Y's rows
        # (ColumnParallelLinear.forward_gathered; --gather-chunks > 1 overlaps chunk i's gather with
        # chunk i+1's GEMM)
        Yfull = torch.empty(M, N, dtype=torch.float16, device=dev)

        def step_full():
            col.forward_gathered(X, out=Yfull, stage=Y, chunks=args.gather_chunks)
        for _ in range(max(2, args.warmup)):
            step_full()
        t_full, _ = _timed(step_full, args.steps, stream, torch, dist, world, dev)
    head = headline(world, M, args.steps, t_slice, t_full, args.gather_chunks)
    value, ms_per_step = head["value"], head["ms_per_step"]

    flops_local = 2.0 * M * n_local * K
    abytes_local = algorithmic_bytes(M, K, n_local, args.bits, args.group)
    achieved_tflops = flops_local / (kernel_ms * 1e-3) / 1e12
    pmc_cfg = {"M": M, "K": K, "N_local": n_local, "bits": args.bits, "group": args.group, "rev": GEMM_REV}
    pmc = load_pmc_traffic(pmc_cfg)
    out = {
        "metric": "int4 dequant+GEMM GiB/s & tok/s per denoise step, 4096×4096, 1/2/4/8 GPU",
        "value": round(value, 1), "unit": "tok/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f16 X x exact int4 weights (f32 group scales), f32 accumulate",
        "data": "synthetic",
        "config": {"workload": (f"int{args.bits}-g{args.group} dequant+GEMM, M={M} tokens x K={K} x N={N}" +
                                ("" if world == 1 else
                                 f", N split column-parallel over {world} ranks ({n_local} columns on rank 0) + "
                                 f"RCCL all-gather of the f16 slices: the full [M, N] Y on every rank")),
                   "M": M, "K": K, "N": N, "bits": args.bits, "group": args.group,
                   "global_batch_tokens": M, "parallelism": f"column-parallel (hidden dim) x{world}" +
                                                            ("" if world == 1 else " + all-gather")},
        "value_from": head["value_from"],
        "gib_per_s": round(algorithmic_bytes(M, K, N, args.bits, args.group) / (ms_per_step * 1e-3) / 2**30, 1),
        "tflops": round(2.0 * M * N * K / (ms_per_step * 1e-3) / 1e12, 1),
        "roofline": {"bound": "mfma", "achieved": round(achieved_tflops, 1), "peak": PEAK_F16_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved_tflops / PEAK_F16_TFLOPS, 4),
                     "traffic": None if pmc is None else pmc[0],
                     "traffic_source": None if pmc is None else pmc[1],
                     "algorithmic_bytes": abytes_local, "kernel_ms": round(kernel_ms, 5),
                     "kernel": f"rank 0's local GEMM, M={M} x K={K} x N={n_local}"},
    }
    if "kernel_only" in head:
        out["kernel_only"] = head["kernel_only"]
    if world > 1:
        full = d.QuantLinear.from_weight(W, None, args.bits, args.group)
        Yf = torch.empty(M, N, dtype=torch.float16, device=dev)
        for _ in range(args.warmup):
            full(X, out=Yf)
        tr, _ = _timed(lambda: full(X, out=Yf), args.steps, stream, torch, dist, world, dev)
        out["replicas"] = {"value": round(M * world * args.steps / tr, 1), "scaling": "weak",
                           "ms_per_step": round(tr / args.steps * 1e3, 5),
                           "note": f"token-parallel replicas: each rank its own {M} tokens x the full weight"}
        full.close()
    if world == 1:
        # the rounded-weight mode on the same weights (side figure; same HIP-event timing)
        lin16 = d.QuantLinear.from_weight(W, None, args.bits, args.group, d.linear.F16W)
        for _ in range(args.warmup):
            lin16(X, out=Y)
        _, k16 = _timed(lambda: lin16(X, out=Y), args.steps, stream, torch, dist, world, dev)
        t16 = flops_local / (k16 * 1e-3) / 1e12
        out["f16_weights"] = {"kernel_ms": round(k16, 5), "achieved_tflops": round(t16, 1),
                              "frac": round(t16 / PEAK_F16_TFLOPS, 4), "value": round(M / (k16 * 1e-3), 1),
                              "note": "DLLM_PRECISION_F16W: weight rounded to f16 before the MFMA (~2.7e-4 "
                                      "more relative error per layer); kernel time only"}
        lin16.close()
    del W
    if not args.no_denoise:
        out["denoise_loop"] = denoise_loop(d, torch, dev)
        if world > 1 and args.tp_steps > 0:
            out["denoise_loop_tp"] = denoise_loop_tp(d, torch, dist, dev, world, args.tp_steps)
        if world > 1 and args.dp_steps > 0:
            if world > 2048:
                raise SystemExit("denoise_loop_dp: the token-parallel loop needs world <= 2048 tokens")
            out["denoise_loop_dp"] = denoise_loop_dp(d, torch, dist, dev, world, args.dp_steps)
    if args.sweep and rank == 0 and world == 1:
        out["m_sweep"] = m_sweep(lin, K, N, args.bits, args.group, torch, dev, stream)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(K, N, args.bits, args.group, M, args.cpu_seconds)
        if "denoise_loop" in out:
            out["denoise_loop"]["cpu_baseline"] = cpu_denoise_step()
    if rank == 0:
        print(json.dumps(out), flush=True)
    lin.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
