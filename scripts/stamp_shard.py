"""Phase breakdown of the exact-weight fold GEMM (wq_gemm_exact_kernel) on the column-shard shapes,
from in-kernel s_memtime stamps (prologue fill / steady k-step / epilogue).

Needs the stamp build:  make -C diffusion-llm-rs_amd/csrc variant VNAME=stamp VFLAGS=-DDLLM_STAMP=1
(lib/libdllm_hip_stamp.so; the product build compiles every stamp hook to nothing).  Per shape: a
300 ms clock pre-warm of back-to-back launches, then one stamped launch; every (block, wave) row
holds s_memtime at entry, after the prologue barrier, at the end of each k-step's MFMA issue and
after its barrier, before the epilogue stores and at exit, plus s_memrealtime (100 MHz, comparable
across XCDs) at entry and exit.  Output: one JSON object per shape (medians over blocks, cycles
and microseconds at the measured in-kernel clock) -> stdout / --out."""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

SLOTS, WAVES, BLOCKS = 64, 16, 2048
PER_STEP = 4
MAXSTEP = (58 - 2) // PER_STEP - 1
EPI, END, RT0, RT1, HWID, XCC = 58, 59, 60, 61, 62, 63


def read_stamps(lib):
    buf = np.zeros(BLOCKS * WAVES * SLOTS, np.uint64)
    rc = lib.dllm_stamp_read_exact(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes))
    assert rc == 0, rc
    return buf.reshape(BLOCKS, WAVES, SLOTS).astype(np.int64)


def analyze(st, nwaves, nk):
    live = st[:, 0, RT0] != 0
    nb = int(live.sum())
    s = st[:nb, :nwaves]
    # in-kernel clock: memtime ticks / realtime ticks (10 ns)
    clk = (s[:, :, END] - s[:, :, 0]) / np.maximum(s[:, :, RT1] - s[:, :, RT0], 1) * 0.1   # GHz
    ghz = float(np.median(clk))
    rt0 = s[:, 0, RT0]
    start_us = (rt0 - rt0.min()) / 100.0
    end_us = (s[:, :, RT1].max(axis=1) - rt0.min()) / 100.0
    pro = s[:, :, 1] - s[:, :, 0]
    steps = min(nk, MAXSTEP + 1)
    P = PER_STEP
    prev = [s[:, :, 1]] + [s[:, :, 5 + P * k] for k in range(steps - 1)]
    dma = np.stack([s[:, :, 2 + P * k] - prev[k] for k in range(steps)], -1)          # the stage's DMA issue
    issue = np.stack([s[:, :, 3 + P * k] - s[:, :, 2 + P * k] for k in range(steps)], -1)   # MFMA issue
    vmw = np.stack([s[:, :, 4 + P * k] - s[:, :, 3 + P * k] for k in range(steps)], -1)     # vmcnt/lgkmcnt wait
    bar = np.stack([s[:, :, 5 + P * k] - s[:, :, 4 + P * k] for k in range(steps)], -1)     # barrier
    last = s[:, :, 5 + P * (steps - 1)]
    combine = s[:, 0, EPI] - last[:, 0]        # wave 0 (k-group 0): the k-group hand-off, if any
    store = s[:, 0, END] - s[:, 0, EPI]
    total = s[:, :, END] - s[:, :, 0]

    def med(a):
        return float(np.median(a))

    to_us = 1.0 / (ghz * 1e3)
    res = {
        "blocks": nb, "waves": nwaves, "k_steps_per_wave": nk, "steps_stamped": steps, "clock_ghz": round(ghz, 3),
        "block_start_spread_us": round(float(start_us.max()), 3),
        "block_start_p50_us": round(float(np.median(start_us)), 3),
        "kernel_span_us": round(float(end_us.max()), 3),
        "block_end_p10_p50_p90_us": [round(float(np.percentile(end_us, q)), 3) for q in (10, 50, 90)],
        "median_cycles": {
            "total": med(total), "prologue": med(pro),
            "step_dma_issue": [round(med(dma[..., k]), 1) for k in range(steps)],
            "step_issue": [round(med(issue[..., k]), 1) for k in range(steps)],
            "step_vmcnt_wait": [round(med(vmw[..., k]), 1) for k in range(steps)],
            "step_barrier": [round(med(bar[..., k]), 1) for k in range(steps)],
            "combine": med(combine), "epilogue_store": med(store)},
    }
    # waves of the block's first / second half (k-group 0 / 1 or SIMD partner waves)
    if nwaves >= 8:
        h = nwaves // 2
        res["halves_step_cycles_median"] = {
            name: [round(med(a[:, :h]), 1), round(med(a[:, h:]), 1)]
            for name, a in (("dma_issue", dma[..., 1:steps - 1]), ("issue", issue[..., 1:steps - 1]),
                            ("vmcnt_wait", vmw[..., 1:steps - 1]),
                            ("barrier", bar[..., 1:steps - 1]))}
    mc = res["median_cycles"]
    scale = nk / steps   # steps past the stamped ones extrapolated at the stamped medians
    res["median_us"] = {
        "total": round(mc["total"] * to_us, 3), "prologue": round(mc["prologue"] * to_us, 3),
        "steps_dma_issue_sum": round(sum(mc["step_dma_issue"]) * scale * to_us, 3),
        "steps_issue_sum": round(sum(mc["step_issue"]) * scale * to_us, 3),
        "steps_vmcnt_wait_sum": round(sum(mc["step_vmcnt_wait"]) * scale * to_us, 3),
        "steps_barrier_sum": round(sum(mc["step_barrier"]) * scale * to_us, 3),
        "combine": round(mc["combine"] * to_us, 3), "epilogue_store": round(mc["epilogue_store"] * to_us, 3)}
    xcc = s[:, 0, XCC] & 0xF
    res["per_xcc_blocks"] = {int(x): int((xcc == x).sum()) for x in np.unique(xcc)}
    # blocks sharing a CU: (XCC, HW_ID bits 8..15 = CU / SH / SE) seen more than once
    cu = (xcc << 16) | ((s[:, 0, HWID] >> 8) & 0xFF)
    _, counts = np.unique(cu, return_counts=True)
    res["distinct_cus"] = int(len(counts))
    res["max_blocks_per_cu"] = int(counts.max())
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=str(ROOT / "diffusion-llm-rs_amd" / "lib" / "libdllm_hip_stamp.so"))
    ap.add_argument("--out", default=None)
    ap.add_argument("--shapes", default="4096x1024,4096x512,2048x2048")
    ap.add_argument("--prewarm-ms", type=float, default=300.0)
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    d = g.load_package()
    lib = d._lib.use(args.lib)
    lib.dllm_stamp_read_exact.restype = C.c_int
    lib.dllm_stamp_read_exact_zero.restype = C.c_int
    K = 4096
    rows = []
    for shp in args.shapes.split(","):
        M, N = (int(v) for v in shp.split("x"))
        gen = torch.Generator(device="cuda").manual_seed(5)
        W = 0.02 * torch.randn(K, N, device="cuda", generator=gen)
        X = torch.randn(M, K, device="cuda", generator=gen).half()
        lin = d.QuantLinear.from_weight(W, None, 4, 128, prefill_only=True)
        Y = torch.empty(M, N, dtype=torch.float16, device="cuda")
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < args.prewarm_ms:
            for _ in range(20):
                lin(X, out=Y)
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            lin(X, out=Y)
        e1.record()
        torch.cuda.synchronize()
        ev_us = e0.elapsed_time(e1) / 20 * 1e3
        assert lib.dllm_stamp_read_exact_zero() == 0
        lin(X, out=Y)
        torch.cuda.synchronize()
        st = read_stamps(lib)
        live = int((st[:, 0, RT0] != 0).sum())
        nw = int((st[0, :, RT0] != 0).sum())
        # k-steps per wave: the last stamped step slot that is non-zero on wave 0 of block 0
        nk = 0
        while nk <= MAXSTEP and st[0, 0, 5 + PER_STEP * nk] != 0:
            nk += 1
        if nk > MAXSTEP:
            nk = 4096 // 128 // (2 if nw == 8 else 1)   # the shard shapes' stages per wave (K 4096, 128-deep)
        r = {"shape": f"{M}x{K}x{N}", "event_us_per_launch": round(ev_us, 2), **analyze(st, nw, nk)}
        r["blocks_seen"] = live
        rows.append(r)
        print(json.dumps(r), flush=True)
        lin.close()
        del W, X, Y
    if args.out:
        Path(args.out).write_text("\n".join(json.dumps(r) for r in rows) + "\n")


if __name__ == "__main__":
    main()
