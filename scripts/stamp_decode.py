"""Phase breakdown of the decode GEMM (wq_decode_kernel, M <= 64) from in-kernel s_memtime stamps
(VERDICT r04 item 4), and of the mid-M exact kernel through scripts/stamp_shard.py's analysis.

Stamp build: make -C diffusion-llm-rs_amd/csrc variant VNAME=stamp VFLAGS=-DDLLM_STAMP=1
VTU="linear_exact.hip linear_wq.hip".  Per M: a chain of 40 distinct int4 g128 4096 x 4096 layers
(weights from HBM, as bench.py's m_sweep) is run warm, then once more with the stamps zeroed before
the LAST layer's launch, whose stamps are read: per (block, wave) s_memtime at entry, after the
round's loads are issued, after its MFMAs are issued, after the wave partials are in LDS, at exit;
s_memrealtime at entry / exit.  Medians over blocks (cycles and us at the in-kernel clock)."""
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
EPI, END, RT0, RT1, HWID, XCC = 58, 59, 60, 61, 62, 63


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=str(ROOT / "diffusion-llm-rs_amd" / "lib" / "libdllm_hip_stamp.so"))
    ap.add_argument("--out", default=None)
    ap.add_argument("--ms", default="1,16,64")
    ap.add_argument("--layers", type=int, default=40)
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    d = g.load_package()
    lib = d._lib.use(args.lib)
    for f in (lib.dllm_stamp_read_dec, lib.dllm_stamp_read_dec_zero):
        f.restype = C.c_int
    K = N = 4096
    gen = torch.Generator(device="cuda").manual_seed(3)
    chain = [d.QuantLinear.from_weight(0.02 * torch.randn(K, N, device="cuda", generator=gen), None, 4, 128)
             for _ in range(args.layers)]
    rows = []
    for M in (int(v) for v in args.ms.split(",")):
        X = torch.randn(M, K, device="cuda", generator=gen).half()
        Y = torch.empty(M, N, dtype=torch.float16, device="cuda")
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            for lyr in chain:
                lyr(X, out=Y)
            torch.cuda.synchronize()
        for lyr in chain[:-1]:
            lyr(X, out=Y)
        torch.cuda.synchronize()
        assert lib.dllm_stamp_read_dec_zero() == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for lyr in chain[:-1]:          # the layers before it, so the last one runs in a warm chain
            lyr(X, out=Y)
        e0.record()
        chain[-1](X, out=Y)
        e1.record()
        torch.cuda.synchronize()
        buf = np.zeros(BLOCKS * WAVES * SLOTS, np.uint64)
        assert lib.dllm_stamp_read_dec(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
        st = buf.reshape(BLOCKS, WAVES, SLOTS).astype(np.int64)
        nb = int((st[:, 0, RT0] != 0).sum())
        s = st[:nb, :8]
        clk = float(np.median((s[:, :, END] - s[:, :, 0]) / np.maximum(s[:, :, RT1] - s[:, :, RT0], 1) * 0.1))
        rt0 = s[:, 0, RT0]
        med = lambda a: float(np.median(a))
        to_us = 1.0 / (clk * 1e3)
        r = {"M": M, "blocks": nb, "clock_ghz": round(clk, 3), "event_us_last_layer": round(e0.elapsed_time(e1) * 1e3, 2),
             "block_start_spread_us": round(float((rt0.max() - rt0.min()) / 100.0), 3),
             "kernel_span_us": round(float((s[:, :, RT1].max() - rt0.min()) / 100.0), 3),
             "median_us": {
                 "entry_to_loads_issued": round(med(s[:, :, 1] - s[:, :, 0]) * to_us, 3),
                 "loads_issued_to_mfmas_issued": round(med(s[:, :, 2] - s[:, :, 1]) * to_us, 3),
                 "to_partials_in_lds": round(med(s[:, :, EPI] - s[:, :, 2]) * to_us, 3),
                 "lds_sum_and_store": round(med(s[:, :, END] - s[:, :, EPI]) * to_us, 3),
                 "total": round(med(s[:, :, END] - s[:, :, 0]) * to_us, 3)}}
        rows.append(r)
        print(json.dumps(r), flush=True)
    for lyr in chain:
        lyr.close()
    if args.out:
        Path(args.out).write_text("\n".join(json.dumps(r) for r in rows) + "\n")


if __name__ == "__main__":
    main()
