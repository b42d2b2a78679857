"""Pairs a rocprofv3 kernel trace of scripts/sweep.py with its M list: per M, the median
duration of the REPS timed wq_* dispatches, HBM-roofline and MFMA-roofline fractions."""
import csv, json, sys
trace, Ms = sys.argv[1], [int(a) for a in sys.argv[2:]]
WARM, REPS, K, N = 5, 20, 4096, 4096
rows = [r for r in csv.DictReader(open(trace)) if "wq_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
i = 0
for M in Ms:
    blk = rows[i + WARM:i + WARM + REPS]
    i += WARM + REPS
    d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in blk)
    med = d[len(d) // 2] * 1e-9
    wbytes = K * N // 2 + (K // 128) * N * 5
    abytes = wbytes + M * K * 2 + M * N * 2
    print(json.dumps({"M": M, "kernel_us": round(med * 1e6, 2), "kernel": blk[0]["Kernel_Name"].split("(")[0][-40:],
                      "GB/s": round(abytes / med / 1e9, 1), "hbm_frac_8TBs": round(abytes / med / 8e12, 3),
                      "TFLOP/s": round(2 * M * N * K / med / 1e12, 1)}))
