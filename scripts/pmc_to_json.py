"""Per-launch HBM traffic of the bench GEMM kernel from rocprofv3 PMC passes (MI355X_MICROARCH.md
HBM section: FETCH_SIZE reads 1/2 of a wide coalesced stream on gfx950 -> doubled, a factor this
repo re-checks with scripts/pmc_calib.py; WRITE_SIZE is exact for 16-B stores; both in KiB).
Usage: pmc_to_json.py <pmc root> <out.json> <kernel substring> [M K N_local bits group [rev]]; the
config (+ the kernel revision tag) is recorded so bench.py only quotes the figure for the same shape
and the same kernel."""
import csv, glob, json, statistics, sys
root, out = sys.argv[1], sys.argv[2]
regex = sys.argv[3] if len(sys.argv) > 3 else "wq_gemm8_kernel<4,"
cfg = None
if len(sys.argv) > 8:
    cfg = dict(zip(("M", "K", "N_local", "bits", "group"), (int(v) for v in sys.argv[4:9])))
    if len(sys.argv) > 9:
        cfg["rev"] = sys.argv[9]
vals = {}
for f in glob.glob(f"{root}/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if regex in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
res = {"kernel": regex}
if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:   # SQ-only records carry no HBM figure
    fetch = statistics.median(vals["FETCH_SIZE"]) * 1024
    write = statistics.median(vals["WRITE_SIZE"]) * 1024
    res.update({"FETCH_SIZE_bytes_raw": fetch, "WRITE_SIZE_bytes": write, "hbm_bytes_per_launch": 2 * fetch + write,
                "correction": "FETCH_SIZE doubled (gfx950 reports 1/2 of wide coalesced reads); Infinity-Cache hits "
                              "are counted",
                "dispatches": len(vals["FETCH_SIZE"])})
if cfg is not None:
    res["config"] = cfg
for k, v in vals.items():
    if k not in ("FETCH_SIZE", "WRITE_SIZE"):
        res[k] = statistics.median(v)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
