"""Per-kernel-template effective clock and MFMA cycle efficiency from scripts/clock_probe.sh output
(GRBM_GUI_ACTIVE summed over the 8 XCDs / kernel-trace duration).  Usage: clock_summary.py DIR M [K N] [FLOP]: FLOP overrides the GEMM's 2 M N K for the efficiency column."""
import collections, csv, sys
from pathlib import Path

d = Path(sys.argv[1])
M = int(sys.argv[2])
K = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
N = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
rows, tr = [], {}
for f in sorted(d.rglob("*counter_collection.csv")):
    rows += [(f.parent, r) for r in csv.DictReader(open(f))]
    for g in f.parent.glob("*kernel_trace.csv"):
        tr.update({(f.parent, r["Dispatch_Id"]): r for r in csv.DictReader(open(g))})
order, agg = [], collections.defaultdict(list)
for parent, r in rows:
    t = tr.get((parent, r["Dispatch_Id"]))
    if t is None:
        continue
    dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) * 1e-9
    kn = r["Kernel_Name"]
    name = kn.split("(")[0] if kn.startswith("void ") else kn
    name = name.replace("void ", "").replace("dllm::", "").replace("(anonymous namespace)::", "")
    key = (name, r["Grid_Size"])
    if key not in agg:
        order.append(key)
    agg[key].append((dur, float(r["Counter_Value"])))
flop = float(sys.argv[5]) if len(sys.argv) > 5 else 2.0 * M * N * K
ideal = flop / (256 * 4 * 1024)   # cycles per SIMD at the f16 MFMA issue peak
for key in order:
    v = agg[key][2:] or agg[key]
    dur = sum(x[0] for x in v) / len(v)
    cyc = sum(x[1] for x in v) / len(v) / 8
    print(f"{key[0]:55s} n={len(v):3d} us={dur * 1e6:9.1f} cyc/XCD={cyc / 1e6:7.3f}M clk={cyc / dur / 1e9:.3f}GHz "
          f"mfma_eff={ideal / cyc:.3f}")
