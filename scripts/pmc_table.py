"""Average each PMC counter per kernel template from scripts/pmc_variants.sh output dirs."""
import collections, csv, sys
from pathlib import Path

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            name = kn.split("(")[0][:70]
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in agg.items():
    print(name)
    for c, v in sorted(cs.items()):
        v = v[2:] or v
        print(f"   {c:28s} {sum(v) / len(v):16.4g}")
