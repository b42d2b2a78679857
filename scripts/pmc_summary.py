"""Summarise rocprofv3 PMC csvs under a directory: mean counter value per kernel (per dispatch)."""
import collections, csv, glob, json, re, sys
root = sys.argv[1]
regex = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(list)
for f in glob.glob(f"{root}/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if regex and regex not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        m = re.search(r"::(\w+<[^()]*>)\(", name) or re.search(r"::(\w+)\(", name)
        agg[(m.group(1) if m else name[:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {f"{k[0]}|{k[1]}": sum(v) / len(v) for k, v in sorted(agg.items())}
print(json.dumps(out, indent=1))
