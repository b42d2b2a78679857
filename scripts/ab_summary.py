"""Summarise gemm_ab.py output: per shape and library, the sorted per-round medians and the Y hash."""
import collections, json, sys
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open(sys.argv[1]):
    r = json.loads(l)
    for k, v in r.items():
        if isinstance(v, dict) and "us" in v:
            d[k][r["lib"].split("/")[-1]].append((v["us"], v["yhash"]))
for k in d:
    for lib, v in d[k].items():
        us = sorted(x[0] for x in v)
        print(f"{k:10s} {lib:28s} min {us[0]:7.2f} med {us[len(us) // 2]:7.2f}  all {us}  hash {v[0][1]}")
