"""Kernel-duration summary of a rocprofv3 SQLite (rocpd) output: per (kernel, grid) count, mean and
median duration in us.  Usage: python scripts/rocpd_stats.py <results.db> [name-regex] [--seq N]"""
import re
import sqlite3
import statistics
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("dllm::(anonymous namespace)::", "")[:90]


def main():
    db, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ".")
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, duration, start from kernels order by start").fetchall()
    rows = [(short(n), g, d / 1e3, s) for n, g, d, s in rows if re.search(pat, n)]
    if "--seq" in sys.argv:
        k = int(sys.argv[sys.argv.index("--seq") + 1])
        for n, g, d, s in rows[:k]:
            print(f"{d:9.2f} us  grid {g:8d}  {n}")
        return
    groups = {}
    for n, g, d, _ in rows:
        groups.setdefault((n, g), []).append(d)
    for (n, g), ds in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(ds):6d} x  mean {statistics.mean(ds):9.2f}  median {statistics.median(ds):9.2f} us  grid {g:8d}  {n}")


if __name__ == "__main__":
    main()
