#!/bin/bash
# Round 6: where the C5 step goes -- product / serial / no-KV loop timings of library $LIB (default
# the product), then a kernel trace of 20 product steps, into gpurun_out/$RECORD/.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${RECORD:-r06_c5b}; mkdir -p $O
export DLLM_LIB=${LIB:-}
timeout -k 10 300 python -u scripts/c5_breakdown.py 50 product,serial,nokv > $O/breakdown.jsonl 2> $O/breakdown.err || exit $?
cat $O/breakdown.jsonl
rm -rf /tmp/prof_c5
ROUNDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_c5 -o c5 --output-format csv -- python3 scripts/c5_breakdown.py 20 ${TRACE_MODE:-product} > $O/trace.log 2>&1 || exit $?
find /tmp/prof_c5 -name "*kernel_stats.csv" -exec cp {} $O/c5_kernel_stats.csv \;
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/c5_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(r["Calls"], round(float(r["AverageNs"])/1e3, 2), round(float(r["TotalDurationNs"])/1e6, 2), r["Name"][:110])
PY
