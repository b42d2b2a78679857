#!/bin/bash
# Round 5: where the C5 step goes now -- product / serial / no-KV loop timings, and a kernel trace of
# the product loop (kernel time summed per step vs the step's wall time).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_c5b; mkdir -p $O
timeout -k 10 300 python -u scripts/c5_breakdown.py 50 product,serial,nokv > $O/breakdown.jsonl 2> $O/breakdown.err || exit $?
rm -rf /tmp/prof_c5
ROUNDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_c5 -o c5 --output-format csv -- python3 scripts/c5_breakdown.py 20 product > $O/trace.log 2>&1 || exit $?
find /tmp/prof_c5 -name "*kernel_stats.csv" -exec cp {} $O/c5_kernel_stats.csv \;
find /tmp/prof_c5 -name "*kernel_trace.csv" -exec cp {} $O/c5_kernel_trace.csv \;
ls -la $O
