#!/bin/bash
# Round 6: C5 kernel timeline (gaps between kernels) under rocprofv3 --kernel-trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06_c5trace; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o c5 --output-format csv -- python3 scripts/c5_trace.py > $OUT/run.log 2>&1
echo "rc=$?"; tail -2 $OUT/run.log
