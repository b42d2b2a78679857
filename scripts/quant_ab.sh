#!/bin/bash
# A/B of the quantize_tensor paths under rocprofv3 kernel-trace stats: fused (default) vs generic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/quant_ab"
mkdir -p "$OUT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/fused" -o qp --output-format csv -- python3 scripts/quant_probe.py 20 > "$OUT/fused.log" 2>&1 || exit $?
DLLM_LIB=lab DLLM_QUANT_GENERIC=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/generic" -o qp --output-format csv -- python3 scripts/quant_probe.py 20 > "$OUT/generic.log" 2>&1 || exit $?
echo done
