#!/bin/bash
# Effective clock / cycles of the dequant-attention kernel (config C4) per DLLM_ATTN_LAB mask:
# one rocprofv3 --pmc GRBM_GUI_ACTIVE pass per mask (the mask is read once per process).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for lab in ${LABS:-0 1 2 4 8}; do
  OUT="$PWD/gpurun_out/attn/lab$lab"
  mkdir -p "$OUT"
  DLLM_ATTN_LAB=$lab timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex "kv_" -d "$OUT" -o clk --output-format csv -- python3 scripts/attn_once.py > "$OUT/run.log" 2>&1
  rc=$?; echo "lab $lab rc=$rc $(tail -1 $OUT/run.log)"
  [ $rc -eq 0 ] || exit $rc
done
