#!/bin/bash
# One rocprofv3 --pmc pass over the C4 attention (scripts/attn_once.py).  PMC="..." (<= 8 SQ).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/attn_pmc/${TAG:-a}"
mkdir -p "$OUT"
DLLM_ATTN_LAB=${LAB:-0} timeout -s KILL 120 rocprofv3 --pmc ${PMC} --kernel-include-regex "kv_attention" -d "$OUT" -o pmc --output-format csv -- python3 scripts/attn_once.py > "$OUT/run.log" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -1 "$OUT/run.log"
exit $rc
