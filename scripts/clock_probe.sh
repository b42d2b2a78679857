#!/bin/bash
# Effective shader clock per GEMM variant: GRBM_GUI_ACTIVE (cycles, summed over the 8 XCDs) per
# dispatch next to the same dispatch's kernel-trace duration.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/clk"
mkdir -p "$OUT"
VARIANTS=${VARIANTS:-4,35,36} timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex "${KREGEX:-wq_gemm}" -d "$OUT" -o clk --output-format csv -- python3 scripts/sweep.py ${SWEEP_M:-4096} > "$OUT/run.log" 2>&1
rc=$?; echo "rc=$rc"; tail -4 "$OUT/run.log"
exit $rc
