#!/bin/bash
# One rocprofv3 --pmc pass over scripts/sweep.py for a list of GEMM variants (A/B counters).
# PMC="..." (one pass, <= 8 SQ counters), VARIANTS, SWEEP_M.  Output: gpurun_out/pmcv/<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${TAG:-pass}
OUT="$PWD/gpurun_out/pmcv/$tag"
mkdir -p "$OUT"
VARIANTS=${VARIANTS:-4} timeout -s KILL 120 rocprofv3 --pmc ${PMC} --kernel-include-regex "${KREGEX:-wq_gemm}" -d "$OUT" -o pmc --output-format csv -- python3 scripts/sweep.py ${SWEEP_M:-16384} > "$OUT/run.log" 2>&1
rc=$?; echo "pmc $tag rc=$rc"; tail -2 "$OUT/run.log"
exit $rc
