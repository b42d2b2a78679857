#!/bin/bash
# PMC passes (one counter set per rocprofv3 run) on a bench.py kernel; sets separated by ';'.
# Usage: KREGEX=<kernel regex> PMC_SETS="A B;C D" bash scripts/pmc_sets.sh <outdir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/${1:-pmcsets}"
mkdir -p "$OUT"
IFS=';' read -ra SETARR <<< "$PMC_SETS"
for C in "${SETARR[@]}"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-include-regex "$KREGEX" -d "$OUT/$tag" -o pmc --output-format csv -- python3 bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu --no-denoise --prewarm-ms 0} > "$OUT/$tag.log" 2>&1
  rc=$?; echo "pmc $tag rc=$rc"
  case $rc in 0) ;; *) tail -3 "$OUT/$tag.log"; exit $rc;; esac
done
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.json"; cat "$OUT/summary.json"
