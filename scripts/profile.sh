#!/bin/bash
# rocprofv3 evidence for the bench's GEMM kernel: kernel-trace stats, then separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  Output under gpurun_out/prof/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/prof"
mkdir -p "$OUT"
BARGS="${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py $BARGS > "$OUT/kt.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; tail -3 "$OUT/kt.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES;SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"}
IFS=';' read -ra SETARR <<< "$SETS"
for C in "${SETARR[@]}"; do
  tag=$(echo $C | cut -d' ' -f1)
  [ -n "$tag" ] || continue
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "${KREGEX:-wq_gemm}" -d "$OUT/pmc_$tag" -o pmc --output-format csv -- python3 bench.py ${PMC_BENCH_ARGS:---steps 5 --warmup 2 --no-cpu --no-denoise --prewarm-ms 0} > "$OUT/pmc_$tag.log" 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; tail -2 "$OUT/pmc_$tag.log"
  case $rc in 124|134|137|139) echo "hard failure; stopping"; exit $rc;; esac
done
find "$OUT" -name "*.csv" | head -50
