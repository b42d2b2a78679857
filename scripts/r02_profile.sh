#!/bin/bash
# Round-2 profile pass on the GPU box: rocprofv3 kernel-trace stats of the default bench, PMC passes
# (FETCH_SIZE / WRITE_SIZE / MFMA busy + clock, each its own run) on the bench GEMM kernel, and
# the FETCH_SIZE calibration on a known streaming read.  Output under gpurun_out/prof2/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/${PROF_OUT:-prof2}"
mkdir -p "$OUT"
KREGEX=${KREGEX:-wq_gemm8_kernel}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-denoise > "$OUT/kt.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; tail -2 "$OUT/kt.log"
[ $rc -eq 0 ] || exit $rc
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-include-regex "$KREGEX" -d "$OUT/pmc_$tag" -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-denoise --prewarm-ms 0 > "$OUT/pmc_$tag.log" 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; tail -1 "$OUT/pmc_$tag.log"
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
done
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex minmax_partial -d "$OUT/calib" -o pmc --output-format csv -- python3 scripts/pmc_calib.py > "$OUT/calib.log" 2>&1
rc=$?; echo "calib rc=$rc"; tail -1 "$OUT/calib.log"
exit $rc
