#!/bin/bash
# SQ instruction/wait breakdown of the bench GEMM (Horner form, M = K = N = 4096) and of the F16W
# kernel on the same shape: one rocprofv3 --pmc run per counter set (<= 8 SQ counters each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/sq"; mkdir -p "$OUT"
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex wq_gemm8_kernel -d "$OUT/p$i" -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-denoise --prewarm-ms 0 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
